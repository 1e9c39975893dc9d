"""Quick timing of the f64-FFT PBS bench leg alone, for one-box A/B runs of two builds of the library (GPU box
helper): python tools/fft_quick.py [reps] [package dir holding tfhe_ntt_amd/]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "tfhe-rs-main_modified_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402  (first: bench.py puts the in-tree package on the path too)
import bench  # noqa: E402

assert os.path.dirname(eng.__file__).startswith(os.path.abspath(PKG)), eng.__file__


class A:
    pbs_batch = 4096
    pbs_steps = 3


dev = torch.device("cuda", 0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    r = bench.bench_pbs_fft(A, eng, torch, dev, 0, 1, lambda: None, None)
    print(json.dumps({"value": r["value"], "kernel_ms": r.get("kernel_ms")}), flush=True)
