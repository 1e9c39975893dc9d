#!/usr/bin/env python3
"""bench.py's config-3 external-product leg alone, repeated (diagnostic A/B of body variants):
python tools/ext_probe.py [reps] [package dir holding tfhe_ntt_amd/] [fft: the f64 leg instead]"""
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
    batch = bench.BATCH


dev = torch.device("cuda", 0)
bench.SIMDS = torch.cuda.get_device_properties(dev).multi_processor_count * 4
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    if len(sys.argv) > 3 and sys.argv[3] == "fft":
        r = bench.bench_ext_product_fft(A, eng, torch, dev, 1, lambda: None, None)
        print(json.dumps({"value": r["value"], "kernel_ms": r["kernel_ms"], "k2_l2": r["k2_l2"]["value"]}), flush=True)
        continue
    r = bench.bench_ext_product(A, eng, torch, dev, 1, lambda: None, None)
    print(json.dumps({"value": r["value"], "kernel_ms": r["kernel_ms"], "valu_frac": r["roofline"]["frac"]}), flush=True)
