"""Quick timing of the config-4 PBS legs (BNF and Solinas) alone, for one-box A/B runs of two builds of the
library (GPU box helper): python tools/pbs_quick.py [package dir holding tfhe_ntt_amd/]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tfhe-rs-main_modified_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402  (first: bench.py puts the in-tree package on the path too)
import bench  # noqa: E402

assert os.path.dirname(eng.__file__).startswith(os.path.abspath(PKG)), eng.__file__


class A:
    pbs_batch = 4096


dev = torch.device("cuda", 0)
for name, fn in (("bnf", lambda: bench.bench_pbs(A, eng, torch, dev, 0, 1, lambda: None, None)),
                 ("sol", lambda: bench.bench_pbs_solinas(A, eng, torch, dev, 1, lambda: None, None))):
    r = fn()
    print(json.dumps({"leg": name, "value": r["value"], "kernel_ms": r["kernel_ms"],
                      "valu_frac": r["roofline"]["frac"]}), flush=True)
