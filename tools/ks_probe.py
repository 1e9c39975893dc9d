#!/usr/bin/env python3
"""Time bench.py's keyswitch leg alone (diagnostic): python tools/ks_probe.py [reps]; PROBE_PKG=<dir> loads another
build of the package (A/B in one session)."""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PROBE_PKG=<dir holding another tfhe_ntt_amd/ with its own .so>: A/B against another build in one session
sys.path[:0] = [ROOT, os.environ.get("PROBE_PKG") or os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402  (before bench, whose import puts the tree's package first on sys.path)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
args = types.SimpleNamespace(pbs_batch=bench.PBS_BATCH)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    r = bench.bench_keyswitch(args, eng, torch, dev, 1, lambda: None, None)
    print(json.dumps({"value": r["value"], "kernel_ms": r["kernel_ms"], "frac": r["roofline"]["frac"],
                      "pkg": os.path.dirname(eng.__file__)}), flush=True)
