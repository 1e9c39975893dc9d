#!/usr/bin/env python3
"""Time bench.py's config-3 external-product leg alone (diagnostic; A/B of launch forms via the environment, e.g.
r5; the persistent form it compared is gone).   python tools/ext_probe.py [batch]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import tfhe_ntt_amd as eng  # noqa: E402

dev = torch.device("cuda", 0)
args = argparse.Namespace(batch=int(sys.argv[1]) if len(sys.argv) > 1 else bench.BATCH)
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
for rep in range(2):
    r = bench.bench_ext_product(args, eng, torch, dev, 1, lambda: None, None)
    print(json.dumps({"rep": rep, "persist": os.environ.get("MI_EXT_PERSIST", "0"), "value": r["value"],
                      "kernel_ms": r["kernel_ms"], "frac": r["roofline"]["frac"]}), flush=True)
