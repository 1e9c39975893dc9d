#!/usr/bin/env python3
"""bench.py's config-3 external-product leg alone, repeated (diagnostic A/B of body variants):
python tools/ext_probe.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import tfhe_ntt_amd as eng  # noqa: E402


class A:
    batch = bench.BATCH


dev = torch.device("cuda", 0)
bench.SIMDS = torch.cuda.get_device_properties(dev).multi_processor_count * 4
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    r = bench.bench_ext_product(A, eng, torch, dev, 1, lambda: None, None)
    print(json.dumps({"value": r["value"], "kernel_ms": r["kernel_ms"], "valu_frac": r["roofline"]["frac"]}), flush=True)
