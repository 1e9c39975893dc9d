#!/usr/bin/env python3
"""Time bench.py's PBS legs at the other shortint shapes only (diagnostic; the numbers the bench reports come from
bench.py itself).   python tools/shape_probe.py [--fft] [message_1_carry_1 message_3_carry_3 message_4_carry_4]
--fft times the f64-FFT legs (bench_pbs_shape_fft) instead of the BNF NTT ones."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PROBE_PKG=<dir holding another tfhe_ntt_amd/ with its own .so>: A/B against another build in one session
sys.path[:0] = [ROOT, os.environ.get("PROBE_PKG") or os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402  (before bench, whose import puts the tree's package first on sys.path)
import bench  # noqa: E402


fft = "--fft" in sys.argv
names = [a for a in sys.argv[1:] if a != "--fft"] or list(bench.SHAPE_LEGS)
for i, nm in enumerate(names):  # "N,k,n,base_log,level,batch" adds an ad-hoc shape
    if "," in nm:
        bench.SHAPE_LEGS[nm] = tuple(int(v) for v in nm.split(","))
dev = torch.device("cuda", 0)
bench.SIMDS = torch.cuda.get_device_properties(dev).multi_processor_count * 4
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
for name in names:
    leg = bench.bench_pbs_shape_fft if fft else bench.bench_pbs_shape
    r = leg(name, None, eng, torch, dev, 1, lambda: None, None)
    print(json.dumps({"shape": name, "value": r["value"], "kernel_ms": r["kernel_ms"], "steps": r["steps"],
                      "engine": r["config"]["engine"]}), flush=True)
