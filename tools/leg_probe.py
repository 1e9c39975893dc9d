#!/usr/bin/env python3
"""Time one of bench.py's legs alone (diagnostic; the numbers the bench reports come from bench.py itself):
  python tools/leg_probe.py <keyswitch|ks32_pbs|ext_product|pbs|pbs_solinas|bsk_conversion|plans> [reps]
PROBE_PKG=<dir holding another tfhe_ntt_amd/ with its own .so> runs another build of the package (A/B in one session)."""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("PROBE_PKG") or os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402  (before bench, whose import puts the tree's package first on sys.path)
import bench  # noqa: E402

leg = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda", 0)
bench.SIMDS = torch.cuda.get_device_properties(dev).multi_processor_count * 4
torch.cuda.set_stream(torch.cuda.Stream(device=dev))
args = types.SimpleNamespace(pbs_batch=bench.PBS_BATCH, batch=bench.BATCH, no_shapes=True, pbs_steps=10)
fn = getattr(bench, "bench_" + leg)
for _ in range(reps):
    if leg in ("pbs", "pbs_fft"):
        r = fn(args, eng, torch, dev, 0, 1, lambda: None, None)
    else:
        r = fn(args, eng, torch, dev, 1, lambda: None, None)
    if "value" not in r:  # a group of legs (plans): one line per member
        for k, v in r.items():
            if isinstance(v, dict) and "value" in v:
                print(json.dumps({"leg": f"{leg}.{k}", "value": v["value"], "unit": v.get("unit"),
                                  "kernel_ms": v.get("kernel_ms"), "frac": (v.get("roofline") or {}).get("frac"),
                                  "pkg": os.path.dirname(eng.__file__)}), flush=True)
        continue
    print(json.dumps({"leg": leg, "value": r["value"], "kernel_ms": r.get("kernel_ms"),
                      "sub": r.get("keyswitch_and_switch"), "pkg": os.path.dirname(eng.__file__)}), flush=True)
