#!/usr/bin/env python3
"""Per-polynomial time of the N = 2048 transform launches against the batch size (diagnostic: how much of a
batch-8192 launch is ramp-up / drain rather than steady issue).   python tools/batch_scaling_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402

P = 0xFFFFFFFF00000001
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(s)
plan = eng.Plan.try_new(2048, P)
big = torch.empty((65536, 2048), dtype=torch.int64, device=dev)
eng.fill_uniform(big, 7, P)
# warm the clock: ~1 s of transforms
for _ in range(400):
    plan.fwd(big[:8192])
    plan.inv(big[:8192])
torch.cuda.synchronize()
rows = []
for batch in (1024, 2048, 4096, 8192, 16384, 32768, 65536, 8192):
    buf = big[:batch]
    reps = max(20, 200 * 8192 // batch)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(s)
    for _ in range(reps):
        plan.fwd(buf)
    e1.record(s)
    for _ in range(reps):
        plan.inv(buf)
    e2.record(s)
    torch.cuda.synchronize()
    f = e0.elapsed_time(e1) / reps * 1e3
    i = e1.elapsed_time(e2) / reps * 1e3
    rows.append({"batch": batch, "fwd_us": f, "inv_us": i, "fwd_ns_per_poly": f / batch * 1e3,
                 "inv_ns_per_poly": i / batch * 1e3,
                 "hbm_frac_pair": 65536 * batch / ((f + i) * 1e-6) / 8e12})
    print(json.dumps(rows[-1]), flush=True)
