#!/usr/bin/env python3
"""A/B of the headline transform between package builds, one child process per measurement, orders rotated
(diagnostic; the reported numbers come from bench.py):
  python tools/headline_ab.py <reps> <pkg-dir> [<pkg-dir> ...]
A pkg-dir holds a tfhe_ntt_amd/ with its own libtfhe_ntt_amd.so (the tree's is tfhe-rs-main_modified_amd).  Each child
warms the GPU for ~1.5 s of fwd+inv steps at the config-2 batch, then times the driver's 20 steps and a 2-s loop with
HIP events on the launching stream and prints us per launch."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, P, BATCH = 2048, 0xFFFFFFFF00000001, 8192


def child(pkg):
    sys.path.insert(0, pkg)
    import torch
    import tfhe_ntt_amd as eng

    dev = torch.device("cuda", 0)
    work = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(work)
    plan = eng.Plan.try_new(N, P, device=0)
    buf = torch.empty((BATCH, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(buf, 1234, P)
    torch.cuda.synchronize()

    def loop(k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(work)
        for _ in range(k):
            plan.fwd(buf)
            plan.inv(buf)
        e1.record(work)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (2 * k)

    t0 = time.time()
    while time.time() - t0 < 1.5:
        loop(200)
    loop(5)
    d20 = loop(20)
    ss = loop(int(2.0 / 115e-6))
    print(json.dumps({"pkg": os.path.basename(pkg.rstrip("/")), "driver20_us": d20, "steady_us": ss,
                      "frac20": BATCH * N * 8 * 2 / (d20 * 1e-6) / 8e12}), flush=True)


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2])
    reps, pkgs = int(sys.argv[1]), sys.argv[2:]
    for r in range(reps):
        order = pkgs[r % len(pkgs):] + pkgs[:r % len(pkgs)]
        for pkg in order:
            rc = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", os.path.abspath(pkg)],
                                timeout=120).returncode
            if rc:
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
