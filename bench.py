#!/usr/bin/env python3
"""Headline benchmark: batched negacyclic NTT, N = 2048, Goldilocks p = 2^64 - 2^32 + 1.

BASELINE.json metric "forward+inverse NTTs/sec, N=2048 u64 prime, batch=8192" (config 2).
One *step* = `Plan::fwd` over a resident batch of 8192 polynomials followed by `Plan::inv` over
the same batch (two kernel launches, as the reference API has two calls; prime64.rs:897,975).
`value` counts fwd+inv pairs per second over the whole job.

Multi-GPU: polynomials are independent, so each rank owns its own 8192-poly
shard (weak scaling) and there is no data-path collective; torch.distributed (RCCL) is used only
for the start/stop barriers and the max-over-ranks time.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-main_modified_amd"))

N = 2048
BATCH = 8192
SOLINAS_P = 0xFFFFFFFF00000001
SEED = 0x74666865 + 2  # 0x74666865 + config id
BYTES_PER_POLY_PASS = 2 * N * 8  # read 16 KiB + write 16 KiB per polynomial per transform
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline leg")
    return ap.parse_args()


def cpu_baseline(seconds: float):
    """The oracle's restatement of the reference AVX-512 path (or scalar), OpenMP over polys.

    TEST/BASELINE infrastructure only: measured beside the GPU, never instead of it.
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    plan = O.Plan.try_new(N, SOLINAS_P)
    sample = max(threads * 8, 256)
    buf = O.fill_uniform(SEED, SOLINAS_P, sample * N)
    avx = O.have_avx512()
    fwd = plan.fwd_avx512_inplace if avx else plan.fwd_scalar_inplace
    inv = plan.inv_avx512_inplace if avx else plan.inv_scalar_inplace
    fwd(buf, threads); inv(buf, threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        fwd(buf, threads)
        inv(buf, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": reps * sample / el,
        "unit": "fwd+inv NTT pairs/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{reps} x ({sample} polys fwd+inv) N=2048 Solinas in {el:.1f}s, "
                   f"{'AVX-512 restatement of generic_solinas.rs fwd/inv_depth_first_avx512' if avx else 'scalar restatement'}, "
                   f"OpenMP {threads} threads, {cpu_model}"),
    }


def load_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/*/pmc_traffic.json)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import tfhe_ntt_amd as eng

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    batch = args.batch
    buf = torch.empty((batch, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(buf, SEED + rank * 0x1000, SOLINAS_P)  # inputs resident in HBM before timing
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        plan.fwd(buf)
        plan.inv(buf)
    torch.cuda.synchronize()

    K = args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        ev[k][0].record()
        plan.fwd(buf)
        ev[k][1].record()
        plan.inv(buf)
        ev[k][2].record()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    fwd_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / K
    inv_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / K
    dom_ms = max(fwd_ms, inv_ms)
    dom = "fwd" if fwd_ms >= inv_ms else "inv"
    bytes_launch = batch * BYTES_PER_POLY_PASS
    achieved = bytes_launch / (dom_ms * 1e-3) / 1e9

    units = world * batch * K
    value = units / elapsed
    out = {
        "metric": "forward+inverse NTTs/sec, N=2048 u64 prime, batch=8192",
        "value": value,
        "unit": "fwd+inv NTT pairs/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: device counter-based splitmix64, uniform in [0,p) (SURVEY.md 8d)",
        "config": {
            "workload": "tfhe-ntt prime64 Plan fwd then inv, N=2048, Solinas p=2^64-2^32+1, batch 8192 per GPU (config 2)",
            "n": N,
            "batch_per_gpu": batch,
            "global_batch": batch * world,
            "parallelism": f"independent shards x{world} (no data-path collective)",
        },
        "kernels": {"fwd_ms": fwd_ms, "inv_ms": inv_ms},
        "roofline": {
            "bound": "hbm",
            "kernel": f"ntt {dom}",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": load_traffic(),
            "algorithmic_bytes_per_launch": bytes_launch,
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
