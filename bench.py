#!/usr/bin/env python3
"""Headline benchmark: batched negacyclic NTT, N = 2048, Goldilocks p = 2^64 - 2^32 + 1.

BASELINE.json metric "forward+inverse NTTs/sec, N=2048 u64 prime, batch=8192" (config 2).
One *step* = `Plan::fwd` over a resident batch of 8192 polynomials followed by `Plan::inv` over
the same batch (two kernel launches, as the reference API has two calls; prime64.rs:897,975).
`value` counts fwd+inv pairs per second over the whole job.

Multi-GPU: polynomials are independent, so each rank owns its own 8192-poly
shard (weak scaling) and there is no data-path collective; torch.distributed (RCCL) is used only
for the start/stop barriers and the max-over-ranks time.

The second half of the metric, "PBS/sec @ shortint default params" (config 4), is measured in the
same run and reported under "pbs": one step = a batch of 4096 programmable bootstraps per GPU at
the PARAM_MESSAGE_2_CARRY_2 shape (n=918, k=1, N=2048, base 2^23, l=1, native 2^64 ciphertexts
through the BNF NTT algorithm, ntt64_bnf_pbs.rs:469-540), one fused kernel launch.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--no-pbs]

``--gpus N`` with N > 1 outside a torch.distributed launch re-launches this script under
``python -m torch.distributed.run --nproc-per-node N`` (as a child process, before anything touches the
GPU) and exits with its status; inside a launch, WORLD_SIZE must equal N.
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
# Integer-VALU issue model of the generated bodies (tools/valu_cost.py: instruction mix x the issue
# costs measured by tools/valu_probe.hip; tests/test_bench_contract.py keeps these in sync), and the
# MI355X peak engine clock it is priced at.
VALU_CYCLES = {"fwd": 13631.3, "inv": 14158.8, "pbs_step": 35057.4, "pbs_sol_step": 35378.7, "ext_bnf": 33859.1}
SIMDS, PEAK_CLOCK_HZ = 256 * 4, 2.4e9
# PARAM_MESSAGE_2_CARRY_2 shape (ks_pbs.rs:29-47)
PBS_N_LWE, PBS_BASE_LOG, PBS_LEVEL, PBS_BATCH = 918, 23, 1, 4096


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults keep every GPU leg busy for seconds (the NTT leg ~1.6 s), so a sampler outside the process
    # sees the work, while the whole run stays well under a minute of GPU time
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-pbs", action="store_true", help="skip the config-4 PBS leg")
    ap.add_argument("--no-shapes", action="store_true",
                    help="skip the other-shortint-shape PBS legs (the PMC passes of tools/profile_session.sh: rocprofv3 "
                         "--pmc segfaults on the host inside the shape-generic f64 engine's launch)")
    ap.add_argument("--pbs-batch", type=int, default=PBS_BATCH)
    ap.add_argument("--pbs-steps", type=int, default=10, help="steps of the config-5 sharded leg (N > 1)")
    ap.add_argument("--steady-seconds", type=float, default=1.0, help="length of the steady_state loop")
    ap.add_argument("--pbs-global", type=int, default=65536, help="config 5 global batch (N > 1 only)")
    # rehearsal of the multi-rank path on a 1-GPU box: every rank on cuda:0, gloo instead of RCCL
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--same-device", action="store_true")
    return ap.parse_args()


LEG_SECONDS = 0.3  # every non-headline leg times at least this much GPU work (no --steps-scaled legs)
# order of the legs in the JSON line (not the order they run in): the driver keeps only the tail of stdout, so the
# config-3 / config-4 legs come last, followed only by the compact legs_summary
LEG_ORDER = ("plans", "pbs_shapes", "pbs_shapes_fft", "keyswitch", "ks_pbs", "ks32_pbs", "ks_pbs_fft", "ext_product_fft",
             "bsk_conversion",
             "pbs_fft", "ext_product", "pbs_solinas", "pbs")


def timed_leg(run, torch, barrier, dist, dev, min_seconds=LEG_SECONDS, min_steps=2, max_steps=200000):
    """Time `run` (one step of a leg) over a time-based step count: one untimed step sizes K so the timed loop
    holds >= min_seconds of GPU work; K agrees over ranks (max).  HIP events on the current (launching) stream
    bracket the loop.  Returns (K, wall seconds max over ranks, kernel ms per step from the events)."""
    import math
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    one = max(time.perf_counter() - t0, 1e-6)
    K = int(min(max_steps, max(min_steps, math.ceil(min_seconds / one))))
    if dist is not None:
        import tfhe_ntt_amd as eng
        K = int(eng.multi_gpu.max_over_ranks(float(K), dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(K):
        run()
    e1.record()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        import tfhe_ntt_amd as eng
        el = eng.multi_gpu.max_over_ranks(el, dev)
    return K, el, e0.elapsed_time(e1) / K


def valu_roofline(waves_per_unit, cycles_per_wave, units, kernel_ms, note):
    """Integer-VALU bound of a leg: issue cycles of the generated body (tools/valu_cost.py) over all SIMDs at the
    peak engine clock, vs the measured kernel time."""
    model_ms = units * waves_per_unit * cycles_per_wave / SIMDS / PEAK_CLOCK_HZ * 1e3
    return {"bound": "valu", "issue_cycles_per_wave_unit": cycles_per_wave, "waves_per_unit": waves_per_unit,
            "model_ms": model_ms, "measured_ms": kernel_ms, "frac": model_ms / kernel_ms, "peak_clock_ghz": 2.4,
            "note": note}


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


def cpu_baseline_pbs(seconds: float):
    """Oracle restatement of programmable_bootstrap_ntt64_bnf (transforms through the AVX-512
    restatement, as the reference's runtime dispatch), one PBS per thread, OpenMP over the batch."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    ctx = O.NttContext(N)
    n_lwe, k = PBS_N_LWE, 1
    bsk = O.fill_uniform(SEED + 20, SOLINAS_P, n_lwe * PBS_LEVEL * 4 * N)
    lut = O.fill_uniform(SEED + 21, 0, 2 * N)
    sample = threads * 2
    lwe = O.fill_uniform(SEED + 22, 0, sample * (n_lwe + 1)).reshape(sample, n_lwe + 1)
    out = np.zeros((sample, k * N + 1), np.uint64)
    O.pbs_set_fast_ntt(True)
    try:
        reps, t0 = 0, time.perf_counter()
        while True:
            ctx.pbs_batch_bnf(lwe, lut, bsk, k, PBS_BASE_LOG, PBS_LEVEL, threads=threads, out=out)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        O.pbs_set_fast_ntt(False)
    return {
        "value": reps * sample / el,
        "unit": "PBS/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{reps} x {sample} BNF PBS (n=918, N=2048, l=1) in {el:.1f}s, restatement of "
                   f"ntt64_bnf_pbs.rs with {'AVX-512' if O.have_avx512() else 'scalar'} transforms, "
                   f"OpenMP {threads} threads"),
    }


def bench_pbs(args, eng, torch, dev, rank, world, barrier, dist):
    """Config 4: batched BNF PBS, key and inputs resident in HBM, one fused launch per step."""
    M = eng.ntt64_pbs
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    n_lwe, batch = PBS_N_LWE, args.pbs_batch
    # synthetic NTT-domain key (60 MB): per-step work does not depend on its values
    bsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(bsk, SEED + 10, SOLINAS_P)
    key = M.NttBootstrapKey(plan, bsk, PBS_BASE_LOG, PBS_LEVEL, M.BNF)
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 11, 0)
    lwe = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 12 + rank * 0x1000, 0)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)
    run = lambda: M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(lwe, out, lut, key)
    K, elapsed, kernel_ms = timed_leg(run, torch, barrier, dist, dev)
    res = {
        "metric": "PBS/sec @ shortint default params",
        "value": world * batch * K / elapsed,
        "unit": "PBS/s",
        "steps": K,
        "ms_per_step": elapsed / K * 1e3,
        "kernel_ms": kernel_ms,
        "ntt_equivalents_per_s": world * batch * K / elapsed * 4 * n_lwe,
        "config": {
            "workload": "programmable_bootstrap_ntt64_bnf, PARAM_MESSAGE_2_CARRY_2 shape n=918 k=1 N=2048 "
                        "base_log=23 level=1, standard modulus switch (config 4)",
            "batch_per_gpu": batch,
            "global_batch": batch * world,
            "key": "synthetic random NTT-domain BSK (60,162,048 B), resident",
        },
        "roofline": valu_roofline(2 * n_lwe, VALU_CYCLES["pbs_step"], batch, kernel_ms,
                                  "integer VALU-bound (3,672 NTTs + 11.3 M modmul-class ops per PBS; 2 waves x n CMUX "
                                  "steps per PBS); per-step HBM traffic is the L2-resident key plus 23.7 KB of LWE "
                                  "in/out per PBS"),
        "cpu_baseline": None,
    }
    if dist is not None:
        res["sharded"] = bench_pbs_sharded(
            args, eng, torch, dev, rank, world, barrier,
            lambda li, lo: M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(li, lo, lut, key), bsk)
    del key
    return res


def bench_pbs_solinas(args, eng, torch, dev, world, barrier, dist):
    """Solinas-modulus PBS (programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized, ntt64_pbs.rs:482-538)
    at the PARAM_MESSAGE_2_CARRY_2 shape with q = p: the reference's own NTT PBS benchmark runs the shortint
    parameter sets with this custom modulus (tfhe-benchmark/benches/core_crypto/pbs_bench.rs:646-905)."""
    M = eng.ntt64_pbs
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    n_lwe, batch = PBS_N_LWE, args.pbs_batch
    bsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(bsk, SEED + 60, SOLINAS_P)
    key = M.NttBootstrapKey(plan, bsk, PBS_BASE_LOG, PBS_LEVEL, M.SOLINAS)
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 61, SOLINAS_P)
    lwe = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 62, SOLINAS_P)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)
    run = lambda: M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(lwe, out, lut, key)
    K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev)
    del key
    return {"metric": "PBS/sec, Solinas modulus (ntt64_pbs), PARAM_MESSAGE_2_CARRY_2 shape", "value": world * batch * K / el,
            "unit": "PBS/s", "steps": K, "ms_per_step": el / K * 1e3, "kernel_ms": kernel_ms,
            "ntt_equivalents_per_s": world * batch * K / el * 4 * n_lwe,
            "config": {"workload": "programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized, q = 2^64 - 2^32 + 1, "
                                   "n=918 k=1 N=2048 base_log=23 level=1 (pbs_bench.rs:646-905 shape)",
                       "batch_per_gpu": batch},
            "roofline": valu_roofline(2 * n_lwe, VALU_CYCLES["pbs_sol_step"], batch, kernel_ms,
                                      "integer VALU-bound; kernel_ms includes the modulus-switch pre-pass "
                                      "(ms_non_native, HBM-bound, ~30 us)"),
            "cpu_baseline": None}


def cpu_baseline_pbs_solinas(seconds: float):
    """Oracle restatement of programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized (ntt64_pbs.rs:482-538) with
    the AVX-512 transform restatement, one PBS per thread, OpenMP over a bounded batch."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    ctx = O.NttContext(N)
    n_lwe, k = PBS_N_LWE, 1
    bsk = O.fill_uniform(SEED + 60, SOLINAS_P, n_lwe * PBS_LEVEL * 4 * N)
    lut = O.fill_uniform(SEED + 61, SOLINAS_P, 2 * N)
    sample = threads * 2
    lwe = O.fill_uniform(SEED + 62, SOLINAS_P, sample * (n_lwe + 1)).reshape(sample, n_lwe + 1)
    out = np.zeros((sample, k * N + 1), np.uint64)
    O.pbs_set_fast_ntt(True)
    try:
        reps, t0 = 0, time.perf_counter()
        while True:
            ctx.pbs_batch_solinas(lwe, lut, bsk, k, PBS_BASE_LOG, PBS_LEVEL, threads=threads, out=out)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        O.pbs_set_fast_ntt(False)
    return {"value": reps * sample / el, "unit": "PBS/s", "cores": threads, "kind": "port",
            "sample": (f"{reps} x {sample} Solinas-modulus PBS (n=918, N=2048, l=1) in {el:.1f}s, restatement of "
                       f"ntt64_pbs.rs with {'AVX-512' if O.have_avx512() else 'scalar'} transforms, "
                       f"OpenMP {threads} threads")}


# the other shortint parameter sets' PBS shapes (shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/
# ks_pbs.rs:8-90): name -> (N, k, n, base_log, level, batch per step)
SHAPE_LEGS = {
    "message_1_carry_1": (512, 4, 879, 23, 1, 4096),
    "message_3_carry_3": (8192, 1, 1077, 15, 2, 1024),
    "message_4_carry_4": (65536, 1, 1117, 11, 3, 192),
}


def bench_pbs_shape(name, args, eng, torch, dev, world, barrier, dist):
    """BNF PBS at another shortint shape (synthetic NTT-domain key and inputs, resident): N = 512 runs the fused
    one-workgroup-per-ciphertext kernel (pbs_kernels.hip), N = 8192 / 65536 the multi-kernel blind rotation
    (pbs_large.hip, accumulators in HBM).  Same time-based timing as the other legs."""
    M = eng.ntt64_pbs
    n, k, n_lwe, base_log, level, batch = SHAPE_LEGS[name]
    plan = eng.Plan.try_new(n, SOLINAS_P, device=dev.index)
    bsk = torch.empty((n_lwe, level, k + 1, k + 1, n), dtype=torch.int64, device=dev)
    eng.fill_uniform(bsk, SEED + 90, SOLINAS_P)
    key = M.NttBootstrapKey(plan, bsk, base_log, level, M.BNF)
    del bsk
    lut = torch.empty((k + 1, n), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 91, 0)
    lwe = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 92, 0)
    out = torch.empty((batch, k * n + 1), dtype=torch.int64, device=dev)
    run = lambda: M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(lwe, out, lut, key)
    K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev, min_steps=3)
    del key
    ntts = n_lwe * (level + 1) * (k + 1)  # forward (level x (k+1)) + inverse (k+1) transforms per CMUX step
    return {"metric": f"PBS/sec, BNF NTT PBS at the {name.upper()} shape", "value": world * batch * K / el,
            "unit": "PBS/s", "steps": K, "ms_per_step": el / K * 1e3, "kernel_ms": kernel_ms,
            "ntt_per_s": world * batch * K / el * ntts,
            "config": {"workload": f"programmable_bootstrap_ntt64_bnf, N={n} k={k} n={n_lwe} base_log={base_log} "
                                   f"level={level} (shortint {name.upper()} shape), synthetic key",
                       "batch_per_gpu": batch,
                       "engine": "multi-kernel blind rotation (pbs_large.hip)" if n >= 8192 else
                                 "fused one-workgroup-per-ciphertext kernel (pbs_kernels.hip)"},
            "cpu_baseline": None}


def cpu_baseline_pbs_shape(name, seconds: float):
    """Oracle restatement of the BNF PBS at the shape (OpenMP, one PBS per thread), bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    n, k, n_lwe, base_log, level, _ = SHAPE_LEGS[name]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    ctx = O.NttContext(n)
    bsk = O.fill_uniform(SEED + 90, SOLINAS_P, n_lwe * level * (k + 1) ** 2 * n)
    lut = O.fill_uniform(SEED + 91, 0, (k + 1) * n)
    sample = threads
    lwe = O.fill_uniform(SEED + 92, 0, sample * (n_lwe + 1)).reshape(sample, n_lwe + 1)
    out = np.zeros((sample, k * n + 1), np.uint64)
    O.pbs_set_fast_ntt(True)
    try:
        reps, t0 = 0, time.perf_counter()
        while True:
            ctx.pbs_batch_bnf(lwe, lut, bsk, k, base_log, level, threads=threads, out=out)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        O.pbs_set_fast_ntt(False)
    return {"value": reps * sample / el, "unit": "PBS/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {sample} BNF PBS (N={n}, k={k}, n={n_lwe}, l={level}) in {el:.1f}s, restatement of "
                      f"ntt64_bnf_pbs.rs, OpenMP {threads} threads"}


def bench_pbs_shape_fft(name, args, eng, torch, dev, world, barrier, dist):
    """The default (f64-FFT) shortint PBS at another parameter set's shape: the shape-generic engine
    (fft64_generic.hip: row / column four-step transforms, accumulators in HBM), synthetic Fourier key resident."""
    F = eng.fft64
    n, k, n_lwe, base_log, level, batch = SHAPE_LEGS[name]
    fft = F.Fft(n, dev.index)
    std = torch.empty((n_lwe, level, k + 1, k + 1, n), dtype=torch.int64, device=dev)
    eng.fill_uniform(std, SEED + 93, 0)
    fbsk = torch.empty((n_lwe, level, k + 1, k + 1, n // 2, 2), dtype=torch.float64, device=dev)
    F.convert_standard_lwe_bootstrap_key_to_fourier(std, fbsk, fft)
    del std
    key = F.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    lut = torch.empty((k + 1, n), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 94, 0)
    lwe = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 95, 0)
    out = torch.empty((batch, k * n + 1), dtype=torch.int64, device=dev)
    run = lambda: F.programmable_bootstrap_lwe_ciphertext(lwe, out, lut, key, F.MS_CENTERED)
    K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev, min_steps=3)
    del key, fbsk
    return {"metric": f"PBS/sec, f64-FFT PBS at the {name.upper()} shape", "value": world * batch * K / el,
            "unit": "PBS/s", "steps": K, "ms_per_step": el / K * 1e3, "kernel_ms": kernel_ms, "dtype": "f64",
            "config": {"workload": f"programmable_bootstrap_lwe_ciphertext (tfhe-fft path), N={n} k={k} n={n_lwe} "
                                   f"base_log={base_log} level={level} (shortint {name.upper()} shape), centered "
                                   "modulus switch, synthetic key",
                       "batch_per_gpu": batch, "engine": "shape-generic f64 engine (fft64_generic.hip)"},
            "cpu_baseline": None, "cpu_baseline_note": NO_FFT_BASELINE}


NO_FFT_BASELINE = ("no comparable CPU baseline: the reference's f64 path is tfhe-fft (AVX-512 / FMA, Rust), absent here; "
                   "cpu_numpy_restatement is a single-thread numpy timing, not a baseline")


def cpu_baseline_pbs_fft(n, k, n_lwe, base_log, level, seconds: float, threads_note="numpy, 1 thread"):
    """The numpy restatement of the f64 PBS (oracle/fft_oracle.py: np.fft transforms, one batch vectorised) on a
    bounded sample: a batch of 8 ciphertexts over the first n' mask elements, timed and scaled to n (every CMUX
    step costs the same)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import fft_oracle as FO

    g = np.random.default_rng(SEED + 96)
    sample, steps = 8, 4
    bsk = g.integers(0, 2**64, size=(steps, level, k + 1, k + 1, n), dtype=np.uint64)
    fbsk = FO.forward_as_torus(bsk)
    lut = g.integers(0, 2**64, size=(k + 1, n), dtype=np.uint64)
    lwe = g.integers(0, 2**64, size=(sample, steps + 1), dtype=np.uint64)
    reps, t0 = 0, time.perf_counter()
    while True:
        FO.pbs(lwe, lut, fbsk, base_log, level)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    per_pbs = el / (reps * sample) * n_lwe / steps
    return {"value": 1.0 / per_pbs, "unit": "PBS/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x {sample} PBS of {steps} CMUX steps (N={n}, k={k}, l={level}) in {el:.1f}s, scaled to "
                      f"n={n_lwe} steps; numpy restatement of fft64_pbs.rs ({threads_note})"}


def bench_pbs_fft(args, eng, torch, dev, rank, world, barrier, dist):
    """The default shortint PBS, f64-FFT path (programmable_bootstrap_lwe_ciphertext, fft64_pbs.rs:924-1060)
    at PARAM_MESSAGE_2_CARRY_2's shape: native 2^64 ciphertexts, Fourier key (60 MB of complex f64) resident."""
    F = eng.fft64
    fft = F.Fft(N, dev.index)
    n_lwe, batch = PBS_N_LWE, args.pbs_batch
    std = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(std, SEED + 80, 0)
    fbsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N // 2, 2), dtype=torch.float64, device=dev)
    F.convert_standard_lwe_bootstrap_key_to_fourier(std, fbsk, fft)
    del std
    key = F.FourierLweBootstrapKey(fbsk, PBS_BASE_LOG, PBS_LEVEL, fft)
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 81, 0)
    lwe = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 82 + rank * 0x1000, 0)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)
    run = lambda: F.programmable_bootstrap_lwe_ciphertext(lwe, out, lut, key)
    K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev)
    res = {"metric": "PBS/sec, f64-FFT path (default shortint PBS), PARAM_MESSAGE_2_CARRY_2 shape",
           "value": world * batch * K / el, "unit": "PBS/s", "steps": K, "ms_per_step": el / K * 1e3,
           "kernel_ms": kernel_ms, "dtype": "f64",
           "config": {"workload": "programmable_bootstrap_lwe_ciphertext (tfhe-fft path), n=918 k=1 N=2048 "
                                  "base_log=23 level=1, standard modulus switch", "batch_per_gpu": batch},
           "cpu_baseline": None, "cpu_baseline_note": NO_FFT_BASELINE}
    if dist is not None:
        res["sharded"] = bench_pbs_sharded(
            args, eng, torch, dev, rank, world, barrier,
            lambda li, lo: F.programmable_bootstrap_lwe_ciphertext(li, lo, lut, key), fbsk)
    del key
    return res


def bench_pbs_sharded(args, eng, torch, dev, rank, world, barrier, pbs, bsk):
    """Config 5: one global batch of PBS (default 65,536) held on the root, scattered over the ranks,
    bootstrapped, gathered back (strong scaling).  The transfers are grouped point-to-point sends from
    the root (multi_gpu.scatter_batch / gather_batch: RCCL over xGMI, the root feeding each peer over
    its own link); the key broadcast is timed once, outside the steady state.  `pbs(lwe_in, lwe_out)` runs
    the bootstrap of one shard with the resident key; `bsk` is the key tensor whose broadcast is timed."""
    mg = eng.multi_gpu
    n_lwe, G, K = PBS_N_LWE, args.pbs_global, args.pbs_steps
    gloo = args.dist_backend == "gloo"  # rehearsal: gloo point-to-point needs host tensors
    tdev = torch.device("cpu") if gloo else dev
    a, b = mg.shard_bounds(G, world, rank)
    mine = b - a
    # key broadcast from the root (replicated read-only state)
    kb = bsk.to(tdev)
    barrier()
    t0 = time.perf_counter()
    mg.broadcast_(kb, src=0)
    torch.cuda.synchronize()
    barrier()
    bcast_s = mg.max_over_ranks(time.perf_counter() - t0, None if gloo else dev)
    del kb
    lwe_all = out_all = None
    if rank == 0:
        lwe_all = torch.empty((G, n_lwe + 1), dtype=torch.int64, device=dev)
        eng.fill_uniform(lwe_all, SEED + 50, 0)
        lwe_all = lwe_all.to(tdev)
        out_all = torch.empty((G, N + 1), dtype=torch.int64, device=tdev)
    shard_in = torch.empty((mine, n_lwe + 1), dtype=torch.int64, device=tdev)
    shard_out = torch.empty((mine, N + 1), dtype=torch.int64, device=dev)
    work_in = shard_in if not gloo else torch.empty((mine, n_lwe + 1), dtype=torch.int64, device=dev)

    def step(transfer):
        if transfer:
            mg.scatter_batch(lwe_all, shard_in, src=0)
            if gloo:
                work_in.copy_(shard_in)
        if mine:  # an empty shard (global batch < ranks) launches nothing
            pbs(work_in, shard_out)
        if transfer:
            mg.gather_batch(shard_out if not gloo else shard_out.cpu(), out_all, dst=0)

    step(True)
    torch.cuda.synchronize()
    times = {}
    for transfer in (False, True):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step(transfer)
        torch.cuda.synchronize()
        barrier()
        times[transfer] = mg.max_over_ranks(time.perf_counter() - t0, None if gloo else dev)
    return {"metric": "PBS/sec, one global batch sharded over the GPUs (config 5)",
            "value": G * K / times[False], "unit": "PBS/s", "scaling": "strong",
            "value_with_scatter_gather": G * K / times[True],
            "ms_per_step": times[False] / K * 1e3, "ms_per_step_with_scatter_gather": times[True] / K * 1e3,
            "steps": K,
            "key_broadcast_ms": bcast_s * 1e3,
            "config": {"global_batch": G, "n_gpus": world, "shard": [a, b],
                       "transfer": "gloo via host (rehearsal)" if gloo else
                                   "RCCL grouped send/recv from rank 0 (xGMI)",
                       "scatter_bytes": G * (n_lwe + 1) * 8, "gather_bytes": G * (N + 1) * 8}}


EXT_BYTES = 32768 + 65536  # in-GLWE read + out-GLWE read/modify/write per product


def bench_ext_product(args, eng, torch, dev, world, barrier, dist):
    """Config 3: batched GGSW x GLWE external product (BNF: native GLWEs, Raw NTT GGSW), l = 1, base 2^23."""
    M = eng.ntt64_pbs
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    batch = args.batch
    ggsw = torch.empty((1, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(ggsw, SEED + 30, SOLINAS_P)
    glwe = torch.empty((batch, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(glwe, SEED + 31, 0)
    out = torch.zeros((batch, 2, N), dtype=torch.int64, device=dev)
    # the GGSW is prepared once (mi_ntt64_ggsw_create: permuted into the bodies' read order), as a key is; the raw-pointer
    # form, which permutes it on every call, is timed beside it (raw_ggsw_per_call)
    prepared = M.NttGgswList(plan, ggsw, PBS_BASE_LOG, 1, M.BNF)
    torch.cuda.synchronize()
    run_raw = lambda: M.add_external_product_ntt64_bnf_assign(plan, out, ggsw, glwe, PBS_BASE_LOG, 1)
    K_raw, el_raw, kernel_ms_raw = timed_leg(run_raw, torch, barrier, dist, dev)
    run = lambda: M.add_external_product_ntt64_bnf_assign(plan, out, prepared, glwe, PBS_BASE_LOG, 1)
    K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev)
    hbm = EXT_BYTES * batch / (kernel_ms * 1e-3) / 1e9
    return {"metric": "GGSW x GLWE external products/sec (config 3)", "value": world * batch * K / el,
            "unit": "external products/s", "steps": K, "ms_per_step": el / K * 1e3, "kernel_ms": kernel_ms,
            "ntt_equivalents_per_s": world * batch * K / el * 4,
            "config": {"workload": "add_external_product_ntt64_bnf_assign, N=2048, k=1, level 1, base_log 23, "
                                   "prepared GGSW (NttGgswList)",
                       "batch_per_gpu": batch},
            "raw_ggsw_per_call": {"value": world * batch * K_raw / el_raw, "kernel_ms": kernel_ms_raw,
                                  "note": "the same products through the raw-pointer call (GGSW permuted per call)"},
            "algorithmic_bytes_per_unit": EXT_BYTES,
            "roofline": dict(valu_roofline(2, VALU_CYCLES["ext_bnf"], batch, kernel_ms,
                                           "bound by integer VALU issue (2 waves per product: decomposition, 2 fwd + "
                                           "2 inv twisted transforms, MAC, modulus switch)"),
                             hbm={"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm / HBM_PEAK_GBS,
                                  "algorithmic_bytes_per_launch": EXT_BYTES * batch}),
            "cpu_baseline": None}


def bench_ext_product_fft(args, eng, torch, dev, world, barrier, dist):
    """Config 3 on the default (f64-FFT) path: add_external_product_assign (fft64_pbs.rs:270-330) of a batch of
    native GLWEs (k = 1, N = 2048, l = 1, base 2^23) with one shared Fourier GGSW; the one-ciphertext workgroups of
    fft64_pbs.hip (2 waves per product).  Also the k = 2, level-2 shape on the same engine."""
    F = eng.fft64
    fft = F.Fft(N, dev.index)
    res = {}
    for k, level, base_log in ((1, 1, PBS_BASE_LOG), (2, 2, 12)):
        batch = args.batch
        std = torch.empty((level, k + 1, k + 1, N), dtype=torch.int64, device=dev)
        eng.fill_uniform(std, SEED + 33 + k, 0)
        fg = torch.empty((level, k + 1, k + 1, N // 2, 2), dtype=torch.float64, device=dev)
        F.convert_standard_lwe_bootstrap_key_to_fourier(std, fg, fft)
        glwe = torch.empty((batch, k + 1, N), dtype=torch.int64, device=dev)
        eng.fill_uniform(glwe, SEED + 35 + k, 0)
        out = torch.zeros((batch, k + 1, N), dtype=torch.int64, device=dev)
        run = lambda: F.add_external_product_assign(out, fg, glwe, base_log, level, fft)
        K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev)
        res[f"k{k}_l{level}"] = {"value": world * batch * K / el, "unit": "external products/s", "steps": K,
                                 "ms_per_step": el / K * 1e3, "kernel_ms": kernel_ms,
                                 "hbm_frac": (k + 1) * N * 8 * 3 * batch / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                 "config": {"k": k, "level": level, "base_log": base_log, "batch_per_gpu": batch}}
    out = res["k1_l1"]
    out.update({"metric": "GGSW x GLWE external products/sec, f64-FFT path (config 3 shape)", "dtype": "f64",
                "config": dict(out["config"], workload="add_external_product_assign (tfhe-fft path), N=2048"),
                "k2_l2": res["k2_l2"]})
    return out


def cpu_baseline_ext(seconds: float):
    """Oracle restatement of add_external_product_ntt64_bnf_assign (ntt64_bnf_pbs.rs:541-681) with the AVX-512
    transform restatement, OpenMP over a bounded batch of products."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    ctx = O.NttContext(N)
    sample = threads * 64
    ggsw = O.fill_uniform(SEED + 30, SOLINAS_P, 4 * N)
    glwe = O.fill_uniform(SEED + 31, 0, sample * 2 * N)
    out = O.fill_uniform(SEED + 32, 0, sample * 2 * N)
    O.pbs_set_fast_ntt(True)
    try:
        reps, t0 = 0, time.perf_counter()
        while True:
            ctx.ext_product_batch_bnf(out, ggsw, glwe, 1, PBS_BASE_LOG, 1, threads=threads)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        O.pbs_set_fast_ntt(False)
    return {"value": reps * sample / el, "unit": "external products/s", "cores": threads, "kind": "port",
            "sample": (f"{reps} x {sample} BNF external products (N=2048, k=1, l=1) in {el:.1f}s, restatement of "
                       f"ntt64_bnf_pbs.rs:541-681 with {'AVX-512' if O.have_avx512() else 'scalar'} transforms, "
                       f"OpenMP {threads} threads")}


def bench_bsk_conversion(args, eng, torch, dev, world, barrier, dist):
    """convert_standard_lwe_bootstrap_key_to_ntt64 (lwe_bootstrap_key_conversion.rs:294-365) of one whole
    PARAM_MESSAGE_2_CARRY_2 key per step: 918 GGSWs x (k+1)^2 x level = 3,672 polynomials, native 2^64
    input modswitched to p, forward NTT, Raw (BNF) output; standard and NTT keys resident in HBM."""
    M = eng.ntt64_pbs
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    shape = (PBS_N_LWE, PBS_LEVEL, 2, 2, N)
    std = torch.empty(shape, dtype=torch.int64, device=dev)
    eng.fill_uniform(std, SEED + 70, 0)
    ntt = torch.empty_like(std)
    run = lambda: M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, std, ntt, normalize=False)
    K, el, ms = timed_leg(run, torch, barrier, dist, dev)
    polys = std.numel() // N
    alg = polys * N * 16  # read the standard key, write the NTT key
    # two keys in flight: consecutive conversions alternate between the leg's stream and a second
    # one (the keys are independent), so one launch's 3,672 waves overlap the next one's instead of each launch
    # running as one partial generation of waves with a drain; wall-clock rate over >= 0.3 s
    side = torch.cuda.Stream(device=dev)
    std2, ntt2 = std.clone(), torch.empty_like(std)
    side.wait_stream(torch.cuda.current_stream(dev))

    def two():
        run()
        with torch.cuda.stream(side):
            M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, std2, ntt2, normalize=False)

    K2, el2, _ = timed_leg(two, torch, barrier, dist, dev)
    two_rate = world * 2 * K2 / el2
    del std2, ntt2
    return {"metric": "bootstrap keys converted to the NTT domain per second", "value": world * K / el,
            "unit": "keys/s", "ms_per_step": el / K * 1e3, "kernel_ms": ms, "steps": K,
            "polys_per_key": polys, "ntt_per_s": world * K * polys / el,
            "two_streams": {"value": two_rate, "unit": "keys/s", "steps": K2,
                            "hbm_frac_wall": alg * two_rate / world / 1e9 / HBM_PEAK_GBS,
                            "note": "two independent keys in flight on two streams; wall-clock rate (includes the "
                                    "gaps), HBM fraction of the algorithmic bytes at that rate"},
            "config": {"workload": "convert_standard_lwe_bootstrap_key_to_ntt64, native 2^64 -> p, Raw, "
                                   "n=918 k=1 N=2048 level=1 (PARAM_MESSAGE_2_CARRY_2)", "batch_per_gpu": 1},
            "roofline": {"bound": "hbm", "achieved": alg / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": alg}}


def cpu_baseline_bsk(seconds: float):
    """Oracle restatement of the sequential conversion (one thread, as the reference's non-par function),
    with the AVX-512 transform restatement where the host has it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    ctx = O.NttContext(N)
    polys = PBS_N_LWE * PBS_LEVEL * 4
    O.pbs_set_fast_ntt(True)
    try:
        std = O.fill_uniform(SEED + 70, 0, polys * N)
        reps, t0 = 0, time.perf_counter()
        while True:
            ctx.bsk_to_ntt(std, 64, False)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        O.pbs_set_fast_ntt(False)
    return {"value": reps / el, "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": f"{reps} whole keys ({polys} polys) in {el:.1f}s, restatement of "
                      f"convert_standard_lwe_bootstrap_key_to_ntt64 "
                      f"({'AVX-512' if O.have_avx512() else 'scalar'} transforms), 1 thread"}


# the other plans of SURVEY.md 8 a13 / f3: the largest primes = 1 mod 2^16 below 2^62 and 2^64
# (largest_prime_in_arithmetic_progression64, prime.rs:130-; the GPU tests' p62 / p64) and a prime32 NTT prime
P62, P64G, P30 = 0x3FFFFFFFFFFF0001, 0xFFFFFFFFFFE40001, 1062862849


def bench_plans(args, eng, torch, dev, world, barrier, dist):
    """Rates of the other SURVEY.md 8 rows at config 2's shape (N = 2048, inputs resident), each over >= 0.3 s of GPU
    work with the HBM fraction of its algorithmic bytes: a7 the core_crypto Ntt64View pair forward_from_decomp +
    add_backward_on_power_of_two_modulus(64) (ntt64.rs:221-266, conversions fused into the twisted bodies), a4
    mul_accumulate (prime64.rs:1182-1222), a13 fwd + inv over generic 62- / 64-bit primes (Montgomery window kernels)
    and prime32 (prime32.rs:632-1025), f3 the native64 CRT negacyclic product (native64.rs:929-1160)."""
    B = args.batch
    out = {"metric": "other plans and the Ntt64View layer at N = 2048 (SURVEY.md 8 a4 / a7 / a13 / f3)"}

    def leg(name, run, units, unit, nbytes, workload):
        K, el, ms = timed_leg(run, torch, barrier, dist, dev)
        achieved = nbytes / (ms * 1e-3) / 1e9
        out[name] = {"value": world * units * K / el, "unit": unit, "ms_per_step": el / K * 1e3, "kernel_ms": ms,
                     "steps": K, "config": {"workload": workload, "batch_per_gpu": units},
                     "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes": nbytes}}

    poly = N * 8
    view = eng.ntt64.Ntt64(SOLINAS_P, N, dev.index).as_view()
    dec = torch.empty((B, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(dec, SEED + 80, 1 << 23)
    dec -= 1 << 22  # signed digits in [-2^22, 2^22)
    ntt, std = torch.empty_like(dec), torch.empty_like(dec)
    eng.fill_uniform(std, SEED + 81, 0)

    def view_step():
        view.forward_from_decomp(ntt, dec)
        view.add_backward_on_power_of_two_modulus(64, std, ntt)

    leg("ntt64_view", view_step, B, "fwd+add_backward pairs/s", B * poly * 6,
        "Ntt64View forward_from_decomp then add_backward_on_power_of_two_modulus(64), Solinas N=2048")
    del dec, ntt, std
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    acc, a, b = (torch.empty((B, N), dtype=torch.int64, device=dev) for _ in range(3))
    for i, t in enumerate((acc, a, b)):
        eng.fill_uniform(t, SEED + 82 + i, SOLINAS_P)
    leg("mul_accumulate", lambda: plan.mul_accumulate(acc, a, b), B, "polys/s", B * poly * 4,
        "Plan::mul_accumulate acc += a b mod p, Solinas N=2048")
    del acc, a, b
    for name, p in (("prime64_p62", P62), ("prime64_p64", P64G)):
        gp = eng.Plan.try_new(N, p, device=dev.index)
        buf = torch.empty((B, N), dtype=torch.int64, device=dev)
        eng.fill_uniform(buf, SEED + 85, p)

        def pair(gp=gp, buf=buf):
            gp.fwd(buf)
            gp.inv(buf)

        leg(name, pair, B, "fwd+inv NTT pairs/s", B * poly * 4, f"prime64 Plan fwd then inv, N=2048, p={p:#x}")
        del buf
    p32 = eng.prime32.Plan.try_new(N, P30, device=dev.index)
    b32 = torch.empty((B, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(b32, SEED + 86, P30)
    b32 = b32.to(torch.int32)

    def pair32():
        p32.fwd(b32)
        p32.inv(b32)

    leg("prime32", pair32, B, "fwd+inv NTT pairs/s", B * N * 4 * 4, f"prime32 Plan fwd then inv, N=2048, p={P30}")
    del b32
    nb = B // 8
    nplan = eng.native64.Plan32.try_new(N, dev.index)
    prod, lhs, rhs = (torch.empty((nb, N), dtype=torch.int64, device=dev) for _ in range(3))
    eng.fill_uniform(lhs, SEED + 87, 0)
    eng.fill_uniform(rhs, SEED + 88, 0)
    leg("native64_polymul", lambda: nplan.negacyclic_polymul(prod, lhs, rhs), nb, "products/s", nb * poly * 3,
        "native64::Plan32 negacyclic_polymul mod 2^64 (CRT over 32-bit primes), N=2048")
    return out


KS_IN, KS_BASE_LOG, KS_LEVEL = 2048, 4, 4  # PARAM_MESSAGE_2_CARRY_2 keyswitch (ks_pbs.rs:38-39): k*N -> n
I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: i8 MFMA = 2x the dense bf16 rate (~2.5 PF)


def bench_keyswitch(args, eng, torch, dev, world, barrier, dist):
    """The keyswitch in front of the PBS (shortint KS-PBS order): batched 2048 -> 918 LWE keyswitch,
    base 2^4, 4 levels, on the int8 matrix cores; key and inputs resident."""
    KS = eng.lwe_keyswitch
    batch = args.pbs_batch
    ksk = torch.empty((KS_IN, KS_LEVEL, PBS_N_LWE + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(ksk, SEED + 40, 0)
    key = KS.LweKeyswitchKey(ksk, KS_BASE_LOG, KS_LEVEL)
    del ksk
    lwe = torch.empty((batch, KS_IN + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 41, 0)
    out = torch.empty((batch, PBS_N_LWE + 1), dtype=torch.int64, device=dev)
    run = lambda: KS.keyswitch_lwe_ciphertext(key, lwe, out)
    K, el, ms = timed_leg(run, torch, barrier, dist, dev)
    # int8 MACs the matrix cores execute: 8 recoded byte planes x (out_dim + 1) columns x in_dim*level digits
    ops = 2.0 * batch * 8 * (PBS_N_LWE + 1) * KS_IN * KS_LEVEL
    frac = ops / (ms * 1e-3) / 1e12 / I8_PEAK_TOPS
    return {"metric": "LWE keyswitches/sec (KS of KS-PBS)", "value": world * batch * K / el, "unit": "KS/s",
            "steps": K, "ms_per_step": el / K * 1e3, "kernel_ms": ms,
            "config": {"workload": "keyswitch_lwe_ciphertext 2048 -> 918, base_log 4, level 4, native modulus",
                       "batch_per_gpu": batch},
            "roofline": {"bound": "mfma", "achieved": ops / (ms * 1e-3) / 1e12, "peak": I8_PEAK_TOPS,
                         "unit": "TOP/s", "frac": frac,
                         # one useful u64 MAC is 8 i8 plane MACs: the useful-work fraction is 1/8 of the utilisation
                         "useful_u64_frac": frac / 8,
                         "note": "digit pass + i8 MFMA GEMM per step; `frac` counts all 8 recoded byte-plane MACs per "
                                 "u64 MAC (matrix-core utilisation), `useful_u64_frac` counts each u64 MAC once"}}


def bench_ks_pbs(args, eng, torch, dev, world, barrier, dist):
    """The shortint KS-PBS order end to end on one stream: big LWE (k N + 1 = 2049) -> keyswitch
    (2048 -> 918, B 2^4, 4 levels) -> BNF PBS (n = 918) -> big LWE, both keys resident."""
    KS, M = eng.lwe_keyswitch, eng.ntt64_pbs
    batch, n_lwe = args.pbs_batch, PBS_N_LWE
    ksk = torch.empty((KS_IN, KS_LEVEL, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(ksk, SEED + 40, 0)
    kkey = KS.LweKeyswitchKey(ksk, KS_BASE_LOG, KS_LEVEL)
    del ksk
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    bsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(bsk, SEED + 10, SOLINAS_P)
    bkey = M.NttBootstrapKey(plan, bsk, PBS_BASE_LOG, PBS_LEVEL, M.BNF)
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 11, 0)
    big = torch.empty((batch, KS_IN + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(big, SEED + 42, 0)
    small = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)

    def run():
        KS.keyswitch_lwe_ciphertext(kkey, big, small)
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(small, out, lut, bkey)

    K, el, _ = timed_leg(run, torch, barrier, dist, dev)
    del bkey, kkey
    return {"metric": "KS-PBS/sec (keyswitch then PBS, PARAM_MESSAGE_2_CARRY_2 shape)",
            "value": world * batch * K / el, "unit": "KS-PBS/s", "ms_per_step": el / K * 1e3, "steps": K,
            "config": {"workload": "keyswitch_lwe_ciphertext 2048 -> 918 (B 2^4, L 4) then "
                                   "programmable_bootstrap_ntt64_bnf (n 918, N 2048, B 2^23, L 1), one stream",
                       "batch_per_gpu": batch}}


KS32_IN, KS32_N_LWE, KS32_BASE_LOG, KS32_LEVEL, KS32_MOD_LOG = 2048, 879, 2, 8, 21


def bench_ks32_pbs(args, eng, torch, dev, world, barrier, dist):
    """The HPU KS32 bootstrap at V1_5_HPU_PARAM_MESSAGE_2_CARRY_2_KS32_PBS_TUNIFORM_2M128 (shortint/parameters/v1_5/
    hpu.rs:57-76), the parameter set of BASELINE.md's one NTT-PBS figure (HPU, 14,167 KS-PBS/s): keyswitch with a scalar
    change (2048 -> 879, base 2^2, 8 levels, u32 output of modulus 2^21), the centered binary modulus switch of the u32
    LWE to 2N, and the NTT BNF bootstrap (n 879, N 2048, base 2^23, level 1) on the switched input — the order of the
    HPU mockup (mockups/tfhe-hpu-mockup/src/lib.rs:720-761, one LUT); both keys resident, one stream."""
    KS, M = eng.lwe_keyswitch, eng.ntt64_pbs
    batch, n_lwe = args.pbs_batch, KS32_N_LWE
    ksk = torch.empty((KS32_IN, KS32_LEVEL, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(ksk, SEED + 70, 0)
    ksk32 = (ksk & ((1 << 32) - 1)).to(torch.int32)  # u32 key words (their low 11 bits need not be 0 for timing)
    del ksk
    kkey = KS.LweKeyswitchKey32(ksk32, KS32_BASE_LOG, KS32_LEVEL, KS32_MOD_LOG)
    del ksk32
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    bsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(bsk, SEED + 71, SOLINAS_P)
    bkey = M.NttBootstrapKey(plan, bsk, PBS_BASE_LOG, PBS_LEVEL, M.BNF)
    del bsk
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 72, 0)
    big = torch.empty((batch, KS32_IN + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(big, SEED + 73, 0)
    small = torch.empty((batch, n_lwe + 1), dtype=torch.int32, device=dev)
    switched = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)
    log2n = (2 * N).bit_length() - 1

    def run_ks():
        KS.keyswitch_lwe_ciphertext_with_scalar_change(kkey, big, small)
        KS.lwe_ciphertext_centered_binary_modulus_switch32(small, switched, log2n)

    def run():
        run_ks()
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(switched, out, lut, bkey, M.MS_PRE_SWITCHED)

    K, el, kernel_ms = timed_leg(run, torch, barrier, dist, dev)
    K_ks, el_ks, ks_ms = timed_leg(run_ks, torch, barrier, dist, dev)
    del bkey, kkey
    return {"metric": "KS-PBS/sec, HPU KS32 parameters (V1_5_HPU_PARAM_MESSAGE_2_CARRY_2_KS32_PBS_TUNIFORM_2M128)",
            "value": world * batch * K / el, "unit": "KS-PBS/s", "ms_per_step": el / K * 1e3, "steps": K,
            "kernel_ms": kernel_ms,
            "ntt_equivalents_per_s": world * batch * K / el * 4 * n_lwe,
            "keyswitch_and_switch": {"value": world * batch * K_ks / el_ks, "unit": "KS/s", "kernel_ms": ks_ms,
                                     "steps": K_ks},
            "vs_hpu_published": {"value": 14167.0, "unit": "KS-PBS/s",
                                 "source": "BASELINE.md: AMD Alveo V80 HPU, batch 12 (hpu-programmable-bootstrapping.md)"},
            "config": {"workload": "keyswitch_lwe_ciphertext_with_scalar_change 2048 -> 879 (B 2^2, L 8, u32 mod 2^21) "
                                   "-> lwe_ciphertext_centered_binary_modulus_switch (u32, 2N) -> NTT BNF PBS "
                                   "(n 879, N 2048, B 2^23, L 1) on the switched input, one stream",
                       "batch_per_gpu": batch}}


def bench_ks_pbs_fft(args, eng, torch, dev, world, barrier, dist):
    """The shortint server key's KS-PBS as tfhe-rs runs it by default: keyswitch (2048 -> 918, B 2^4, L 4) then the
    f64-FFT PBS (n 918, N 2048, B 2^23, L 1), both keys resident, one stream."""
    KS, F = eng.lwe_keyswitch, eng.fft64
    batch, n_lwe = args.pbs_batch, PBS_N_LWE
    ksk = torch.empty((KS_IN, KS_LEVEL, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(ksk, SEED + 40, 0)
    kkey = KS.LweKeyswitchKey(ksk, KS_BASE_LOG, KS_LEVEL)
    del ksk
    fft = F.Fft(N, dev.index)
    std = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(std, SEED + 80, 0)
    fbsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N // 2, 2), dtype=torch.float64, device=dev)
    F.convert_standard_lwe_bootstrap_key_to_fourier(std, fbsk, fft)
    del std
    bkey = F.FourierLweBootstrapKey(fbsk, PBS_BASE_LOG, PBS_LEVEL, fft)
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 11, 0)
    big = torch.empty((batch, KS_IN + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(big, SEED + 42, 0)
    small = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)

    def run():
        KS.keyswitch_lwe_ciphertext(kkey, big, small)
        F.programmable_bootstrap_lwe_ciphertext(small, out, lut, bkey)

    K, el, _ = timed_leg(run, torch, barrier, dist, dev)
    del bkey, kkey
    return {"metric": "KS-PBS/sec, default shortint path (keyswitch then f64-FFT PBS), PARAM_MESSAGE_2_CARRY_2 shape",
            "value": world * batch * K / el, "unit": "KS-PBS/s", "ms_per_step": el / K * 1e3, "steps": K,
            "config": {"workload": "keyswitch_lwe_ciphertext 2048 -> 918 (B 2^4, L 4) then "
                                   "programmable_bootstrap_lwe_ciphertext (f64 FFT; n 918, N 2048, B 2^23, L 1), one stream",
                       "batch_per_gpu": batch}}


def cpu_baseline_ks(seconds: float):
    """Oracle restatement of keyswitch_lwe_ciphertext_native_mod_compatible, OpenMP over ciphertexts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    ksk = O.fill_uniform(SEED + 40, 0, KS_IN * KS_LEVEL * (PBS_N_LWE + 1))
    sample = threads * 4
    lwe = O.fill_uniform(SEED + 41, 0, sample * (KS_IN + 1)).reshape(sample, KS_IN + 1)
    reps, t0 = 0, time.perf_counter()
    while True:
        O.lwe_keyswitch(ksk, lwe, PBS_N_LWE, KS_BASE_LOG, KS_LEVEL, threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": reps * sample / el, "unit": "KS/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {sample} keyswitches 2048 -> 918 (B 2^4, L 4) in {el:.1f}s, restatement of "
                      f"lwe_keyswitch.rs:137-227, OpenMP {threads} threads"}


def bench_default_stream(eng, torch, dev, work):
    """the entry points that take device scratch (the Solinas PBS's modulus-switch pre-pass, the keyswitch
    digits, the shape-generic f64 engine) called on torch's default stream — the legacy null stream — against the
    same calls on a created stream.  Small batches, so the per-call host cost shows: `enqueue_us` is the host time
    per call with the calls back to back (a host-blocking sync inside a call would show here), `us_per_call` the
    time per call to the final synchronize.  Before r4 every null-stream call synchronised and freed its scratch."""
    M, KS, F = eng.ntt64_pbs, eng.lwe_keyswitch, eng.fft64
    batch, n_lwe, R = 4, PBS_N_LWE, 200
    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    bsk = torch.empty((n_lwe, PBS_LEVEL, 2, 2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(bsk, SEED + 90, SOLINAS_P)
    skey = M.NttBootstrapKey(plan, bsk, PBS_BASE_LOG, PBS_LEVEL, M.SOLINAS)
    del bsk
    lut = torch.empty((2, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(lut, SEED + 91, SOLINAS_P)
    lwe = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, SEED + 92, SOLINAS_P)
    out = torch.empty((batch, N + 1), dtype=torch.int64, device=dev)
    ksk = torch.empty((KS_IN, KS_LEVEL, n_lwe + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(ksk, SEED + 93, 0)
    kkey = KS.LweKeyswitchKey(ksk, KS_BASE_LOG, KS_LEVEL)
    del ksk
    big = torch.empty((batch, KS_IN + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(big, SEED + 94, 0)
    small = torch.empty((batch, n_lwe + 1), dtype=torch.int64, device=dev)
    n_g, nl_g = 1024, 64  # the shape-generic f64 engine (N != 2048)
    fft = F.Fft(n_g, dev.index)
    std = torch.empty((nl_g, 2, 2, 2, n_g), dtype=torch.int64, device=dev)
    eng.fill_uniform(std, SEED + 95, 0)
    fbsk = torch.empty((nl_g, 2, 2, 2, n_g // 2, 2), dtype=torch.float64, device=dev)
    F.convert_standard_lwe_bootstrap_key_to_fourier(std, fbsk, fft)
    del std
    fkey = F.FourierLweBootstrapKey(fbsk, 12, 2, fft)
    flut = torch.empty((2, n_g), dtype=torch.int64, device=dev)
    eng.fill_uniform(flut, SEED + 96, 0)
    flwe = torch.empty((batch, nl_g + 1), dtype=torch.int64, device=dev)
    eng.fill_uniform(flwe, SEED + 97, 0)
    fout = torch.empty((batch, n_g + 1), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    cases = {
        "pbs_solinas_n2048": lambda: M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(lwe, out, lut, skey),
        "keyswitch_2048_to_918": lambda: KS.keyswitch_lwe_ciphertext(kkey, big, small),
        "pbs_fft_generic_n1024": lambda: F.programmable_bootstrap_lwe_ciphertext(flwe, fout, flut, fkey),
    }
    rows = {}
    for name, run in cases.items():
        row = {}
        for sname, stream in (("default_stream", torch.cuda.default_stream(dev)), ("created_stream", work)):
            with torch.cuda.stream(stream):
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(R):
                    run()
                t_enq = time.perf_counter() - t0
                torch.cuda.synchronize()
                t_all = time.perf_counter() - t0
            row[sname] = {"enqueue_us": t_enq / R * 1e6, "us_per_call": t_all / R * 1e6}
        rows[name] = row
    del skey, kkey, fkey
    return {"note": f"{R} back-to-back calls at batch {batch} per case and stream (null stream = torch's default)",
            "cases": rows}


def bench_host_path(eng, torch):
    """Config 1 plumbing and VERDICT r2 item 6: the per-polynomial host form of Plan::fwd + Plan::inv
    (`mi_ntt64_fwd_host` / `_inv_host`: copy in, transform, copy out on a pooled private stream, the drop-in for
    Ntt64View::forward / add_backward, ntt64.rs:89-137) against the oracle's CPU transform of the same
    polynomials: latency at batch 1 for N = 1024 / 2048, and the crossover batch from which one host call beats
    the CPU (1 thread, as the reference's per-call transform, and all cores).  Host buffers, PCIe-inclusive: never
    the headline `value`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    avx = O.have_avx512()

    def best(fn, reps):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2]

    res = {"unit": "us per fwd+inv call pair (median)", "cpu_kind": ("AVX-512" if avx else "scalar") + " restatement",
           "cpu_threads_all": threads, "sizes": {}}
    for n in (1024, 2048):
        plan = eng.Plan.try_new(n, SOLINAS_P)
        ora = O.Plan.try_new(n, SOLINAS_P)
        fwd = ora.fwd_avx512_inplace if avx else ora.fwd_scalar_inplace
        inv = ora.inv_avx512_inplace if avx else ora.inv_scalar_inplace
        rows, cross1, crossall = [], None, None
        for batch in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024):
            x = O.fill_uniform(SEED + batch, SOLINAS_P, batch * n).reshape(batch, n)
            ref = ora.inv(ora.fwd(x))
            y = x.copy()
            plan.fwd(y)
            plan.inv(y)
            assert np.array_equal(y, ref), "host path mismatch vs oracle"
            reps = 50 if batch <= 64 else 10

            def gpu():
                plan.fwd(y)
                plan.inv(y)

            g = best(gpu, reps) * 1e6
            c1 = best(lambda: (fwd(y, 1), inv(y, 1)), reps) * 1e6
            ca = best(lambda: (fwd(y, threads), inv(y, threads)), reps) * 1e6
            rows.append({"batch": batch, "gpu_host_us": g, "cpu_1t_us": c1, "cpu_all_us": ca})
            if cross1 is None and g < c1:
                cross1 = batch
            if crossall is None and g < ca:
                crossall = batch
        res["sizes"][str(n)] = {"rows": rows, "crossover_batch_vs_cpu_1t": cross1,
                                "crossover_batch_vs_cpu_all_cores": crossall,
                                "single_poly_gpu_us": rows[0]["gpu_host_us"], "single_poly_cpu_1t_us": rows[0]["cpu_1t_us"]}
    return res


def load_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/*/pmc_traffic.json)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def relaunch_distributed(n: int) -> int:
    """One process per GPU: run this script under torch.distributed.run with N ranks (a child process;
    this process has not touched the GPU) and return its exit status."""
    import socket
    import subprocess

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    import torch
    import tfhe_ntt_amd as eng

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(0 if args.same_device else local)
        dist.init_process_group(backend=args.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    global SIMDS
    SIMDS = torch.cuda.get_device_properties(dev).multi_processor_count * 4
    # every leg runs on a dedicated stream: on the legacy default stream each dependent launch costs
    # ~5 us more (tools/graph_probe.py: 150 vs ~160 us per fwd+inv step)
    work = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(work)

    plan = eng.Plan.try_new(N, SOLINAS_P, device=dev.index)
    batch = args.batch
    buf = torch.empty((batch, N), dtype=torch.int64, device=dev)
    eng.fill_uniform(buf, SEED + rank * 0x1000, SOLINAS_P)  # inputs resident in HBM before timing
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    K = args.steps

    def headline(K, W):
        """W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier + synchronize; HIP events on the
        launching stream (`work`, torch's current stream, which the plan launches on) bracket the timed region:
        their interval / (2 K) is the average duration of the 2 K timed launches, gaps included."""
        for _ in range(W):
            plan.fwd(buf)
            plan.inv(buf)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(work)
        for _ in range(K):
            plan.fwd(buf)
            plan.inv(buf)
        ev1.record(work)
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        if dist is not None:
            elapsed = eng.multi_gpu.max_over_ranks(elapsed, dev)
        return elapsed, ev0.elapsed_time(ev1) / (2 * K)

    bytes_launch = batch * BYTES_PER_POLY_PASS
    # Cold start: the K steps straight from an idle GPU, before any other work (the engine clock is still ramping:
    # reported, not the headline).  The component legs then keep the GPU busy for several seconds, and the headline
    # below is the same W + K steps at the clock the chip holds under sustained load.
    cold_el, cold_launch = headline(K, args.warmup)
    cold = {"value": world * batch * K / cold_el, "ms_per_step": cold_el / K * 1e3, "timed_launch_ms": cold_launch,
            "roofline_frac": bytes_launch / (cold_launch * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": "the same W + K steps measured first, from an idle GPU, before any leg ran"}
    legs = {}
    if not args.no_pbs:
        if not args.no_shapes:
            legs["pbs_shapes"] = {name: bench_pbs_shape(name, args, eng, torch, dev, world, barrier, dist)
                                  for name in SHAPE_LEGS}
        legs["pbs"] = bench_pbs(args, eng, torch, dev, rank, world, barrier, dist)
        legs["pbs_solinas"] = bench_pbs_solinas(args, eng, torch, dev, world, barrier, dist)
        legs["pbs_fft"] = bench_pbs_fft(args, eng, torch, dev, rank, world, barrier, dist)
        if not args.no_shapes:
            legs["pbs_shapes_fft"] = {name: bench_pbs_shape_fft(name, args, eng, torch, dev, world, barrier, dist)
                                      for name in SHAPE_LEGS}
        legs["keyswitch"] = bench_keyswitch(args, eng, torch, dev, world, barrier, dist)
        legs["ks_pbs"] = bench_ks_pbs(args, eng, torch, dev, world, barrier, dist)
        legs["ks32_pbs"] = bench_ks32_pbs(args, eng, torch, dev, world, barrier, dist)
        legs["ks_pbs_fft"] = bench_ks_pbs_fft(args, eng, torch, dev, world, barrier, dist)
        legs["ext_product_fft"] = bench_ext_product_fft(args, eng, torch, dev, world, barrier, dist)
        legs["bsk_conversion"] = bench_bsk_conversion(args, eng, torch, dev, world, barrier, dist)
        legs["plans"] = bench_plans(args, eng, torch, dev, world, barrier, dist)
        # last before the headline: the external product, an integer-VALU load like the transform's, so the headline
        # always follows the same kind of work (the held clock depends on what ran just before)
        legs["ext_product"] = bench_ext_product(args, eng, torch, dev, world, barrier, dist)

    elapsed, launch_ms = headline(K, args.warmup)

    # steady state: a time-based loop of >= --steady-seconds after the timed region (same stream, same buffer)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ss_k = max(1, int(args.steady_seconds / max(2 * launch_ms * 1e-3, 1e-6)))
    if dist is not None:
        ss_k = int(eng.multi_gpu.max_over_ranks(float(ss_k), dev))
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(work)
    for _ in range(ss_k):
        plan.fwd(buf)
        plan.inv(buf)
    e1.record(work)
    torch.cuda.synchronize()
    barrier()
    ss_el = time.perf_counter() - t0
    if dist is not None:
        ss_el = eng.multi_gpu.max_over_ranks(ss_el, dev)
    ss_launch = e0.elapsed_time(e1) / (2 * ss_k)
    steady = {"value": world * batch * ss_k / ss_el, "steps": ss_k, "seconds": ss_el, "timed_launch_ms": ss_launch,
              "roofline_frac": bytes_launch / (ss_launch * 1e-3) / 1e9 / HBM_PEAK_GBS,
              "note": "fwd+inv loop of >= --steady-seconds right after the timed region"}

    # per-direction split (informational), from a separate loop of back-to-back launches of one kernel;
    # the roofline below uses the timed launches
    split_k = min(K, 500)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(work)
    for k in range(split_k):
        plan.fwd(buf)
    e1.record(work)
    for k in range(split_k):
        plan.inv(buf)
    e2.record(work)
    torch.cuda.synchronize()
    fwd_ms = e0.elapsed_time(e1) / split_k
    inv_ms = e1.elapsed_time(e2) / split_k
    achieved = bytes_launch / (launch_ms * 1e-3) / 1e9

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
            "order": "cold_start (W + K steps from idle) -> component legs (external product last) -> headline "
                     "(W + K steps) -> steady_state",
            "hip_runtime": eng._lib.hip_runtimes(),
            "build": eng._lib.build_provenance(),
        },
        "kernels": {"timed_launch_ms": launch_ms, "fwd_ms": fwd_ms, "inv_ms": inv_ms,
                    "note": "timed_launch_ms: HIP events around the timed region / (2 K launches); "
                            f"fwd_ms / inv_ms: {split_k} back-to-back launches of one direction after it"},
        # the binding limit: integer VALU issue (SIMD cycles per launch at the peak clock vs measured)
        "valu_bound": {
            kind: {"issue_cycles_per_poly": VALU_CYCLES[kind],
                   "model_ms": batch * VALU_CYCLES[kind] / SIMDS / PEAK_CLOCK_HZ * 1e3,
                   "measured_ms": ms,
                   "frac": batch * VALU_CYCLES[kind] / SIMDS / PEAK_CLOCK_HZ * 1e3 / ms}
            for kind, ms in (("fwd", fwd_ms), ("inv", inv_ms))},
        "roofline": {
            "bound": "hbm",
            "kernel": "ntt_tw_body_kernel fwd / inv (average over the 2 K timed launches)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": load_traffic(),
            "traffic_source": "constant: PMC FETCH_SIZE + WRITE_SIZE per launch from the committed rocprofv3 passes "
                              "(profiles/pmc_traffic.json), not measured in this run",
            "algorithmic_bytes_per_launch": bytes_launch,
        },
        "cpu_baseline": None,
        "cold_start": cold,
        "steady_state": steady,
    }
    if rank == 0 and world == 1:
        out["host_path"] = bench_host_path(eng, torch)
        if not args.no_pbs and not args.no_shapes:  # (it runs the shape-generic f64 engine, as the shape legs do)
            out["default_stream"] = bench_default_stream(eng, torch, dev, work)
    # the driver keeps only the tail of stdout: the bulky legs first, configs 3 and 4 (external product, PBS) last
    for name in LEG_ORDER:
        if name in legs:
            out[name] = legs[name]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        if not args.no_pbs:
            out["ext_product"]["cpu_baseline"] = cpu_baseline_ext(min(args.cpu_seconds, 4.0))
            out["pbs"]["cpu_baseline"] = cpu_baseline_pbs(min(args.cpu_seconds, 8.0))
            out["pbs_solinas"]["cpu_baseline"] = cpu_baseline_pbs_solinas(min(args.cpu_seconds, 6.0))
            out["keyswitch"]["cpu_baseline"] = cpu_baseline_ks(min(args.cpu_seconds, 4.0))
            out["bsk_conversion"]["cpu_baseline"] = cpu_baseline_bsk(min(args.cpu_seconds, 3.0))
            for name in ("message_1_carry_1", "message_3_carry_3") if not args.no_shapes else ():
                # (4_4: ~0.1 s per CMUX step per core, unbounded)
                out["pbs_shapes"][name]["cpu_baseline"] = cpu_baseline_pbs_shape(name, min(args.cpu_seconds, 4.0))
            # the f64 legs' CPU figure is a single-thread numpy restatement, not comparable with the reference's
            # AVX-512 tfhe-fft: reported under its own key, never as `cpu_baseline`
            out["pbs_fft"]["cpu_numpy_restatement"] = cpu_baseline_pbs_fft(N, 1, PBS_N_LWE, PBS_BASE_LOG, PBS_LEVEL,
                                                                           min(args.cpu_seconds, 3.0))
            for name, (n_, k_, nl_, bl_, lv_, _) in (SHAPE_LEGS.items() if not args.no_shapes else ()):
                out["pbs_shapes_fft"][name]["cpu_numpy_restatement"] = cpu_baseline_pbs_fft(
                    n_, k_, nl_, bl_, lv_, min(args.cpu_seconds, 3.0))
    if rank == 0:
        full_path = write_full_record(out)
        # the driver parses the LAST stdout line and keeps only the tail: one compact line (<= LINE_MAX_BYTES)
        print(json.dumps(compact_line(out, full_path)), flush=True)
    if dist is not None:
        dist.destroy_process_group()


LINE_MAX_BYTES = 12 * 1024  # the parsed line must fit the driver's captured tail
FULL_RECORD = os.path.join("gpurun_out", "bench_full.json")


def write_full_record(out):
    """The whole record (host path, default-stream, per-shape legs, CPU baselines of every leg) goes to a file, not
    stdout. Returns the path written, or None when the tree is read-only."""
    path = os.path.join(ROOT, FULL_RECORD)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return FULL_RECORD
    except OSError as e:
        print(f"bench.py: full record not written ({e})", file=sys.stderr)
        return None


def compact_line(out, full_path=None):
    """The one JSON line the driver parses: the contract's keys, the headline's roofline and CPU baseline, and one
    short row per leg. Everything else stays in the full record."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: out.get(k) for k in keep}
    cfg = out.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "n", "batch_per_gpu", "global_batch", "parallelism") if k in cfg}
    build = cfg.get("build") or {}
    if build:
        line["config"]["source_sha16"] = (build.get("so_source_hash") or "")[:16]
        line["config"]["build_matches_tree"] = build.get("match")
    roof = out.get("roofline") or {}
    line["roofline"] = {k: roof.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                "traffic_source", "algorithmic_bytes_per_launch", "kernel")}
    line["cpu_baseline"] = out.get("cpu_baseline")
    kern = out.get("kernels") or {}
    line["kernels"] = {k: kern.get(k) for k in ("timed_launch_ms", "fwd_ms", "inv_ms")}
    line["valu_bound_frac"] = {k: v.get("frac") for k, v in (out.get("valu_bound") or {}).items()}
    # the sustained rate beside the K-step burst: the >= 1 s loop right after the timed region, and
    # the same K steps from an idle GPU
    for key in ("steady_state", "cold_start"):
        d = out.get(key) or {}
        if d:
            line[key] = {k: d.get(k) for k in ("value", "roofline_frac", "seconds", "steps") if d.get(k) is not None}
    line["legs_summary"] = legs_summary(out)
    line["full_record"] = full_path
    return line


def legs_summary(out):
    """One compact row per leg: value, unit, ms_per_step, steps, roofline frac + bound, CPU baseline value, and for
    the NTT-built legs `alg_frac` = the leg's NTT-equivalents/s over the standalone transform's single-transform
    rate (2 x the headline pairs/s), the algorithmic view beside the VALU-model `frac`."""
    rows = {}
    single_rate = 2.0 * out["value"] if out.get("value") else None

    def row(d):
        roof = d.get("roofline") or {}
        r = {"value": d.get("value"), "unit": d.get("unit"), "ms_per_step": d.get("ms_per_step"),
             "steps": d.get("steps"), "frac": roof.get("frac"), "bound": roof.get("bound")}
        cpu = d.get("cpu_baseline") or {}
        if cpu.get("value") is not None:
            r["cpu"] = cpu["value"]
        if d.get("ntt_equivalents_per_s") and single_rate:
            r["alg_frac"] = d["ntt_equivalents_per_s"] / single_rate
        return {k: v for k, v in r.items() if v is not None}

    for name in LEG_ORDER:
        d = out.get(name)
        if not isinstance(d, dict):
            continue
        if "value" in d:
            rows[name] = row(d)
        # nested legs with their own value: the shape legs' entries, and config 5 under pbs.sharded / pbs_fft.sharded
        # (N > 1 ranks) with and without the scatter / gather transfers
        for k, v in d.items():
            if isinstance(v, dict) and "value" in v:
                r = row(v)
                for extra in ("value_with_scatter_gather", "ms_per_step_with_scatter_gather", "scaling"):
                    if v.get(extra) is not None:
                        r[extra] = v[extra]
                rows[f"{name}.{k}"] = r
    return rows


if __name__ == "__main__":
    main()
