"""Eager vs hipGraph-replayed fwd+inv steps (N = 2048, batch 8192): how much of a step is the
dependent-launch gap.  python tools/graph_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-main_modified_amd"))
import torch  # noqa: E402
import tfhe_ntt_amd as eng  # noqa: E402

N, B, K = 2048, 8192, 200
plan = eng.Plan.try_new(N, eng.SOLINAS_P)
buf = torch.empty((B, N), dtype=torch.int64, device="cuda")
eng.fill_uniform(buf, 1, eng.SOLINAS_P)
s = torch.cuda.Stream()
torch.cuda.synchronize()


def timeit(fn, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e6


with torch.cuda.stream(s):
    for _ in range(10):
        plan.fwd(buf); plan.inv(buf)
    eager = timeit(lambda: (plan.fwd(buf), plan.inv(buf)), K)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=s):
        plan.fwd(buf)
        plan.inv(buf)
    g1.replay()
    one = timeit(g1.replay, K)
    g10 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g10, stream=s):
        for _ in range(10):
            plan.fwd(buf)
            plan.inv(buf)
    g10.replay()
    ten = timeit(g10.replay, K // 10) / 10
    fw = timeit(lambda: plan.fwd(buf), K)
print(f"eager {eager:.1f} us/step  graph(1 step) {one:.1f}  graph(10 steps) {ten:.1f}  fwd-only eager {fw:.1f}")
