"""The per-polynomial host form of Plan::fwd / Plan::inv (`mi_ntt64_fwd_host` / `_inv_host`): the drop-in for
Ntt64View::forward / add_backward, which the reference calls one polynomial at a time from rayon workers
(tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:89-137).  Bit-exact vs the oracle, safe from concurrent host
threads (each call borrows its own staging slot and stream), and never synchronises other streams of the
process: a transform queued on another stream keeps running while host calls complete."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


@pytest.mark.parametrize("n", [1024, 2048, 4096])
def test_host_single_poly_bit_exact(engine, oracle, n):
    plan, ora = engine.Plan.try_new(n, P), oracle.Plan.try_new(n, P)
    for seed in range(3):
        x = oracle.fill_uniform(0xC0FF + seed + n, P, n)
        y = x.copy()
        plan.fwd(y)
        assert np.array_equal(y, ora.fwd(x))
        plan.inv(y)
        assert np.array_equal(y, ora.inv(ora.fwd(x)))


def test_host_batches_grow_the_staging_slot(engine, oracle):
    """A small call, then larger ones (the slot's buffers grow), then a small one again; batch 128 (2 MiB) is the
    last in-place call on the mapped host buffer, 129 the first staged one (c_api.cpp ZERO_COPY_BYTES)."""
    plan, ora = engine.Plan.try_new(2048, P), oracle.Plan.try_new(2048, P)
    for batch in (1, 64, 128, 129, 3):
        x = oracle.fill_uniform(0xB0 + batch, P, batch * 2048).reshape(batch, 2048)
        y = x.copy()
        plan.fwd(y)
        assert np.array_equal(y, ora.fwd(x))


def test_host_concurrent_threads(engine, oracle):
    """8 host threads x 40 single-polynomial fwd+inv round trips on one shared plan (the reference's Arc<Plan>
    shared across rayon workers): every result bit-exact."""
    plan, ora = engine.Plan.try_new(2048, P), oracle.Plan.try_new(2048, P)
    errors = []

    def worker(t):
        try:
            for i in range(40):
                x = oracle.fill_uniform(1000 * t + i, P, 2048)
                y = x.copy()
                plan.fwd(y)
                if not np.array_equal(y, ora.fwd(x)):
                    errors.append((t, i, "fwd"))
                plan.inv(y)
                if not np.array_equal(y, ora.inv(ora.fwd(x))):
                    errors.append((t, i, "inv"))
        except Exception as e:  # surface it in the main thread
            errors.append((t, repr(e)))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:5]


def test_host_call_does_not_wait_for_other_streams(engine):
    """A host call returns while a long transform loop queued on another stream is still running (the old path
    called hipDeviceSynchronize, which waited for it).  The loop is 80 launches over a 1 GiB batch (~35 ms of GPU
    work, few enough launches that queueing them never blocks the host), and the host path is warmed first so
    its staging slot exists."""
    import torch
    plan = engine.Plan.try_new(2048, P)
    x = np.arange(2048, dtype=np.uint64)
    plan.fwd(x)  # warm: the staging slot of this device exists and is large enough
    busy = torch.zeros((65536, 2048), dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    done = torch.cuda.Event()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for _ in range(40):
            plan.fwd(busy)
            plan.inv(busy)
        done.record(s)
    plan.fwd(x)
    assert not done.query(), "the host call waited for an unrelated stream"
    torch.cuda.synchronize()


@pytest.mark.parametrize("n,prime", [(32768, "solinas"), (1024, "p62"), (64, "solinas")])
def test_host_other_plans(engine, oracle, n, prime):
    """The host form over the large-N passes (N = 2^15 on the mapped buffer) and a Montgomery-path prime."""
    p = P if prime == "solinas" else oracle.largest_prime_in_arithmetic_progression64(1 << 16, 1, 1 << 61, 1 << 62)
    plan, ora = engine.Plan.try_new(n, p), oracle.Plan.try_new(n, p)
    x = oracle.fill_uniform(0xD00D + n, p, 2 * n).reshape(2, n)
    y = x.copy()
    plan.fwd(y)
    assert np.array_equal(y, ora.fwd(x))
    plan.inv(y)
    assert np.array_equal(y, ora.inv(ora.fwd(x)))
