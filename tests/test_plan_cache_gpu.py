"""The process-wide plan cache of ``Ntt64::new`` (tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:27-79)
behind ``mi_ntt64_plan_cached`` / ``Plan.cached`` (`-m gpu`: plans upload their tables)."""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


def test_cached_plan_is_shared_and_correct(engine, oracle):
    import torch
    a = engine.Plan.cached(2048, P)
    b = engine.Plan.cached(2048, P)
    assert a.handle.value == b.handle.value  # one plan per (N, p, device)
    assert engine.Plan.cached(1024, P).handle.value != a.handle.value
    del b  # dropping a cached handle never frees the shared plan
    x = oracle.fill_uniform(0xCAC4E, P, 3 * 2048).reshape(3, 2048)
    t = torch.from_numpy(x.view(np.int64)).cuda()
    a.fwd(t)
    assert np.array_equal(t.cpu().numpy().view(np.uint64), oracle.Plan.try_new(2048, P).fwd(x))
    assert engine.Plan.cached(2048, P).handle.value == a.handle.value


def test_cached_plan_concurrent_first_use(engine):
    """Many threads asking for a new (N, p) at once all get the one plan built once."""
    p62 = 4611686018427322369  # a Shoup-range prime (prime64.rs:1311)
    out, errs = [], []

    def get():
        try:
            out.append(engine.Plan.cached(512, p62).handle.value)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    threads = [threading.Thread(target=get) for _ in range(16)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errs and len(set(out)) == 1


def test_cached_plan_errors(engine):
    """Where Plan::try_new is None the reference's Ntt64::new panics; here the status is returned, and
    the failure is cached like a plan (every later lookup reports it)."""
    for _ in range(2):
        with pytest.raises(engine.MiError) as e:
            engine.Plan.cached(2048, 1024)
        assert e.value.status == 2  # MI_ERR_NOT_PRIME
    L = engine._lib.lib()
    h = ctypes.c_void_p()
    assert L.mi_ntt64_plan_cached(100, P, 0, ctypes.byref(h)) == 1  # not a power of two
    assert L.mi_ntt64_plan_destroy(engine.Plan.cached(2048, P).handle) == 0  # no-op on a cached plan
    assert engine.Plan.cached(2048, P).ntt_size() == 2048
