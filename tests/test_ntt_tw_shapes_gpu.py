"""GPU parity of the twisted N = 2048 transform kernel (ntt_tw_body_kernel, one wave per polynomial; the
forward runs 1-wave workgroups, the inverse 4-wave ones) on ragged batches (not multiples of 4) and padded
strides (`-m gpu`): bit-exact against the oracle (Plan::fwd / Plan::inv, prime64.rs:897-1046), padding and
the row after the batch never written.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SOLINAS_P = 0xFFFFFFFF00000001


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("batch,stride", [(1, 2048), (7, 2048), (2051, 2048), (300, 2048 + 8), (5000, 2048)])
def test_twisted_kernel_shapes(engine, oracle, batch, stride):
    n = 2048
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    full = oracle.fill_uniform(0x5EED + batch, SOLINAS_P, (batch + 1) * stride).reshape(batch + 1, stride)
    x = np.ascontiguousarray(full[:batch, :n])
    t = dev(full)
    plan.fwd(t[:batch, :n])
    out = host(t)
    fx = ora.fwd(x, threads=8)
    assert np.array_equal(out[:batch, :n], fx)
    assert np.array_equal(out[:batch, n:], full[:batch, n:])  # padding never written
    assert np.array_equal(out[batch], full[batch])            # nor the row after the batch
    plan.inv(t[:batch, :n])
    out = host(t)
    assert np.array_equal(out[:batch, :n], ora.inv(fx, threads=8))
    assert np.array_equal(out[:batch, n:], full[:batch, n:])
    assert np.array_equal(out[batch], full[batch])
