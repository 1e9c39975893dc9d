"""GPU parity of the secondary plans (`-m gpu`): prime32::Plan on u32 buffers vs
the oracle transform for the same (N, p), and every native / native_binary plan kind's
negacyclic_polymul vs the exact convolution mod 2^W (the property the reference's tests assert,
native64.rs:1200-1240).  Bit-exact."""
import random

import numpy as np
import pytest

import native_oracle as NO

pytestmark = pytest.mark.gpu


def dev(a, dtype):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(dtype)).cuda()


def host(t, dtype):
    return t.cpu().numpy().view(dtype)


def _primes32(oracle):
    lo30 = oracle.largest_prime_in_arithmetic_progression64(1 << 16, 1, 1 << 30, 1 << 31)
    lo31 = oracle.largest_prime_in_arithmetic_progression64(1 << 16, 1, 1 << 31, 1 << 32)
    return [1062862849, 1073479681, lo30, lo31, NO.PRIMES32[9]]


@pytest.mark.parametrize("n", [32, 1024, 2048, 32768])
def test_prime32_plan_parity(engine, oracle, n):
    import torch
    for p in _primes32(oracle):
        plan = engine.prime32.Plan.try_new(n, p)
        ref = oracle.Plan.try_new(n, p)
        assert plan is not None and plan.modulus() == p and plan.ntt_size() == n
        g = np.random.default_rng(p % 1000 + n)
        x = g.integers(0, p, size=(5, n), dtype=np.uint64).astype(np.uint32)
        x[0, :3] = [0, p - 1, 1]
        x[1] = p - 1  # a whole row at the top of the range (the Shoup32 sums and products near 2^32 at lo31)
        t = dev(x, np.int32)
        plan.fwd(t)
        want = np.stack([ref.fwd(r.astype(np.uint64)) for r in x])
        assert np.array_equal(host(t, np.uint32).astype(np.uint64), want)
        plan.inv(t)
        assert np.array_equal(host(t, np.uint32).astype(np.uint64), np.stack([ref.inv(r) for r in want]))
        # pointwise ops
        a = g.integers(0, p, size=(5, n), dtype=np.uint64).astype(np.uint32)
        b = g.integers(0, p, size=(5, n), dtype=np.uint64).astype(np.uint32)
        c = g.integers(0, p, size=(5, n), dtype=np.uint64).astype(np.uint32)
        ta, tb, tc = dev(a, np.int32), dev(b, np.int32), dev(c, np.int32)
        plan.mul_accumulate(tc, ta, tb)
        want_c = (c.astype(object) + a.astype(object) * b.astype(object)) % p
        assert np.array_equal(host(tc, np.uint32).astype(object), want_c)
        plan.mul_assign_normalize(ta, tb)
        ninv = pow(n, p - 2, p)
        assert np.array_equal(host(ta, np.uint32).astype(object), a.astype(object) * b.astype(object) % p * ninv % p)
        plan.normalize(tb)
        assert np.array_equal(host(tb, np.uint32).astype(object), b.astype(object) * ninv % p)
    torch.cuda.synchronize()


def test_prime32_try_new_none(engine):
    assert engine.prime32.Plan.try_new(16, 1062862849) is None     # N < 32 (prime32.rs:666)
    assert engine.prime32.Plan.try_new(48, 1062862849) is None     # not a power of two
    assert engine.prime32.Plan.try_new(64, 1062862851) is None     # not prime
    assert engine.prime32.Plan.try_new(64, 97) is None             # no primitive 128-th root


def _conv_wrap(a, b, width):
    """Negacyclic product mod 2^width with numpy wrapping arithmetic (width 32 / 64)."""
    dt = np.uint64
    n = a.shape[-1]
    out = np.zeros(n, dt)
    a, b = a.astype(dt), b.astype(dt)
    with np.errstate(over="ignore"):
        for i in range(n):
            if a[i] == 0:
                continue
            term = a[i] * b
            out[i:] += term[: n - i]
            out[:i] -= term[n - i:]
    if width == 32:
        out &= np.uint64(0xFFFFFFFF)
    return out


def _words(vals, width):
    if width == 32:
        return np.array(vals, dtype=np.uint64).astype(np.uint32).view(np.int32)
    if width == 64:
        return np.array(vals, dtype=np.uint64).view(np.int64)
    return np.array([[v & (2**64 - 1), v >> 64] for v in vals], dtype=np.uint64).view(np.int64)


def _unwords(a, width):
    if width == 32:
        return [int(v) for v in a.view(np.uint32).reshape(-1)]
    if width == 64:
        return [int(v) for v in a.view(np.uint64).reshape(-1)]
    w = a.view(np.uint64).reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in w]


@pytest.mark.parametrize("kind", range(len(NO.KINDS)))
@pytest.mark.parametrize("n", [32, 256])
def test_native_polymul_parity(engine, kind, n):
    import torch
    name, width, binary, bits, k = NO.KINDS[kind]
    mod, sub = name.split(".")
    plan = getattr(getattr(engine, mod), sub).try_new(n)
    assert plan is not None and plan.ntt_size() == n
    rnd = random.Random(kind * 100 + n)
    batch = 2
    lhs = [[rnd.getrandbits(width) for _ in range(n)] for _ in range(batch)]
    rhs = [[rnd.getrandbits(1) if binary else rnd.getrandbits(width) for _ in range(n)] for _ in range(batch)]
    lhs[0][0] = (1 << width) - 1  # extremes
    if not binary:
        rhs[0][0] = (1 << width) - 1
    shape = (batch, n, 2) if width == 128 else (batch, n)
    tl = torch.from_numpy(np.stack([_words(r, width) for r in lhs]).reshape(shape)).cuda()
    tr = torch.from_numpy(np.stack([_words(r, width) for r in rhs]).reshape(shape)).cuda()
    tp = torch.zeros_like(tl)
    plan.negacyclic_polymul(tp, tl, tr)
    got = tp.cpu().numpy()
    for b in range(batch):
        assert _unwords(got[b], width) == NO.schoolbook(lhs[b], rhs[b], width), (name, b)


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 5, 6, 7, 8])
def test_native_polymul_n2048(engine, kind):
    """N = 2048 for the 32/64-bit kinds, checked with wrapping numpy arithmetic."""
    import torch
    name, width, binary, bits, k = NO.KINDS[kind]
    mod, sub = name.split(".")
    n = 2048
    plan = getattr(getattr(engine, mod), sub).try_new(n)
    g = np.random.default_rng(kind)
    hi = 2**width
    lhs = g.integers(0, hi, size=(3, n), dtype=np.uint64)
    rhs = g.integers(0, 2, size=(3, n), dtype=np.uint64) if binary else g.integers(0, hi, size=(3, n), dtype=np.uint64)
    cast = (lambda a: a.astype(np.uint32).view(np.int32)) if width == 32 else (lambda a: a.view(np.int64))
    tl, tr = torch.from_numpy(cast(lhs)).cuda(), torch.from_numpy(cast(rhs)).cuda()
    tp = torch.zeros_like(tl)
    plan.negacyclic_polymul(tp, tl, tr)
    got = tp.cpu().numpy()
    got = got.view(np.uint32).astype(np.uint64) if width == 32 else got.view(np.uint64)
    for b in range(3):
        assert np.array_equal(got[b], _conv_wrap(lhs[b], rhs[b], width)), (name, b)


def test_native_try_new_none(engine):
    assert engine.native64.Plan32.try_new(16) is None  # component prime32 plans need N >= 32
    assert engine.native64.Plan52.try_new(16) is not None
    assert engine.native64.Plan32.try_new(100) is None
