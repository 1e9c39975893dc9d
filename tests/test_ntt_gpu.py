"""GPU parity of the HIP NTT path against the CPU oracle, through the C ABI (`-m gpu`).

Bar: bit-exact.  Small sizes compare every output with the oracle; the headline size
(N = 2048, batch 8192) is compared in full against the multi-threaded oracle plus the
size-independent round trip inv(fwd(x)) = N x.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SOLINAS_P = 0xFFFFFFFF00000001


def _primes(oracle):
    f = oracle.largest_prime_in_arithmetic_progression64
    return {
        "solinas": SOLINAS_P,
        "p64": f(1 << 16, 1, 1 << 63, 2**64 - 1),
        "p63": f(1 << 16, 1, 1 << 62, 1 << 63),
        "p62": f(1 << 16, 1, 1 << 61, 1 << 62),
        "p50": f(1 << 16, 1, 1 << 49, 1 << 50),
        "p30": 1062862849,
    }


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("logn", list(range(4, 19)))
def test_fwd_inv_all_sizes_solinas(engine, oracle, logn):
    """N = 16 ... 2^18; N > 2^14 runs the two-pass large-N path (top stages + 2^14 blocks)."""
    n = 1 << logn
    batch = max(1, min(37, (1 << 17) // n))  # ragged (not a multiple of the polys-per-workgroup)
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    x = oracle.fill_uniform(0x74666865 + logn, SOLINAS_P, batch * n).reshape(batch, n)
    t = dev(x)
    plan.fwd(t)
    fx = ora.fwd(x, threads=8)
    assert np.array_equal(host(t), fx)
    plan.inv(t)
    assert np.array_equal(host(t), ora.inv(fx, threads=8))
    t = dev(x)
    plan.inv(t)
    assert np.array_equal(host(t), ora.inv(x, threads=8))


@pytest.mark.parametrize("logn,batch", [(19, 2), (20, 1), (21, 1), (22, 1), (24, 1)])
def test_fwd_inv_beyond_2_18(engine, oracle, logn, batch):
    """N = 2^19 ... 2^24 (plans past the reference's root table, find_root_solinas_64, roots.rs:96-107):
    k = logn - 14 top stages run in passes of at most 4 (s0 = 0, 4, ...) before the 2^14 blocks; bit-exact vs the
    oracle both directions, plus a non-Solinas prime with 2^22 | p - 1 at N = 2^21."""
    n = 1 << logn
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    x = oracle.fill_uniform(0x1A26E + logn, SOLINAS_P, batch * n).reshape(batch, n)
    t = dev(x)
    plan.fwd(t)
    fx = ora.fwd(x, threads=16)
    assert np.array_equal(host(t), fx)
    plan.inv(t)
    assert np.array_equal(host(t), ora.inv(fx, threads=16))
    if logn == 21:
        p = oracle.largest_prime_in_arithmetic_progression64(1 << 22, 1, 1 << 62, 1 << 63)
        plan, ora = engine.Plan.try_new(n, p), oracle.Plan.try_new(n, p)
        x = oracle.fill_uniform(0x1A26F, p, n).reshape(1, n)
        t = dev(x)
        plan.fwd(t)
        assert np.array_equal(host(t), ora.fwd(x, threads=16))
        t = dev(x)
        plan.inv(t)
        assert np.array_equal(host(t), ora.inv(x, threads=16))


@pytest.mark.parametrize("name", ["p64", "p63", "p62", "p50", "p30"])
@pytest.mark.parametrize("logn", [4, 5, 10, 11, 12, 15, 16])
def test_fwd_inv_other_primes(engine, oracle, name, logn):
    p = _primes(oracle)[name]
    n = 1 << logn
    plan, ora = engine.Plan.try_new(n, p), oracle.Plan.try_new(n, p)
    assert (plan is None) == (ora is None)  # no 2N-th root: None on both sides
    if ora is None:
        return
    batch = 5 if logn < 15 else 2
    x = oracle.fill_uniform(17 + logn, p, batch * n).reshape(batch, n)
    t = dev(x)
    plan.fwd(t)
    assert np.array_equal(host(t), ora.fwd(x))
    t = dev(x)
    plan.inv(t)
    assert np.array_equal(host(t), ora.inv(x))


@pytest.mark.parametrize("logn,batch", [(12, 5), (13, 3), (14, 3), (15, 3), (17, 2), (19, 2)])
def test_large_n_strided_batch(engine, oracle, logn, batch):
    """Large-N path on a padded-stride batch (2^12 ... 2^14: the one-launch split transform, ntt_tw_fused_kernel):
    bit-exact, gaps never written, inv(fwd(x)) = N x."""
    import torch
    n = 1 << logn
    stride = n + 64
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    full = oracle.fill_uniform(0xB16 + logn, SOLINAS_P, batch * stride).reshape(batch, stride)
    t = dev(full)
    plan.fwd(t[:, :n])
    out = host(t)
    fx = ora.fwd(np.ascontiguousarray(full[:, :n]), threads=8)
    assert np.array_equal(out[:, :n], fx) and np.array_equal(out[:, n:], full[:, n:])
    plan.inv(t[:, :n])
    back = host(t)[:, :n]
    want = np.array([[oracle.mul_mod(int(v), n, SOLINAS_P) for v in row[:64]] for row in full[:, :n]], np.uint64)
    assert np.array_equal(back[:, :64], want)
    assert np.array_equal(back, ora.inv(fx, threads=8))


def test_strided_batch_leaves_gaps_untouched(engine, oracle):
    import torch

    n, batch, stride = 2048, 9, 2048 + 64
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    full = oracle.fill_uniform(3, SOLINAS_P, batch * stride).reshape(batch, stride)
    t = dev(full)
    view = t[:, :n]
    assert view.stride(0) == stride
    plan.fwd(view)
    out = host(t)
    assert np.array_equal(out[:, n:], full[:, n:])  # padding never written
    assert np.array_equal(out[:, :n], ora.fwd(np.ascontiguousarray(full[:, :n])))
    torch.cuda.synchronize()


def test_empty_batch_and_length_mismatch(engine):
    import torch

    plan = engine.Plan.try_new(2048, SOLINAS_P)
    plan.fwd(torch.zeros((0, 2048), dtype=torch.int64, device="cuda"))  # no-op, like an empty loop
    with pytest.raises(ValueError):
        plan.fwd(torch.zeros(2047, dtype=torch.int64, device="cuda"))
    with pytest.raises(ValueError):
        plan.inv(np.zeros(1000, np.uint64))


def test_edge_values(engine, oracle):
    # all-zero, all p-1, single spikes, alternating extremes
    n = 2048
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    rows = [np.zeros(n, np.uint64), np.full(n, SOLINAS_P - 1, np.uint64), np.ones(n, np.uint64)]
    spike = np.zeros(n, np.uint64); spike[n - 1] = SOLINAS_P - 1; rows.append(spike)
    alt = np.where(np.arange(n) % 2 == 0, SOLINAS_P - 1, 0).astype(np.uint64); rows.append(alt)
    hi = np.full(n, 0xFFFFFFFF00000000, np.uint64); rows.append(hi)   # p - 1 and the 2^64-2^32 corner
    x = np.stack(rows)
    t = dev(x); plan.fwd(t); assert np.array_equal(host(t), ora.fwd(x))
    t = dev(x); plan.inv(t); assert np.array_equal(host(t), ora.inv(x))


@pytest.mark.parametrize("name", ["solinas", "p64", "p62", "p30"])
def test_pointwise_ops(engine, oracle, name):
    p = _primes(oracle)[name]
    n, batch = 1024, 7
    plan, ora = engine.Plan.try_new(n, p), oracle.Plan.try_new(n, p)
    a, b, c = (oracle.fill_uniform(s, p, batch * n).reshape(batch, n) for s in (21, 22, 23))
    t = dev(a); plan.normalize(t); assert np.array_equal(host(t), ora.normalize(a))
    t = dev(a); plan.mul_assign_normalize(t, dev(b)); assert np.array_equal(host(t), ora.mul_assign_normalize(a, b))
    t = dev(c); plan.mul_accumulate(t, dev(a), dev(b)); assert np.array_equal(host(t), ora.mul_accumulate(c, a, b))
    # odd stride -> scalar access path
    full = np.concatenate([c, np.zeros((batch, 1), np.uint64)], axis=1)
    tf = dev(full); v = tf[:, :n]
    plan.mul_accumulate(v, dev(np.concatenate([a, a[:, :1]], 1))[:, :n], dev(np.concatenate([b, b[:, :1]], 1))[:, :n])
    assert np.array_equal(host(tf)[:, :n], ora.mul_accumulate(c, a, b))
    # even stride > N -> the 16-byte path with the per-row offset (the contiguous batch above takes the flat path)
    full2 = np.concatenate([c, np.zeros((batch, 2), np.uint64)], axis=1)
    tf2 = dev(full2); v2 = tf2[:, :n]
    plan.mul_accumulate(v2, dev(np.concatenate([a, a[:, :2]], 1))[:, :n], dev(np.concatenate([b, b[:, :2]], 1))[:, :n])
    assert np.array_equal(host(tf2)[:, :n], ora.mul_accumulate(c, a, b)) and (host(tf2)[:, n:] == 0).all()


def test_polymul_through_ntt(engine, oracle):
    # prime64.rs:1305-1361 end to end on device: inv(mul_assign_normalize(fwd a, fwd b)) = a (*) b
    n = 1024
    for p in (SOLINAS_P, _primes(oracle)["p62"]):
        plan = engine.Plan.try_new(n, p)
        a, b = oracle.fill_uniform(31, p, n), oracle.fill_uniform(32, p, n)
        ta, tb = dev(a), dev(b)
        plan.fwd(ta); plan.fwd(tb)
        plan.mul_assign_normalize(ta, tb)
        plan.inv(ta)
        assert np.array_equal(host(ta), oracle.negacyclic_convolution(n, p, a, b))


def test_device_generator_matches_oracle(engine, oracle):
    import torch

    for p in (SOLINAS_P, 1062862849, 0):
        t = torch.empty(100003, dtype=torch.int64, device="cuda")
        engine.fill_uniform(t, 0x74666865 + 2, p)
        assert np.array_equal(host(t), oracle.fill_uniform(0x74666865 + 2, p, 100003))


def test_headline_batch_full_parity(engine, oracle):
    """Config 2 shape: N=2048, batch 8192 — full comparison with the oracle + round trip."""
    import torch

    n, batch = 2048, 8192
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    t = torch.empty((batch, n), dtype=torch.int64, device="cuda")
    engine.fill_uniform(t, 0x74666865 + 2, SOLINAS_P)
    x = host(t).copy()
    assert np.array_equal(x.reshape(-1), oracle.fill_uniform(0x74666865 + 2, SOLINAS_P, batch * n))
    plan.fwd(t)
    fx = host(t).copy()
    ref = x.copy().reshape(-1)
    ora.fwd_scalar_inplace(ref, 8)  # the canonical scalar restatement (generic_solinas.rs:449-481)
    assert np.array_equal(fx.reshape(-1), ref)
    plan.inv(t)
    back = host(t)
    # size-independent property: inv(fwd(x)) == N x mod p, i.e. normalize(inv(fwd(x))) == x
    assert np.array_equal(ora.normalize(back), x)


def test_split_transform_chunked_batch(engine, oracle):
    """The split transform (N = 4096: one top stage + the twisted 2048 body on 2 blocks per polynomial) on a batch
    past the top pass's 65,535-polynomial grid.y chunk: the polynomials on both sides of the chunk edge equal the
    oracle, and normalize(inv(fwd(x))) == x over the whole batch (checked on the device)."""
    import torch
    n, batch = 4096, 65535 + 4
    plan, ora = engine.Plan.try_new(n, SOLINAS_P), oracle.Plan.try_new(n, SOLINAS_P)
    x = torch.empty((batch, n), dtype=torch.int64, device="cuda")
    engine.fill_uniform(x, 0x5917, SOLINAS_P)
    t = x.clone()
    plan.fwd(t)
    rows = [0, 1, 65533, 65534, 65535, 65536, batch - 1]
    xs = host(x[rows])
    assert np.array_equal(host(t[rows]), ora.fwd(xs, threads=8))
    plan.inv(t)
    plan.normalize(t)
    assert torch.equal(t, x)
