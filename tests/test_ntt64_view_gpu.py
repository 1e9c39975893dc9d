"""GPU parity of the Ntt64View layer (ntt64.rs:89-266) and the u64 LWE modulus switch (modulus_switch.rs:14-104) as
batched device operations (`-m gpu`), through the C ABI, against the oracle's restatement (pbs_oracle.c
ora_ntt64_view_*, ora_lwe_ms64).  Bit-exact, both the operation's output and what it leaves in the reference's scratch
buffer (`ntt` after add_backward).

The Solinas N = 2048 plan runs the fused twisted bodies (csrc/ntt64_view.hip, tools/gen_view_kernel.py) and is tested
at the full config-2 batch (8192 polynomials); the other plans run the generic prologue / epilogue around their own
transform (window kernels, split transform, large-N passes, a Montgomery prime) on smaller batches.
Corners: 0, p - 1, 2^64 - 1, 2^63; the OR-rounding ties of the p -> 2^w switch (v with (v 2^w + (p - 1) / 2) mod p at
0 and p - 1); decomposition digits -2^22 and 2^22; widths 64, 63, 33, 32, 21, 1.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001
M64 = (1 << 64) - 1


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def _ctx(oracle, n, p=P):
    return oracle.NttContext(n, p)


def _ties(width, p, count):
    """v < p at the rounding boundary of ((v << w) | p >> 1) / p (ntt64.rs:184-196): (v 2^w + (p - 1) / 2) mod p equal
    to 0 (the quotient just steps up) and to p - 1 (just below the step) — exact when the OR is an add (w >= 63 for the
    Solinas prime); other widths get the same v's, the oracle decides."""
    inv = pow(pow(2, width, p), p - 2, p)
    half = (p - 1) // 2
    out = []
    for r in range(count):
        target = (-half - r) % p  # v 2^w = target mod p  =>  v 2^w + half = -r mod p
        out.append((target * inv) % p)
    return out


def _std_input(oracle, seed, batch, n, p=P, canonical=True):
    x = oracle.fill_uniform(seed, p if canonical else 0, batch * n).reshape(batch, n)
    x[0, :4] = [0, p - 1, 1, p // 2] if canonical else [0, M64, 1 << 63, p]
    if not canonical:
        x[0, 4:8] = [p - 1, (1 << 63) - 1, 1, 2]
    return x


@pytest.mark.parametrize("normalized", [False, True])
def test_forward_full_batch(engine, oracle, normalized):
    """forward / forward_normalized (ntt64.rs:89-108) on the config-2 batch, out of place and in place."""
    n, batch = 2048, 8192
    view = engine.ntt64.Ntt64(P, n).as_view()
    ctx = _ctx(oracle, n)
    x = _std_input(oracle, 0x5101, batch, n)
    want = ctx.forward_normalized(x, threads=16) if normalized else ctx.forward(x, threads=16)
    src, dst = dev(x), dev(np.zeros_like(x))
    (view.forward_normalized if normalized else view.forward)(dst, src)
    assert np.array_equal(host(dst), want)
    assert np.array_equal(host(src), x), "the standard buffer is read only"
    (view.forward_normalized if normalized else view.forward)(src, src)  # in place
    assert np.array_equal(host(src), want)


@pytest.mark.parametrize("width", [64, 63, 33, 32, 21, 1])
def test_forward_from_power_of_two_modulus_full_batch(engine, oracle, width):
    """forward_from_power_of_two_modulus (ntt64.rs:166-177, 201-214) at every width class: MSB-aligned inputs (the
    reference's power-of-two encoding) plus arbitrary low bits (the switch ignores them), 0, 2^64 - 1, 2^63."""
    n, batch = 2048, 8192 if width in (64, 21) else 1024
    view = engine.ntt64.Ntt64(P, n).as_view()
    ctx = _ctx(oracle, n)
    x = _std_input(oracle, 0x5102 + width, batch, n, canonical=False)
    x[1::2] = (x[1::2] >> np.uint64(64 - width)) << np.uint64(64 - width)
    want = ctx.forward_from_power_of_two_modulus(width, x, threads=16)
    src, dst = dev(x), dev(np.zeros_like(x))
    view.forward_from_power_of_two_modulus(width, dst, src)
    assert np.array_equal(host(dst), want)


def test_forward_from_decomp_full_batch(engine, oracle):
    """forward_from_decomp (ntt64.rs:221-240): signed digits of a 2^23-base decomposition in [-2^22, 2^22] as
    wrapping u64, the extremes -2^22 and 2^22, and arbitrary u64 words (the rule is x + p for every x < 0 as i64)."""
    n, batch = 2048, 8192
    view = engine.ntt64.Ntt64(P, n).as_view()
    ctx = _ctx(oracle, n)
    g = np.random.Generator(np.random.PCG64(0x5103))
    d = g.integers(-(1 << 22), (1 << 22) + 1, size=(batch, n), dtype=np.int64).astype(np.uint64)
    d[0, :4] = np.array([-(1 << 22), 1 << 22, -1, 0], dtype=np.int64).astype(np.uint64)
    d[1] = g.integers(0, 2**64, size=n, dtype=np.uint64)
    d[2, :4] = [1 << 63, M64, (1 << 63) - 1, P]
    want = ctx.forward_from_decomp(d, threads=16)
    src, dst = dev(d), dev(np.zeros_like(d))
    view.forward_from_decomp(dst, src)
    assert np.array_equal(host(dst), want)


def test_add_backward_full_batch(engine, oracle):
    """add_backward (ntt64.rs:110-131): standard = wrapping_add_custom_mod(standard, inv(ntt), p); ntt is left
    holding inv(ntt), as Plan::inv in place leaves it."""
    n, batch = 2048, 8192
    view = engine.ntt64.Ntt64(P, n).as_view()
    ctx = _ctx(oracle, n)
    y = _std_input(oracle, 0x5104, batch, n)
    st = _std_input(oracle, 0x5105, batch, n)
    st[0, :4] = [P - 1, P - 1, 0, P - 1]
    want_st, want_y = ctx.add_backward(st, y, threads=16)
    ts, ty = dev(st), dev(y)
    view.add_backward(ts, ty)
    assert np.array_equal(host(ty), want_y)
    assert np.array_equal(host(ts), want_st)


@pytest.mark.parametrize("width", [64, 63, 32, 21, 1])
def test_add_backward_on_power_of_two_modulus_full_batch(engine, oracle, width):
    """add_backward_on_power_of_two_modulus (ntt64.rs:184-196, 244-266): ntt = (((v << w) | p >> 1) / p) << (64 - w)
    of v = inv(ntt), standard += ntt (wrapping).  The inverse's outputs include the rounding ties: the NTT input is
    fwd(t) of a t that holds them (inv(fwd(t)) = N t, so t carries the ties times N^-1)."""
    n, batch = 2048, 8192 if width in (64, 21) else 1024
    view = engine.ntt64.Ntt64(P, n).as_view()
    ctx = _ctx(oracle, n)
    plan = oracle.Plan.try_new(n, P)
    n_inv = plan.n_inv
    t = _std_input(oracle, 0x5106 + width, batch, n)
    ties = _ties(width, P, 16) + [0, P - 1]
    t[0, :len(ties)] = [(v * n_inv) % P for v in ties]
    y = ctx.forward(t, threads=16)
    st = oracle.fill_uniform(0x5107 + width, 0, batch * n).reshape(batch, n)
    want_st, want_y = ctx.add_backward_on_power_of_two_modulus(width, st, y, threads=16)
    assert [int(v) for v in plan.inv(y[:1])[0, :len(ties)]] == ties, "the ties reach the switch"
    ts, ty = dev(st), dev(y)
    view.add_backward_on_power_of_two_modulus(width, ts, ty)
    assert np.array_equal(host(ty), want_y)
    assert np.array_equal(host(ts), want_st)


def _other_plans(oracle):
    f = oracle.largest_prime_in_arithmetic_progression64
    return [(1024, P), (4096, P), (8192, P), (32768, P), (2048, f(1 << 16, 1, 1 << 63, 2**64 - 1)),
            (512, f(1 << 16, 1, 1 << 61, 1 << 62))]


@pytest.mark.parametrize("idx", range(6))
def test_view_generic_plans(engine, oracle, idx):
    """Every Ntt64View op on the plans that do not run the fused bodies: the window kernels (N = 512 / 1024, a 64-bit
    and a 62-bit Montgomery prime), the split transform (4096, 8192) and the large-N passes (32768)."""
    n, p = _other_plans(oracle)[idx]
    batch = max(2, min(67, (1 << 17) // n))
    view = engine.ntt64.Ntt64(p, n).as_view()
    ctx = _ctx(oracle, n, p)
    x = _std_input(oracle, 0x5200 + idx, batch, n, p)
    xw = _std_input(oracle, 0x5210 + idx, batch, n, canonical=False)
    for name, args, want in [
        ("forward", (), ctx.forward(x)),
        ("forward_normalized", (), ctx.forward_normalized(x)),
    ]:
        dst = dev(np.zeros_like(x))
        getattr(view, name)(*args, dst, dev(x))
        assert np.array_equal(host(dst), want), name
    for w in (64, 21):
        dst = dev(np.zeros_like(xw))
        view.forward_from_power_of_two_modulus(w, dst, dev(xw))
        assert np.array_equal(host(dst), ctx.forward_from_power_of_two_modulus(w, xw)), w
    g = np.random.Generator(np.random.PCG64(0x5230 + idx))
    d = g.integers(-(1 << 22), (1 << 22) + 1, size=(batch, n), dtype=np.int64).astype(np.uint64)
    dst = dev(np.zeros_like(d))
    view.forward_from_decomp(dst, dev(d))
    assert np.array_equal(host(dst), ctx.forward_from_decomp(d))
    st = _std_input(oracle, 0x5220 + idx, batch, n, p)
    ws, wy = ctx.add_backward(st, x)
    ts, ty = dev(st), dev(x)
    view.add_backward(ts, ty)
    assert np.array_equal(host(ty), wy) and np.array_equal(host(ts), ws)
    for w in (64, 33):
        ws, wy = ctx.add_backward_on_power_of_two_modulus(w, xw, x)
        ts, ty = dev(xw), dev(x)
        view.add_backward_on_power_of_two_modulus(w, ts, ty)
        assert np.array_equal(host(ty), wy) and np.array_equal(host(ts), ws), w


def test_view_strided_batch(engine, oracle):
    """Row stride > N (a view into a wider buffer, e.g. one GLWE's polynomials): untouched padding, exact rows."""
    import torch
    n, batch, stride = 2048, 37, 2048 + 64
    view = engine.ntt64.Ntt64(P, n).as_view()
    ctx = _ctx(oracle, n)
    x = _std_input(oracle, 0x5300, batch, n)
    buf = torch.full((batch, stride), 7, dtype=torch.int64, device="cuda")
    src = torch.full((batch, stride), 5, dtype=torch.int64, device="cuda")  # both operands share one row stride
    src[:, :n] = dev(x)
    view.forward(buf[:, :n], src[:, :n])
    got = host(buf)
    assert np.array_equal(got[:, :n], ctx.forward(x)) and (got[:, n:] == 7).all()
    st = torch.full((batch, stride), 0, dtype=torch.int64, device="cuda")
    view.add_backward_on_power_of_two_modulus(64, st[:, :n], buf[:, :n])
    ws, _ = ctx.add_backward_on_power_of_two_modulus(64, np.zeros_like(x), ctx.forward(x))
    assert np.array_equal(host(st)[:, :n], ws) and (host(st)[:, n:] == 0).all()


def test_view_errors(engine):
    import torch
    view = engine.ntt64.Ntt64(P, 2048).as_view()
    a = torch.zeros((4, 2048), dtype=torch.int64, device="cuda")
    b = torch.zeros((4, 2048), dtype=torch.int64, device="cuda")
    for w in (0, 65):
        with pytest.raises(engine.MiError):
            view.forward_from_power_of_two_modulus(w, a, b)
        with pytest.raises(engine.MiError):
            view.add_backward_on_power_of_two_modulus(w, a, b)
    with pytest.raises(engine.MiError):  # add_backward operands must be disjoint
        view.add_backward(a, a)
    big = torch.zeros((5, 2048), dtype=torch.int64, device="cuda")
    with pytest.raises(engine.MiError):  # partial overlap
        view.forward(big[1:], big[:4])
    with pytest.raises(ValueError):
        view.forward(a, torch.zeros((3, 2048), dtype=torch.int64, device="cuda"))


@pytest.mark.parametrize("log_mod", [12, 1, 63, 64])
@pytest.mark.parametrize("centered", [False, True])
def test_lwe_modulus_switch_u64(engine, oracle, log_mod, centered):
    """lwe_ciphertext_[centered_binary_]modulus_switch at Scalar = u64 (modulus_switch.rs:14-104), materialised as the
    lazy switched ciphertext reads it; the centered form refuses log_mod = 64 (the reference's half_case shift
    underflows there)."""
    KS = engine.lwe_keyswitch
    if centered and log_mod == 64:
        with pytest.raises(engine.MiError):
            KS.lwe_ciphertext_modulus_switch(dev(np.zeros((2, 9), np.uint64)), dev(np.zeros((2, 9), np.uint64)), 64,
                                             centered=True)
        return
    g = np.random.Generator(np.random.PCG64(log_mod * 5 + centered))
    dim, batch = 918, 513
    lwe = g.integers(0, 2**64, size=(batch, dim + 1), dtype=np.uint64)
    lwe[1::2] = (lwe[1::2] >> np.uint64(40)) << np.uint64(40)
    lwe[0, :5] = [0, M64, 1 << 63, (1 << 63) - 1, 1 << 51]
    want = oracle.lwe_ms64(lwe, log_mod, centered)
    out = dev(np.zeros((batch, dim + 1), np.uint64))
    KS.lwe_ciphertext_modulus_switch(dev(lwe), out, log_mod, centered)
    assert np.array_equal(host(out), want)
    if log_mod < 64:
        assert (host(out) < np.uint64(1 << log_mod)).all()


def test_lwe_modulus_switch_u64_reference_kat(engine):
    """modulus_switch.rs:274-299 test_ms_halving_correction: mask (1, 1), body 0, log 12: both mask rounding errors
    are -1, so the body correction is -1 - half_case and the switched body is ms(2^64 - 1 - 2^51) = 4095."""
    KS = engine.lwe_keyswitch
    out = dev(np.zeros((1, 3), np.uint64))
    KS.lwe_ciphertext_centered_binary_modulus_switch(dev(np.array([[1, 1, 0]], np.uint64)), out, 12)
    assert host(out).tolist() == [[0, 0, 4095]]


def test_view_empty_batch(engine):
    """A zero-row batch is a no-op for the six view operations and the u64 switch (the reference's per-polynomial
    loops run zero times): no launch, no error, the operands untouched."""
    import torch
    view = engine.ntt64.Ntt64(P, 2048).as_view()
    a = torch.zeros((0, 2048), dtype=torch.int64, device="cuda")
    b = torch.zeros((0, 2048), dtype=torch.int64, device="cuda")
    view.forward(a, b)
    view.forward_normalized(a, b)
    view.forward_from_power_of_two_modulus(64, a, b)
    view.forward_from_decomp(a, b)
    view.add_backward(a, b)
    view.add_backward_on_power_of_two_modulus(21, a, b)
    lwe = torch.zeros((0, 919), dtype=torch.int64, device="cuda")
    engine.lwe_keyswitch.lwe_ciphertext_modulus_switch(lwe, torch.zeros_like(lwe), 12, centered=True)
    torch.cuda.synchronize()
    assert a.numel() == 0 and b.numel() == 0
