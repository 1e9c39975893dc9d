"""Corner-case checks of the modular building blocks the generated transform / PBS bodies are made of
(tools/gen_tw_kernel.py: tmul, tmul_lane, ct, gs, gmul, canon), emulated instruction by instruction
(tools/asm_emu.py) on adversarial 64-bit inputs — 0, 1, p - 1, p, p + 1, 2^64 - 1, values around 2^32,
2^63 and random ones, in every lane — against Python integers.  The whole-body tests
(tests/test_tw_codegen.py) only see random data; the carry corners these blocks must get right occur
with probability ~2^-32 there.  No GPU."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import asm_emu  # noqa: E402
import gen_tw_kernel as G  # noqa: E402

P = 0xFFFFFFFF00000001
M64 = (1 << 64) - 1
EPS = (1 << 32) - 1


def corner_values(rnd, canonical):
    base = [0, 1, 2, P - 1, P - 2, EPS, EPS + 1, 1 << 32, (1 << 32) + 1, 1 << 63, (1 << 63) - 1, (1 << 63) + 1,
            P >> 1, (P >> 1) + 1, 0xFFFFFFFE00000000, 0xFFFFFFFE00000001, 0x00000001FFFFFFFF, 0x7FFFFFFF80000000]
    if not canonical:
        base += [P, P + 1, P + 2, M64, M64 - 1, M64 - EPS, M64 - EPS + 1, 0xFFFFFFFF80000000]
    vals = [v for v in base if canonical is False or v < P]
    while len(vals) < 64:
        hi = rnd.choice([0, 0xFFFFFFFF, 0xFFFFFFFE, rnd.getrandbits(32)])
        v = (hi << 32) | rnd.choice([0, 1, EPS, rnd.getrandbits(32)])
        vals.append(v % P if canonical else v)
    return vals[:64]


def run_seg(sg, regs_in, pairs_out, in_order=False):
    """Emulate a Seg on one wave; regs_in: {pair_base: list of 64 u64}; returns {pair_base: list}."""
    w = asm_emu.Wave({}, {})
    w.s[G.S_X15] = np.uint64(0x11111111)
    w.s[G.S_PAR], w.s[G.S_PAR + 1] = np.uint64(0xAAAAAAAA), np.uint64(0xAAAAAAAA)
    w.s[G.S_EXE], w.s[G.S_EXE + 1] = np.uint64(0xFFFFFFFF), np.uint64(0xFFFFFFFF)  # the body's saved EXEC
    for b, vals in regs_in.items():
        arr = np.array(vals, dtype=np.uint64)
        w.v[b] = arr & np.uint64(0xFFFFFFFF)
        w.v[b + 1] = arr >> np.uint64(32)
    for i, op in enumerate(sg.ops):
        op.idx = i
    w.run(sg.emit_in_order() if in_order else sg.schedule())
    return {b: [int(lo) | (int(hi) << 32) for lo, hi in zip(w.v[b], w.v[b + 1])] for b in pairs_out}


def slot():
    return G.Slot(8, G.SG0)


X_A, X_B = 64, 66  # data pairs


@pytest.mark.parametrize("S", range(0, 192))
def test_tmul_all_exponents(S):
    rnd = random.Random(S)
    xs = corner_values(rnd, canonical=False)  # tmul takes any 64-bit value
    sg = G.Seg()
    sl = slot()
    neg = G.tmul(sg, S, f"v{X_A}", f"v{X_A + 1}", G.pv(X_A), sl, sl.v[2], sl.v[3])
    out = run_seg(sg, {X_A: xs}, [8 + 2])[10]
    for x, t in zip(xs, out):
        want = x * pow(2, S, P) % P
        assert t < P, (S, hex(x), hex(t))
        assert (P - t) % P == want if neg else t == want, (S, hex(x))


def _pair_exponents():
    tabs = G.load_tables()
    out = []
    for name in ("CYC_FWD", "CYC_INV"):
        E = tabs[name][5]
        out += [(E[k], E[k + 16]) for k in range(16) if G.lane_tmul_applies(E[k], E[k + 16])]
    return out


@pytest.mark.parametrize("Se,So", _pair_exponents())
def test_tmul_lane(Se, So):
    rnd = random.Random(Se * 1000 + So)
    xs = corner_values(rnd, canonical=False)
    xs = xs[:32] + xs[:32]  # every value in an even and in an odd lane
    sg = G.Seg()
    sl = slot()
    par3 = "v30"
    sg.add(f"v_cndmask_b32_e64 {par3}, 0, 3, s[{G.S_PAR}:{G.S_PAR + 1}]", [], [par3])
    neg = G.tmul_lane(sg, Se, So, (f"v{X_A}", f"v{X_A + 1}", G.pv(X_A)), sl, sl.v[2], sl.v[3], par3, ("v28", "v29"))
    out = run_seg(sg, {X_A: xs}, [10])[10]
    for lane, (x, t) in enumerate(zip(xs, out)):
        S = So if lane & 1 else Se
        want = x * pow(2, S, P) % P
        assert t < P
        assert ((P - t) % P if neg else t) == want, (Se, So, lane, hex(x))


@pytest.mark.parametrize("S", [0, 3, 24, 30, 33, 48, 63, 64, 72, 93, 96, 99, 120, 144, 160, 168, 189])
@pytest.mark.parametrize("ac,bc", [(False, False), (True, False), (False, True), (True, True)])
def test_gs_butterfly(S, ac, bc):
    rnd = random.Random(S * 4 + 2 * ac + bc)
    a = corner_values(rnd, ac)
    b = corner_values(random.Random(rnd.random()), bc)
    rnd.shuffle(b)
    if ac and bc:  # the largest sums / differences of canonical values
        a[:3], b[:3] = [P - 1, P - 1, 0], [P - 1, 0, P - 1]
    sg = G.Seg()
    sc, dc = G.gs(sg, slot(), G.X([X_A, X_B], 0), G.X([X_A, X_B], 1), S, ac, bc)
    assert dc and sc == (ac and bc)
    out = run_seg(sg, {X_A: a, X_B: b}, [X_A, X_B])
    w = pow(2, S, P)
    for x, y, s, d in zip(a, b, out[X_A], out[X_B]):
        assert s % P == (x + y) % P and (s < P or not sc)
        assert d < P and d == (x - y) * w % P


@pytest.mark.parametrize("S", [0, 3, 24, 30, 48, 63, 72, 93, 96, 120, 144, 189])
@pytest.mark.parametrize("bc", [False, True])
def test_ct_butterfly(S, bc):
    rnd = random.Random(S + 1000 * bc)
    a = corner_values(rnd, False)
    b = corner_values(random.Random(rnd.random()), bc)
    sg = G.Seg()
    sl = slot()
    A, B = G.X([X_A, X_B], 0), G.X([X_A, X_B], 1)
    if S % 96 == 0 and bc:
        G.ct_core(sg, sl, A, B, S >= 96, tsrc=(B[0], B[1]))
    else:
        G.ct(sg, sl, A, B, S)
    out = run_seg(sg, {X_A: a, X_B: b}, [X_A, X_B])
    w = pow(2, S, P)
    for x, y, s, d in zip(a, b, out[X_A], out[X_B]):
        assert s % P == (x + y * w) % P and d % P == (x - y * w) % P


def test_gmul_and_canon():
    rnd = random.Random(5)
    xs = corner_values(rnd, False)
    ws = corner_values(random.Random(6), True)
    sg = G.Seg()
    ms = G.MulSlot(8, G.SG0)
    G.gmul(sg, ms, G.X([X_A], 0), "v70", "v71", f"v{X_A}", f"v{X_A + 1}")
    out = run_seg(sg, {X_A: xs, 70: ws}, [X_A])[X_A]
    for x, w, t in zip(xs, ws, out):
        assert t == x * w % P
    sg = G.Seg()
    G.canon(sg, slot(), G.X([X_A], 0))
    out = run_seg(sg, {X_A: xs}, [X_A])[X_A]
    assert out == [x % P for x in xs]


@pytest.mark.parametrize("S", [0, 3, 24, 30, 33, 48, 63, 64, 72, 93, 96, 99, 120, 144, 168, 189])
@pytest.mark.parametrize("shuffle", range(4))
def test_ct_butterfly_canonical_outputs(S, shuffle):
    """The forward's last stage: canon(a), t = tmul(b), ct_core_canon -> both outputs canonical."""
    rnd = random.Random(S * 8 + shuffle)
    a = corner_values(rnd, False)
    b = corner_values(random.Random(rnd.random()), False)
    rnd.shuffle(a)
    rnd.shuffle(b)
    if shuffle == 0:  # the largest sums / differences of canonical values
        a[:4], b[:4] = [P - 1, P - 1, 0, M64], [P - 1, 0, P - 1, M64]
    sg = G.Seg()
    sl = slot()
    A, B = G.X([X_A, X_B], 0), G.X([X_A, X_B], 1)
    G.canon(sg, sl, A)
    neg = G.tmul(sg, S, B[0], B[1], B[2], sl, sl.v[2], sl.v[3])
    G.ct_core_canon(sg, sl, A, B, neg)
    out = run_seg(sg, {X_A: a, X_B: b}, [X_A, X_B])
    w = pow(2, S, P)
    for x, y, s, d in zip(a, b, out[X_A], out[X_B]):
        assert s < P and d < P, (S, hex(x), hex(y), hex(s), hex(d))
        assert s == (x + y * w) % P and d == (x - y * w) % P, (S, hex(x), hex(y))


def test_modswitch_native_corners():
    """modswitch_native (the key conversion's native 2^64 -> Z_p switch) == (x p + 2^63) >> 64, ntt64.rs:166-178."""
    rnd = random.Random(11)
    for rep in range(4):
        xs = corner_values(rnd, False)
        if rep == 0:
            xs[:12] = [0, 1, M64, M64 - 1, 1 << 63, (1 << 63) - 1, 0xFFFFFFFF00000000, 0x80000000FFFFFFFF,
                       0x7FFFFFFF00000000, 0x7FFFFFFFFFFFFFFF, 0x80000000_80000000, 0x7FFFFFFF_80000000]
        sg = G.Seg()
        sg.add(f"s_mov_b32 s{G.S_H31}, 0x80000000", [], [f"s{G.S_H31}"], "salu")
        G.modswitch_native(sg, slot(), G.X([X_A], 0))
        out = run_seg(sg, {X_A: xs}, [X_A])[X_A]
        for x, y in zip(xs, out):
            assert y == (x * P + (1 << 63)) >> 64 and y < P, hex(x)
