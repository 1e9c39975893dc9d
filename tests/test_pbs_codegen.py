"""CPU checks of the generated blind-rotation asm (tools/gen_pbs_kernel.py, no GPU): the committed
header matches its generator, and a 2-wave emulation of the body (tools/asm_emu.py) followed by the
wrapper's final rotation + sample extraction (pbs_tw.hip) equals the oracle BNF PBS bit for bit."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from test_tw_codegen import _tables

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "tfhe-rs-main_modified_amd", "csrc", "pbs_tw_body.hpp")
P = 0xFFFFFFFF00000001
N = 2048


def test_pbs_header_is_generated():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_pbs_kernel.py")], capture_output=True,
                         text=True, check=True).stdout
    assert out == open(HDR).read(), "regenerate csrc/pbs_tw_body.hpp with tools/gen_pbs_kernel.py"


def _extract(acc, body, oracle):
    """pbs_tw.hip epilogue: rotate by -ms(b), sample-extract coefficient 0."""
    glwe = np.concatenate([oracle.poly_monomial_div(acc[c], oracle.modulus_switch(body, 12)) for c in range(2)])
    return oracle.sample_extract(glwe, N, 1)


@pytest.mark.parametrize("seed,base_log", [(1, 23), (2, 10), (3, 31)])
def test_emulated_pbs_matches_oracle(oracle, seed, base_log):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_emu
    plan, tf, ti = _tables(oracle)
    ctx = oracle.NttContext(N)
    rnd = random.Random(seed)
    n_lwe = 4
    bsk = np.array([rnd.randrange(P) for _ in range(n_lwe * 4 * N)], dtype=np.uint64)
    n_inv = int(plan.n_inv)
    bsk_norm = np.array([int(v) * n_inv % P for v in bsk], dtype=np.uint64)
    lut = np.array([rnd.getrandbits(64) for _ in range(2 * N)], dtype=np.uint64)
    # mask values: ms = 0 (skipped step), ms >= N (negacyclic wrap), ms = 2047 / 1 (extremes), random
    ms_vals = [0, 2048 + 5, 2047, 1] if seed == 1 else [rnd.randrange(4096) for _ in range(n_lwe)]
    lwe = [(m << 52) + rnd.getrandbits(50) - (1 << 50) & (2**64 - 1) for m in ms_vals] + [rnd.getrandbits(64)]
    lwe = np.array(lwe, dtype=np.uint64)
    want = ctx.pbs(lwe, lut, bsk, 1, base_log, 1, bnf=True)
    acc = asm_emu.run_pbs(HDR, lwe, lut, bsk_norm, tf + ti, base_log, n_lwe)
    got = _extract(acc, int(lwe[-1]), oracle)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("cmux", [False, True])
def test_emulated_ext_product_matches_oracle(oracle, cmux):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_emu
    plan, tf, ti = _tables(oracle)
    n_inv = int(plan.n_inv)
    ti_norm = [v * n_inv % P for v in ti[:N]] + ti[N:]
    ctx = oracle.NttContext(N)
    rnd = random.Random(7 + cmux)
    ggsw = np.array([rnd.randrange(P) for _ in range(4 * N)], dtype=np.uint64)
    glwe = np.array([rnd.getrandbits(64) for _ in range(2 * N)], dtype=np.uint64)
    out = np.array([rnd.getrandbits(64) for _ in range(2 * N)], dtype=np.uint64)
    g, o = asm_emu.run_ext(HDR, glwe, out, ggsw, tf + ti + ti_norm, 23, cmux)
    if cmux:
        want = ctx.cmux(out, glwe, ggsw, 1, 23, 1, bnf=True)
        assert np.array_equal(g.reshape(-1), glwe - out)
    else:
        want = ctx.ext_product(out, ggsw, glwe, 1, 23, 1, bnf=True)
    assert np.array_equal(o.reshape(-1), want)


@pytest.mark.parametrize("base_log", [23, 10, 31, 1])
def test_emulated_decomposition_corners(oracle, base_log):
    """The level-1 decomposition of the generated body on the rounding corners: the one unbalanced tie
    (top B+1 bits = 1 0..0, i.e. x in [2^63, 2^63 + 2^(63-B))), the balanced tie just below it, the
    extremes, and both neighbours of every corner; external product vs the oracle, bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_emu
    plan, tf, ti = _tables(oracle)
    n_inv = int(plan.n_inv)
    ti_norm = [v * n_inv % P for v in ti[:N]] + ti[N:]
    ctx = oracle.NttContext(N)
    rnd = random.Random(base_log)
    q = 1 << (63 - base_log)
    corners = [1 << 63, (1 << 63) + 1, (1 << 63) + q - 1, (1 << 63) + q, (1 << 63) - 1, (1 << 63) - q,
               (1 << 63) - q - 1, 0, 1, 2**64 - 1, 2**64 - q, q - 1, q, (1 << 62), (1 << 62) - 1]
    vals = []
    for c in corners:
        vals += [(c + d) % 2**64 for d in (-1, 0, 1)]
    glwe = np.array((vals * (2 * N // len(vals) + 1))[: 2 * N], dtype=np.uint64)
    rnd.shuffle(glwe)
    ggsw = np.array([rnd.randrange(P) for _ in range(4 * N)], dtype=np.uint64)
    out = np.array([rnd.getrandbits(64) for _ in range(2 * N)], dtype=np.uint64)
    _, o = asm_emu.run_ext(HDR, glwe, out, ggsw, tf + ti + ti_norm, base_log, False)
    assert np.array_equal(o.reshape(-1), ctx.ext_product(out, ggsw, glwe, 1, base_log, 1, bnf=True))


def _sol_ms(a):
    """pbs_tw.hip's pre-switch of a Solinas mask element (ms_non_native mod 2N)."""
    import oracle as O
    return O.pbs_modulus_switch_non_native(int(a), N, P) % (2 * N)


@pytest.mark.parametrize("seed,base_log", [(1, 23), (2, 10), (3, 31), (4, 1)])
def test_emulated_solinas_pbs_matches_oracle(oracle, seed, base_log):
    """Solinas-modulus blind rotation (ntt64_pbs.rs:213-286): the body on the pre-switched mask and the
    wrapper's LUT pre-rotation / sample extraction vs the oracle PBS, bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_emu
    plan, tf, ti = _tables(oracle)
    ctx = oracle.NttContext(N)
    rnd = random.Random(100 + seed)
    n_lwe = 4
    bsk = np.array([rnd.randrange(P) for _ in range(n_lwe * 4 * N)], dtype=np.uint64)  # Normalize key
    lut = np.array([rnd.randrange(P) for _ in range(2 * N)], dtype=np.uint64)
    lut[:4] = [0, P - 1, 1, P // 2]
    # mask: 0 (skipped), values that switch to 0 / 2N / the wrap, extremes, random
    lwe = [0, P - 1, P // 2, 1] if seed == 1 else [rnd.randrange(P) for _ in range(n_lwe)]
    lwe = np.array(lwe + [rnd.randrange(P)], dtype=np.uint64)
    want = ctx.pbs(lwe, lut, bsk, 1, base_log, 1, bnf=False)
    msb = oracle.pbs_modulus_switch_non_native(int(lwe[-1]), N, P)
    acc0 = np.stack([oracle.poly_monomial_div(lut[c * N:(c + 1) * N], msb, P) for c in range(2)])
    msed = np.array([_sol_ms(a) for a in lwe[:-1]] + [0], dtype=np.uint64)
    acc = asm_emu.run_pbs(HDR, msed, lut, bsk, tf + ti, base_log, n_lwe, name="sol_l1", acc0=acc0)
    got = oracle.sample_extract(acc.reshape(-1), N, 1, P)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("cmux", [False, True])
@pytest.mark.parametrize("base_log", [23, 10, 31, 1])
def test_emulated_solinas_ext_product_corners(oracle, cmux, base_log):
    """Solinas external product / CMUX (ntt64_pbs.rs:553-702) with the non-native decomposition's
    corners: the sign threshold p/2 + 1 and its neighbours, 0, 1, p - 1 and the rounding boundaries
    k 2^(63-B) +- 1 of the magnitude, on both sides of the threshold."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_emu
    plan, tf, ti = _tables(oracle)
    ctx = oracle.NttContext(N)
    rnd = random.Random(base_log + 50 * cmux)
    half = P // 2 + 1
    q = 1 << (63 - base_log)
    corners = [half, half - 1, half + 1, P // 2, 0, 1, 2, P - 1, P - 2, q, q - 1, q // 2, q // 2 + 1, 3 * q // 2,
               (1 << 62), (1 << 63) - 1 - P // 2]
    vals = []
    for c in corners:
        for d in (-1, 0, 1):
            vals += [(c + d) % P, (P - c - d) % P]
    glwe = np.array((vals * (2 * N // len(vals) + 1))[: 2 * N], dtype=np.uint64)
    rnd.shuffle(glwe)
    ggsw = np.array([rnd.randrange(P) for _ in range(4 * N)], dtype=np.uint64)
    out = np.array([rnd.randrange(P) for _ in range(2 * N)], dtype=np.uint64)
    g, o = asm_emu.run_ext(HDR, glwe, out, ggsw, tf + ti, base_log, cmux, sol=True)
    if cmux:
        want = ctx.cmux(out, glwe, ggsw, 1, base_log, 1, bnf=False)
        assert np.array_equal(g.reshape(-1), np.array([(int(a) - int(b)) % P for a, b in zip(glwe, out)], np.uint64))
    else:
        want = ctx.ext_product(out, ggsw, glwe, 1, base_log, 1, bnf=False)
    assert np.array_equal(o.reshape(-1), want)
