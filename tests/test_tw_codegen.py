"""CPU checks of the generated twisted-transform asm (no GPU): the committed body header matches what
tools/gen_tw_kernel.py generates, and emulating it instruction by instruction (tools/asm_emu.py) on
seeded polynomials gives the oracle's forward / inverse transform bit for bit."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "tfhe-rs-main_modified_amd", "csrc", "ntt64_tw_body.hpp")
P = 0xFFFFFFFF00000001


def test_body_header_is_generated():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_tw_kernel.py")], capture_output=True,
                         text=True, check=True).stdout
    assert out == open(HDR).read(), "regenerate csrc/ntt64_tw_body.hpp with tools/gen_tw_kernel.py"


@pytest.fixture(scope="module")
def emu():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_emu
    return asm_emu


def _tables(oracle):
    plan = oracle.Plan.try_new(2048, P)
    tw = [int(v) for v in plan.twid]
    br = lambda x, b: int(format(x, f"0{b}b")[::-1], 2)
    psi = tw[br(1, 11)]
    omega = pow(psi, 64, P)
    f, i = [], []
    for blk in range(32):
        rho = pow(psi, 2 * br(blk, 5) + 1, P)
        rinv = pow(rho, P - 2, P)
        f += [pow(rho, j, P) for j in range(64)]
        i += [pow(rinv, j, P) for j in range(64)]
    f += [pow(omega, br(g, 5), P) for g in range(32)]
    i += [pow(pow(omega, br(g, 5), P), P - 2, P) for g in range(32)]
    return plan, f, i


@pytest.mark.parametrize("seed", [1, 2])
def test_emulated_body_matches_oracle(emu, oracle, seed):
    plan, tf, ti = _tables(oracle)
    rnd = random.Random(seed)
    x = [rnd.randrange(P) for _ in range(2048)]
    if seed == 2:  # edge values
        x[:6] = [0, P - 1, 1, P - 1, 2**32 - 1, 2**32]
    got = emu.run_body(HDR, "fwd", x, tf)
    want = plan.fwd(np.array(x, dtype=np.uint64))
    assert np.array_equal(got, want)
    back = emu.run_body(HDR, "inv", [int(v) for v in want], ti)
    assert np.array_equal(back, plan.inv(want))
