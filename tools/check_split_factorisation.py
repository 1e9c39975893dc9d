#!/usr/bin/env python3
"""CPU check of the split transform's factorisation (ntt64_kernels.hip launch_ntt_split) against the oracle.

forward_N = the reference's first t = log2 N - 11 CT stages (generic_solinas.rs:449-481, twid[m + i]), then per
2048-block b: element j times alpha_b^j, alpha_b = psi_N^(2 bitrev_t(b) + 1 - 2^t mod 2N), then the N = 2048 forward
of the 2048-point Solinas plan.  inverse_N = per block the 2048 inverse, times alpha_b^-j, then the t GS stages in
reverse (generic_solinas.rs:483-514), unnormalised.  Test infrastructure only (imports the oracle).

  python tools/check_split_factorisation.py [log2N ...]     (default 12 13 14)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import oracle as O  # noqa: E402

P = 0xFFFFFFFF00000001


def br(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def alpha_exponent(b, t, n):
    return (2 * br(b, t) + 1 - (1 << t)) % (2 * n)


def check(logn, seed=7):
    n, t = 1 << logn, logn - 11
    plan, p2048 = O.Plan.try_new(n, P), O.Plan.try_new(2048, P)
    tw = np.array([int(v) for v in plan.twid], dtype=object)
    itw = np.array([int(v) for v in plan.inv_twid], dtype=object)
    psi = int(tw[br(1, logn)])
    x = O.fill_uniform(seed + logn, P, n)
    ref = plan.fwd(x.copy())
    y = np.array([int(v) for v in x], dtype=object)
    for s in range(t):  # CT stage with m = 2^s groups, pair distance n / 2m
        m, half = 1 << s, n >> (s + 1)
        v = y.reshape(m, 2, half)
        w = tw[m:2 * m].reshape(m, 1)
        b = (v[:, 1, :] * w) % P
        v[:, 0, :], v[:, 1, :] = (v[:, 0, :] + b) % P, (v[:, 0, :] - b) % P
    out = np.zeros(n, np.uint64)
    j = np.arange(2048)
    for b in range(1 << t):
        a = pow(psi, alpha_exponent(b, t, n), P)
        pw = np.array([pow(a, int(k), P) for k in j], dtype=object)
        out[b * 2048:(b + 1) * 2048] = p2048.fwd(np.array((y[b * 2048:(b + 1) * 2048] * pw) % P, dtype=np.uint64))
    fwd_ok = np.array_equal(out, ref)
    z = np.zeros(n, dtype=object)
    for b in range(1 << t):
        ai = pow(pow(psi, alpha_exponent(b, t, n), P), P - 2, P)
        pw = np.array([pow(ai, int(k), P) for k in j], dtype=object)
        blk = p2048.inv(ref[b * 2048:(b + 1) * 2048].copy()).astype(object)
        z[b * 2048:(b + 1) * 2048] = (blk * pw) % P
    for s in reversed(range(t)):  # GS stage, m = 2^s groups
        m, half = 1 << s, n >> (s + 1)
        v = z.reshape(m, 2, half)
        w = itw[m:2 * m].reshape(m, 1)
        a0, a1 = v[:, 0, :].copy(), v[:, 1, :].copy()
        v[:, 0, :], v[:, 1, :] = (a0 + a1) % P, ((a0 - a1) * w) % P
    inv_ok = np.array_equal(np.array(z, dtype=np.uint64), plan.inv(ref.copy()))
    return fwd_ok, inv_ok


if __name__ == "__main__":
    for lg in [int(a) for a in sys.argv[1:]] or [12, 13, 14]:
        print(f"N = 2^{lg}: forward, inverse == oracle:", check(lg))
