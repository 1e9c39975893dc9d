"""Generate the committed golden fixtures for the prime64 NTT path.

The reference (Rust tfhe-ntt) cannot be built in this image (no cargo/rustc) and ships no
stored NTT outputs, so the fixtures are produced by the CPU oracle (oracle/ntt_oracle.c) — a
restatement pinned by the reference's own KATs and property tests (tests/test_oracle.py) — and
each fixture is self-checked here against those properties before it is written:

  * inv(fwd(x)) == N * x                                     (prime64.rs:1339-1356)
  * inv(fwd(a) (.) fwd(b)) * N^-1 == negacyclic(a, b)        (prime64.rs:1264-1361)
  * every output is canonical (< p)                          (prime64.rs:1328-1333)
(the closed form of SURVEY.md F5 is checked in tests/test_oracle.py)

Moduli: the six primes of the reference's test_product (prime64.rs:1308-1315) plus the 61-bit
prime of the pointwise tests (prime64.rs:1460) and the prime32 doc-example prime (lib.rs:31).

Run:  python tests/golden/make_golden.py     (writes tests/golden/prime64_p<p>_n<n>.npz, large_solinas_n*.npz and
      consumers_n2048.npz — the external product / CMUX / key conversion / PBS cases)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

SEED = 0x74666865


def golden_primes():
    ap = O.largest_prime_in_arithmetic_progression64
    return {
        "p50": ap(1 << 16, 1, 1 << 49, 1 << 50),
        "p51": ap(1 << 16, 1, 1 << 50, 1 << 51),
        "p61": ap(1 << 16, 1, 1 << 60, 1 << 61),
        "p62": ap(1 << 16, 1, 1 << 61, 1 << 62),
        "p63": ap(1 << 16, 1, 1 << 62, 1 << 63),
        "solinas": O.SOLINAS_P,
        "p64": ap(1 << 16, 1, 1 << 63, 2**64 - 1),
        "p30": 1062862849,
    }


SIZES = {"solinas": [16, 32, 64, 1024, 2048], "default": [16, 32, 1024]}


def make_one(name, p, n):
    batch = 3 if n < 1024 else 1
    plan = O.Plan.try_new(n, p)
    assert plan is not None, (name, n)
    seed = SEED + (n << 8) + sum(map(ord, name))
    x = O.fill_uniform(seed, p, batch * n).reshape(batch, n)
    y = O.fill_uniform(seed + 1, p, batch * n).reshape(batch, n)
    acc = O.fill_uniform(seed + 2, p, batch * n).reshape(batch, n)
    fx, fy = plan.fwd(x), plan.fwd(y)
    ix = plan.inv(x)
    # property checks before writing anything
    assert np.array_equal(plan.inv(fx), np.array([[O.mul_mod(int(v), n, p) for v in row] for row in x], np.uint64))
    if n <= 1024:
        conv = O.negacyclic_convolution(n, p, x[0], y[0])
        prod = plan.mul_assign_normalize(fx[:1], fy[:1])
        assert np.array_equal(plan.inv(prod)[0], conv)
    assert all(int(v) < p for v in fx.reshape(-1)) and all(int(v) < p for v in ix.reshape(-1))
    return dict(
        p=np.array([p], np.uint64), n=np.array([n], np.uint64),
        twid=plan.twid, inv_twid=plan.inv_twid, n_inv=np.array([plan.n_inv], np.uint64),
        x=x, y=y, acc=acc,
        fwd_x=fx, fwd_y=fy, inv_x=ix,
        normalize_fx=plan.normalize(fx),
        mul_assign_normalize_fx_fy=plan.mul_assign_normalize(fx, fy),
        mul_accumulate_acc_fx_fy=plan.mul_accumulate(acc, fx, fy),
    )


def make_large(n):
    """A single-polynomial Solinas fixture beyond one workgroup (the engine's two-pass large-N path):
    x, fwd(x), inv(x) only, self-checked by inv(fwd(x)) = N x and canonical outputs."""
    p = O.SOLINAS_P
    plan = O.Plan.try_new(n, p)
    x = O.fill_uniform(SEED + n, p, n).reshape(1, n)
    fx, ix = plan.fwd(x, threads=8), plan.inv(x, threads=8)
    back = plan.inv(fx, threads=8)
    assert all(int(b) == O.mul_mod(int(v), n, p) for b, v in zip(back[0], x[0]))
    assert int(fx.max()) < p and int(ix.max()) < p
    return dict(p=np.array([p], np.uint64), n=np.array([n], np.uint64), x=x, fwd_x=fx, inv_x=ix)


LARGE_SIZES = [32768]


def make_consumers():
    """The core_crypto consumers at the hot shape (N = 2048, k = 1, Solinas NTT), one fixed-seed case each
    (an external-product case and a BNF CMUX step with a fixed-seed GGSW; plus key conversion and
    a short PBS of both variants).  The oracle's outputs are written with their inputs; the PBS case is
    self-checked by the blind-rotation identity with a zero mask (the result is the LUT rotated by the body)."""
    n, p, k = 2048, O.SOLINAS_P, 1
    ctx = O.NttContext(n)
    s = SEED + 0xC0
    u = lambda seed, q, shape: O.fill_uniform(seed, q, int(np.prod(shape))).reshape(shape)
    d = {}
    # key conversion (Raw, native input) and (Normalize, mod-p input)
    d["bsk_std_native"] = u(s + 1, 0, (2, 1, 2, 2, n))
    d["bsk_ntt_raw"] = ctx.bsk_to_ntt(d["bsk_std_native"].reshape(-1), 64, False).reshape(2, 1, 2, 2, n)
    d["bsk_std_solinas"] = u(s + 2, p, (2, 1, 2, 2, n))
    d["bsk_ntt_normalize"] = ctx.bsk_to_ntt(d["bsk_std_solinas"].reshape(-1), 0, True).reshape(2, 1, 2, 2, n)
    # external products: BNF level 1 (B 23) and level 2 (B 12); Solinas level 1
    d["ggsw_l1"] = u(s + 3, p, (1, 2, 2, n))
    d["ggsw_l2"] = u(s + 4, p, (2, 2, 2, n))
    d["glwe_native"], d["out_native"] = u(s + 5, 0, (2, n)), u(s + 6, 0, (2, n))
    d["glwe_solinas"], d["out_solinas"] = u(s + 7, p, (2, n)), u(s + 8, p, (2, n))
    d["ext_bnf_l1"] = ctx.ext_product(d["out_native"], d["ggsw_l1"], d["glwe_native"], k, 23, 1, bnf=True)
    d["ext_bnf_l2"] = ctx.ext_product(d["out_native"], d["ggsw_l2"], d["glwe_native"], k, 12, 2, bnf=True)
    d["ext_solinas_l1"] = ctx.ext_product(d["out_solinas"], d["ggsw_l1"], d["glwe_solinas"], k, 23, 1, bnf=False)
    # one BNF CMUX step
    d["cmux_ct0"], d["cmux_ct1"] = u(s + 9, 0, (2, n)), u(s + 10, 0, (2, n))
    d["cmux_bnf_ct0"] = ctx.cmux(d["cmux_ct0"], d["cmux_ct1"], d["ggsw_l1"], k, 23, 1, bnf=True)
    # short PBS (n_lwe = 2) of both variants on the converted keys; a zero-mask input checks the identity
    d["lut_native"], d["lut_solinas"] = u(s + 11, 0, (2, n)), u(s + 12, p, (2, n))
    lwe_native = u(s + 13, 0, (3, 3))
    lwe_native[0, :2] = 0
    lwe_solinas = u(s + 14, p, (3, 3))
    d["lwe_native"], d["lwe_solinas"] = lwe_native, lwe_solinas
    d["pbs_bnf"] = np.stack([ctx.pbs(lwe_native[b], d["lut_native"], d["bsk_ntt_raw"], k, 23, 1, bnf=True)
                             for b in range(3)])
    d["pbs_solinas"] = np.stack([ctx.pbs(lwe_solinas[b], d["lut_solinas"], d["bsk_ntt_normalize"], k, 23, 1,
                                         bnf=False) for b in range(3)])
    # identity: zero mask -> sample extract of LUT * X^-round(b 2N / 2^64)
    b0 = int(lwe_native[0, 2])
    ms = ((b0 + (1 << 51)) >> 52) % (2 * n)
    lut = d["lut_native"].astype(object)
    rot = [[(lut[c][(m + ms) % n] if (m + ms) % (2 * n) < n else -lut[c][(m + ms) % n]) % 2**64 for m in range(n)]
           for c in range(2)]
    want0 = [rot[0][0]] + [(-rot[0][n - j]) % 2**64 for j in range(1, n)] + [rot[1][0]]
    assert [int(v) for v in d["pbs_bnf"][0]] == want0
    return d


def main():
    path = os.path.join(HERE, "consumers_n2048.npz")
    np.savez_compressed(path, **make_consumers())
    print("wrote", os.path.relpath(path, ROOT))
    for n in LARGE_SIZES:
        path = os.path.join(HERE, f"large_solinas_n{n}.npz")
        np.savez_compressed(path, **make_large(n))
        print("wrote", os.path.relpath(path, ROOT))
    for name, p in golden_primes().items():
        for n in SIZES.get(name, SIZES["default"]):
            if O.Plan.try_new(n, p) is None:
                continue
            d = make_one(name, p, n)
            path = os.path.join(HERE, f"prime64_{name}_n{n}.npz")
            np.savez_compressed(path, **d)
            print("wrote", os.path.relpath(path, ROOT))


if __name__ == "__main__":
    main()
