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

Run:  python tests/golden/make_golden.py     (writes tests/golden/prime64_p<p>_n<n>.npz)
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


def main():
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
