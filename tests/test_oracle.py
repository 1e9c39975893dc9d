"""Pin the CPU oracle to the reference's own known-answer and property tests (no GPU).

The reference cannot be compiled here (Rust, no cargo), so these KATs/properties — copied as
*data* from the reference's test modules — are what make the oracle trustworthy.
"""
import os
import sys

import numpy as np
import pytest

SOLINAS_P = 0xFFFFFFFF00000001


def test_solinas_root_kat(oracle):
    # roots.rs:150-172 test_primitive_root_solinas
    table = [(32, 8), (64, 2198989700608), (128, 14041890976876060974), (256, 14430643036723656017),
             (512, 4440654710286119610), (1024, 8816101479115663336), (2048, 10974926054405199669),
             (4096, 1206500561358145487), (8192, 10930245224889659871), (16384, 3333600369887534767),
             (32768, 15893793146607301539)]
    for n, root in table:
        assert oracle.find_root_solinas_64(2 * n) == root
        assert oracle.exp_mod(root, 2 * n, SOLINAS_P) == 1


def test_is_prime_kat(oracle):
    # prime.rs:184-204 test_is_prime
    primes = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89, 97,
              101, 103, 107, 109, 113, 127, 131, 137, 139, 149, 151, 157, 163, 167, 173, 179, 181, 191, 193,
              197, 199, 211, 223, 227, 229, 233, 239, 241, 251, 257, 263, 269, 271, 277, 281, 283, 293, 307,
              311, 313, 317, 331, 337, 347, 349, 353, 359, 367, 373, 379, 383, 389, 397, 401, 409, 419, 421,
              431, 433, 439, 443, 449, 457, 461, 463, 467, 479, 487, 491, 499, 503, 509, 521, 523, 541, 547,
              557, 563, 569, 571, 577, 587, 593, 599, 601, 607, 613, 617, 619, 631, 641, 643, 647, 653, 659,
              661, 673, 677, 683, 691, 701, 709, 719, 727, 733, 739, 743, 751, 757, 761, 769, 773, 787, 797,
              809, 811, 821, 823, 827, 829, 839, 853, 857, 859, 863, 877, 881, 883, 887, 907, 911, 919, 929,
              937, 941, 947, 953, 967, 971, 977, 983, 991, 997]
    ps = set(primes)
    for n in range(1000):
        assert oracle.is_prime64(n) == (n in ps), n
    assert oracle.is_prime64(SOLINAS_P)


def test_prime_search_kat(oracle):
    # prime.rs:199-213 test_prime_search
    f = oracle.largest_prime_in_arithmetic_progression64
    M = 2**64 - 1
    assert f(0, 2, 1, 4) == 2
    assert f(0, 2, 2, 2) == 2
    assert f(0, 2, 2, 1) is None
    assert f(1, 0, 14, 16) is None
    assert f(1, 0, 14, 17) == 17
    assert f(1, 0, 17, 18) == 17
    assert f(2, 1, 14, 16) is None
    assert f(2, 1, 14, 17) == 17
    assert f(2, 1, 17, 18) == 17
    assert f(6, 5, 0, M) == 18446744073709551557
    assert f(6, 1, 0, M) == 18446744073709551427


def test_plan_none_cases(oracle):
    # prime64.rs:1988-1990 test_plan_crash_github_11 + the try_new guards prime64.rs:769-775
    assert oracle.Plan.try_new(2048, 1024) is None
    assert oracle.Plan.try_new(8, SOLINAS_P) is None
    assert oracle.Plan.try_new(48, SOLINAS_P) is None
    assert oracle.Plan.try_new(2048, 2**61 - 1) is None  # prime, but 4096 does not divide p-1
    assert oracle.Plan.try_new(16, SOLINAS_P) is not None


def test_tonelli_shanks_roots(oracle):
    # roots for the reference's test primes (values restated in SURVEY.md §8c)
    f = oracle.largest_prime_in_arithmetic_progression64
    cases = {
        f(1 << 16, 1, 1 << 61, 1 << 62): (2953159431647451165, 3710688476054411196),
        f(1 << 16, 1, 1 << 62, 1 << 63): (1982205562075138180, 524101119581882958),
        f(1 << 16, 1, 1 << 63, 2**64 - 1): (16689193157577585518, 6356787237574732451),
        f(1 << 16, 1, 1 << 60, 1 << 61): (1275689310943844420, 632406636641850464),
    }
    assert list(cases) == [4611686018427322369, 9223372036853661697, 18446744073707716609, 2305843009211662337]
    for p, (r1024, r2048) in cases.items():
        assert oracle.find_primitive_root64(p, 2048) == r1024
        assert oracle.find_primitive_root64(p, 4096) == r2048
    assert oracle.find_primitive_root64(1062862849, 2048) == 306208274
    assert oracle.find_primitive_root64(1062862849, 4096) == 675605923


def _test_primes(oracle):
    f = oracle.largest_prime_in_arithmetic_progression64
    return [f(1 << 16, 1, 1 << 49, 1 << 50), f(1 << 16, 1, 1 << 50, 1 << 51), f(1 << 16, 1, 1 << 61, 1 << 62),
            f(1 << 16, 1, 1 << 62, 1 << 63), SOLINAS_P, f(1 << 16, 1, 1 << 63, 2**64 - 1)]


@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 512, 1024])
def test_product_property(oracle, n):
    # prime64.rs:1305-1361 test_product, restated against the oracle
    for i, p in enumerate(_test_primes(oracle)):
        plan = oracle.Plan.try_new(n, p)
        lhs = oracle.fill_uniform(1000 + 7 * n + i, p, n)
        rhs = oracle.fill_uniform(2000 + 7 * n + i, p, n)
        conv = oracle.negacyclic_convolution(n, p, lhs, rhs)
        lf, rf = plan.fwd(lhs), plan.fwd(rhs)
        assert int(lf.max()) < p and int(rf.max()) < p
        prod = np.array([oracle.mul_mod(int(a), int(b), p) for a, b in zip(lf, rf)], np.uint64)
        prod = plan.inv(prod)
        assert int(prod.max()) < p
        assert all(int(prod[k]) == oracle.mul_mod(int(conv[k]), n, p) for k in range(n))
        assert np.array_equal(plan.inv(plan.mul_assign_normalize(lf, rf)), conv)


def test_closed_form_f5(oracle):
    # fwd(x)[j] = sum_i x_i psi^((2 bitrev(j) + 1) i); fwd(e_0) = 1, fwd(e_1)[j] = psi^(2brev(j)+1)
    n, p, psi = 2048, SOLINAS_P, 10974926054405199669
    plan = oracle.Plan.try_new(n, p)
    e0 = np.zeros(n, np.uint64); e0[0] = 1
    assert np.all(plan.fwd(e0) == 1)
    e1 = np.zeros(n, np.uint64); e1[1] = 1
    f = plan.fwd(e1)
    br = lambda j: int(format(j, "011b")[::-1], 2)
    for j in range(0, n, 13):
        assert int(f[j]) == oracle.exp_mod(psi, 2 * br(j) + 1, p)
    # inverse is the unnormalised inverse: inv(fwd(x)) = N x
    x = oracle.fill_uniform(7, p, n)
    assert np.array_equal(plan.inv(plan.fwd(x)), np.array([oracle.mul_mod(int(v), n, p) for v in x], np.uint64))


def test_prime32_doc_roundtrip(oracle):
    # lib.rs:25-49 (prime32 doc example, p = 1062862849, N = 32) through the prime64 plan
    p, n = 1062862849, 32
    plan = oracle.Plan.try_new(n, p)
    data = np.arange(n, dtype=np.uint64)
    assert np.array_equal(plan.inv(plan.fwd(data)), data * n)


def test_pointwise_ops(oracle):
    # prime64.rs:1457-1555: pointwise ops vs u128 arithmetic
    for p in _test_primes(oracle):
        n = 128
        plan = oracle.Plan.try_new(n, p)
        a, b, c = (oracle.fill_uniform(s, p, n) for s in (11, 12, 13))
        ninv = oracle.exp_mod(n, p - 2, p)
        assert plan.n_inv == ninv
        mul = lambda u, v: (int(u) * int(v)) % p
        assert [int(v) for v in plan.normalize(a)] == [mul(x, ninv) for x in a]
        assert [int(v) for v in plan.mul_assign_normalize(a, b)] == [mul(mul(x, y), ninv) for x, y in zip(a, b)]
        assert [int(v) for v in plan.mul_accumulate(c, a, b)] == [(int(z) + mul(x, y)) % p for x, y, z in zip(a, b, c)]


def test_avx512_baseline_matches_scalar(oracle):
    if not oracle.have_avx512():
        pytest.skip("host lacks AVX-512F")
    for n in (16, 32, 1024, 2048, 4096):
        plan = oracle.Plan.try_new(n, SOLINAS_P)
        x = oracle.fill_uniform(99 + n, SOLINAS_P, 8 * n)
        y = x.copy()
        assert plan.fwd_avx512_inplace(y, 2)
        assert np.array_equal(y, plan.fwd(x))
        z = y.copy()
        assert plan.inv_avx512_inplace(z, 2)
        assert np.array_equal(z, plan.inv(y))


def test_generator_range(oracle):
    for p in (SOLINAS_P, 1062862849, 2**62 + 1, 0):
        v = oracle.fill_uniform(5, p, 4096)
        if p:
            assert int(v.max()) < p
    assert len(set(oracle.fill_uniform(5, SOLINAS_P, 4096).tolist())) == 4096


@pytest.mark.parametrize("logn", [12, 13, 14, 15, 16, 17])
def test_split_factorisation(logn):
    """The split transform's factorisation (ntt64_kernels.hip launch_ntt_split): t = log2 N - 11 reference stages, the
    block twist alpha_b^j, the 2048-point plan's transform per block == the N-point oracle transform, both directions."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import check_split_factorisation as C
    assert C.check(logn) == (True, True)
