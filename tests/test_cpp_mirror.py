"""The C++ host mirror of prime64::Plan (include/tfhe_ntt_amd.hpp) running the reference's own
prime64.rs tests (tests/cpp/test_prime64.cpp).

CPU: the mirror builds against the C ABI, its try_new None cases pass without a device, and the
hard-coded test primes equal the oracle's restatement of largest_prime_in_arithmetic_progression64
(prime.rs).  GPU: the full restated suite (test_product over 6 primes x N = 16..1024,
normalize / mul_assign_normalize / mul_accumulate vs u128 %, slice-length panics).
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")
BIN = os.path.join(CPP, "test_prime64")


def _build():
    subprocess.run(["make", "-C", CPP, "-s"], check=True)
    assert os.path.exists(BIN)


def test_mirror_builds_and_none_cases_pass():
    _build()
    r = subprocess.run([BIN, "--cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "passed" in r.stdout


def test_hardcoded_primes_match_oracle(oracle):
    src = open(os.path.join(CPP, "test_prime64.cpp")).read()
    lists = {name: [int(v) if v != "SOLINAS" else 0xFFFFFFFF00000001 for v in re.findall(r"(\d+)ull|(SOLINAS)", body) for v in v if v]
             for name, body in re.findall(r"(PRODUCT_PRIMES|MACC_PRIMES)\[\] = \{([^}]*)\}", src)}
    f = oracle.largest_prime_in_arithmetic_progression64
    M = 2**64 - 1
    assert lists["PRODUCT_PRIMES"] == [f(1 << 16, 1, 1 << 49, 1 << 50), f(1 << 16, 1, 1 << 50, 1 << 51),
                                       f(1 << 16, 1, 1 << 61, 1 << 62), f(1 << 16, 1, 1 << 62, 1 << 63),
                                       0xFFFFFFFF00000001, f(1 << 16, 1, 1 << 63, M)]
    assert lists["MACC_PRIMES"] == [f(1 << 16, 1, 0, 1 << 51), f(1 << 16, 1, 0, 1 << 61),
                                    f(1 << 16, 1, 0, 1 << 62), f(1 << 16, 1, 0, 1 << 63), f(1 << 16, 1, 0, M)]


@pytest.mark.gpu
def test_mirror_reference_suite_on_gpu():
    assert os.path.exists(BIN), "tests/cpp/test_prime64 must be built beforehand (__graft_entry__.build())"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "all tests passed" in r.stdout


@pytest.mark.gpu
def test_core_crypto_mirror_on_gpu():
    """C++ core_crypto mirror (key conversion, external product, PBS, keyswitch) vs the oracle."""
    exe = os.path.join(CPP, "test_core_crypto")
    assert os.path.exists(exe), "tests/cpp/test_core_crypto must be built beforehand (__graft_entry__.build())"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "all tests passed" in r.stdout
