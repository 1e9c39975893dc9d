"""ctypes view of the CPU oracle (oracle/libntt_oracle.so).

TEST INFRASTRUCTURE ONLY.  This module is imported by tests/, by
``__graft_entry__.smoke()`` and by ``bench.py``'s ``cpu_baseline`` leg — as the
*checker* and the CPU baseline, never as the thing measured or shipped.  The
product package (``tfhe-rs-main_modified_amd/``) never imports it.

Every function restates the reference named in ``ntt_oracle.h`` /
``pbs_oracle.h`` (file:line citations live next to each C function).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libntt_oracle.so")

SOLINAS_P = 0xFFFFFFFF00000001

_u64 = ctypes.c_uint64
_sz = ctypes.c_size_t
_p64 = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc only; no reference sources are used)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        sigs = {
            "ora_mul_mod": (_u64, [_u64, _u64, _u64]),
            "ora_exp_mod": (_u64, [_u64, _u64, _u64]),
            "ora_is_prime64": (ctypes.c_int, [_u64]),
            "ora_largest_prime_in_ap": (ctypes.c_int, [_u64, _u64, _u64, _u64, _p64]),
            "ora_find_primitive_root64": (ctypes.c_int, [_u64, _u64, _p64]),
            "ora_find_root_solinas64": (ctypes.c_int, [_u64, _p64]),
            "ora_plan_init": (ctypes.c_int, [_sz, _u64, _p64, _p64, _p64]),
            "ora_fwd": (None, [_sz, _u64, _p64, _p64]),
            "ora_inv": (None, [_sz, _u64, _p64, _p64]),
            "ora_fwd_batch": (None, [_sz, _u64, _p64, _p64, _sz, _sz, ctypes.c_int]),
            "ora_inv_batch": (None, [_sz, _u64, _p64, _p64, _sz, _sz, ctypes.c_int]),
            "ora_mul_accumulate": (None, [_sz, _u64, _p64, _p64, _p64]),
            "ora_normalize": (None, [_sz, _u64, _u64, _p64]),
            "ora_mul_assign_normalize": (None, [_sz, _u64, _u64, _p64, _p64]),
            "ora_negacyclic_convolution": (None, [_sz, _u64, _p64, _p64, _p64]),
            "ora_have_avx512": (ctypes.c_int, []),
            "ora_fwd_batch_avx512": (ctypes.c_int, [_sz, _p64, _p64, _sz, _sz, ctypes.c_int]),
            "ora_inv_batch_avx512": (ctypes.c_int, [_sz, _p64, _p64, _sz, _sz, ctypes.c_int]),
            "ora_fill_uniform": (None, [_u64, _u64, _p64, _sz]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_p64)


def _opt(fn, *args):
    out = _u64(0)
    ok = fn(*args, ctypes.byref(out))
    return int(out.value) if ok else None


# ---- number theory -------------------------------------------------------
def mul_mod(a, b, p):
    return int(lib().ora_mul_mod(a, b, p))


def exp_mod(base, pow_, p):
    return int(lib().ora_exp_mod(base, pow_, p))


def is_prime64(n):
    return bool(lib().ora_is_prime64(n))


def largest_prime_in_arithmetic_progression64(factor, offset, lo, hi):
    return _opt(lib().ora_largest_prime_in_ap, factor, offset, lo, hi)


def find_primitive_root64(p, degree):
    return _opt(lib().ora_find_primitive_root64, p, degree)


def find_root_solinas_64(degree):
    return _opt(lib().ora_find_root_solinas64, degree)


# ---- Plan ------------------------------------------------------------------
class Plan:
    """Oracle twin of ``tfhe_ntt::prime64::Plan`` (prime64.rs:245-1222)."""

    def __init__(self, n, p, twid, inv_twid, n_inv):
        self.n, self.p, self.twid, self.inv_twid, self.n_inv = n, p, twid, inv_twid, n_inv

    @staticmethod
    def try_new(n: int, p: int):
        twid = np.zeros(max(n, 1), np.uint64)
        inv = np.zeros(max(n, 1), np.uint64)
        n_inv = _u64(0)
        ok = lib().ora_plan_init(n, p, _ptr(twid), _ptr(inv), ctypes.byref(n_inv))
        return Plan(n, p, twid, inv, int(n_inv.value)) if ok else None

    def ntt_size(self):
        return self.n

    def modulus(self):
        return self.p

    def _batch(self, buf):
        buf = np.ascontiguousarray(buf, dtype=np.uint64)
        assert buf.size % self.n == 0, "buffer length must be a multiple of the NTT size"
        return buf

    def fwd(self, buf: np.ndarray, threads: int = 1) -> np.ndarray:
        out = self._batch(buf).copy()
        lib().ora_fwd_batch(self.n, self.p, _ptr(self.twid), _ptr(out), out.size // self.n, self.n, threads)
        return out.reshape(np.shape(buf))

    def inv(self, buf: np.ndarray, threads: int = 1) -> np.ndarray:
        out = self._batch(buf).copy()
        lib().ora_inv_batch(self.n, self.p, _ptr(self.inv_twid), _ptr(out), out.size // self.n, self.n, threads)
        return out.reshape(np.shape(buf))

    def normalize(self, x):
        out = self._batch(x).copy()
        lib().ora_normalize(out.size, self.p, self.n_inv, _ptr(out))
        return out.reshape(np.shape(x))

    def mul_assign_normalize(self, lhs, rhs):
        out = self._batch(lhs).copy()
        r = np.ascontiguousarray(rhs, dtype=np.uint64).reshape(-1)
        lib().ora_mul_assign_normalize(out.size, self.p, self.n_inv, _ptr(out), _ptr(r))
        return out.reshape(np.shape(lhs))

    def mul_accumulate(self, acc, lhs, rhs):
        out = self._batch(acc).copy()
        l = np.ascontiguousarray(lhs, dtype=np.uint64).reshape(-1)
        r = np.ascontiguousarray(rhs, dtype=np.uint64).reshape(-1)
        lib().ora_mul_accumulate(out.size, self.p, _ptr(out), _ptr(l), _ptr(r))
        return out.reshape(np.shape(acc))

    # CPU baseline (restated AVX-512 fast path, Solinas only)
    def fwd_avx512_inplace(self, buf: np.ndarray, threads: int) -> bool:
        assert self.p == SOLINAS_P
        return bool(lib().ora_fwd_batch_avx512(self.n, _ptr(self.twid), _ptr(buf), buf.size // self.n, self.n, threads))

    def inv_avx512_inplace(self, buf: np.ndarray, threads: int) -> bool:
        assert self.p == SOLINAS_P
        return bool(lib().ora_inv_batch_avx512(self.n, _ptr(self.inv_twid), _ptr(buf), buf.size // self.n, self.n, threads))

    def fwd_scalar_inplace(self, buf: np.ndarray, threads: int) -> None:
        lib().ora_fwd_batch(self.n, self.p, _ptr(self.twid), _ptr(buf), buf.size // self.n, self.n, threads)

    def inv_scalar_inplace(self, buf: np.ndarray, threads: int) -> None:
        lib().ora_inv_batch(self.n, self.p, _ptr(self.inv_twid), _ptr(buf), buf.size // self.n, self.n, threads)


def have_avx512() -> bool:
    return bool(lib().ora_have_avx512())


def negacyclic_convolution(n, p, lhs, rhs):
    out = np.zeros(n, np.uint64)
    l = np.ascontiguousarray(lhs, dtype=np.uint64)
    r = np.ascontiguousarray(rhs, dtype=np.uint64)
    lib().ora_negacyclic_convolution(n, p, _ptr(l), _ptr(r), _ptr(out))
    return out


def fill_uniform(seed: int, p: int, count: int) -> np.ndarray:
    out = np.zeros(count, np.uint64)
    lib().ora_fill_uniform(seed & 0xFFFFFFFFFFFFFFFF, p, _ptr(out), count)
    return out


# ---- core_crypto consumers (pbs_oracle.h) ------------------------------------------------
class _Tables(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("p", ctypes.c_uint64), ("twid", _p64), ("inv_twid", _p64),
                ("n_inv", ctypes.c_uint64)]


_PBS_SIGS = {
    "ora_decomp_init_native": (_u64, [_u64, ctypes.c_int, ctypes.c_int]),
    "ora_decompose_one_level": (_u64, [ctypes.c_int, _p64]),
    "ora_modswitch_p2_to_prime": (_u64, [_u64, ctypes.c_uint, _u64]),
    "ora_modswitch_prime_to_p2": (_u64, [_u64, ctypes.c_uint, _u64]),
    "ora_modulus_switch": (_u64, [_u64, ctypes.c_uint]),
    "ora_pbs_modulus_switch_non_native": (_u64, [_u64, _sz, _u64]),
    "ora_poly_monomial_mul": (None, [_p64, _sz, _sz, _u64]),
    "ora_poly_monomial_div": (None, [_p64, _sz, _sz, _u64]),
    "ora_sample_extract": (None, [_p64, _p64, _sz, ctypes.c_int, _u64]),
}
_T = ctypes.POINTER(_Tables)
for _name in ("ora_ext_product_bnf", "ora_ext_product_solinas"):
    _PBS_SIGS[_name] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64])
for _name in ("ora_cmux_bnf", "ora_cmux_solinas"):
    _PBS_SIGS[_name] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64])
_PBS_SIGS["ora_blind_rotate_bnf"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _u64, _p64, _sz])
for _name in ("ora_pbs_bnf", "ora_pbs_solinas"):
    _PBS_SIGS[_name] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _p64, _sz])
_PBS_SIGS["ora_bsk_to_ntt"] = (None, [_T, _p64, _p64, _sz, ctypes.c_uint, ctypes.c_int])
_PBS_SIGS["ora_pbs_bnf_batch"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _p64, _sz, _sz,
                                         ctypes.c_int, ctypes.c_int])
_PBS_SIGS["ora_pbs_bnf_ms"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _p64, _sz, ctypes.c_int])
_PBS_SIGS["ora_centered_ms_body_correction"] = (_u64, [_p64, _sz, ctypes.c_uint])
_PBS_SIGS["ora_pbs_set_fast_ntt"] = (None, [ctypes.c_int])
_PBS_SIGS["ora_pbs_solinas_batch"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _p64, _sz, _sz,
                                         ctypes.c_int])
_PBS_SIGS["ora_ext_product_bnf_batch"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _sz, ctypes.c_int])
_PBS_SIGS["ora_blind_rotate_solinas"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _sz,
                                              ctypes.c_int])
_PBS_SIGS["ora_sample_extract_nth"] = (None, [_p64, _p64, _sz, ctypes.c_int, _sz, _u64])
_PBS_SIGS["ora_blind_rotate_bnf_batch"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64, _sz,
                                                _sz, ctypes.c_int, ctypes.c_int])
_PBS_SIGS["ora_blind_rotate_solinas_batch"] = (None, [_T, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64, _p64, _p64,
                                                    _sz, _sz, ctypes.c_int, ctypes.c_int])
_PBS_SIGS["ora_ntt64_view_forward_batch"] = (None, [_T, ctypes.c_int, ctypes.c_uint, ctypes.c_int, _p64, _p64, _sz,
                                                   _sz, ctypes.c_int])
_PBS_SIGS["ora_ntt64_view_add_backward_batch"] = (None, [_T, ctypes.c_uint, _p64, _p64, _sz, _sz, ctypes.c_int])
_PBS_SIGS["ora_lwe_ms64"] = (None, [_p64, _sz, ctypes.c_uint, ctypes.c_int, _p64])
_pbs_ready = False


def _plib():
    global _pbs_ready
    L = lib()
    if not _pbs_ready:
        for name, (res, args) in _PBS_SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _pbs_ready = True
    return L


def _u(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


class NttContext:
    """Oracle twin of core_crypto's Ntt64 + the NTT PBS algorithms for one (N, p)."""

    def __init__(self, n: int, p: int = SOLINAS_P):
        self.plan = Plan.try_new(n, p)
        assert self.plan is not None
        self.n, self.p = n, p
        self._t = _Tables(n, p, _ptr(self.plan.twid), _ptr(self.plan.inv_twid), self.plan.n_inv)

    @property
    def tables(self):
        return ctypes.byref(self._t)

    def ext_product(self, out, ggsw, glwe, k, base_log, level, bnf=True):
        out = _u(out).copy()
        fn = _plib().ora_ext_product_bnf if bnf else _plib().ora_ext_product_solinas
        fn(self.tables, k, base_log, level, _ptr(out), _ptr(_u(ggsw)), _ptr(_u(glwe)))
        return out

    def ext_product_batch_bnf(self, out, ggsw, glwe, k, base_log, level, threads=8):
        out = _u(out).copy()
        batch = out.size // ((k + 1) * self.n)
        _plib().ora_ext_product_bnf_batch(self.tables, k, base_log, level, _ptr(out), _ptr(_u(ggsw)),
                                         _ptr(_u(glwe)), batch, threads)
        return out

    def cmux(self, ct0, ct1, ggsw, k, base_log, level, bnf=True):
        ct0, ct1 = _u(ct0).copy(), _u(ct1).copy()
        fn = _plib().ora_cmux_bnf if bnf else _plib().ora_cmux_solinas
        fn(self.tables, k, base_log, level, _ptr(ct0), _ptr(ct1), _ptr(_u(ggsw)))
        return ct0

    def blind_rotate_bnf(self, acc, msed_mask, msed_body, bsk, k, base_log, level):
        acc = _u(acc).copy()
        m = _u(msed_mask)
        _plib().ora_blind_rotate_bnf(self.tables, k, base_log, level, _ptr(acc), _ptr(m), int(msed_body),
                                     _ptr(_u(bsk)), m.size)
        return acc

    def blind_rotate_solinas(self, acc, lwe_in, bsk, k, base_log, level, pre_switched=False):
        acc = _u(acc).copy()
        lwe_in = _u(lwe_in)
        _plib().ora_blind_rotate_solinas(self.tables, k, base_log, level, _ptr(acc), _ptr(lwe_in), _ptr(_u(bsk)),
                                         lwe_in.size - 1, int(pre_switched))
        return acc

    def blind_rotate_batch(self, acc, lwe_in, bsk, k, base_log, level, bnf=True, ms_mode=0, threads=8):
        """acc (batch, k+1, N) rotated item by item (a new array); BNF ms_mode 0 standard / 1 centered / 2 pre-switched,
        Solinas 0 (raw mod p) or 2 (pre-switched)."""
        acc = _u(acc).copy()
        lwe_in = _u(lwe_in)
        batch, n_lwe = lwe_in.shape[0], lwe_in.shape[1] - 1
        if bnf:
            _plib().ora_blind_rotate_bnf_batch(self.tables, k, base_log, level, _ptr(acc), _ptr(lwe_in), _ptr(_u(bsk)),
                                               n_lwe, batch, int(ms_mode), threads)
        else:
            assert ms_mode in (0, 2)
            _plib().ora_blind_rotate_solinas_batch(self.tables, k, base_log, level, _ptr(acc), _ptr(lwe_in),
                                                   _ptr(_u(bsk)), n_lwe, batch, int(ms_mode == 2), threads)
        return acc

    def pbs(self, lwe_in, lut, bsk, k, base_log, level, bnf=True, centered=False):
        lwe_in = _u(lwe_in)
        out = np.zeros(k * self.n + 1, np.uint64)
        if bnf:
            _plib().ora_pbs_bnf_ms(self.tables, k, base_log, level, _ptr(out), _ptr(lwe_in), _ptr(_u(lut)),
                                   _ptr(_u(bsk)), lwe_in.size - 1, int(centered))
        else:
            assert not centered
            _plib().ora_pbs_solinas(self.tables, k, base_log, level, _ptr(out), _ptr(lwe_in), _ptr(_u(lut)),
                                    _ptr(_u(bsk)), lwe_in.size - 1)
        return out

    def pbs_batch_bnf(self, lwe_in, lut, bsk, k, base_log, level, threads=8, centered=False, out=None):
        lwe_in = _u(lwe_in)
        batch, n_lwe = lwe_in.shape[0], lwe_in.shape[1] - 1
        if out is None:
            out = np.zeros((batch, k * self.n + 1), np.uint64)
        _plib().ora_pbs_bnf_batch(self.tables, k, base_log, level, _ptr(out), _ptr(lwe_in), _ptr(_u(lut)),
                                  _ptr(_u(bsk)), n_lwe, batch, int(centered), threads)
        return out

    def pbs_batch_solinas(self, lwe_in, lut, bsk, k, base_log, level, threads=8, out=None):
        lwe_in = _u(lwe_in)
        batch, n_lwe = lwe_in.shape[0], lwe_in.shape[1] - 1
        if out is None:
            out = np.zeros((batch, k * self.n + 1), np.uint64)
        _plib().ora_pbs_solinas_batch(self.tables, k, base_log, level, _ptr(out), _ptr(lwe_in), _ptr(_u(lut)),
                                      _ptr(_u(bsk)), n_lwe, batch, threads)
        return out

    def bsk_to_ntt(self, bsk_std, in_width=64, normalize=False):
        src = _u(bsk_std)
        dst = np.zeros_like(src)
        _plib().ora_bsk_to_ntt(self.tables, _ptr(src), _ptr(dst), src.size // self.n, in_width, int(normalize))
        return dst


    # ---- the Ntt64View layer (ntt64.rs:89-266), over a (batch, N) array (new arrays returned) ----
    def _view_fwd(self, kind, width, normalize, standard, threads):
        src = _u(standard).reshape(-1, self.n)
        dst = np.zeros_like(src)
        _plib().ora_ntt64_view_forward_batch(self.tables, kind, width, int(normalize), _ptr(dst), _ptr(src),
                                             src.shape[0], self.n, threads)
        return dst.reshape(np.shape(standard))

    def forward(self, standard, threads=8):
        return self._view_fwd(0, 0, False, standard, threads)

    def forward_normalized(self, standard, threads=8):
        return self._view_fwd(0, 0, True, standard, threads)

    def forward_from_power_of_two_modulus(self, input_modulus_width, standard, threads=8):
        return self._view_fwd(1, input_modulus_width, False, standard, threads)

    def forward_from_decomp(self, decomp, threads=8):
        return self._view_fwd(2, 0, False, decomp, threads)

    def _view_add(self, width, standard, ntt, threads):
        st = _u(standard).reshape(-1, self.n).copy()
        y = _u(ntt).reshape(-1, self.n).copy()
        _plib().ora_ntt64_view_add_backward_batch(self.tables, width, _ptr(st), _ptr(y), st.shape[0], self.n, threads)
        return st.reshape(np.shape(standard)), y.reshape(np.shape(ntt))

    def add_backward(self, standard, ntt, threads=8):
        """-> (standard after the call, ntt after the call)"""
        return self._view_add(0, standard, ntt, threads)

    def add_backward_on_power_of_two_modulus(self, output_modulus_width, standard, ntt, threads=8):
        return self._view_add(output_modulus_width, standard, ntt, threads)


def pbs_set_fast_ntt(on: bool) -> None:
    """Route the PBS restatement's transforms through the AVX-512 restatement (CPU baseline only)."""
    _plib().ora_pbs_set_fast_ntt(int(on))


def centered_ms_body_correction(mask, log_modulus):
    m = _u(mask)
    return int(_plib().ora_centered_ms_body_correction(_ptr(m), m.size, log_modulus))


def decomp_init_native(x, base_log, level):
    return int(_plib().ora_decomp_init_native(x, base_log, level))


def decompose_one_level(base_log, state):
    s = _u64(state)
    t = _plib().ora_decompose_one_level(base_log, ctypes.byref(s))
    return int(t), int(s.value)


def modswitch_p2_to_prime(v, width, p=SOLINAS_P):
    return int(_plib().ora_modswitch_p2_to_prime(v, width, p))


def modswitch_prime_to_p2(v, width, p=SOLINAS_P):
    return int(_plib().ora_modswitch_prime_to_p2(v, width, p))


def modulus_switch(x, log_modulus):
    return int(_plib().ora_modulus_switch(x, log_modulus))


def pbs_modulus_switch_non_native(x, n, q):
    return int(_plib().ora_pbs_modulus_switch_non_native(x, n, q))


def poly_monomial_mul(poly, degree, q=0):
    a = _u(poly).copy()
    _plib().ora_poly_monomial_mul(_ptr(a), a.size, degree, q)
    return a


def poly_monomial_div(poly, degree, q=0):
    a = _u(poly).copy()
    _plib().ora_poly_monomial_div(_ptr(a), a.size, degree, q)
    return a


def sample_extract(glwe, n, k, q=0):
    out = np.zeros(k * n + 1, np.uint64)
    _plib().ora_sample_extract(_ptr(_u(glwe)), _ptr(out), n, k, q)
    return out


def sample_extract_nth(glwe, n, k, nth, q=0):
    out = np.zeros(k * n + 1, np.uint64)
    _plib().ora_sample_extract_nth(_ptr(_u(glwe)), _ptr(out), n, k, nth, q)
    return out


# ---- LWE keyswitch (ks_oracle.h) ---------------------------------------------------------
_KS_SIGS = {
    "ora_lwe_keyswitch": (None, [_p64, _sz, _sz, ctypes.c_int, ctypes.c_int, _p64, _p64]),
    "ora_lwe_keyswitch_batch": (None, [_p64, _sz, _sz, ctypes.c_int, ctypes.c_int, _p64, _p64, _sz, ctypes.c_int]),
    "ora_lwe_keyswitch32_batch": (None, [ctypes.c_void_p, _sz, _sz, ctypes.c_int, ctypes.c_int, ctypes.c_int, _p64,
                                         ctypes.c_void_p, _sz, ctypes.c_int]),
    "ora_lwe_ms32": (None, [ctypes.c_void_p, _sz, ctypes.c_int, ctypes.c_int, _p64]),
}
_ks_ready = False


def _klib():
    global _ks_ready
    L = lib()
    if not _ks_ready:
        for name, (res, args) in _KS_SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _ks_ready = True
    return L


def lwe_keyswitch(ksk, lwe_in, out_dim, base_log, level, threads=8):
    """keyswitch_lwe_ciphertext (lwe_keyswitch.rs:137-227) over a batch: lwe_in (..., in_dim + 1),
    ksk (in_dim, level, out_dim + 1) -> (..., out_dim + 1)."""
    k = _u(ksk)
    x = _u(lwe_in)
    in_dim = x.shape[-1] - 1
    assert k.size == in_dim * level * (out_dim + 1), "ksk shape"
    batch = x.size // (in_dim + 1)
    out = np.zeros(x.shape[:-1] + (out_dim + 1,), np.uint64)
    _klib().ora_lwe_keyswitch_batch(_ptr(k), in_dim, out_dim, base_log, level, _ptr(x), _ptr(out), batch, threads)
    return out


def lwe_keyswitch32(ksk, lwe_in, out_dim, base_log, level, out_mod_log, threads=8):
    """keyswitch_lwe_ciphertext_with_scalar_change (lwe_keyswitch.rs:331-447) over a batch: lwe_in u64
    (..., in_dim + 1), ksk u32 (in_dim, level, out_dim + 1) -> u32 (..., out_dim + 1)."""
    k = np.ascontiguousarray(ksk, dtype=np.uint32)
    x = _u(lwe_in)
    in_dim = x.shape[-1] - 1
    assert k.size == in_dim * level * (out_dim + 1), "ksk shape"
    batch = x.size // (in_dim + 1)
    out = np.zeros(x.shape[:-1] + (out_dim + 1,), np.uint32)
    _klib().ora_lwe_keyswitch32_batch(k.ctypes.data, in_dim, out_dim, base_log, level, out_mod_log, _ptr(x),
                                      out.ctypes.data, batch, threads)
    return out


def lwe_ms64(lwe, log_mod, centered):
    """lwe_ciphertext_[centered_binary_]modulus_switch of u64 LWEs (modulus_switch.rs:14-104) -> u64 values in
    [0, 2^log_mod), same shape."""
    x = np.ascontiguousarray(lwe, dtype=np.uint64)
    dim = x.shape[-1] - 1
    out = np.zeros(x.shape, np.uint64)
    flat, oflat = x.reshape(-1, dim + 1), out.reshape(-1, dim + 1)
    for b in range(flat.shape[0]):
        row = np.ascontiguousarray(flat[b])
        orow = np.zeros(dim + 1, np.uint64)
        _plib().ora_lwe_ms64(_ptr(row), dim, log_mod, 1 if centered else 0, _ptr(orow))
        oflat[b] = orow
    return out


def lwe_ms32(lwe, log_mod, centered):
    """lwe_ciphertext_[centered_binary_]modulus_switch of u32 LWEs (modulus_switch.rs:14-104) -> u64 values in
    [0, 2^log_mod), same shape."""
    x = np.ascontiguousarray(lwe, dtype=np.uint32)
    dim = x.shape[-1] - 1
    out = np.zeros(x.shape, np.uint64)
    flat, oflat = x.reshape(-1, dim + 1), out.reshape(-1, dim + 1)
    for b in range(flat.shape[0]):
        row = np.ascontiguousarray(flat[b])
        orow = np.zeros(dim + 1, np.uint64)
        _klib().ora_lwe_ms32(row.ctypes.data, dim, log_mod, 1 if centered else 0, _ptr(orow))
        oflat[b] = orow
    return out
