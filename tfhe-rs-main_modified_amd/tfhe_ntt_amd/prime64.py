"""Host-side mirror of ``tfhe_ntt::prime64::Plan`` over the MI355X C ABI.

Same names, argument meaning and error behaviour as the reference
(/root/reference/tfhe-ntt/src/prime64.rs:245-1222):

* ``Plan.try_new(n, p)`` returns ``None`` exactly where the reference does
  (N < 16, N not a power of two, p not prime, no primitive 2N-th root; prime64.rs:764-775);
* ``fwd`` / ``inv`` / ``normalize`` / ``mul_assign_normalize`` / ``mul_accumulate`` work in place;
  a length mismatch raises (the reference panics on ``assert_eq!``, prime64.rs:898,976).

Buffers may be HIP device tensors (``torch`` uint64/int64 on a ``cuda`` device — the batched fast
path, launched on the tensor device's current stream) or host ``numpy`` uint64 arrays (copied in
and out; the single-poly ``&mut [u64]`` shape of the reference API).  A buffer of shape
``(..., N)`` is a batch of polynomials.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from ._lib import MiError, check, lib

SOLINAS_P = 0xFFFFFFFF00000001

_NONE_STATUSES = (_lib.MI_ERR_INVALID_ARG, _lib.MI_ERR_NOT_PRIME, _lib.MI_ERR_NO_ROOT)


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


class Plan:
    """Negacyclic NTT plan for a 64-bit prime, living on one HIP device."""

    __slots__ = ("_h", "_n", "_p", "_device", "_cached")

    def __init__(self, handle, n: int, p: int, device: int, cached: bool = False):
        self._h, self._n, self._p, self._device, self._cached = handle, n, p, device, cached

    # -- construction ------------------------------------------------------------------
    @classmethod
    def try_new(cls, polynomial_size: int, modulus: int, device: int = 0) -> Optional["Plan"]:
        h = ctypes.c_void_p()
        st = lib().mi_ntt64_plan_create(polynomial_size, modulus, device, ctypes.byref(h))
        if st in _NONE_STATUSES:
            return None
        check(st)
        return cls(h, polynomial_size, modulus, device)

    @classmethod
    def cached(cls, polynomial_size: int, modulus: int, device: int = 0) -> "Plan":
        """The shared plan of ``Ntt64::new`` (ntt64.rs:27-79): one plan per (N, p, device) for the whole
        process, built on first use; raises where the reference panics (no plan for (N, p))."""
        h = ctypes.c_void_p()
        check(lib().mi_ntt64_plan_cached(polynomial_size, modulus, device, ctypes.byref(h)))
        return cls(h, polynomial_size, modulus, device, cached=True)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and not getattr(self, "_cached", False):
            try:
                lib().mi_ntt64_plan_destroy(h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    @property
    def device(self) -> int:
        return self._device

    def ntt_size(self) -> int:
        return self._n

    def modulus(self) -> int:
        return self._p

    def twiddles(self):
        """(twid, inv_twid, n_inv) host copies, reference layout (prime64.rs:184-203, 844)."""
        n = self._n
        tw = np.zeros(n, np.uint64)
        itw = np.zeros(n, np.uint64)
        ninv = ctypes.c_uint64(0)
        p64 = ctypes.POINTER(ctypes.c_uint64)
        check(lib().mi_ntt64_plan_twiddles(self._h, tw.ctypes.data_as(p64), itw.ctypes.data_as(p64),
                                           ctypes.byref(ninv)))
        return tw, itw, int(ninv.value)

    # -- layout helpers ------------------------------------------------------------------
    def _dev_layout(self, t, name="buf"):
        import torch

        if not t.is_cuda:
            raise ValueError(f"{name} must be a HIP device tensor or a numpy array")
        if t.dtype not in (torch.uint64, torch.int64):
            raise TypeError(f"{name} must hold 64-bit integers, got {t.dtype}")
        n = self._n
        if t.dim() == 0 or t.shape[-1] != n:
            raise ValueError(f"assertion failed: {name}.len() == ntt_size ({tuple(t.shape)} vs N={n})")
        if t.stride(-1) != 1:
            raise ValueError(f"{name} rows must be contiguous")
        if t.dim() == 1:
            return 1, n
        if t.dim() == 2:
            return t.shape[0], (t.stride(0) if t.shape[0] > 1 else n)
        if not t.is_contiguous():
            raise ValueError(f"{name} with more than 2 dims must be contiguous")
        return t.numel() // n, n

    def _stream(self, t):
        import torch

        return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def _host_layout(self, a, name="buf"):
        if not isinstance(a, np.ndarray) or a.dtype != np.uint64:
            raise TypeError(f"{name} must be a numpy uint64 array or a device tensor")
        if a.size % self._n != 0 or a.shape[-1] != self._n:
            raise ValueError(f"assertion failed: {name}.len() == ntt_size ({a.shape} vs N={self._n})")
        if not a.flags["C_CONTIGUOUS"] or not a.flags["WRITEABLE"]:
            raise ValueError(f"{name} must be a writeable C-contiguous array")
        return a.size // self._n

    # -- transforms (prime64.rs:897-1046) ------------------------------------------------
    def fwd(self, buf) -> None:
        self._transform(True, buf)

    def inv(self, buf) -> None:
        self._transform(False, buf)

    def _transform(self, fwd: bool, buf) -> None:
        L = lib()
        if _is_torch(buf):
            batch, stride = self._dev_layout(buf)
            fn = L.mi_ntt64_fwd_batch if fwd else L.mi_ntt64_inv_batch
            check(fn(self._h, ctypes.c_void_p(buf.data_ptr()), batch, stride, self._stream(buf)))
        else:
            batch = self._host_layout(buf)
            fn = L.mi_ntt64_fwd_host if fwd else L.mi_ntt64_inv_host
            check(fn(self._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), batch))

    # -- pointwise ops (prime64.rs:1050-1222) --------------------------------------------
    # device tensors run async on the tensor's stream; numpy uint64 arrays (the reference's `&mut [u64]` slices) go
    # through the library's pooled staging slots (mi_ntt64_*_host: copy in, run, copy out, no allocation per call)
    def normalize(self, values) -> None:
        if not _is_torch(values):
            b = self._host_layout(values, "values")
            check(lib().mi_ntt64_normalize_host(self._h, _u64p(values), b))
            return
        b, s = self._dev_layout(values, "values")
        check(lib().mi_ntt64_normalize_batch(self._h, ctypes.c_void_p(values.data_ptr()), b, s, self._stream(values)))

    def mul_assign_normalize(self, lhs, rhs) -> None:
        if not _is_torch(lhs):
            b = self._same_host_layout(lhs, rhs)
            check(lib().mi_ntt64_mul_assign_normalize_host(self._h, _u64p(lhs), _u64p(rhs), b))
            return
        b, s = self._same_layout(lhs, rhs)
        check(lib().mi_ntt64_mul_assign_normalize_batch(self._h, ctypes.c_void_p(lhs.data_ptr()),
                                                        ctypes.c_void_p(rhs.data_ptr()), b, s, self._stream(lhs)))

    def mul_accumulate(self, acc, lhs, rhs) -> None:
        if not _is_torch(acc):
            b = self._same_host_layout(acc, lhs, rhs)
            check(lib().mi_ntt64_mul_accumulate_host(self._h, _u64p(acc), _u64p(lhs), _u64p(rhs), b))
            return
        b, s = self._same_layout(acc, lhs, rhs)
        check(lib().mi_ntt64_mul_accumulate_batch(self._h, ctypes.c_void_p(acc.data_ptr()),
                                                  ctypes.c_void_p(lhs.data_ptr()), ctypes.c_void_p(rhs.data_ptr()),
                                                  b, s, self._stream(acc)))

    def _same_host_layout(self, out, *ins):
        b = self._host_layout(out)
        for a in ins:
            if not isinstance(a, np.ndarray) or a.dtype != np.uint64 or not a.flags["C_CONTIGUOUS"]:
                raise TypeError("host pointwise operands must be C-contiguous numpy uint64 arrays")
            if a.shape != out.shape:
                raise ValueError(f"assertion `left == right` failed: operand shapes {out.shape} vs {a.shape}")
        return b

    def _same_layout(self, *ts):
        if not all(_is_torch(t) for t in ts):
            raise TypeError("pointwise ops take HIP device tensors")
        layouts = [self._dev_layout(t) for t in ts]
        if any(l != layouts[0] for l in layouts):
            raise ValueError(f"operand layouts differ: {layouts}")
        return layouts[0]

    def __repr__(self):
        return f"Plan {{ ntt_size: {self._n}, modulus: {self._p} }}"


def _u64p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def fill_uniform(t, seed: int, p: int = SOLINAS_P) -> None:
    """Fill a device tensor with the §8d synthetic stream (same values as the oracle generator)."""
    import torch

    check(lib().mi_fill_uniform(ctypes.c_void_p(t.data_ptr()), t.numel(), seed & (2**64 - 1), p,
                                t.device.index or 0, ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)))


__all__ = ["Plan", "SOLINAS_P", "MiError", "fill_uniform"]
