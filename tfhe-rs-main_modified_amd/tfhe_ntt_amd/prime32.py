"""Host-side mirror of ``tfhe_ntt::prime32::Plan`` (/root/reference/tfhe-ntt/src/prime32.rs:632-1025)
over the MI355X C ABI: the prime64 transform and pointwise ops on u32 buffers, p < 2^32.

``Plan.try_new(n, p)`` returns ``None`` where the reference does (N < 32, N not a power of two, p not
prime, no primitive 2N-th root; prime32.rs:662-671).  Buffers are HIP device tensors of 32-bit
integers (``torch.int32`` / ``torch.uint32``, values read as u32) shaped ``(..., N)``.
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import _lib
from ._lib import check, lib
from .prime64 import _is_torch

_NONE_STATUSES = (_lib.MI_ERR_INVALID_ARG, _lib.MI_ERR_NOT_PRIME, _lib.MI_ERR_NO_ROOT)


class Plan:
    """Negacyclic NTT plan for a 32-bit prime, living on one HIP device."""

    __slots__ = ("_h", "_n", "_p", "_device")

    def __init__(self, handle, n: int, p: int, device: int):
        self._h, self._n, self._p, self._device = handle, n, p, device

    @classmethod
    def try_new(cls, polynomial_size: int, modulus: int, device: int = 0) -> Optional["Plan"]:
        if not 0 < modulus < 2**32:
            raise OverflowError("modulus must fit in u32")
        h = ctypes.c_void_p()
        st = lib().mi_ntt32_plan_create(polynomial_size, modulus, device, ctypes.byref(h))
        if st in _NONE_STATUSES:
            return None
        check(st)
        return cls(h, polynomial_size, modulus, device)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_ntt32_plan_destroy(h)
            except Exception:
                pass
            self._h = None

    def ntt_size(self) -> int:
        return self._n

    def modulus(self) -> int:
        return self._p

    def _layout(self, t, name="buf"):
        import torch

        if not _is_torch(t) or not t.is_cuda:
            raise ValueError(f"{name} must be a HIP device tensor")
        if t.dtype not in (torch.int32, getattr(torch, "uint32", torch.int32)):
            raise TypeError(f"{name} must hold 32-bit integers, got {t.dtype}")
        n = self._n
        if t.dim() == 0 or t.shape[-1] != n:
            raise ValueError(f"assertion failed: {name}.len() == ntt_size ({tuple(t.shape)} vs N={n})")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        return t.numel() // n, n

    @staticmethod
    def _stream(t):
        import torch

        return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def fwd(self, buf) -> None:
        b, s = self._layout(buf)
        check(lib().mi_ntt32_fwd_batch(self._h, ctypes.c_void_p(buf.data_ptr()), b, s, self._stream(buf)))

    def inv(self, buf) -> None:
        b, s = self._layout(buf)
        check(lib().mi_ntt32_inv_batch(self._h, ctypes.c_void_p(buf.data_ptr()), b, s, self._stream(buf)))

    def normalize(self, values) -> None:
        b, s = self._layout(values, "values")
        check(lib().mi_ntt32_normalize_batch(self._h, ctypes.c_void_p(values.data_ptr()), b, s, self._stream(values)))

    def mul_assign_normalize(self, lhs, rhs) -> None:
        b, s = self._same(lhs, rhs)
        check(lib().mi_ntt32_mul_assign_normalize_batch(self._h, ctypes.c_void_p(lhs.data_ptr()),
                                                        ctypes.c_void_p(rhs.data_ptr()), b, s, self._stream(lhs)))

    def mul_accumulate(self, acc, lhs, rhs) -> None:
        b, s = self._same(acc, lhs, rhs)
        check(lib().mi_ntt32_mul_accumulate_batch(self._h, ctypes.c_void_p(acc.data_ptr()),
                                                  ctypes.c_void_p(lhs.data_ptr()), ctypes.c_void_p(rhs.data_ptr()),
                                                  b, s, self._stream(acc)))

    def _same(self, *ts):
        layouts = [self._layout(t) for t in ts]
        if any(l != layouts[0] for l in layouts):
            raise ValueError(f"operand layouts differ: {layouts}")
        return layouts[0]

    def __repr__(self):
        return f"Plan {{ ntt_size: {self._n}, modulus: {self._p} }}"


__all__ = ["Plan"]
