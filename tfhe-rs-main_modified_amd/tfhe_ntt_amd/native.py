"""Host-side mirror of tfhe-ntt's exact native-modulus plans (reference paths relative to
/root/reference/tfhe-ntt/src): ``native32::{Plan32, Plan52}`` (native32.rs), ``native64::{Plan32,
Plan52}`` (native64.rs), ``native128::Plan32`` (native128.rs) and the binary-RHS plans
``native_binary{32,64,128}`` — ``negacyclic_polymul(prod, lhs, rhs)`` in Z_{2^W}[X]/(X^N + 1), computed
as a CRT over the reference's NTT primes on the GPU (``mi_native_polymul_batch``).

Usage mirrors the reference modules: ``native64.Plan32.try_new(n)`` etc.  Buffers are HIP device
tensors of shape ``(..., N)`` with 32-bit (W = 32) or 64-bit (W = 64) integers, or ``(..., N, 2)``
64-bit words (lo, hi) for W = 128; a leading batch dimension multiplies many polynomial pairs.
"""
from __future__ import annotations

import ctypes
from types import SimpleNamespace
from typing import Optional

from . import _lib
from ._lib import check, lib

_NONE_STATUSES = (_lib.MI_ERR_INVALID_ARG, _lib.MI_ERR_NOT_PRIME, _lib.MI_ERR_NO_ROOT)


class _NativePlan:
    KIND = -1
    WIDTH = 64

    __slots__ = ("_h", "_n", "_device")

    def __init__(self, handle, n, device):
        self._h, self._n, self._device = handle, n, device

    @classmethod
    def try_new(cls, n: int, device: int = 0) -> Optional["_NativePlan"]:
        h = ctypes.c_void_p()
        st = lib().mi_native_plan_create(cls.KIND, n, device, ctypes.byref(h))
        if st in _NONE_STATUSES:
            return None
        check(st)
        return cls(h, n, device)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_native_plan_destroy(h)
            except Exception:
                pass
            self._h = None

    def ntt_size(self) -> int:
        return self._n

    def _batch(self, t, name):
        import torch

        if not (hasattr(t, "is_cuda") and t.is_cuda):
            raise ValueError(f"{name} must be a HIP device tensor")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        word_dims = 1 if self.WIDTH == 128 else 0
        want = (torch.int32, getattr(torch, "uint32", torch.int32)) if self.WIDTH == 32 else \
            (torch.int64, torch.uint64)
        if t.dtype not in want:
            raise TypeError(f"{name}: wrong dtype {t.dtype} for {self.WIDTH}-bit coefficients")
        if self.WIDTH == 128 and (t.dim() < 2 or t.shape[-1] != 2):
            raise ValueError(f"{name}: u128 coefficients are (..., N, 2) 64-bit words")
        if t.dim() <= word_dims or t.shape[-1 - word_dims] != self._n:
            raise ValueError(f"assertion failed: {name}.len() == n ({tuple(t.shape)} vs N={self._n})")
        return t.numel() // (self._n * (2 if self.WIDTH == 128 else 1))

    def negacyclic_polymul(self, prod, lhs, rhs) -> None:
        import torch

        b = self._batch(prod, "prod")
        if self._batch(lhs, "lhs") != b or self._batch(rhs, "rhs") != b:
            raise ValueError("prod, lhs and rhs must hold the same number of polynomials")
        stream = ctypes.c_void_p(torch.cuda.current_stream(prod.device).cuda_stream)
        check(lib().mi_native_polymul_batch(self._h, ctypes.c_void_p(prod.data_ptr()), ctypes.c_void_p(lhs.data_ptr()),
                                            ctypes.c_void_p(rhs.data_ptr()), b, stream))


def _plan(name, kind, width):
    return type(name, (_NativePlan,), {"KIND": kind, "WIDTH": width, "__slots__": ()})


native32 = SimpleNamespace(Plan32=_plan("Plan32", 0, 32), Plan52=_plan("Plan52", 1, 32))
native64 = SimpleNamespace(Plan32=_plan("Plan32", 2, 64), Plan52=_plan("Plan52", 3, 64))
native128 = SimpleNamespace(Plan32=_plan("Plan32", 4, 128))
native_binary32 = SimpleNamespace(Plan32=_plan("Plan32", 5, 32), Plan52=_plan("Plan52", 6, 32))
native_binary64 = SimpleNamespace(Plan32=_plan("Plan32", 7, 64), Plan52=_plan("Plan52", 8, 64))
native_binary128 = SimpleNamespace(Plan32=_plan("Plan32", 9, 128))

__all__ = ["native32", "native64", "native128", "native_binary32", "native_binary64", "native_binary128"]
