"""Host-side mirror of core_crypto's ``Ntt64`` / ``Ntt64View`` over the C ABI (``mi_ntt64_*_batch`` view entry points).

Reference: tfhe/src/core_crypto/commons/math/ntt/ntt64.rs — ``Ntt64::new`` (:33-76, the process-wide PLANS cache) and the
six ``Ntt64View`` helpers (:89-266) that every tfhe-rs NTT consumer calls per polynomial.  Here each call takes a batch:
device tensors of shape (..., N) (u64 / i64 storage, rows contiguous, the same layout for both operands), run async on
the tensor's current stream.  Argument order and meaning are the reference's (``forward(ntt, standard)``,
``add_backward(standard, ntt)``, ...).  As in the reference, ``add_backward*`` leave ``ntt`` holding the inverse
transform (switched to 2^w for the power-of-two form).  Length mismatches raise ``ValueError`` where the reference
panics on ``assert_eq!``.
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib
from .prime64 import Plan, _is_torch


class Ntt64View:
    """``Ntt64View`` (ntt64.rs:14-17, 80-266) over a plan of this package."""

    def __init__(self, plan: Plan):
        self.plan = plan

    def polynomial_size(self) -> int:
        return self.plan.ntt_size()

    def custom_modulus(self) -> int:
        return self.plan.modulus()

    def _pair(self, out, inp, out_name, in_name):
        if not (_is_torch(out) and _is_torch(inp)):
            raise TypeError("Ntt64View ops take HIP device tensors")
        lo = self.plan._dev_layout(out, out_name)
        li = self.plan._dev_layout(inp, in_name)
        if lo != li:
            raise ValueError(f"assertion `left == right` failed: {out_name} / {in_name} layouts {lo} vs {li}")
        return lo

    def _fwd(self, fn, ntt, standard, *lead):
        b, s = self._pair(ntt, standard, "ntt", "standard")
        check(fn(self.plan.handle, *lead, ctypes.c_void_p(ntt.data_ptr()), ctypes.c_void_p(standard.data_ptr()), b, s,
                 self.plan._stream(ntt)))

    def forward(self, ntt, standard) -> None:
        """ntt = Plan::fwd(standard) (ntt64.rs:89-95)."""
        self._fwd(lib().mi_ntt64_forward_batch, ntt, standard)

    def forward_normalized(self, ntt, standard) -> None:
        """ntt = normalize(Plan::fwd(standard)) (ntt64.rs:97-108)."""
        self._fwd(lib().mi_ntt64_forward_normalized_batch, ntt, standard)

    def forward_from_power_of_two_modulus(self, input_modulus_width: int, ntt, standard) -> None:
        """ntt = Plan::fwd(switch_{2^w -> p}(standard)) (ntt64.rs:166-177, 201-214); MSB-aligned inputs."""
        self._fwd(lib().mi_ntt64_forward_from_power_of_two_modulus_batch, ntt, standard,
                  ctypes.c_uint(input_modulus_width))

    def forward_from_decomp(self, ntt, decomp) -> None:
        """ntt = Plan::fwd(d), d = x + p for the digits negative as an i64 (ntt64.rs:221-240)."""
        self._fwd(lib().mi_ntt64_forward_from_decomp_batch, ntt, decomp)

    def _add(self, fn, standard, ntt, *lead):
        b, s = self._pair(standard, ntt, "standard", "ntt")
        check(fn(self.plan.handle, *lead, ctypes.c_void_p(standard.data_ptr()), ctypes.c_void_p(ntt.data_ptr()), b, s,
                 self.plan._stream(standard)))

    def add_backward(self, standard, ntt) -> None:
        """ntt = Plan::inv(ntt); standard = wrapping_add_custom_mod(standard, ntt, p) (ntt64.rs:110-131)."""
        self._add(lib().mi_ntt64_add_backward_batch, standard, ntt)

    def add_backward_on_power_of_two_modulus(self, output_modulus_width: int, standard, ntt) -> None:
        """ntt = switch_{p -> 2^w}(Plan::inv(ntt)); standard += ntt wrapping (ntt64.rs:184-196, 244-266)."""
        self._add(lib().mi_ntt64_add_backward_on_power_of_two_modulus_batch, standard, ntt,
                  ctypes.c_uint(output_modulus_width))


class Ntt64:
    """``Ntt64::new(modulus, size)`` (ntt64.rs:33-76): the plan of (size, modulus) from the process-wide cache
    (``mi_ntt64_plan_cached``: built once per device, shared by every caller and thread)."""

    def __init__(self, modulus: int, polynomial_size: int, device: int = 0):
        self.plan = Plan.cached(polynomial_size, modulus, device)

    def as_view(self) -> Ntt64View:
        return Ntt64View(self.plan)


__all__ = ["Ntt64", "Ntt64View"]
