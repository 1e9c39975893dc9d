"""Host-side mirror of the core_crypto LWE keyswitch over the C ABI (``mi_lwe_*``).

Reference (paths relative to /root/reference/tfhe/src/core_crypto):

* ``LweKeyswitchKey``            entities/lwe_keyswitch_key.rs (in_dim blocks x level LWEs of out_dim + 1)
* ``keyswitch_lwe_ciphertext``   algorithms/lwe_keyswitch.rs:103-227 (native 2^64 modulus)
* ``keyswitch_lwe_ciphertext_with_scalar_change``  algorithms/lwe_keyswitch.rs:331-447 (u64 -> u32 LWEs, the HPU
  KS32 parameter sets, shortint/parameters/v1_5/hpu.rs:57-76)
* ``lwe_ciphertext_modulus_switch`` / ``lwe_ciphertext_centered_binary_modulus_switch`` of u32 LWEs (the KS32
  bootstrap's input, mockups/tfhe-hpu-mockup/src/lib.rs:720-736) and of u64 LWEs (the native-modulus ciphertexts in
  front of every other blind rotation), algorithms/modulus_switch.rs:14-104

The reference keyswitches one ciphertext per call; here a leading batch dimension is allowed (one
launch on the int8 matrix cores, csrc/keyswitch.hip).  Shape mismatches raise ``ValueError`` where
the reference panics on ``assert!``.
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib
from .ntt64_pbs import _dev, _stream


class LweKeyswitchKey:
    """A device keyswitch key prepared for ``keyswitch_lwe_ciphertext`` (``mi_lwe_ksk``).

    ``ksk``: device tensor (in_dim, level, out_dim + 1) of u64 in the reference layout (levels as
    generate_lwe_keyswitch_key stores them, lwe_keyswitch_key_generation.rs:169-199).  A private
    matrix-core copy is made; ``ksk`` may be released afterwards."""

    def __init__(self, ksk, base_log: int, level: int):
        if ksk.dim() != 3 or ksk.shape[1] != level:
            raise ValueError(f"assertion failed: ksk shape {tuple(ksk.shape)} != (in_dim, {level}, out_dim + 1)")
        self.input_key_lwe_dimension = int(ksk.shape[0])
        self.output_key_lwe_dimension = int(ksk.shape[2]) - 1
        self.decomposition_base_log, self.decomposition_level_count = base_log, level
        self.device = ksk.device
        h = ctypes.c_void_p()
        check(lib().mi_lwe_ksk_create(_dev(ksk, "ksk"), self.input_key_lwe_dimension,
                                      self.output_key_lwe_dimension, base_log, level,
                                      ksk.device.index or 0, _stream(ksk), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_lwe_ksk_destroy(h)
            except Exception:
                pass
            self._h = None


def keyswitch_lwe_ciphertext(lwe_keyswitch_key: LweKeyswitchKey, input_lwe_ciphertext, output_lwe_ciphertext) -> None:
    """output = keyswitch(input) for every ciphertext of the batch (lwe_keyswitch.rs:137-227)."""
    k = lwe_keyswitch_key
    n_in, n_out = k.input_key_lwe_dimension + 1, k.output_key_lwe_dimension + 1
    if input_lwe_ciphertext.shape[-1] != n_in:
        raise ValueError(f"assertion failed: Mismatched input LweDimension {input_lwe_ciphertext.shape[-1] - 1} "
                         f"!= {k.input_key_lwe_dimension}")
    if output_lwe_ciphertext.shape[-1] != n_out:
        raise ValueError(f"assertion failed: Mismatched output LweDimension {output_lwe_ciphertext.shape[-1] - 1} "
                         f"!= {k.output_key_lwe_dimension}")
    batch = input_lwe_ciphertext.numel() // n_in
    if output_lwe_ciphertext.numel() // n_out != batch:
        raise ValueError("assertion failed: input and output batch sizes differ")
    check(lib().mi_lwe_keyswitch_batch(k._h, _dev(output_lwe_ciphertext, "output_lwe_ciphertext"),
                                       _dev(input_lwe_ciphertext, "input_lwe_ciphertext"), batch,
                                       _stream(output_lwe_ciphertext)))


def _dev32(t, name):
    import torch

    if not (type(t).__module__.startswith("torch") and t.is_cuda):
        raise TypeError(f"{name} must be a HIP device tensor")
    if t.dtype not in (torch.uint32, torch.int32):
        raise TypeError(f"{name} must hold 32-bit integers, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


class LweKeyswitchKey32:
    """An LweKeyswitchKey<Vec<u32>> prepared for ``keyswitch_lwe_ciphertext_with_scalar_change`` (``mi_lwe_ksk32``).

    ``ksk``: device tensor (in_dim, level, out_dim + 1) of u32 (int32 storage) in the reference layout; the output
    ciphertext modulus is 2^``out_modulus_log`` (the HPU's post_keyswitch_ciphertext_modulus 2^21), its values in the
    MSBs of the words as the reference stores non-native power-of-two moduli."""

    def __init__(self, ksk, base_log: int, level: int, out_modulus_log: int = 32):
        if ksk.dim() != 3 or ksk.shape[1] != level:
            raise ValueError(f"assertion failed: ksk shape {tuple(ksk.shape)} != (in_dim, {level}, out_dim + 1)")
        self.input_key_lwe_dimension = int(ksk.shape[0])
        self.output_key_lwe_dimension = int(ksk.shape[2]) - 1
        self.decomposition_base_log, self.decomposition_level_count = base_log, level
        self.out_modulus_log = out_modulus_log
        self.device = ksk.device
        h = ctypes.c_void_p()
        check(lib().mi_lwe_ksk32_create(_dev32(ksk, "ksk"), self.input_key_lwe_dimension,
                                        self.output_key_lwe_dimension, base_log, level, out_modulus_log,
                                        ksk.device.index or 0, _stream(ksk), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_lwe_ksk32_destroy(h)
            except Exception:
                pass
            self._h = None


def keyswitch_lwe_ciphertext_with_scalar_change(lwe_keyswitch_key: LweKeyswitchKey32, input_lwe_ciphertext,
                                                output_lwe_ciphertext) -> None:
    """u32 output = keyswitch(u64 input) for every ciphertext of the batch (lwe_keyswitch.rs:331-447)."""
    k = lwe_keyswitch_key
    n_in, n_out = k.input_key_lwe_dimension + 1, k.output_key_lwe_dimension + 1
    if input_lwe_ciphertext.shape[-1] != n_in:
        raise ValueError(f"assertion failed: Mismatched input LweDimension {input_lwe_ciphertext.shape[-1] - 1} "
                         f"!= {k.input_key_lwe_dimension}")
    if output_lwe_ciphertext.shape[-1] != n_out:
        raise ValueError(f"assertion failed: Mismatched output LweDimension {output_lwe_ciphertext.shape[-1] - 1} "
                         f"!= {k.output_key_lwe_dimension}")
    batch = input_lwe_ciphertext.numel() // n_in
    if output_lwe_ciphertext.numel() // n_out != batch:
        raise ValueError("assertion failed: input and output batch sizes differ")
    check(lib().mi_lwe_keyswitch32_batch(k._h, _dev32(output_lwe_ciphertext, "output_lwe_ciphertext"),
                                         _dev(input_lwe_ciphertext, "input_lwe_ciphertext"), batch,
                                         _stream(output_lwe_ciphertext)))


MS_STANDARD, MS_CENTERED = 0, 1


def lwe_ciphertext_modulus_switch32(lwe_in, switched_out, log_modulus: int, centered: bool = False) -> None:
    """The (centered binary) modulus switch of u32 LWEs (modulus_switch.rs:14-104 at Scalar = u32), materialised:
    switched_out (u64 storage, same shape as lwe_in) gets every value in [0, 2^log_modulus), the MI_MS_PRE_SWITCHED
    input of the blind rotation / PBS."""
    if tuple(switched_out.shape) != tuple(lwe_in.shape):
        raise ValueError(f"assertion failed: shapes {tuple(lwe_in.shape)} != {tuple(switched_out.shape)}")
    size = lwe_in.shape[-1]
    batch = lwe_in.numel() // size
    check(lib().mi_lwe_modulus_switch32_batch(_dev(switched_out, "switched_out"), _dev32(lwe_in, "lwe_in"), size - 1,
                                              batch, log_modulus, MS_CENTERED if centered else MS_STANDARD,
                                              lwe_in.device.index or 0, _stream(lwe_in)))


def lwe_ciphertext_centered_binary_modulus_switch32(lwe_in, switched_out, log_modulus: int) -> None:
    lwe_ciphertext_modulus_switch32(lwe_in, switched_out, log_modulus, centered=True)


def lwe_ciphertext_modulus_switch(lwe_in, switched_out, log_modulus: int, centered: bool = False) -> None:
    """The (centered binary) modulus switch of u64 LWEs (modulus_switch.rs:14-104 at Scalar = u64), materialised as
    the LazyStandardModulusSwitchedLweCiphertext reads it (modulus_switched_lwe_ciphertext.rs:150-175): switched_out
    (same shape as lwe_in) gets every value in [0, 2^log_modulus), the MI_MS_PRE_SWITCHED input of the blind rotation
    / PBS.  log_modulus in [1, 64] (standard) or [1, 63] (centered: the reference's half_case shift underflows at 64)."""
    if tuple(switched_out.shape) != tuple(lwe_in.shape):
        raise ValueError(f"assertion failed: shapes {tuple(lwe_in.shape)} != {tuple(switched_out.shape)}")
    size = lwe_in.shape[-1]
    batch = lwe_in.numel() // size
    check(lib().mi_lwe_modulus_switch_batch(_dev(switched_out, "switched_out"), _dev(lwe_in, "lwe_in"), size - 1,
                                            batch, log_modulus, MS_CENTERED if centered else MS_STANDARD,
                                            lwe_in.device.index or 0, _stream(lwe_in)))


def lwe_ciphertext_centered_binary_modulus_switch(lwe_in, switched_out, log_modulus: int) -> None:
    lwe_ciphertext_modulus_switch(lwe_in, switched_out, log_modulus, centered=True)


__all__ = ["LweKeyswitchKey", "keyswitch_lwe_ciphertext", "LweKeyswitchKey32",
           "keyswitch_lwe_ciphertext_with_scalar_change", "lwe_ciphertext_modulus_switch32",
           "lwe_ciphertext_centered_binary_modulus_switch32", "lwe_ciphertext_modulus_switch",
           "lwe_ciphertext_centered_binary_modulus_switch"]
