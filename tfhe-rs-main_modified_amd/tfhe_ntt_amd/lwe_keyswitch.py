"""Host-side mirror of the core_crypto LWE keyswitch over the C ABI (``mi_lwe_*``).

Reference (paths relative to /root/reference/tfhe/src/core_crypto):

* ``LweKeyswitchKey``            entities/lwe_keyswitch_key.rs (in_dim blocks x level LWEs of out_dim + 1)
* ``keyswitch_lwe_ciphertext``   algorithms/lwe_keyswitch.rs:103-227 (native 2^64 modulus)

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


__all__ = ["LweKeyswitchKey", "keyswitch_lwe_ciphertext"]
