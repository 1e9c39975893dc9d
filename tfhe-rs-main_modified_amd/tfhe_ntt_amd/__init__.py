"""MI355X-native negacyclic NTT engine for TFHE (host-side mirror of tfhe-ntt / core_crypto Ntt64).

The compute path is ``libtfhe_ntt_amd.so`` (HIP kernels for gfx950 behind the C ABI in
``include/tfhe_ntt_amd.h``); this package only binds it.  Importing it without the built library
raises ``ImportError`` — there is no CPU fallback.
"""
from ._lib import MiError, lib as _load_lib
from .prime64 import SOLINAS_P, Plan, fill_uniform

_load_lib()

from . import fft64, fourier_bsk_format, lwe_keyswitch, multi_gpu, ntt64, ntt64_pbs, ntt_bsk_format, prime32  # noqa: E402,E501  (core_crypto consumers; key formats; batch sharding; u32 plans)
from .native import (native32, native64, native128, native_binary32, native_binary64,  # noqa: E402
                     native_binary128)

__all__ = ["Plan", "SOLINAS_P", "MiError", "fill_uniform", "fft64", "ntt64", "ntt64_pbs", "lwe_keyswitch", "multi_gpu", "prime32", "native32",
           "native64", "native128", "native_binary32", "native_binary64", "native_binary128"]
