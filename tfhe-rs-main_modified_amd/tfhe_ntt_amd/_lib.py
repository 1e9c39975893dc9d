"""ctypes binding of ``libtfhe_ntt_amd.so`` (the C ABI in ``include/tfhe_ntt_amd.h``).

The library is built in-tree by ``make -C tfhe-rs-main_modified_amd`` (``__graft_entry__.build()``).
There is deliberately no CPU fallback: if the shared object is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libtfhe_ntt_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), "include", "tfhe_ntt_amd.h")

MI_OK = 0
MI_ERR_INVALID_ARG = 1
MI_ERR_NOT_PRIME = 2
MI_ERR_NO_ROOT = 3
MI_ERR_HIP = 4
MI_ERR_OOM = 5
MI_ERR_UNSUPPORTED = 6

_u64 = ctypes.c_uint64
_sz = ctypes.c_size_t
_int = ctypes.c_int
_vp = ctypes.c_void_p
_p64 = ctypes.POINTER(ctypes.c_uint64)


class MiError(RuntimeError):
    """A non-OK ``mi_status`` returned through the C ABI."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{message} (status {status})")
        self.status = status


_SIGS = {
    "mi_status_string": (ctypes.c_char_p, [_int]),
    "mi_last_error_message": (ctypes.c_char_p, []),
    "mi_build_source_hash": (ctypes.c_char_p, []),
    "mi_ntt64_plan_create": (_int, [_sz, _u64, _int, ctypes.POINTER(_vp)]),
    "mi_ntt64_plan_destroy": (_int, [_vp]),
    "mi_ntt64_plan_cached": (_int, [_sz, _u64, _int, ctypes.POINTER(_vp)]),
    "mi_ntt64_plan_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_u64), ctypes.POINTER(_int)]),
    "mi_ntt64_plan_twiddles": (_int, [_vp, _p64, _p64, _p64]),
    "mi_ntt64_fwd_batch": (_int, [_vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_inv_batch": (_int, [_vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_normalize_batch": (_int, [_vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_mul_assign_normalize_batch": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_mul_accumulate_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_forward_batch": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_forward_normalized_batch": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_forward_from_power_of_two_modulus_batch": (_int, [_vp, ctypes.c_uint, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_forward_from_decomp_batch": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_add_backward_batch": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_add_backward_on_power_of_two_modulus_batch": (_int, [_vp, ctypes.c_uint, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt64_fwd_host": (_int, [_vp, _p64, _sz]),
    "mi_ntt64_inv_host": (_int, [_vp, _p64, _sz]),
    "mi_ntt64_normalize_host": (_int, [_vp, _p64, _sz]),
    "mi_ntt64_mul_assign_normalize_host": (_int, [_vp, _p64, _p64, _sz]),
    "mi_ntt64_mul_accumulate_host": (_int, [_vp, _p64, _p64, _p64, _sz]),
    "mi_fill_uniform": (_int, [_vp, _sz, _u64, _u64, _int, _vp]),
    "mi_bsk_to_ntt64": (_int, [_vp, _vp, _vp, _sz, ctypes.c_uint, _int, _vp]),
    "mi_ext_product_ntt64_batch": (_int, [_vp, _vp, _vp, _vp, _int, _int, _int, _sz, _int, _vp]),
    "mi_cmux_ntt64_batch": (_int, [_vp, _vp, _vp, _vp, _int, _int, _int, _sz, _int, _vp]),
    "mi_ext_product_ntt64_batch_indexed": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _int, _int, _int, _sz, _int, _vp]),
    "mi_cmux_ntt64_batch_indexed": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _int, _int, _int, _sz, _int, _vp]),
    "mi_pbs_ntt64_key_create": (_int, [_vp, _vp, _sz, _int, _int, _int, _int, _vp, ctypes.POINTER(_vp)]),
    "mi_pbs_ntt64_key_destroy": (_int, [_vp]),
    "mi_pbs_ntt64_key_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_int), ctypes.POINTER(_int),
                                     ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "mi_ntt_bsk_parse": (_int, [_vp, _sz, _int, _vp]),
    "mi_ntt_bsk_serialized_size": (_int, [_vp, _int, ctypes.POINTER(_sz)]),
    "mi_ntt_bsk_write": (_int, [_vp, _vp, _int, _vp, _sz]),
    "mi_pbs_ntt64_key_load": (_int, [_vp, _vp, _sz, _int, _int, _vp, ctypes.POINTER(_vp)]),
    "mi_pbs_ntt64_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _int, _vp]),
    "mi_ntt64_ggsw_create": (_int, [_vp, _vp, _sz, _int, _int, _int, _int, _vp, ctypes.POINTER(_vp)]),
    "mi_ntt64_ggsw_destroy": (_int, [_vp]),
    "mi_ntt64_ggsw_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_int), ctypes.POINTER(_int),
                                  ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "mi_ext_product_ntt64_prepared_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
    "mi_cmux_ntt64_prepared_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
    "mi_pbs_ntt64_batch_lut_indexed": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _sz, _int, _vp]),
    "mi_blind_rotate_ntt64_batch": (_int, [_vp, _vp, _vp, _sz, _int, _vp]),
    "mi_sample_extract_batch": (_int, [_vp, _vp, _sz, _int, _sz, _sz, _sz, _sz, _u64, _int, _vp]),
    "mi_scratch_trim": (_int, [_int, ctypes.POINTER(_sz)]),
    "mi_scratch_bytes": (_int, [_int, ctypes.POINTER(_sz)]),
    "mi_multi_gpu_create": (_int, [_vp, _int, ctypes.POINTER(_vp)]),
    "mi_multi_gpu_destroy": (_int, [_vp]),
    "mi_multi_gpu_count": (_int, [_vp, ctypes.POINTER(_int)]),
    "mi_multi_gpu_info": (_int, [_vp, _int, ctypes.POINTER(_int), ctypes.POINTER(_vp)]),
    "mi_multi_gpu_synchronize": (_int, [_vp]),
    "mi_multi_gpu_active_count": (_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    "mi_multi_gpu_shard": (_int, [_sz, _int, _int, ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    "mi_multi_gpu_broadcast": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_multi_gpu_scatter": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_multi_gpu_gather": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_pbs_ntt64_multi_gpu": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _int, _vp]),
    "mi_pbs_ntt64_multi_gpu_ordered": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _int, _vp, _vp]),
    "mi_fft64_pbs_multi_gpu": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _int, _vp]),
    "mi_fft64_pbs_multi_gpu_ordered": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _int, _vp, _vp]),
    "mi_fft64_plan_create": (_int, [_sz, _int, ctypes.POINTER(_vp)]),
    "mi_fft64_plan_cached": (_int, [_sz, _int, ctypes.POINTER(_vp)]),
    "mi_fft64_plan_destroy": (_int, [_vp]),
    "mi_fft64_plan_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_int)]),
    "mi_fft64_fourier_order": (_int, [_vp, ctypes.POINTER(ctypes.c_uint32)]),
    "mi_fft64_forward_torus_batch": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_fft64_to_standard_order": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_fft64_from_standard_order": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_fft64_backward_torus_batch": (_int, [_vp, _vp, _vp, _sz, _int, _vp]),
    "mi_bsk_to_fourier64": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_fft64_ext_product_batch": (_int, [_vp, _vp, _vp, _vp, _int, _int, _int, _sz, _vp]),
    "mi_fft64_cmux_batch": (_int, [_vp, _vp, _vp, _vp, _int, _int, _int, _sz, _vp]),
    "mi_fft64_pbs_key_create": (_int, [_vp, _vp, _sz, _int, _int, _int, ctypes.POINTER(_vp)]),
    "mi_fft64_pbs_key_destroy": (_int, [_vp]),
    "mi_fft64_pbs_key_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_int), ctypes.POINTER(_int),
                                     ctypes.POINTER(_int)]),
    "mi_fft64_pbs_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _int, _vp]),
    "mi_fft64_pbs_batch_lut_indexed": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, _sz, _int, _vp]),
    "mi_fft64_blind_rotate_batch": (_int, [_vp, _vp, _vp, _sz, _int, _vp]),
    "mi_fft64_bsk_serialized_size": (_int, [_sz, _sz, _int, _int, _int, ctypes.POINTER(_sz)]),
    "mi_fft64_pbs_key_load": (_int, [_vp, _vp, _sz, _int, _vp, ctypes.POINTER(_vp)]),
    "mi_fft64_pbs_key_write": (_int, [_vp, _int, _vp, _sz, _vp]),
    "mi_ntt32_plan_create": (_int, [_sz, ctypes.c_uint32, _int, ctypes.POINTER(_vp)]),
    "mi_ntt32_plan_destroy": (_int, [_vp]),
    "mi_ntt32_plan_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(_int)]),
    "mi_ntt32_fwd_batch": (_int, [_vp, _vp, _sz, _sz, _vp]),
    "mi_ntt32_inv_batch": (_int, [_vp, _vp, _sz, _sz, _vp]),
    "mi_ntt32_normalize_batch": (_int, [_vp, _vp, _sz, _sz, _vp]),
    "mi_ntt32_mul_assign_normalize_batch": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_ntt32_mul_accumulate_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _sz, _vp]),
    "mi_native_plan_create": (_int, [_int, _sz, _int, ctypes.POINTER(_vp)]),
    "mi_native_plan_destroy": (_int, [_vp]),
    "mi_native_plan_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "mi_native_polymul_batch": (_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
    "mi_lwe_ksk_create": (_int, [_vp, _sz, _sz, _int, _int, _int, _vp, ctypes.POINTER(_vp)]),
    "mi_lwe_ksk_destroy": (_int, [_vp]),
    "mi_lwe_ksk_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_sz), ctypes.POINTER(_int),
                               ctypes.POINTER(_int)]),
    "mi_lwe_keyswitch_batch": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_lwe_ksk32_create": (_int, [_vp, _sz, _sz, _int, _int, _int, _int, _vp, ctypes.POINTER(_vp)]),
    "mi_lwe_ksk32_destroy": (_int, [_vp]),
    "mi_lwe_ksk32_info": (_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_sz), ctypes.POINTER(_int),
                                 ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "mi_lwe_keyswitch32_batch": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "mi_lwe_modulus_switch32_batch": (_int, [_vp, _vp, _sz, _sz, _int, _int, _int, _vp]),
    "mi_lwe_modulus_switch_batch": (_int, [_vp, _vp, _sz, _sz, _int, _int, _int, _vp]),
}



class NttBskHeader(ctypes.Structure):
    """``mi_ntt_bsk_header`` (include/tfhe_ntt_amd.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("polynomial_size", "glwe_size", "level", "base_log", "modulus_lo",
                                               "modulus_hi", "input_lwe_dimension", "count", "data_offset")]


_lib = None


def _init_torch_device_runtime() -> None:
    """Bring torch's HIP context up before the engine's first HIP call.

    torch ships its own libamdhip64; the engine links /opt/rocm's.  Measured on the MI355X: either
    runtime fully initialised first is fine, but after a bare ``torch.cuda.is_available()`` (which
    pytest collection and most scripts call) the engine's first ``hipSetDevice`` fails.  Completing
    torch's initialisation here removes that order dependence.  No device -> nothing to do."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C tfhe-rs-main_modified_amd` "
                "(there is no CPU fallback for the HIP engine)")
        _init_torch_device_runtime()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def hip_runtimes() -> list[str]:
    """Paths of every libamdhip64 mapped into this process (/proc/self/maps).  The engine links
    ``libamdhip64.so.7`` by SONAME, so in a process where torch has already loaded its bundled runtime the engine
    shares that one (one HIP runtime per process); without torch it resolves /opt/rocm's through its RUNPATH."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return sorted(paths)


def build_provenance() -> dict:
    """The loaded library's embedded source hash against the hash of the sources beside it (tools/source_hash.py,
    when the repository tree is present): `match` False means the .so was not built from this tree."""
    so = (lib().mi_build_source_hash() or b"").decode()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    tool = os.path.join(root, "tools", "source_hash.py")
    tree = None
    if os.path.exists(tool):
        import importlib.util

        spec = importlib.util.spec_from_file_location("_mi_source_hash", tool)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        tree = mod.source_hash(root)
    return {"so_source_hash": so, "tree_source_hash": tree, "match": (tree == so) if tree else None,
            "so_path": LIB_PATH}


def check(status: int) -> None:
    if status != MI_OK:
        L = lib()
        detail = (L.mi_last_error_message() or b"").decode()
        text = (L.mi_status_string(status) or b"").decode()
        raise MiError(status, f"{text}: {detail}" if detail else text)


def declared_symbols(header: str = HEADER_PATH) -> list[str]:
    """Every function the public header declares (used by the ABI export test)."""
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mi_[a-z0-9_]+)\s*\(", src)))
