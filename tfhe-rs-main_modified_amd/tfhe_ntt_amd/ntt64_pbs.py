"""Host-side mirror of the core_crypto NTT64 consumers (external product, CMUX, PBS) over the C ABI.

Function names follow the reference (paths relative to /root/reference/tfhe/src/core_crypto):

* ``convert_standard_lwe_bootstrap_key_to_ntt64``    algorithms/lwe_bootstrap_key_conversion.rs:294-365
* ``add_external_product_ntt64_assign``              algorithms/lwe_programmable_bootstrapping/ntt64_pbs.rs:553-663
* ``add_external_product_ntt64_bnf_assign``          .../ntt64_bnf_pbs.rs:541-681
* ``cmux_ntt64_assign`` / ``cmux_ntt64_bnf_assign``   ntt64_pbs.rs:669-680 / ntt64_bnf_pbs.rs:683-705
* ``programmable_bootstrap_ntt64[_bnf]_lwe_ciphertext_mem_optimized``
                                                     ntt64_pbs.rs:482-538 / ntt64_bnf_pbs.rs:469-540
* ``blind_rotate_ntt64[_bnf]_assign``                 ntt64_pbs.rs:176-286 / ntt64_bnf_pbs.rs:174-266
* ``extract_lwe_sample_from_glwe_ciphertext``        algorithms/glwe_sample_extraction.rs:89-160

Every operand is a HIP device tensor (uint64 / int64).  The reference works on one ciphertext per
call; here a leading batch dimension is allowed everywhere (the reference's rayon loop over
ciphertexts, ``pbs_bench.rs:865-886``, becomes one launch).  Shape mismatches raise ``ValueError``
(the reference panics on ``assert_eq!``).
"""
from __future__ import annotations

import ctypes

from ._lib import MiError, check, lib

SOLINAS = 0
BNF = 1
MS_STANDARD = 0
MS_CENTERED = 1
MS_PRE_SWITCHED = 2  # lwe_in already modulus-switched to [0, 2N) (ModulusSwitchedLweCiphertext)


def _dev(t, name):
    import torch

    if not (type(t).__module__.startswith("torch") and t.is_cuda):
        raise TypeError(f"{name} must be a HIP device tensor")
    if t.dtype not in (torch.uint64, torch.int64):
        raise TypeError(f"{name} must hold 64-bit integers, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _stream(t):
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _glwe_batch(t, k, n, name):
    if t.dim() < 2 or tuple(t.shape[-2:]) != (k + 1, n):
        raise ValueError(f"assertion failed: {name} shape {tuple(t.shape)} != (..., {k + 1}, {n})")
    return t.numel() // ((k + 1) * n)


def _ggsw_shape(plan, ggsw, level, k):
    n = plan.ntt_size()
    want = (level, k + 1, k + 1, n)
    if tuple(ggsw.shape[-4:]) != want or ggsw.numel() != level * (k + 1) ** 2 * n:
        raise ValueError(f"assertion failed: ggsw shape {tuple(ggsw.shape)} != {want}")


def convert_standard_lwe_bootstrap_key_to_ntt64(plan, input_bsk, output_bsk, normalize: bool = False,
                                                input_modulus_width: int | None = 64) -> None:
    """output_bsk = fwd(switch(input_bsk)) [* N^-1] polynomial by polynomial.

    ``input_modulus_width``: 64 for native-modulus keys (``Ntt64::modswitch_requirement``,
    ntt64.rs:142-159), the power-of-two width for other 2^w moduli, ``None`` for keys already mod p.
    ``normalize``: ``NttLweBootstrapKeyOption::Normalize`` (Solinas PBS) vs ``Raw`` (BNF PBS)."""
    n = plan.ntt_size()
    if input_bsk.shape != output_bsk.shape or input_bsk.numel() % n:
        raise ValueError("assertion failed: input/output bootstrap key shapes differ")
    check(lib().mi_bsk_to_ntt64(plan.handle, _dev(input_bsk, "input_bsk"), _dev(output_bsk, "output_bsk"),
                                input_bsk.numel() // n, int(input_modulus_width or 0), int(bool(normalize)),
                                _stream(output_bsk)))


class NttGgswList:
    """GGSWs made ready for repeated external products / CMUXes (``mi_ntt64_ggsw``): the reference's
    NttGgswCiphertextList (entities/ntt_ggsw_ciphertext_list.rs) held in the NTT domain.  ``ggsw`` is the device tensor
    (n_ggsw, level, k+1, k+1, N) (or one GGSW (level, k+1, k+1, N)).  The fused N = 2048, k = 1, level-1 bodies read a
    private copy permuted once into their order (made on the tensor's current stream); other shapes reference the
    tensor (keep it alive).  Pass it wherever a ``ggsw`` tensor is accepted below."""

    def __init__(self, plan, ggsw, base_log: int, level: int, variant: int):
        n = plan.ntt_size()
        if ggsw.dim() == 4:
            ggsw = ggsw.unsqueeze(0)
        k = int(ggsw.shape[2]) - 1 if ggsw.dim() == 5 else 0
        if ggsw.dim() != 5 or tuple(ggsw.shape[1:]) != (level, k + 1, k + 1, n):
            raise ValueError(f"assertion failed: ggsw shape {tuple(ggsw.shape)} != (n_ggsw, {level}, k + 1, k + 1, {n})")
        self.plan, self.ggsw, self.base_log, self.level, self.variant = plan, ggsw, base_log, level, variant
        self.glwe_dimension, self.n_ggsw = k, int(ggsw.shape[0])
        h = ctypes.c_void_p()
        check(lib().mi_ntt64_ggsw_create(plan.handle, _dev(ggsw, "ggsw"), self.n_ggsw, k, base_log, level, variant,
                                         _stream(ggsw), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_ntt64_ggsw_destroy(h)
            except Exception:
                pass
            self._h = None


def _ext_prepared(pg, out, glwe, base_log, level, variant, cmux, ggsw_index):
    n = pg.plan.ntt_size()
    k = pg.glwe_dimension
    if (base_log, level, variant) != (pg.base_log, pg.level, pg.variant):
        raise ValueError("the prepared GGSW list was made for another decomposition / variant")
    b = _glwe_batch(out, k, n, "out")
    if glwe.shape != out.shape:
        raise ValueError(f"assertion failed: glwe shape {tuple(glwe.shape)} != out shape {tuple(out.shape)}")
    idx = None if ggsw_index is None else _index(ggsw_index, b, out.device, "ggsw_index")
    fn = lib().mi_cmux_ntt64_prepared_batch if cmux else lib().mi_ext_product_ntt64_prepared_batch
    check(fn(pg._h, _dev(out, "out"), _dev(glwe, "glwe"), idx, b, _stream(out)))


def _ext(plan, out, ggsw, glwe, base_log, level, variant, cmux, ggsw_index=None):
    if isinstance(ggsw, NttGgswList):
        return _ext_prepared(ggsw, out, glwe, base_log, level, variant, cmux, ggsw_index)
    n = plan.ntt_size()
    if out.dim() < 2:
        raise ValueError(f"assertion failed: out shape {tuple(out.shape)} != (..., k + 1, {n})")
    k = int(out.shape[-2]) - 1  # the GLWE dimension follows the operands (GlweSize = k + 1)
    b = _glwe_batch(out, k, n, "out")
    if glwe.shape != out.shape:
        raise ValueError(f"assertion failed: glwe shape {tuple(glwe.shape)} != out shape {tuple(out.shape)}")
    if ggsw_index is None:
        _ggsw_shape(plan, ggsw, level, k)
        fn = lib().mi_cmux_ntt64_batch if cmux else lib().mi_ext_product_ntt64_batch
        check(fn(plan.handle, _dev(out, "out"), _dev(glwe, "glwe"), _dev(ggsw, "ggsw"), k, base_log, level, b,
                 variant, _stream(out)))
        return
    # one GGSW per item: ggsw = (n_ggsw, level, k+1, k+1, N), ggsw_index = `b` int32 / uint32 device indices
    want = (level, k + 1, k + 1, n)
    if ggsw.dim() != 5 or tuple(ggsw.shape[1:]) != want:
        raise ValueError(f"assertion failed: ggsw list shape {tuple(ggsw.shape)} != (n_ggsw, *{want})")
    import torch

    if (ggsw_index.dtype not in (torch.int32, torch.uint32) or ggsw_index.numel() != b or not ggsw_index.is_cuda
            or not ggsw_index.is_contiguous() or ggsw_index.device != out.device):
        raise ValueError(f"assertion failed: ggsw_index must be {b} contiguous int32 indices on the GLWEs' device")
    fn = lib().mi_cmux_ntt64_batch_indexed if cmux else lib().mi_ext_product_ntt64_batch_indexed
    check(fn(plan.handle, _dev(out, "out"), _dev(glwe, "glwe"), _dev(ggsw, "ggsw"),
             ctypes.c_void_p(ggsw_index.data_ptr()), int(ggsw.shape[0]), k, base_log, level, b, variant, _stream(out)))


def add_external_product_ntt64_assign(plan, out, ggsw, glwe, base_log: int, level: int, ggsw_index=None) -> None:
    """out += ggsw (.) glwe modulo the Solinas prime; ``ggsw`` NTT-domain (converted Normalize).  With
    ``ggsw_index`` (int32 device tensor, one entry per item) ``ggsw`` is a list (n_ggsw, level, k+1, k+1, N) and
    item b uses ``ggsw[ggsw_index[b]]`` (an out-of-range index leaves the item untouched)."""
    _ext(plan, out, ggsw, glwe, base_log, level, SOLINAS, False, ggsw_index)


def add_external_product_ntt64_bnf_assign(plan, out, ggsw, glwe, base_log: int, level: int, ggsw_index=None) -> None:
    """out += ggsw (.) glwe on native 2^64 ciphertexts; ``ggsw`` NTT-domain (converted Raw); ``ggsw_index`` as
    ``add_external_product_ntt64_assign``."""
    _ext(plan, out, ggsw, glwe, base_log, level, BNF, False, ggsw_index)


def cmux_ntt64_assign(plan, ct0, ct1, ggsw, base_log: int, level: int, ggsw_index=None) -> None:
    """ct0 = cmux(ggsw, ct0, ct1) mod p; like the reference, ct1 is left holding ct1 - ct0."""
    _ext(plan, ct0, ggsw, ct1, base_log, level, SOLINAS, True, ggsw_index)


def cmux_ntt64_bnf_assign(plan, ct0, ct1, ggsw, base_log: int, level: int, ggsw_index=None) -> None:
    _ext(plan, ct0, ggsw, ct1, base_log, level, BNF, True, ggsw_index)


class NttBootstrapKey:
    """An NTT-domain bootstrap key bound to a plan (``mi_pbs_ntt64_key``).

    ``bsk`` is the device tensor (n_lwe, level, k+1, k+1, N) (k = the GLWE dimension) produced by
    ``convert_standard_lwe_bootstrap_key_to_ntt64``: Raw for ``BNF`` (a private copy with N^-1
    folded in is made once, on the tensor's current stream), Normalize for ``SOLINAS`` (referenced;
    keep the tensor alive; the fused N = 2048, k = 1, level-1 engine copies either variant once, into the
    order its blind rotation reads)."""

    def __init__(self, plan, bsk, base_log: int, level: int, variant: int = BNF):
        n = plan.ntt_size()
        k = int(bsk.shape[2]) - 1 if bsk.dim() == 5 else 1
        if bsk.dim() != 5 or tuple(bsk.shape[1:]) != (level, k + 1, k + 1, n):
            raise ValueError(f"assertion failed: bsk shape {tuple(bsk.shape)} != (n_lwe, {level}, k + 1, k + 1, {n})")
        self._bind(plan, bsk, int(bsk.shape[0]), k, base_log, level, variant)
        h = ctypes.c_void_p()
        check(lib().mi_pbs_ntt64_key_create(plan.handle, _dev(bsk, "bsk"), self.input_lwe_dimension, k, base_log,
                                            level, variant, _stream(bsk), ctypes.byref(h)))
        self._h = h

    def _bind(self, plan, bsk, n_lwe, k, base_log, level, variant):
        self.plan, self.bsk, self.base_log, self.level, self.variant = plan, bsk, base_log, level, variant
        self.input_lwe_dimension = n_lwe
        self.glwe_dimension, self.polynomial_size = k, plan.ntt_size()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_pbs_ntt64_key_destroy(h)
            except Exception:
                pass
            self._h = None

    def output_lwe_size(self) -> int:
        return self.glwe_dimension * self.polynomial_size + 1

    def serialize(self, versioned: bool = False) -> bytes:
        """Bytes of the reference's NttLweBootstrapKey (``ntt_bsk_format``: ``bincode::serialize`` or, with
        ``versioned``, bincode of ``versionize()``).  The ciphertext modulus is the plan's NTT prime for
        both variants, as the reference stores it (ntt64_bnf_pbs.rs:44-94).  Needs the source tensor
        (keys made by ``load`` own only their device copy)."""
        from .ntt_bsk_format import serialize_ntt_bsk
        if self.bsk is None:
            raise ValueError("key was loaded from bytes; serialise the original bytes instead")
        return serialize_ntt_bsk(self.bsk.detach().cpu().numpy(), self.polynomial_size, self.glwe_dimension + 1,
                                 self.level, self.base_log, self.plan.modulus(), versioned)

    @classmethod
    def load(cls, plan, buf: bytes, variant: int, versioned: bool = False, stream=None):
        """Serialised key bytes straight into HBM through the C ABI loader (``mi_pbs_ntt64_key_load``: one
        host-to-device copy, no re-layout).  ``variant`` is explicit because Raw (BNF) and Normalize
        (Solinas) keys store the same fields; the stored modulus must be the plan's prime."""
        import torch
        buf = bytes(buf)
        h = ctypes.c_void_p()
        s = stream if stream is not None else torch.cuda.current_stream(torch.device("cuda", plan.device))
        check(lib().mi_pbs_ntt64_key_load(plan.handle, buf, len(buf), int(bool(versioned)), variant,
                                          ctypes.c_void_p(s.cuda_stream), ctypes.byref(h)))
        n_lwe, k, bl, lv, var = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().mi_pbs_ntt64_key_info(h, ctypes.byref(n_lwe), ctypes.byref(k), ctypes.byref(bl), ctypes.byref(lv),
                                          ctypes.byref(var)))
        key = cls.__new__(cls)
        key._bind(plan, None, n_lwe.value, k.value, bl.value, lv.value, var.value)
        key._h = h
        return key

    @classmethod
    def deserialize(cls, plan, buf: bytes, variant: int, versioned: bool = False, device=None):
        """Parses the bytes on the host (``ntt_bsk_format``), uploads the key tensor and binds it to ``plan``
        (the key keeps the tensor, so it can be re-serialised).  ``variant`` as in ``load``."""
        import numpy as np
        import torch
        from .ntt_bsk_format import NttBskFormatError, deserialize_ntt_bsk
        data, f = deserialize_ntt_bsk(buf, versioned)
        if f["polynomial_size"] != plan.ntt_size():
            raise NttBskFormatError(f"key polynomial size {f['polynomial_size']} != plan size {plan.ntt_size()}")
        if f["ciphertext_modulus"] != plan.modulus():
            raise NttBskFormatError(f"key ciphertext modulus {f['ciphertext_modulus']} is not the plan's NTT prime")
        dev = device if device is not None else torch.device("cuda", plan.device)
        bsk = torch.from_numpy(data.view(np.int64)).to(dev)
        return cls(plan, bsk, f["decomposition_base_log"], f["decomposition_level_count"], variant)


def _lwe_batch(key, lwe_in):
    n_in = key.input_lwe_dimension + 1
    if lwe_in.shape[-1] != n_in:
        raise ValueError(f"assertion failed: input lwe size {lwe_in.shape[-1]} != {n_in}")
    return lwe_in.numel() // n_in


def _index(idx, count, device, name):
    import torch

    if (idx.dtype not in (torch.int32, torch.uint32) or idx.numel() != count or not idx.is_cuda
            or not idx.is_contiguous() or idx.device != device):
        raise ValueError(f"assertion failed: {name} must be {count} contiguous int32 indices on the LWEs' device")
    return ctypes.c_void_p(idx.data_ptr())


def _pbs(key, lwe_in, lwe_out, accumulator, ms_mode, lut_index=None):
    batch = _lwe_batch(key, lwe_in)
    if lwe_out.shape[-1] != key.output_lwe_size() or lwe_out.numel() // key.output_lwe_size() != batch:
        raise ValueError(f"assertion failed: output lwe shape {tuple(lwe_out.shape)}")
    glwe = (key.glwe_dimension + 1, key.polynomial_size)
    if lut_index is None:
        if tuple(accumulator.shape) != glwe:
            raise ValueError(f"assertion failed: accumulator shape {tuple(accumulator.shape)}")
        check(lib().mi_pbs_ntt64_batch(key._h, _dev(lwe_out, "lwe_out"), _dev(lwe_in, "lwe_in"),
                                       _dev(accumulator, "accumulator"), batch, ms_mode, _stream(lwe_out)))
        return
    if accumulator.dim() != 3 or tuple(accumulator.shape[1:]) != glwe:
        raise ValueError(f"assertion failed: accumulator list shape {tuple(accumulator.shape)} != (n_lut, *{glwe})")
    check(lib().mi_pbs_ntt64_batch_lut_indexed(key._h, _dev(lwe_out, "lwe_out"), _dev(lwe_in, "lwe_in"),
                                               _dev(accumulator, "accumulator"),
                                               _index(lut_index, batch, lwe_in.device, "lut_index"),
                                               int(accumulator.shape[0]), batch, ms_mode, _stream(lwe_out)))


def programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(lwe_in, lwe_out, accumulator, key,
                                                                  ms_mode: int = MS_STANDARD, lut_index=None) -> None:
    """Batched BNF PBS of native-modulus LWEs (ntt64_bnf_pbs.rs:469-540).  With ``lut_index`` (int32 device tensor,
    one entry per item) ``accumulator`` is a list (n_lut, k+1, N) and item b bootstraps through
    ``accumulator[lut_index[b]]`` (an out-of-range index leaves ``lwe_out[b]`` untouched)."""
    if key.variant != BNF:
        raise ValueError("key was not prepared for the BNF variant")
    _pbs(key, lwe_in, lwe_out, accumulator, ms_mode, lut_index)


def programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(lwe_in, lwe_out, accumulator, key,
                                                              ms_mode: int = MS_STANDARD, lut_index=None) -> None:
    """Batched PBS of LWEs modulo the Solinas prime (ntt64_pbs.rs:482-538); ms_mode STANDARD or
    PRE_SWITCHED; ``lut_index`` as for the BNF form."""
    if key.variant != SOLINAS:
        raise ValueError("key was not prepared for the Solinas variant")
    if ms_mode == MS_CENTERED:
        raise ValueError("centered modulus switch applies to native-modulus (BNF) inputs")
    _pbs(key, lwe_in, lwe_out, accumulator, ms_mode, lut_index)


def _blind_rotate(key, lwe_in, lut, ms_mode):
    batch = _lwe_batch(key, lwe_in)
    glwe = (key.glwe_dimension + 1, key.polynomial_size)
    if lut.dim() < 2 or tuple(lut.shape[-2:]) != glwe or lut.numel() != batch * glwe[0] * glwe[1]:
        raise ValueError(f"assertion failed: lut shape {tuple(lut.shape)} != ({batch}, *{glwe})")
    check(lib().mi_blind_rotate_ntt64_batch(key._h, _dev(lut, "lut"), _dev(lwe_in, "lwe_in"), batch, ms_mode,
                                            _stream(lut)))


def blind_rotate_ntt64_bnf_assign(msed_input, lut, key, ms_mode: int = MS_PRE_SWITCHED) -> None:
    """blind_rotate_ntt64_bnf_assign[_mem_optimized] (ntt64_bnf_pbs.rs:174-266), batched and in place: every item's
    GLWE ``lut[b]`` is rotated by ``msed_input[b]``.  The reference's input is a ModulusSwitchedLweCiphertext:
    ``MS_PRE_SWITCHED`` (default) takes the switched values (in [0, 2N)); ``MS_STANDARD`` / ``MS_CENTERED`` take the
    native LWE and switch it on the device (lwe_ciphertext_modulus_switch / the centered binary switch)."""
    if key.variant != BNF:
        raise ValueError("key was not prepared for the BNF variant")
    _blind_rotate(key, msed_input, lut, ms_mode)


def blind_rotate_ntt64_assign(lwe_in, lut, key, ms_mode: int = MS_STANDARD) -> None:
    """blind_rotate_ntt64_assign[_mem_optimized] (ntt64_pbs.rs:176-286), batched and in place: LWEs modulo the Solinas
    prime (or ``MS_PRE_SWITCHED`` values)."""
    if key.variant != SOLINAS:
        raise ValueError("key was not prepared for the Solinas variant")
    if ms_mode == MS_CENTERED:
        raise ValueError("centered modulus switch applies to native-modulus (BNF) inputs")
    _blind_rotate(key, lwe_in, lut, ms_mode)


def extract_lwe_sample_from_glwe_ciphertext(glwe, lwe_out, nth: int = 0, nth_stride: int = 0, nth_count: int = 1,
                                            modulus: int = 0) -> None:
    """extract_lwe_sample_from_glwe_ciphertext (glwe_sample_extraction.rs:89-160) over a batch of GLWEs
    (..., k+1, N): lwe_out[b, j] = the LWE of coefficient ``nth + j * nth_stride`` of glwe[b], j < nth_count
    (lwe_out: (batch, nth_count, k N + 1), or (batch, k N + 1) when nth_count is 1).  ``modulus`` 0 = native 2^64,
    else the custom modulus (e.g. the Solinas prime)."""
    if glwe.dim() < 2:
        raise ValueError(f"assertion failed: glwe shape {tuple(glwe.shape)}")
    kp1, n = int(glwe.shape[-2]), int(glwe.shape[-1])
    batch = glwe.numel() // (kp1 * n)
    out_len = (kp1 - 1) * n + 1
    if lwe_out.shape[-1] != out_len or lwe_out.numel() != batch * nth_count * out_len:
        raise ValueError(f"assertion failed: lwe_out shape {tuple(lwe_out.shape)} != ({batch}, {nth_count}, {out_len})")
    if lwe_out.device != glwe.device:
        raise ValueError("glwe and lwe_out must be on one device")
    check(lib().mi_sample_extract_batch(_dev(lwe_out, "lwe_out"), _dev(glwe, "glwe"), n, kp1 - 1, batch, int(nth),
                                        int(nth_stride), int(nth_count), int(modulus), glwe.device.index,
                                        _stream(glwe)))


def scratch_trim(device: int = -1) -> int:
    """Frees the idle blocks of the engine's scratch pool (``mi_scratch_trim``); returns the bytes released."""
    out = ctypes.c_size_t()
    check(lib().mi_scratch_trim(int(device), ctypes.byref(out)))
    return out.value


def scratch_bytes(device: int = -1) -> int:
    out = ctypes.c_size_t()
    check(lib().mi_scratch_bytes(int(device), ctypes.byref(out)))
    return out.value


__all__ = [
    "SOLINAS", "BNF", "MS_STANDARD", "MS_CENTERED", "MS_PRE_SWITCHED", "MiError", "NttBootstrapKey", "NttGgswList",
    "convert_standard_lwe_bootstrap_key_to_ntt64", "add_external_product_ntt64_assign",
    "add_external_product_ntt64_bnf_assign", "cmux_ntt64_assign", "cmux_ntt64_bnf_assign",
    "programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized",
    "programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized", "blind_rotate_ntt64_bnf_assign",
    "blind_rotate_ntt64_assign", "extract_lwe_sample_from_glwe_ciphertext", "scratch_trim", "scratch_bytes",
]
