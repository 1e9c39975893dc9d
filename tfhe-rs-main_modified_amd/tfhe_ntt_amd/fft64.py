"""Host-side mirror of the core_crypto f64-FFT PBS path (the default shortint PBS) over the C ABI.

Names follow the reference (paths relative to /root/reference/tfhe/src/core_crypto):

* ``Fft``                                            fft_impl/fft64/math/fft/mod.rs:82-224 (``Fft::new``)
* ``Fft.forward_as_torus`` / ``backward_as_torus``    fft_impl/fft64/math/fft/mod.rs:406-511
* ``convert_standard_lwe_bootstrap_key_to_fourier``  algorithms/lwe_bootstrap_key_conversion.rs:20-43
* ``add_external_product_assign`` / ``cmux_assign``  algorithms/lwe_programmable_bootstrapping/fft64_pbs.rs:270-330, 510-560
* ``FourierLweBootstrapKey``, ``programmable_bootstrap_lwe_ciphertext``  fft64_pbs.rs:924-1060
* ``batch_programmable_bootstrap_lwe_ciphertext`` (one accumulator per input), ``blind_rotate_assign``
                                                     fft64_pbs.rs:1055-1127, 186-250
* ``Fft.to_standard_order`` / ``from_standard_order``  the serialised (natural) Fourier order of
  tfhe-fft/src/unordered.rs:943-1020; ``FourierLweBootstrapKey.serialize`` / ``deserialize``: the reference's
  bytes of the key (``fourier_bsk_format``)

Fourier buffers are float64 device tensors with a trailing (N/2, 2) = (complex, re/im) shape in this
engine's frequency order (``Fft.fourier_order``); ``to_standard_order`` / ``from_standard_order`` convert to and
from the natural order the reference serialises, so keys move between the two in either direction.  A leading batch
dimension is allowed everywhere.  Results are f64 computations: decryption-exact and within the FFT error
bound of the reference, not bit-identical to it.
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib
from .ntt64_pbs import MS_CENTERED, MS_PRE_SWITCHED, MS_STANDARD, _dev, _stream  # noqa: F401


def _fdev(t, name):
    import torch

    if not (type(t).__module__.startswith("torch") and t.is_cuda):
        raise TypeError(f"{name} must be a HIP device tensor")
    if t.dtype != torch.float64:
        raise TypeError(f"{name} must hold float64 (re, im pairs), got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


class Fft:
    """``Fft::new(PolynomialSize)``: the plan-cached twiddles / twisting factors on ``device``."""

    def __init__(self, polynomial_size: int, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().mi_fft64_plan_cached(polynomial_size, device, ctypes.byref(h)))
        self.handle, self.device, self.n = h, device, polynomial_size

    def polynomial_size(self) -> int:
        return self.n

    def fourier_order(self):
        """numpy uint32 array: Fourier position -> DFT frequency index."""
        import numpy as np

        out = np.zeros(self.n // 2, np.uint32)
        check(lib().mi_fft64_fourier_order(self.handle, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
        return out

    def _fourier_shape(self, std, fourier):
        n = self.n
        if std.shape[-1] != n or std.numel() % n:
            raise ValueError(f"assertion failed: standard polynomial size {std.shape[-1]} != {n}")
        if tuple(fourier.shape[-2:]) != (n // 2, 2) or fourier.numel() // n != std.numel() // n:
            raise ValueError(f"assertion failed: fourier shape {tuple(fourier.shape)} != (..., {n // 2}, 2)")
        return std.numel() // n

    def forward_as_torus(self, fourier, standard) -> None:
        b = self._fourier_shape(standard, fourier)
        check(lib().mi_fft64_forward_torus_batch(self.handle, _fdev(fourier, "fourier"), _dev(standard, "standard"), b,
                                                 _stream(standard)))

    def backward_as_torus(self, standard, fourier, add: bool = False) -> None:
        b = self._fourier_shape(standard, fourier)
        check(lib().mi_fft64_backward_torus_batch(self.handle, _dev(standard, "standard"), _fdev(fourier, "fourier"), b,
                                                  int(bool(add)), _stream(standard)))

    def add_backward_as_torus(self, standard, fourier) -> None:
        self.backward_as_torus(standard, fourier, add=True)

    def _reorder(self, out, inp, to_std):
        m = self.n // 2
        if tuple(inp.shape[-2:]) != (m, 2) or out.shape != inp.shape:
            raise ValueError(f"assertion failed: fourier shapes {tuple(out.shape)} / {tuple(inp.shape)} != (..., {m}, 2)")
        fn = lib().mi_fft64_to_standard_order if to_std else lib().mi_fft64_from_standard_order
        check(fn(self.handle, _fdev(out, "out"), _fdev(inp, "in"), inp.numel() // (2 * m), _stream(inp)))

    def to_standard_order(self, out, fourier) -> None:
        """out = fourier (this engine's order) in the natural DFT order the reference serialises
        (Plan::serialize_fourier_buffer); ``out is fourier`` converts in place."""
        self._reorder(out, fourier, True)

    def from_standard_order(self, out, standard_order) -> None:
        """The reverse (Plan::deserialize_fourier_buffer): natural order -> this engine's order."""
        self._reorder(out, standard_order, False)


def convert_standard_lwe_bootstrap_key_to_fourier(input_bsk, output_bsk, fft: Fft | None = None) -> None:
    """output_bsk (n_lwe, level, k+1, k+1, N/2, 2) float64 = forward_as_torus of every polynomial of
    input_bsk (n_lwe, level, k+1, k+1, N)."""
    n = int(input_bsk.shape[-1])
    fft = fft or Fft(n, input_bsk.device.index or 0)
    if tuple(output_bsk.shape[:-2]) != tuple(input_bsk.shape[:-1]) or tuple(output_bsk.shape[-2:]) != (n // 2, 2):
        raise ValueError("assertion failed: output key shape does not match the input key")
    check(lib().mi_bsk_to_fourier64(fft.handle, _dev(input_bsk, "input_bsk"), _fdev(output_bsk, "output_bsk"),
                                    input_bsk.numel() // n, _stream(input_bsk)))


def _ggsw_k(ggsw, level, n):
    if ggsw.dim() < 5:
        raise ValueError(f"assertion failed: fourier ggsw shape {tuple(ggsw.shape)}")
    k = int(ggsw.shape[-4]) - 1
    want = (level, k + 1, k + 1, n // 2, 2)
    if tuple(ggsw.shape[-5:]) != want or ggsw.numel() != level * (k + 1) ** 2 * n:
        raise ValueError(f"assertion failed: fourier ggsw shape {tuple(ggsw.shape)} != {want}")
    return k


def _ext(fft, out, ggsw, glwe, base_log, level, cmux):
    n = fft.n
    k = _ggsw_k(ggsw, level, n)
    if out.dim() < 2 or tuple(out.shape[-2:]) != (k + 1, n):
        raise ValueError(f"assertion failed: out shape {tuple(out.shape)} != (..., {k + 1}, {n})")
    if glwe.shape != out.shape:
        raise ValueError(f"assertion failed: glwe shape {tuple(glwe.shape)} != out shape {tuple(out.shape)}")
    b = out.numel() // ((k + 1) * n)
    fn = lib().mi_fft64_cmux_batch if cmux else lib().mi_fft64_ext_product_batch
    check(fn(fft.handle, _dev(out, "out"), _dev(glwe, "glwe"), _fdev(ggsw, "ggsw"), k, base_log, level, b, _stream(out)))


def add_external_product_assign(out, ggsw, glwe, base_log: int, level: int, fft: Fft | None = None) -> None:
    """out += ggsw (.) glwe (native 2^64 GLWEs, Fourier GGSW (level, k+1, k+1, N/2, 2))."""
    _ext(fft or Fft(int(out.shape[-1]), out.device.index or 0), out, ggsw, glwe, base_log, level, False)


def cmux_assign(ct0, ct1, ggsw, base_log: int, level: int, fft: Fft | None = None) -> None:
    """ct0 = cmux(ggsw, ct0, ct1); like the reference, ct1 is left holding ct1 - ct0."""
    _ext(fft or Fft(int(ct0.shape[-1]), ct0.device.index or 0), ct0, ggsw, ct1, base_log, level, True)


class FourierLweBootstrapKey:
    """A Fourier-domain bootstrap key (n_lwe, level, k+1, k+1, N/2, 2) float64 bound to an ``Fft`` plan
    (``mi_fft64_pbs_key``; the tensor is referenced, keep it alive)."""

    def __init__(self, fbsk, base_log: int, level: int, fft: Fft | None = None):
        if fbsk.dim() != 6 or fbsk.shape[1] != level or fbsk.shape[-1] != 2 or fbsk.shape[2] != fbsk.shape[3]:
            raise ValueError(f"assertion failed: fourier bsk shape {tuple(fbsk.shape)}")
        n = 2 * int(fbsk.shape[-2])
        self.fft = fft or Fft(n, fbsk.device.index or 0)
        self.fbsk, self.base_log, self.level = fbsk, base_log, level
        self.input_lwe_dimension = int(fbsk.shape[0])
        self.glwe_dimension, self.polynomial_size = int(fbsk.shape[2]) - 1, n
        h = ctypes.c_void_p()
        check(lib().mi_fft64_pbs_key_create(self.fft.handle, _fdev(fbsk, "fbsk"), self.input_lwe_dimension,
                                            self.glwe_dimension, base_log, level, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().mi_fft64_pbs_key_destroy(h)
            except Exception:
                pass
            self._h = None

    def output_lwe_size(self) -> int:
        return self.glwe_dimension * self.polynomial_size + 1

    def serialize(self, versioned: bool = False) -> bytes:
        """The reference's bytes of this key (``bincode::serialize(&FourierLweBootstrapKey)``, or of its
        ``versionize()`` form), written by the library (``mi_fft64_pbs_key_write``: natural Fourier order, see
        ``fourier_bsk_format``)."""
        size = ctypes.c_size_t()
        check(lib().mi_fft64_bsk_serialized_size(self.polynomial_size, self.input_lwe_dimension, self.glwe_dimension,
                                                 self.level, int(bool(versioned)), ctypes.byref(size)))
        out = ctypes.create_string_buffer(size.value)
        check(lib().mi_fft64_pbs_key_write(self._h, int(bool(versioned)), out, size.value, self._stream()))
        return out.raw

    def _stream(self):
        import torch

        return ctypes.c_void_p(torch.cuda.current_stream(torch.device("cuda", self.fft.device)).cuda_stream)

    @classmethod
    def load(cls, buf: bytes, versioned: bool = False, fft: Fft | None = None, device: int = 0):
        """A key from the reference's bytes through the library (``mi_fft64_pbs_key_load``: validated, one strided
        upload, reordered into this engine's order on the device; the key owns that copy, ``fbsk`` is None).
        Without ``fft`` the plan is the cached one of the polynomial size the bytes declare."""
        if fft is None:
            head = 8 if versioned else 0  # the list's u64 sequence length, then u64 polynomial_size
            if len(buf) < head + 16:
                raise ValueError("Fourier BSK: truncated")
            fft = Fft(int.from_bytes(bytes(buf[head + 8:head + 16]), "little"), device)
        self = cls.__new__(cls)
        self.fft, self.fbsk = fft, None
        h = ctypes.c_void_p()
        check(lib().mi_fft64_pbs_key_load(fft.handle, buf, len(buf), int(bool(versioned)), self._stream(),
                                          ctypes.byref(h)))
        self._h = h
        n_lwe, k, bl, lv = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().mi_fft64_pbs_key_info(h, ctypes.byref(n_lwe), ctypes.byref(k), ctypes.byref(bl), ctypes.byref(lv)))
        self.input_lwe_dimension, self.glwe_dimension = n_lwe.value, k.value
        self.base_log, self.level, self.polynomial_size = bl.value, lv.value, fft.n
        return self

    @classmethod
    def deserialize(cls, buf: bytes, versioned: bool = False, device=None, fft: Fft | None = None):
        """A key from the reference's bytes parsed on the host by ``fourier_bsk_format`` (the Python mirror of the
        layout), copied to ``device`` as a tensor the key references, reordered into this engine's order in
        place on the device."""
        from .fourier_bsk_format import deserialize_fourier_bsk

        import torch

        data, info = deserialize_fourier_bsk(buf, versioned)
        if device is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        else:
            dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        fft = fft or Fft(info["polynomial_size"], dev.index)
        fbsk = torch.from_numpy(data).to(dev)
        fft.from_standard_order(fbsk, fbsk)
        return cls(fbsk, info["decomposition_base_log"], info["decomposition_level_count"], fft)


def _lwe_batch(key, lwe_in):
    n_in = key.input_lwe_dimension + 1
    if lwe_in.shape[-1] != n_in:
        raise ValueError(f"assertion failed: input lwe size {lwe_in.shape[-1]} != {n_in}")
    return lwe_in.numel() // n_in


def programmable_bootstrap_lwe_ciphertext(lwe_in, lwe_out, accumulator, key: FourierLweBootstrapKey,
                                          ms_mode: int = MS_STANDARD, lut_index=None) -> None:
    """Batched f64-FFT PBS of native-modulus LWEs (fft64_pbs.rs:924-1060).  ``accumulator`` (k+1, N) is shared; with
    ``lut_index`` (int32 device tensor, one entry per item) it is a list (n_lut, k+1, N) and item b bootstraps through
    ``accumulator[lut_index[b]]`` (an out-of-range index leaves ``lwe_out[b]`` untouched)."""
    from .ntt64_pbs import _index
    batch = _lwe_batch(key, lwe_in)
    if lwe_out.shape[-1] != key.output_lwe_size() or lwe_out.numel() // key.output_lwe_size() != batch:
        raise ValueError(f"assertion failed: output lwe shape {tuple(lwe_out.shape)}")
    glwe = (key.glwe_dimension + 1, key.polynomial_size)
    if lut_index is None:
        if tuple(accumulator.shape) != glwe:
            raise ValueError(f"assertion failed: accumulator shape {tuple(accumulator.shape)}")
        check(lib().mi_fft64_pbs_batch(key._h, _dev(lwe_out, "lwe_out"), _dev(lwe_in, "lwe_in"),
                                       _dev(accumulator, "accumulator"), batch, ms_mode, _stream(lwe_out)))
        return
    if accumulator.dim() != 3 or tuple(accumulator.shape[1:]) != glwe:
        raise ValueError(f"assertion failed: accumulator list shape {tuple(accumulator.shape)} != (n_lut, *{glwe})")
    check(lib().mi_fft64_pbs_batch_lut_indexed(key._h, _dev(lwe_out, "lwe_out"), _dev(lwe_in, "lwe_in"),
                                               _dev(accumulator, "accumulator"),
                                               _index(lut_index, batch, lwe_in.device, "lut_index"),
                                               int(accumulator.shape[0]), batch, ms_mode, _stream(lwe_out)))


def batch_programmable_bootstrap_lwe_ciphertext(lwe_in, lwe_out, accumulators, key: FourierLweBootstrapKey,
                                                ms_mode: int = MS_STANDARD) -> None:
    """batch_programmable_bootstrap_lwe_ciphertext_mem_optimized (fft64_pbs.rs:1055-1127): one accumulator per input
    (``accumulators``: (batch, k+1, N))."""
    batch = _lwe_batch(key, lwe_in)
    glwe = (key.glwe_dimension + 1, key.polynomial_size)
    if lwe_out.shape[-1] != key.output_lwe_size() or lwe_out.numel() // key.output_lwe_size() != batch:
        raise ValueError(f"assertion failed: output lwe shape {tuple(lwe_out.shape)}")
    if accumulators.dim() != 3 or tuple(accumulators.shape) != (batch, *glwe):
        raise ValueError(f"assertion failed: accumulator list shape {tuple(accumulators.shape)} != ({batch}, *{glwe})")
    check(lib().mi_fft64_pbs_batch_lut_indexed(key._h, _dev(lwe_out, "lwe_out"), _dev(lwe_in, "lwe_in"),
                                               _dev(accumulators, "accumulators"), None, batch, batch, ms_mode,
                                               _stream(lwe_out)))


def blind_rotate_assign(msed_input, lut, key: FourierLweBootstrapKey, ms_mode: int = MS_PRE_SWITCHED) -> None:
    """blind_rotate_assign (fft64_pbs.rs:186-250), batched and in place: lut (batch, k+1, N), every item rotated by its
    own input; ``MS_PRE_SWITCHED`` (default) takes the ModulusSwitchedLweCiphertext values, ``MS_STANDARD`` /
    ``MS_CENTERED`` the native LWE switched on the device."""
    batch = _lwe_batch(key, msed_input)
    glwe = (key.glwe_dimension + 1, key.polynomial_size)
    if lut.dim() < 2 or tuple(lut.shape[-2:]) != glwe or lut.numel() != batch * glwe[0] * glwe[1]:
        raise ValueError(f"assertion failed: lut shape {tuple(lut.shape)} != ({batch}, *{glwe})")
    check(lib().mi_fft64_blind_rotate_batch(key._h, _dev(lut, "lut"), _dev(msed_input, "msed_input"), batch, ms_mode,
                                            _stream(lut)))


__all__ = ["Fft", "FourierLweBootstrapKey", "convert_standard_lwe_bootstrap_key_to_fourier",
           "add_external_product_assign", "cmux_assign", "programmable_bootstrap_lwe_ciphertext",
           "batch_programmable_bootstrap_lwe_ciphertext", "blind_rotate_assign",
           "MS_STANDARD", "MS_CENTERED", "MS_PRE_SWITCHED"]
