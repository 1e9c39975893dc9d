"""CPU tests of the serialised FourierLweBootstrapKey layout (tfhe_ntt_amd.fourier_bsk_format).

The bytes follow the serde derive order of FourierLweBootstrapKey (fft_impl/fft64/crypto/bootstrap.rs:30-39), the
custom Serialize of FourierPolynomialList (fft_impl/fft64/math/fft/mod.rs:642-690) and bincode 1.3's default
encoding; the reference holds no serialised key, so the layout is checked against a hand-assembled byte string
(parity of the bytes unpinned by fixtures) and the parser's refusals.  The GPU side (device reorder into this
engine's order, PBS with a loaded key) is in tests/test_fft_gpu.py.
"""
import struct

import numpy as np
import pytest

from tfhe_ntt_amd import fourier_bsk_format as FB


def tiny(seed=0, n_lwe=2, level=1, glwe=2, n=4):
    g = np.random.default_rng(seed)
    return g.standard_normal((n_lwe, level, glwe, glwe, n // 2, 2))


def test_layout_by_hand():
    n, glwe, level, base_log = 4, 2, 1, 23
    data = tiny(1, n_lwe=1)
    polys = data.reshape(4, 2, 2)
    want = struct.pack("<QQQ", 2 + 4, n, 4)
    for p in polys:
        want += struct.pack("<Q", 2) + struct.pack("<4d", p[0, 0], p[0, 1], p[1, 0], p[1, 1])
    want += struct.pack("<QQQQ", 1, glwe, base_log, level)
    assert FB.serialize_fourier_bsk(data, n, glwe, level, base_log) == want
    vwant = struct.pack("<II", 1, 0) + want[:-32] + b"".join(
        struct.pack("<IQ", 0, v) for v in (1, glwe, base_log, level))
    assert FB.serialize_fourier_bsk(data, n, glwe, level, base_log, versioned=True) == vwant


@pytest.mark.parametrize("versioned", [False, True])
@pytest.mark.parametrize("shape", [(3, 1, 2, 2, 1024), (2, 2, 3, 3, 512), (1, 3, 2, 2, 8)])
def test_round_trip(versioned, shape):
    n_lwe, level, glwe, _, m = shape
    data = np.random.default_rng(sum(shape)).standard_normal(shape + (2,))
    buf = FB.serialize_fourier_bsk(data, 2 * m, glwe, level, 7, versioned)
    got, info = FB.deserialize_fourier_bsk(buf, versioned)
    assert np.array_equal(got, data)
    assert info == dict(polynomial_size=2 * m, glwe_size=glwe, decomposition_level_count=level,
                        decomposition_base_log=7, input_lwe_dimension=n_lwe)
    # complex input serialises the same bytes
    assert FB.serialize_fourier_bsk(data[..., 0] + 1j * data[..., 1], 2 * m, glwe, level, 7, versioned) == buf


def test_refusals():
    data = tiny(2)
    buf = FB.serialize_fourier_bsk(data, 4, 2, 1, 23)
    vbuf = FB.serialize_fourier_bsk(data, 4, 2, 1, 23, versioned=True)
    bad = []
    bad.append((buf[:-1], False))                                        # truncated
    bad.append((buf + b"\0", False))                                     # trailing byte
    bad.append((struct.pack("<Q", 7) + buf[8:], False))                  # sequence length != 2 + chunks
    bad.append((buf[:8] + struct.pack("<Q", 6) + buf[16:], False))       # polynomial size not a power of two
    bad.append((buf[:24] + struct.pack("<Q", 3) + buf[32:], False))      # a polynomial of the wrong length
    bad.append((buf[:-32] + struct.pack("<QQQQ", 3, 2, 23, 1), False))   # 8 polys are not 3 GGSWs
    bad.append((buf[:-32] + struct.pack("<QQQQ", 2, 2, 23, 0), False))   # level 0
    bad.append((struct.pack("<I", 0) + vbuf[4:], True))                  # deprecated V0
    bad.append((struct.pack("<II", 2, 0) + vbuf[8:], True))              # unknown version
    bad.append((vbuf[:-12] + struct.pack("<IQ", 1, 1), True))            # unknown field version
    for b, v in bad:
        with pytest.raises(FB.FourierBskFormatError):
            FB.deserialize_fourier_bsk(b, v)
    with pytest.raises(FB.FourierBskFormatError):
        FB.serialize_fourier_bsk(data[:1, :, :1], 4, 2, 1, 23)          # not a whole GGSW
    with pytest.raises(FB.FourierBskFormatError):
        FB.serialize_fourier_bsk(data, 6, 2, 1, 23)
