"""GPU tests of the f64-FFT path's per-item accumulators and GLWE-output blind rotation (`-m gpu`).

Reference (paths relative to /root/reference/tfhe/src/core_crypto/algorithms/lwe_programmable_bootstrapping):
  blind_rotate_assign                                      fft64_pbs.rs:186-250
  batch_programmable_bootstrap_lwe_ciphertext_mem_optimized fft64_pbs.rs:1055-1127 (one accumulator per input)
The f64 path is not bit-exact against any restatement (its FFT rounding), so these check the engine against itself
bit for bit where the arithmetic is the same (blind rotation + extraction at 0 == the PBS; a per-item accumulator ==
the shared-LUT PBS run with that LUT) and decryption under real keys (the many-LUT extraction of the HPU mockup,
mockups/tfhe-hpu-mockup/src/lib.rs:736-761), on the one-wave N = 2048 engine and the shape-generic one.
"""
import numpy as np
import pytest

import tfhe_helpers as H

pytestmark = pytest.mark.gpu


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def _key(engine, n, k, n_lwe, base_log, level, seed):
    import torch
    g = H.rng(seed)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17)
    fft = engine.fft64.Fft(n)
    fbsk = torch.zeros((n_lwe, level, k + 1, k + 1, n // 2, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    return g, lwe_sk, glwe_sk, engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft), fbsk


# (N, k, level, base_log): the one-wave engine (k 1, level 1: 4 ciphertexts per workgroup; k 2: one per workgroup),
# the shape-generic engine (N 1024, N 512 with k 4)
SHAPES = [(2048, 1, 1, 23), (2048, 2, 1, 23), (1024, 1, 2, 12), (512, 4, 1, 23)]


@pytest.mark.parametrize("n,k,level,base_log", SHAPES)
def test_blind_rotate_extract_equals_pbs(engine, n, k, level, base_log):
    """blind_rotate_assign on per-item copies of the LUT, then extraction at 0 == the PBS, bit for bit; and
    batch_programmable_bootstrap with per-item accumulators == the shared-LUT PBS per LUT."""
    import torch
    F, M = engine.fft64, engine.ntt64_pbs
    n_lwe, batch = 24, 6
    g, lwe_sk, glwe_sk, key, _ = _key(engine, n, k, n_lwe, base_log, level, 8100 + n + k)
    lut = H.uniform_u64(g, (k + 1, n))
    lwe = H.uniform_u64(g, (batch, n_lwe + 1))
    for ms in (F.MS_STANDARD, F.MS_CENTERED):
        want = dev(np.zeros((batch, k * n + 1), np.uint64))
        F.programmable_bootstrap_lwe_ciphertext(dev(lwe), want, dev(lut), key, ms)
        acc = dev(np.broadcast_to(lut, (batch, k + 1, n)).copy())
        F.blind_rotate_assign(dev(lwe), acc, key, ms)
        got = dev(np.zeros((batch, k * n + 1), np.uint64))
        M.extract_lwe_sample_from_glwe_ciphertext(acc, got, 0)
        assert torch.equal(got, want), ms
    # per-item accumulators: item b with LUT b equals the shared-LUT PBS of LUT b
    luts = H.uniform_u64(g, (batch, k + 1, n))
    out = dev(np.zeros((batch, k * n + 1), np.uint64))
    F.batch_programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(luts), key)
    for b in range(batch):
        one = dev(np.zeros((batch, k * n + 1), np.uint64))
        F.programmable_bootstrap_lwe_ciphertext(dev(lwe), one, dev(luts[b]), key)
        assert torch.equal(out[b], one[b]), b
    # indexed: an out-of-range index leaves the item untouched
    idx = np.array([1, 0, 9, 1, 0, 1], np.int32)
    sentinel = H.uniform_u64(g, (batch, k * n + 1))
    out = dev(sentinel)
    F.programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(luts[:2]), key, lut_index=torch.from_numpy(idx).cuda())
    got = host(out)
    assert np.array_equal(got[2], sentinel[2])
    for b in (0, 1, 3, 5):
        one = dev(np.zeros((batch, k * n + 1), np.uint64))
        F.programmable_bootstrap_lwe_ciphertext(dev(lwe), one, dev(luts[idx[b]]), key)
        assert np.array_equal(got[b], host(one)[b]), b


def test_many_lut_blind_rotate_real_keys(engine):
    """The many-LUT PBS on the f64 path: blind_rotate_assign on a fill_many_lut_accumulator GLWE, lut_nb extractions
    at fn_idx * fn_stride; every sample decrypts to its function's value (N = 2048, k = 1, level 1, msg 2 + carry 2)."""
    from test_blind_rotate_gpu import many_lut_accumulator
    F, M = engine.fft64, engine.ntt64_pbs
    n, k, n_lwe, base_log, level, lut_nb = 2048, 1, 64, 23, 1, 4
    g, lwe_sk, glwe_sk, key, _ = _key(engine, n, k, n_lwe, base_log, level, 8500)
    functions = [lambda m, j=j: (m * (j + 2) + 1) % 16 for j in range(lut_nb)]
    acc0, fn_stride, delta, max_degree = many_lut_accumulator(n, k, 4, 4, functions)
    msgs = list(range(max_degree + 1)) * 4
    lwe = np.stack([H.lwe_encrypt(g, m * delta, lwe_sk, 30, 0) for m in msgs])
    acc = dev(np.broadcast_to(acc0, (len(msgs), k + 1, n)).copy())
    F.blind_rotate_assign(dev(lwe), acc, key, F.MS_STANDARD)
    out = dev(np.zeros((len(msgs), lut_nb, k * n + 1), np.uint64))
    M.extract_lwe_sample_from_glwe_ciphertext(acc, out, 0, fn_stride, lut_nb)
    got = host(out)
    sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for b, m in enumerate(msgs):
        for j in range(lut_nb):
            assert H.decode(H.lwe_decrypt(got[b, j], sk, 0), delta, 16, 0) % 16 == functions[j](m), (m, j)
