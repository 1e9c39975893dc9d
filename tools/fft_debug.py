"""Debug helper: run the config-4 FFT PBS test scenario on the GPU and save outputs (gpurun_out/)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-main_modified_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import tfhe_helpers as H
import tfhe_ntt_amd as eng
N, M = 2048, 1024
n_lwe, base_log, level, msg_mod, batch = 918, 23, 1, 16, 4096
delta = (1 << 63) // msg_mod
g = H.rng(64918)
lwe_sk = H.binary_key(g, n_lwe)
glwe_sk = H.binary_key(g, (1, N))
bsk = H.bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, 17)
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()
fft = eng.fft64.Fft(N)
fbsk = torch.zeros((n_lwe, level, 2, 2, M, 2), dtype=torch.float64, device="cuda")
eng.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
f = lambda x: (7 * x + 2) % msg_mod
lut = H.pbs_lut(N, 1, msg_mod, delta, f)
msgs = np.arange(batch) % msg_mod
lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 45)
key = eng.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
out = dev(np.zeros((batch, N + 1), np.uint64))
eng.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(lut), key)
got = out.cpu().numpy().view(np.uint64)
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/fft_got.npy", got[[0, 1, 2047, batch - 1]])
print("saved")
