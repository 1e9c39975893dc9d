"""Repeat the shape-generic f64 engine's key conversion and external product on fixed inputs and report any run whose
output differs from the first (GPU box diagnostic): python tools/fftg_determinism_probe.py [n] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tfhe-rs-main_modified_amd")]
import torch  # noqa: E402

import tfhe_ntt_amd as eng  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
m = n // 2
rng = np.random.default_rng(7)
u64 = lambda shape: torch.from_numpy(rng.integers(0, 2**63, size=shape, dtype=np.int64) * 2 + 1).cuda()
fft = eng.fft64.Fft(n)
ggsw, glwe, out0 = u64((1, 2, 2, n)), u64((1, 2, n)), u64((1, 2, n))
# the C++ mirror's sequence: forward_as_torus, to / from the standard order (in place), backward_as_torus
x = u64((2, n))
four = torch.zeros((2, m, 2), dtype=torch.float64, device="cuda")
fft.forward_as_torus(four, x)
h0 = four.cpu()
nat = torch.zeros_like(four)
fft.to_standard_order(nat, four)
fft.from_standard_order(nat, nat)
h1 = nat.cpu()
print(f"standard-order round trip: {int((h0 != h1).sum())} of {h0.numel()} differ; NaN in h0: {int(torch.isnan(h0).sum())}",
      flush=True)
first_fg = first_out = None
bad_fg = bad_out = 0
for r in range(reps):
    fg = torch.zeros((1, 2, 2, m, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(fg, ggsw)
    out = out0.clone()
    eng.fft64.add_external_product_assign(out, fg, glwe.clone(), 23, 1, fft)
    torch.cuda.synchronize()
    if first_fg is None:
        first_fg, first_out = fg.clone(), out.clone()
        continue
    if not torch.equal(fg, first_fg):
        bad_fg += 1
        print(f"rep {r}: key conversion differs ({int((fg != first_fg).sum())} values)", flush=True)
    if not torch.equal(out, first_out):
        bad_out += 1
        d = (out != first_out)
        print(f"rep {r}: external product differs at {int(d.sum())} coefficients, first {d.nonzero()[:4].tolist()}",
              flush=True)
print(f"n={n} reps={reps}: key conversion mismatches {bad_fg}, external-product mismatches {bad_out}", flush=True)
