"""Quick timing of the f64-FFT PBS bench leg alone (GPU box helper)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-main_modified_amd")]
import torch, bench
import tfhe_ntt_amd as eng
class A: pbs_batch = 4096; pbs_steps = 3
dev = torch.device("cuda", 0)
print(json.dumps(bench.bench_pbs_fft(A, eng, torch, dev, 0, 1, lambda: None, None)), flush=True)
