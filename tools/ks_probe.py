"""Run the PARAM_MESSAGE_2_CARRY_2 keyswitch (2048 -> 918, B 2^4, L 4) a few times on synthetic data, for
rocprofv3 kernel-trace / PMC passes on the keyswitch kernels alone (bench.py runs every leg)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-main_modified_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import tfhe_ntt_amd as eng

    KS = eng.lwe_keyswitch
    dev = torch.device("cuda", 0)
    ksk = torch.empty((2048, 4, 919), dtype=torch.int64, device=dev)
    eng.fill_uniform(ksk, 0x74666865 + 40, 0)
    key = KS.LweKeyswitchKey(ksk, 4, 4)
    lwe = torch.empty((args.batch, 2049), dtype=torch.int64, device=dev)
    eng.fill_uniform(lwe, 0x74666865 + 41, 0)
    out = torch.empty((args.batch, 919), dtype=torch.int64, device=dev)
    for _ in range(args.reps):
        KS.keyswitch_lwe_ciphertext(key, lwe, out)
    torch.cuda.synchronize()
    print(f"ks_probe: {args.reps} x {args.batch} keyswitches done")


if __name__ == "__main__":
    main()
