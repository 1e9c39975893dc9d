#!/usr/bin/env python3
"""GPU probe: the Solinas transform at N = 2^11 ... 2^20 through the C ABI of a given library build (default: the
in-tree one; 2^12 and up run the split transform there, launch_ntt_split), time per launch and HBM fraction at
2 x 8 B per coefficient (one read + one write per transform: the algorithmic bytes).
  python tools/split_probe.py [--lib path/to/libtfhe_ntt_amd.so] [reps]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0xFFFFFFFF00000001
args = sys.argv[1:]
lib_path = os.path.join(ROOT, "tfhe-rs-main_modified_amd", "tfhe_ntt_amd", "libtfhe_ntt_amd.so")
if args and args[0] == "--lib":
    lib_path, args = args[1], args[2:]
reps = int(args[0]) if args else 20
L = ctypes.CDLL(lib_path)
L.mi_ntt64_plan_create.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
for f in (L.mi_ntt64_fwd_batch, L.mi_ntt64_inv_batch):
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
L.mi_fill_uniform.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                              ctypes.c_void_p]
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
sp = ctypes.c_void_p(s.cuda_stream)
print("library:", lib_path, flush=True)
for logn in range(11, 21):
    n = 1 << logn
    batch = (1 << 27) >> logn  # 1 GiB of coefficients
    h = ctypes.c_void_p()
    assert L.mi_ntt64_plan_create(n, P, 0, ctypes.byref(h)) == 0
    buf = torch.empty((batch, n), dtype=torch.int64, device="cuda")
    assert L.mi_fill_uniform(ctypes.c_void_p(buf.data_ptr()), buf.numel(), 7 + logn, P, 0, sp) == 0
    res = {}
    for name, fn in (("fwd", L.mi_ntt64_fwd_batch), ("inv", L.mi_ntt64_inv_batch)):
        for _ in range(3):
            assert fn(h, ctypes.c_void_p(buf.data_ptr()), batch, n, sp) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn(h, ctypes.c_void_p(buf.data_ptr()), batch, n, sp)
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / reps
    gb = 2 * 8 * n * batch / 1e9
    print(f"N=2^{logn} batch {batch}: fwd {res['fwd'] * 1e3:8.1f} us ({gb / res['fwd'] * 1e3 / 8000:.3f} of HBM), "
          f"inv {res['inv'] * 1e3:8.1f} us ({gb / res['inv'] * 1e3 / 8000:.3f}); ns per poly fwd "
          f"{res['fwd'] * 1e6 / batch:.1f}", flush=True)
    del buf
