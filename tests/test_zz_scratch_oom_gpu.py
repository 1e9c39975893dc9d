"""The scratch pool under device-memory pressure and across destroyed streams (`-m gpu`; named to run last: it fills
the card).

ADVICE r5: since the pool keeps a large idle block for the large requests it was made for, a small request allocates
a new block; when that hipMalloc fails the request must still be served — from the large idle block, or after the
pool frees its idle blocks — instead of returning OOM where the pre-r5 pool succeeded (csrc/scratch.cpp
scratch_alloc).  The keyswitch's digit buffer is the scratch request here (batch 131,072: a 1 GiB block; batch 16:
128 KiB), its output checked against the same call made before the card was full.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fill_device(torch, dev, floor_bytes=1 << 20):
    """Allocate device memory in halving chunk sizes until even `floor_bytes` fails; returns the tensors held."""
    held, size = [], 8 << 30
    while size >= floor_bytes:
        try:
            held.append(torch.empty(size, dtype=torch.uint8, device=dev))
        except torch.cuda.OutOfMemoryError:
            size //= 2
    return held


def test_blocks_last_used_on_a_destroyed_stream(engine, oracle):
    """A DeviceSet's streams are destroyed with it (mi_multi_gpu_destroy) while scratch blocks whose last use ran on
    them sit idle in the pool.  Reusing or trimming those blocks must not wait on the dead streams' events (on ROCm that
    fails with hipErrorCapturedEvent and leaves the runtime's sticky error for the next torch launch to report): the
    destroy marks them retired (scratch_stream_retired), and any other dead-stream event falls back to a device-wide
    wait (scratch.cpp wait_last_use).  The keyswitch after the destroy reuses such a block and must stay exact."""
    import gc

    import torch
    KS = engine.lwe_keyswitch
    M = engine.ntt64_pbs
    dev = torch.device("cuda:0")
    M.scratch_trim(0)
    g = np.random.Generator(np.random.PCG64(0x5D))
    n_lwe, batch, N = 16, 64, 2048
    P = 0xFFFFFFFF00000001
    plan = engine.Plan.try_new(N, P)
    bsk = torch.from_numpy(g.integers(0, P, size=(n_lwe, 1, 2, 2, N), dtype=np.uint64).view(np.int64)).to(dev)
    key = M.NttBootstrapKey(plan, bsk, 23, 1, M.BNF)
    lut = torch.from_numpy(g.integers(0, 2**64, size=(2, N), dtype=np.uint64).view(np.int64)).to(dev)
    src = torch.from_numpy(g.integers(0, 2**64, size=(batch, n_lwe + 1), dtype=np.uint64).view(np.int64)).to(dev)
    ds = engine.multi_gpu.DeviceSet([0, 0])
    out = torch.zeros((batch, N + 1), dtype=torch.int64, device=dev)
    ds.programmable_bootstrap([key, key], src, out, [lut, lut])
    ds.synchronize()
    held = M.scratch_bytes(0)
    assert held > 0  # the DeviceSet's staging blocks are idle in the pool
    del ds
    gc.collect()
    # a scratch user on the caller's stream reuses an idle block last used on a destroyed stream
    in_dim, out_dim = 64, 32
    ksk = torch.from_numpy(g.integers(0, 2**64, size=(in_dim, 2, out_dim + 1), dtype=np.uint64).view(np.int64)).to(dev)
    kkey = KS.LweKeyswitchKey(ksk, 8, 2)
    lin = torch.from_numpy(g.integers(0, 2**64, size=(4, in_dim + 1), dtype=np.uint64).view(np.int64)).to(dev)
    lout = torch.zeros((4, out_dim + 1), dtype=torch.int64, device=dev)
    KS.keyswitch_lwe_ciphertext(kkey, lin, lout)
    torch.cuda.synchronize()
    want = oracle.lwe_keyswitch(ksk.cpu().numpy().view(np.uint64), lin.cpu().numpy().view(np.uint64), out_dim, 8, 2)
    assert np.array_equal(lout.cpu().numpy().view(np.uint64), want)
    M.scratch_trim(0)
    z = torch.zeros((1 << 20,), dtype=torch.int64, device=dev)  # the next torch launch sees no stale HIP error
    torch.cuda.synchronize()
    assert int(z.sum()) == 0


def test_small_request_served_when_device_memory_is_full(engine, oracle):
    import torch
    KS = engine.lwe_keyswitch
    M = engine.ntt64_pbs
    dev = torch.device("cuda:0")
    in_dim, out_dim, base_log, level = 2048, 918, 4, 4
    g = np.random.Generator(np.random.PCG64(0x5C))
    ksk = torch.from_numpy(g.integers(0, 2**64, size=(in_dim, level, out_dim + 1), dtype=np.uint64).view(np.int64)).to(dev)
    key = KS.LweKeyswitchKey(ksk, base_log, level)
    del ksk
    small_in = torch.from_numpy(g.integers(0, 2**64, size=(16, in_dim + 1), dtype=np.uint64).view(np.int64)).to(dev)
    small_out = torch.zeros((16, out_dim + 1), dtype=torch.int64, device=dev)
    KS.keyswitch_lwe_ciphertext(key, small_in, small_out)
    torch.cuda.synchronize()
    want = small_out.clone()
    M.scratch_trim(0)
    # a large call leaves a 1 GiB idle block behind
    big_in = torch.zeros((131072, in_dim + 1), dtype=torch.int64, device=dev)
    big_out = torch.zeros((131072, out_dim + 1), dtype=torch.int64, device=dev)
    KS.keyswitch_lwe_ciphertext(key, big_in, big_out)
    torch.cuda.synchronize()
    del big_in, big_out
    torch.cuda.empty_cache()
    assert M.scratch_bytes(0) >= 1 << 30
    held = []
    small_out.zero_()
    try:
        held = _fill_device(torch, dev)
        KS.keyswitch_lwe_ciphertext(key, small_in, small_out)  # its new 1 MiB block cannot be allocated
        torch.cuda.synchronize()
    finally:
        del held
        torch.cuda.empty_cache()
        M.scratch_trim(0)
    # compared once the card has room again: torch's own comparison kernel loads its code object lazily, which needs
    # device memory
    assert torch.equal(small_out, want)
