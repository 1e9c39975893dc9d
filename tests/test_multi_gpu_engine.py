"""Config 5's split through the real engine.

* CPU: the C-ABI shard arithmetic (``mi_multi_gpu_shard`` / ``_active_count``) equals the reference's
  get_num_inputs_on_gpu / get_gpu_offset / get_active_gpu_count (helper_multi_gpu.cu:42-98, restated
  below with its float ceil) and ``multi_gpu.shard_bounds``.
* GPU, one process: ``DeviceSet([0, 0, 0])`` scatters a batch from entry 0, bootstraps every shard with the
  real PBS and gathers it back (``mi_pbs_ntt64_multi_gpu``): identical to one launch and to the oracle.
* GPU, two processes (world size 2, gloo, both ranks on cuda:0 — the one-GPU rehearsal of the RCCL path):
  the root holds the global LWE batch and the key, broadcasts the key, scatters the batch, every rank runs
  the real NTT and PBS on its shard, the root gathers; the gathered result equals the single-rank run and
  the oracle.
"""
import math
import os
import socket

import numpy as np
import pytest

import tfhe_helpers as H

P = 0xFFFFFFFF00000001
N = 2048


def _ref_inputs_on_gpu(total, i, count):
    """helper_multi_gpu.cu:66-98, restated as written (float ceil, cutoff)."""
    if count > total:
        return 1 if i < total else 0
    if total % count == 0:
        small = large = total // count
        cutoff = 0
    else:
        y = math.ceil(total / count) * count - total
        cutoff = count - y
        small, large = total // count, math.ceil(total / count)
    return large if i < cutoff else small


def test_shard_arithmetic_matches_reference(engine):
    mg = engine.multi_gpu
    for total in (0, 1, 5, 8, 9, 4095, 4096, 65536, 65537):
        for count in (1, 2, 3, 7, 8):
            off = 0
            for i in range(count):
                n = _ref_inputs_on_gpu(total, i, count)
                assert mg.lib_shard(total, i, count) == (off, off + n), (total, count, i)
                if total >= count:
                    assert mg.shard_bounds(total, count, i) == (off, off + n)
                off += n
    for num_inputs in (0, 1, 12, 13, 100, 10**6):
        for g in (1, 2, 8):
            assert mg.lib_active_count(num_inputs, g) == min(max(1, -(-num_inputs // 12)), g)
    with pytest.raises(engine.MiError):
        mg.lib_shard(10, 3, 3)


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def _host(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.gpu
def test_device_set_gather_waits_for_the_caller_stream(engine):
    """mi_multi_gpu_gather's copies are ordered after the work already queued on the caller's stream (the header's
    contract): a zero-fill of the destination queued behind a long transform loop on that stream must land before
    the gathered shards, not over them (r4: the gather used to start its copies at once, and a zero-fill still queued
    on the caller stream could overwrite them; seen once in test_device_set_pbs_scatter_gather)."""
    import torch
    ds = engine.multi_gpu.DeviceSet([0, 0, 0])
    g = H.rng(4242)
    total, width = 7, 33
    shards_h = [H.uniform_u64(g, (b - a, width)) for a, b in (ds.shard(total, i) for i in range(3))]
    shards = [_dev(x) for x in shards_h]
    torch.cuda.synchronize()
    plan = engine.Plan.try_new(N, P)
    busy = torch.zeros((8192, N), dtype=torch.int64, device="cuda")
    dst = torch.full((total, width), 7, dtype=torch.int64, device="cuda")
    for _ in range(20):  # ~2 ms of work queued on the caller (current) stream ahead of the zero-fill
        plan.fwd(busy)
    dst.zero_()
    ds.gather(dst, shards)
    torch.cuda.synchronize()
    assert np.array_equal(_host(dst), np.concatenate(shards_h))


@pytest.mark.gpu
@pytest.mark.parametrize("entries,batch", [(2, 9), (3, 10), (3, 2)])
def test_device_set_pbs_scatter_gather(engine, oracle, entries, batch):
    import torch
    M = engine.ntt64_pbs
    g = H.rng(900 + entries + batch)
    n_lwe = 20
    plan = engine.Plan.try_new(N, P)
    bsk = g.integers(0, P, size=(n_lwe, 1, 2, 2, N), dtype=np.uint64)
    lut = H.uniform_u64(g, (2, N))
    lwe = H.uniform_u64(g, (batch, n_lwe + 1))
    key = M.NttBootstrapKey(plan, _dev(bsk), 23, 1, M.BNF)
    ds = engine.multi_gpu.DeviceSet([0] * entries)
    # scatter / gather round trip and broadcast
    src = _dev(lwe)
    shards = [torch.empty((b - a, n_lwe + 1), dtype=torch.int64, device="cuda") for a, b in
              (ds.shard(batch, i) for i in range(entries))]
    ds.scatter(src, shards)
    back = torch.zeros_like(src)
    ds.gather(back, shards)
    torch.cuda.synchronize()
    assert np.array_equal(_host(back), lwe)
    copies = [torch.zeros(2, N, dtype=torch.int64, device="cuda") for _ in range(entries)]
    lt = _dev(lut)
    ds.broadcast(lt, copies)
    ds.synchronize()
    assert all(np.array_equal(_host(c), lut) for c in copies)
    # the multi-device PBS == one launch == the oracle
    out_multi = torch.zeros((batch, N + 1), dtype=torch.int64, device="cuda")
    ds.programmable_bootstrap([key] * entries, src, out_multi, copies)
    out_one = torch.zeros_like(out_multi)
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(src, out_one, lt, key)
    torch.cuda.synchronize()
    assert np.array_equal(_host(out_multi), _host(out_one))
    ctx = oracle.NttContext(N)
    assert np.array_equal(_host(out_multi)[-1], ctx.pbs(lwe[-1], lut.reshape(-1), bsk.reshape(-1), 1, 23, 1, bnf=True))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


GLOBAL_PBS, GLOBAL_POLYS, N_LWE = 11, 13, 24


def _rank_main(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tfhe-rs-main_modified_amd"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import tfhe_ntt_amd as eng
        mg, M = eng.multi_gpu, eng.ntt64_pbs
        torch.cuda.set_device(0)
        plan = eng.Plan.try_new(N, P)
        g = H.rng(4242)
        # the root's state: key, LUT, global batches (host tensors: gloo moves host memory)
        if rank == 0:
            bsk = torch.from_numpy(g.integers(0, P, size=(N_LWE, 1, 2, 2, N), dtype=np.uint64).view(np.int64))
            lut = torch.from_numpy(H.uniform_u64(g, (2, N)).view(np.int64))
            lwe_all = torch.from_numpy(H.uniform_u64(g, (GLOBAL_PBS, N_LWE + 1)).view(np.int64))
            polys_all = torch.from_numpy(g.integers(0, P, size=(GLOBAL_POLYS, N), dtype=np.uint64).view(np.int64))
        else:
            bsk = torch.zeros((N_LWE, 1, 2, 2, N), dtype=torch.int64)
            lut = torch.zeros((2, N), dtype=torch.int64)
            lwe_all = polys_all = None
        mg.broadcast_(bsk)
        mg.broadcast_(lut)
        a, b = mg.shard_bounds(GLOBAL_PBS, world, rank)
        lwe = torch.empty((b - a, N_LWE + 1), dtype=torch.int64)
        mg.scatter_batch(lwe_all, lwe)
        pa, pb = mg.shard_bounds(GLOBAL_POLYS, world, rank)
        polys = torch.empty((pb - pa, N), dtype=torch.int64)
        mg.scatter_batch(polys_all, polys)
        # the real engine on this rank's shard
        key = M.NttBootstrapKey(plan, bsk.cuda(), 23, 1, M.BNF)
        out = torch.zeros((b - a, N + 1), dtype=torch.int64, device="cuda")
        if b > a:
            M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(lwe.cuda(), out, lut.cuda(), key)
        tp = polys.cuda()
        if pb > pa:
            plan.fwd(tp)
        torch.cuda.synchronize()
        out_all = torch.zeros((GLOBAL_PBS, N + 1), dtype=torch.int64) if rank == 0 else None
        fwd_all = torch.zeros((GLOBAL_POLYS, N), dtype=torch.int64) if rank == 0 else None
        mg.gather_batch(out.cpu(), out_all)
        mg.gather_batch(tp.cpu(), fwd_all)
        if rank == 0:
            # single-rank reference run of the same global batches
            one = torch.zeros((GLOBAL_PBS, N + 1), dtype=torch.int64, device="cuda")
            M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(lwe_all.cuda(), one, lut.cuda(), key)
            tp1 = polys_all.cuda()
            plan.fwd(tp1)
            torch.cuda.synchronize()
            assert torch.equal(out_all, one.cpu()), "sharded PBS != single-rank PBS"
            assert torch.equal(fwd_all, tp1.cpu()), "sharded NTT != single-rank NTT"
            np.save(os.environ["MI_MG_OUT"] + "_pbs.npy", out_all.numpy())
            np.save(os.environ["MI_MG_OUT"] + "_fwd.npy", fwd_all.numpy())
            np.save(os.environ["MI_MG_OUT"] + "_in.npy", lwe_all.numpy())
            np.save(os.environ["MI_MG_OUT"] + "_polys.npy", polys_all.numpy())
            np.save(os.environ["MI_MG_OUT"] + "_bsk.npy", bsk.numpy())
            np.save(os.environ["MI_MG_OUT"] + "_lut.npy", lut.numpy())
        q.put((rank, "ok"))
    except Exception as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_real_engine(oracle, tmp_path):
    import torch.multiprocessing as mp
    os.environ["MI_MG_OUT"] = str(tmp_path / "mg")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    results = sorted(q.get(timeout=5) for _ in range(2))
    assert not alive and results == [(0, "ok"), (1, "ok")], results
    base = str(tmp_path / "mg")
    out = np.load(base + "_pbs.npy").view(np.uint64)
    lwe = np.load(base + "_in.npy").view(np.uint64)
    bsk = np.load(base + "_bsk.npy").view(np.uint64)
    lut = np.load(base + "_lut.npy").view(np.uint64)
    want = oracle.NttContext(N).pbs_batch_bnf(lwe, lut.reshape(-1), bsk.reshape(-1), 1, 23, 1, threads=8)
    assert np.array_equal(out, want)
    polys = np.load(base + "_polys.npy").view(np.uint64)
    assert np.array_equal(np.load(base + "_fwd.npy").view(np.uint64), oracle.Plan.try_new(N, P).fwd(polys))


@pytest.mark.gpu
def test_device_set_active_count_13_on_8(engine, oracle):
    """get_active_gpu_count inside mi_pbs_ntt64_multi_gpu (helper_multi_gpu.cu:42-49): 13 bootstraps on an
    8-entry set run on the first ceil(13 / 12) = 2 entries (7 + 6).  The other six entries get no key and no
    LUT (None): the call succeeds only if they are never read.  Output == one launch == the oracle."""
    import torch
    M = engine.ntt64_pbs
    g = H.rng(1308)
    n_lwe, batch = 20, 13
    plan = engine.Plan.try_new(N, P)
    bsk = g.integers(0, P, size=(n_lwe, 1, 2, 2, N), dtype=np.uint64)
    lut = H.uniform_u64(g, (2, N))
    lwe = H.uniform_u64(g, (batch, n_lwe + 1))
    key = M.NttBootstrapKey(plan, _dev(bsk), 23, 1, M.BNF)
    ds = engine.multi_gpu.DeviceSet([0] * 8)
    assert ds.active_count(batch) == 2
    lt = _dev(lut)
    out_multi = torch.zeros((batch, N + 1), dtype=torch.int64, device="cuda")
    ds.programmable_bootstrap([key, key] + [None] * 6, _dev(lwe), out_multi, [lt, lt] + [None] * 6)
    with pytest.raises(ValueError):  # an active entry without a LUT is refused before the ABI
        ds.programmable_bootstrap([key] * 8, _dev(lwe), out_multi, [lt] + [None] * 7)
    out_one = torch.zeros_like(out_multi)
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(_dev(lwe), out_one, lt, key)
    torch.cuda.synchronize()
    assert np.array_equal(_host(out_multi), _host(out_one))
    want = oracle.NttContext(N).pbs_batch_bnf(lwe[[0, 6, 7, 12]], lut.reshape(-1), bsk.reshape(-1), 1, 23, 1, threads=8)
    assert np.array_equal(_host(out_multi)[[0, 6, 7, 12]], want)


@pytest.mark.gpu
def test_device_set_producer_stream_ordering(engine):
    """Every shard is ordered after the stream that produced its LUT, not only after the caller's
    stream: the LUT copies are queued on a producer stream behind ~2 ms of transforms, and the PBS is queued on
    another stream (torch's default stream) with that producer passed through mi_pbs_ntt64_multi_gpu_ordered.  An
    unordered read would bootstrap with the zero LUTs.  The producer stream is then ordered after the PBS: work
    queued on it next (zeroing the LUTs) must not reach the bootstrap."""
    import ctypes

    import torch
    from tfhe_ntt_amd._lib import check, lib
    M = engine.ntt64_pbs
    g = H.rng(77)
    n_lwe, batch, entries = 16, 48, 4
    plan = engine.Plan.try_new(N, P)
    bsk = g.integers(0, P, size=(n_lwe, 1, 2, 2, N), dtype=np.uint64)
    lut = H.uniform_u64(g, (2, N))
    lwe = H.uniform_u64(g, (batch, n_lwe + 1))
    key = M.NttBootstrapKey(plan, _dev(bsk), 23, 1, M.BNF)
    src_lut, src_lwe = _dev(lut), _dev(lwe)
    ref = torch.zeros((batch, N + 1), dtype=torch.int64, device="cuda")
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(src_lwe, ref, src_lut, key)
    busy = torch.zeros((4096, N), dtype=torch.int64, device="cuda")
    luts = [torch.zeros((2, N), dtype=torch.int64, device="cuda") for _ in range(entries)]
    out = torch.zeros_like(ref)
    torch.cuda.synchronize()
    ds = engine.multi_gpu.DeviceSet([0] * entries)
    assert ds.active_count(batch) == entries
    producer = torch.cuda.Stream()
    caller = torch.cuda.default_stream()
    with torch.cuda.stream(producer):
        for _ in range(20):
            plan.fwd(busy)
            plan.inv(busy)
        for t in luts:
            t.copy_(src_lut)
    kp = (ctypes.c_void_p * entries)(*[key._h.value] * entries)
    lp = (ctypes.c_void_p * entries)(*[t.data_ptr() for t in luts])
    ps = (ctypes.c_void_p * entries)(*[producer.cuda_stream] * entries)
    check(lib().mi_pbs_ntt64_multi_gpu_ordered(ds._h, kp, ctypes.c_void_p(out.data_ptr()),
                                               ctypes.c_void_p(src_lwe.data_ptr()), lp, batch, 0,
                                               ctypes.c_void_p(caller.cuda_stream), ps))
    with torch.cuda.stream(producer):
        for t in luts:
            t.zero_()
    torch.cuda.synchronize()
    assert np.array_equal(_host(out), _host(ref))


@pytest.mark.gpu
def test_device_set_two_distinct_devices(engine):
    """The cross-device path (peer copies, per-device keys, producer ordering on a second device); skipped on a
    one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    M = engine.ntt64_pbs
    g = H.rng(2002)
    n_lwe, batch = 16, 40
    bsk = g.integers(0, P, size=(n_lwe, 1, 2, 2, N), dtype=np.uint64)
    lut = H.uniform_u64(g, (2, N))
    lwe = H.uniform_u64(g, (batch, n_lwe + 1))
    keys, luts = [], []
    for d in (0, 1):
        with torch.cuda.device(d):
            plan = engine.Plan.try_new(N, P, device=d)
            keys.append(M.NttBootstrapKey(plan, _dev(bsk).to(f"cuda:{d}"), 23, 1, M.BNF))
            luts.append(_dev(lut).to(f"cuda:{d}"))
    ds = engine.multi_gpu.DeviceSet([0, 1])
    out = torch.zeros((batch, N + 1), dtype=torch.int64, device="cuda:0")
    ds.programmable_bootstrap(keys, _dev(lwe), out, luts)
    one = torch.zeros_like(out)
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(_dev(lwe), one, luts[0], keys[0])
    torch.cuda.synchronize()
    assert np.array_equal(_host(out), _host(one))


@pytest.mark.gpu
def test_config5_device_set_65536_real_keys(engine, oracle):
    """BASELINE config 5's workload on the HIP path: one global batch of 65,536 PBS at PARAM_MESSAGE_2_CARRY_2
    (n = 918, N = 2048, B = 2^23, l = 1, TUniform 2^45 LWE / 2^17 GLWE noise bounds, ks_pbs.rs:29-47) under real
    keys, split by mi_pbs_ntt64_multi_gpu over an 8-entry DeviceSet (one card stands in for the 8 GPUs: every
    entry is device 0, so the split, the scatter / gather copies and the 8 shard launches all run).
    * every one of the 65,536 outputs decrypts to f(m);
    * the sharded output equals one single-launch run of the whole batch, bit for bit;
    * 72 ciphertexts spread over all eight shards (every 1024th, plus each shard's first and last) equal the
      oracle PBS bit for bit."""
    import torch
    n_lwe, base_log, level, msg_mod, batch, entries = 918, 23, 1, 16, 65536, 8
    delta = (1 << 63) // msg_mod
    g = H.rng(65536918)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (1, N))
    bsk = H.bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, 17)
    f = lambda x: (3 * x + 1) % msg_mod
    lut = H.pbs_lut(N, 1, msg_mod, delta, f)
    msgs = (np.arange(batch) * 7 + 3) % msg_mod
    M = engine.ntt64_pbs
    plan = engine.Plan.try_new(N, P)
    gkey = _dev(np.zeros_like(bsk))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, _dev(bsk), gkey, normalize=False, input_modulus_width=64)
    nbsk = _host(gkey)
    key = M.NttBootstrapKey(plan, gkey, base_log, level, M.BNF)
    lwe = np.concatenate([H.lwe_encrypt_batch(g, msgs[i:i + 8192].astype(np.uint64) * np.uint64(delta), lwe_sk, 45)
                          for i in range(0, batch, 8192)])
    lt = _dev(lut)
    src = _dev(lwe)
    ds = engine.multi_gpu.DeviceSet([0] * entries)
    assert ds.active_count(batch) == entries
    out = torch.zeros((batch, N + 1), dtype=torch.int64, device="cuda")
    ds.programmable_bootstrap([key] * entries, src, out, [lt] * entries)
    one = torch.zeros_like(out)
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(src, one, lt, key)
    torch.cuda.synchronize()
    assert torch.equal(out, one), "sharded PBS != single launch"
    got = _host(out)
    del one, src
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    want_dec = np.array([f(int(m)) for m in range(msg_mod)], np.uint64)[msgs]
    for i in range(0, batch, 8192):
        pts = H.lwe_decrypt_batch(got[i:i + 8192], out_sk)
        with np.errstate(over="ignore"):
            dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
        assert np.array_equal(dec, want_dec[i:i + 8192]), f"decryption mismatch in rows {i}..{i + 8191}"
    edges = [b for i in range(entries) for b in (i * batch // entries, (i + 1) * batch // entries - 1)]
    idx = np.unique(np.concatenate([np.arange(0, batch, 1024), edges]))
    want = oracle.NttContext(N).pbs_batch_bnf(lwe[idx], lut.reshape(-1), nbsk.reshape(-1), 1, base_log, level,
                                              threads=16)
    assert np.array_equal(got[idx], want)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,level,base_log,entries,batch", [(2048, 1, 1, 23, 8, 4096), (512, 4, 1, 23, 3, 37)])
def test_device_set_fft_pbs_real_keys(engine, oracle, n, k, level, base_log, entries, batch):
    """The default f64-FFT PBS through the same multi-GPU bootstrap (`mi_fft64_pbs_multi_gpu_ordered`): config 4's
    shape (N = 2048, the one-wave engine, 8 entries, 4096 ciphertexts) and the MESSAGE_1_CARRY_1 shape (N = 512,
    k = 4, the generic engine, a ragged 37 over 3 entries).  The sharded output equals one launch bit for bit (each
    ciphertext's f64 arithmetic does not depend on which shard or workgroup holds it) and every output decrypts."""
    import torch
    F = engine.fft64
    n_lwe, msg_mod = 64, 16
    delta = (1 << 63) // msg_mod
    g = H.rng(7700 + n + entries)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen_fast(g, oracle, lwe_sk, glwe_sk, base_log, level, 17)
    fft = F.Fft(n)
    fbsk = torch.zeros((n_lwe, level, k + 1, k + 1, n // 2, 2), dtype=torch.float64, device="cuda")
    F.convert_standard_lwe_bootstrap_key_to_fourier(_dev(bsk), fbsk, fft)
    key = F.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    f = lambda x: (3 * x + 5) % msg_mod
    lut = _dev(H.pbs_lut(n, k, msg_mod, delta, f))
    msgs = np.arange(batch) % msg_mod
    src = _dev(H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 30))
    ds = engine.multi_gpu.DeviceSet([0] * entries)
    active = ds.active_count(batch)
    out = torch.zeros((batch, k * n + 1), dtype=torch.int64, device="cuda")
    ds.programmable_bootstrap([key] * active + [None] * (entries - active), src, out,
                              [lut] * active + [None] * (entries - active), F.MS_CENTERED)
    one = torch.zeros_like(out)
    F.programmable_bootstrap_lwe_ciphertext(src, one, lut, key, F.MS_CENTERED)
    torch.cuda.synchronize()
    assert torch.equal(out, one), "sharded f64 PBS != single launch"
    pts = H.lwe_decrypt_batch(_host(out), H.glwe_sk_as_lwe_sk(glwe_sk))
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert np.array_equal(dec, np.array([f(int(m)) for m in msgs], np.uint64))
    with pytest.raises(ValueError):  # one engine per call
        ntt_key = engine.ntt64_pbs.NttBootstrapKey(engine.Plan.try_new(2048, P),
                                                   _dev(np.zeros((n_lwe, 1, 2, 2, 2048), np.uint64)), 23, 1,
                                                   engine.ntt64_pbs.BNF)
        ds.programmable_bootstrap([key, ntt_key] + [key] * (entries - 2), src, out, [lut] * entries)
