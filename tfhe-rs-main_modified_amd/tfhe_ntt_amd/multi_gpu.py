"""Batch sharding of independent polynomials / bootstraps over the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU
for the tests).  Polynomials (config 2), external products (config 3) and bootstraps (configs 4-5)
are independent, so the data path has no collective: each rank transforms its own contiguous
shard.  Collectives appear only at the edges, mirroring the CUDA backend's multi-GPU helpers
(/root/reference/backends/tfhe-cuda-backend/cuda/src/utils/helper_multi_gpu.cu:10-98):

* ``shard_bounds``   — contiguous split, the first ``B % G`` ranks take one extra item
                       (helper_multi_gpu.cu:55-87 get_num_inputs_on_gpu / get_gpu_offset);
* ``broadcast_``     — replicate read-only state (plan-independent key material: the NTT-domain
                       bootstrap key, LUTs) from the root once;
* ``scatter_batch`` / ``gather_batch`` — root-held batch out to the shards and results back
                       (grouped point-to-point: xGMI is point-to-point, so the root talks to each
                       peer over its own link instead of a ring);
* ``max_over_ranks`` — the benchmark's whole-job time.

``DeviceSet`` is the single-process form of the same split over the C ABI (``mi_multi_gpu_*``): one host
process driving several devices, as tfhe-rs's ``CudaStreams`` do — peer-to-peer scatter / gather /
broadcast from the first device and a whole multi-GPU PBS (``mi_pbs_ntt64_multi_gpu``).
"""
from __future__ import annotations


def shard_bounds(total: int, world: int, rank: int) -> tuple[int, int]:
    """[start, stop) of ``rank``'s contiguous shard of ``total`` items over ``world`` ranks."""
    if world <= 0 or not 0 <= rank < world or total < 0:
        raise ValueError(f"bad shard request total={total} world={world} rank={rank}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _dist():
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialised")
    return dist


def broadcast_(tensor, src: int = 0):
    """In-place broadcast of read-only state (e.g. the 60 MB NTT bootstrap key) from ``src``."""
    _dist().broadcast(tensor, src=src)
    return tensor


def scatter_batch(global_batch, out_shard, src: int = 0) -> None:
    """Root sends each rank its contiguous shard of ``global_batch`` (leading dim = items);
    every rank receives into ``out_shard``.  ``global_batch`` is only read on ``src``."""
    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == src:
        total = global_batch.shape[0]
        ops = []
        for r in range(world):
            a, b = shard_bounds(total, world, r)
            if r == src:
                out_shard.copy_(global_batch[a:b])
            elif b > a:
                ops.append(dist.P2POp(dist.isend, global_batch[a:b].contiguous(), r))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
    elif out_shard.shape[0] > 0:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, out_shard, src)]):
            w.wait()


def gather_batch(shard, global_out, dst: int = 0) -> None:
    """Inverse of ``scatter_batch``: every rank's shard lands in ``global_out`` on ``dst``."""
    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == dst:
        total = global_out.shape[0]
        ops, views = [], []
        for r in range(world):
            a, b = shard_bounds(total, world, r)
            if r == dst:
                global_out[a:b].copy_(shard)
            elif b > a:
                buf = global_out[a:b] if global_out[a:b].is_contiguous() else global_out[a:b].clone()
                views.append((buf, a, b))
                ops.append(dist.P2POp(dist.irecv, buf, r))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        for buf, a, b in views:
            if buf.data_ptr() != global_out[a:b].data_ptr():
                global_out[a:b].copy_(buf)
    elif shard.shape[0] > 0:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, shard.contiguous(), dst)]):
            w.wait()


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host float over all ranks (whole-job time = slowest rank)."""
    import torch

    dist = _dist()
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class DeviceSet:
    """A set of HIP devices with one stream each (``mi_multi_gpu``); entry 0 holds whole batches.  A device
    may repeat (``DeviceSet([0, 0])`` rehearses the split on one GPU)."""

    def __init__(self, devices):
        import ctypes

        from ._lib import check, lib
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        check(lib().mi_multi_gpu_create(ctypes.cast(arr, ctypes.c_void_p), len(self.devices), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                from ._lib import lib
                lib().mi_multi_gpu_destroy(h)
            except Exception:
                pass
            self._h = None

    def __len__(self):
        return len(self.devices)

    def shard(self, total: int, index: int):
        """[offset, offset + n) of entry ``index`` (``mi_multi_gpu_shard``)."""
        return lib_shard(total, index, len(self.devices))

    @staticmethod
    def _ptrs(ts):
        import ctypes
        return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])

    @staticmethod
    def _stream(t):
        import ctypes

        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def synchronize(self):
        from ._lib import check, lib
        check(lib().mi_multi_gpu_synchronize(self._h))

    def broadcast(self, src, dsts):
        import ctypes

        from ._lib import check, lib
        check(lib().mi_multi_gpu_broadcast(self._h, ctypes.c_void_p(src.data_ptr()), self._ptrs(dsts),
                                           src.numel() * src.element_size(), self._stream(src)))

    def scatter(self, src, dsts):
        """``dsts[i]`` (on ``devices[i]``) <- shard i of ``src`` (leading dim = units, on ``devices[0]``)."""
        import ctypes

        from ._lib import check, lib
        unit = src[0].numel() * src.element_size() if src.shape[0] else 0
        check(lib().mi_multi_gpu_scatter(self._h, ctypes.c_void_p(src.data_ptr()), self._ptrs(dsts), src.shape[0],
                                         unit, self._stream(src)))

    def gather(self, dst, srcs):
        import ctypes

        from ._lib import check, lib
        unit = dst[0].numel() * dst.element_size() if dst.shape[0] else 0
        check(lib().mi_multi_gpu_gather(self._h, ctypes.c_void_p(dst.data_ptr()), self._ptrs(srcs), dst.shape[0],
                                        unit, self._stream(dst)))

    def active_count(self, batch: int) -> int:
        """How many leading entries a batch of ``batch`` bootstraps runs on (``get_active_gpu_count``)."""
        return lib_active_count(batch, len(self.devices))

    def programmable_bootstrap(self, keys, lwe_in, lwe_out, luts, ms_mode: int = 0):
        """Batched PBS over the set (``mi_pbs_ntt64_multi_gpu_ordered``, or ``mi_fft64_pbs_multi_gpu_ordered`` for
        ``fft64.FourierLweBootstrapKey`` keys: the default f64-FFT path): ``keys[i]`` / ``luts[i]`` on
        ``devices[i]``, ``lwe_in`` / ``lwe_out`` on ``devices[0]``; results land in ``lwe_out`` as one launch
        would.  Only the first ``active_count(batch)`` entries run (their keys / LUTs are the only ones read;
        the others may be None).  Each device's current torch stream is passed as the producer of its key and
        LUT: shard i starts after it, and it waits for shard i's last read, so torch's caching allocator may
        reuse a LUT's memory on that stream as soon as this returns (no ``record_stream`` needed)."""
        import ctypes

        import torch

        from ._lib import check, lib
        if len(keys) != len(self.devices) or len(luts) != len(self.devices):
            raise ValueError("one key (or None) and one LUT (or None) per device of the set")
        k0 = keys[0]
        n_in, n_out = k0.input_lwe_dimension + 1, k0.output_lwe_size()
        batch = lwe_in.numel() // n_in
        if lwe_in.shape[-1] != n_in or lwe_out.shape[-1] != n_out or lwe_out.numel() // n_out != batch:
            raise ValueError("assertion failed: lwe shapes do not match the key")
        active = self.active_count(batch) if batch else 0
        for i in range(active):
            if keys[i] is None or luts[i] is None:
                raise ValueError(f"entry {i} is active for a batch of {batch}: it needs a key and a LUT")
        kp = (ctypes.c_void_p * len(keys))(*[k._h.value if k is not None else None for k in keys])
        lp = (ctypes.c_void_p * len(luts))(*[t.data_ptr() if t is not None else None for t in luts])
        prod = (ctypes.c_void_p * len(self.devices))(
            *[torch.cuda.current_stream(torch.device("cuda", d)).cuda_stream for d in self.devices])
        from .fft64 import FourierLweBootstrapKey
        fft = isinstance(k0, FourierLweBootstrapKey)
        if any(k is not None and isinstance(k, FourierLweBootstrapKey) != fft for k in keys):
            raise ValueError("keys mix the NTT and the f64-FFT engines")
        fn = lib().mi_fft64_pbs_multi_gpu_ordered if fft else lib().mi_pbs_ntt64_multi_gpu_ordered
        check(fn(self._h, kp, ctypes.c_void_p(lwe_out.data_ptr()), ctypes.c_void_p(lwe_in.data_ptr()), lp, batch,
                 ms_mode, self._stream(lwe_out), prod))


def lib_shard(total: int, index: int, count: int):
    """``mi_multi_gpu_shard`` (get_gpu_offset / get_num_inputs_on_gpu, helper_multi_gpu.cu:51-98)."""
    import ctypes

    from ._lib import check, lib
    off, n = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().mi_multi_gpu_shard(total, index, count, ctypes.byref(off), ctypes.byref(n)))
    return off.value, off.value + n.value


def lib_active_count(num_inputs: int, gpu_count: int) -> int:
    """``mi_multi_gpu_active_count`` (get_active_gpu_count, helper_multi_gpu.cu:42-49)."""
    import ctypes

    from ._lib import check, lib
    out = ctypes.c_uint32()
    check(lib().mi_multi_gpu_active_count(num_inputs, gpu_count, ctypes.byref(out)))
    return out.value


__all__ = ["shard_bounds", "broadcast_", "scatter_batch", "gather_batch", "max_over_ranks", "DeviceSet",
           "lib_shard", "lib_active_count"]
