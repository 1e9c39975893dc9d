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


__all__ = ["shard_bounds", "broadcast_", "scatter_batch", "gather_batch", "max_over_ranks"]
