"""Multi-rank batch sharding on CPU: world_size-2 gloo process groups.

The GPU path uses the same functions over RCCL; only the backend and the tensor device differ.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tfhe-rs-main_modified_amd")


def _multi_gpu():
    # import the module file directly: no libtfhe_ntt_amd.so needed for the host-side logic
    import importlib.util

    spec = importlib.util.spec_from_file_location("mg", os.path.join(PKG, "tfhe_ntt_amd", "multi_gpu.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_shard_bounds_cover_and_balance():
    mg = _multi_gpu()
    for total in (0, 1, 7, 8, 65536, 65537, 4095):
        for world in (1, 2, 3, 8):
            spans = [mg.shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
    with pytest.raises(ValueError):
        mg.shard_bounds(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mg = _multi_gpu()
        # replicated key material
        key = torch.arange(16, dtype=torch.int64) if rank == 0 else torch.zeros(16, dtype=torch.int64)
        mg.broadcast_(key)
        assert torch.equal(key, torch.arange(16, dtype=torch.int64))
        # root-held batch of "LWE ciphertexts" scattered, transformed per shard, gathered back
        a, b = mg.shard_bounds(total, world, rank)
        glob = torch.arange(total * 5, dtype=torch.int64).reshape(total, 5) if rank == 0 else None
        shard = torch.empty((b - a, 5), dtype=torch.int64)
        mg.scatter_batch(glob, shard)
        assert torch.equal(shard, torch.arange(a * 5, b * 5, dtype=torch.int64).reshape(b - a, 5))
        shard = shard * 3 + rank * 0  # the per-shard "bootstrap"
        out = torch.empty((total, 5), dtype=torch.int64) if rank == 0 else None
        mg.gather_batch(shard, out)
        if rank == 0:
            assert torch.equal(out, torch.arange(total * 5, dtype=torch.int64).reshape(total, 5) * 3)
        t = mg.max_over_ranks(1.0 + rank)
        assert t == float(world)
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent instead of hanging
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [9, 2, 1])
def test_gloo_world2_scatter_compute_gather(total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    results = sorted(q.get(timeout=5) for _ in range(world))
    for p in procs:
        if p.is_alive():
            p.kill()
    assert results == [(0, "ok"), (1, "ok")], results


class _FakeDist:
    """Records the point-to-point ops scatter_batch / gather_batch build (the RCCL path's op construction, checked
    without a process group or a GPU)."""

    def __init__(self, world, rank):
        self.world, self.rank, self.posted = world, rank, []
        self.isend, self.irecv = "isend", "irecv"

    def get_world_size(self):
        return self.world

    def get_rank(self):
        return self.rank

    def P2POp(self, op, tensor, peer):  # noqa: N802 (torch.distributed's name)
        return (op, tensor, peer)

    def batch_isend_irecv(self, ops):
        assert ops, "an empty op list must not be posted"
        self.posted.append(list(ops))

        class W:
            def wait(self):
                pass
        return [W() for _ in ops]


@pytest.mark.parametrize("total,world", [(13, 8), (5, 8), (65536, 8), (7, 2)])
@pytest.mark.parametrize("device", ["cpu", "meta"])
def test_p2p_op_construction(monkeypatch, total, world, device):
    """scatter_batch / gather_batch on every rank of an 8-rank job: the root posts one send (scatter) / receive
    (gather) per non-empty peer shard, on a contiguous slice of the right rows, on the batch's own device (meta
    tensors stand in for device tensors: nothing is moved to the host); an empty shard posts nothing on either side;
    the root's own shard is a local copy."""
    mg = _multi_gpu()
    width = 919
    glob = torch.arange(total * width, dtype=torch.int64).reshape(total, width).to(device)
    for rank in range(world):
        fd = _FakeDist(world, rank)
        monkeypatch.setattr(mg, "_dist", lambda fd=fd: fd)
        a, b = mg.shard_bounds(total, world, rank)
        shard = torch.empty((b - a, width), dtype=torch.int64, device=device)
        mg.scatter_batch(glob if rank == 0 else None, shard, src=0)
        if rank == 0:
            ops = fd.posted[0] if fd.posted else []
            peers = [p for _, _, p in ops]
            want = [r for r in range(1, world) if mg.shard_bounds(total, world, r)[1] > mg.shard_bounds(total, world, r)[0]]
            assert peers == want
            for op, t, p in ops:
                pa, pb = mg.shard_bounds(total, world, p)
                assert op == "isend" and tuple(t.shape) == (pb - pa, width) and t.is_contiguous()
                assert t.device.type == device and t.dtype == torch.int64
                if device == "cpu":
                    assert torch.equal(t, glob[pa:pb])
            if device == "cpu":
                assert torch.equal(shard, glob[a:b])
        else:
            if b == a:
                assert fd.posted == []
            else:
                (op, t, p), = fd.posted[0]
                assert op == "irecv" and p == 0 and t.data_ptr() == shard.data_ptr()
        # gather back into a column-sliced (non-contiguous) global buffer on the root
        fd.posted.clear()
        out = torch.zeros((total, width + 1), dtype=torch.int64, device=device)[:, :width] if rank == 0 else None
        mg.gather_batch(shard, out, dst=0)
        if rank == 0:
            ops = fd.posted[0] if fd.posted else []
            for op, t, p in ops:
                pa, pb = mg.shard_bounds(total, world, p)
                assert op == "irecv" and tuple(t.shape) == (pb - pa, width) and t.is_contiguous()
                assert t.device.type == device
            assert len(ops) == len(want)
        elif b == a:
            assert fd.posted == []
        else:
            (op, t, p), = fd.posted[0]
            assert op == "isend" and p == 0 and tuple(t.shape) == (b - a, width)
