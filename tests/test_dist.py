"""Multi-rank gather of compressed chunks (SURVEY 8.1 row e) with the gloo backend on CPU, world size 2.

Each rank fabricates the chunk headers and payload of its own block range (the same layout the
encoder produces), the ranks gather to rank 0 with br-archive_amd/dist.py, and rank 0 checks that the
assembled stream holds every block in global order.
"""
import importlib
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_rank_output(rank, nb):
    """Headers + payload of nb blocks as rank `rank` would produce them (deterministic per global block)."""
    import numpy as np
    import torch

    dist_mod = importlib.import_module("br-archive_amd.dist")
    first, n = dist_mod.shard_blocks(nb, rank)
    hdr = np.zeros((n, 268), np.uint8)
    pays = []
    for i in range(n):
        g = first + i
        size = 17 + (g * 37) % 101 if g % 5 else 0  # some empty payloads
        hdr[i, 0:4] = np.frombuffer(np.uint32(g).tobytes(), np.uint8)
        hdr[i, 264:268] = np.frombuffer(np.uint32(size).tobytes(), np.uint8)
        pays.append(((np.arange(size) * (g + 3)) % 251).astype(np.uint8))
    pay = np.concatenate(pays) if pays else np.zeros(0, np.uint8)
    total = pay.size
    buf = np.zeros(total + 64, np.uint8)
    buf[:total] = pay
    return torch.from_numpy(hdr), torch.tensor([total], dtype=torch.int64), torch.from_numpy(buf), pays


def _worker(rank, world, port, nb, q):
    try:
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist_mod = importlib.import_module("br-archive_amd.dist")
        hdr, size, pay, _ = _fake_rank_output(rank, nb)
        g = dist_mod.ChunkGather(dist, rank, world)
        for _ in range(2):  # second call reuses the receive buffers
            parts = g(hdr, size, pay)
        ok = True
        if rank == 0:
            hdrs, pays, offs = dist_mod.assemble(parts)
            ok = hdrs.shape[0] == nb * world
            for r in range(world):
                _, _, _, want = _fake_rank_output(r, nb)
                for i, p in enumerate(want):
                    gb = r * nb + i
                    ok &= int.from_bytes(hdrs[gb, 0:4].numpy().tobytes(), "little") == gb
                    got = pays[offs[gb]: offs[gb + 1]].numpy()
                    ok &= got.tobytes() == p.tobytes()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, bool(ok)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2])
def test_gather_chunks_gloo(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 7, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}, res


def test_shard_blocks():
    dist_mod = importlib.import_module("br-archive_amd.dist")
    assert dist_mod.shard_blocks(256, 0) == (0, 256)
    assert dist_mod.shard_blocks(256, 3) == (768, 256)
