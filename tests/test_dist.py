"""Multi-rank gather of compressed chunks (SURVEY 8.1 row e, BASELINE configs[3]) with the gloo
backend on CPU, world size 2 and 3.

Every rank encodes its round-robin share of a global stream (global block b on rank b mod G) with the
oracle -- real chunk headers and Huffman payloads, the same layout bra_gpu_encode_blocks writes --
computes its share of the chunk-stream CRC32C the way bra_gpu_chunks_crc32c_shard does (raw CRC of
each hdr || chunk moved to the end of the GLOBAL stream), and the ranks gather to rank 0 with
br-archive_amd/dist.py.  Rank 0 interleaves the parts back into global block order and checks
headers, payloads and the merged CRC against the oracle's single-process encode of the whole stream
and its chained chunk CRC (lib_bra_io_file_chunks.c:248-249).
"""
import importlib
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BS = 4096
KINDS = (0, 1, 2)  # text, random, sym16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_blocks(total):
    bra = importlib.import_module("br-archive_amd")
    nb = (total + BS - 1) // BS
    return [bra.synth_block(KINDS[g % 3], g, min(BS, total - g * BS)) for g in range(nb)]


def _mem_header(ch) -> bytes:
    """The 268-byte in-memory bra_io_chunk_header_t (lib_bra_types.h:63-68): pi as a full u32."""
    return ch.primary_index.to_bytes(4, "little") + ch.lengths + ch.orig_size.to_bytes(4, "little") + ch.encoded_size.to_bytes(4, "little")


def _crc_share(orc, chunks, blocks, mine, nb, total, with_init, prev=0):
    """Host restatement of the device shard CRC: crc(S, prev) = ~((~prev) x^(8|S|)) ^ XOR_g L(X_g) x^(8 after_g),
    X_g = hdr_g || chunk_g, L the raw CRC (zero register, no final complement) = ~crc(X, 0xFFFFFFFF)."""
    M = 0xFFFFFFFF
    stream_len = total + 268 * nb

    def shift(a, n):  # a * x^(8n): bra_crc32c_combine(a, 0, n)
        return orc.crc32c_combine(a, 0, n) & M

    v = (~shift(~prev & M, stream_len)) & M if with_init else 0
    for g, ch in zip(mine, chunks):
        x = _mem_header(ch) + blocks[g]
        raw = (~orc.crc32c(x, M)) & M
        after = sum(268 + len(blocks[k]) for k in range(g + 1, nb))
        v ^= shift(raw, after)
    return v


def _rank_output(orc, rank, world, total):
    import numpy as np
    import torch

    dmod = importlib.import_module("br-archive_amd.dist")
    blocks = _global_blocks(total)
    nb = len(blocks)
    mine = dmod.shard_blocks(nb, rank, world)
    assert dmod.shard_bytes(total, BS, rank, world) == sum(len(blocks[g]) for g in mine)
    chunks = [orc.encode_block(blocks[g]) for g in mine]
    hdr = np.zeros((len(mine), 268), np.uint8)
    sizes = []
    for i, ch in enumerate(chunks):
        hdr[i] = np.frombuffer(_mem_header(ch), np.uint8)
        sizes.append(len(ch.payload))
    off = np.zeros(len(mine) + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    pay = np.frombuffer(b"".join(ch.payload for ch in chunks) + b"\0" * 64, np.uint8).copy()
    crc = _crc_share(orc, chunks, blocks, mine, nb, total, rank == 0)
    crc_t = torch.tensor([np.uint32(crc).view(np.int32)], dtype=torch.int32)
    return torch.from_numpy(hdr), torch.from_numpy(off), torch.from_numpy(pay), crc_t


def _worker(rank, world, port, total, q, bound=False):
    try:
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist

        from oracle import Oracle

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dmod = importlib.import_module("br-archive_amd.dist")
        orc = Oracle()
        hdr, off, pay, crc = _rank_output(orc, rank, world, total)
        if bound:
            # sizes from the geometry: the payload travels at its bound (its tail is padding)
            g = dmod.ChunkGather(dist, rank, world, geometry=(total, BS))
            pb = dmod.shard_payload_bound(total, BS, rank, world)
            assert pb >= pay.numel() - 64
            pay = torch.cat([pay, torch.full((pb + 64 - pay.numel(),), 0xEE, dtype=torch.uint8)])
        else:
            g = dmod.ChunkGather(dist, rank, world)
        for _ in range(2):  # the second call reuses the receive buffers
            parts = g(hdr, off, pay, crc)
        ok = True
        if rank == 0:
            hdrs, offs, pays = dmod.assemble_host(parts, round_robin=True)
            blocks = _global_blocks(total)
            want = [orc.encode_block(b) for b in blocks]
            ok = hdrs.shape[0] == len(blocks)
            for gb, ch in enumerate(want):
                ok &= hdrs[gb].numpy().tobytes() == _mem_header(ch)
                ok &= pays[int(offs[gb]): int(offs[gb + 1])].numpy().tobytes() == ch.payload
            whole = orc.chunks_crc32c(b"".join(_mem_header(ch) for ch in want), b"".join(blocks), BS, 0)
            ok &= dmod.merge_crc(parts) == whole
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, bool(ok)))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("world,total,bound", [(2, 7 * BS - 3096, False), (3, 8 * BS, False), (2, 1 * BS, False), (2, 7 * BS - 3096, True),
                                               (3, 8 * BS, True)])
def test_gather_chunks_gloo(world, total, bound):
    """bound: sizes from the geometry (no size all_gather), payloads at their bound."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q, bound)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}, res


def test_shard_blocks_round_robin():
    dmod = importlib.import_module("br-archive_amd.dist")
    assert dmod.shard_blocks(2048, 3, 8)[:3] == [3, 11, 19]
    assert len(dmod.shard_blocks(2048, 3, 8)) == 256
    assert sorted(g for r in range(3) for g in dmod.shard_blocks(10, r, 3)) == list(range(10))
    # only the rank holding the global last block gets a short one
    assert [dmod.shard_bytes(10 * BS - 5, BS, r, 3) for r in range(3)] == [4 * BS - 5, 3 * BS, 3 * BS]
    assert dmod.shard_bytes(BS, BS, 1, 2) == 0


def test_bench_spawns_torchrun_before_touching_the_gpu():
    # bench.py --gpus N (N > 1) without a torchrun environment relaunches itself as N ranks
    src = open(os.path.join(ROOT, "bench.py")).read()
    main = src[src.index("def main():"):]
    assert main.index("spawn_torchrun(args)") < main.index("import torch")
    assert "torch.distributed.run" in src and "--nproc-per-node" in src
