"""Multi-GPU sharding of the block codec (SURVEY.md 8.1 row e).

Blocks are independent, so ranks never talk while they encode: rank r owns the contiguous block
range `shard_blocks(...)` of the global stream (weak scaling: every rank encodes the same number of
blocks).  The one exchange step gathers the compressed chunks to rank 0 in global block order:

  1. all_gather of each rank's payload byte count (one int64 per rank),
  2. per peer one send/recv of its chunk headers (nblocks x 268 B, `bra_io_chunk_header_t`) and
     one of its payload bytes, posted together with batch_isend_irecv.

With the "nccl" backend (RCCL on ROCm) the tensors are device tensors and the copies run over
xGMI; the same code runs with "gloo" on CPU tensors (tests/test_dist.py).
"""
from __future__ import annotations

HEADER_BYTES = 268


def shard_blocks(nblocks_per_rank: int, rank: int) -> tuple[int, int]:
    """Global block range [first, first + n) that `rank` encodes."""
    return rank * nblocks_per_rank, nblocks_per_rank


class ChunkGather:
    """Gathers (headers, payload) of every rank to rank 0; receive buffers are kept between calls."""

    def __init__(self, dist, rank: int, world: int):
        self.dist, self.rank, self.world = dist, rank, world
        self.bufs: dict[int, tuple] = {}

    def __call__(self, hdr, payload_bytes, pay):
        """hdr: uint8 [nb, 268]; payload_bytes: int64 tensor [1] (this rank's payload size);
        pay: uint8 payload buffer.  Returns on rank 0 a list over ranks of (hdr, payload view);
        None elsewhere."""
        import torch

        dist, rank, world = self.dist, self.rank, self.world
        sizes = [torch.empty_like(payload_bytes) for _ in range(world)]
        dist.all_gather(sizes, payload_bytes)
        sizes = [int(s.item()) for s in sizes]
        ops = []
        if rank == 0:
            for r in range(1, world):
                if r not in self.bufs or self.bufs[r][1].numel() < sizes[r] or self.bufs[r][0].shape != hdr.shape:
                    self.bufs[r] = (torch.empty_like(hdr), torch.empty((int(sizes[r] * 1.1) + 4096,), dtype=torch.uint8, device=pay.device))
                ops.append(dist.P2POp(dist.irecv, self.bufs[r][0], r))
                if sizes[r]:
                    ops.append(dist.P2POp(dist.irecv, self.bufs[r][1][: sizes[r]], r))
        else:
            ops.append(dist.P2POp(dist.isend, hdr, 0))
            if sizes[rank]:
                ops.append(dist.P2POp(dist.isend, pay[: sizes[rank]], 0))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if rank != 0:
            return None
        parts = [(hdr, pay[: sizes[0]])]
        for r in range(1, world):
            parts.append((self.bufs[r][0], self.bufs[r][1][: sizes[r]]))
        return parts


def assemble(parts):
    """Concatenate gathered parts in global block order: (headers [N, 268], payload, offsets [N+1])."""
    import torch

    hdrs = torch.cat([h for h, _ in parts], 0)
    pays = torch.cat([p for _, p in parts], 0)
    sizes = hdrs[:, 264:268].contiguous().view(torch.int32).to(torch.int64).flatten()  # encoded_size field
    offs = torch.zeros(hdrs.shape[0] + 1, dtype=torch.int64, device=hdrs.device)
    offs[1:] = torch.cumsum(sizes, 0)
    return hdrs, pays, offs
