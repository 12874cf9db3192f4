"""Multi-GPU sharding of the block codec (SURVEY.md 8.1 row e; BASELINE configs[3]).

Blocks are independent, so ranks never talk while they encode.  Global block b of the input stream
is encoded by rank b mod G (round robin, as configs[3] states); a rank's blocks sit back to back in
its own HBM in ascending global order.  The one exchange step gathers the compressed chunks to
rank 0:

  1. all_gather of each rank's payload byte count (one int64 per rank) -- or, when the gather knows
     the global geometry, nothing: every rank's block count and payload bound follow from it
     (`shard_payload_bound`), so no rank waits on the host for another rank's encode,
  2. per peer one send/recv of its chunk headers (nblocks x 268 B, `bra_io_chunk_header_t`), its
     payload offsets, its payload bytes (the exact count, or the bound: the assembly reads the
     offsets on the device) and its 4-byte share of the chunk-stream CRC, posted together with
     batch_isend_irecv,
  3. on rank 0, `BlockCodec.assemble_shards` interleaves the parts back into global block order on
     the device, and the CRC shares XOR to the CRC32C of the whole chunk stream (every rank computed
     its share with `chunks_crc32c_shard`, positions taken in the global stream).

With the "nccl" backend (RCCL on ROCm) the tensors are device tensors and the copies run over
xGMI; the same gather runs with "gloo" on CPU tensors (tests/test_dist.py), where
`assemble_host` is the host-side interleave used to check it, and with "gloo" on device tensors
through host copies (`bench.py --gpus 2 --backend gloo`: ranks sharing one GPU rehearse the N > 1
bench path end to end).
"""
from __future__ import annotations

HEADER_BYTES = 268


def num_blocks(total: int, block_size: int) -> int:
    return (total + block_size - 1) // block_size


def shard_blocks(nblocks: int, rank: int, world: int) -> list[int]:
    """Global block indices rank `rank` encodes (round robin: b -> b mod world), ascending."""
    return list(range(rank, nblocks, world))


def shard_bytes(total: int, block_size: int, rank: int, world: int) -> int:
    """Bytes of input rank `rank` holds: its blocks, only the global last one may be short."""
    nb = num_blocks(total, block_size)
    mine = shard_blocks(nb, rank, world)
    if not mine:
        return 0
    last = mine[-1]
    return (len(mine) - 1) * block_size + min(block_size, total - last * block_size)


def shard_payload_bound(total: int, block_size: int, rank: int, world: int) -> int:
    """Payload bytes rank `rank`'s blocks can take at most: per block its PackBits RLE capacity
    (n + ceil(n / 128) + 16, csrc/rle.h) plus a 16-byte word of padding, + 64 -- the bound the encode
    chain itself relies on (csrc/capi.hip encode_impl, `cap_ok`): an optimal prefix code over byte
    symbols is never longer than the 8-bit code of the RLE bytes."""
    nb = num_blocks(total, block_size)
    r = 64
    for b in shard_blocks(nb, rank, world):
        n = min(block_size, total - b * block_size)
        r += n + (n + 127) // 128 + 16 + 16
    return r


class ChunkGather:
    """Gathers (headers, offsets, payload, crc share) of every rank to rank 0; receive buffers are
    kept between calls.  With `geometry` = (global_total, block_size) (round-robin shards) the
    payloads travel at their bound and no sizes are exchanged: the call queues its transfers
    without a host wait (RCCL); the assembly reads the received offsets on the device."""

    def __init__(self, dist, rank: int, world: int, geometry: tuple[int, int] | None = None):
        self.dist, self.rank, self.world = dist, rank, world
        self.bufs: dict[int, tuple] = {}
        self.bounds = None
        self.last_bytes = 0
        if geometry is not None:
            total, bs = geometry
            nb = num_blocks(total, bs)
            self.bounds = [(len(shard_blocks(nb, r, world)), shard_payload_bound(total, bs, r, world)) for r in range(world)]

    def __call__(self, hdr, off, pay, crc):
        """hdr: uint8 [nb, 268]; off: int64 [nb + 1] (off[nb] = this rank's payload bytes); pay: uint8
        payload buffer; crc: int32 [1] CRC share.  Returns on rank 0 a list over ranks of
        (hdr, off, payload view, crc share); None elsewhere."""
        import torch

        dist, rank, world = self.dist, self.rank, self.world
        # gloo with device tensors (the one-GPU rehearsal of the N > 1 path): the exchange goes
        # through host copies; RCCL moves the device tensors themselves
        host = hdr.is_cuda and dist.get_backend() == "gloo"
        dev = hdr.device
        if self.bounds is not None:
            nbs = [b[0] for b in self.bounds]
            sizes = [b[1] for b in self.bounds]
            if hdr.shape[0] != nbs[rank] or pay.numel() < sizes[rank]:
                raise ValueError("ChunkGather: this rank's output does not match the geometry's shard")
            if host:
                hdr, off, pay, crc = hdr.cpu(), off.cpu(), pay[: sizes[rank]].cpu(), crc.cpu()
        else:
            if host:
                hdr, off, pay, crc = hdr.cpu(), off.cpu(), pay[: int(off[-1].item())].cpu(), crc.cpu()
            # (payload bytes, block count) of every rank in one small all_gather
            meta = torch.cat([off[-1:], torch.full((1,), hdr.shape[0], dtype=torch.int64, device=off.device)])
            metas = [torch.empty_like(meta) for _ in range(world)]
            dist.all_gather(metas, meta)
            metas = [m.tolist() for m in metas]  # (the host waits for every rank's encode here)
            sizes = [int(m[0]) for m in metas]
            nbs = [int(m[1]) for m in metas]
        ops = []
        if rank == 0:
            for r in range(1, world):
                b = self.bufs.get(r)
                if b is None or b[2].numel() < sizes[r] or b[0].shape[0] != nbs[r]:
                    b = (torch.empty((nbs[r], HEADER_BYTES), dtype=torch.uint8, device=hdr.device),
                         torch.empty((nbs[r] + 1,), dtype=torch.int64, device=hdr.device),
                         torch.empty((sizes[r] if self.bounds else int(sizes[r] * 1.1) + 4096,), dtype=torch.uint8, device=pay.device),
                         torch.empty((1,), dtype=torch.int32, device=hdr.device))
                    self.bufs[r] = b
                ops.append(dist.P2POp(dist.irecv, b[0], r))
                ops.append(dist.P2POp(dist.irecv, b[1], r))
                ops.append(dist.P2POp(dist.irecv, b[3], r))
                if sizes[r]:
                    ops.append(dist.P2POp(dist.irecv, b[2][: sizes[r]], r))
        else:
            ops.append(dist.P2POp(dist.isend, hdr, 0))
            ops.append(dist.P2POp(dist.isend, off, 0))
            ops.append(dist.P2POp(dist.isend, crc, 0))
            if sizes[rank]:
                ops.append(dist.P2POp(dist.isend, pay[: sizes[rank]], 0))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        # bytes that crossed to rank 0 in this call (headers, offsets, CRC shares, payloads)
        self.last_bytes = sum(nbs[r] * HEADER_BYTES + (nbs[r] + 1) * 8 + 4 + sizes[r] for r in range(1, world))
        if rank != 0:
            return None
        parts = [(hdr, off, pay[: sizes[0]], crc)]
        for r in range(1, world):
            b = self.bufs[r]
            parts.append((b[0], b[1], b[2][: sizes[r]], b[3]))
        if host:
            parts = [tuple(t.to(dev) for t in p) for p in parts]
        return parts


def merge_crc(parts) -> int:
    """CRC32C of the global chunk stream from the ranks' shares (XOR; see chunks_crc32c_shard)."""
    v = 0
    for p in parts:
        v ^= int(p[3].item()) & 0xFFFFFFFF
    return v


def merge_crc_device(parts):
    """merge_crc on the device: the XOR of the ranks' int32 shares, without a host round trip."""
    v = parts[0][3]
    for p in parts[1:]:
        v = v ^ p[3]
    return v


def assemble(codec, parts, round_robin: bool = True, stream=None):
    """Device assembly on rank 0: (headers [N, 268], offsets [N + 1], payload) in global block order.

    The assembly kernels run on `stream` (default: torch's current stream).  That is the stream the
    RCCL receives were made to wait on (`Work.wait()` in ChunkGather orders the current stream after
    the P2P kernels; it does not block the host), so the kernels read the peers' receive buffers
    only after they have arrived."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(parts[0][0].device)
    return codec.assemble_shards([(h, o, p) for h, o, p, _ in parts], round_robin=round_robin, stream=stream)


def assemble_host(parts, round_robin: bool = True):
    """Host restatement of the same interleave for CPU tensors (the gloo test checks the gather with it)."""
    import torch

    world = len(parts)
    nbs = [int(h.shape[0]) for h, _, _, _ in parts]
    nb = sum(nbs)
    order = []
    for g in range(nb):
        if round_robin:
            order.append((g % world, g // world))
        else:
            r, first = 0, 0
            while g >= first + nbs[r]:
                first += nbs[r]
                r += 1
            order.append((r, g - first))
    hdrs = torch.stack([parts[r][0][i] for r, i in order]) if nb else torch.empty((0, HEADER_BYTES), dtype=torch.uint8)
    pays = [parts[r][2][int(parts[r][1][i]): int(parts[r][1][i]) + int.from_bytes(parts[r][0][i, 264:268].numpy().tobytes(), "little")]
            for r, i in order]
    pay = torch.cat(pays) if pays else torch.empty((0,), dtype=torch.uint8)
    sizes = torch.tensor([p.numel() for p in pays], dtype=torch.int64)
    offs = torch.zeros(nb + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(sizes, 0)
    return hdrs, offs, pay
