"""Localisation helpers for the .BRa chunk-stream tests (test infrastructure, not product).

A chunk record on disk is 3-byte LE pi + packed bra_huffman_t (264 B) + payload
(lib_bra_io_file_chunks.c:76-95, 217-256).  These helpers split a device chunk stream into its
records, compare each record with the reference digests of tests/golden/digests.json, and -- when a
decoded chunk differs from its input -- name the first decode stage whose output differs from the
oracle's restatement of the reference for that chunk.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REC_HDR = 267


def load_digests() -> dict:
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        return json.load(f)


def split_records(stream: bytes):
    """[(pi, meta 264 B, payload)] of a chunk stream; raises on a truncated one."""
    recs, pos = [], 0
    while pos < len(stream):
        if pos + REC_HDR > len(stream):
            raise AssertionError(f"truncated record header at {pos}")
        pi = int.from_bytes(stream[pos: pos + 3], "little")
        meta = stream[pos + 3: pos + REC_HDR]
        esz = int.from_bytes(meta[260:264], "little")
        if pos + REC_HDR + esz > len(stream):
            raise AssertionError(f"truncated payload of record {len(recs)}")
        recs.append((pi, meta, stream[pos + REC_HDR: pos + REC_HDR + esz]))
        pos += REC_HDR + esz
    return recs


def record_digest(pi: int, meta: bytes, payload: bytes) -> str:
    """sha256(pi u32 LE || bra_huffman_t || payload): the digest make_digests.py stores."""
    return hashlib.sha256(pi.to_bytes(4, "little") + meta + payload).hexdigest()


def records_vs_reference(stream: bytes, w: dict):
    """Chunk indices whose record differs from the reference digests of workload w."""
    recs = split_records(stream)
    if len(recs) != w["nblocks"]:
        raise AssertionError(f"{len(recs)} records, reference has {w['nblocks']}")
    bad = []
    for b, (pi, meta, pay) in enumerate(recs):
        esz = int.from_bytes(meta[260:264], "little")
        if (pi, esz, record_digest(pi, meta, pay)) != (w["pi"][b], w["encoded_size"][b], w["sha256"][b]):
            bad.append(b)
    return bad


def headers_in_memory(stream: bytes) -> bytes:
    """The 268-byte in-memory headers of every record, back to back (the CRC input, :248-249)."""
    return b"".join(pi.to_bytes(4, "little") + meta for pi, meta, _ in split_records(stream))


def bad_chunks(out: np.ndarray, data: np.ndarray, bs: int):
    """Chunk indices where the decoded bytes differ from the input."""
    n = min(out.size, data.size)
    diff = np.flatnonzero(out[:n] != data[:n])
    ids = sorted(set((diff // bs).tolist()))
    if out.size != data.size:
        ids.append(-1)
    return ids


def decode_diagnosis(codec, orc, data: np.ndarray, b: int, bs: int, total: int) -> str:
    """First decode stage of chunk b (of the codec's last decode, chunks packed at b * bs) whose
    output differs from the oracle: RLE decode output (= MTF symbols), MTF decode output (= BWT
    last column), else the inverse BWT."""
    lo, hi = b * bs, min(total, (b + 1) * bs)
    blk = data[lo:hi].tobytes()
    ref_L, _ = orc.bwt_encode(blk)
    ref_M = orc.mtf_encode(ref_L)
    M = codec.stage_copy(1, total)[lo:hi]
    d = np.flatnonzero(M != np.frombuffer(ref_M, np.uint8))
    if d.size:
        return f"chunk {b}: Huffman/RLE decode output differs at {d.size} bytes (first {d[:4].tolist()})"
    L = codec.stage_copy(0, total)[lo:hi]
    d = np.flatnonzero(L != np.frombuffer(ref_L, np.uint8))
    if d.size:
        return f"chunk {b}: MTF decode output differs at {d.size} bytes (first {d[:4].tolist()})"
    return f"chunk {b}: Huffman, RLE and MTF decode ok; inverse BWT output differs"


def cyclic_sa(blk: np.ndarray) -> np.ndarray:
    """Sorted cyclic rotations of blk (ties by index, as the reference's stable qsort_r): prefix
    doubling over ranks with numpy (a 256 KiB block takes well under a second)."""
    n = blk.size
    rank = blk.astype(np.int64)
    sa = np.argsort(rank, kind="stable")
    k = 1
    while k < n:
        key2 = rank[(np.arange(n) + k) % n]
        sa = np.lexsort((np.arange(n), key2, rank))
        r1, r2 = rank[sa], key2[sa]
        head = np.empty(n, bool)
        head[0] = True
        head[1:] = (r1[1:] != r1[:-1]) | (r2[1:] != r2[:-1])
        new = np.empty(n, np.int64)
        new[sa] = np.cumsum(head) - 1
        rank = new
        if head.all():
            break
        k *= 2
    return sa


def _lcp(blk: np.ndarray, i: int, j: int, cap: int = 4096) -> int:
    n = blk.size
    for t in range(min(cap, n)):
        if blk[(i + t) % n] != blk[(j + t) % n]:
            return t
    return cap


def sa_diagnosis(codec, blk: np.ndarray, lo: int, total: int, save: str | None = None) -> str:
    """Where the device's suffix array of a block (stage 5, u32 per element at the block offset)
    departs from the reference order: whether it is still a permutation (a data-movement error
    loses or duplicates rotations; a sort error only misorders them), the span of the differing
    slots and the common-prefix depths there (which MSD level / job size the span belongs to)."""
    n = blk.size
    sa_dev = codec.stage_copy(5, 4 * total).view(np.uint32)[lo:lo + n].astype(np.int64)
    sa_ref = cyclic_sa(blk)
    d = np.flatnonzero(sa_dev != sa_ref)
    if not d.size:
        return "SA equal (L / pi written wrongly after the sort)"
    perm = np.array_equal(np.sort(sa_dev), np.arange(n))
    a, z = int(d[0]), int(d[-1])
    # the group of slots sharing the span's common prefix in the reference order: its size tells
    # the job class (<= 256 wave job, <= 1024 workgroup job) that sorted it
    dep = min(_lcp(blk, int(sa_ref[a]), int(sa_ref[z])), 4096)
    g0, g1 = a, z
    while g0 > 0 and _lcp(blk, int(sa_ref[g0 - 1]), int(sa_ref[a])) >= dep:
        g0 -= 1
    while g1 + 1 < n and _lcp(blk, int(sa_ref[g1 + 1]), int(sa_ref[a])) >= dep:
        g1 += 1
    inner = [_lcp(blk, int(sa_ref[i]), int(sa_ref[i + 1])) for i in range(a, min(z, a + 64))]
    msg = (f"SA {d.size} slots differ in [{a}, {z}] ({'permutation' if perm else 'NOT a permutation'}); "
           f"common prefix of the span {dep} bytes, group of that prefix [{g0}, {g1}] ({g1 - g0 + 1} slots); "
           f"adjacent lcps in span min {min(inner) if inner else -1} max {max(inner) if inner else -1}; "
           f"dev slots {sa_dev[a:a + 6].tolist()} ref {sa_ref[a:a + 6].tolist()}")
    save = save or (os.path.join(os.environ["BRA_DIAG_DIR"], f"sa_{lo}.npz") if os.environ.get("BRA_DIAG_DIR") else None)
    if save:
        np.savez_compressed(save, blk=blk, sa_dev=sa_dev, sa_ref=sa_ref)
    return msg


def encode_diagnosis(codec, orc, data: np.ndarray, b: int, bs: int, total: int, stream: bytes) -> str:
    """First encode stage of chunk b (of the codec's last encode, blocks at b * bs) whose output
    differs from the oracle: BWT last column and primary index, MTF of the device's own BWT output,
    then the record (RLE / Huffman)."""
    lo, hi = b * bs, min(total, (b + 1) * bs)
    blk = data[lo:hi].tobytes()
    ref_L, ref_pi = orc.bwt_encode(blk)
    recs = split_records(stream)
    pi = recs[b][0] if b < len(recs) else -1
    L = codec.stage_copy(0, total)[lo:hi]
    d = np.flatnonzero(L != np.frombuffer(ref_L, np.uint8))
    if d.size or pi != ref_pi:
        return (f"chunk {b}: BWT differs (L at {d.size} bytes, first {d[:4].tolist()}; pi {pi} vs {ref_pi}); "
                + sa_diagnosis(codec, data[lo:hi], lo, total))
    M = codec.stage_copy(1, total)[lo:hi]
    d = np.flatnonzero(M != np.frombuffer(orc.mtf_encode(L.tobytes()), np.uint8))
    if d.size:
        return f"chunk {b}: BWT ok; MTF differs at {d.size} bytes (first {d[:4].tolist()})"
    ref = orc.encode_block(blk)
    _, meta, pay = recs[b]
    return (f"chunk {b}: BWT and MTF ok; record differs: lengths {'ok' if meta[:256] == ref.lengths else 'differ'}, "
            f"sizes {int.from_bytes(meta[256:260], 'little'), int.from_bytes(meta[260:264], 'little')} vs {ref.orig_size, ref.encoded_size}, "
            f"payload {'ok' if pay == ref.payload else 'differs'}")
