"""The .BRa chunk stream on CPU: CRC32C, combine, chunk framing.

1. The CRC32C restatement (oracle/bra_oracle.c) against the known answers of the reference's own
   test/test_bra_crc32c.cpp (hard-coded here) and, when oracle/_ref/libbralib.so is present,
   against the reference's bra_crc32c / bra_crc32c_combine on seeded random cases.
2. The oracle's chunk loop (framing + running CRC + entry CRC) against tests/golden/chunks.json,
   which holds what the reference's bra_io_file_chunks_compress_file produced on the same inputs
   (tests/golden/make_chunks_golden.py).
3. The product library's host-side CRC helpers (bra_gpu_crc32c_combine, bra_gpu_entry_crc32c)
   against the oracle -- host arithmetic only, no GPU call.
"""
import hashlib
import importlib
import json
import os
import random

import numpy as np
import pytest

from oracle import ReferenceLib, have_reflib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNKS = os.path.join(ROOT, "tests", "golden", "chunks.json")
CS = 256 * 1024


def _synth(kind, total):
    bra = importlib.import_module("br-archive_amd")
    return bra.synth_fill(kind, total, CS).tobytes()


def _case_input(g) -> bytes:
    """Input bytes of a chunks.json case (the rule of tests/golden/make_chunks_golden.py)."""
    if "file" in g:
        with open(os.path.join(os.path.dirname(CHUNKS), g["file"]), "rb") as f:
            return f.read()
    if "parts" in g:
        bra = importlib.import_module("br-archive_amd")
        return b"".join(bra.synth_fill(k, n, CS, first_block=fb).tobytes() for k, n, fb in g["parts"])
    return _synth(g["kind"], g["total"])


# ---- 1. CRC32C known answers (test/test_bra_crc32c.cpp:19-132) ------------------------------------
def test_crc32c_kat(orc):
    d1, d2 = b"123456789", b"Hello World!"
    assert orc.crc32c(d1) == 0xE3069283
    assert orc.crc32c(d1[5:], orc.crc32c(d1[:5])) == 0xE3069283
    assert orc.crc32c(b"") == 0
    assert orc.crc32c(d2) == 0xFE6CF1DC
    assert orc.crc32c_combine(orc.crc32c(d2[:6]), orc.crc32c(d2[6:]), 6) == orc.crc32c(d2)
    buf = bytes((i * 7 + 3) & 0xFF for i in range(1000))
    for split in (0, 1, 333, 999, 1000):
        c = orc.crc32c_combine(orc.crc32c(buf[:split]), orc.crc32c(buf[split:]), 1000 - split)
        assert c == orc.crc32c(buf), split


@pytest.mark.skipif(not have_reflib(), reason="reference lib_bra build (oracle/_ref/libbralib.so) not present")
def test_crc32c_vs_reference(orc):
    R = ReferenceLib()
    rng = random.Random(11)
    for _ in range(200):
        n = rng.choice([0, 1, 7, 8, 15, 16, 17, 255, 4096, rng.randrange(20000)])
        data = bytes(rng.getrandbits(8) for _ in range(n))
        prev = rng.getrandbits(32)
        assert orc.crc32c(data, prev) == R.crc32c(data, prev)
        a, b, lb = rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(32)
        assert orc.crc32c_combine(a, b, lb) == R.crc32c_combine(a, b, lb)


# ---- 2. the chunk loop vs the reference's output ---------------------------------------------------
def _golden():
    with open(CHUNKS) as f:
        return json.load(f)


@pytest.mark.parametrize("name", sorted(_golden()))
def test_oracle_chunk_loop_vs_golden(orc, name):
    g = _golden()[name]
    data = _case_input(g)
    assert len(data) == g["total"]
    stream, crc, chunks = orc.compress_chunks(data, CS)
    compressed = len(stream) < len(data)
    assert compressed == g["compressed"]
    if not compressed:
        return
    assert len(stream) == g["stream_size"]
    assert hashlib.sha256(stream).hexdigest() == g["stream_sha256"]
    assert orc.entry_crc32c(g["entry_crc_before"], len(stream), crc, len(data)) == g["entry_crc"]
    # per-chunk CRC of header + data, and the running fold of them
    running = 0
    for b, ch in enumerate(chunks):
        hdr = ch.primary_index.to_bytes(4, "little") + ch.lengths + ch.orig_size.to_bytes(4, "little") + ch.encoded_size.to_bytes(4, "little")
        part = data[b * CS: (b + 1) * CS]
        assert orc.crc32c(part, orc.crc32c(hdr)) == g["chunk_crcs"][b], b
        running = orc.crc32c_combine(running, g["chunk_crcs"][b], 268 + len(part))
    assert running == crc
    assert [ch.encoded_size for ch in chunks] == g["encoded_sizes"]
    if not g["ref_decodes"]:
        # the reference writes this stream but its decoder rejects it, because
        # one chunk's Huffman payload exceeds BRA_MAX_CHUNK_SIZE (lib_bra_io_file_chunks.c:36-40)
        assert max(g["encoded_sizes"]) > CS
    else:
        assert g["ref_decode_crc"] == crc


@pytest.mark.skipif(not have_reflib(), reason="reference lib_bra build (oracle/_ref/libbralib.so) not present")
def test_oracle_chunk_loop_vs_reference_run(orc, tmp_path):
    """Fresh inputs through the reference's compress loop and the oracle (ragged tails)."""
    R = ReferenceLib()
    for kind, total in ((0, 3 * CS + 17), (2, CS - 1), (0, 1000)):
        data = _synth(kind, total)
        ok, dst, cb, ca, _ = R.compress_file(data, str(tmp_path))
        stream, crc, _ = orc.compress_chunks(data, CS)
        assert ok == (len(stream) < len(data))
        if ok:
            assert dst[8:] == stream and int.from_bytes(dst[:8], "little") == len(stream)
            assert orc.entry_crc32c(cb, len(stream), crc, len(data)) == ca


# ---- 3. product host helpers (no GPU) -------------------------------------------------------------
def test_product_host_crc_helpers(orc):
    bra = importlib.import_module("br-archive_amd")
    rng = random.Random(5)
    for _ in range(300):
        a, b, lb = rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(32)
        assert bra.crc32c_combine(a, b, lb) == orc.crc32c_combine(a, b, lb)
    # 64-bit lengths: shifting by 2^32 + k equals two 2^31 shifts then k
    for _ in range(20):
        a, b, k = rng.getrandbits(32), rng.getrandbits(32), rng.randrange(1, 1 << 20)
        step = orc.crc32c_combine(orc.crc32c_combine(a, 0, 1 << 31), 0, 1 << 31)
        assert bra.crc32c_combine(a, b, (1 << 32) + k) == orc.crc32c_combine(step, b, k)
    for g in _golden().values():
        if g["compressed"]:
            me, tsz, data_size = g["entry_crc_before"], g["stream_size"], g["total"]
            crc = rng.getrandbits(32)
            assert bra.entry_crc32c(me, tsz, crc, data_size) == orc.entry_crc32c(me, tsz, crc, data_size)
    # sizes above 4 GiB keep the reference's 32-bit combine length
    assert bra.entry_crc32c(1, 1 << 33, 2, (5 << 32) + 3) == orc.entry_crc32c(1, 1 << 33, 2, (5 << 32) + 3)
