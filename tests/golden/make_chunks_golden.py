"""Generate tests/golden/chunks.json from the REFERENCE chunk loop (rows f1/f2).

Run in the build container (where /root/reference exists):
    make -C oracle ref && python tests/golden/make_chunks_golden.py

For every case the input is a deterministic synthetic buffer (br-archive_amd/csrc/bra_synth.c,
bra_synth_fill(kind, 0, ..., total, 262144)), and the expected values come from
oracle/_ref/libbralib.so, i.e. the reference's own bra_io_file_chunks_compress_file
(src/io/lib_bra_io_file_chunks.c:169-312) run on a real file by oracle/ref_chunks.c:
  * compressed   -- the call succeeded (False: the reference switched the entry to STORED);
  * stream_size / stream_sha256 -- the chunk records the reference writes after the 8-byte
    data_size of the meta entry (what bra_gpu_compress_chunks must produce byte for byte);
  * entry_crc    -- me->crc32 after the call (lib_bra_io_file_chunks.c:291-292), from a fresh
    entry whose CRC is BRA_CRC32C_INIT;
  * chunk_crcs   -- the CRC32C of every 268-byte in-memory header + chunk (parsed back from the
    stream with the reference's bra_crc32c, so the fixture also pins the header layout).
The fixture stores digests and CRCs only (JSON data, no code).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ReferenceLib, have_reflib  # noqa: E402

CASES = [  # (name, synth kind, total bytes)
    ("text_600000", 0, 600000),
    ("text_262144", 0, 262144),
    ("text_262145", 0, 262145),
    ("sym16_524288", 2, 524288),
    ("random_100000", 1, 100000),
]
# Inputs made of parts [synth kind, bytes, first synthetic block] or the reference's own fixture file:
#   mixed_text_random -- SURVEY 0.5 / row f4: compressible text chunks around ONE uniform-random
#                        256 KiB chunk.  The reference still archives the file compressed (the
#                        tmpfile is smaller than the input), but the random chunk's Huffman payload
#                        exceeds BRA_MAX_CHUNK_SIZE, so its own decoder rejects the stream
#                        (lib_bra_io_file_chunks.c:36-40): `ref_decodes` is false.
#   lorem_txt         -- test/fixtures/lorem.txt (3039 B, the input of test_bra_unbra_comp_2,
#                        test/test_bra.cpp:353-398), committed as tests/golden/lorem.txt.
PART_CASES = [
    ("mixed_text_random", {"parts": [[0, 2 * 262144, 0], [1, 262144, 0], [0, 100000, 3]]}),
    ("lorem_txt", {"file": "lorem.txt"}),
]
# Decode-only cases: a case's reference stream with one chunk header patched.  The reference's loop
# writes every chunk before the bad one, then fails (lib_bra_io_file_chunks.c:340-411); the fixture
# pins that prefix (`ref_decode_prefix_size` / `_sha256`) and the verdict.
#   text_600000_bad_pi -- chunk 2 (75712 B) gets primary index 100000: the header is valid
#                         (pi < BRA_MAX_CHUNK_SIZE) but pi >= the decoded size (:385-389).
# (written to tests/golden/chunks_decode.json)
DECODE_CASES = [
    ("text_600000_bad_pi", {"base": "text_600000", "patch_chunk": 2, "patch_pi": 100000}),
]


def patch_stream(stream: bytes, chunk: int, pi: int) -> bytes:
    """The chunk stream with record `chunk`'s 3-byte primary index set to pi."""
    pos = 0
    for _ in range(chunk):
        pos += 267 + int.from_bytes(stream[pos + 263: pos + 267], "little")
    return stream[:pos] + pi.to_bytes(3, "little") + stream[pos + 3:]


def synth(kind: int, total: int) -> bytes:
    import numpy as np

    bra = __import__("importlib").import_module("br-archive_amd")
    a = np.empty(total, dtype=np.uint8)
    bra.synth_lib().bra_synth_fill(kind, 0, a.ctypes.data, total, 262144)
    return a.tobytes()


def case_input(rec: dict) -> bytes:
    """The input bytes of a chunks.json case (same rule as tests/test_gpu_chunks.py)."""
    import numpy as np

    if "file" in rec:
        return open(os.path.join(ROOT, "tests", "golden", rec["file"]), "rb").read()
    if "parts" in rec:
        bra = __import__("importlib").import_module("br-archive_amd")
        return np.concatenate([bra.synth_fill(k, n, 262144, first_block=fb) for k, n, fb in rec["parts"]]).tobytes()
    return synth(rec["kind"], rec["total"])


def main():
    if not have_reflib():
        sys.exit("oracle/_ref/libbralib.so missing: run `make -C oracle ref` where /root/reference exists")
    lorem = os.path.join(ROOT, "tests", "golden", "lorem.txt")
    if not os.path.exists(lorem):  # the reference's own fixture file, kept as test data
        with open("/root/reference/test/fixtures/lorem.txt", "rb") as f, open(lorem, "wb") as g:
            g.write(f.read())
    R = ReferenceLib()
    out = {}
    cases = [(name, {"kind": kind, "total": total}) for name, kind, total in CASES] + PART_CASES
    for name, spec in cases:
        data = case_input(spec)
        with tempfile.TemporaryDirectory() as d:
            ok, dst, cb, ca, attr = R.compress_file(data, d)
        rec = dict(spec, total=len(data), compressed=ok, attr=attr, entry_crc_before=cb, entry_crc=ca)
        if ok:
            tsz = int.from_bytes(dst[:8], "little")
            stream = dst[8:]
            assert len(stream) == tsz, (name, len(stream), tsz)
            crcs, pos, b = [], 0, 0
            while pos < len(stream):
                esz = int.from_bytes(stream[pos + 263: pos + 267], "little")
                hdr = stream[pos: pos + 3] + b"\0" + stream[pos + 3: pos + 267]
                chunk = data[b * 262144: (b + 1) * 262144]
                crcs.append(R.crc32c(chunk, R.crc32c(hdr)))
                pos += 267 + esz
                b += 1
            with tempfile.TemporaryDirectory() as d:
                dok, dec, dcrc = R.decompress_file(stream, d)
            esizes = []
            pos = 0
            while pos < len(stream):
                esizes.append(int.from_bytes(stream[pos + 263: pos + 267], "little"))
                pos += 267 + esizes[-1]
            rec.update(stream_size=tsz, stream_sha256=hashlib.sha256(stream).hexdigest(), chunk_crcs=crcs, encoded_sizes=esizes,
                       ref_decodes=dok and dec == data, ref_decode_crc=dcrc if dok else None)
            if not dok:
                rec.update(ref_decode_prefix_size=len(dec), ref_decode_prefix_sha256=hashlib.sha256(dec).hexdigest())
        out[name] = rec
        print(name, {k: v for k, v in rec.items() if k != "chunk_crcs"}, flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "chunks.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    dec_out = {}
    for name, spec in DECODE_CASES:
        base = dict(cases)[spec["base"]]
        data = case_input(base)
        with tempfile.TemporaryDirectory() as d:
            ok, dst, _, _, _ = R.compress_file(data, d)
        assert ok, name
        stream = patch_stream(dst[8:], spec["patch_chunk"], spec["patch_pi"])
        with tempfile.TemporaryDirectory() as d:
            dok, dec, dcrc = R.decompress_file(stream, d)
        rec = dict(spec, stream_sha256=hashlib.sha256(stream).hexdigest(), ref_decodes=bool(dok and dec == data),
                   ref_decode_crc=dcrc if dok else None, ref_decode_prefix_size=len(dec), ref_decode_prefix_sha256=hashlib.sha256(dec).hexdigest())
        dec_out[name] = rec
        print(name, rec, flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "chunks_decode.json"), "w") as f:
        json.dump(dec_out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
