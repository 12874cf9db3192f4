"""lib_bra itself on the GPU encoders (SURVEY 8.1 rows b and f1): the reference front end links
against libbra_hip.so and produces the reference's bytes.

Two builds made by oracle/Makefile (target gpulib) from the reference's own lib_bra sources:
  * libbralib_hipenc.so -- lib_bra WITHOUT src/encoders/*.c, its own chunk loop
    (lib_bra_io_file_chunks.c) unchanged: every chunk goes through the 14 drop-in entry points of
    libbra_hip.so;
  * libbralib_gpu.so    -- lib_bra without src/encoders/*.c and without lib_bra_io_file_chunks.c,
    plus the batched front end br-archive_amd/frontend/bra_io_file_chunks_gpu.c (one device call
    per 256 chunks);
  * libbralib_gpu_b2.so -- the same front end built with BATCH_CHUNKS=2, so every multi-chunk
    case spans several batches (the CRC combine across batches, decode batches that end at the
    batch limit, the serial error path after a failed batch).
Both must reproduce tests/golden/chunks.json (the reference lib_bra's own tmpfile bytes, entry
CRCs, STORED decisions, decoder verdicts and decode CRCs) exactly.  Each build runs in its own
process (tests/frontend_driver.py).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "chunks.json")))
DECODE = json.load(open(os.path.join(ROOT, "tests", "golden", "chunks_decode.json")))


@pytest.mark.parametrize("lib", ["libbralib_hipenc.so", "libbralib_gpu.so", "libbralib_gpu_b2.so"])
def test_lib_bra_chunk_loop_on_gpu(lib, tmp_path):
    path = os.path.join(ROOT, "oracle", "_ref", lib)
    assert os.path.exists(path), f"{lib} not built (make -C oracle gpulib where the reference tree exists)"
    res = tmp_path / "result.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "frontend_driver.py"), path, str(res)], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(res.read_text())
    for name, g in GOLDEN.items():
        o = got[name]
        assert o["compressed"] == g["compressed"] and o["attr"] == g["attr"], name
        assert (o["entry_crc_before"], o["entry_crc"]) == (g["entry_crc_before"], g["entry_crc"]), name
        if not g["compressed"]:
            continue
        assert (o["stream_size"], o["stream_sha256"]) == (g["stream_size"], g["stream_sha256"]), name
        assert o["decodes"] == g["ref_decodes"], name
        if g["ref_decodes"]:
            assert o["decode_crc"] == g["ref_decode_crc"], name
        else:  # the reference wrote every chunk before the bad record: so must the drop-in
            assert (o["decode_prefix_size"], o["decode_prefix_sha256"]) == (g["ref_decode_prefix_size"], g["ref_decode_prefix_sha256"]), name
    for name, g in DECODE.items():
        o = got[name]
        assert o["stream_sha256"] == g["stream_sha256"], name
        assert o["decodes"] == g["ref_decodes"], name
        assert (o["decode_prefix_size"], o["decode_prefix_sha256"]) == (g["ref_decode_prefix_size"], g["ref_decode_prefix_sha256"]), name
