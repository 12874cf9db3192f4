"""Drive a lib_bra build's chunk loop on the GPU box (helper of tests/test_gpu_frontend.py).

    python tests/frontend_driver.py <lib.so> <out.json>

<lib.so> is oracle/_ref/libbralib_hipenc.so (the reference lib_bra with its own chunk loop, its
encoders replaced by libbra_hip.so) or oracle/_ref/libbralib_gpu.so (lib_bra with the batched front
end br-archive_amd/frontend/bra_io_file_chunks_gpu.c).  For every case of tests/golden/chunks.json
it runs bra_io_file_chunks_compress_file and bra_io_file_chunks_decompress_file through that
library (oracle/ref_chunks.c) and writes one JSON object to <out.json> (lib_bra prints its progress
on stdout): per case the stream digest, the entry
CRCs, whether the decode succeeded and gave the input back, and the decode CRC.  Runs in its own
process so that the two lib_bra builds never share a symbol scope.
"""
import hashlib
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import ReferenceLib  # noqa: E402
from test_chunks import _case_input  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_chunks_golden import patch_stream  # noqa: E402


def main():
    lib = ReferenceLib(sys.argv[1])
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "chunks.json")))
    out = {}
    for name, g in sorted(golden.items()):
        data = _case_input(g)
        with tempfile.TemporaryDirectory() as d:
            ok, dst, cb, ca, attr = lib.compress_file(data, d)
        rec = {"compressed": ok, "attr": attr, "entry_crc_before": cb, "entry_crc": ca}
        if ok:
            stream = dst[8:]
            rec.update(stream_size=int.from_bytes(dst[:8], "little"), stream_sha256=hashlib.sha256(stream).hexdigest())
            with tempfile.TemporaryDirectory() as d:
                dok, dec, dcrc = lib.decompress_file(stream, d)
            rec.update(decodes=bool(dok and dec == data), decode_crc=dcrc if dok else None)
            if not dok:
                rec.update(decode_prefix_size=len(dec), decode_prefix_sha256=hashlib.sha256(dec).hexdigest())
        out[name] = rec
    # decode-only cases: a patched stream; the decoder must fail after writing the same prefix
    for name, spec in sorted(json.load(open(os.path.join(ROOT, "tests", "golden", "chunks_decode.json"))).items()):
        data = _case_input(golden[spec["base"]])
        with tempfile.TemporaryDirectory() as d:
            ok, dst, _, _, _ = lib.compress_file(data, d)
        stream = patch_stream(dst[8:], spec["patch_chunk"], spec["patch_pi"])
        with tempfile.TemporaryDirectory() as d:
            dok, dec, dcrc = lib.decompress_file(stream, d)
        out[name] = {"stream_sha256": hashlib.sha256(stream).hexdigest(), "decodes": bool(dok and dec == data),
                     "decode_crc": dcrc if dok else None, "decode_prefix_size": len(dec), "decode_prefix_sha256": hashlib.sha256(dec).hexdigest()}
    with open(sys.argv[2], "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
