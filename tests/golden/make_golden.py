"""Generate tests/golden/golden.npz from the REFERENCE encoders.

Run in the build container (where /root/reference exists):
    make -C oracle && python tests/golden/make_golden.py

Every expected value is produced by oracle/_ref/libbraref.so, i.e. the reference's own
src/encoders compiled in place by oracle/Makefile.  Inputs are
  * the known-answer strings of the reference's test/test_bra_encoders.cpp,
  * blocks from br-archive_amd/csrc/bra_synth.c (text / random / sym16 / tiled, several sizes,
    ragged and power-of-two), periodic and run-heavy edge cases,
  * config 1 of BASELINE.json: test/test.txt tiled to 65,536 bytes (the reference needs ~50 s
    for its BWT; pass --skip-cfg1 to leave that case out).
The archive holds only data (uint8/uint32 arrays): it loads with numpy.load(allow_pickle=False).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import Reference, have_ref  # noqa: E402


def synth_lib():
    so = "/tmp/bra_synth_golden.so"
    src = os.path.join(ROOT, "br-archive_amd", "csrc", "bra_synth.c")
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", so, src, "-lm"])
    lib = C.CDLL(so)
    lib.bra_synth_block.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_uint64]
    return lib


def synth(lib, kind: int, idx: int, n: int) -> bytes:
    b = (C.c_uint8 * n)()
    lib.bra_synth_block(kind, idx, b, n)
    return bytes(b)


def cases(lib, skip_cfg1: bool):
    yield "kat_banana", b"BANANA"
    yield "kat_fox", b"The quick brown fox jumps over the lazy dog."
    yield "kat_aaaaa", b"AAAAA"
    yield "kat_rle2", b"AAAAABBBCD"
    yield "kat_rle3", b"ABCDEFGH"
    yield "kat_rle1", b"A" * 10
    yield "one_byte", b"\x07"
    yield "two_same", b"zz"
    yield "abab", b"abab"
    yield "baba", b"baba"
    yield "zeros_4096", b"\0" * 4096
    yield "ff_300", b"\xff" * 300
    yield "period3_999", b"xyz" * 333
    yield "period7_ragged", (b"abcabca" * 100)[:697]
    runs = b"".join(bytes([i % 5]) * L for i, L in enumerate([1, 2, 3, 127, 128, 129, 130, 131, 255, 256, 257, 258, 2, 1, 300]))
    yield "runs_mixed", runs
    for kind, name in ((0, "text"), (1, "random"), (2, "sym16"), (3, "tiled")):
        for n in (1, 2, 3, 7, 64, 255, 256, 257, 1000, 4096, 65535):
            if kind == 3 and n > 4096:
                continue
            yield f"{name}_{n}", synth(lib, kind, 7 + n, n)
    yield "text_65536", synth(lib, 0, 1, 65536)
    yield "random_65536", synth(lib, 1, 1, 65536)
    if not skip_cfg1:
        yield "cfg1_tiled_65536", synth(lib, 3, 0, 65536)


def main():
    if not have_ref():
        sys.exit("oracle/_ref/libbraref.so missing: run `make -C oracle ref` with /root/reference present")
    skip = "--skip-cfg1" in sys.argv
    R = Reference()
    lib = synth_lib()
    arrays = {}
    names = []
    for name, data in cases(lib, skip):
        t = time.time()
        ch = R.encode_block(data)
        dec = R.decode_block(ch)
        assert dec == data, name
        arrays[f"{name}/input"] = np.frombuffer(data, np.uint8)
        arrays[f"{name}/bwt"] = np.frombuffer(ch.bwt, np.uint8)
        arrays[f"{name}/mtf"] = np.frombuffer(ch.mtf, np.uint8)
        arrays[f"{name}/rle"] = np.frombuffer(ch.rle, np.uint8)
        arrays[f"{name}/lengths"] = np.frombuffer(ch.lengths, np.uint8)
        arrays[f"{name}/payload"] = np.frombuffer(ch.payload, np.uint8)
        arrays[f"{name}/scalars"] = np.array([ch.primary_index, ch.orig_size, ch.encoded_size], np.uint32)
        names.append(name)
        print(f"{name:24s} n={len(data):6d} pi={ch.primary_index:6d} rle={len(ch.rle):6d} "
              f"payload={ch.encoded_size:6d}  ({time.time() - t:.2f}s)", flush=True)
    arrays["names"] = np.array(names)
    out = os.path.join(ROOT, "tests", "golden", "golden.npz")
    np.savez_compressed(out, **arrays)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
