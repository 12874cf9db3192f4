"""Generate tests/golden/digests.json: per-block digests of the REFERENCE encoder at the benchmark sizes.

Run in the build container (where /root/reference exists):
    make -C oracle ref && python tests/golden/make_digests.py
    ONLY=text_1MiB_x2048,sym16_8MiB_x256 python tests/golden/make_digests.py   # some workloads only

For each BASELINE workload below, every block of the deterministic synthetic input
(br-archive_amd/csrc/bra_synth.c, the same bytes bench.py encodes on one GPU) goes through the
reference's own src/encoders (oracle/_ref/libbraref.so: bra_bwt_encode2 -> bra_mtf_encode2 ->
bra_rle_encode -> bra_huffman_encode, the chain of lib_bra_io_file_chunks.c:217-245), and the
fixture stores sha256(pi as u32 LE || bra_huffman_t (264 B) || payload) per block, plus the
per-block pi and encoded_size in the clear.  The GPU test (tests/test_gpu_fullsize.py) compares
EVERY block of the same workload against it.  Data only (JSON digests), no code.
"""
from __future__ import annotations

import hashlib
import importlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import Reference, have_ref  # noqa: E402

# name -> (synth kind, block size, blocks): BASELINE configs[1] (text), configs[2] (random) at the
# 256 MiB single-GPU size, configs[4] (sym16 8 MiB blocks) at its per-GPU share of 2 GiB / 8, and
# the two 8-GPU configurations at their FULL global shape: configs[3] = 2048 x 1 MiB text blocks
# (2 GiB; rank r of 8 encodes blocks r, r + 8, ...) and configs[4] = 256 x 8 MiB sym16 blocks.
WORKLOADS = {
    "text_1MiB_x256": (0, 1 << 20, 256),
    "random_1MiB_x256": (1, 1 << 20, 256),
    "sym16_8MiB_x32": (2, 8 << 20, 32),
    "text_1MiB_x2048": (0, 1 << 20, 2048),
    "sym16_8MiB_x256": (2, 8 << 20, 256),
    # the .BRa geometry: bra -c always encodes 256 KiB chunks (lib_bra_io_file_chunks.c:199-201,
    # BRA_MAX_CHUNK_SIZE, lib_bra_defs.h:93) -- 1024 chunks = the 256 MiB chunk stream of
    # tests/test_gpu_chunks.py::test_full_size_chunk_stream
    "text_256KiB_x1024": (0, 256 << 10, 1024),
    "random_256KiB_x1024": (1, 256 << 10, 1024),
    "sym16_256KiB_x1024": (2, 256 << 10, 1024),
}


def digest(pi: int, lens: bytes, osz: int, esz: int, payload: bytes) -> str:
    h = hashlib.sha256()
    h.update(pi.to_bytes(4, "little") + lens + osz.to_bytes(4, "little") + esz.to_bytes(4, "little") + payload)
    return h.hexdigest()


def main():
    if not have_ref():
        sys.exit("oracle/_ref/libbraref.so missing: run `make -C oracle ref` where /root/reference exists")
    bra = importlib.import_module("br-archive_amd")
    ref = Reference()
    path = os.path.join(ROOT, "tests", "golden", "digests.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    only = [w for w in os.environ.get("ONLY", "").split(",") if w]
    threads = int(os.environ.get("THREADS", os.cpu_count() or 8))
    for name, (kind, bs, nb) in WORKLOADS.items():
        if only and name not in only:
            continue
        t0 = time.time()

        def one(b):
            # one block at a time (a 2 GiB workload is never held whole)
            ch = ref.encode_block(bra.synth_fill(kind, bs, bs, first_block=b).tobytes())
            return ch.primary_index, ch.encoded_size, digest(ch.primary_index, ch.lengths, ch.orig_size, ch.encoded_size, ch.payload)

        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(one, range(nb)))
        out[name] = {
            "kind": kind, "block_size": bs, "nblocks": nb, "first_block": 0, "stride": 1,
            "pi": [r[0] for r in res], "encoded_size": [r[1] for r in res], "sha256": [r[2] for r in res],
        }
        print(f"{name}: {nb} blocks in {time.time() - t0:.1f} s", flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
