"""Repeat full-size encodes in one process and compare every block with the reference digests
(tests/golden/digests.json): sym16 8 MiB shards and text 1 MiB batches, N rounds.  Prints one line
per round (mismatching global blocks), exits 1 on any mismatch.  GPU box diagnostic."""
import hashlib
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bra = importlib.import_module("br-archive_amd")
D = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))


def digest(hdr_row, payload):
    pi, lens, osz, esz = bra.parse_header(hdr_row.tobytes())
    h = hashlib.sha256()
    h.update(pi.to_bytes(4, "little") + lens + osz.to_bytes(4, "little") + esz.to_bytes(4, "little"))
    h.update(payload)
    return h.hexdigest()


def run(codec, name, rank, world):
    w = D[name]
    bs, nbg = w["block_size"], w["nblocks"]
    ids = list(range(rank, nbg, world))
    d = torch.from_numpy(bra.synth_fill(w["kind"], len(ids) * bs, bs, first_block=rank, stride=world)).cuda()
    hdr, off, pay = codec.encode(d, bs)
    torch.cuda.synchronize()
    H, O, P = hdr.cpu().numpy(), off.cpu().numpy(), pay.cpu().numpy()
    return [g for i, g in enumerate(ids) if digest(H[i], P[O[i]:O[i + 1]].tobytes()) != w["sha256"][g]]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    codec = bra.BlockCodec(0)
    bad_any = False
    for r in range(rounds):
        t0 = time.time()
        out = {}
        for name, rank, world in [("sym16_8MiB_x256", 7, 8), ("sym16_8MiB_x256", 3, 8), ("text_1MiB_x256", 0, 1), ("random_1MiB_x256", 0, 1)]:
            out[f"{name}/{rank}"] = run(codec, name, rank, world)
        bad = {k: v for k, v in out.items() if v}
        bad_any |= bool(bad)
        print(f"round {r}: {time.time() - t0:.1f} s, mismatches {bad if bad else 'none'}", flush=True)
    sys.exit(1 if bad_any else 0)


if __name__ == "__main__":
    main()
