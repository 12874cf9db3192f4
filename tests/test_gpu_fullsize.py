"""Full-size parity: EVERY block of the benchmark workloads against the reference encoder.

tests/golden/digests.json (made by tests/golden/make_digests.py from the reference's own
src/encoders, compiled here as oracle/_ref/libbraref.so) holds, per block, the primary index, the
encoded size and sha256(pi u32 LE || bra_huffman_t || payload) for:
  * text_1MiB_x256    BASELINE configs[1]: 256 x 1 MiB synthetic text (the bench workload);
  * random_1MiB_x256  BASELINE configs[2]: 256 MiB of uniform-random bytes in 1 MiB blocks;
  * sym16_8MiB_x32    BASELINE configs[4]: 8 MiB 16-symbol blocks, one GPU's share of 2 GiB / 8.
  * text_1MiB_x2048   BASELINE configs[3] at its FULL shape: 2048 x 1 MiB text blocks (2 GiB);
  * sym16_8MiB_x256   BASELINE configs[4] at its FULL shape: 256 x 8 MiB sym16 blocks (2 GiB).
The GPU encodes the same bytes through the batch C-ABI (bra_gpu_encode_blocks) and every block's
digest must match: bit-exact at the sizes the benchmark measures, not only on samples.  The two
8-GPU configurations are encoded the way bench.py shards them (rank r of 8 holds global blocks
r, r + 8, ...: 256 MiB per rank): the shards of ranks 0 and 7 are compared block by block, and all
8 shards are encoded on one device, assembled in global order (bra_gpu_assemble_shards) and checked
whole: every one of the 2048 / 256 blocks against the reference, the merged CRC shares against the
chunk-stream CRC32C of the assembled stream, and the decode of the assembled stream.
"""
import hashlib
import importlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))


@pytest.fixture(scope="module")
def bra():
    return importlib.import_module("br-archive_amd")


@pytest.fixture(scope="module")
def codec(bra):
    c = bra.BlockCodec(0)
    yield c
    c.close()


SINGLE = sorted(n for n, w in DIGESTS.items() if w["block_size"] * w["nblocks"] <= (256 << 20))
WORLD = 8
FULL = ["text_1MiB_x2048", "sym16_8MiB_x256"]


def _digest(bra, hdr_row, payload):
    pi, lens, osz, esz = bra.parse_header(hdr_row.tobytes())
    h = hashlib.sha256()
    h.update(pi.to_bytes(4, "little") + lens + osz.to_bytes(4, "little") + esz.to_bytes(4, "little"))
    h.update(payload)
    return pi, esz, h.hexdigest()


def _mismatches(bra, w, hdr, off, pay, global_ids):
    hdr_h, off_h, pay_h = hdr.cpu().numpy(), off.cpu().numpy(), pay.cpu().numpy()
    bad = []
    for i, g in enumerate(global_ids):
        esz = int.from_bytes(hdr_h[i, 264:268].tobytes(), "little")
        got = _digest(bra, hdr_h[i], pay_h[off_h[i]:off_h[i] + esz].tobytes())
        if got != (w["pi"][g], w["encoded_size"][g], w["sha256"][g]):
            bad.append(g)
    return bad


@pytest.mark.parametrize("name", SINGLE)
def test_every_block_matches_reference(bra, codec, name):
    import torch

    w = DIGESTS[name]
    bs, nb = w["block_size"], w["nblocks"]
    data = bra.synth_fill(w["kind"], bs * nb, bs, first_block=w["first_block"], stride=w["stride"])
    d = torch.from_numpy(data).cuda()
    hdr, off, pay = codec.encode(d, bs)
    torch.cuda.synchronize()
    hdr_h, off_h, pay_h = hdr.cpu().numpy(), off.cpu().numpy(), pay.cpu().numpy()
    bad = []
    for b in range(nb):
        pi, lens, osz, esz = bra.parse_header(hdr_h[b].tobytes())
        h = hashlib.sha256()
        h.update(pi.to_bytes(4, "little") + lens + osz.to_bytes(4, "little") + esz.to_bytes(4, "little"))
        h.update(pay_h[off_h[b]:off_h[b] + esz].tobytes())
        if (pi, esz, h.hexdigest()) != (w["pi"][b], w["encoded_size"][b], w["sha256"][b]):
            bad.append(b)
    assert not bad, f"{len(bad)} of {nb} blocks differ from the reference, first {bad[:8]}"
    # and the whole batch decodes back to the input
    out = codec.decode(hdr, off, pay, bs * nb, bs)
    assert torch.equal(out, d)


@pytest.mark.parametrize("rank", [0, WORLD - 1])
@pytest.mark.parametrize("name", FULL)
def test_round_robin_shard_matches_reference(bra, codec, name, rank):
    """One rank's shard of an 8-GPU configuration (bench.py's layout), every block vs the reference."""
    import torch

    w = DIGESTS[name]
    bs, nbg = w["block_size"], w["nblocks"]
    ids = list(range(rank, nbg, WORLD))
    data = bra.synth_fill(w["kind"], bs * len(ids), bs, first_block=rank, stride=WORLD)
    d = torch.from_numpy(data).cuda()
    hdr, off, pay = codec.encode(d, bs)
    torch.cuda.synchronize()
    bad = _mismatches(bra, w, hdr, off, pay, ids)
    assert not bad, f"{len(bad)} of {len(ids)} blocks of rank {rank} differ from the reference, first {bad[:8]}"


@pytest.mark.parametrize("name", FULL)
def test_eight_shards_assembled_match_reference(bra, codec, name):
    """All 8 shards of an 8-GPU configuration encoded on one device, their chunk records assembled
    in global block order and their CRC shares merged exactly as rank 0 does after the RCCL gather
    (br-archive_amd/dist.py): the 2 GiB global stream must be the reference's, block for block."""
    import torch

    dmod = __import__("importlib").import_module("br-archive_amd.dist")
    w = DIGESTS[name]
    bs, nbg = w["block_size"], w["nblocks"]
    total = bs * nbg
    parts, shards = [], []
    for r in range(WORLD):
        nb_r = len(dmod.shard_blocks(nbg, r, WORLD))
        d = torch.from_numpy(bra.synth_fill(w["kind"], nb_r * bs, bs, first_block=r, stride=WORLD)).cuda()
        hdr, off, pay = codec.encode(d, bs)
        crc = codec.chunks_crc32c_shard(d, hdr, bs, r, WORLD, total, r == 0)
        parts.append((hdr, off, pay[: int(off[nb_r].item())].clone(), crc))
        shards.append(d.view(nb_r, bs))
        del pay
    torch.cuda.synchronize()
    H, O, P = dmod.assemble(codec, parts, round_robin=True)
    torch.cuda.synchronize()
    bad = _mismatches(bra, w, H, O, P, list(range(nbg)))
    assert not bad, f"{len(bad)} of {nbg} assembled blocks differ from the reference, first {bad[:8]}"
    glob = torch.stack(shards, dim=1).reshape(-1)  # global block g = 8 i + r is block i of shard r
    assert dmod.merge_crc(parts) == codec.chunks_crc32c(glob, H, bs)
    out = codec.decode(H, O, P, total, bs)
    assert torch.equal(out, glob)
