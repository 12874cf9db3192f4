"""Full-size parity: EVERY block of the benchmark workloads against the reference encoder.

tests/golden/digests.json (made by tests/golden/make_digests.py from the reference's own
src/encoders, compiled here as oracle/_ref/libbraref.so) holds, per block, the primary index, the
encoded size and sha256(pi u32 LE || bra_huffman_t || payload) for:
  * text_1MiB_x256    BASELINE configs[1]: 256 x 1 MiB synthetic text (the bench workload);
  * random_1MiB_x256  BASELINE configs[2]: 256 MiB of uniform-random bytes in 1 MiB blocks;
  * sym16_8MiB_x32    BASELINE configs[4]: 8 MiB 16-symbol blocks, one GPU's share of 2 GiB / 8.
The GPU encodes the same bytes through the batch C-ABI (bra_gpu_encode_blocks) and every block's
digest must match: bit-exact at the sizes the benchmark measures, not only on samples.
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


@pytest.mark.parametrize("name", sorted(DIGESTS))
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
