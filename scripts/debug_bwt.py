"""Debug helper: GPU BWT (stage 0 + pi) of synthetic blocks vs the oracle, per kind / size."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import Oracle

bra = importlib.import_module("br-archive_amd")
orc = Oracle()
codec = bra.BlockCodec(0)
for kind, bs, nb in [(int(a.split(":")[0]), int(a.split(":")[1]), int(a.split(":")[2])) for a in sys.argv[1:]]:
    data = bra.synth_fill(kind, bs * nb, bs)
    d = torch.from_numpy(data).cuda()
    hdr, off, pay = codec.encode(d, bs)
    torch.cuda.synchronize()
    L = codec.stage_copy(0, bs * nb)
    hdr_h = hdr.cpu().numpy()
    for b in range(nb):
        blk = data[b * bs:(b + 1) * bs].tobytes()
        ref_L, ref_pi = orc.bwt_encode(blk)
        pi = bra.parse_header(hdr_h[b].tobytes())[0]
        got = L[b * bs:(b + 1) * bs].tobytes()
        nbad = int((np.frombuffer(got, np.uint8) != np.frombuffer(ref_L, np.uint8)).sum())
        print(f"kind {kind} bs {bs} block {b}: pi gpu {pi} ref {ref_pi} {'OK' if pi == ref_pi else 'BAD'}; L {'OK' if got == ref_L else f'BAD ({nbad} bytes)'}", flush=True)
