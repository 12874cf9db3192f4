"""Single-block C-ABI BWT at sizes past the batched path's 2^24 block limit (csrc/bwt_large.hip):
round trips through bra_bwt_encode2 / bra_bwt_decode2, the oracle on a random 2^24 + 1 block, and
pi of a periodic block against its closed form."""
import importlib, sys, time
import numpy as np
sys.path.insert(0, ".")
bra = importlib.import_module("br-archive_amd")
from oracle import Oracle
orc = Oracle("oracle/liboracle.so")
ok_all = True
def check(name, x, oracle=False, pi_expect=None):
    global ok_all
    t = time.time()
    r = bra.bwt_encode(x)
    dt = time.time() - t
    if r is None:
        print(name, "encode failed", flush=True); ok_all = False; return
    L, pi = r
    rt = bra.bwt_decode(L, pi) == x
    line = f"{name} n={len(x)} encode {dt:.2f}s round_trip={rt}"
    ok = rt
    if pi_expect is not None:
        line += f" pi={pi} expect={pi_expect}"; ok &= pi == pi_expect
    if oracle:
        t = time.time(); RL, rpi = orc.bwt_encode(x)
        same = RL == L and rpi == pi
        line += f" oracle={same} ({time.time()-t:.1f}s)"; ok &= same
    print(line, flush=True)
    ok_all &= ok
n1 = (1 << 24) + 1
check("random", bra.synth_fill(1, n1, n1).tobytes(), oracle=True)
check("text", bra.synth_fill(0, 40 << 20, 40 << 20).tobytes())
check("sym16", bra.synth_fill(2, 40 << 20, 40 << 20).tobytes())
p = b"abracadabra"
k = (17 << 20) // len(p)
rots = [p[i:] + p[:i] for i in range(len(p))]
check("periodic", p * k, pi_expect=k * sum(r < p for r in rots))
check("zeros", bytes(1 << 24), pi_expect=0)
print("ALL OK" if ok_all else "FAILED", flush=True)
sys.exit(0 if ok_all else 1)
