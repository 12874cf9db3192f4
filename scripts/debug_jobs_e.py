"""Debug helper: BWT of the runs_mixed golden input with the single-wave jobs switched per class."""
import importlib, os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if len(sys.argv) == 1:
    for v in ("0", "1", "2", "3"):
        r = subprocess.run([sys.executable, __file__, v], env=dict(os.environ, BRA_JOBS_E=v), capture_output=True, text=True)
        print("BRA_JOBS_E", v, r.stdout.strip(), r.stderr.strip()[-300:])
    sys.exit(0)
import numpy as np
bra = importlib.import_module("br-archive_amd")
from oracle import Oracle
orc = Oracle()
runs = b"".join(bytes([i % 5]) * L for i, L in enumerate([1, 2, 3, 127, 128, 129, 130, 131, 255, 256, 257, 258, 2, 1, 300]))
cases = {"runs_mixed": runs}
rng = np.random.default_rng(5)
cases["runs_rand"] = bytes(np.repeat(rng.integers(0, 4, 400, dtype=np.uint8), rng.integers(1, 40, 400)).tolist())
cases["text_64k"] = bra.synth_block(0, 3, 65536)
for name, x in cases.items():
    L, pi = bra.bwt_encode(x)
    L2, pi2 = orc.bwt_encode(x)
    bad = [i for i in range(len(x)) if L[i] != L2[i]]
    print(name, len(x), "pi", pi, pi2, "Lbad", len(bad), bad[:5])
