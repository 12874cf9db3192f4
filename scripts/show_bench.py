"""Print the headline and per-kernel timings of a bench.py --profile-all JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "GB/s  ms/step", d["ms_per_step"], "stages", d["pipeline"]["stage_ms"], "rt", d["pipeline"]["roundtrip_bit_exact"])
for k, v in d.get("kernels", {}).items():
    if not k.startswith("stage"):
        print(f"  {k:16s} {v['ms']:9.3f} ms x{v['launches'] // d['steps']:3d}/step  {v['GBps']:8.1f} GB/s")
