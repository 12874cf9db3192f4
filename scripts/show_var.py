"""Summarise gpu_var.sh results: value and the main kernel slots per variant."""
import json, os, sys
d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if not f.endswith(".json"):
        continue
    try:
        j = json.load(open(os.path.join(d, f)))
    except Exception as e:
        print(f, "unreadable", e); continue
    k = j.get("kernels", {})
    steps = j["steps"]
    top = sorted(((n, v["ms"] * v["launches"] / steps) for n, v in k.items() if not n.startswith("stage")), key=lambda x: -x[1])[:8]
    print(f"{f:14s} {j['value']:7.3f} GB/s ok={j['pipeline']['roundtrip_bit_exact']}  " + "  ".join(f"{n}={t:.2f}" for n, t in top))
