"""Per-kernel instruction counts from a gpu_pmc_var.sh pass (measurement tooling).
usage: pmc_insts.py <dir> [kernel substring ...]"""
import collections, csv, glob, sys
d = sys.argv[1]
want = sys.argv[2:] or ["k_jobs", "k_mjobs"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if any(w in n for w in want):
            k = n.replace("void bra::(anonymous namespace)::", "").replace("bra::(anonymous namespace)::", "").split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if any(w in n for w in want):
            k = n.replace("void bra::(anonymous namespace)::", "").replace("bra::(anonymous namespace)::", "").split("(")[0]
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, c in agg.items():
    t = dur.get(k, 0.0)
    util = c["SQ_INSTS_VALU"] * 4 / (t / 1e3 * 2.4e9 * 1024) if t else 0
    print(f"{k:28s} ms {t:8.3f} valu {c['SQ_INSTS_VALU'] / 1e6:9.1f}M salu {c['SQ_INSTS_SALU'] / 1e6:8.1f}M lds {c['SQ_INSTS_LDS'] / 1e6:7.1f}M "
          f"vmem {c['SQ_INSTS_VMEM_RD'] / 1e6:7.1f}M smem {c['SQ_INSTS_SMEM'] / 1e6:6.1f}M waves {c['SQ_WAVES']:.0f} valu_util {util:.2f}")
