"""Per-kernel mean of every counter in rocprofv3 --pmc pass directories (measurement tooling).
usage: pmc_dump.py <dir> [kernel-substring ...]"""
import collections, csv, glob, os, re, sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = re.sub(r"bra::\(anonymous namespace\)::|\(anonymous namespace\)::|^void ", "", r["Kernel_Name"]).split("(")[0].strip()
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
pats = sys.argv[2:]
for k in sorted(agg):
    if pats and not any(p in k for p in pats):
        continue
    c = agg[k]
    print(k)
    for n in sorted(c):
        v = c[n]
        print(f"    {n:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
