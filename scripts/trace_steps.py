"""Print the dispatch sequence of the last encode step from a rocprofv3 kernel-trace csv:
kernel, duration (us), gap before it (us)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step starts at the last k_l0_hist
starts = [i for i, r in enumerate(rows) if "k_l0_hist" in r["Kernel_Name"]]
i0 = starts[-1] if starts else 0
end = int(rows[i0]["Start_Timestamp"])
tot = {}
first = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("bra::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
    if len(sys.argv) > 2:
        print(f"{name:42s} {(e - s) / 1e3:9.1f} gap {(s - end) / 1e3:8.1f}  grid {r.get('Grid_Size_X', r.get('Grid_Size',''))}")
    t = tot.setdefault(name, [0, 0, 0.0])
    t[0] += 1; t[1] += e - s; t[2] += max(0, s - end) / 1e3
    end = max(end, e)
print(f"step span {(end - first) / 1e6:.3f} ms")
busy = sum(v[1] for v in tot.values()) / 1e6
print(f"busy {busy:.3f} ms, gaps {sum(v[2] for v in tot.values()) / 1e3:.3f} ms")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:42s} n={v[0]:4d} {v[1] / 1e6:8.3f} ms  gaps-before {v[2] / 1e3:7.3f} ms")
