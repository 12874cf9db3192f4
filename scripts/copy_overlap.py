"""How much of the host<->device copy time ran under kernels, from a rocprofv3 trace (measurement
tooling): python scripts/copy_overlap.py <dir with run_kernel_trace.csv, run_memory_copy_trace.csv>

Copies are the memory-copy records (SDMA) plus blit-kernel copies (__amd_rocclr_copyBuffer* in
the kernel trace: pinned device->host copies run as kernels).  For every copy of at least 1 MB the
time covered by some other (non-copy) kernel is summed; printed as JSON per direction, with the
window from the first large copy to the end of the last event and the kernels' busy time in it."""
import csv
import json
import os
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, busy):
    return sum(max(0, min(b, y) - max(a, x)) for x, y in busy)


def main(d):
    ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    ms = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))))
    copies, kern = [], []
    for r in ks:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        (copies if "copyBuffer" in r["Kernel_Name"] else kern).append((a, b, "blit"))
    for r in ms:
        copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", "").lower()))
    big = [c for c in copies if c[1] - c[0] > 100_000]  # ns: the batch copies, not the mailbox words
    if not big:
        return {}
    t0 = min(c[0] for c in big)
    t1 = max(max(b for _, b, _ in copies), max((b for _, b in ((k[0], k[1]) for k in kern)), default=0))
    busy = union([(a, b) for a, b, _ in kern if b > t0])
    res = {"window_ms": round((t1 - t0) / 1e6, 3), "kernel_busy_ms": round(sum(min(b, t1) - max(a, t0) for a, b in busy) / 1e6, 3)}
    for kind in sorted({c[2] for c in big}):
        sel = [c for c in big if c[2] == kind]
        tot = sum(b - a for a, b, _ in sel)
        cov = sum(covered(a, b, busy) for a, b, _ in sel)
        res[kind] = {"copies": len(sel), "ms": round(tot / 1e6, 3), "under_kernels_ms": round(cov / 1e6, 3), "under_kernels_frac": round(cov / max(tot, 1), 3)}
    return res


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1])))
