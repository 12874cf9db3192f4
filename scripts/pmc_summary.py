"""Summarise rocprofv3 --pmc passes per kernel (test/measurement tooling, not product code).

usage: pmc_summary.py <run_dir>  -- reads <run_dir>/{fetch,write,sq1,grbm}/run_counter_collection.csv.
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reports half of the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM section), so hbm_bytes = 2 * FETCH + WRITE.
VALU: SQ_INSTS_VALU = wave-level VALU instructions issued; GRBM_GUI_ACTIVE is summed over the 8 XCDs,
so a dispatch lasts GRBM_GUI_ACTIVE / 8 cycles on 256 CUs x 4 SIMDs = 1024 VALU issue ports.
valu_frac = SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 * 1024 * R_MAX), where R_MAX is the issue rate a
VALU-only kernel at full occupancy reaches (scripts/micro/valu_cal.hip, profiles/r06_valu_calibration.json:
0.380 wave-instructions per SIMD per cycle): 1.0 = the calibrated VALU issue ceiling.  (Round 5 used
4 * SQ_ACTIVE_INST_VALU / (cycles * 1024), which reads 1.52 on the calibration kernel: SQ_ACTIVE_INST_VALU
equals SQ_INSTS_VALU there, one count per wave-instruction.)
"""
import collections
import csv
import json
import os
import re
import sys

N_SIMD = 256 * 4  # VALU issue ports: 256 CUs x 4 SIMDs


def valu_rate_max():
    """Calibrated VALU issue ceiling (wave-instructions per SIMD per cycle)."""
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06_valu_calibration.json")
    try:
        return float(json.load(open(p))["valu_wave_insts_per_simd_per_cycle_max"])
    except (OSError, KeyError, ValueError):
        return 0.3804


def valu_frac(insts, gui_active):
    return round(insts / (gui_active / 8 * N_SIMD * valu_rate_max()), 4)


def short(name):
    n = re.sub(r"bra::\(anonymous namespace\)::|\(anonymous namespace\)::|^void ", "", name)
    return n.split("(")[0].strip()


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(d):
    f = load(os.path.join(d, "fetch", "run_counter_collection.csv"))
    w = load(os.path.join(d, "write", "run_counter_collection.csv"))
    sq = load(os.path.join(d, "sq1", "run_counter_collection.csv"))
    gr = load(os.path.join(d, "grbm", "run_counter_collection.csv"))
    out = {}
    for k in sorted(set(f) | set(w)):
        fs = f[k].get("FETCH_SIZE", [0.0])
        ws = w[k].get("WRITE_SIZE", [0.0])
        e = {"launches": len(fs), "fetch_kib_per_launch": sum(fs) / len(fs), "write_kib_per_launch": sum(ws) / len(ws)}
        e["hbm_bytes_per_launch"] = int((2 * e["fetch_kib_per_launch"] + e["write_kib_per_launch"]) * 1024)
        c = sq.get(k)
        if c and c.get("SQ_WAVE_CYCLES"):
            wc = sum(c["SQ_WAVE_CYCLES"])
            e["sq_frac_of_wave_cycles"] = {n: round(sum(v) / wc, 3) for n, v in c.items() if n.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
            e["valu_insts_per_lds_inst"] = round(sum(c.get("SQ_INSTS_VALU", [0])) / max(1.0, sum(c.get("SQ_INSTS_LDS", [0]))), 2)
            n = len(c["SQ_WAVE_CYCLES"])
            e["valu_insts_per_launch"] = sum(c.get("SQ_INSTS_VALU", [0])) / n
            e["active_valu_quads_per_launch"] = sum(c.get("SQ_ACTIVE_INST_VALU", [0])) / n
        g = gr.get(k)
        if g and g.get("GRBM_GUI_ACTIVE"):
            e["gui_active_per_launch"] = sum(g["GRBM_GUI_ACTIVE"]) / len(g["GRBM_GUI_ACTIVE"])
            if "valu_insts_per_launch" in e:
                e["valu_frac"] = valu_frac(e["valu_insts_per_launch"], e["gui_active_per_launch"])
        out[k] = e
    return out


if __name__ == "__main__":
    res = main(sys.argv[1])
    for k, e in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]):
        print(f"{k[:34]:34s} n={e['launches']:3d} hbm/launch {e['hbm_bytes_per_launch'] / 1e6:10.2f} MB", e.get("sq_frac_of_wave_cycles", ""),
              e.get("valu_insts_per_lds_inst", ""), e.get("valu_frac", ""))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
