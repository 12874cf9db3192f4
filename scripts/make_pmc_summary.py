"""Build / update profiles/pmc_summary.json (HBM bytes per profiler-slot launch) from a gpurun PMC directory.

usage: make_pmc_summary.py <run_dir> <workload key> [<out.json>]
  <workload key>  "<kind>_<block size>" as bench.py looks it up (e.g. text_1048576, random_1048576,
                  sym16_8388608): the input kind and block size of the bench command the passes ran.
The file holds one entry per workload key: {"workloads": {key: {"source", "kernels": {slot: ...}}}};
other keys already in the file are kept.  A slot's launch is the group of kernels its BRA_PROF scope
covers (bwt.mjobs = the workgroup-job kernels of one encode, one per size class); hbm bytes =
2 * FETCH_SIZE + WRITE_SIZE (the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md); with the SQ
and GRBM passes, the slot's VALU instructions per launch and valu_frac (scripts/pmc_summary.py).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import main as summarize, valu_frac  # noqa: E402

SLOTS = {
    "bwt.pack": ["k_alpha", "k_pack_desc", "k_pack"],
    "bwt.l0_hist": ["k_l0_hist"], "bwt.l0_scatter": ["k_l0_scatter"], "bwt.hist": ["k_hist<0u>"], "bwt.scan": ["k_scan<0u>"],
    "bwt.scatter": ["k_scatter", "k_scatter_p"], "bwt.jobs": ["k_jobs<0u>"],
    "bwt.mjobs": ["k_mjobs<0u, 2>", "k_mjobs<0u, 4>", "k_mjobs<0u, 8>", "k_mjobs<0u, 16>"],
    "mtf.lastocc": ["k_mtf_lastocc"], "mtf.scan": ["k_mtf_scan"], "mtf.encode": ["k_mtf_encode_pos", "k_mtf_encode_reg", "k_mtf_encode_wave"],
    "rle.runs": ["k_rle_runs"], "rle.link": ["k_rle_link"], "rle.sizes": ["k_rle_sizes"], "rle.offsets": ["k_rle_offsets"],
    "rle.write": ["k_rle_write"], "huf.build": ["k_huff_build"], "huf.offsets": ["k_huff_offsets"], "huf.tilebits": ["k_huff_tilebits"],
    "huf.tilescan": ["k_huff_tilescan"], "huf.zero": ["k_huff_zero"], "huf.pack": ["k_huff_pack"],
}

if __name__ == "__main__":
    d, key = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                                             "pmc_summary.json")
    k = summarize(d)
    res = json.load(open(out)) if os.path.exists(out) else {}
    if "workloads" not in res:
        res = {"workloads": {}}
    entry = {"source": d, "kernels": {}}
    for slot, names in SLOTS.items():
        have = [k[n] for n in names if n in k]
        if not have:
            continue
        ks = entry["kernels"][slot] = {
            "hbm_bytes_per_launch": int(sum(e["hbm_bytes_per_launch"] for e in have)),
            "kernels": {n: k[n] for n in names if n in k},
        }
        # VALU of the slot's launch: its kernels run one after the other, so their cycles add
        if all("valu_insts_per_launch" in e for e in have):
            ks["valu_insts_per_launch"] = int(sum(e["valu_insts_per_launch"] for e in have))
        if all("valu_frac" in e for e in have):
            ks["valu_frac"] = valu_frac(sum(e["valu_insts_per_launch"] for e in have), sum(e["gui_active_per_launch"] for e in have))
    res["workloads"][key] = entry
    res["valu_frac_basis"] = "SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs x 0.380): profiles/r06_valu_calibration.json"
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for s_, e in entry["kernels"].items():
        print(f"{key} {s_:14s} {e['hbm_bytes_per_launch'] / 1e6:10.1f} MB per launch")
