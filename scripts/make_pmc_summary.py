"""Build profiles/pmc_summary.json (HBM bytes per profiler-slot launch) from a gpurun PMC directory.

usage: make_pmc_summary.py <run_dir> <workload string> <out.json>
A slot's launch is the group of kernels its BRA_PROF scope covers (bwt.mjobs = the 2- and 4-wave
workgroup-job kernels of one encode); hbm bytes = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 correction).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import main as summarize  # noqa: E402

SLOTS = {
    "bwt.l0_hist": ["k_l0_hist"], "bwt.l0_scatter": ["k_l0_scatter"], "bwt.hist": ["k_hist<0u>"], "bwt.scan": ["k_scan<0u>"],
    "bwt.scatter": ["k_scatter", "k_scatter_p"], "bwt.jobs": ["k_jobs<0u>"], "bwt.mjobs": ["k_mjobs<0u, 2>", "k_mjobs<0u, 4>"],
    "mtf.lastocc": ["k_mtf_lastocc"], "mtf.scan": ["k_mtf_scan"], "mtf.encode": ["k_mtf_encode"],
    "rle.runs": ["k_rle_runs"], "rle.link": ["k_rle_link"], "rle.sizes": ["k_rle_sizes"], "rle.offsets": ["k_rle_offsets"],
    "rle.write": ["k_rle_write"], "huf.build": ["k_huff_build"], "huf.offsets": ["k_huff_offsets"], "huf.tilebits": ["k_huff_tilebits"],
    "huf.tilescan": ["k_huff_tilescan"], "huf.zero": ["k_huff_zero"], "huf.pack": ["k_huff_pack"],
}

if __name__ == "__main__":
    d, workload, out = sys.argv[1], sys.argv[2], sys.argv[3]
    k = summarize(d)
    res = {"source": d, "kernels": {}}
    for slot, names in SLOTS.items():
        have = [k[n] for n in names if n in k]
        if not have:
            continue
        res["kernels"][slot] = {
            "workload": workload,
            "hbm_bytes_per_launch": int(sum(e["hbm_bytes_per_launch"] for e in have)),
            "kernels": {n: k[n] for n in names if n in k},
        }
    json.dump(res, open(out, "w"), indent=1)
    for s_, e in res["kernels"].items():
        print(f"{s_:14s} {e['hbm_bytes_per_launch'] / 1e6:10.1f} MB per launch")
