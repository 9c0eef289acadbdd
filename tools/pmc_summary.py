"""Summarise rocprofv3 CSVs of a bench.py run into profiles/<tag>_summary.json.

    python tools/pmc_summary.py <tag> <kernel_stats.csv> <fetch.csv> <write.csv> <sq.csv>

Only the batched launches (grid = instances × 512 threads) are summarised.
FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3.  MI355X_MICROARCH.md
(§HBM) says FETCH_SIZE counts 1/2 of a wide coalesced stream on gfx950; this
kernel's loads are 4–8-byte scalar per-thread loads (not calibrated), so both
the raw value and the ×2 reading are recorded.
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, grid_min):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "sw_plan_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) >= grid_min:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    tag, stats, fetch, write, sq = sys.argv[1:6]
    grid_min = (int(sys.argv[6]) if len(sys.argv) > 6 else 512) * 512
    f, nf = per_kernel(fetch, grid_min)
    w, nw = per_kernel(write, grid_min)
    s, ns = per_kernel(sq, grid_min)
    kstats = [r for r in csv.DictReader(open(stats)) if "sw_plan_kernel" in r["Name"]]
    out = {
        "workload": {"instances": int(sys.argv[6]) if len(sys.argv) > 6 else 512, "jobs": 900, "rounds": 30},
        "kernel_stats": kstats,
        "batched_launches": {"FETCH_SIZE_KB": f.get("FETCH_SIZE"), "WRITE_SIZE_KB": w.get("WRITE_SIZE"),
                             "launches": {**nf, **nw}},
        "hbm_bytes_per_launch_raw": 1024 * ((f.get("FETCH_SIZE") or 0) + (w.get("WRITE_SIZE") or 0)),
        "hbm_bytes_per_launch_fetch_x2": 1024 * (2 * (f.get("FETCH_SIZE") or 0) + (w.get("WRITE_SIZE") or 0)),
        "sq": s,
        "sq_wait_fraction": (s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"]) if s.get("SQ_WAVE_CYCLES") else None,
    }
    json.dump(out, open(f"profiles/{tag}_summary.json", "w"), indent=1)
    print(json.dumps(out["batched_launches"]), out["hbm_bytes_per_launch_raw"], out["sq_wait_fraction"])


if __name__ == "__main__":
    main()
