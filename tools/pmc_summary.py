"""Summarise rocprofv3 CSVs of a bench.py run into profiles/<tag>_summary.json.

    python tools/pmc_summary.py <tag> <kernel_stats.csv> <fetch.csv> <write.csv> <sq.csv> [batch]

Only the batched launches (grid = instances × 512 threads) are summarised.
One step of the solve is four launches on one stream (sw_level_kernel,
sw_pack_kernel, sw_plan_kernel for the instances the pack kernel leaves,
sw_p2x_kernel); each counter is averaged per kernel over its launches and the
per-step value is the sum over the four.  FETCH_SIZE / WRITE_SIZE are
reported in KB by rocprofv3; MI355X_MICROARCH.md (§HBM) says FETCH_SIZE counts
1/2 of a wide coalesced stream on gfx950, so both the raw value and the ×2
reading are recorded.
"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = ("sw_level_kernel", "sw_pack_kernel", "sw_plan_kernel", "sw_p2x_kernel")


def kernel_of(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def per_kernel(path, grid_min):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = kernel_of(r["Kernel_Name"])
        if k and int(r["Grid_Size"]) >= grid_min:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    means = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}
    total = defaultdict(float)
    for d in means.values():
        for c, v in d.items():
            total[c] += v
    return means, dict(total)


def main():
    tag, stats, fetch, write, sq = sys.argv[1:6]
    batch = int(sys.argv[6]) if len(sys.argv) > 6 else 512
    grid_min = batch * 512
    fk, f = per_kernel(fetch, grid_min)
    wk, w = per_kernel(write, grid_min)
    sk, s = per_kernel(sq, grid_min)
    kstats = [r for r in csv.DictReader(open(stats)) if kernel_of(r["Name"])]
    out = {
        "workload": {"instances": batch, "jobs": 900, "rounds": 30},
        "kernel_stats": kstats,
        "per_kernel": {"FETCH_SIZE_KB": {k: v.get("FETCH_SIZE") for k, v in fk.items()},
                       "WRITE_SIZE_KB": {k: v.get("WRITE_SIZE") for k, v in wk.items()},
                       "sq": sk},
        "hbm_bytes_per_launch_raw": 1024 * (f.get("FETCH_SIZE", 0) + w.get("WRITE_SIZE", 0)),
        "hbm_bytes_per_launch_fetch_x2": 1024 * (2 * f.get("FETCH_SIZE", 0) + w.get("WRITE_SIZE", 0)),
        "sq": s,
        "sq_wait_fraction": (s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"]) if s.get("SQ_WAVE_CYCLES") else None,
        "note": "per step = sum over the four solve kernels of each kernel's mean per launch",
    }
    json.dump(out, open(f"profiles/{tag}_summary.json", "w"), indent=1)
    print(out["hbm_bytes_per_launch_raw"], out["hbm_bytes_per_launch_fetch_x2"], out["sq_wait_fraction"])


if __name__ == "__main__":
    main()
