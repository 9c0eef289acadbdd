"""Per-kernel instruction mix from tools/pmc_insts.sh, per solved instance.

    python tools/insts_summary.py gpurun_out/<tag> [batch] > profiles/<tag>_insts.json

SQ counters are summed over every wave of a dispatch; dividing by the
dispatch's instance count (the batch for the solve kernels) gives the per-
instance figure.  `valu_issue_ms` prices the VALU count at one wave64 VALU
instruction per CU per cycle (four SIMD16 units, four cycles per wave64
instruction) over the 256 CUs at 2.4 GHz: when it is close to the kernel's
measured duration the kernel is VALU-issue bound.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

CUS, CLK = 256, 2.4e9


def _name(s):
    return re.sub(r"^void ", "", s).split("(")[0]


def main(d, batch):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "insts", "**", "*counter_collection.csv"),
                                              recursive=True)[0])))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    meta = {}
    for r in rows:
        k = _name(r["Kernel_Name"])
        if not k.startswith("sw_"):
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        meta[k] = {"scratch_bytes_per_lane": int(r["Scratch_Size"]), "grid": int(r["Grid_Size"]),
                   "wg": int(r["Workgroup_Size"])}
    stats = {}
    for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[_name(r["Name"])] = float(r["AverageNs"]) / 1e6
    out = {"batch": batch, "kernels": {}}
    for k, c in sorted(acc.items()):
        n = len(disp[k])
        inst = meta[k]["grid"] // meta[k]["wg"]
        per = {name: round(v / n / inst, 1) for name, v in sorted(c.items())}
        valu_ms = c["SQ_INSTS_VALU"] / n / CUS / CLK * 1e3
        out["kernels"][k] = {"dispatches": n, "instances_per_dispatch": inst, **meta[k],
                             "per_instance": per, "valu_issue_ms": round(valu_ms, 3),
                             "measured_ms": round(stats[k], 3) if k in stats else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 32768)
