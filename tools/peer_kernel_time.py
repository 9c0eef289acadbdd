"""Per-rank kernel time per C4 solve from a rocprofv3 kernel trace of
tools/peer_timing.py (W ranks as processes on one GPU): each process's
kernel durations summed and divided by its solves (k_setup launches, one per
solve).  The ranks share the GPU, so wall time per solve does not fall with
W here; the per-rank kernel work is what a rank on its own GPU would run.
k_xchg (the peer exchange) spends most of its time waiting for the other
ranks' flags, so the work is also reported without it ("excl_xchg").
    python tools/peer_kernel_time.py <rocprofv3 output dir> [W]"""
import collections
import csv
import glob
import json
import os
import sys

rows = []
for f in sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        r["_file"] = os.path.basename(f)
        rows.append(r)
per = collections.defaultdict(lambda: [0.0, 0, collections.Counter()])
for r in rows:
    p = f'{r["_file"]}:{r.get("Thread_Id", "")}'  # one launching thread per rank process
    d = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    per[p][0] += d
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    if name.startswith("k_setup"):
        per[p][1] += 1
    per[p][2][name.split("(")[0].split("<")[0][:40]] += d
out = {}
for p, (tot, solves, by) in per.items():
    if solves == 0:
        continue
    out[p] = {"solves": solves, "kernel_us_per_solve": round(tot / solves / 1e3, 2),
              "kernel_us_per_solve_excl_xchg": round((tot - by.get("k_xchg", 0.0)) / solves / 1e3, 2),
              "top": {k: round(v / solves / 1e3, 2) for k, v in by.most_common(8)}}
ex = [v["kernel_us_per_solve_excl_xchg"] for v in out.values()]
print(json.dumps({"world": int(sys.argv[2]) if len(sys.argv) > 2 else None,
                  "mean_excl_xchg_us": round(sum(ex) / len(ex), 2) if ex else None, "ranks": out}))
