"""Per-solve kernel time of the C4 line from a rocprofv3 kernel-stats CSV
(tools/gpu_shard_check.sh): python tools/c4_stats.py <run_kernel_stats.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
solves = [int(r["Calls"]) for r in rows if "k_setup" in r["Name"]][0]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"solves {solves}; kernel time per solve {tot / solves / 1e3:.1f} us")
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f'{r["Name"][:64]:64s} {int(r["Calls"]) / solves:5.1f}/solve avg {float(r["AverageNs"]) / 1e3:7.2f} us'
          f'  {float(r["TotalDurationNs"]) / solves / 1e3:7.2f} us/solve')
