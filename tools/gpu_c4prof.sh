#!/bin/bash
# rocprofv3 kernel stats of the C4 bench line (one 10k x 30 sharded solve per step).
#   gpurun --timeout 600 -- bash tools/gpu_c4prof.sh <tag>
set -o pipefail
TAG=${1:-c4prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 20 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
python3 - $OUT <<'PY'
import csv, sys, os
p = os.path.join(sys.argv[1], "prof_c4", "run_kernel_stats.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.2f} tot_ms {float(r["TotalDurationNs"])/1e6:8.3f}')
PY
exit $rc
