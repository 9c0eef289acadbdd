#!/bin/bash
# Sharded-path GPU session: parity tests, C4 bench line, rocprofv3 kernel stats.
set -o pipefail
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; cat $OUT/bench_c4.json
python3 - $OUT/prof_c4/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:56]:56s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.2f} {r["Percentage"][:5]}%')
PY
exit $rc
