#!/bin/bash
# Round-2 evidence: PMC passes of the default C3 bench (tools/gpu_pmc_c3.sh,
# 8192 instances), then the default line without the CPU leg and the C4 line
# alone (the C4 sub-record's timing against the standalone C4 run).
#   gpurun --timeout 900 -- bash tools/gpu_pmc_r2.sh <tag>
set -o pipefail
TAG=${1:-pmc_r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_pmc_c3.sh $TAG/pmc 8192 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/bench_nocpu.json 2> $OUT/bench_nocpu.err &&
timeout -k 10 120 python -u bench.py --workload c4 > $OUT/c4.json 2> $OUT/c4.err &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 100 > $OUT/c4_100.json 2> $OUT/c4_100.err
rc=$?
echo "exit $rc"
for f in bench_nocpu c4 c4_100; do python3 -c "
import json
d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1])
c=d.get('c4_sharded') or d
print('$f', round(d['value']), 'c4 ms', c.get('ms_per_solve', c.get('ms_per_step')), c.get('collective_steps'))" || true; done
exit $rc
