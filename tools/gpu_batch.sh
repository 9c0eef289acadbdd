#!/bin/bash
# Headline bench at the default batch (C3 + C4), rocprofv3 kernel stats, PMC
# passes at that batch, and a batch sweep of the C3 rate.
#   gpurun --timeout 1200 -- bash tools/gpu_batch.sh <tag>
set -o pipefail
TAG=${1:-batch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_bench_prof.sh $TAG > $OUT/bench_prof.log 2>&1 &&
bash tools/gpu_pmc_c3.sh ${TAG}_pmc 8192 > $OUT/pmc.log 2>&1 &&
for b in 2048 4096 8192 16384; do
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --batch $b > $OUT/sweep_$b.json 2> $OUT/sweep_$b.err || exit $?
done
rc=$?
echo "exit $rc"; cat $OUT/bench_prof.log | cut -c1-300
for b in 2048 4096 8192 16384; do python3 -c "
import json; d=json.loads(open('$OUT/sweep_$b.json').read().strip().splitlines()[-1]); print($b, round(d['value']), round(d['ms_per_step'],3))"; done
exit $rc
