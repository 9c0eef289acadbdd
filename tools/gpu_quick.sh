#!/bin/bash
# Quick check of one change: the default C3 bench line (no CPU leg), kernel
# stats of the C3 step, then the GPU suite.
#   gpurun --timeout 900 -- bash tools/gpu_quick.sh <tag>
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 1 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 150 python -u tools/c5_stages.py > $OUT/c5_stages.json 2> $OUT/c5_stages.err &&
timeout -k 10 200 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1 &&
timeout -k 10 200 python -u tools/stamps.py --c5 > $OUT/stamps_c5.log 2>&1
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; cat $OUT/c5_stages.json; grep -h "mean cycles\|exchange kernel" $OUT/stamps.log $OUT/stamps_c5.log
python3 - <<PY
import json, csv, glob
d = json.load(open('$OUT/bench_c3.json'))
print('C3', round(d['value']), d['ms_per_step'], d.get('single_instance_ms'), (d.get('c5_sweep') or {}).get('value'), (d.get('c5_sweep') or {}).get('passes_per_instance_by_G'))
for f in glob.glob('$OUT/prof_c3/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('%-60s %6s %10.3f ms avg' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))
PY
exit $rc
