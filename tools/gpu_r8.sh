#!/bin/bash
# Round-6 check of one build: the pack-kernel GPU tests, the default C3 line
# (no CPU leg), kernel stats of the C3 step and the PMC passes at the bench
# batch.   gpurun --timeout 900 -- bash tools/gpu_r8.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r8}
K=${2:-"host_boundary or gpu_fuzz or gpu_parity"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
bash tools/pmc_c3.sh $TAG/pmc 32768
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log
python3 - <<PY
import json, csv, glob
d = json.load(open('$OUT/bench_c3.json'))
print('C3', round(d['value']), d['ms_per_step'], d.get('single_instance_ms'), (d.get('c5_sweep') or {}).get('value'), (d.get('c4_sharded') or {}).get('ms_per_solve'))
for f in glob.glob('$OUT/pmc/stats/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('%-60s %6s %10.3f ms avg' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))
PY
exit $rc
