#!/bin/bash
# Round-5 check: GPU suite, default bench line without the CPU leg, C4 line,
# phase stamps.   gpurun --timeout 1200 -- bash tools/gpu_r7.sh <tag>
set -o pipefail
TAG=${1:-r7}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 120 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; head -30 $OUT/stamps.log
python3 -c "
import json
for f in ['$OUT/bench_c3.json', '$OUT/bench_c4.json']:
    try:
        d = json.load(open(f)); print(f, round(d['value']), d['ms_per_step'], d.get('single_instance_ms'), (d.get('c5_sweep') or {}).get('value'), (d.get('c5_sweep') or {}).get('passes_per_instance_by_G'))
    except Exception as e: print(f, e)"
exit $rc
