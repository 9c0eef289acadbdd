#!/bin/bash
# Quick check: GPU parity suite, the C4 bench line (in-tree vs an alternative
# build), and the phase stamps of the diagnostic build.
#   gpurun --timeout 600 -- bash tools/gpu_c4q.sh <tag> <alt.so>
set -o pipefail
TAG=${1:-c4q}; ALT=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py --workload c4 > $OUT/c4a.json 2> $OUT/c4a.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py --workload c4 > $OUT/c4b.json 2> $OUT/c4b.err &&
timeout -k 10 120 python -u bench.py --workload c4 > $OUT/c4a2.json 2> $OUT/c4a2.err &&
timeout -k 10 200 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_gpu.log; head -12 $OUT/stamps.log
for f in c4a c4b c4a2; do python3 -c "
import json
try:
    d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4), d.get('collective_steps'))
except Exception as e: print('$f', e)"; done
exit $rc
