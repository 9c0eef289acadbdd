#!/bin/bash
# A/B on one box: GPU parity suite on the in-tree library, then the C3 and C4
# bench lines of the in-tree library (a) against an alternative build (b),
# interleaved, and the phase stamps of the diagnostic build.
#   gpurun --timeout 900 -- bash tools/gpu_ab3.sh <tag> <alt.so>
set -o pipefail
TAG=${1:-ab3}; ALT=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-legs"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py $B > $OUT/a1.json 2> $OUT/a1.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py $B > $OUT/b1.json 2> $OUT/b1.err &&
timeout -k 10 120 python -u bench.py $B > $OUT/a2.json 2> $OUT/a2.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py $B > $OUT/b2.json 2> $OUT/b2.err &&
timeout -k 10 120 python -u bench.py --workload c4 > $OUT/c4a.json 2> $OUT/c4a.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py --workload c4 > $OUT/c4b.json 2> $OUT/c4b.err &&
timeout -k 10 200 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_gpu.log; head -12 $OUT/stamps.log
for f in a1 b1 a2 b2 c4a c4b; do python3 -c "
import json
try:
    d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4), d.get('cycles_per_instance'), d.get('collective_steps'))
except Exception as e: print('$f', e)"; done
exit $rc
