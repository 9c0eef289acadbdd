#!/bin/bash
# A/B of the C3 bench between the in-tree library and an alternative build,
# after the GPU parity suite.   gpurun -- bash tools/gpu_ab2.sh <tag> <alt.so>
set -o pipefail
TAG=${1:-ab}; ALT=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/a1.json 2> $OUT/a1.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/b1.json 2> $OUT/b1.err &&
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/a2.json 2> $OUT/a2.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/b2.json 2> $OUT/b2.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_gpu.log
for f in a1 b1 a2 b2; do python3 -c "
import json
try:
    d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4), d.get('single_instance_ms'), d['roofline'].get('passes_per_instance'))
except Exception as e: print('$f', e)"; done
exit $rc
