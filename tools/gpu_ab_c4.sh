#!/bin/bash
# A/B of the sharded C4 solve on one box: GPU parity suite on the in-tree
# library, then bench.py --workload c4 for the in-tree library (a) and an
# alternative build (b), interleaved, and the default line (C5 / C4 legs).
#   gpurun --timeout 900 -- bash tools/gpu_ab_c4.sh <tag> <alt.so>
set -o pipefail
TAG=${1:-abc4}; ALT=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
C="--workload c4 --steps 100 --warmup 5"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py $C > $OUT/a1.json 2> $OUT/a1.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py $C > $OUT/b1.json 2> $OUT/b1.err &&
timeout -k 10 120 python -u bench.py $C > $OUT/a2.json 2> $OUT/a2.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py $C > $OUT/b2.json 2> $OUT/b2.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/default.json 2> $OUT/default.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_gpu.log
for f in a1 b1 a2 b2; do python3 -c "
import json
try:
    d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],4), d.get('collective_steps'))
except Exception as e: print('$f', e)"; done
python3 -c "
import json
d=json.loads(open('$OUT/default.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('c5_sweep')), json.dumps(d.get('c4_sharded')))"
exit $rc
