#!/bin/bash
# A/B of a plan-kernel change: GPU parity suite, the C3 line of the in-tree
# library (a) vs an alternative build (b) interleaved, the per-config sweep of
# both, and the phase stamps of the diagnostic build.
#   gpurun --timeout 900 -- bash tools/gpu_ab_pack.sh <tag> <alt.so>
set -o pipefail
TAG=${1:-abpack}; ALT=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-legs"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py $B > $OUT/a1.json 2> $OUT/a1.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py $B > $OUT/b1.json 2> $OUT/b1.err &&
timeout -k 10 120 python -u bench.py $B > $OUT/a2.json 2> $OUT/a2.err &&
SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py $B > $OUT/b2.json 2> $OUT/b2.err &&
timeout -k 10 200 python -u tools/config_sweep.py > $OUT/sweep_a.log 2>&1 &&
SW_LIB_PATH=$ALT timeout -k 10 200 python -u tools/config_sweep.py > $OUT/sweep_b.log 2>&1 &&
timeout -k 10 200 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log
for f in a1 b1 a2 b2; do python3 -c "
import json
try:
    d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4), d.get('cycles_per_instance'))
except Exception as e: print('$f', e)"; done
head -3 $OUT/sweep_a.log; head -3 $OUT/sweep_b.log; head -12 $OUT/stamps.log
exit $rc
