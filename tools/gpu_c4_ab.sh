#!/bin/bash
# C4 check of one change: the shard GPU tests, then the C4 line at W = 1
# (100 solves, three times).
#   gpurun --timeout 600 -- bash tools/gpu_c4_ab.sh <tag>
set -o pipefail
TAG=${1:-c4ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_p2.py tests/test_c4_digest.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_shard.log 2>&1 || { tail -20 $OUT/pytest_shard.log; exit 1; }
tail -1 $OUT/pytest_shard.log
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --workload c4 --steps 100 --warmup 5 > $OUT/bench_c4_$i.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_c4_$i.json')); print('C4 W=1 ms', d['ms_per_step'])"
done
