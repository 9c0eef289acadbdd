#!/bin/bash
# Sharded-engine loop: GPU shard tests, the C4 bench line and its kernel trace.
#   gpurun --timeout 600 -- bash tools/gpu_c4.sh <tag>
set -o pipefail
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_shard.log 2>&1 &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_shard.log; cat $OUT/bench_c4.json
exit $rc
