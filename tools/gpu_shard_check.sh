#!/bin/bash
# GPU session for the sharded path: its parity tests, then timings.
set -o pipefail
TAG=${1:-shard}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u tools/shard_timing.py 5 > $OUT/timing.log 2>&1
rc=$?
echo "exit $rc"; tail -5 $OUT/pytest_gpu.log; cat $OUT/timing.log
exit $rc
