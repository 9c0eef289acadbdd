#!/bin/bash
# Re-entry check of the restored tree: GPU parity suite and the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r2d_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_gpu.log; cat $OUT/bench.json
exit $rc
