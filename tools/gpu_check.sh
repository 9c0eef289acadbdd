#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh <tag>
# Every GPU step runs under its own time limit; steps are chained with &&.
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; cat $OUT/smoke.log; cat $OUT/bench.json
exit $rc
