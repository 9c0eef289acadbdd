#!/bin/bash
# Microbenchmarks (tools/micro) then the C4 quick check.
set -o pipefail
TAG=${1:-micro}
mkdir -p gpurun_out/$TAG
timeout -k 10 60 ./tools/micro/barrier_bench > gpurun_out/$TAG/barrier_bench.log 2>&1
rc=$?
cat gpurun_out/$TAG/barrier_bench.log
exit $rc
