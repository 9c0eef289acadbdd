#!/bin/bash
# Phase stamps of the plan kernel (diagnostic build libshockwave_amd_stamps.so).
#   gpurun -- bash tools/gpu_stamps.sh <tag> [instances]
set -o pipefail
TAG=${1:-stamps}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python -u tools/stamps.py ${2:-256} > $OUT/stamps.log 2>&1
rc=$?
cat $OUT/stamps.log
exit $rc
