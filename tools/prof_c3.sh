#!/bin/bash
# rocprofv3 kernel stats of the C3 bench (no legs): per-kernel time of the
# level-search, pack, full (slow-path) and P2 exchange kernels.
#   gpurun --timeout 600 -- bash tools/prof_c3.sh <tag> [batch]
set -o pipefail
TAG=${1:-prof_c3}
B=${2:-32768}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 1 --batch $B > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "exit $rc"
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -20
exit $rc
