#!/bin/bash
# Instruction mix per solve kernel (one rocprofv3 pass, kernel-trace only) and
# the kernel stats of the same C3 bench command.
#   gpurun --timeout 600 -- bash tools/pmc_insts.sh <tag> [batch]
set -o pipefail
TAG=${1:-pmc_insts}
B=${2:-32768}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline --no-legs --steps 3 --warmup 1 --batch $B"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD > $OUT/stats.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/insts -o run -- $CMD > $OUT/insts.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
