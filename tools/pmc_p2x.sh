#!/bin/bash
# rocprofv3 counter passes over the C3 bench, for the P2 exchange kernel
# (sw_p2x_kernel): instruction mix, waits and LDS behaviour, each pass its own
# run with kernel trace only.
#   gpurun --timeout 600 -- bash tools/pmc_p2x.sh <tag> [batch]
set -o pipefail
TAG=${1:-pmc_p2x}
B=${2:-2048}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline --no-legs --steps 2 --warmup 1 --batch $B"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/sq1 -o run -- $CMD > $OUT/sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d $OUT/sq2 -o run -- $CMD > $OUT/sq2.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
