#!/bin/bash
# rocprofv3 passes over the C3 bench (each its own run, kernel-trace only):
# kernel stats, FETCH_SIZE, WRITE_SIZE, SQ counters; then, in the build container:
#   python tools/pmc_summary.py <tag> gpurun_out/<tag>/{stats/run_kernel_stats,fetch/run_counter_collection,write/run_counter_collection,sq/run_counter_collection}.csv <batch>
#   gpurun --timeout 600 -- bash tools/pmc_c3.sh <tag> [batch]
set -o pipefail
TAG=${1:-pmc_c3}
B=${2:-2048}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline --no-legs --steps 3 --warmup 1 --batch $B"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD > $OUT/stats.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq -o run -- $CMD > $OUT/sq.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
