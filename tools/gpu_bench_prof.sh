#!/bin/bash
# Bench lines (C3 headline, C4 sharded) and rocprofv3 kernel stats (CSV) of each.
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; cat $OUT/bench_c3.json $OUT/bench_c4.json; find $OUT -name "*stats*"
exit $rc
