#!/bin/bash
# Round-2 GPU session: parity suite, smoke, the default bench line (C3 replicas
# + the sharded C4 sub-record), rocprofv3 kernel stats of the bench.
#   gpurun --timeout 900 -- bash tools/gpu_r2.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r2}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log; cat $OUT/bench.json; tail -5 $OUT/bench.err
exit $rc
