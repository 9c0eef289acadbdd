#!/bin/bash
# Full GPU session: parity tests, smoke, bench lines (C3 headline, C4 sharded),
# rocprofv3 kernel stats of both, and the Fig-9 simulations with the HIP solvers.
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
T220="220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err &&
for g in 64 128 256; do
  timeout -k 10 200 python -u tools/sim_parity.py --solver gpu --trace $T220 --gpus $g --out $OUT/sim_220_$g.json > $OUT/sim_220_$g.log 2>&1 || exit $?
done
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log; cat $OUT/bench_c3.json $OUT/bench_c4.json; cat $OUT/sim_220_*.log | cut -c1-220
exit $rc
