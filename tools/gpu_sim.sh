#!/bin/bash
# GPU session: gpu tests, then the Fig-9 simulations with the HIP solvers.
#   gpurun --timeout 900 -- bash tools/gpu_sim.sh <tag>
set -o pipefail
TAG=${1:-sim}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
T220="220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
T120="120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
T900="900_0.2_5_100_5_15_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --solver gpu --trace $T220 --gpus 64 --out $OUT/sim_220_64.json > $OUT/sim_220_64.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --solver gpu --trace $T120 --gpus 64 --out $OUT/sim_120_64.json > $OUT/sim_120_64.log 2>&1 &&
timeout -k 10 300 python -u tools/sim_parity.py --solver gpu --trace $T900 --gpus 256 --future-rounds 30 --out $OUT/sim_900_256.json > $OUT/sim_900_256.log 2>&1
rc=$?
echo "exit $rc"; tail -5 $OUT/pytest_gpu.log; cat $OUT/sim_*.log
exit $rc
