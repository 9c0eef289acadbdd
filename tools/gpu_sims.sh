#!/bin/bash
# BASELINE C1 / C2 (and the 220-job Fig-9 trace) as full simulations on the
# GPU solvers (sw_plan_solve for Shockwave, sw_mmf_allocate for
# MaxMinFairness), one JSON per run with wall time and solve time.
#   gpurun --timeout 600 -- bash tools/gpu_sims.sh <tag>
set -o pipefail
TAG=${1:-sims}
OUT=gpurun_out/$TAG
mkdir -p $OUT
T120="120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
T220="220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
timeout -k 10 200 python -u tools/sim_parity.py --solver gpu --trace "$T120" --gpus 32 --max-jobs 50 --out $OUT/c1_32.json > $OUT/c1.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --solver gpu --trace "$T120" --gpus 64 --out $OUT/c2_64.json > $OUT/c2.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --solver gpu --trace "$T220" --gpus 64 --out $OUT/fig9_64.json > $OUT/fig9.log 2>&1
rc=$?
for f in $OUT/*.json; do python3 -c "
import json; d=json.load(open('$f'))
for k,v in d['runs'].items(): print('$f', k, {x: v[x] for x in ('makespan','avg_jct','worst_ftf','solves','solve_seconds','wall_s')})"; done
exit $rc
