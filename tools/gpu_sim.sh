#!/bin/bash
# Fig-9 / C1 / C2 simulations with the GPU solvers (tools/sim_parity.py).
#   gpurun --timeout 900 -- bash tools/gpu_sim.sh <tag>
set -o pipefail
TAG=${1:-sim}
OUT=gpurun_out/$TAG; mkdir -p $OUT
T120="120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
timeout -k 10 200 python -u tools/sim_parity.py --trace $T120 --gpus 32 --max-jobs 50 --solver gpu --out $OUT/gpu_sim_c1_32.json > $OUT/c1.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --trace $T120 --gpus 64 --solver gpu --out $OUT/gpu_sim_c2_64.json > $OUT/c2.log 2>&1 &&
for g in 64 128 256; do
  timeout -k 10 300 python -u tools/sim_parity.py --gpus $g --solver gpu --out $OUT/gpu_sim_fig9_$g.json > $OUT/fig9_$g.log 2>&1 || exit 1
done
rc=$?
python3 - <<PY
import json, glob
for f in sorted(glob.glob('$OUT/gpu_sim_*.json')):
    d = json.load(open(f))
    for p, r in d['runs'].items():
        print(f.split('/')[-1], p, round(r['makespan']), round(r['avg_jct']), r['worst_ftf'], r.get('solves'), round(r.get('solve_seconds', 0), 3))
PY
exit $rc
