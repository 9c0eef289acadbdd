#!/bin/bash
# C4 bench A/B, interleaved 3x (100 solves each): in-tree library vs an alternative.
#   gpurun --timeout 600 -- bash tools/gpu_c4ab.sh <tag> <alt.so>
set -o pipefail
TAG=${1:-c4ab}; ALT=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --workload c4 --steps 100 > $OUT/a$i.json 2> $OUT/a$i.err &&
  SW_LIB_PATH=$ALT timeout -k 10 120 python -u bench.py --workload c4 --steps 100 > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
done
for f in a1 b1 a2 b2 a3 b3; do python3 -c "
import json
d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4), d.get('collective_steps'))"; done
