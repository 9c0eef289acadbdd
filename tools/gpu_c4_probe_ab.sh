#!/bin/bash
# The price probe's grid (SW_PROBE_BLOCKS) on the C4 line at W = 1, three runs each.
#   gpurun --timeout 600 -- bash tools/gpu_c4_probe_ab.sh <tag>
set -o pipefail
TAG=${1:-c4probe}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  for pb in 256 0 128; do
    SW_PROBE_BLOCKS=$pb timeout -k 10 120 python -u bench.py --workload c4 --steps 100 --warmup 5 > $OUT/c4_pb${pb}_r$r.json 2> $OUT/c4_pb${pb}_r$r.err || exit 1
  done
done
python3 - <<PY
import json, glob
for pb in (256, 0, 128):
    v = [json.load(open(f))['ms_per_step'] for f in sorted(glob.glob('$OUT/c4_pb%d_r*.json' % pb))]
    print('SW_PROBE_BLOCKS', pb, 'ms', [round(x, 4) for x in v])
PY
