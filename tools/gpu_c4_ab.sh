#!/bin/bash
# Interleaved A/B of an environment switch on the C4 line (W = 1), one box:
#   gpurun --timeout 900 -- bash tools/gpu_c4_ab.sh <tag> VAR v1 v2 [v3]
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3 4; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 120 python -u bench.py --workload c4 --steps 200 --warmup 5 > $OUT/c4_${v}_r$r.json 2> $OUT/c4_${v}_r$r.err || exit 1
  done
done
python3 - "$OUT" "$@" <<'PY'
import json, glob, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    ms = [json.load(open(f))['ms_per_step'] for f in sorted(glob.glob(f'{out}/c4_{v}_r*.json'))]
    print(v, 'ms', [round(x, 4) for x in ms], 'mean', round(sum(ms) / len(ms), 4))
PY
