#!/bin/bash
# Interleaved A/B of library builds (SW_LIB_PATH) on the C3 line without legs
# and on the C5 sweep (tools/c5_stages.py), three rounds:
#   gpurun --timeout 900 -- bash tools/gpu_ab_c3c5.sh <tag> lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  i=0
  for lib in "$@"; do
    SW_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-legs --steps 20 --warmup 3 > $OUT/v${i}_r$r.json 2> $OUT/v${i}_r$r.err || exit 1
    SW_LIB_PATH=$lib timeout -k 10 120 python -u tools/c5_stages.py > $OUT/c5_v${i}_r$r.json 2> $OUT/c5_v${i}_r$r.err || exit 1
    i=$((i+1))
  done
done
python3 - "$OUT" "$@" <<'PY'
import json, glob, sys
out = sys.argv[1]
for i, lib in enumerate(sys.argv[2:]):
    v = [json.load(open(f))['value'] for f in sorted(glob.glob(f'{out}/v{i}_r*.json'))]
    c = [json.load(open(f))['plan_ms'] for f in sorted(glob.glob(f'{out}/c5_v{i}_r*.json'))]
    print(json.dumps({"lib": lib, "c3_Msolves": [round(x / 1e6, 4) for x in v], "c3_mean": round(sum(v) / len(v) / 1e6, 4),
                      "c5_ms": [round(x, 4) for x in c], "c5_mean_ms": round(sum(c) / len(c), 4)}))
PY
