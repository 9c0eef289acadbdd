#!/bin/bash
# Interleaved A/B of sw_batch_run's stream count (SW_RUN_STREAMS) on the C5
# sweep (tools/c5_stages.py), three rounds each of the stream counts in NS (default 1 2 4).
#   gpurun --timeout 600 -- bash tools/gpu_streams_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
for r in 1 2 3; do
  for n in ${NS:-1 2 4}; do
    SW_RUN_STREAMS=$n timeout -k 10 120 python -u tools/c5_stages.py > $OUT/c5_s${n}_r$r.json 2> $OUT/c5_s${n}_r$r.err || exit 1
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
out = sys.argv[1]
for n in sorted({int(f.split("_s")[1].split("_")[0]) for f in glob.glob(f"{out}/c5_s*_r*.json")}):
    c = [json.load(open(f))['plan_ms'] for f in sorted(glob.glob(f'{out}/c5_s{n}_r*.json'))]
    print(json.dumps({"streams": n, "c5_ms": [round(x, 4) for x in c], "c5_mean_ms": round(sum(c) / len(c), 4)}))
PY
