#!/bin/bash
# Interleaved A/B of sw_batch_run's stream count (SW_RUN_STREAMS) on the C3
# line without legs, three rounds each of the counts in NS (default 1 2 4).
#   gpurun --timeout 600 -- bash tools/gpu_streams_c3_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
for r in 1 2 3; do
  for n in ${NS:-1 2 4}; do
    SW_RUN_STREAMS=$n timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-legs --steps 20 --warmup 3 > $OUT/c3_s${n}_r$r.json 2> $OUT/c3_s${n}_r$r.err || exit 1
  done
done
python3 - "$OUT" <<'PY'
import json, glob, sys
out = sys.argv[1]
for n in sorted({int(f.split("_s")[-1].split("_")[0]) for f in glob.glob(f"{out}/c3_s*_r*.json")}):
    v = [json.load(open(f))['value'] for f in sorted(glob.glob(f'{out}/c3_s{n}_r*.json'))]
    print(json.dumps({"streams": n, "c3_Msolves": [round(x / 1e6, 4) for x in v], "c3_mean": round(sum(v) / len(v) / 1e6, 4)}))
PY
