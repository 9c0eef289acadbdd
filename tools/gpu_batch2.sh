#!/bin/bash
# C3 bench at several batch sizes (instances per launch), no legs.
set -o pipefail
TAG=${1:-batch2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for b in 4096 8192 16384 32768; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-legs --batch $b --steps 10 > $OUT/b$b.json 2> $OUT/b$b.err || exit 1
done
for b in 4096 8192 16384 32768; do python3 -c "
import json
d=json.loads(open('$OUT/b$b.json').read().strip().splitlines()[-1]); print($b, round(d['value']), round(d['ms_per_step'],3), round(d['cycles_per_instance']))"; done
