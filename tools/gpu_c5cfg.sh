#!/bin/bash
# C5 sweep stage times under the launch-form thresholds (SW_SPLIT_MIN,
# SW_FUSE_MAX).   gpurun --timeout 600 -- bash tools/gpu_c5cfg.sh <tag>
set -o pipefail
TAG=${1:-c5cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/c5_stages.py > $OUT/default.json 2> $OUT/default.err &&
SW_SPLIT_MIN=256 timeout -k 10 120 python -u tools/c5_stages.py > $OUT/split256.json 2> $OUT/split256.err &&
SW_FUSE_MAX=1024 timeout -k 10 120 python -u tools/c5_stages.py > $OUT/fuse1024.json 2> $OUT/fuse1024.err
rc=$?
for f in $OUT/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['plan_ms'],4), round(d['p2x_ms'],4), round(d['plan_ms']+d['p2x_ms'],4))"; done
exit $rc
