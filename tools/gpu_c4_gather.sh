#!/bin/bash
# C4 after the gathered search brackets: the shard GPU tests, the C4 line
# three times, its kernel trace, and W = 2 / 4 on one GPU.
#   gpurun --timeout 900 -- bash tools/gpu_c4_gather.sh <tag>
set -o pipefail
TAG=${1:-c4g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_shard.py tests/test_gpu_p2.py tests/test_c4_digest.py > $OUT/pytest_shard.log 2>&1 || { tail -30 $OUT/pytest_shard.log; exit 1; }
tail -3 $OUT/pytest_shard.log
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --workload c4 --steps 100 --warmup 5 > $OUT/c4_r$r.json 2> $OUT/c4_r$r.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 20 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err || exit 1
timeout -k 10 200 python -u tools/peer_timing.py 2 100 > $OUT/peer_w2.json 2> $OUT/peer_w2.err || exit 1
timeout -k 10 200 python -u tools/peer_timing.py 4 100 > $OUT/peer_w4.json 2> $OUT/peer_w4.err || exit 1
python3 - <<PY
import json, glob
v = [json.load(open(f)) for f in sorted(glob.glob('$OUT/c4_r*.json'))]
print('c4 ms', [round(x['ms_per_step'], 4) for x in v], 'steps', [x.get('collective_steps') for x in v],
      'digest', [x.get('matches_twin_digest') for x in v])
PY
cat $OUT/peer_w2.json $OUT/peer_w4.json
