#!/bin/bash
# Shard placement loop variants: E chosen by the active entries (default),
# E by the entries (SW_SHARD_PACK_SEL=0), 4-wave loops (SEL=0, NT=256):
# C4 at W = 1 and peer timing at W = 2 / 4; shard tests on the default.
#   gpurun --timeout 900 -- bash tools/gpu_nt.sh <tag>
set -o pipefail
TAG=${1:-nt}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_p2.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 &&
for cfg in "sel" "old:SW_SHARD_PACK_SEL=0" "nt256:SW_SHARD_PACK_SEL=0 SW_SHARD_PACK_NT=256"; do
  name=${cfg%%:*}; envs=""; [ "$cfg" != "$name" ] && envs=${cfg#*:}
  env $envs timeout -k 10 120 python -u bench.py --workload c4 --steps 60 --warmup 3 > $OUT/c4_$name.json 2>/dev/null || exit 1
  env $envs timeout -k 10 200 python -u tools/peer_timing.py 2 100 > $OUT/peer2_$name.json 2>/dev/null || exit 1
  env $envs timeout -k 10 200 python -u tools/peer_timing.py 4 100 > $OUT/peer4_$name.json 2>/dev/null || exit 1
done &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer2 -o run_%pid% -- python3 tools/peer_timing.py 2 40 > $OUT/prof_peer2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer4 -o run_%pid% -- python3 tools/peer_timing.py 4 40 > $OUT/prof_peer4.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rr -o run -- python3 tools/rr_c4.py 10 > $OUT/rr_c4.json 2> $OUT/rr_c4.err
rc=$?
cat $OUT/rr_c4.json; grep -h "k_rr\b\|k_rr(" $OUT/prof_rr/run_kernel_stats.csv | cut -d, -f1-5
tail -1 $OUT/pytest.log
for name in sel old nt256; do
  python3 -c "
import json
a=json.load(open('$OUT/c4_$name.json')); b=[l for l in open('$OUT/peer2_$name.json') if 'world' in l]; c=[l for l in open('$OUT/peer4_$name.json') if 'world' in l]
print('$name', round(a['ms_per_step'],4), round(json.loads(b[-1])['ms_per_solve'],4), round(json.loads(c[-1])['ms_per_solve'],4))"
done
python3 tools/peer_kernel_time.py $OUT/prof_peer2 2 | cut -c1-300
python3 tools/peer_kernel_time.py $OUT/prof_peer4 4 | cut -c1-300
exit $rc
