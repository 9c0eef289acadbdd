#!/bin/bash
# C4 with the one-wave placement loop at different thresholds, shard tests,
# per-rank kernel time at W = 2 / 4 (processes on one GPU).
#   gpurun --timeout 900 -- bash tools/gpu_c4_wave.sh <tag>
set -o pipefail
TAG=${1:-c4w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_p2.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_shard.log 2>&1 &&
for wa in 0 2048 4096; do
  SW_SHARD_WAVE_A=$wa timeout -k 10 120 python -u bench.py --workload c4 --steps 40 --warmup 3 > $OUT/bench_c4_wa$wa.json 2> $OUT/bench_c4_wa$wa.err || exit 1
done &&
SW_SHARD_WAVE_A=0 timeout -k 10 200 python -u tools/peer_timing.py 4 60 > $OUT/peer_w4_wa0.json 2> $OUT/peer_w4_wa0.err &&
timeout -k 10 200 python -u tools/peer_timing.py 4 60 > $OUT/peer_w4.json 2> $OUT/peer_w4.err &&
timeout -k 10 200 python -u tools/peer_timing.py 2 60 > $OUT/peer_w2.json 2> $OUT/peer_w2.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer4 -o run_%pid% -- python3 tools/peer_timing.py 4 40 > $OUT/prof_peer4.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer2 -o run_%pid% -- python3 tools/peer_timing.py 2 40 > $OUT/prof_peer2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 40 --warmup 3 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_shard.log
for f in $OUT/bench_c4_wa*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d.get('ms_per_step'), d.get('value'))" ; done
cat $OUT/peer_w*.json
python3 tools/peer_kernel_time.py $OUT/prof_peer2 2 | cut -c1-900
python3 tools/peer_kernel_time.py $OUT/prof_peer4 4 | cut -c1-1500
exit $rc
