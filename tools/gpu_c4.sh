#!/bin/bash
# C4 check: shard GPU tests, the C4 line at W = 1, peer-transport timing and
# per-rank kernel time at W = 2 / 4 (processes on one GPU), C4 kernel stats.
#   gpurun --timeout 900 -- bash tools/gpu_c4.sh <tag>
set -o pipefail
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_p2.py tests/test_c4_digest.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_shard.log 2>&1 &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 60 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 200 python -u tools/peer_timing.py 2 100 > $OUT/peer_w2.json 2> $OUT/peer_w2.err &&
timeout -k 10 200 python -u tools/peer_timing.py 4 100 > $OUT/peer_w4.json 2> $OUT/peer_w4.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer2 -o run_%pid% -- python3 tools/peer_timing.py 2 40 > $OUT/prof_peer2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer4 -o run_%pid% -- python3 tools/peer_timing.py 4 40 > $OUT/prof_peer4.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 40 --warmup 3 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_shard.log
python3 -c "import json; d=json.load(open('$OUT/bench_c4.json')); print('C4 W=1 ms', d.get('ms_per_step'))"
grep -h ms_per_solve $OUT/peer_w*.json
python3 tools/peer_kernel_time.py $OUT/prof_c4 1 > $OUT/kernel_w1.json
python3 tools/peer_kernel_time.py $OUT/prof_peer2 2 > $OUT/kernel_w2.json
python3 tools/peer_kernel_time.py $OUT/prof_peer4 4 > $OUT/kernel_w4.json
cut -c1-700 $OUT/kernel_w1.json $OUT/kernel_w2.json; cut -c1-1400 $OUT/kernel_w4.json
exit $rc
