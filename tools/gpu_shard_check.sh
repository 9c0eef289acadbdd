#!/bin/bash
# Sharded-engine check: the GPU shard tests, the C4 line, the peer timing at
# W = 2 / 4 on one GPU, and a rocprofv3 kernel trace of the C4 line.
#   gpurun --timeout 900 -- bash tools/gpu_shard_check.sh <tag>
set -o pipefail
TAG=${1:-shard}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_c4_digest.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 200 python -u tools/peer_timing.py 2 100 > $OUT/peer_w2.json 2> $OUT/peer_w2.err &&
timeout -k 10 200 python -u tools/peer_timing.py 4 100 > $OUT/peer_w4.json 2> $OUT/peer_w4.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 32 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log; cat $OUT/bench_c4.json; cat $OUT/peer_w2.json $OUT/peer_w4.json
[ $rc -eq 0 ] || exit $rc
# per-rank kernel time at W = 2 / 4 (processes on one GPU)
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer2 -o run_%pid% -- python3 tools/peer_timing.py 2 40 > $OUT/prof_peer2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer4 -o run_%pid% -- python3 tools/peer_timing.py 4 40 > $OUT/prof_peer4.log 2>&1 &&
python3 tools/peer_kernel_time.py $OUT/prof_peer2 2 > $OUT/peer_kernel_w2.json &&
python3 tools/peer_kernel_time.py $OUT/prof_peer4 4 > $OUT/peer_kernel_w4.json
rc=$?
cat $OUT/peer_kernel_w2.json $OUT/peer_kernel_w4.json
exit $rc
