#!/bin/bash
# Evidence set for one build, one call: GPU parity suite, smoke, the
# default bench line, rocprofv3 kernel stats of the C3 bench (no legs) and of
# the C4 line, PMC passes at the default batch, phase stamps, the peer-transport
# C4 timing at W = 2 / 4 as processes on one GPU, the host-boundary timing
# (tools/boundary.py) and the C5 sweep's stage times (tools/c5_stages.py).
#   gpurun --timeout 1200 -- bash tools/gpu_evidence.sh <tag>
set -o pipefail
TAG=${1:-evidence}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B=32768
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 1 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 20 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err &&
bash tools/pmc_c3.sh $TAG/pmc $B &&
bash tools/pmc_insts.sh $TAG/insts $B &&
timeout -k 10 200 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1 &&
timeout -k 10 200 python -u tools/peer_timing.py 2 100 > $OUT/peer_w2.json 2> $OUT/peer_w2.err &&
timeout -k 10 200 python -u tools/peer_timing.py 4 100 > $OUT/peer_w4.json 2> $OUT/peer_w4.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer2 -o run_%pid% -- python3 tools/peer_timing.py 2 40 > $OUT/prof_peer2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_peer4 -o run_%pid% -- python3 tools/peer_timing.py 4 40 > $OUT/prof_peer4.log 2>&1 &&
timeout -k 10 120 python -u tools/boundary.py > $OUT/boundary.json 2> $OUT/boundary.err &&
timeout -k 10 120 python -u tools/c5_stages.py > $OUT/c5_stages.json 2> $OUT/c5_stages.err &&
timeout -k 10 200 python -u tools/stamps.py --c5 > $OUT/stamps_c5.log 2>&1 &&
timeout -k 10 120 python -u tools/mmf_types_timing.py > $OUT/mmf_types_timing.json 2> $OUT/mmf_types_timing.err
rc=$?
echo "exit $rc"; tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log; cat $OUT/bench.json; head -14 $OUT/stamps.log
exit $rc
