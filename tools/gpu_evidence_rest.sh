#!/bin/bash
# The second half of tools/gpu_final_r9.sh (phase stamps, peer-transport C4
# timing, host boundary, C5 stages, MMF types, GPU <-> twin fuzz scans), for a
# call whose first half already ran.  Needs libshockwave_amd_stamps.so built
# (make -C shockwave-replication_amd/csrc stamps).
#   gpurun --timeout 1200 -- bash tools/gpu_evidence_rest.sh <tag>
set -o pipefail
TAG=${1:-evidence}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/stamps.py 256 > $OUT/stamps.log 2>&1 &&
timeout -k 10 200 python -u tools/peer_timing.py 2 100 > $OUT/peer_w2.json 2> $OUT/peer_w2.err &&
timeout -k 10 200 python -u tools/peer_timing.py 4 100 > $OUT/peer_w4.json 2> $OUT/peer_w4.err &&
timeout -k 10 120 python -u tools/boundary.py > $OUT/boundary.json 2> $OUT/boundary.err &&
timeout -k 10 120 python -u tools/c5_stages.py > $OUT/c5_stages.json 2> $OUT/c5_stages.err &&
timeout -k 10 200 python -u tools/stamps.py --c5 > $OUT/stamps_c5.log 2>&1 &&
timeout -k 10 120 python -u tools/mmf_types_timing.py > $OUT/mmf_types_timing.json 2> $OUT/mmf_types_timing.err &&
timeout -k 10 200 python -u tools/fuzz_scan.py 4096 > $OUT/fuzz_scan_4096.log 2>&1 &&
timeout -k 10 200 python -u tools/fuzz_scan.py 8800 --onchip 2200 > $OUT/fuzz_scan_onchip_8800.log 2>&1 &&
timeout -k 10 200 python -u tools/fuzz_scan.py 4096 --onchip 512 > $OUT/fuzz_scan_onchip_4096.log 2>&1
rc=$?
echo "exit $rc"; head -14 $OUT/stamps.log; cat $OUT/peer_w2.json $OUT/peer_w4.json; tail -n 2 $OUT/fuzz_scan_*.log
exit $rc
