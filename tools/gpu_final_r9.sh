#!/bin/bash
# Round 6 evidence: tools/gpu_evidence.sh <tag>, then the GPU <-> twin fuzz
# scans of the three launch forms (batches of 512, on-chip split batches of
# 2200 and of 512).
#   gpurun --timeout 1200 -- bash tools/gpu_final_r9.sh <tag>
set -o pipefail
TAG=${1:-r9ev}
bash tools/gpu_evidence.sh $TAG || exit 1
O=gpurun_out/$TAG
timeout -k 10 200 python -u tools/fuzz_scan.py 4096 > $O/fuzz_scan_4096.log 2>&1 &&
timeout -k 10 200 python -u tools/fuzz_scan.py 8800 --onchip 2200 > $O/fuzz_scan_onchip_8800.log 2>&1 &&
timeout -k 10 200 python -u tools/fuzz_scan.py 4096 --onchip 512 > $O/fuzz_scan_onchip_4096.log 2>&1
rc=$?
tail -n 2 $O/fuzz_scan_*.log
exit $rc
