# GPU ↔ twin fuzz scans over the round-3 launch forms (on-chip batches):
# split kernels (2048 per batch), full kernel + exchange kernel (600), fused (200).
set -o pipefail
O=gpurun_out/scan; mkdir -p $O
timeout -k 10 500 python -u tools/fuzz_scan.py 32768 --onchip 2048 > $O/split.log 2>&1 &&
timeout -k 10 200 python -u tools/fuzz_scan.py 9600 --onchip 600 > $O/mono.log 2>&1 &&
timeout -k 10 200 python -u tools/fuzz_scan.py 8000 --onchip 200 > $O/fused.log 2>&1
rc=$?
tail -n 2 $O/split.log $O/mono.log $O/fused.log; exit $rc
