set -o pipefail
mkdir -p gpurun_out/r3t
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3t/pytest_gpu.log 2>&1 &&
for c in 1 2 4 8; do SW_PIPELINE_CHUNKS=$c timeout -k 10 120 python -u tools/boundary.py >> gpurun_out/r3t/boundary.jsonl 2>>gpurun_out/r3t/boundary.err || exit 1; done &&
SW_HOST_THREADS=8 timeout -k 10 120 python -u tools/boundary.py >> gpurun_out/r3t/boundary.jsonl 2>>gpurun_out/r3t/boundary.err
rc=$?
tail -3 gpurun_out/r3t/pytest_gpu.log; cat gpurun_out/r3t/boundary.jsonl; exit $rc
