set -o pipefail
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-legs > $O/bench.json 2>$O/bench.err &&
timeout -k 10 100 python -u tools/stamps.py 256 > $O/stamps.log 2>&1 &&
timeout -k 10 100 python -u tools/stamps.py --c4 > $O/stamps_c4.log 2>&1 &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $O/c4.json 2>$O/c4.err
rc=$?
tail -n 1 $O/pytest.log; grep "P2 exchange" $O/stamps.log $O/stamps_c4.log; exit $rc
