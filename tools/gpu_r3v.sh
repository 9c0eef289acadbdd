set -o pipefail
O=gpurun_out/r3v; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_host_boundary.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/boundary.py > $O/boundary.jsonl 2>$O/boundary.err &&
timeout -k 10 120 python -u tools/c5_stages.py > $O/c5.json 2>$O/c5.err &&
SW_SPLIT_MIN=256 timeout -k 10 120 python -u tools/c5_stages.py >> $O/c5.json 2>>$O/c5.err &&
export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 tools/c5_stages.py > $O/c5_prof.json 2>$O/c5_prof.err
rc=$?
tail -2 $O/pytest.log; cat $O/boundary.jsonl $O/c5.json; exit $rc
