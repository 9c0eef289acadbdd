#!/bin/bash
# The raises (sw_arith.h SW_RAISE_ITERS) on the GPU: the plan kernel's and the
# shard engine's re-solve paths against their twins, then the C3 line.
#   gpurun --timeout 900 -- bash tools/gpu_raise.sh <tag>
set -o pipefail
TAG=${1:-raise}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_frag_fuzz.py tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_p2.py tests/test_gpu_fuzz.py \
  tests/test_gpu_sim.py tests/test_oracle_c3.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print(b['value'],b['single_instance_ms'],b['c5_sweep']['value'],b['c4_sharded']['ms_per_solve'])"
