#!/bin/bash
# Iteration loop on the GPU box: all gpu tests, C3 bench (no CPU leg), C4 bench,
# rocprofv3 kernel stats of both.
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
timeout -k 10 120 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 > $OUT/prof_c4.json 2> $OUT/prof_c4.err
rc=$?
echo "exit $rc"; tail -3 $OUT/pytest_gpu.log
python3 - $OUT <<'PY'
import csv, json, sys, os
o = sys.argv[1]
for f in ("bench_c3.json", "bench_c4.json"):
    p = os.path.join(o, f)
    if os.path.exists(p) and os.path.getsize(p):
        d = json.loads(open(p).read().strip().splitlines()[-1])
        print(f, round(d["value"], 1), d["unit"], "ms/step", round(d["ms_per_step"], 4),
              "single_ms", d.get("single_instance_ms"), "frac", (d.get("roofline") or {}).get("frac"))
for w in ("prof_c3", "prof_c4"):
    p = os.path.join(o, w, "run_kernel_stats.csv")
    if os.path.exists(p):
        print(w)
        for r in csv.DictReader(open(p)):
            print(f'  {r["Name"][:54]:54s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.2f} {r["Percentage"][:5]}%')
PY
exit $rc
