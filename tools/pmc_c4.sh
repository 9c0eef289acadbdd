#!/bin/bash
# PMC pass (SQ counters) over the C4 sharded solve; kernel-trace only, no other tracing.
set -o pipefail
OUT=gpurun_out/${1:-pmc_c4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq -o run -- python3 tools/shard_timing.py 2 > $OUT/sq.log 2>&1
rc=$?
python3 - $OUT/sq/run_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:48]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    calls = max(n[(k, c)] for c in d)
    print(k, "calls", calls, {c: round(v / calls) for c, v in sorted(d.items())})
PY
exit $rc
