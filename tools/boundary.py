"""Host-boundary timing of sw_plan_solve_batch on the C3 bench batch (32,768
instances, 900 jobs x 30 rounds): byte plans and bit-packed plans, 5 calls
each after one warm call.  SW_PIPELINE_CHUNKS / SW_HOST_THREADS in the
environment select the pipeline's chunk count and host threads.
    python tools/boundary.py [batch]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "shockwave-replication_amd"))
import numpy as np  # noqa: E402

import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
batch = [ss.synth_problem(i, 900, 256, 30, 120.0, 1e5, 5.0) for i in range(n)]
solver = sn.Solver(device=0)
lib = solver.lib
probs = (sn.SwProblem * n)(*[a.c_problem() for a in batch])
ress = (sn.SwResult * n)(*[a.c_result() for a in batch])
out = {"batch": n, "chunks_env": os.environ.get("SW_PIPELINE_CHUNKS"),
       "threads_env": os.environ.get("SW_HOST_THREADS")}
for mode in ("bytes", "masks"):
    if mode == "masks":
        masks = [np.zeros(a.N, dtype=np.uint64) for a in batch]
        for i in range(n):
            ress[i].plan = None
            ress[i].plan_masks = masks[i].ctypes.data_as(C.POINTER(C.c_uint64))
    assert lib.sw_plan_solve_batch(solver.h, n, probs, ress) >= 0
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        assert lib.sw_plan_solve_batch(solver.h, n, probs, ress) >= 0
        t.append(time.perf_counter() - t0)
    out[mode + "_ms"] = [round(x * 1e3, 2) for x in t]
    out[mode + "_solves_per_s"] = n / float(np.median(t))
print(json.dumps(out))
