"""Wall time per sw_mmf_allocate_types call (the heterogeneity-aware
MaxMinFairness LP on the GPU) at Gavel-like sizes, with the pivots taken and
the HiGHS level for comparison.    python tools/mmf_types_timing.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import sw_native as sn  # noqa: E402

s = sn.Solver(device=0)
rng = np.random.default_rng(0)
out = []
for m, n in [(50, 3), (100, 3), (200, 3), (400, 3), (200, 8)]:
    W = rng.integers(m // 4 + 1, m // 2 + 2, size=n).astype(np.int32)
    sf = rng.choice([1, 2, 4, 8], size=m, p=[0.6, 0.3, 0.09, 0.01]).astype(np.int32)
    c = rng.uniform(0.2, 3.0, size=(m, n)) * sf[:, None]
    s.mmf_allocate_types(W, sf, c)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        x, t, piv = s.mmf_allocate_types(W, sf, c)
    dt = (time.perf_counter() - t0) / reps
    out.append({"jobs": m, "types": n, "ms_per_call": dt * 1e3, "pivots": piv, "level": t})
s.close()
print(json.dumps(out))
