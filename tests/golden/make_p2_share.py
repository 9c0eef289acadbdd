"""Generate tests/golden/p2_share.json: the HiGHS optimum of the reference's P2
MILP (shockwave.py:281-328, restated in oracle/milp_ref.py, gap 1e-4) on the
planned counts of large C4-shaped instances (3,000 and 5,000 jobs × 30 rounds,
G scaled with the jobs as in C4, k = 1e5, λ = 5; sw_synth).  The sharded
solve keeps the single instance's counts (its P1), so tests/test_shard.py holds
the share placement's P2 at worlds 2, 4 and 8 to this optimum.

    python tests/golden/make_p2_share.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("tests", "shockwave-replication_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import milp_ref as mr  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402
from helpers import to_oracle  # noqa: E402

CASES = [(5, 3000, 854), (6, 5000, 1424)]  # (seed, N, G): G/N as in C4 (2848 / 10,000)


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libplan_twin.so"))
    sn.declare_solver_api(lib, "twin_")
    out = []
    for seed, N, G in CASES:
        a = ss.synth_problem(seed, N, G, 30, 120.0, 1e5, 5.0)
        pr, res = a.c_problem(), a.c_result()
        assert lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res)) >= 0
        n = a.plan.sum(1).astype(np.int64)
        y, st, obj, dt = mr.solve_p2(to_oracle(a), n, time_limit=600.0, rel_gap=1e-4)
        assert y is not None
        out.append({"seed": seed, "N": N, "G": G, "T": 30, "k": 1e5, "lam": 5.0,
                    "counts": n.astype(int).tolist(), "p2_milp": float(obj), "milp_status": st,
                    "single_p2": float(res.p2_objective), "seconds": round(dt, 1)})
        print(seed, N, G, st, obj, res.p2_objective / obj)
    json.dump({"generator": "tests/golden/make_p2_share.py", "milp_gap": 1e-4, "cases": out},
              open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "p2_share.json"), "w"))


if __name__ == "__main__":
    main()
