"""Generates tests/golden/twin_plans.json: plan digests of the CPU twin
(oracle/plan_twin.c) on seeded instances at the reference cluster
configurations (scale_{32,64,128,256}gpus.json's k and lambda).

History: first pinned with the plain price bisection (commit aed1d81), kept
through the snapped searches (same results); re-pinned in
round 2 when the P2 cascade gained the width-profile repair (sw_repair.h),
which changes placements on purpose, and in round 3 when P2 gained the
exchange step (sw_p2x.h, negative-cycle cancelling), and in round 5 when the level
search became a branch and bound (sw_bnb.h) and P1 gained the pattern placement
(sw_profile_search).  Performance-only changes must keep
these digests; tests/test_twin_plans.py checks the twin and the GPU kernel
against them.  Regenerate only when the algorithm is meant to change:

    python tests/golden/make_twin_plans.py oracle/_build/libplan_twin.so
"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd")]
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

# (G, k, lambda, N, T): scale_256gpus.json, scale_128gpus.json, scale_64gpus.json
CONFIGS = [(256, 1e5, 5.0, 900, 30), (128, 1e-3, 15.0, 300, 30), (64, 10.0, 5.0, 300, 20),
           (32, 1e5, 5.0, 50, 20)]
SEEDS = range(8)


def digest(lib_path):
    lib = ctypes.CDLL(lib_path)
    sn.declare_solver_api(lib, "twin_")
    out = []
    for G, k, lam, N, T in CONFIGS:
        for seed in SEEDS:
            a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
            b = sn.ProblemArrays(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, tuple(a.bases))
            pr, res = b.c_problem(), b.c_result()
            rc = lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
            out.append({"G": G, "k": k, "lam": lam, "N": N, "T": T, "seed": seed, "rc": int(rc),
                        "objective": float(res.objective).hex(),
                        "plan_md5": hashlib.md5(b.plan.tobytes()).hexdigest(),
                        "counts_md5": hashlib.md5(b.planned.tobytes()).hexdigest()})
    return out


if __name__ == "__main__":
    rows = digest(sys.argv[1])
    json.dump({"source": "oracle/plan_twin.c, round 5 (level branch and bound, pattern placement)", "cases": rows},
              open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "twin_plans.json"), "w"),
              indent=0)
    print(len(rows), "cases")
