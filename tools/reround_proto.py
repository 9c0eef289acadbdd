"""Prototype (test infrastructure, CPU only): per-round exact re-optimisation
of the twin's P1 plan on the FRAG cases of tests/test_oracle.py that stay
above 1e-3 of the MILP.  For each round t in turn,
every subset of jobs that fits G replaces the round's current set when the
exact P1 objective (milp_ref.evaluate_counts, makespan term included) rises;
passes until none does.  Brute force over subsets: N <= 14 only.
    python tools/reround_proto.py"""
import sys, ctypes, itertools
sys.path.insert(0,'tests'); sys.path.insert(0,'shockwave-replication_amd'); sys.path.insert(0,'oracle'); sys.path.insert(0,'.')
import numpy as np
import sw_native as sn, sw_synth as ss
import milp_ref as mr
from helpers import to_oracle
import os
os.chdir(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL('oracle/_build/libplan_twin.so'); sn.declare_solver_api(lib, "twin_")
cases = [(0, 12, 8, 1e-3), (1, 12, 8, 1e-3), (2, 10, 12, 1e-3), (10, 8, 8, 1.0), (10, 8, 8, 1e5)]
for (seed,N,G,k) in cases:
    a = ss.synth_problem(seed, N, G, 6, 120.0, k, 5.0, width_p=(0.4, 0.3, 0.2, 0.1))
    P = to_oracle(a)
    sol = mr.plan_solve(P, rel_gap=1e-6, time_limit=60)
    ref = mr.evaluate_counts(P, sol.n)[0]
    pr, res = a.c_problem(), a.c_result()
    lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
    y = a.plan.copy().astype(bool)
    T = a.T; w = np.asarray(a.w)
    n = y.sum(1)
    J = mr.evaluate_counts(P, n)[0]
    g0 = (ref-J)/abs(ref)
    Tj = None
    for pas in range(4):
        changed=False
        for t in range(T):
            cur = y[:,t].copy()
            base = n - cur
            best = (J, cur)
            elig = [j for j in range(N) if w[j] <= G]
            for r in range(len(elig)+1):
                for S in itertools.combinations(elig, r):
                    if w[list(S)].sum() > G: continue
                    nn = base.copy(); nn[list(S)] += 1
                    Jn = mr.evaluate_counts(P, nn)[0]
                    if Jn > best[0] * (1 - 1e-12) + 1e-12 and Jn > best[0]:
                        m = np.zeros(N, bool); m[list(S)] = True
                        best = (Jn, m)
            if best[0] > J:
                y[:,t] = best[1]; n = y.sum(1); J = best[0]; changed=True
        if not changed: break
    print(seed,N,G,k, "gap before", g0, "after", (ref-J)/abs(ref), "passes", pas+1)
