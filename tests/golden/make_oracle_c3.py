"""Generate tests/golden/oracle_c3.json: the reference model solved by the
oracle (oracle/milp_ref.py, HiGHS) at the headline sizes — 12 C3 instances
(900 jobs x 30 rounds, G=256, k=1e5, lambda=5) and 16 C5-mix instances
(900 x 30, G in {32, 64, 128, 256} with the matching scale_*gpus.json k and
lambda) — so the GPU kernel can be checked against the ORACLE at the
configuration the bench is quoted on, not only against the bit-exact twin.

    python tests/golden/make_oracle_c3.py [--procs 6] [--missing]

Per instance it records (all in the maximisation sense of shockwave.py:363-379):

  p1        the reference P1 MILP (shockwave.py:330-382), gap 1e-4: the
            objective J, utility term U and makespan M of its planned counts
            (closed-form evaluation, milp_ref.evaluate_counts), and HiGHS'
            dual bound;
  p1_lp     the LP relaxation of the same model (x, SOS2 binaries in [0, 1]):
            an upper bound of the P1 optimum;
  mk_min    the smallest makespan any plan reaches (same rows, objective
            min M) and its dual lower bound;
  util_at   the utility term alone at that makespan: max U s.t. every job's
            makespan <= mk_min (SURVEY.md Appendix A.4 — at k >= 10 the
            k*M term is ~1e5..1e9 and swamps a relative check of J), with
            its LP-relaxation bound;
  p2        the reference P2 MILP (shockwave.py:281-328) on the planned
            counts the CPU twin (= the GPU kernel, bit for bit) returns, gap
            1e-4, with a digest of those counts so a stale fixture is caught.

Inputs are not stored: they are regenerated from (seed, N, G, T, k, lambda)
by sw_synth.synth_problem and pinned by a SHA-256 of the six input arrays.
Only numbers are stored; no reference source.
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_c3.json")

# (name, seed, N, G, T) — C3 seeds are disjoint from the bench's (0 … 8191 per rank)
C3_CASES = [("c3", 500_000 + i, 900, 256, 30) for i in range(12)]
C5_CASES = [("c5", 600_000 + i, 900, (32, 64, 128, 256)[i % 4], 30) for i in range(16)]


def inputs_digest(a):
    h = hashlib.sha256()
    for arr in (a.w, a.d, a.F, a.E, a.R, a.p):
        h.update(np.ascontiguousarray(arr).tobytes())
    return h.hexdigest()[:32]


def counts_digest(n):
    return hashlib.sha256(np.ascontiguousarray(n, dtype=np.int32).tobytes()).hexdigest()[:32]


def problem(case):
    import sw_synth as ss

    name, seed, N, G, T = case
    cfg = ss.CLUSTER_CONFIG[G]
    return ss.synth_problem(seed, N, G, T, 120.0, cfg["k"], cfg["lam"])


def solve_case(case):
    import milp_ref as mr
    import ctypes
    import sw_native as sn

    name, seed, N, G, T = case
    a = problem(case)
    P = mr.Problem(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, list(a.bases))
    rec = {"name": name, "seed": seed, "N": N, "G": G, "T": T, "k": a.k,
           "lam": float(__import__("sw_synth").CLUSTER_CONFIG[G]["lam"]),
           "inputs_sha": inputs_digest(a)}
    t0 = time.perf_counter()
    st, xv, obj, bound, dt = mr.solve_p1(P, rel_gap=1e-4, time_limit=600.0)
    n = (xv > 0.5).sum(axis=1)
    J, U, M = mr.evaluate_counts(P, n)
    rec["p1"] = {"status": st, "J": J, "U": U, "M": M, "solver_obj": obj, "dual_bound": bound,
                 "seconds": dt, "feasible": mr.check_plan(P, (xv > 0.5).astype(np.uint8))}
    st, _, obj, _, dt = mr.solve_p1(P, relax=True, time_limit=600.0)
    rec["p1_lp"] = {"status": st, "bound": obj, "seconds": dt}
    # smallest makespan (objective: min M)
    st, xv, obj, bound, dt = mr.solve_p1(P, rel_gap=1e-9, time_limit=600.0, utility_weight=0.0,
                                         makespan_weight=1.0)
    nm = (xv > 0.5).sum(axis=1)
    Mmin = mr.evaluate_counts(P, nm)[2]
    rec["mk_min"] = {"status": st, "M": Mmin, "lower_bound": -bound, "seconds": dt}
    # utility at that makespan (the cap carries a relative 1e-12 for rounding)
    cap = Mmin * (1 + 1e-12) + 1e-9
    st, xv, obj, bound, dt = mr.solve_p1(P, rel_gap=1e-5, time_limit=400.0, makespan_weight=0.0,
                                         makespan_cap=cap)
    nu = (xv > 0.5).sum(axis=1)
    _, Uu, Mu = mr.evaluate_counts(P, nu)
    st_lp, _, ub_lp, _, dt_lp = mr.solve_p1(P, relax=True, time_limit=600.0, makespan_weight=0.0,
                                            makespan_cap=cap)
    rec["util_at"] = {"status": st, "M_cap": cap, "U": Uu, "M": Mu, "dual_bound": bound,
                      "lp_bound": ub_lp, "seconds": dt + dt_lp}
    solve_p2_part(rec)
    rec["seconds_total"] = time.perf_counter() - t0
    print(f"{name} seed {seed} G={G}: J_ref {rec['p1']['J']:.9g} J_twin {rec['twin']['J']:.9g} "
          f"U* {Uu:.6g} U_twin {rec['twin']['U']:.6g} M* {Mmin:.6g} M_twin {rec['twin']['M']:.6g} "
          f"p2 {rec['twin']['p2_objective'] / max(rec['p2']['objective'], 1e-300):.4f}x  "
          f"{rec['seconds_total']:.0f}s", flush=True)
    return rec


def solve_p2_part(rec):
    """The solver-dependent part: the twin's (= the GPU's) planned counts and
    the reference P2 MILP on exactly those counts (refreshed by --p2-only
    when the placement algorithm changes; the P1-side oracle stays)."""
    import milp_ref as mr
    import ctypes
    import sw_native as sn

    a = problem((rec["name"], rec["seed"], rec["N"], rec["G"], rec["T"]))
    assert inputs_digest(a) == rec["inputs_sha"]
    P = mr.Problem(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, list(a.bases))
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libplan_twin.so"))
    sn.declare_solver_api(lib, "twin_")
    pr, res = a.c_problem(), a.c_result()
    rc = lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
    assert rc >= 0
    nt = a.planned.astype(np.int64)
    y2, st2, p2obj, dt2 = mr.solve_p2(P, nt, time_limit=600.0, rel_gap=1e-4)
    rec["p2"] = {"status": st2, "objective": p2obj, "counts_sha": counts_digest(a.planned),
                 "seconds": dt2}
    rec["twin"] = {"J": res.objective, "U": res.utility, "M": res.makespan,
                   "p2_objective": res.p2_objective, "status": res.status}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=6)
    ap.add_argument("--only", default="")
    ap.add_argument("--missing", action="store_true",
                    help="keep the records already in the file, solve only the cases it lacks")
    ap.add_argument("--p2-only", dest="p2_only", action="store_true",
                    help="keep the P1-side oracle records, redo the twin counts and P2 MILPs")
    args = ap.parse_args()
    if args.p2_only:
        d = json.load(open(OUT))
        with mp.get_context("spawn").Pool(args.procs) as pool:
            d["cases"] = pool.map(solve_p2_part, d["cases"], chunksize=1)
        for r in d["cases"]:
            print(r["name"], r["seed"], r["G"], "p2 %.4fx" % (r["twin"]["p2_objective"] /
                                                           max(r["p2"]["objective"], 1e-300)))
        json.dump(d, open(OUT, "w"), indent=1)
        return
    cases = C3_CASES + C5_CASES
    if args.only:
        cases = [c for c in cases if f"{c[0]}:{c[1]}" in args.only.split(",")]
    have = {}
    if args.missing and os.path.exists(OUT):
        have = {(r["name"], r["seed"]): r for r in json.load(open(OUT))["cases"]}
    todo = [c for c in cases if (c[0], c[1]) not in have]
    with mp.get_context("spawn").Pool(args.procs) as pool:
        new = dict(zip([(c[0], c[1]) for c in todo], pool.map(solve_case, todo, chunksize=1)))
    recs = [have.get((c[0], c[1])) or new[(c[0], c[1])] for c in cases]
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_oracle_c3.py",
                   "oracle": "oracle/milp_ref.py (HiGHS restatement of shockwave.py:281-388)",
                   "scipy": __import__("scipy").__version__,
                   "cases": recs}, f, indent=1)
    print(f"wrote {OUT}: {len(recs)} cases")


if __name__ == "__main__":
    main()
