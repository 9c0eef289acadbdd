"""Prototype (test infrastructure, CPU only) of the per-round exact
re-optimisation of a re-solved P1 plan, run on the
twin's plans against the MILP oracle.

For each round t in turn, with every other round fixed (b_j = n_j - y_jt),
the round's job set S is re-chosen to maximise the exact P1 objective
    sum_j f_j(b_j + [j in S]) - k * max_j g_j(b_j + [j in S])
subject to sum_{j in S} w_j <= G.  The utility part is a 0/1 knapsack with
values v_j = f_j(b_j + 1) - f_j(b_j); the makespan part is handled by
enumerating its level theta: every job with g_j(b_j) > theta must be in S
(and needs g_j(b_j + 1) <= theta), the others are optional.  Levels are
visited ascending after the unconstrained one, and the scan stops once the
unconstrained knapsack value minus k * (previous level) cannot beat the best.

    python tools/reround_proto.py frag          # the seeded FRAG cases
    python tools/reround_proto.py fuzz 600      # random, widths up to G
    python tools/reround_proto.py check         # knapsack form == brute force
"""
import ctypes
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "shockwave-replication_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import milp_ref as mr  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402
from fuzzcases import fuzz_problem  # noqa: E402
from helpers import to_oracle  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "oracle/_build/libplan_twin.so"))
sn.declare_solver_api(lib, "twin_")
STATS = dict(dps=0, cells=0, rounds=0, moves=0)


def rows(a):
    N, T = a.N, a.T
    f = np.zeros((N, T + 1)); g = np.zeros((N, T + 1)); key = np.zeros((N, T), np.float32)
    dp = ctypes.POINTER(ctypes.c_double)
    lib.twin_job_rows(ctypes.byref(a.c_problem()), f.ctypes.data_as(dp), g.ctypes.data_as(dp),
                      key.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return f, g


def knap(items, w, v, cap):
    """0/1 knapsack over items in job order; strict improvement keeps the
    earlier choice; the smallest capacity reaching the maximum."""
    if cap < 0:
        return None, None
    tot = sum(w[j] for j in items)
    if tot <= cap:
        return sum(v[j] for j in items), list(items)
    STATS["dps"] += 1
    STATS["cells"] += len(items) * (cap + 1)
    dp = [0.0] * (cap + 1)
    take = []
    for j in items:
        tk = [False] * (cap + 1)
        for c in range(cap, w[j] - 1, -1):
            x = dp[c - w[j]] + v[j]
            if x > dp[c]:
                dp[c] = x
                tk[c] = True
        take.append(tk)
    c = max(range(cap + 1), key=lambda i: (dp[i], -i))
    best = dp[c]
    S = []
    for i in range(len(items) - 1, -1, -1):
        if take[i][c]:
            S.append(items[i])
            c -= w[items[i]]
    return best, S[::-1]


def best_round_set(b, elig, w, G, k, f, g):
    """Exact optimum of one round's set given the other rounds' counts b."""
    N = len(b)
    idx = np.arange(N)
    v = np.where(elig, f[idx, np.minimum(b + 1, f.shape[1] - 1)] - f[idx, b], 0.0)
    h0 = g[idx, b]
    h1 = np.where(elig, g[idx, np.minimum(b + 1, g.shape[1] - 1)], h0)
    opt_all = [j for j in range(N) if elig[j] and v[j] > 0 and w[j] <= G]
    D, S = knap(opt_all, w, v, G)

    def mk(S):
        inS = np.zeros(N, bool); inS[S] = True
        return float(np.max(np.where(inS, h1, h0))) if N else 0.0

    best = (D - k * mk(S), S)
    thetas = sorted(set(h0.tolist()) | set(h1.tolist()) | {0.0})
    prev = None
    for th in thetas:
        if prev is not None and D - k * prev <= best[0]:
            break
        prev = th
        forced = [j for j in range(N) if h0[j] > th]
        if any((not elig[j]) or h1[j] > th for j in forced):
            continue
        cap = G - sum(w[j] for j in forced)
        if cap < 0:
            continue
        opt = [j for j in opt_all if h0[j] <= th and w[j] <= cap]
        val, So = knap(opt, w, v, cap)
        S2 = sorted(forced + So)
        J2 = sum(v[j] for j in forced) + val - k * mk(S2)
        if J2 > best[0]:
            best = (J2, S2)
    return best


def reround(a, y, f, g, passes=4, brute=False):
    y = y.astype(bool).copy()
    N, T, G, k = a.N, a.T, a.G, a.k
    w = np.asarray(a.w, dtype=np.int64)
    elig = w <= G
    for _ in range(passes):
        changed = False
        for t in range(T):
            STATS["rounds"] += 1
            n = y.sum(1)
            cur = y[:, t]
            b = n - cur
            idx = np.arange(N)
            v = np.where(elig, f[idx, np.minimum(b + 1, T)] - f[idx, b], 0.0)
            h0 = g[idx, b]
            h1 = np.where(elig, g[idx, np.minimum(b + 1, T)], h0)
            Jcur = float(v[cur].sum()) - k * (float(np.max(np.where(cur, h1, h0))) if N else 0.0)
            if brute:
                bestJ, bestS = Jcur, None
                el = [j for j in range(N) if elig[j]]
                for r in range(len(el) + 1):
                    for S in itertools.combinations(el, r):
                        if w[list(S)].sum() > G:
                            continue
                        m = np.zeros(N, bool); m[list(S)] = True
                        J = float(v[m].sum()) - k * float(np.max(np.where(m, h1, h0)))
                        if J > bestJ:
                            bestJ, bestS = J, list(S)
                J2, S2 = bestJ, bestS
            else:
                J2, S2 = best_round_set(b, elig, w, G, k, f, g)
            if S2 is not None and J2 > Jcur + 1e-12 * (abs(Jcur) + 1e-300):
                m = np.zeros(N, bool); m[S2] = True
                y[:, t] = m
                changed = True
                STATS["moves"] += 1
        if not changed:
            break
    return y


def run_case(a, label, rel_gap=1e-6):
    P = to_oracle(a)
    try:
        sol = mr.plan_solve(P, rel_gap=rel_gap, time_limit=30)
    except AssertionError:
        return None
    ref = mr.evaluate_counts(P, sol.n)[0]
    pr, res = a.c_problem(), a.c_result()
    lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
    rep = res.status & sn.SW_STATUS_P1_REPACKED
    got = mr.evaluate_counts(P, a.plan.sum(1))[0]
    g0 = (ref - got) / abs(ref) if ref else 0.0
    g1 = g0
    if rep:
        f, gg = rows(a)
        y = reround(a, a.plan, f, gg)
        assert mr.check_plan(P, y.astype(int))
        g1 = (ref - mr.evaluate_counts(P, y.sum(1))[0]) / abs(ref) if ref else 0.0
    return g0, g1, rep


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "frag"
    if mode == "check":  # knapsack form == brute force on small rounds
        for s in range(40):
            a = ss.synth_problem(s, 9, 8, 5, 120.0, [1.0, 1e-3, 1e5][s % 3], 5.0,
                                 width_p=(0.4, 0.3, 0.2, 0.1))
            pr, res = a.c_problem(), a.c_result()
            lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
            f, g = rows(a)
            y1 = reround(a, a.plan, f, g, passes=1)
            y2 = reround(a, a.plan, f, g, passes=1, brute=True)
            P = to_oracle(a)
            J1 = mr.evaluate_counts(P, y1.sum(1))[0]
            J2 = mr.evaluate_counts(P, y2.sum(1))[0]
            assert abs(J1 - J2) <= 1e-9 * abs(J2), (s, J1, J2)
        print("knapsack form == brute force on 40 cases")
        return
    if mode == "frag":
        cases = [(s, N, G, k) for s in range(6) for (N, G) in ((8, 8), (12, 8), (10, 12), (14, 15))
                 for k in (1.0, 1e-3)] + [(10, 8, 8, 1.0), (10, 8, 8, 1e5), (1, 12, 8, 1e-3)]
        probs = [(f"s{s}_N{N}_G{G}_k{k:g}",
                  ss.synth_problem(s, N, G, 6, 120.0, k, 5.0, width_p=(0.4, 0.3, 0.2, 0.1)))
                 for s, N, G, k in cases]
    else:
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 600
        probs = []
        s = 0
        while len(probs) < n:
            b = fuzz_problem(50_000 + s, max_n=80, trace_widths=(mode == "fuzztrace"))
            s += 1
            if b.G < 1:
                continue
            probs.append((f"fz{50_000 + s - 1}",
                          sn.ProblemArrays(b.w, b.d, b.F, b.E, b.R, b.p, min(b.T, 12), b.G,
                                           b.delta, b.k, tuple(b.bases))))
    over0 = over1 = nrep = unsolved = 0
    worst0 = worst1 = 0.0
    for label, a in probs:
        r = run_case(a, label)
        if r is None:
            unsolved += 1
            continue
        g0, g1, rep = r
        nrep += bool(rep)
        over0 += g0 > 1e-3
        over1 += g1 > 1e-3
        worst0, worst1 = max(worst0, g0), max(worst1, g1)
        if g0 > 1e-3 or g1 > 1e-3:
            print(f"{label} N={a.N} G={a.G} T={a.T} k={a.k:.3g} maxw={a.w.max()} "
                  f"gap {g0:.3g} -> {g1:.3g}", flush=True)
    print(f"{len(probs)} cases ({unsolved} unsolved by HiGHS), {nrep} repacked; "
          f"above 1e-3: {over0} -> {over1}; worst {worst0:.3g} -> {worst1:.3g}; {STATS}")


if __name__ == "__main__":
    main()
