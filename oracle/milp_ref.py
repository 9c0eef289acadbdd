"""oracle/milp_ref.py — TEST INFRASTRUCTURE (the reference oracle).

CPU restatement of the reference Shockwave plan solve, model for model, as
mixed-integer programs solved with HiGHS (``scipy.optimize.milp``, scipy
1.15.3) instead of CVXPY + Gurobi.  Only tests/, ``__graft_entry__.smoke()``
and bench.py's ``cpu_baseline`` leg may import this module; the product path
never does.

Parity status: **unpinned**.  The reference solve cannot run in this image
(``import shockwave`` → ModuleNotFoundError: cvxpy; gurobipy absent, no
licence) and the reference tests contain no Shockwave case (SURVEY.md §4,
§8c).  This restatement is cross-checked instead against exhaustive
enumeration of the same model on tiny instances (tests/test_oracle.py) and
its inputs come from the reference's own estimators (tests/golden/).

Line map (reference scheduler/shockwave.py):
  P1  _eisenberg_gale_program                     :330-388
      x[j][t] boolean, Σ_j w_j x[j][t] ≤ G        :45-75
      e_j ≥ 0, d_j e_j ≤ Δ Σ_t x[j][t]            :114, :122-129
      SOS2 boundaries / adjacency / weights        :162-179
      L_j = Σ_b ω_jb ℓ_b, ℓ_b = log(max(β_b,1e-6)) :99-105, :180
      makespan_j = max(0, R_j − d_j e_j)           :260-263
      maximize Σ p_j L_j/(N·T) − k·max_j makespan_j :363-379
  P2  _prioritize_unfair_jobs                      :281-328
      Σ_t y[j][t] = n_j (P1's planned rounds)      :294-303
      capacity                                     :306
      minimize Σ_{n_j>0} p_j (Σ_t t·y[j][t]) / n_j  :309-322
      no planned job → keep P1 x                   :319-320
      no P2 solution → keep P1 x                   :325-326
  solver options MIPGap / TimeLimit                :400-411
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
from scipy.optimize import LinearConstraint, milp


def log_bases(bases):
    """shockwave.py:99-105 — log of each breakpoint, log(0) replaced by log(1e-6)."""
    return [math.log(1e-6) if b == 0.0 else math.log(b) for b in bases]


@dataclass
class Problem:
    """The numbers the reference feeds into P1/P2 (see include/shockwave_amd.h)."""

    w: np.ndarray  # int, nworkers
    d: np.ndarray  # float, interpolated epoch duration
    F: np.ndarray  # int, completed epochs
    E: np.ndarray  # int, total epochs
    R: np.ndarray  # float, remaining runtime (call #2)
    p: np.ndarray  # float, priority FTF**lambda
    T: int
    G: int
    delta: float
    k: float
    bases: list = field(default_factory=lambda: [0.0, 0.2, 0.4, 0.6, 0.8, 1.0])

    @property
    def N(self):
        return int(len(self.w))


@dataclass
class Solution:
    status: str
    x: np.ndarray  # P1 plan [N][T] 0/1
    n: np.ndarray  # planned rounds per job
    objective: float  # P1 objective as reported by the solver
    bound: float  # P1 dual (upper) bound
    y: np.ndarray  # final plan after P2 (or P1 fallback)
    p2_objective: float
    p2_status: str
    seconds_p1: float
    seconds_p2: float


def _lp_status(res):
    return {0: "optimal", 1: "time_limit", 2: "infeasible", 3: "unbounded", 4: "other"}.get(
        res.status, str(res.status)
    )


def build_p1(prob: Problem, utility_weight=1.0, makespan_weight=None, makespan_cap=None):
    """Assemble P1 exactly as shockwave.py:330-379 (SOS2 formulation of :162-179).

    The defaults give the reference model.  The stage problems of the
    utility-term parity checks reuse the same rows:
    ``utility_weight=0, makespan_weight=1`` minimises the makespan alone;
    ``makespan_weight=0, makespan_cap=M`` maximises the utility term with every
    job's makespan ≤ M.
    """
    N, T, B = prob.N, prob.T, len(prob.bases)
    ell = log_bases(prob.bases)
    beta = list(prob.bases)
    nx, ne, nz, na, nw, nt = N * T, N, N * B, N * (B - 1), N * B, N
    ox = 0
    oe = ox + nx
    oz = oe + ne
    oa = oz + nz
    ow = oa + na
    ot = ow + nw
    oM = ot + nt
    nv = oM + 1
    c = np.zeros(nv)
    integ = np.zeros(nv)
    integ[ox:ox + nx] = 1
    integ[oz:oz + nz] = 1
    integ[oa:oa + na] = 1
    lb = np.zeros(nv)
    ub = np.full(nv, np.inf)
    ub[ox:ox + nx] = 1
    ub[oz:oz + nz] = 1
    ub[oa:oa + na] = 1
    lb[oM] = -np.inf
    if makespan_cap is not None:
        ub[oM] = float(makespan_cap)
    NT = float(N * T)
    for j in range(N):
        for b in range(B):
            # minimise −(p_j ℓ_b / (N·T)) ω_jb
            c[ow + j * B + b] = -utility_weight * (prob.p[j] * ell[b]) / NT
    c[oM] = prob.k if makespan_weight is None else float(makespan_weight)
    rows, cols, vals, rlo, rhi = [], [], [], [], []
    r = 0

    def add(coefs, lo, hi):
        nonlocal r
        for col, v in coefs:
            rows.append(r)
            cols.append(col)
            vals.append(v)
        rlo.append(lo)
        rhi.append(hi)
        r += 1

    # per-round capacity  (shockwave.py:64-75)
    for t in range(T):
        add([(ox + j * T + t, float(prob.w[j])) for j in range(N)], -np.inf, float(prob.G))
    for j in range(N):
        zj = oz + j * B
        aj = oa + j * (B - 1)
        wj = ow + j * B
        # Σ boundaries == 2 (:164)
        add([(zj + b, 1.0) for b in range(B)], 2.0, 2.0)
        for i in range(B - 1):
            # adjacent[i] >= b[i] + b[i+1] − 1 ; adjacent[i] <= b[i], b[i+1]  (:167-170)
            add([(zj + i, 1.0), (zj + i + 1, 1.0), (aj + i, -1.0)], -np.inf, 1.0)
            add([(aj + i, 1.0), (zj + i, -1.0)], -np.inf, 0.0)
            add([(aj + i, 1.0), (zj + i + 1, -1.0)], -np.inf, 0.0)
        # Σ adjacent == 1 (:172)
        add([(aj + i, 1.0) for i in range(B - 1)], 1.0, 1.0)
        # Σ ω == 1 (:174)
        add([(wj + b, 1.0) for b in range(B)], 1.0, 1.0)
        # ω <= boundaries (:176, added B times in the reference; once suffices)
        for b in range(B):
            add([(wj + b, 1.0), (zj + b, -1.0)], -np.inf, 0.0)
        # Σ ω β == (F + e) / E  (:132-134, :177-179)
        E = float(prob.E[j])
        coefs = [(wj + b, beta[b]) for b in range(B) if beta[b] != 0.0]
        coefs.append((oe + j, -1.0 / E))
        add(coefs, float(prob.F[j]) / E, float(prob.F[j]) / E)
        # d e ≤ Δ Σ_t x  (:126-129)
        coefs = [(oe + j, float(prob.d[j]))] + [(ox + j * T + t, -prob.delta) for t in range(T)]
        add(coefs, -np.inf, 0.0)
        # makespan_j = max(0, R − d e) → t_j ≥ R − d e, t_j ≥ 0  (:260-263)
        add([(ot + j, 1.0), (oe + j, float(prob.d[j]))], float(prob.R[j]), np.inf)
        # M ≥ t_j  (cp.max, :363)
        add([(oM, 1.0), (ot + j, -1.0)], 0.0, np.inf)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(r, nv))
    layout = dict(ox=ox, oe=oe, oM=oM, nv=nv)
    return c, integ, (lb, ub), LinearConstraint(A, np.array(rlo), np.array(rhi)), layout


def solve_p1(prob: Problem, rel_gap=1e-3, time_limit=15.0, relax=False, **variant):
    """P1 (shockwave.py:330-382) with HiGHS; ``variant`` as build_p1.  Returns
    (status, x values, objective, dual bound, seconds) in the maximisation
    sense of the built objective; relax=True solves the LP relaxation (every
    binary in [0, 1]), whose optimum is an upper bound of the MILP."""
    c, integ, (lb, ub), cons, lay = build_p1(prob, **variant)
    from scipy.optimize import Bounds

    opts = {"disp": False, "time_limit": float(time_limit)}
    if not relax:
        opts["mip_rel_gap"] = float(rel_gap)
    t0 = time.perf_counter()
    res = milp(c, integrality=(np.zeros_like(integ) if relax else integ), bounds=Bounds(lb, ub),
               constraints=[cons], options=opts)
    dt = time.perf_counter() - t0
    if res.x is None:
        raise AssertionError(f"P1 has no solution (status {_lp_status(res)})")  # shockwave.py:382
    N, T = prob.N, prob.T
    xv = res.x[lay["ox"]:lay["ox"] + N * T].reshape(N, T)
    obj = -float(res.fun)
    bound = -float(getattr(res, "mip_dual_bound", res.fun) if not relax else res.fun)
    return _lp_status(res), xv, obj, bound, dt


def solve_p2(prob: Problem, n_planned, time_limit=15.0, rel_gap=1e-3):
    """shockwave.py:281-328 (returns None when the reference would keep P1's x)."""
    N, T = prob.N, prob.T
    if not any(n_planned[j] > 0 for j in range(N)):
        return None, "no_planned", 0.0, 0.0  # :319-320
    nv = N * T
    c = np.zeros(nv)
    for j in range(N):
        if n_planned[j] > 0:
            for t in range(T):
                c[j * T + t] = prob.p[j] * t / float(n_planned[j])
    rows, cols, vals, rlo, rhi = [], [], [], [], []
    r = 0
    for j in range(N):
        for t in range(T):
            rows.append(r); cols.append(j * T + t); vals.append(1.0)
        rlo.append(float(n_planned[j])); rhi.append(float(n_planned[j])); r += 1
    for t in range(T):
        for j in range(N):
            rows.append(r); cols.append(j * T + t); vals.append(float(prob.w[j]))
        rlo.append(-np.inf); rhi.append(float(prob.G)); r += 1
    A = sp.csr_matrix((vals, (rows, cols)), shape=(r, nv))
    from scipy.optimize import Bounds

    t0 = time.perf_counter()
    res = milp(c, integrality=np.ones(nv), bounds=Bounds(np.zeros(nv), np.ones(nv)),
               constraints=[LinearConstraint(A, np.array(rlo), np.array(rhi))],
               options={"disp": False, "time_limit": float(time_limit), "mip_rel_gap": float(rel_gap)})
    dt = time.perf_counter() - t0
    if res.x is None:
        return None, _lp_status(res), 0.0, dt  # :325-326
    return np.rint(res.x).reshape(N, T).astype(np.uint8), _lp_status(res), float(res.fun), dt


def plan_solve(prob: Problem, rel_gap=1e-3, time_limit=15.0) -> Solution:
    """One full reference plan solve: P1 → P2 → schedule (shockwave.py:330-398)."""
    st, xv, obj, bound, t1 = solve_p1(prob, rel_gap, time_limit)
    x = (xv > 0.5).astype(np.uint8)
    n = x.sum(axis=1).astype(np.int64)
    y, st2, p2obj, t2 = solve_p2(prob, n, time_limit, rel_gap)
    if y is None:
        y = x
    return Solution(st, x, n, obj, bound, y, p2obj, st2, t1, t2)


# ---------------------------------------------------------------------------
# Independent evaluation of the P1 objective for a given plan (closed form of
# the optimal e_j, ω for fixed x; used to compare plans from any solver).
# ---------------------------------------------------------------------------
def phi(u, bases):
    ell = log_bases(bases)
    B = len(bases)
    for b in range(B - 1):
        if u <= bases[b + 1] or b == B - 2:
            t = (u - bases[b]) / (bases[b + 1] - bases[b])
            return ell[b] + (ell[b + 1] - ell[b]) * t
    raise ValueError(u)


def evaluate_counts(prob: Problem, n):
    """(objective, utility, makespan) of planned-round counts n under P1."""
    N, T = prob.N, prob.T
    util = 0.0
    mk = 0.0
    for j in range(N):
        e = min(prob.delta * float(n[j]) / float(prob.d[j]), float(prob.E[j] - prob.F[j]))
        u = (float(prob.F[j]) + e) / float(prob.E[j])
        util += prob.p[j] * phi(u, prob.bases) / float(N * T)
        mk = max(mk, max(0.0, float(prob.R[j]) - float(prob.d[j]) * e))
    return util - prob.k * mk, util, mk


def p2_objective(prob: Problem, y):
    n = y.sum(axis=1)
    tt = np.arange(prob.T)
    return float(sum(prob.p[j] * float(y[j] @ tt) / float(n[j]) for j in range(prob.N) if n[j] > 0))


def check_plan(prob: Problem, y):
    """Feasibility of a 0/1 plan: per-round capacity (shockwave.py:64-75)."""
    y = np.asarray(y)
    load = (y * np.asarray(prob.w)[:, None]).sum(axis=0)
    return bool(np.all(load <= prob.G)) and y.shape == (prob.N, prob.T)


def brute_force_p1(prob: Problem):
    """Exhaustive optimum of P1 over every 0/1 x (tiny N·T only)."""
    N, T = prob.N, prob.T
    assert N * T <= 16
    best = (-math.inf, None)
    for mask in range(1 << (N * T)):
        x = np.array([(mask >> i) & 1 for i in range(N * T)], dtype=np.int64).reshape(N, T)
        if not check_plan(prob, x):
            continue
        obj, _, _ = evaluate_counts(prob, x.sum(axis=1))
        if obj > best[0]:
            best = (obj, x)
    return best


class MilpSolver:
    """ShockwaveScheduler's solver interface (``solve(ProblemArrays) -> dict``)
    backed by the MILP restatement — the reference's solve path (P1 → P2 →
    read-back, shockwave.py:330-411) with HiGHS in place of Gurobi.  Used by
    the simulator-parity tests and tools/sim_parity.py as the oracle run."""

    def __init__(self, rel_gap=1e-3, time_limit=15.0, perm_seed=None):
        """perm_seed: solve every model with its jobs in a seeded random order
        (the same problem; HiGHS then walks a different path and may stop at a
        different solution inside the gap) — samples the oracle's own
        indeterminacy at a given gap."""
        self.rel_gap = rel_gap
        self.time_limit = time_limit
        self.perm_seed = perm_seed
        self.seconds = 0.0
        self.calls = 0

    def solve(self, arrays):
        perm = np.arange(arrays.N)
        if self.perm_seed is not None:
            perm = np.random.default_rng([self.perm_seed, self.calls]).permutation(arrays.N)
        prob = Problem(arrays.w[perm], arrays.d[perm], arrays.F[perm], arrays.E[perm],
                       arrays.R[perm], arrays.p[perm], arrays.T, arrays.G, arrays.delta,
                       arrays.k, list(arrays.bases))
        t0 = time.perf_counter()
        sol = plan_solve(prob, self.rel_gap, self.time_limit)
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        y = np.empty_like(sol.y)
        y[perm] = sol.y
        y = y.astype(np.uint8)
        return {"rc": 0 if sol.p2_status in ("optimal", "no_planned", "time_limit") else 1,
                "plan": y, "planned_rounds": y.sum(axis=1).astype(np.int32),
                "objective": sol.objective, "utility": float("nan"), "makespan": float("nan"),
                "p2_objective": sol.p2_objective, "bound": sol.bound, "iters": 0, "status": 0}
