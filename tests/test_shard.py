"""Sharded single-instance solve (include/shockwave_amd.h sw_dist_*).

The controller (csrc/sw_shard_ctl.h) runs here on the CPU shard engine
(oracle/shard_twin.c) with W ranks as threads (a barrier-based allgather) and,
for the multi-process path, as W=2 processes over torch.distributed gloo.

The contract.  The CPU shard engine is the specification the
GPU engine (csrc/sw_shard.hip) matches bit for bit at every world size
(tests/test_gpu_shard.py).  The placement runs in V = sw_share_count(N, G, W)
shares (each placed alone in its share of every round, sw_share_caps): V = W,
except for large instances (≥ 4,096 jobs on ≥ 512 GPUs), which take V = 8 at
every W ≤ 8.  Against the single-instance solve (the twin, oracle/plan_twin.c,
= the GPU plan kernel):
  * V = 1 (W = 1, not large): the same result, bit for bit (plan rows, counts,
    every objective);
  * V > 1: the plan rows and the P2 objective depend on V (not on W: a large
    instance gives the same result at W = 1, 2, 4, 8); P1 — counts,
    objective, utility, makespan, bound and the P1 status bits — is the
    single-instance solve's bit for bit (the same level search, every count
    placed), or better when only the shares could place the level search's
    counts; P2 stays within SHARE_P2_RATIO of the single instance's.  Only
    `iters` differs at every W (it counts collective steps).
"""
import ctypes
import os
import threading

import numpy as np
import pytest

import sw_native as sn
import sw_synth as ss
from conftest import TWIN_SO, _build_twin
from helpers import check_plan_valid

SCALARS = ("objective", "utility", "makespan", "p2_objective", "bound")


class ThreadGroup:
    """W ranks as threads of this process: allgather through shared slots."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world

    def member(self, rank):
        group = self

        class Member:
            def allgather_bytes(self, data):
                group.slots[rank] = data
                group.barrier.wait()
                out = list(group.slots)
                group.barrier.wait()
                return out

        return Member()


@pytest.fixture(scope="module")
def shard_lib():
    _build_twin()
    lib = ctypes.CDLL(TWIN_SO)
    lib.shard_twin_solve.argtypes = [ctypes.POINTER(sn.SwHostComm), ctypes.c_int32, ctypes.c_int32,
                                     ctypes.POINTER(sn.SwProblem), ctypes.c_int64, ctypes.c_int64,
                                     ctypes.POINTER(sn.SwResult)]
    lib.shard_twin_solve.restype = ctypes.c_int
    return lib


def shard_solve_rank(lib, comm, rank, world, a):
    lo, hi = sn.shard_range(a.N, world, rank)
    loc = a.slice(lo, hi)
    pr, res = loc.c_problem(), loc.c_result()
    rc = lib.shard_twin_solve(ctypes.byref(comm.c), rank, world, ctypes.byref(pr), lo, a.N,
                              ctypes.byref(res))
    return lo, hi, sn.result_dict(res, loc, rc)


def run_threads(lib, a, world):
    group = ThreadGroup(world)
    out = [None] * world
    errs = []

    def work(r):
        try:
            comm = sn.HostComm(group.member(r))
            out[r] = shard_solve_rank(lib, comm, r, world, a)
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)
            group.barrier.abort()

    ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs, errs
    return assemble(a, out)


def assemble(a, parts):
    plan = np.zeros((a.N, a.T), np.uint8)
    cnt = np.zeros(a.N, np.int32)
    r0 = parts[0][2]
    for lo, hi, r in parts:
        assert r["rc"] >= 0, r["rc"]
        for key in SCALARS + ("status", "rc", "iters"):
            assert np.float64(r[key]).tobytes() == np.float64(r0[key]).tobytes(), key
        plan[lo:hi] = r["plan"]
        cnt[lo:hi] = r["planned_rounds"]
    return dict(r0, plan=plan, planned_rounds=cnt)


P1_BITS = sn.SW_STATUS_P1_REPACKED | sn.SW_STATUS_NO_PLANNED | sn.SW_STATUS_P1_UNCERTIFIED
# the share placement's P2 against the single instance's (both after the
# exchange step), and against the HiGHS optimum of the reference P2 MILP on
# the large fixtures: worst measured 1.00196 (case N1500 at W = 8) and
# 1.00158 (the 3,000-job fixture at W = 8) — the reference's own P2 gap is
# 1e-3 (shockwave.py:405), so 1.002 is its bar plus the measured margin
SHARE_P2_RATIO = 1.002


def assert_share_contract(rs, rt, what):
    """W > 1 against the single-instance result rt (the module docstring)."""
    assert rs["rc"] >= 0, what
    if (rs["status"] & P1_BITS) == (rt["status"] & P1_BITS):
        assert np.array_equal(rs["planned_rounds"], rt["planned_rounds"]), f"{what}: counts"
        for key in ("objective", "utility", "makespan", "bound"):
            assert np.float64(rs[key]).tobytes() == np.float64(rt[key]).tobytes(), \
                f"{what}: {key} {rs[key]!r} vs {rt[key]!r}"
        if rt["p2_objective"] > 0:
            assert rs["p2_objective"] <= rt["p2_objective"] * SHARE_P2_RATIO, \
                (what, rs["p2_objective"], rt["p2_objective"])
    else:  # the shares placed the level search's counts, the gathered orders could not
        assert rt["status"] & sn.SW_STATUS_P1_REPACKED and not rs["status"] & sn.SW_STATUS_P1_REPACKED, what
        assert rs["objective"] >= rt["objective"], what


def share_count(N, G, world):
    """sw_share_count (csrc/sw_shard_ctl.h)."""
    return 8 if world < 8 and 4096 <= N <= 65536 and G >= 512 else world


def assert_contract(rs, rt, world, what, N=0, G=0):
    if share_count(N, G, world) == 1:
        assert_same_as_single(rs, rt, what)
    else:
        assert_share_contract(rs, rt, what)


def assert_same_as_single(rs, rt, what):
    assert rs["status"] == rt["status"], what
    assert rs["rc"] == rt["rc"], what
    assert np.array_equal(rs["planned_rounds"], rt["planned_rounds"]), f"{what}: counts"
    assert np.array_equal(rs["plan"], rt["plan"]), f"{what}: plan"
    for key in SCALARS:
        assert np.float64(rs[key]).tobytes() == np.float64(rt[key]).tobytes(), \
            f"{what}: {key} {rs[key]!r} vs {rt[key]!r}"


CASES = [
    # (seed, N, G, T, k, lam)
    (0, 12, 4, 6, 1e5, 5.0),
    (1, 50, 32, 20, 1e-3, 15.0),
    (2, 120, 64, 20, 1e-3, 15.0),
    (3, 120, 128, 20, 1e1, 5.0),
    (4, 300, 64, 64, 1e1, 5.0),
    (5, 200, 32, 40, 0.5, 3.0),
    (6, 900, 256, 30, 1e5, 5.0),
    (7, 1500, 400, 30, 1e5, 5.0),
    (8, 40, 8, 10, 0.0, 5.0),
    (9, 30, 6, 12, 1e2, 5.0),
]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("case", CASES, ids=[f"N{c[1]}_G{c[2]}_T{c[3]}_k{c[4]:g}" for c in CASES])
def test_sharded_vs_single(case, world, shard_lib, twin):
    seed, N, G, T, k, lam = case
    a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
    rs = run_threads(shard_lib, a, world)
    rt = twin.solve(a)
    check_plan_valid(a, rs)
    assert_contract(rs, rt, world, f"W={world} case {case}", N, G)


def test_sharded_edge_cases(shard_lib, twin):
    # empty instance; jobs wider than the cluster; one job; all-equal jobs (ties)
    a0 = ss.synth_problem(1, 0, 8, 5, 120.0, 1e5, 5.0)
    rs = run_threads(shard_lib, a0, 2)
    assert rs["status"] & sn.SW_STATUS_NO_PLANNED
    a = ss.synth_problem(2, 64, 4, 10, 120.0, 1e2, 5.0)
    a.w[::3] = 8  # wider than G=4: never schedulable
    assert_share_contract(run_threads(shard_lib, a, 4), twin.solve(a), "wide jobs")
    a1 = ss.synth_problem(3, 1, 8, 5, 120.0, 1e5, 5.0)
    assert_share_contract(run_threads(shard_lib, a1, 8), twin.solve(a1), "one job")
    at = ss.synth_problem(4, 96, 16, 8, 120.0, 1e1, 5.0)
    for arr in (at.w, at.d, at.F, at.E, at.R, at.p):
        arr[:] = arr[0]
    assert_share_contract(run_threads(shard_lib, at, 4), twin.solve(at), "ties")


def test_shard_range_rule():
    for N in (0, 1, 511, 512, 513, 10_000):
        for W in (1, 2, 8, 512):
            spans = [sn.shard_range(N, W, r) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == N
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
    with pytest.raises(ValueError):
        sn.shard_range(100, 3, 0)


def test_shard_rejects_wrong_slice(shard_lib):
    a = ss.synth_problem(0, 100, 32, 10, 120.0, 1e5, 5.0)
    group = ThreadGroup(1)
    comm = sn.HostComm(group.member(0))
    loc = a.slice(0, 50)  # W=1 must hold every job
    pr, res = loc.c_problem(), loc.c_result()
    rc = shard_lib.shard_twin_solve(ctypes.byref(comm.c), 0, 1, ctypes.byref(pr), 0, a.N,
                                    ctypes.byref(res))
    assert rc == sn.SW_ERR_INVALID


# ---- multi-process: world_size 2 over torch.distributed gloo ----------------

def _gloo_worker(rank, world, port, outdir, cases):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = ctypes.CDLL(TWIN_SO)
    lib.shard_twin_solve.argtypes = [ctypes.POINTER(sn.SwHostComm), ctypes.c_int32, ctypes.c_int32,
                                     ctypes.POINTER(sn.SwProblem), ctypes.c_int64, ctypes.c_int64,
                                     ctypes.POINTER(sn.SwResult)]
    lib.shard_twin_solve.restype = ctypes.c_int
    comm = sn.HostComm(sn.TorchGroupComm())
    for ci, case in enumerate(cases):
        seed, N, G, T, k, lam = case
        a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
        lo, hi, r = shard_solve_rank(lib, comm, rank, world, a)
        np.savez(os.path.join(outdir, f"c{ci}_r{rank}.npz"), lo=lo, hi=hi, plan=r["plan"],
                 cnt=r["planned_rounds"],
                 scal=np.array([r[k] for k in SCALARS], dtype=np.float64),
                 meta=np.array([r["rc"], r["status"], r["iters"]], dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_gloo_world2(tmp_path, shard_lib, twin):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cases = [CASES[1], CASES[6], CASES[7]]
    mp.spawn(_gloo_worker, args=(2, port, str(tmp_path), cases), nprocs=2, join=True)
    for ci, case in enumerate(cases):
        seed, N, G, T, k, lam = case
        a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
        parts = []
        for r in range(2):
            z = np.load(tmp_path / f"c{ci}_r{r}.npz")
            res = {key: float(v) for key, v in zip(SCALARS, z["scal"])}
            res.update(rc=int(z["meta"][0]), status=int(z["meta"][1]), iters=int(z["meta"][2]),
                       plan=z["plan"], planned_rounds=z["cnt"])
            parts.append((int(z["lo"]), int(z["hi"]), res))
        rs = assemble(a, parts)
        # processes over gloo = threads in one process: the same engine, bit for bit
        assert_same_as_single(rs, run_threads(shard_lib, a, 2), f"gloo case {case}")
        assert_share_contract(rs, twin.solve(a), f"gloo case {case}")


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_fuzz_vs_single(world, shard_lib, twin):
    """The fuzz instances of tests/fuzzcases.py (validator-range inputs, exact
    duplicate jobs, finished jobs, zero priorities, custom base grids)."""
    from fuzzcases import fuzz_problem

    for s in range(0, 48):
        a = fuzz_problem(s)
        rs = run_threads(shard_lib, a, world)
        check_plan_valid(a, rs)
        assert_contract(rs, twin.solve(a), world, f"W={world} fuzz seed {s}", a.N, a.G)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_pattern_placement_equals_single(world, shard_lib, twin):
    """Frag-fuzz instances whose level-search counts only the round-pattern
    search places (sw_profile_search: 50115 with widths {1, 2, 4, 8} on 13
    GPUs, 50417, 50439) or that the branch and bound changes (50104, 12 width
    classes), and 50169, where a raise (one more round for a width-6 job, the
    plan re-placed; sw_arith.h SW_RAISE_ITERS) closes a 0.52 gap: the
    controller's pattern step gathers the classes' count histograms
    (class_caps, SW_CLASS_HIST) and runs the same search."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_frag_fuzz as mk

    for s in (50115, 50417, 50439, 50104, 50169):
        a = mk.instance(s)
        rs = run_threads(shard_lib, a, world)
        check_plan_valid(a, rs)
        rt = twin.solve(a)
        assert_contract(rs, rt, world, f"W={world} frag seed {s}", a.N, a.G)
        if s == 50115:
            assert not rt["status"] & sn.SW_STATUS_P1_REPACKED  # placed as counted


@pytest.mark.parametrize("world", [2, 4, 8])
def test_share_p2_vs_milp_on_large_instances(world, shard_lib, twin):
    """The share placement's P2 at 3,000 and 5,000 jobs (C4-shaped) against
    the HiGHS optimum of the reference P2 MILP on the same counts
    (tests/golden/p2_share.json): the counts are the single instance's, and
    the P2 objective stays within SHARE_P2_RATIO of the optimum."""
    import json

    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "p2_share.json")))["cases"]
    for c in gold:
        a = ss.synth_problem(c["seed"], c["N"], c["G"], c["T"], 120.0, c["k"], c["lam"])
        rs = run_threads(shard_lib, a, world)
        check_plan_valid(a, rs)
        assert np.array_equal(rs["planned_rounds"], np.asarray(c["counts"], np.int32))
        assert rs["p2_objective"] <= c["p2_milp"] * SHARE_P2_RATIO, \
            (c["N"], world, rs["p2_objective"] / c["p2_milp"])
        assert_share_contract(rs, twin.solve(a), f"N={c['N']} W={world}")


def _share_caps_ref(loads, W, rank, T, G):
    """sw_share_caps restated in exact integers."""
    L = sum(loads)
    C = G * T
    if L <= 0 or L > C or T < 1:
        return None
    S = C - L
    rest = S - sum(S * x // L for x in loads)
    B = [loads[r] + S * loads[r] // L + (1 if r < rest else 0) for r in range(W)]
    cursor = sum(b % T for b in B[:rank]) % T
    base, ext = divmod(B[rank], T)
    return [base + (1 if (t - cursor) % T < ext else 0) for t in range(T)], B[rank]


def test_share_caps_properties(shard_lib):
    """Every round's shares sum to G; rank r's shares sum to its budget
    B_r ≥ its load and differ by at most one across rounds; world 1 is G in
    every round; an empty or over-full load is refused."""
    import ctypes

    f = shard_lib.shard_share_caps
    f.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                  ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]
    f.restype = ctypes.c_int
    rng = np.random.default_rng(7)

    def caps_of(loads, W, r, T, G):
        ld = np.ascontiguousarray(loads, dtype=np.int64)
        out = np.zeros(T, dtype=np.int32)
        rc = f(ld.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), W, r, T, G,
               out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return rc, out

    for _ in range(300):
        W = int(rng.choice([1, 2, 4, 8, 16]))
        T = int(rng.integers(1, 65))
        G = int(rng.integers(1, 5000))
        loads = rng.integers(0, G * T // W + 1, size=W)
        if loads.sum() == 0:
            loads[0] = 1
        rows = []
        for r in range(W):
            rc, caps = caps_of(loads, W, r, T, G)
            ref = _share_caps_ref([int(x) for x in loads], W, r, T, G)
            assert rc == 0 and ref is not None
            assert caps.tolist() == ref[0], (W, r, T, G)
            assert int(caps.sum()) == ref[1] >= int(loads[r])
            assert caps.max() - caps.min() <= 1
            rows.append(caps)
        assert (np.sum(rows, axis=0) == G).all()
        if W == 1:
            assert (rows[0] == G).all()
    assert caps_of([0, 0], 2, 0, 4, 10)[0] == -1
    assert caps_of([30, 11], 2, 0, 4, 10)[0] == -1


def test_large_instance_same_at_every_world(shard_lib, twin):
    """A large instance (5,000 jobs on 1,424 GPUs: V = 8 shares at every
    W ≤ 8) gives one result at W = 1, 2, 4, 8 — plan rows, counts and every
    objective bit for bit; at W = 16 (V = W) the shares are its own."""
    a = ss.synth_problem(11, 5000, 1424, 30, 120.0, 1e5, 5.0)
    r1 = run_threads(shard_lib, a, 1)
    check_plan_valid(a, r1)
    assert_share_contract(r1, twin.solve(a), "W=1 large")
    for world in (2, 4, 8):
        assert_same_as_single(run_threads(shard_lib, a, world), r1, f"W={world} vs W=1")
    r16 = run_threads(shard_lib, a, 16)
    check_plan_valid(a, r16)
    assert_share_contract(r16, twin.solve(a), "W=16 large")


def test_search_resolve_matches_brute_force(shard_lib):
    """The gathered step of the sharded searches (sw_search_resolve,
    DESIGN.md §7.2): the smallest x in [lo, hi) with chi + Σ_{v_i > x} w_i ≤
    bud, else hi — against a scan over every x of small brackets, with ties,
    items at both ends and budgets on either side of every partial sum."""
    fn = shard_lib.shard_search_resolve
    fn.restype = ctypes.c_uint64
    fn.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                   ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
    rng = np.random.default_rng(7)
    for _ in range(400):
        lo = int(rng.integers(0, 1 << 40))
        span = int(rng.integers(1, 40))
        hi = lo + span
        n = int(rng.integers(0, 12))
        v = np.sort(rng.integers(lo, hi + 1, size=n)).astype(np.uint64)
        w = rng.integers(1, 6, size=n).astype(np.int64)
        chi = int(rng.integers(0, 4))
        tot = chi + int(w.sum())
        for bud in range(max(0, chi - 1), tot + 2):
            want = hi
            for x in range(lo, hi):
                if chi + int(w[v > x].sum()) <= bud:
                    want = x
                    break
            got = fn(lo, hi, chi, bud, v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                     w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n)
            assert got == want, (lo, hi, chi, bud, v.tolist(), w.tolist(), got, want)
