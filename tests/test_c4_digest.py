"""The committed C4 digests (tests/golden/c4_digest.json) that bench.py's
c4_sharded sub-record checks at every N are the CPU solves of that instance —
the twin's single-instance solve (top level) and the CPU shard engine's at
worlds 1, 2, 4, 8 (by_world; DESIGN.md §7.2: the C4 instance is placed in
SW_VSHARES = 8 shares at every world size, so the four are one digest) — so a
stale digest fails here, on the CPU, before a GPU run; and on the GPU the
RCCL-sharded engine at world 1 reproduces the world-1 digest."""
import hashlib
import json
import os

import numpy as np
import pytest

import sw_synth as ss

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                   "c4_digest.json")))
# The LP relaxation of the reference P1 (shockwave.py:330-382, binaries relaxed
# to [0, 1]) on the same instance, solved once by HiGHS
# (tests/golden/make_c4_lp.py): an upper bound on every integer plan's J.
LP = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c4_lp.json")))


def c4():
    c = ss.C4
    return ss.synth_problem(GOLD["seed"], c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])


def digest(plan, counts):
    return (hashlib.sha256(np.ascontiguousarray(plan).tobytes()).hexdigest()[:32],
            hashlib.sha256(np.ascontiguousarray(counts, dtype=np.int32).tobytes()).hexdigest()[:32])


def inputs_sha(a):
    h = hashlib.sha256()
    for arr in (a.w, a.d, a.F, a.E, a.R, a.p):
        h.update(np.ascontiguousarray(arr).tobytes())
    return h.hexdigest()[:32]


def check_lp_bound(J):
    """(LP − J) / |J| ≤ 1e-3: the LP relaxation certifies the C4 objective to
    the north star's tolerance (and J never exceeds the bound)."""
    assert LP["lp_status"] == "optimal"
    gap = (LP["lp_bound"] - J) / abs(J)
    assert -1e-9 <= gap <= 1e-3, (J, LP["lp_bound"], gap)


def test_c4_digest_is_the_twin_solve(twin):
    a = c4()
    r = twin.solve(a)
    assert digest(r["plan"], r["planned_rounds"]) == (GOLD["plan_sha"], GOLD["counts_sha"])
    assert float(r["objective"]).hex() == GOLD["objective_hex"]


def test_c4_world_digests_are_one():
    ref = GOLD["by_world"]["1"]
    assert all(GOLD["by_world"][w] == ref for w in ("2", "4", "8"))
    assert ref["counts_sha"] == GOLD["counts_sha"] and ref["objective_hex"] == GOLD["objective_hex"]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c4_world_digests_are_the_shard_engine(world, twin):
    """The CPU shard engine at W (threads) reproduces the committed digest of W,
    and keeps the single-instance P1 objective (the share placement places
    every count); its P2 stays within the contract's ratio."""
    import ctypes

    import sw_native as sn
    import test_shard as ts
    from conftest import TWIN_SO

    lib = ctypes.CDLL(TWIN_SO)
    lib.shard_twin_solve.argtypes = [ctypes.POINTER(sn.SwHostComm), ctypes.c_int32, ctypes.c_int32,
                                     ctypes.POINTER(sn.SwProblem), ctypes.c_int64, ctypes.c_int64,
                                     ctypes.POINTER(sn.SwResult)]
    lib.shard_twin_solve.restype = ctypes.c_int
    a = c4()
    r = ts.run_threads(lib, a, world)
    g = GOLD["by_world"][str(world)]
    assert digest(r["plan"], r["planned_rounds"]) == (g["plan_sha"], g["counts_sha"])
    assert float(r["objective"]).hex() == g["objective_hex"] == GOLD["objective_hex"]
    ts.assert_share_contract(r, twin.solve(a), f"C4 W={world}")


def test_c4_objective_within_lp_bound(twin):
    a = c4()
    assert inputs_sha(a) == LP["inputs_sha"], "C4 inputs changed: regenerate tests/golden/c4_lp.json"
    check_lp_bound(twin.solve(a)["objective"])


@pytest.mark.gpu
def test_gpu_rccl_world1_reproduces_c4_digest():
    import sw_native as sn

    a = c4()
    s = sn.Solver(device=0)
    s.dist_init(sn.unique_id(), 0, 1)
    r = s.dist_solve(a, 0, a.N)
    s.close()
    g = GOLD["by_world"]["1"]
    assert digest(r["plan"], r["planned_rounds"]) == (g["plan_sha"], g["counts_sha"])
    assert float(r["objective"]).hex() == g["objective_hex"] == GOLD["objective_hex"]
    check_lp_bound(r["objective"])
