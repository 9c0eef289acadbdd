"""The committed C4 digest (tests/golden/c4_digest.json) that bench.py's
c4_sharded sub-record checks at every N is the CPU twin's solve of that
instance (so a stale digest fails here, on the CPU, before a GPU run); and on
the GPU the RCCL-sharded engine at world 1 reproduces it."""
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
    assert digest(r["plan"], r["planned_rounds"]) == (GOLD["plan_sha"], GOLD["counts_sha"])
    assert float(r["objective"]).hex() == GOLD["objective_hex"]
    check_lp_bound(r["objective"])
