"""Width fragmentation against the reference MILP on 600 random instances
whose widths reach the cluster size (tests/golden/frag_fuzz.json, made by
tests/golden/make_frag_fuzz.py: fuzzcases.fuzz_problem(seed, max_n=80), T
capped at 12, HiGHS at gap 1e-6 on the restated P1 of shockwave.py:330-382).

The reference packs any widths exactly (a MILP over x_jt, capacity rows
:64-75).  The count-then-pack reduction with the level search's branch and
bound (sw_bnb.h), the pattern placement (sw_profile_search), the reduced-
budget re-solve, the fill and the per-round exact re-optimisation
(sw_reround.h) and the raises (one job one more round, the plan re-placed by
the pattern search; sw_arith.h SW_RAISE_ITERS) bring 591 of the 599 solved
instances within the north star's 1e-3 (round 5: 590, round 4: 588; before
the re-optimisation: 567, worst gap 0.61).  Every
instance whose widths lie in the reference traces' domain {1, 2, 4, 8} is
within 1e-3 (seed 50115, the one that was not, now finds the MILP's level and
places its counts by a round-pattern search).  The 8 that stay above all have
other widths (non-power-of-two classes, up to 12 of them); they are recorded
here with their measured gap as a ceiling, so a regression fails and a fix
shows (seed 50169, at 0.52 in round 5, is within 1e-3 since the raises), and
the solver flags each one: SW_STATUS_P1_UNCERTIFIED says the plan is
not certified within 1e-3 of `bound`, which is a valid upper bound on the
MILP optimum (checked on all 599).  One of the 8 (seed 50445) is an instance
HiGHS itself stopped at its time limit.
"""
import json
import os
import sys

import numpy as np
import pytest

import milp_ref as mr
import sw_native as sn
from helpers import assert_same_result, check_plan_valid, to_oracle

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_frag_fuzz as mk  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frag_fuzz.json")
REL_TOL = 1e-3
# seed -> measured relative gap to the MILP (twin = GPU bit for bit); none
# of them has widths within {1, 2, 4, 8} only
EXCEPTIONS = {50078: 5.2e-3, 50104: 1.5e-3, 50265: 1.91e-2, 50334: 1.46e-2,
              50404: 1.17e-2, 50432: 1.7e-3, 50445: 2.41e-2, 50498: 1.24e-2}
# the bound is the Lagrangian bound of fp32-keyed prices: valid to fp32 key
# resolution (a relative 1e-7 of the objective's scale)
BOUND_TOL = 1e-7


def _cases():
    return json.load(open(GOLD))["cases"] if os.path.exists(GOLD) else []


CASES = _cases()


def _instance(c):
    a = mk.instance(c["seed"])
    assert mk.inputs_sha(a) == c["inputs_sha"], "instance changed: regenerate frag_fuzz.json"
    return a


def _check(c, a, r):
    check_plan_valid(a, r)
    got = mr.evaluate_counts(to_oracle(a), r["planned_rounds"])[0]
    ref = c["J"]
    gap = (ref - got) / abs(ref) if ref else 0.0
    bar = EXCEPTIONS.get(c["seed"], REL_TOL)
    assert gap <= bar * (1 + 1e-6), (c["seed"], a.N, a.G, a.k, gap, bar)
    # the certificate: bound ≥ the MILP optimum, and a plan not flagged is
    # within 1e-3 of the bound (so of the MILP)
    assert ref <= r["bound"] + BOUND_TOL * abs(r["bound"]) + 1e-12, (c["seed"], ref, r["bound"])
    if c["seed"] in EXCEPTIONS:
        assert r["status"] & sn.SW_STATUS_P1_UNCERTIFIED, (c["seed"], "miss not flagged")
    if not r["status"] & sn.SW_STATUS_P1_UNCERTIFIED:
        assert r["bound"] - got <= 1e-3 * abs(got) + 1e-12, (c["seed"], got, r["bound"])
    return gap


def test_exceptions_outside_trace_widths():
    """Every remaining miss has widths outside the traces' {1, 2, 4, 8}."""
    for s in EXCEPTIONS:
        a = mk.instance(s)
        assert set(a.w[a.w <= a.G].tolist()) - {1, 2, 4, 8}, s


def test_fixture_complete():
    assert len(CASES) == 600
    assert sum("J" in c for c in CASES) >= 590
    wide = sum(1 for c in CASES if (lambda a: (a.w[a.w <= a.G] * 2 > a.G).any())(_instance(c)))
    assert wide >= 150, wide  # jobs wider than G/2 are common


def test_twin_frag_fuzz_vs_milp(twin):
    gaps = []
    for c in CASES:
        if "J" not in c:
            continue
        gaps.append(_check(c, _instance(c), twin.solve(_instance(c))))
    above = sum(g > REL_TOL for g in gaps)
    assert above <= len(EXCEPTIONS), above


@pytest.mark.gpu
def test_gpu_frag_fuzz_vs_milp_one_launch(gpu_solver, twin):
    """All 600 in one batched launch of the HIP kernel: each equal to the twin
    bit for bit and held to the same bars."""
    probs = [_instance(c) for c in CASES]
    rs = gpu_solver.solve_batch(probs)
    rep = 0
    for c, a, r in zip(CASES, probs, rs):
        assert_same_result(r, twin.solve(a), f"seed {c['seed']}")
        rep += bool(r["status"] & sn.SW_STATUS_P1_REPACKED)
        if "J" in c:
            _check(c, a, r)
    assert rep >= 200, rep
    assert np.all([r["rc"] >= 0 for r in rs])
