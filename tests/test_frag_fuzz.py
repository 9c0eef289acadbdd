"""Width fragmentation against the reference MILP on 600 random instances
whose widths reach the cluster size (tests/golden/frag_fuzz.json, made by
tests/golden/make_frag_fuzz.py: fuzzcases.fuzz_problem(seed, max_n=80), T
capped at 12, HiGHS at gap 1e-6 on the restated P1 of shockwave.py:330-382).

The reference packs any widths exactly (a MILP over x_jt, capacity rows
:64-75).  The count-then-pack reduction, its reduced-budget re-solve, the fill
and the per-round exact re-optimisation (sw_reround.h) bring 588 of the 599
solved instances within the north star's 1e-3 (before the re-optimisation:
567, worst gap 0.61).  The 11 that stay above are recorded here with their
measured gap as a ceiling, so a regression fails and a fix shows: each is a
local optimum of the per-round neighbourhood (the MILP's better plan needs
jobs moved between several rounds at once: e.g. seed 50169, G = 7 with widths
{1, 2, 2, 3, 4, 6, 6} and k = 0, where the MILP fits a 6-wide job a fourth
round by repacking three other rounds; its objective is a near-cancelling
sum, |J| = 4e-3 against per-job utilities up to 6e7, so the relative gap is
large).  Two of the 11 are instances HiGHS itself stopped at its time limit.
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
# seed -> measured relative gap to the MILP (twin = GPU bit for bit)
EXCEPTIONS = {50078: 5.2e-3, 50104: 1.5e-3, 50115: 2.95e-3, 50169: 0.52, 50265: 1.91e-2,
              50334: 1.46e-2, 50404: 1.17e-2, 50417: 4.9e-3, 50432: 1.7e-3, 50445: 2.41e-2,
              50498: 1.24e-2}


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
    return gap


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
