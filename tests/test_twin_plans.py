"""Plan digests pinned across algorithm changes that must not change results.

tests/golden/twin_plans.json holds, for 32 seeded instances at the reference
cluster configurations (scale_{32,64,128,256}gpus.json's k and lambda), the
objective bits and MD5 digests of the plan and counts of the CPU twin
(generator: tests/golden/make_twin_plans.py; re-pinned when the P2 cascade
gained the width-profile repair, and when P1 gained the fill of stranded
capacity, which changed case 25, a re-solved one, to a higher objective).  Performance-only changes of the kernel or
the searches must keep them: the twin and the GPU kernel must both reproduce
every digest.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import sw_native as sn
import sw_synth as ss

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "twin_plans.json")))["cases"]


def _arrays(c):
    a = ss.synth_problem(c["seed"], c["N"], c["G"], c["T"], 120.0, c["k"], c["lam"])
    return sn.ProblemArrays(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, tuple(a.bases))


def _check(c, objective, plan, counts):
    assert float(objective).hex() == c["objective"], (c, objective)
    assert hashlib.md5(np.ascontiguousarray(plan, dtype=np.uint8).tobytes()).hexdigest() == c["plan_md5"], c
    assert hashlib.md5(np.ascontiguousarray(counts, dtype=np.int32).tobytes()).hexdigest() == c["counts_md5"], c


@pytest.mark.parametrize("i", range(len(GOLD)))
def test_twin_reproduces_pinned_plans(i, twin):
    c = GOLD[i]
    b = _arrays(c)
    r = twin.solve(b)
    assert r["rc"] == c["rc"]
    _check(c, r["objective"], r["plan"], r["planned_rounds"])


@pytest.mark.gpu
def test_gpu_reproduces_pinned_plans(gpu_solver):
    """All 32 instances in one batched launch of the plan kernel."""
    batch = [_arrays(c) for c in GOLD]
    res = gpu_solver.solve_batch(batch)
    for c, r in zip(GOLD, res):
        _check(c, r["objective"], r["plan"], r["planned_rounds"])
