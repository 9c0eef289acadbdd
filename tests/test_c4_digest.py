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


def c4():
    c = ss.C4
    return ss.synth_problem(GOLD["seed"], c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])


def digest(plan, counts):
    return (hashlib.sha256(np.ascontiguousarray(plan).tobytes()).hexdigest()[:32],
            hashlib.sha256(np.ascontiguousarray(counts, dtype=np.int32).tobytes()).hexdigest()[:32])


def test_c4_digest_is_the_twin_solve(twin):
    a = c4()
    r = twin.solve(a)
    assert digest(r["plan"], r["planned_rounds"]) == (GOLD["plan_sha"], GOLD["counts_sha"])
    assert float(r["objective"]).hex() == GOLD["objective_hex"]


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
