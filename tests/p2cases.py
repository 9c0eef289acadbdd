"""Captured simulator instances that exercise every P2 placement (fixture
tests/golden/p2_cases.json, made by tests/golden/make_p2_cases.py)."""
import json
import os

import numpy as np

import sw_native as sn

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "p2_cases.json")
KIND_BITS = {"density": 0, "weight": sn.SW_STATUS_P2_WEIGHT_ORDER,
             "classwise": sn.SW_STATUS_P2_CLASSWISE, "repaired": sn.SW_STATUS_P2_REPAIRED}


def load_cases():
    return json.load(open(GOLDEN))


def arrays(c, tile=1):
    """ProblemArrays of a case; tile > 1 repeats the jobs and scales G (a
    larger instance with the same structure, for the HBM-workspace path)."""
    rep = lambda v: np.tile(np.asarray(v), tile)  # noqa: E731
    return sn.ProblemArrays(rep(c["w"]), rep(c["d"]), rep(c["F"]), rep(c["E"]), rep(c["R"]),
                            rep(c["p"]), c["T"], c["G"] * tile, c["delta"], c["k"],
                            tuple(c["bases"]))
