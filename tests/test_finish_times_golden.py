"""The drop-in ShockwaveScheduler computes the plan-solve inputs exactly as
the REFERENCE code does (tests/golden/finish_times.json, produced by running
the reference's _compute_finish_times / _compute_interpolated_finish_time
(shockwave.py:224-279, AST-executed) on the reference's own
ShockwaveJobMetadata objects — tests/golden/make_finish_times.py).

Every solve's d_j (:116-120), R_j (call #2, :261), FTF_j (:266-278, with the
finish-time history appended every solve) and p_j = FTF_j**lambda (:368) must
match bit for bit, across arrivals, throughput updates, completions,
deletions and the non-idempotent estimator calls.
"""
import json
import os

import numpy as np
import pytest

from job_metadata import ShockwaveJobMetadata
from shockwave import ShockwaveScheduler

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "finish_times.json")
SCEN = json.load(open(GOLD))["scenarios"]


def hexes(a):
    return [float(x).hex() for x in a]


@pytest.mark.parametrize("si", range(len(SCEN)))
def test_solve_inputs_match_reference_execution(si):
    sc = SCEN[si]
    cfg = dict(sc["config"])
    cfg.update({"k": 1.0, "log_approximation_bases": [0.0, 0.2, 0.4, 0.6, 0.8, 1.0]})
    s = ShockwaveScheduler(cfg, solver=object())  # inputs only: no solve is made
    solves = iter(sc["solves"])
    n_checked = 0
    for ev in sc["events"]:
        kind = ev[0]
        if kind == "add":
            jid = ev[1]
            prof = sc["profiles"][str(jid)]
            md = ShockwaveJobMetadata(prof, cfg["time_per_iteration"], prof["scale_factor"])
            md.submit(float.fromhex(ev[2]))
            s.add_metadata(jid, md)
        elif kind == "tput":
            s.job_metadata[ev[1]].update_throughput_schedule(ev[2], float.fromhex(ev[3]), ev[4])
        elif kind == "complete":
            s.job_metadata[ev[1]].complete(ev[2])
        elif kind == "delete":
            s.delete_metadata(ev[1])
        elif kind == "round":
            s.round_index = ev[1]
        elif kind == "solve":
            want = next(solves)
            assert s.round_index == want["round_index"]
            assert list(s.job_metadata) == want["ids"]
            a = s._gather_inputs()
            assert hexes(a.d) == want["d"], "d_j (shockwave.py:116-120)"
            assert hexes(a.R) == want["R"], "R_j (call #2, shockwave.py:261)"
            assert hexes(a.p) == want["p"], "p_j = FTF**lambda (shockwave.py:368)"
            for jid, f in zip(want["ids"], want["ftf"]):
                hist = s.finish_time_estimates[jid]
                assert hist[-1][0] == s.round_index
            n_checked += 1
    assert n_checked == len(sc["solves"]) > 0


def test_fixture_exercises_history_and_deletions():
    kinds = {ev[0] for sc in SCEN for ev in sc["events"]}
    assert {"add", "tput", "complete", "delete", "solve", "round"} <= kinds
    # interpolation with more than one estimate in the history
    assert any(len(sc["solves"]) > 1 for sc in SCEN)
    ftf = np.array([float.fromhex(x) for sc in SCEN for sv in sc["solves"] for x in sv["ftf"]])
    assert np.all(np.isfinite(ftf)) and np.all(ftf > 0)
