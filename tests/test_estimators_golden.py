"""The host estimators (product job_metadata.py) vs golden vectors produced
by the REFERENCE's own scheduler/job_metadata.py (tests/golden/make_golden.py).

Bit-exact: every returned value is compared as a float hex string.
"""
import json
import os

import numpy as np
import pytest

from job_metadata import ShockwaveJobMetadata

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "estimators.json")


def _cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("ci", range(120))
def test_estimator_sequence_bit_exact(ci):
    case = _cases()[ci]
    prof = case["profile"]
    md = ShockwaveJobMetadata(prof, case["round_duration"], prof["scale_factor"])
    outs = iter(case["outs"])
    for op in case["ops"]:
        if op[0] == "tput":
            md.update_throughput_schedule(op[1], float.fromhex(op[2]), op[3])
        elif op[0] == "complete":
            md.complete(op[1])
        else:
            exp = next(outs)
            md.recompute_epoch_duration()
            d = md.interpolated_epoch_duration()
            r2 = md.compute_remaining_runtime()
            r3 = md.compute_remaining_runtime()
            s = md.completed_duration()
            r4 = md.compute_remaining_runtime()
            got = {"d": d, "R_mk": r2, "R_jct": r3, "sum_done": s, "R_fin": r4}
            for k, v in got.items():
                assert float(v).hex() == exp[k], (ci, k, float(v).hex(), exp[k])
            assert md.completed_epochs == exp["F"]
            dur = [float(x).hex() for x in md.epoch_durations[:5]] + \
                  [float(sum(md.epoch_durations)).hex()]
            assert dur == exp["durations_sha"]
            bm = md.compute_bs_epoch_duration()
            assert {str(k): float(v).hex() for k, v in bm.items()} == exp["bs_map"]


def test_remaining_runtime_complete_job_returns_one():
    prof = _cases()[0]["profile"]
    md = ShockwaveJobMetadata(prof, 120, 1)
    md.complete()
    assert md.compute_remaining_runtime() == 1.0


def test_complete_asserts_progress_bound():
    prof = _cases()[0]["profile"]
    md = ShockwaveJobMetadata(prof, 120, 1)
    with pytest.raises(AssertionError):
        md.complete(prof["num_epochs"] + 1)


def test_epoch_durations_rounded_at_least_one_second():
    prof = dict(_cases()[0]["profile"])
    prof["duration_every_epoch"] = [0.2, 1.4, 2.6] + prof["duration_every_epoch"][3:]
    md = ShockwaveJobMetadata(prof, 120, 1)
    assert md.epoch_durations[0] == 1.0 and md.epoch_durations[1] == 1.0
    if len(md.epoch_durations) > 2:
        assert md.epoch_durations[2] == 3.0
