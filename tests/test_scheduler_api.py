"""The drop-in ShockwaveScheduler: reference semantics of the policy API
(shockwave.py:12-91, :224-279, :390-398) with the solve injected.

On CPU the product path has no solver (no GPU, no fallback), so these tests
inject the CPU twin explicitly; the scheduler on the HIP solver is exercised
on the GPU by test_gpu_sim.py (whole simulations through ShockwaveScheduler).
"""
import copy
import random

import numpy as np
import pytest

import sw_native as sn
from job_metadata import ShockwaveJobMetadata
from shockwave import ShockwaveScheduler

CONFIG = {
    "num_gpus": 8, "time_per_iteration": 120, "future_rounds": 6, "lambda": 5.0, "k": 10.0,
    "rhomax": 1.0, "log_approximation_bases": [0.0, 0.2, 0.4, 0.6, 0.8, 1.0],
    "gpu_ram": 16, "solver_rel_gap": 1e-3, "solver_num_threads": 24, "solver_timeout": 15,
}


def profile(rng, E):
    bs = [rng.choice([32, 64]) for _ in range(E)]
    dur = [rng.uniform(20, 400) for _ in range(E)]
    return {"num_epochs": E, "num_samples_per_epoch": 50000, "scale_factor": rng.choice([1, 1, 2, 4]),
            "duration": sum(dur), "bs_every_epoch": bs, "mem_every_epoch": [1.0] * E,
            "util_every_epoch": [1.0] * E, "duration_every_epoch": dur}


class Recorder:
    """Wraps the twin; records the SoA arrays each solve received."""

    def __init__(self, twin):
        self.twin = twin
        self.calls = []

    def solve(self, arrays):
        self.calls.append(arrays)
        return self.twin.solve(arrays)


def make(twin, n_jobs=10, seed=0):
    rng = random.Random(seed)
    rec = Recorder(twin)
    s = ShockwaveScheduler(dict(CONFIG), solver=rec)
    for j in range(n_jobs):
        md = ShockwaveJobMetadata(profile(rng, rng.randint(3, 30)), CONFIG["time_per_iteration"],
                                  None)
        md.submit(0.0)
        s.add_metadata(j, md)
    return s, rec


def test_schedule_covers_horizon_and_is_feasible(twin):
    s, rec = make(twin)
    sched = s.current_round_schedule()
    assert len(rec.calls) == 1
    assert sorted(s.schedules.keys()) == list(range(CONFIG["future_rounds"]))
    ids = list(s.job_metadata.keys())
    for r, jobs in s.schedules.items():
        # insertion order preserved (shockwave.py:394-396)
        assert jobs == [j for j in ids if j in jobs]
        assert sum(s.job_metadata[j].nworkers for j in jobs) <= CONFIG["num_gpus"]
    assert sched == s.schedules[0]


def test_cache_and_recompute_flag(twin):
    s, rec = make(twin)
    s.current_round_schedule()
    s.current_round_schedule()
    assert len(rec.calls) == 1  # cached (shockwave.py:80-83)
    s.increment_round()
    s.current_round_schedule()
    assert len(rec.calls) == 1  # next round still cached
    s.set_recompute_flag()
    s.current_round_schedule()
    assert len(rec.calls) == 2 and not s.recompute_flag
    s.increment_round()
    # after a re-solve the cache covers round_index .. round_index + T - 1
    assert s.round_index + CONFIG["future_rounds"] - 2 in s.schedules


def test_arrivals_do_not_trigger_resolve(twin):
    s, rec = make(twin)
    s.current_round_schedule()
    s.add_metadata(99, ShockwaveJobMetadata(profile(random.Random(5), 5), 120, 1))
    s.increment_round()
    s.current_round_schedule()
    assert len(rec.calls) == 1


def test_inputs_follow_reference_call_order(twin):
    """d, R, FTF and p follow shockwave.py:111-134 then :255-278 exactly."""
    s, rec = make(twin, n_jobs=6, seed=3)
    # measured throughput so the estimators actually rescale
    for j, md in s.job_metadata.items():
        md.update_throughput_schedule(2, 5.0 + j, md.epoch_batch_sizes[0])
        md.complete(min(md.total_epochs, 1 + j % 3))
    shadow = {j: copy.deepcopy(md) for j, md in s.job_metadata.items()}
    s.round_index = 4
    s.current_round_schedule()
    a = rec.calls[0]
    N, G = len(shadow), CONFIG["num_gpus"]
    for i, (j, md) in enumerate(shadow.items()):
        md.recompute_epoch_duration()
        d = np.mean(md.epoch_durations[: md.completed_epochs + 1])
        assert a.d[i] == d
    for i, (j, md) in enumerate(shadow.items()):
        r_mk = md.compute_remaining_runtime()
        r_jct = md.compute_remaining_runtime()
        fin = sum(md.epoch_durations[: md.completed_epochs]) + md.compute_remaining_runtime()
        jct = (4 + CONFIG["future_rounds"]) * CONFIG["time_per_iteration"] + r_jct * (N / G)
        ftf = jct / fin  # first solve: the history holds one estimate
        assert a.R[i] == r_mk
        assert s.finish_time_estimates[j] == [(4, fin)]
        assert a.p[i] == ftf ** CONFIG["lambda"]
        assert a.w[i] == md.nworkers and a.F[i] == md.completed_epochs


def test_finish_time_history_appends_every_solve(twin):
    s, rec = make(twin, n_jobs=4)
    s.current_round_schedule()
    s.set_recompute_flag()
    s.increment_round()
    s.current_round_schedule()
    for hist in s.finish_time_estimates.values():
        assert [r for r, _ in hist] == [0, 1]


def test_interpolated_finish_time_weights():
    s = ShockwaveScheduler(dict(CONFIG), solver=object())
    s.finish_time_estimates["a"] = [(0, 100.0), (2, 200.0), (6, 400.0)]
    # windows [2, 4] → weights [1/3, 2/3] over the first two estimates
    exp = 0.9 * (100.0 / 3 + 200.0 * 2 / 3) + 0.1 * 400.0
    assert s._compute_interpolated_finish_time("a") == pytest.approx(exp, rel=1e-15)
    s.finish_time_estimates["b"] = [(3, 50.0)]
    assert s._compute_interpolated_finish_time("b") == pytest.approx(50.0)


def test_delete_metadata_and_empty_schedule(twin):
    s, rec = make(twin, n_jobs=2)
    assert s.delete_metadata(0) is not None and s.delete_metadata(0) is None
    s.delete_metadata(1)
    assert s.current_round_schedule() == []


def test_default_solver_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    s = ShockwaveScheduler(dict(CONFIG))
    s.add_metadata(0, ShockwaveJobMetadata(profile(random.Random(1), 4), 120, 1))
    with pytest.raises(sn.NativeError):
        s.current_round_schedule()
