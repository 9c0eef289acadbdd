"""Round-loop simulator counterpart (sw_sim.py).

CPU: the loop runs with the bit-exact CPU twins of the two HIP kernels
(oracle/plan_twin.c, oracle/mmf_twin.c) injected, so the numbers here are
the numbers the GPU produces (tests/test_gpu_sim.py checks that on the GPU).
"""
import contextlib
import io
import json
import os

import numpy as np
import pytest

import mmf_ref
import sw_sim
import sw_trace as st

TRACE120 = os.path.join(st.DATA_DIR, "traces",
                        "120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace")
CFG64 = json.load(open(os.path.join(st.DATA_DIR, "configs", "scale_64gpus.json")))


def run(policy, twin, gpus=16, max_jobs=40, **kw):
    with contextlib.redirect_stdout(io.StringIO()):
        return sw_sim.run_trace(policy, TRACE120, gpus, 120, CFG64, shockwave_solver=twin,
                                mmf_allocator=mmf_ref.twin_allocator, max_jobs=max_jobs, **kw)


class CapacityCheck:
    """Wraps the twin; checks every plan against the per-round capacity."""

    def __init__(self, twin):
        self.twin = twin
        self.solves = 0

    def solve(self, arrays):
        r = self.twin.solve(arrays)
        load = (r["plan"].astype(np.int64) * arrays.w[:, None]).sum(axis=0)
        assert np.all(load <= arrays.G)
        self.solves += 1
        return r


@pytest.mark.parametrize("policy", ["shockwave", "max_min_fairness"])
def test_all_jobs_finish_and_metrics_are_consistent(twin, policy):
    r = run(policy, CapacityCheck(twin))
    assert r["jobs_completed"] == 40
    assert r["makespan"] > 0 and r["avg_jct"] > 0
    assert 0 < r["utilization"] <= 1.0
    assert 0.0 <= r["unfair_fraction"] <= 100.0
    assert r["solves"] >= 1


def test_deterministic(twin):
    a = run("shockwave", twin)
    b = run("shockwave", twin)
    for k in ("makespan", "avg_jct", "worst_ftf", "unfair_fraction", "rounds", "solves"):
        assert a[k] == b[k], k


def test_round_loop_invariants(twin):
    """Never more workers than GPUs in a round, every scheduled job is active,
    and job start timestamps are their trace arrival times (scheduler.py:616)."""
    tp = st.load_throughputs()
    jobs, arr = st.parse_trace(TRACE120)
    jobs, arr = jobs[:30], arr[:30]
    prof = st.synthesize_profiles(jobs, tp)
    cfg = dict(CFG64, time_per_iteration=120, num_gpus=8)
    sim = sw_sim.Simulator("shockwave", tp, prof, 120, shockwave_config=cfg, shockwave_solver=twin)
    orig = sim._schedule_jobs_on_workers
    rounds = []

    def checked():
        out = orig()
        used = [w for ws in out.values() for w in ws]
        assert len(used) == len(set(used)) <= 8
        assert all(j in sim._jobs for j in out)
        rounds.append(len(out))
        return out

    sim._schedule_jobs_on_workers = checked
    with contextlib.redirect_stdout(io.StringIO()):
        sim.simulate(8, arr, jobs)
    assert sum(rounds) > 0
    assert sim._per_job_start_timestamps == {i: a for i, a in enumerate(arr)}
    ftf, unfair = sim.get_finish_time_fairness()
    assert len(ftf) == sum(v is not None for v in sim._job_completion_times.values())


def test_shockwave_is_fairer_than_max_min_fairness(twin):
    """The paper's qualitative result (README.md:33-35) on the 120-job trace."""
    s = run("shockwave", twin, gpus=64, max_jobs=None)
    g = run("max_min_fairness", twin, gpus=64, max_jobs=None)
    assert s["worst_ftf"] < g["worst_ftf"]
    assert s["unfair_fraction"] <= g["unfair_fraction"]
    assert s["makespan"] < g["makespan"] * 1.05


def test_bs_scaling_preserves_epochs():
    """_scale_bs_and_iters keeps the epoch count (scheduler.py:3563-3580)."""
    tp = st.load_throughputs()
    jobs, _ = st.parse_trace(TRACE120)
    job = jobs[1]  # ResNet-18 (batch size 32), accordion
    sim = sw_sim.Simulator("max_min_fairness", tp, st.synthesize_profiles([job], tp), 120)
    sim._worker_ids = list(range(4))
    jid = sim.add_job(job, 0.0)
    spe = st.steps_per_epoch(job.model, job.batch_size)
    epochs = sim._num_epochs(job.model, job.batch_size, job.total_steps)
    sim._total_steps_run[jid] = 11 * spe + 3
    sim._bs_scale[jid] = sw_sim.BS_BIG
    sim._scale_bs_and_iters(jid)
    assert job.batch_size == st.MAX_BS["ResNet-18"]
    assert sim._num_epochs(job.model, job.batch_size, job.total_steps) == epochs
    assert sim._total_steps_run[jid] == 12 * st.steps_per_epoch(job.model, job.batch_size)
    assert sim._throughputs[jid] == tp[(job.job_type, job.scale_factor)]


def test_unknown_policy_rejected():
    with pytest.raises(ValueError):
        sw_sim.Simulator("fifo", {}, {})
