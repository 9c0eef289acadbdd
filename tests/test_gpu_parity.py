"""GPU plan kernel vs the CPU bit-exact twin, through the C-ABI.

The bar (north star): the relaxed-plan rounding into the per-round schedule is
deterministic and bit-exact vs a CPU reimplementation — so every field of the
result (plan bytes, counts, objective bits, iteration count) must match.
"""
import numpy as np
import pytest

import sw_synth as ss
from helpers import assert_same_result, check_plan_valid

pytestmark = pytest.mark.gpu

CASES = [
    # (seed, N, G, T, k, lam)
    (0, 12, 4, 6, 1e5, 5.0),
    (1, 20, 8, 8, 1e-3, 15.0),
    (2, 30, 8, 10, 1e1, 5.0),
    (3, 50, 32, 20, 1e-3, 15.0),
    (4, 120, 64, 20, 1e-3, 15.0),
    (5, 120, 128, 20, 1e1, 5.0),
    (6, 120, 256, 20, 1e5, 5.0),
    (7, 900, 256, 30, 1e5, 5.0),
    (8, 900, 64, 20, 1e-3, 15.0),
    (9, 1024, 256, 30, 1e5, 5.0),
    (10, 300, 64, 64, 1e1, 5.0),
    (11, 200, 32, 40, 0.5, 3.0),
]


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[1]}_G{c[2]}_T{c[3]}_k{c[4]:g}" for c in CASES])
def test_gpu_matches_twin(case, gpu_solver, twin):
    seed, N, G, T, k, lam = case
    a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
    rg = gpu_solver.solve(a)
    rt = twin.solve(a)
    check_plan_valid(a, rg)
    assert_same_result(rg, rt, f"case {case}")


@pytest.mark.parametrize("wide", [16, 32, 200])
def test_gpu_wide_jobs_match_twin(wide, gpu_solver, twin):
    """Jobs of width ≥ 16 (the round loop's width tail once packed w in 4 bits)."""
    a = ss.synth_problem(21, 300, 512, 20, 120.0, 1e1, 5.0)
    a.w[::7] = wide
    a.w[::11] = 3
    rg = gpu_solver.solve(a)
    check_plan_valid(a, rg)
    assert_same_result(rg, twin.solve(a), f"wide={wide}")


def test_gpu_large_instance_workspace_path(gpu_solver, twin):
    """N > 1024 takes the HBM-workspace path of the kernel."""
    a = ss.synth_problem(42, 2500, 700, 30, 120.0, 1e5, 5.0)
    rg = gpu_solver.solve(a)
    rt = twin.solve(a)
    check_plan_valid(a, rg)
    assert_same_result(rg, rt, "N=2500")


def test_gpu_batch_matches_single(gpu_solver, twin):
    probs = ss.sweep_problems(8, N=150, seed0=100)
    rb = gpu_solver.solve_batch(probs)
    for a, r in zip(probs, rb):
        assert_same_result(r, twin.solve(a), "batch")


def test_gpu_deterministic(gpu_solver):
    a = ss.c3_problem(3)
    r1 = gpu_solver.solve(a)
    r2 = gpu_solver.solve(a)
    assert_same_result(r1, r2, "repeat")


EDGE = [
    dict(),
    dict(regularizer=0.0),
    dict(nworkers=[4, 1], num_gpus=2),
    dict(completed_epochs=[10, 1], priority=[0.0, 2.0], remaining_runtime=[1.0, 150.0]),
    dict(num_gpus=0),
    dict(priority=[1e300, 1e-300]),
]


@pytest.mark.parametrize("kw", EDGE, ids=[str(i) for i in range(len(EDGE))])
def test_gpu_edge_cases_match_twin(kw, gpu_solver, twin):
    import sw_native as sn

    base = dict(nworkers=[1, 2], epoch_duration=[100.0, 50.0], completed_epochs=[0, 1],
                total_epochs=[10, 4], remaining_runtime=[1000.0, 150.0], priority=[1.0, 2.0],
                future_rounds=4, num_gpus=2, round_duration=120.0, regularizer=1.0)
    base.update(kw)
    a = sn.ProblemArrays(**base)
    assert_same_result(gpu_solver.solve(a), twin.solve(a), str(kw))


def test_gpu_empty_problem(gpu_solver):
    import sw_native as sn

    a = sn.ProblemArrays([], [], [], [], [], [], 4, 2, 120.0, 1.0)
    r = gpu_solver.solve(a)
    assert r["plan"].shape == (0, 4)
    assert r["status"] & sn.SW_STATUS_NO_PLANNED


def test_gpu_rejects_invalid(gpu_solver):
    import sw_native as sn

    a = sn.ProblemArrays([0], [1.0], [0], [1], [1.0], [1.0], 4, 2, 120.0, 1.0)
    with pytest.raises(sn.NativeError):
        gpu_solver.solve(a)


def test_gpu_resolve_with_job_indices_above_65535(gpu_solver, twin):
    """A re-solved instance (SW_STATUS_P1_REPACKED: the per-round
    re-optimisation runs) whose active jobs sit at indices ≥ 66,000 — 66,000
    finished jobs first, then a 40-job width-fragmented instance — so the
    knapsack's items carry job indices above 16 bits (sw_reround_dev.h keeps
    the full index).  The workspace path of sw_plan_solve equals
    the twin bit for bit."""
    import sw_native as sn
    import sw_synth as ss

    b = ss.synth_problem(0, 40, 12, 12, 120.0, 1.0, 5.0, width_p=(0.4, 0.3, 0.2, 0.1))
    pad = 66000
    a = sn.ProblemArrays(np.concatenate([np.ones(pad, np.int32), b.w]),
                         np.concatenate([np.full(pad, 1.0), b.d]),
                         np.concatenate([np.full(pad, 10, np.int32), b.F]),
                         np.concatenate([np.full(pad, 10, np.int32), b.E]),
                         np.concatenate([np.zeros(pad), b.R]), np.concatenate([np.zeros(pad), b.p]),
                         b.T, b.G, b.delta, b.k, tuple(b.bases))
    rt = twin.solve(a)
    assert rt["status"] & sn.SW_STATUS_P1_REPACKED
    assert rt["planned_rounds"][pad:].sum() > 0 and rt["planned_rounds"][:pad].sum() == 0
    rg = gpu_solver.solve(a)
    check_plan_valid(a, rg)
    assert_same_result(rg, rt, "N=66040 re-solved")
