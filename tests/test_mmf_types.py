"""The heterogeneity-aware MaxMinFairness allocation over worker types
(policies/max_min_fairness.py:44-100, policy.py:57-63; sw_mmf_allocate_types,
csrc/sw_mmf_lp.h): the CPU twin of the simplex kernel against the reference's
LP solved by HiGHS (the level to 1e-9, feasibility, optimality of the vertex),
the unit-throughput reduction of the Fig-9 policy, the host mirror of the
policy classes; GPU: the kernel against the twin bit for bit.  The reference's
ECOS returns an interior point of the optimal face, this kernel a vertex: the
allocation itself is parity-unpinned where the optimum is not unique."""
import os
import sys

import numpy as np
import pytest

import mmf_ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "shockwave-replication_amd"))
import max_min_fairness as mmfp  # noqa: E402


def lp_cases():
    rng = np.random.default_rng(11)
    out = []
    for m, n in [(1, 1), (1, 3), (2, 2), (5, 3), (12, 2), (40, 3), (60, 4), (120, 3), (200, 3), (33, 8)]:
        W = rng.integers(1, 3 * m + 2, size=n).astype(np.int32)
        sf = rng.choice([1, 2, 4, 8], size=m, p=[0.6, 0.3, 0.09, 0.01]).astype(np.int32)
        thr = rng.uniform(0.2, 3.0, size=(m, n))
        pw = rng.choice([1.0, 1.0, 2.0, 5.0], size=m)
        out.append((W, sf, thr * (sf / pw)[:, None]))
    # zero throughput on a type, a type with no workers, a tight cluster
    W = np.array([4, 0, 2], dtype=np.int32)
    sf = np.array([1, 2, 1, 4], dtype=np.int32)
    c = np.array([[1.0, 2.0, 0.0], [0.5, 0.0, 1.5], [2.0, 1.0, 1.0], [0.0, 3.0, 1.0]])
    out.append((W, sf, c))
    return out


def check_optimal(W, sf, c, x, t, tol=1e-9):
    t_lp, _ = mmf_ref.lp_level_types(W, sf, c)
    assert abs(t - t_lp) <= tol * max(1.0, abs(t_lp)), (t, t_lp)
    assert (x >= -tol).all()
    assert (x.sum(axis=1) <= 1.0 + tol).all()
    assert ((sf[:, None] * x).sum(axis=0) <= W + tol * np.maximum(W, 1)).all()
    assert ((c * x).sum(axis=1) >= t - tol * max(1.0, abs(t))).all()  # every job reaches t*


@pytest.mark.parametrize("i", range(len(lp_cases())))
def test_twin_types_vs_highs(i):
    W, sf, c = lp_cases()[i]
    x, t, piv = mmf_ref.twin_allocate_types(W, sf, c)
    check_optimal(W, sf, c, x, t)
    assert piv > 0 or t == 0.0


def test_twin_types_fuzz_vs_highs():
    rng = np.random.default_rng(5)
    for _ in range(150):
        m, n = int(rng.integers(1, 50)), int(rng.integers(1, 6))
        W = rng.integers(0, 30, size=n).astype(np.int32)
        W[rng.integers(0, n)] += 1
        sf = rng.choice([1, 2, 4, 8], size=m).astype(np.int32)
        c = rng.uniform(0.0, 4.0, size=(m, n)) * sf[:, None]
        c[rng.random(size=(m, n)) < 0.1] = 0.0
        x, t, _ = mmf_ref.twin_allocate_types(W, sf, c)
        check_optimal(W, sf, c, x, t)


def test_unit_throughputs_reduce_to_the_aggregate_level():
    """The Fig-9 policy (every throughput 1.0): coef[j][k] = c_j for every type,
    so only the total capacity matters — t* = min(min_j c_j, ΣW / Σ_j sf_j/c_j),
    the one-type kernel's level on Σ_k W_k workers."""
    rng = np.random.default_rng(3)
    for _ in range(40):
        m, n = int(rng.integers(1, 80)), int(rng.integers(1, 4))
        W = rng.integers(1, 40, size=n).astype(np.int32)
        sf = rng.choice([1, 2, 4, 8], size=m).astype(np.int32)
        cj = sf / rng.choice([1.0, 2.0, 5.0], size=m)
        _, t, _ = mmf_ref.twin_allocate_types(W, sf, np.repeat(cj[:, None], n, axis=1))
        _, t1, _ = mmf_ref.twin_allocate(sf, cj, int(W.sum()))
        assert abs(t - t1) <= 1e-12 * max(1.0, t1), (t, t1)


class _TwinEngine:
    """The native engine's two calls, backed by the CPU twins (tests only)."""

    def mmf_allocate(self, sf, c, G):
        return mmf_ref.twin_allocate(sf, c, G)

    def mmf_allocate_types(self, W, sf, c):
        return mmf_ref.twin_allocate_types(W, sf, c)


def _policy_inputs(seed, types):
    rng = np.random.default_rng(seed)
    jobs = [f"j{i:03d}" for i in rng.permutation(30)]
    thr = {j: {wt: float(rng.uniform(0.5, 4.0)) for wt in types} for j in jobs}
    sf = {j: int(rng.choice([1, 2, 4, 8], p=[0.6, 0.3, 0.09, 0.01])) for j in jobs}
    pw = {j: float(rng.choice([1.0, 2.0])) for j in jobs}
    spec = {wt: int(rng.integers(4, 24)) for wt in types}
    return thr, sf, pw, spec


def test_policy_mirror_flattens_and_solves_like_the_reference():
    """MaxMinFairnessPolicyWithPerf.get_allocation: jobs by sorted id, types by
    sorted name (policy.py:28-44), the coefficient matrix of
    max_min_fairness.py:54-87, the LP's level, shares clipped to [0, 1]."""
    types = ["v100", "k80", "p100"]
    thr, sf, pw, spec = _policy_inputs(1, types)
    pol = mmfp.MaxMinFairnessPolicyWithPerf(native=_TwinEngine())
    alloc = pol.get_allocation(thr, sf, pw, spec)
    assert sorted(alloc) == sorted(thr)
    assert all(sorted(alloc[j]) == sorted(types) for j in alloc)
    coef, sfa, (job_ids, wts), W = pol.coefficients(thr, sf, pw, spec)
    assert job_ids == sorted(thr) and wts == sorted(types) and W == [spec[w] for w in sorted(types)]
    # the coefficient matrix restated elementwise
    m, n = len(job_ids), len(wts)
    xp = np.array([[spec[w] / m for w in wts]] * m)
    xp = xp / xp.sum(axis=1).max()
    for i, j in enumerate(job_ids):
        prop = sum(thr[j][w] * xp[i, k] for k, w in enumerate(wts))
        for k, w in enumerate(wts):
            assert coef[i, k] == pytest.approx(thr[j][w] * (1.0 / pw[j]) / prop * sf[j], rel=1e-15)
    x = np.array([[alloc[j][w] for w in wts] for j in job_ids])
    assert ((x >= 0.0) & (x <= 1.0)).all()
    t_lp, _ = mmf_ref.lp_level_types(W, sfa, coef)
    assert (coef * x).sum(axis=1).min() == pytest.approx(t_lp, rel=1e-9)
    assert pol.get_allocation({}, {}, {}, spec) is None


def test_unit_policy_mirror_uses_unit_throughputs():
    types = ["k80", "v100"]
    thr, sf, pw, spec = _policy_inputs(2, types)
    pol = mmfp.MaxMinFairnessPolicy(native=_TwinEngine())
    alloc = pol.get_allocation(thr, sf, pw, spec)
    ones = {j: {w: 1.0 for w in types} for j in thr}
    ref = mmfp.MaxMinFairnessPolicyWithPerf(native=_TwinEngine()).get_allocation(ones, sf, pw, spec)
    assert alloc == ref


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(len(lp_cases())))
def test_gpu_types_bit_exact_vs_twin(gpu_solver, i):
    W, sf, c = lp_cases()[i]
    xg, tg, pg = gpu_solver.mmf_allocate_types(W, sf, c)
    xt, tt, pt = mmf_ref.twin_allocate_types(W, sf, c)
    assert pg == pt
    assert tg.hex() == tt.hex()
    assert np.array_equal(xg.view(np.uint64), xt.view(np.uint64))
    check_optimal(W, sf, c, xg, tg)


@pytest.mark.gpu
def test_gpu_types_fuzz_bit_exact_vs_twin(gpu_solver):
    rng = np.random.default_rng(9)
    for _ in range(40):
        m, n = int(rng.integers(1, 120)), int(rng.integers(1, 5))
        W = rng.integers(1, 60, size=n).astype(np.int32)
        sf = rng.choice([1, 2, 4, 8], size=m).astype(np.int32)
        c = rng.uniform(0.0, 4.0, size=(m, n)) * sf[:, None]
        xg, tg, pg = gpu_solver.mmf_allocate_types(W, sf, c)
        xt, tt, pt = mmf_ref.twin_allocate_types(W, sf, c)
        assert pg == pt and tg.hex() == tt.hex()
        assert np.array_equal(xg.view(np.uint64), xt.view(np.uint64))


@pytest.mark.gpu
def test_gpu_types_rejects_bad_input(gpu_solver):
    import sw_native as sn

    with pytest.raises(sn.NativeError):
        gpu_solver.mmf_allocate_types([4, 2], [1, 0], np.ones((2, 2)))
    with pytest.raises(sn.NativeError):
        gpu_solver.mmf_allocate_types([4, -1], [1, 1], np.ones((2, 2)))
    with pytest.raises(sn.NativeError):
        gpu_solver.mmf_allocate_types([4, 2], [1, 1], np.array([[1.0, np.nan], [1.0, 1.0]]))
    x, t, p = gpu_solver.mmf_allocate_types([4, 2], [], np.zeros((0, 2)))
    assert x.shape == (0, 2) and t == 0.0
    # above the limits: too many jobs (invalid), a tableau above 256 MB (capacity)
    with pytest.raises(sn.NativeError) as e:
        gpu_solver.mmf_allocate_types([4], np.ones(2049, dtype=np.int32), np.ones((2049, 1)))
    assert e.value.code == sn.SW_ERR_INVALID
    with pytest.raises(sn.NativeError) as e:
        gpu_solver.mmf_allocate_types(np.full(16, 8), np.ones(2048, dtype=np.int32), np.ones((2048, 16)))
    assert e.value.code == sn.SW_ERR_CAPACITY


@pytest.mark.gpu
def test_gpu_policy_mirror_three_types(gpu_solver):
    types = ["k80", "p100", "v100"]
    thr, sf, pw, spec = _policy_inputs(4, types)
    pol = mmfp.MaxMinFairnessPolicyWithPerf(native=gpu_solver)
    alloc = pol.get_allocation(thr, sf, pw, spec)
    coef, sfa, (job_ids, wts), W = pol.coefficients(thr, sf, pw, spec)
    x = np.array([[alloc[j][w] for w in wts] for j in job_ids])
    t_lp, _ = mmf_ref.lp_level_types(W, sfa, coef)
    assert (coef * x).sum(axis=1).min() == pytest.approx(t_lp, rel=1e-9)
