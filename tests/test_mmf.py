"""MaxMinFairness allocation (Gavel baseline, sw_mmf_allocate): the CPU twin
against the reference LP solved by HiGHS, and the analytic-centre conditions.
GPU: the HIP kernel against the twin, bit for bit."""
import numpy as np
import pytest

import mmf_ref


def instances():
    rng = np.random.default_rng(7)
    out = []
    for n, G in [(1, 4), (3, 2), (5, 64), (40, 32), (120, 64), (700, 256), (1500, 256),
                 (60, 256), (200, 1024), (2, 1)]:
        sf = rng.choice([1, 2, 4, 8], size=n, p=[0.6, 0.3, 0.09, 0.01]).astype(np.int32)
        pw = rng.choice([1.0, 1.0, 1.0, 5.0], size=n)
        out.append((sf, sf / pw, G))
    sf = np.array([2, 4, 8, 2], dtype=np.int32)  # no unit-width job: t* = 2
    out.append((sf, sf.astype(float), 64))
    return out


def check_lp_optimal(sf, c, G, x, t, mu):
    """The allocation against the reference LP (policies/max_min_fairness.py:73-100,
    solved by HiGHS in oracle/mmf_ref.lp_level): the level t* to 1e-9, feasibility,
    and the optimality conditions of the allocation (the unique optimum when
    capacity binds; otherwise the analytic centre's barrier stationarity — the
    point the reference's interior-point ECOS converges to; ECOS itself is
    absent here, so which optimal point it returns is parity-unpinned)."""
    t_lp, _ = mmf_ref.lp_level(sf, c, G)
    assert abs(t - t_lp) <= 1e-9 * max(1.0, abs(t_lp)), (t, t_lp)
    # feasible and optimal: every job gets at least t*, capacity and bounds hold
    assert np.all(x >= -1e-15) and np.all(x <= 1.0 + 1e-15)
    assert float(np.dot(sf, x)) <= G * (1 + 1e-12)
    assert np.min(c * x) >= t * (1 - 1e-12)
    if mu == 0.0:  # capacity binds: the unique optimum
        assert np.allclose(x, t / c, rtol=0, atol=1e-15)
    else:  # analytic centre: stationarity of the barrier on the free jobs
        free = c > t
        slack = G - float(np.dot(sf, x))
        assert abs(mu * slack - 1.0) < 1e-9
        xf, cf, sff = x[free], c[free], sf[free]
        h = 1 / xf - 1 / (1 - xf) + cf / (cf * xf - t) - sff * mu
        scale = 1 / xf + 1 / (1 - xf) + cf / (cf * xf - t)
        assert np.all(np.abs(h) <= 1e-9 * scale)
        assert np.all(x[~free] == 1.0)


@pytest.mark.parametrize("case", range(len(instances())))
def test_twin_level_matches_lp(case):
    sf, c, G = instances()[case]
    x, t, mu = mmf_ref.twin_allocate(sf, c, G)
    check_lp_optimal(sf, c, G, x, t, mu)


def test_twin_empty_and_deterministic():
    x, t, mu = mmf_ref.twin_allocate([], [], 8)
    assert len(x) == 0 and t == 0.0
    sf, c, G = instances()[5]
    a = mmf_ref.twin_allocate(sf, c, G)
    b = mmf_ref.twin_allocate(sf, c, G)
    assert a[0].tobytes() == b[0].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(instances())))
def test_gpu_mmf_bit_exact_vs_twin(gpu_solver, case):
    sf, c, G = instances()[case]
    xg, tg, mug = gpu_solver.mmf_allocate(sf, c, G)
    # the HIP allocation itself against the reference LP (not only the twin)
    check_lp_optimal(sf, c, G, xg, tg, mug)
    xt, tt, mut = mmf_ref.twin_allocate(sf, c, G)
    assert xg.tobytes() == xt.tobytes()
    assert np.float64(tg).tobytes() == np.float64(tt).tobytes()
    assert np.float64(mug).tobytes() == np.float64(mut).tobytes()


@pytest.mark.gpu
def test_gpu_mmf_rejects_bad_input(gpu_solver):
    import sw_native as sn
    with pytest.raises(sn.NativeError):
        gpu_solver.mmf_allocate([1, 0], [1.0, 1.0], 4)
    with pytest.raises(sn.NativeError):
        gpu_solver.mmf_allocate([1, 1], [1.0, -1.0], 4)


def fuzz_instances(n_cases, seed=11, max_n=5000):
    """Random MaxMinFairness inputs: sizes 1..max_n (log-uniform), clusters of
    1..2048 GPUs, scale factors from the traces or up to 255, coefficients over
    six decades, exact duplicates."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_cases):
        n = int(np.exp(rng.uniform(0.0, np.log(max_n + 1))))
        n = max(1, min(n, max_n))
        G = int(np.exp(rng.uniform(0.0, np.log(2049))))
        if rng.random() < 0.7:
            sf = rng.choice([1, 2, 4, 8], size=n, p=rng.dirichlet(np.ones(4)))
        else:
            sf = rng.integers(1, 256, size=n)
        c = 10.0 ** rng.uniform(-3, 3, size=n)
        if n >= 4 and rng.random() < 0.5:
            k = int(rng.integers(1, n // 2 + 1))
            dst, src = rng.integers(0, n, size=k), rng.integers(0, n, size=k)
            sf[dst], c[dst] = sf[src], c[src]
        out.append((sf.astype(np.int32), c, G))
    return out


def test_twin_level_matches_lp_fuzz():
    for sf, c, G in fuzz_instances(200, seed=5, max_n=300):
        x, t, mu = mmf_ref.twin_allocate(sf, c, G)
        check_lp_optimal(sf, c, G, x, t, mu)


@pytest.mark.gpu
def test_gpu_mmf_fuzz_bit_exact_vs_twin(gpu_solver):
    for i, (sf, c, G) in enumerate(fuzz_instances(300)):
        xg, tg, mug = gpu_solver.mmf_allocate(sf, c, G)
        if len(sf) <= 1000 and i % 3 == 0:  # the LP check on a third (HiGHS time)
            check_lp_optimal(sf, c, G, xg, tg, mug)
        xt, tt, mut = mmf_ref.twin_allocate(sf, c, G)
        assert xg.tobytes() == xt.tobytes(), (i, len(sf), G)
        assert np.float64(tg).tobytes() == np.float64(tt).tobytes(), (i, len(sf), G)
        assert np.float64(mug).tobytes() == np.float64(mut).tobytes(), (i, len(sf), G)
