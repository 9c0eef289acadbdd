"""Small helpers shared by tests (no product logic)."""
import numpy as np

import milp_ref as mr


def to_oracle(a):
    """ProblemArrays → oracle Problem (same numbers)."""
    return mr.Problem(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, list(a.bases))


def assert_same_result(r1, r2, what=""):
    """Bit-exact equality of two solver results (plan, counts, every scalar)."""
    assert r1["status"] == r2["status"], f"{what}: status {r1['status']} vs {r2['status']}"
    assert np.array_equal(r1["planned_rounds"], r2["planned_rounds"]), f"{what}: counts differ"
    assert np.array_equal(r1["plan"], r2["plan"]), f"{what}: plans differ"
    for key in ("objective", "utility", "makespan", "p2_objective", "bound"):
        a, b = r1[key], r2[key]
        assert np.float64(a).tobytes() == np.float64(b).tobytes(), f"{what}: {key} {a!r} vs {b!r}"
    assert r1["iters"] == r2["iters"], f"{what}: iters {r1['iters']} vs {r2['iters']}"


def check_plan_valid(a, r):
    """Plan is 0/1, respects per-round capacity, counts match, no job wider than G."""
    y = r["plan"]
    assert y.shape == (a.N, a.T)
    assert set(np.unique(y)).issubset({0, 1})
    load = (y.astype(np.int64) * a.w[:, None]).sum(axis=0)
    assert np.all(load <= a.G), f"capacity violated: {load.max()} > {a.G}"
    assert np.array_equal(y.sum(axis=1), r["planned_rounds"])
