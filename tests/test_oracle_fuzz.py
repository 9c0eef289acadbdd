"""The plan algorithm (CPU twin, bit-identical to the GPU kernel and the
sharded engine) against the MILP oracle on random instances
(tests/fuzzcases.py, widths from the reference traces' {1, 2, 4, 8}).

Inside the reference's regime (clusters of ≥ 32 GPUs, scale_{32..256}gpus.json)
every instance must be within the north star's 1e-3 of the MILP optimum: 307
instances (N ≤ 60, T ≤ 12, any k, λ, base grid, duplicates, finished jobs).
Below it, width fragmentation is the recorded exception:
measured over the first 1,300 seeds at N ≤ 80, T ≤ 12, 1 of 1,057 instances
with G ≥ 2·max width exceeds 1e-3 (G = 22: 2.8e-3), and 4 of 175 with
G < 2·max width (worst 6.8e-2)."""
import pytest

import milp_ref as mr
import sw_native as sn
from fuzzcases import fuzz_problem
from helpers import check_plan_valid, to_oracle

REL_TOL = 1e-3


def _reference_regime(lo, hi, max_n=60, max_t=12):
    out = []
    for s in range(lo, hi):
        b = fuzz_problem(s, max_n=max_n, trace_widths=True)
        if b.G < 32:
            continue
        out.append((s, sn.ProblemArrays(b.w, b.d, b.F, b.E, b.R, b.p, min(b.T, max_t), b.G,
                                        b.delta, b.k, tuple(b.bases))))
    return out


@pytest.mark.parametrize("block", range(8))
def test_twin_within_1e3_of_milp_on_fuzz(block, twin):
    cases = _reference_regime(60 * block, 60 * block + 60)
    unsolved = 0
    for s, a in cases:
        P = to_oracle(a)
        try:
            sol = mr.plan_solve(P, rel_gap=1e-6, time_limit=30)
        except AssertionError:  # HiGHS gives up on badly scaled objectives (p up to 1e25)
            unsolved += 1
            continue
        ref = mr.evaluate_counts(P, sol.n)[0]
        r = twin.solve(a)
        check_plan_valid(a, r)
        got = mr.evaluate_counts(P, r["planned_rounds"])[0]
        assert got >= ref - REL_TOL * abs(ref), (s, a.N, a.G, a.T, a.k, got, ref)
    assert unsolved <= len(cases) // 10, (unsolved, len(cases))
