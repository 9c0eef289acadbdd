"""The CPU twin over the fuzz instances (tests/fuzzcases.py) that
tests/test_gpu_fuzz.py compares the GPU against: every input the validator
accepts gives a valid schedule, and a repeated solve is bit-identical."""
from fuzzcases import fuzz_problem
from helpers import assert_same_result, check_plan_valid


def test_twin_fuzz_plans_valid(twin):
    for s in range(0, 4096, 4):
        a = fuzz_problem(s)
        r = twin.solve(a)
        check_plan_valid(a, r)
        if s % 64 == 0:
            assert_same_result(r, twin.solve(a), f"seed {s}")


def test_twin_fuzz_workspace_sizes_valid(twin):
    for s in range(0, 48, 4):
        a = fuzz_problem(100_000 + s, max_n=3000, min_n=1025)
        check_plan_valid(a, twin.solve(a))
