"""The P2 placement cascade on the GPU: batched kernel (on-chip and
HBM-workspace paths) and the sharded engine against the CPU twin, bit for bit,
on the captured simulator instances (tests/golden/p2_cases.json)."""
import pytest

from helpers import assert_same_result, check_plan_valid
from p2cases import arrays, load_cases
from test_gpu_shard import gpu_shard_threads
from test_shard import assert_same_as_single

pytestmark = pytest.mark.gpu
CASES = load_cases()


@pytest.mark.parametrize("i", range(len(CASES)))
def test_gpu_p2_cascade_matches_twin(gpu_solver, twin, i):
    a = arrays(CASES[i])
    rg, rt = gpu_solver.solve(a), twin.solve(a)
    check_plan_valid(a, rg)
    assert_same_result(rg, rt, f"case {i} ({CASES[i]['kind']})")


@pytest.mark.parametrize("i", [4, 5, 12, 14])
def test_gpu_p2_cascade_tiled_matches_twin(gpu_solver, twin, i):
    """×8 tiles: N > 1024 for cases 4 and 5 (HBM-workspace path, class-wise)."""
    a = arrays(CASES[i], 8)
    rg, rt = gpu_solver.solve(a), twin.solve(a)
    check_plan_valid(a, rg)
    assert_same_result(rg, rt, f"case {i} x8")


def test_gpu_p2_batched_mixed(gpu_solver, twin):
    batch = [arrays(c) for c in CASES]
    for a, rg in zip(batch, gpu_solver.solve_batch(batch)):
        assert_same_result(rg, twin.solve(a), "batched")


@pytest.mark.parametrize("i,tile,world", [(3, 1, 2), (6, 1, 2), (4, 8, 2)])
def test_gpu_shard_p2_cascade(twin, i, tile, world):
    a = arrays(CASES[i], tile)
    assert_same_as_single(gpu_shard_threads(a, world), twin.solve(a), f"case {i} x{tile} W={world}")
