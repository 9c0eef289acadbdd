"""The P2 placement cascade on the GPU: batched kernel (on-chip and
HBM-workspace paths) against the CPU twin, and the sharded engine against the
CPU shard engine, bit for bit, on the captured simulator instances
(tests/golden/p2_cases.json)."""
import pytest

from helpers import assert_same_result, check_plan_valid
from p2cases import arrays, load_cases
from test_gpu_shard import gpu_shard_threads
from test_shard import assert_same_as_single, assert_share_contract, run_threads, shard_lib  # noqa: F401

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
def test_gpu_shard_p2_cascade(shard_lib, twin, i, tile, world):  # noqa: F811
    """The sharded contract: the GPU shard engine equals the
    CPU shard engine at the same world size bit for bit; against the single
    instance, P1 bit for bit and the share placement's P2 within its ratio."""
    a = arrays(CASES[i], tile)
    rg = gpu_shard_threads(a, world)
    check_plan_valid(a, rg)
    what = f"case {i} x{tile} W={world}"
    assert_same_as_single(rg, run_threads(shard_lib, a, world), what)
    assert_share_contract(rg, twin.solve(a), what)
