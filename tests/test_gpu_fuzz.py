"""Randomised GPU ↔ twin parity (tests/fuzzcases.py): 4,096 instances that
cover the validator's whole accepted range, solved as heterogeneous batches of
512 (mixed T, G, k, base grids and widths in one launch), plus 48 instances
above 1,024 jobs on the HBM-workspace path.  Every field of every result must
be bit-identical with oracle/plan_twin.c, and every plan must be a valid
schedule."""
import pytest

from fuzzcases import fuzz_problem
from helpers import assert_same_result, check_plan_valid

pytestmark = pytest.mark.gpu

CHUNK = 512


@pytest.mark.parametrize("chunk", range(8))
def test_gpu_fuzz_batches_match_twin(chunk, gpu_solver, twin):
    probs = [fuzz_problem(s) for s in range(chunk * CHUNK, (chunk + 1) * CHUNK)]
    rb = gpu_solver.solve_batch(probs)
    for i, (a, r) in enumerate(zip(probs, rb)):
        what = f"seed {chunk * CHUNK + i} N={a.N} G={a.G} T={a.T} k={a.k:g}"
        check_plan_valid(a, r)
        assert_same_result(r, twin.solve(a), what)


def test_gpu_fuzz_workspace_path_matches_twin(gpu_solver, twin):
    probs = [fuzz_problem(100_000 + s, max_n=3000, min_n=1025) for s in range(48)]
    rb = gpu_solver.solve_batch(probs)
    for i, (a, r) in enumerate(zip(probs, rb)):
        check_plan_valid(a, r)
        assert_same_result(r, twin.solve(a), f"seed {100_000 + i} N={a.N} G={a.G} T={a.T}")


@pytest.mark.parametrize("count", [600, 1100])
def test_gpu_fuzz_onchip_batch_paths_match_twin(count, gpu_solver, twin):
    """On-chip batches (T ≤ 32, N ≤ 1024) take one of three launch forms by
    size (sw_api.hip launch): up to 256 instances the full kernel with the
    exchange step fused (every single solve and small batch in this suite);
    600 here: the full kernel, then sw_p2x_kernel; more than 1,024 (1,100
    here): the split kernels (level search, pack, slow-path full kernel),
    then sw_p2x_kernel.  All must give the twin's results bit for bit."""
    probs = []
    s = 200_000
    while len(probs) < count:
        a = fuzz_problem(s)
        s += 1
        if a.T <= 32:
            probs.append(a)
    rb = gpu_solver.solve_batch(probs)
    for i, (a, r) in enumerate(zip(probs, rb)):
        check_plan_valid(a, r)
        assert_same_result(r, twin.solve(a), f"{count}-batch case {i} N={a.N} G={a.G} T={a.T}")


def test_gpu_split_pack_loop_widths_match_twin(gpu_solver, twin):
    """The split path's pack kernel runs its one-wave round loop with 2, 4, 6
    or 8 positions per lane by the instance's active-job count A
    (csrc/sw_pack.h sw_pack_rounds_one); one 1,100-instance batch of C3-shaped
    instances whose sizes put A in every one of those ranges (and above 512,
    where the slow-path kernel takes over), each instance bit-identical with
    the twin."""
    import sw_synth as ss
    sizes = [(60, 32), (150, 64), (300, 96), (420, 128), (600, 160), (900, 256), (1024, 384),
             (1024, 512)]
    probs = [ss.synth_problem(7000 + i, *sizes[i % len(sizes)]) for i in range(1100)]
    rb = gpu_solver.solve_batch(probs)
    ranges = set()
    for i, (a, r) in enumerate(zip(probs, rb)):
        check_plan_valid(a, r)
        assert_same_result(r, twin.solve(a), f"case {i} N={a.N} G={a.G}")
        act = int((r["planned_rounds"] > 0).sum())
        ranges.add(0 if act <= 128 else 1 if act <= 256 else 2 if act <= 384 else 3 if act <= 512 else 4)
    assert {0, 1, 2, 3, 4} <= ranges, ranges  # 4: more than 512, the slow-path kernel
