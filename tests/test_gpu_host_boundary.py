"""The host boundary of sw_plan_solve_batch: the bit-packed plan option
(sw_result.plan_masks, ABI 2) and the chunk pipeline large on-chip batches
take (sw_api.hip solve_pipelined: H2D, kernels and D2H of neighbouring chunks
overlapped, host staging and unpacking in parallel threads).  Results must be
the device-resident path's (sw_batch_upload / run / download, one launch) and
the twin's, bit for bit."""
import numpy as np
import pytest

from fuzzcases import fuzz_problem
from helpers import assert_same_result, check_plan_valid

pytestmark = pytest.mark.gpu


def pack_bits(plan: np.ndarray) -> np.ndarray:
    T = plan.shape[1]
    w = (np.uint64(1) << np.arange(T, dtype=np.uint64))
    return (plan.astype(np.uint64) * w[None, :]).sum(axis=1, dtype=np.uint64)


def onchip(n: int, seed0: int) -> list:
    out, s = [], seed0
    while len(out) < n:
        a = fuzz_problem(s)
        s += 1
        if a.T <= 32:
            out.append(a)
    return out


def test_gpu_plan_masks_match_plan_bytes_and_twin(gpu_solver, twin):
    probs = onchip(300, 300_000)
    rb = gpu_solver.solve_batch(probs, masks=True)
    for i, (a, r) in enumerate(zip(probs, rb)):
        assert np.array_equal(r["plan_masks"], pack_bits(r["plan"])), f"case {i}"
        rt = twin.solve(a)
        assert_same_result(r, rt, f"case {i}")
        assert np.array_equal(r["plan_masks"], pack_bits(rt["plan"])), f"case {i} vs twin"


def test_gpu_masks_only_leaves_plan_untouched(gpu_solver):
    probs = onchip(64, 310_000)
    for a in probs:
        a.plan[:] = 7
    rb = gpu_solver.solve_batch(probs, masks=True, plan=False)
    ref = gpu_solver.solve_batch(probs)
    for a, r, q in zip(probs, rb, ref):
        assert np.array_equal(r["plan_masks"], pack_bits(q["plan"]))
        assert r["objective"] == q["objective"] and r["status"] == q["status"]


def test_gpu_pipelined_batch_matches_device_resident_and_twin(gpu_solver, twin):
    """4,608 on-chip instances: at least two 2,048-instance chunks through the
    pipeline (SW_PIPELINE_CHUNKS default 4, ≥ 2,048 per chunk)."""
    probs = onchip(4608, 320_000)
    rp = gpu_solver.solve_batch(probs, masks=True)
    gpu_solver.upload(probs)
    gpu_solver.run()
    rd = gpu_solver.download()
    for i, (a, p, d) in enumerate(zip(probs, rp, rd)):
        assert_same_result(p, d, f"pipelined vs resident, case {i}")
        assert np.array_equal(p["plan_masks"], pack_bits(d["plan"])), f"case {i}"
    for i in range(0, len(probs), 16):
        check_plan_valid(probs[i], rp[i])
        assert_same_result(rp[i], twin.solve(probs[i]), f"pipelined vs twin, case {i}")


def test_gpu_pipelined_invalid_problem_names_index_and_keeps_batch(gpu_solver):
    import sw_native as sn

    probs = onchip(4608, 330_000)
    gpu_solver.upload(probs[:8])
    gpu_solver.run()
    before = gpu_solver.download()
    bad = probs[3001]
    bad.w[0] = 0  # nworkers < 1
    with pytest.raises(sn.NativeError, match="index 3001"):
        gpu_solver.solve_batch(probs)
    gpu_solver.run()  # the previously uploaded batch is still described
    after = gpu_solver.download()
    for b, c in zip(before, after):
        assert_same_result(b, c, "batch kept")


def test_gpu_pipelined_batch_with_empty_instances_and_no_outputs(gpu_solver, twin):
    """Empty instances (no jobs) anywhere in a pipelined batch, chunk
    boundaries included, and a call that asks for no per-job outputs at all
    (plan = plan_masks = planned_rounds = NULL): every result field still
    matches the twin."""
    import ctypes

    import sw_native as sn
    import sw_synth as ss

    probs = onchip(4608, 340_000)
    for i in list(range(0, 4608, 97)) + [2303, 2304, 4607]:
        probs[i] = ss.synth_problem(i, 0, 16, 10, 120.0, 1.0, 5.0)
    rb = gpu_solver.solve_batch(probs)
    for i in range(0, 4608, 7):
        assert_same_result(rb[i], twin.solve(probs[i]), f"case {i} N={probs[i].N}")
    cp = (sn.SwProblem * len(probs))(*[a.c_problem() for a in probs])
    cr = (sn.SwResult * len(probs))()
    assert gpu_solver.lib.sw_plan_solve_batch(gpu_solver.h, len(probs), cp, cr) >= 0
    for i in range(0, 4608, 7):
        assert cr[i].objective == rb[i]["objective"] and cr[i].status == rb[i]["status"], i
        assert cr[i].p2_objective == rb[i]["p2_objective"], i


def test_gpu_resident_split_batch_keep_masks(gpu_solver, twin):
    """The split kernels' pack tail (sw_kernels.hip pack_tail: the exchange
    step's arrays in LDS, the masks stored only when kept): a 600-instance
    device-resident batch gives the same plans and results with and without
    the masks, the kept masks are the plan bytes packed, and a download that
    asks for masks after a run that did not keep them is refused."""
    import sw_native as sn

    probs = onchip(600, 350_000)
    gpu_solver.upload(probs)
    gpu_solver.keep_masks(True)
    gpu_solver.run()
    with_m = gpu_solver.download(masks=True)
    gpu_solver.keep_masks(False)
    gpu_solver.run()
    without = gpu_solver.download()
    with pytest.raises(sn.NativeError, match="plan_masks"):
        gpu_solver.download(masks=True)
    gpu_solver.keep_masks(True)
    for i, (a, m, n) in enumerate(zip(probs, with_m, without)):
        assert_same_result(m, n, f"case {i}")
        assert np.array_equal(m["plan_masks"], pack_bits(m["plan"])), f"case {i}"
    for i in range(0, len(probs), 5):
        assert_same_result(without[i], twin.solve(probs[i]), f"case {i} vs twin")
