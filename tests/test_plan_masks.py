"""The bit-packed plan of ABI 2 (sw_result.plan_masks, include/shockwave_amd.h):
the CPU twin writes it too, so its layout (bit t of job j's word = plan[j][t])
is pinned here without a GPU; the GPU side is tests/test_gpu_host_boundary.py."""
import ctypes

import numpy as np
import pytest

import sw_native as sn
import sw_synth as ss
from conftest import TWIN_SO, _build_twin


def pack_bits(plan: np.ndarray) -> np.ndarray:
    w = np.uint64(1) << np.arange(plan.shape[1], dtype=np.uint64)
    return (plan.astype(np.uint64) * w[None, :]).sum(axis=1, dtype=np.uint64)


@pytest.mark.parametrize("seed,N,G,T", [(0, 40, 16, 10), (1, 300, 64, 30), (2, 12, 8, 64), (3, 0, 8, 5)])
def test_twin_plan_masks_match_plan_bytes(seed, N, G, T):
    _build_twin()
    lib = ctypes.CDLL(TWIN_SO)
    sn.declare_solver_api(lib, "twin_")
    a = ss.synth_problem(seed, N, G, T, 120.0, 1e1, 5.0)
    pr, res = a.c_problem(), a.c_result()
    masks = np.full(max(N, 1), 0xDEAD, dtype=np.uint64)
    res.plan_masks = masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    assert lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res)) >= 0
    assert np.array_equal(masks[:N], pack_bits(a.plan))
    if N == 0:
        assert masks[0] == 0xDEAD  # nothing written past the jobs
