"""The simulator on the GPU: the HIP plan kernel and the HIP MaxMinFairness
kernel inside the round loop give exactly the metrics of the same loop run
with their CPU twins (bit-exact kernels ⇒ identical schedules ⇒ identical
simulations)."""
import contextlib
import io
import json
import os

import pytest

import mmf_ref
import sw_native as sn
import sw_sim
import sw_trace as st

TRACES = {
    120: "120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace",
    220: "220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace",
}
CFG64 = json.load(open(os.path.join(st.DATA_DIR, "configs", "scale_64gpus.json")))


def sim(policy, trace, gpus, solver, mmf):
    with contextlib.redirect_stdout(io.StringIO()):
        return sw_sim.run_trace(policy, os.path.join(st.DATA_DIR, "traces", TRACES[trace]), gpus,
                                120, CFG64, shockwave_solver=solver, mmf_allocator=mmf)


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["shockwave", "max_min_fairness"])
@pytest.mark.parametrize("trace,gpus", [(120, 64), (220, 64)])
def test_gpu_simulation_equals_twin_simulation(gpu_solver, twin, policy, trace, gpus):
    g = sim(policy, trace, gpus, gpu_solver, sn.MmfAllocator(solver=gpu_solver))
    c = sim(policy, trace, gpus, twin, mmf_ref.twin_allocator)
    for k in ("makespan", "avg_jct", "worst_ftf", "unfair_fraction", "rounds", "solves",
              "jobs_completed"):
        assert g[k] == c[k], (k, g[k], c[k])
