"""The simulator on the GPU: the HIP plan kernel and the HIP MaxMinFairness
kernel inside the round loop give exactly the metrics of the same loop run
with their CPU twins (bit-exact kernels ⇒ identical schedules ⇒ identical
simulations).  Cases: BASELINE C1 (the 120-job trace's first 50 jobs on 32
GPUs), C2 (the 120-job trace on 64 GPUs) and the 220-job Fig-9 trace; the
twin simulations are held to the MILP-oracle envelope in test_sim_parity.py."""
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


def sim(policy, trace, gpus, solver, mmf, max_jobs=None):
    with contextlib.redirect_stdout(io.StringIO()):
        return sw_sim.run_trace(policy, os.path.join(st.DATA_DIR, "traces", TRACES[trace]), gpus,
                                120, CFG64, shockwave_solver=solver, mmf_allocator=mmf,
                                max_jobs=max_jobs)


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["shockwave", "max_min_fairness"])
@pytest.mark.parametrize("trace,gpus,max_jobs", [(120, 32, 50), (120, 64, None), (220, 64, None)],
                         ids=["C1_50jobs_32gpus", "C2_120jobs_64gpus", "fig9_220jobs_64gpus"])
def test_gpu_simulation_equals_twin_simulation(gpu_solver, twin, policy, trace, gpus, max_jobs):
    g = sim(policy, trace, gpus, gpu_solver, sn.MmfAllocator(solver=gpu_solver), max_jobs)
    c = sim(policy, trace, gpus, twin, mmf_ref.twin_allocator, max_jobs)
    for k in ("makespan", "avg_jct", "worst_ftf", "unfair_fraction", "rounds", "solves",
              "jobs_completed"):
        assert g[k] == c[k], (k, g[k], c[k])
