"""Generate tests/golden/sim_milp_220.json: Fig-9 simulation metrics of the
220-job trace with the Shockwave plan solved by the MILP restatement of the
reference solve (oracle/milp_ref.py: HiGHS, gap 1e-3, 15 s per MILP, as
scale_*gpus.json), at 64 / 128 / 256 GPUs — the oracle run the simulator
parity test compares against.  At 64 GPUs the MILP is also run at gap 1e-4:
the spread between the two is the MILP path's own run-to-run variability.

    python tests/golden/make_sim_milp.py        (≈ 6 min on one core)
"""
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "oracle")]
import milp_ref  # noqa: E402
import sw_sim  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sim_milp_220.json")
TRACE = os.path.join(ROOT, "data", "traces",
                     "220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace")
KEYS = ("makespan", "avg_jct", "worst_ftf", "unfair_fraction", "rounds", "solves", "jobs_completed")


def main():
    out = {}
    for g, gap in ((256, 1e-3), (128, 1e-3), (64, 1e-3), (64, 1e-4)):
        cfg = json.load(open(os.path.join(ROOT, "data", "configs", f"scale_{g}gpus.json")))
        t0 = time.time()
        with contextlib.redirect_stdout(io.StringIO()):
            r = sw_sim.run_trace("shockwave", TRACE, g, 120, cfg,
                                 shockwave_solver=milp_ref.MilpSolver(rel_gap=gap))
        out[f"{g}_gap{gap:g}"] = {k: r[k] for k in KEYS}
        print(g, gap, round(time.time() - t0), out[f"{g}_gap{gap:g}"], flush=True)
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
