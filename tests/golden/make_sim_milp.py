"""Generate the MILP-oracle simulation fixtures: Fig-9 metrics with every
Shockwave plan solved by the MILP restatement of the reference solve
(oracle/milp_ref.py: HiGHS, gap 1e-3, 15 s per MILP, as scale_*gpus.json).

    python tests/golden/make_sim_milp.py [--procs 6] [--only KEY,...]

Files and runs (KEY = what the parity tests look up):
  sim_milp_220.json   the 220-job trace (replicated Fig-9):
      "{G}_gap0.001"          G = 64, 128, 256
      "64_gap0.0001"          the same at gap 1e-4
      "64_gap0.001_perm{s}"   s = 1..5: the SAME model with its jobs in a
                              seeded random order (MilpSolver(perm_seed=s)).
                              HiGHS then stops at a different solution inside
                              the same gap; the spread of these runs is the
                              oracle's own indeterminacy at 64 GPUs.
  sim_milp_120.json   the 120-job trace:
      "C2_64", "C2_64_perm{s}"   BASELINE config 2 (64 GPUs, 120 jobs)
      "C1_32", "C1_32_perm{s}"   BASELINE config 1: the first 50 jobs on 32
                                 GPUs (no 50-job trace or 32-GPU JSON exists:
                                 SURVEY.md §8(d); scale_64gpus.json is used)
Each record also keeps the per-job completion times.
"""
import argparse
import contextlib
import io
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "oracle")]
HERE = os.path.dirname(os.path.abspath(__file__))
T220 = "220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
T120 = "120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
KEYS = ("makespan", "avg_jct", "worst_ftf", "unfair_fraction", "rounds", "solves",
        "jobs_completed", "jcts")

# (file, key, trace, gpus, config gpus, max_jobs, gap, perm_seed)
RUNS = ([("sim_milp_220.json", f"{g}_gap0.001", T220, g, g, None, 1e-3, None) for g in (256, 128, 64)]
        + [("sim_milp_220.json", "64_gap0.0001", T220, 64, 64, None, 1e-4, None)]
        + [("sim_milp_220.json", f"64_gap0.001_perm{s}", T220, 64, 64, None, 1e-3, s)
           for s in range(1, 6)]
        + [("sim_milp_120.json", "C2_64", T120, 64, 64, None, 1e-3, None)]
        + [("sim_milp_120.json", f"C2_64_perm{s}", T120, 64, 64, None, 1e-3, s) for s in range(1, 4)]
        + [("sim_milp_120.json", "C1_32", T120, 32, 64, 50, 1e-3, None)]
        + [("sim_milp_120.json", f"C1_32_perm{s}", T120, 32, 64, 50, 1e-3, s) for s in range(1, 4)])


def run(spec):
    import milp_ref
    import mmf_ref
    import sw_sim

    fname, key, trace, g, cg, max_jobs, gap, perm = spec
    cfg = json.load(open(os.path.join(ROOT, "data", "configs", f"scale_{cg}gpus.json")))
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        r = sw_sim.run_trace("shockwave", os.path.join(ROOT, "data", "traces", trace), g, 120, cfg,
                             shockwave_solver=milp_ref.MilpSolver(rel_gap=gap, perm_seed=perm),
                             mmf_allocator=mmf_ref.twin_allocator, max_jobs=max_jobs)
    rec = {k: r[k] for k in KEYS}
    rec.update({"trace": trace, "gpus": g, "config": f"scale_{cg}gpus.json", "max_jobs": max_jobs,
                "gap": gap, "perm_seed": perm, "seconds": time.time() - t0})
    print(fname, key, round(rec["seconds"]), rec["makespan"], rec["avg_jct"], rec["worst_ftf"],
          flush=True)
    return fname, key, rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=6)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    runs = [r for r in RUNS if not args.only or r[1] in args.only.split(",")]
    with mp.get_context("spawn").Pool(args.procs) as pool:
        done = pool.map(run, runs, chunksize=1)
    for fname in sorted({d[0] for d in done}):
        path = os.path.join(HERE, fname)
        out = json.load(open(path)) if os.path.exists(path) else {}
        for f, key, rec in done:
            if f == fname:
                out[key] = rec
        json.dump(out, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
