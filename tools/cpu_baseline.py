"""The CPU comparators of SURVEY.md §8(d), measured on the host this runs on.

    python tools/cpu_baseline.py [--procs 16] [--instances 16] [--out profiles/<tag>_cpu_baseline.json]

All three time the repo's HiGHS restatement of the reference MILPs
(oracle/milp_ref.py; test infrastructure, never the product path) on C3-shaped
instances (900 jobs x 30 rounds, G = 256, k = 1e5, lambda = 5):
  (i)   latency: one process, P1 + P2 MILPs (gap 1e-3, 15 s limit per MILP as
        scale_*gpus.json), wall clock including model build;
  (ii)  the LP relaxation of P1 alone (x, z continuous) — a stronger, looser
        comparator: it returns fractional counts, no plan;
  (iii) all-cores throughput: one process per core on independent instances
        (C5-style replicas), completed instances / wall clock.
A solve whose P1 MILP finds no incumbent within its limit is the reference's
AssertionError (shockwave.py:382): it is recorded and not counted as a solve.
The host's CPU model and core counts are recorded with the numbers.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))


def _problem(seed):
    import milp_ref as mr
    import sw_synth as ss
    a = ss.synth_problem(10_000 + seed, 900, 256, 30, 120.0, 1e5, 5.0)
    return mr.Problem(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, list(a.bases))


def _solve(seed):
    import milp_ref as mr
    P = _problem(seed)
    t0 = time.perf_counter()
    try:
        sol = mr.plan_solve(P, rel_gap=1e-3, time_limit=15.0)
    except AssertionError:  # no P1 incumbent within the limit (shockwave.py:382)
        return time.perf_counter() - t0, "no_solution", None
    return time.perf_counter() - t0, sol.status, sol.p2_status


def _relax(seed):
    import milp_ref as mr
    P = _problem(seed)
    t0 = time.perf_counter()
    try:
        st, _x, obj, _bound, _t = mr.solve_p1(P, 1e-3, 120.0, relax=True)
    except AssertionError:
        return time.perf_counter() - t0, "no_solution", None
    return time.perf_counter() - t0, st, obj


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def one(mode, seed):
    """Worker mode for bench.py's cpu_baseline leg: one timed solve (or LP
    relaxation) of one seed, printed as one JSON line."""
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ.setdefault(k, "1")
    dt, st, extra = (_solve if mode == "solve" else _relax)(seed)
    print(json.dumps({"mode": mode, "seed": seed, "seconds": dt, "status": st,
                      "p2_status" if mode == "solve" else "objective": extra}))


def main():
    if len(sys.argv) == 3 and sys.argv[1] in ("--one", "--relax"):
        return one("solve" if sys.argv[1] == "--one" else "relax", int(sys.argv[2]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--instances", type=int, default=16)
    ap.add_argument("--latency-runs", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[k] = "1"  # one core per process for (iii); HiGHS MIP is serial anyway
    host = {"cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0))}
    lat = [_solve(s) for s in range(args.latency_runs)]
    rel = [_relax(s) for s in range(args.latency_runs)]
    procs = max(1, min(args.procs, host["affinity"]))
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(procs) as pool:
        many = pool.map(_solve, range(100, 100 + args.instances))
    wall = time.perf_counter() - t0
    out = {
        "host": host,
        "workload": "C3: 900 jobs x 30 rounds, G=256, k=1e5, lambda=5 (sw_synth seeds 10000+)",
        "latency": {"seconds": [r[0] for r in lat], "mean_s": sum(r[0] for r in lat) / len(lat),
                    "status": [[r[1], r[2]] for r in lat],
                    "plan_solves_per_s": sum(r[1] != "no_solution" for r in lat) / sum(r[0] for r in lat),
                    "cores": 1},
        "lp_relaxation_p1": {"seconds": [r[0] for r in rel], "mean_s": sum(r[0] for r in rel) / len(rel),
                             "status": [r[1] for r in rel],
                             "note": "P1 with x and the SOS2 binaries continuous; no rounding, no P2"},
        "all_cores": {"processes": procs, "instances": args.instances, "wall_s": wall,
                      "completed": sum(r[1] != "no_solution" for r in many),
                      "plan_solves_per_s": sum(r[1] != "no_solution" for r in many) / wall,
                      "per_instance_s": [r[0] for r in many],
                      "status": sorted({f"{r[1]}/{r[2]}" for r in many})},
    }
    txt = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
