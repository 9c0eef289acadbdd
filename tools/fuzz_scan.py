"""List every fuzz instance (tests/fuzzcases.py) whose GPU result differs from
the twin's, with the fields that differ; batched and single solves.

    python tools/fuzz_scan.py [n_instances] [--single]
    python tools/fuzz_scan.py n_instances --onchip CHUNK   # T <= 32 only, CHUNK per batch

With --onchip every instance is on-chip (N <= 1024, T <= 32), so the launch
form follows the chunk size (sw_api.hip launch): <= 256 the full kernel with
the exchange step fused, > 256 the split kernels (level kernel, then the pack
kernel with the exchange step fused, then the full kernel with it for the
instances the pack kernel leaves).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("tests", "shockwave-replication_amd", "oracle")]
import fuzzcases as fz  # noqa: E402
import sw_native as sn  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libplan_twin.so"))
sn.declare_solver_api(lib, "twin_")


def twin(a):
    pr, res = a.c_problem(), a.c_result()
    rc = lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
    return sn.result_dict(res, a, rc)


def diff(r1, r2):
    out = []
    for k in ("status", "iters"):
        if r1[k] != r2[k]:
            out.append(f"{k} {r1[k]} vs {r2[k]}")
    if not np.array_equal(r1["planned_rounds"], r2["planned_rounds"]):
        out.append(f"counts differ at {np.flatnonzero(r1['planned_rounds'] != r2['planned_rounds'])[:8]}")
    elif not np.array_equal(r1["plan"], r2["plan"]):
        out.append("plans differ")
    for k in ("objective", "utility", "makespan", "p2_objective", "bound"):
        if np.float64(r1[k]).tobytes() != np.float64(r2[k]).tobytes():
            out.append(f"{k} {r1[k]!r} vs {r2[k]!r}")
    return out


def ablate(seeds):
    """Which generator feature a mismatch needs: re-solve each seed with one
    feature left out at a time."""
    s = sn.Solver(device=0)
    feats = ("done", "smalld", "r0", "p0", "dup", "bases", "done+dup")
    for seed in seeds:
        row = []
        for f in feats:
            a = fz.fuzz_problem(seed, off=tuple(f.split("+")))
            row.append(f"{f}:{'x' if diff(s.solve(a), twin(a)) else '.'}")
        print(f"seed {seed}: " + " ".join(row), flush=True)
    s.close()


def paths(seeds):
    """Each seed alone (on-chip path when N <= 1024 and T <= 32), next to an
    N = 1025 instance (workspace path, 32-key rows) and next to a T = 64
    instance (workspace path, 64-key rows)."""
    s = sn.Solver(device=0)
    big = fz.fuzz_problem(7, max_n=1025, min_n=1025)
    big = sn.ProblemArrays(big.w, big.d, big.F, big.E, big.R, big.p, 2, big.G, big.delta, big.k)
    t64 = sn.ProblemArrays([1], [10.0], [0], [5], [50.0], [1.0], 64, 4, 120.0, 1.0)
    for seed in seeds:
        a = fz.fuzz_problem(seed)
        rt = twin(a)
        out = []
        for name, mate in (("alone", None), ("ws32", big), ("ws64", t64)):
            if mate is not None and name == "ws32" and a.T > 32:
                out.append(f"{name}:-")
                continue
            r = s.solve(a) if mate is None else s.solve_batch([a, mate])[0]
            out.append(f"{name}:{'x' if diff(r, rt) else '.'}")
        print(f"seed {seed} N={a.N} G={a.G} T={a.T}: " + " ".join(out), flush=True)
    s.close()


def main():
    if "--paths" in sys.argv:
        return paths([int(x) for x in sys.argv[2].split(",")])
    if "--ablate" in sys.argv:
        return ablate([int(x) for x in sys.argv[2].split(",")])
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    single = "--single" in sys.argv
    chunk = int(sys.argv[sys.argv.index("--onchip") + 1]) if "--onchip" in sys.argv else 512
    seeds = list(range(n))
    if "--onchip" in sys.argv:
        seeds, s0 = [], 0
        while len(seeds) < n:
            if fz.fuzz_problem(s0).T <= 32:
                seeds.append(s0)
            s0 += 1
    s = sn.Solver(device=0)
    bad = 0
    iters = []  # (passes, seed, N, T, G, k): the search's pass count per instance
    for c0 in range(0, n, chunk):
        probs = [fz.fuzz_problem(i) for i in seeds[c0:c0 + chunk]]
        rb = [s.solve(a) for a in probs] if single else s.solve_batch(probs)
        for i, (a, r) in enumerate(zip(probs, rb)):
            iters.append((int(r["iters"]), seeds[c0 + i], a.N, a.T, a.G, float(a.k)))
            d = diff(r, twin(a))
            if d:
                bad += 1
                print(f"seed {seeds[c0 + i]} N={a.N} G={a.G} T={a.T} k={a.k:g} nb={len(a.bases)} "
                      f"wmax={a.w.max()}: " + "; ".join(d), flush=True)
        if (c0 // chunk + 1) % max(1, 4096 // chunk) == 0:
            print(f"... {c0 + chunk} solved, {bad} differ", flush=True)
    form = "single" if single else f"batched by {chunk}" + (" (on-chip)" if "--onchip" in sys.argv else "")
    print(f"{bad} of {n} differ ({form})", flush=True)
    # search passes (the searches' pass counts, worst cases first)
    its = np.array([x[0] for x in iters])
    print(f"passes per instance: mean {its.mean():.1f}, p50 {np.percentile(its, 50):.0f}, "
          f"p99 {np.percentile(its, 99):.0f}, max {its.max()}", flush=True)
    for x in sorted(iters, reverse=True)[:5]:
        print(f"  {x[0]} passes: seed {x[1]} N={x[2]} T={x[3]} G={x[4]} k={x[5]:g}", flush=True)
    s.close()


if __name__ == "__main__":
    main()
