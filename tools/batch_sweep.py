"""Batch-size sweep of the C3 plan kernel and single-instance latency per P2
placement kind (diagnostics for DESIGN.md §6).

    python tools/batch_sweep.py > gpurun_out/<tag>/batch_sweep.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def timed(solver, steps):
    solver.run()
    solver.download()
    t0 = time.perf_counter()
    for _ in range(steps):
        solver.run()
    solver.download()
    return (time.perf_counter() - t0) / steps


def main():
    out = {"batch": [], "kinds": []}
    pool = [ss.synth_problem(i, 900, 256, 30, 120.0, 1e5, 5.0) for i in range(4096)]
    for b in (64, 256, 512, 1024, 2048, 4096):
        s = sn.Solver(device=0)
        s.upload(pool[:b])
        dt = timed(s, 10)
        st = np.array([r["status"] for r in s.download()])
        out["batch"].append({"batch": b, "ms_per_step": dt * 1e3, "solves_per_s": b / dt,
                             "frac_weight": float(np.mean((st & 8) > 0)),
                             "frac_classwise": float(np.mean((st & 16) > 0))})
        print(json.dumps(out["batch"][-1]), flush=True)
        s.close()
    from p2cases import arrays, load_cases
    s = sn.Solver(device=0)
    for c in load_cases():
        a = arrays(c)
        s.upload([a])
        out["kinds"].append({"kind": c["kind"], "N": a.N, "ms": timed(s, 20) * 1e3})
    s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
