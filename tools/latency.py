"""Single-instance plan-solve latency (the scheduler's call pattern) on
simulator-captured instances (tests/golden/p2_cases.json) and C3 instances."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402
from p2cases import arrays, load_cases  # noqa: E402


def lat(s, a, reps=20):
    s.upload([a])
    s.run()
    s.download()
    t0 = time.perf_counter()
    for _ in range(reps):
        s.run()
    s.download()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    s = sn.Solver(device=0)
    out = {"sim_cases_ms": [], "c3_ms": []}
    for c in load_cases():
        out["sim_cases_ms"].append((c["kind"], len(c["w"]), round(lat(s, arrays(c)), 4)))
    for i in range(8):
        out["c3_ms"].append(round(lat(s, ss.c3_problem(i)), 4))
    out["sim_mean_ms"] = float(np.mean([x[2] for x in out["sim_cases_ms"]]))
    out["c3_mean_ms"] = float(np.mean(out["c3_ms"]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
