"""The per-round re-optimisation (k_rr, sw_reround_dev.h) on re-solved
(SW_STATUS_P1_REPACKED) 10,000-job instances through the sharded engine at
world 1: small clusters with wide jobs, the only C4-size shape
that re-solves.  Prints the wall time per solve; run under rocprofv3
--kernel-trace --stats for k_rr's share.
    python tools/rr_c4.py [solves]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
s = sn.Solver(device=0)
s.dist_init(sn.unique_id(), 0, 1)
out = []
for (seed, G, T) in [(1, 12, 12), (1, 13, 30)]:
    a = ss.synth_problem(seed, 10000, G, T, 120.0, 1.0, 5.0, width_p=(0.4, 0.3, 0.2, 0.1))
    r = s.dist_solve(a, 0, a.N)
    t0 = time.perf_counter()
    for _ in range(n):
        r = s.dist_solve(a, 0, a.N)
    dt = (time.perf_counter() - t0) / n
    out.append({"seed": seed, "N": a.N, "G": G, "T": T, "status": r["status"],
                "repacked": bool(r["status"] & sn.SW_STATUS_P1_REPACKED), "steps": r["iters"],
                "ms_per_solve": dt * 1e3})
s.close()
print(json.dumps(out))
