"""Diagnostics: one small sharded solve at world 1 (RCCL) with the fast
path's stage trace (SW_FAST_TRACE=1), compared with the twin."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

a = ss.synth_problem(0, 12, 4, 6, 120.0, 1e5, 5.0)
s = sn.Solver(device=0)
s.dist_init(sn.unique_id(), 0, 1)
print("init ok", flush=True)
r = s.dist_solve(a, 0, a.N)
print("solved", r["objective"], r["status"], r["iters"], flush=True)
