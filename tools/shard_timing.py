"""Time one C4-shaped instance (10k jobs × 30 rounds) on one GPU:
the sharded engine at world 1 (RCCL), the sharded engine at W ranks on the
same GPU with host collectives (threads), and the batched kernel (one
workgroup, HBM-workspace path).  Prints JSON lines."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "tests")]
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    c = ss.C4
    for N in (900, c["N"]):
        G = 256 if N == 900 else c["G"]
        a = ss.synth_problem(5, N, G, 30, 120.0, 1e5, 5.0)
        s = sn.Solver(device=0)
        s.dist_init(sn.unique_id(), 0, 1)
        r = s.dist_solve(a, 0, a.N)
        t = time.perf_counter()
        for _ in range(reps):
            r = s.dist_solve(a, 0, a.N)
        dt = (time.perf_counter() - t) / reps
        s.close()
        b = sn.Solver(device=0)
        rb = b.solve(a)
        t = time.perf_counter()
        for _ in range(reps):
            rb = b.solve(a)
        db = (time.perf_counter() - t) / reps
        b.close()
        same = bool((r["plan"] == rb["plan"]).all() and r["objective"] == rb["objective"])
        print(json.dumps({"N": N, "shard_w1_rccl_ms": dt * 1e3, "steps": r["iters"],
                          "ms_per_step": dt * 1e3 / max(r["iters"], 1),
                          "batched_kernel_ms": db * 1e3, "identical": same}), flush=True)


if __name__ == "__main__":
    main()
