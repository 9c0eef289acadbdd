"""C4-shaped instances other than the bench's seed: per seed, the sharded
solve at world 1 (RCCL, device-resident inputs) — ms per solve, collective
steps, status — to show how often the device-side common path (fast_solve,
DESIGN.md §7.2) applies.  python tools/c4_seeds.py [first] [count] [solves]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))

import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def main():
    import torch

    first = int(sys.argv[1]) if len(sys.argv) > 1 else 70
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    solves = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    c = ss.C4
    s = sn.Solver(device=0)
    s.dist_init(sn.unique_id(), 0, 1)
    out = []
    for seed in range(first, first + count):
        a = ss.synth_problem(seed, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
        shard = sn.DeviceShard(a, "cuda:0")
        for _ in range(3):
            r = s.dist_solve_dev(shard, 0, a.N)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(solves):
            r = s.dist_solve_dev(shard, 0, a.N)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / solves * 1e3
        out.append({"seed": seed, "ms_per_solve": ms, "collective_steps": r["iters"], "status": r["status"]})
        print(json.dumps(out[-1]), flush=True)
    s.close()


if __name__ == "__main__":
    main()
