"""One rank of the peer-transport test (tests/test_gpu_shard.py): a separate
process on cuda:0, host collectives over gloo for the setup, then
sw_dist_enable_peer so that every step's collective goes through the other
process's IPC-mapped exchange region.  Writes this rank's rows and the global
scalars of each case to <outdir>/c<case>_r<rank>.npz.

    python tests/peer_worker.py <rank> <world> <port> <outdir> <cases.json>
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))

SCALARS = ("objective", "utility", "makespan", "p2_objective", "bound")


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    outdir, cases = sys.argv[4], json.load(open(sys.argv[5]))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    import sw_native as sn
    import sw_synth as ss

    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = sn.Solver(device=0)
    s.dist_init_host(sn.HostComm(sn.TorchGroupComm()), rank, world)
    s.dist_enable_peer(max(c[1] for c in cases))
    for ci, (seed, N, G, T, k, lam) in enumerate(cases):
        a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
        lo, hi = sn.shard_range(a.N, world, rank)
        r = s.dist_solve(a.slice(lo, hi), lo, a.N)
        np.savez(os.path.join(outdir, f"c{ci}_r{rank}.npz"), lo=lo, hi=hi, plan=r["plan"],
                 cnt=r["planned_rounds"], scal=np.array([r[x] for x in SCALARS], dtype=np.float64),
                 meta=np.array([r["rc"], r["status"], r["iters"]], dtype=np.int64))
    s.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
