"""One rank of the peer-transport test (tests/test_gpu_shard.py): a separate
process on cuda:0, host collectives over gloo for the setup, then
sw_dist_enable_peer so that every step's collective goes through the other
process's IPC-mapped exchange region.  Writes this rank's rows and the global
scalars of each case to <outdir>/c<case>_r<rank>.npz.

    python tests/peer_worker.py <rank> <world> <port> <outdir> <cases.json> [late]

"late": rank 1 enters the first solve 1.5 s after rank 0, with a 300 ms peer
timeout (SW_PEER_TIMEOUT_MS); each rank records the outcome of that solve and
of one more solve on the same handle to <outdir>/late_r<rank>.json.
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

    late = len(sys.argv) > 6 and sys.argv[6] == "late"
    if late:
        os.environ["SW_PEER_TIMEOUT_MS"] = "300"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = sn.Solver(device=0)
    s.dist_init_host(sn.HostComm(sn.TorchGroupComm()), rank, world)
    s.dist_enable_peer(max(c[1] for c in cases))
    if late:
        import time

        seed, N, G, T, k, lam = cases[0]
        a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
        lo, hi = sn.shard_range(a.N, world, rank)
        out = []
        dist.barrier()
        if rank == 1:
            time.sleep(1.5)
        for _ in range(2):
            try:
                r = s.dist_solve(a.slice(lo, hi), lo, a.N)
                out.append(["ok", int(r["rc"])])
            except sn.NativeError as e:
                out.append(["error", str(e)])
        json.dump(out, open(os.path.join(outdir, f"late_r{rank}.json"), "w"))
        s.close()
        dist.barrier()
        dist.destroy_process_group()
        return
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
