"""Time the sharded C4 solve with the peer-memory step transport at W ranks
as W processes on ONE GPU (the only multi-rank layout a one-GPU box allows;
the ranks share the GPU, so this bounds the per-solve time from above and
shows the exchange working under load, it is not a multi-GPU figure).

    python tools/peer_timing.py [W] [solves]      (spawns W workers)
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port, solves):
    sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import sw_native as sn
    import sw_synth as ss

    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = ss.C4
    a = ss.synth_problem(77, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    lo, hi = sn.shard_range(a.N, world, rank)
    s = sn.Solver(device=0)
    s.dist_init_host(sn.HostComm(sn.TorchGroupComm()), rank, world)
    s.dist_enable_peer(a.N)
    shard = sn.DeviceShard(a.slice(lo, hi), "cuda:0")
    torch.cuda.synchronize()
    for _ in range(5):
        r = s.dist_solve_dev(shard, lo, a.N)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(solves):
        r = s.dist_solve_dev(shard, lo, a.N)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"world": world, "solves": solves, "ms_per_solve": float(t.item()) / solves * 1e3,
                          "collective_steps": r["iters"], "objective": r["objective"],
                          "layout": f"{world} processes on one GPU, peer transport"}), flush=True)
    s.close()
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        return worker(*map(int, sys.argv[2:6]))
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    solves = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ps = [subprocess.Popen([sys.executable, __file__, "--worker", str(r), str(world), str(port), str(solves)])
          for r in range(world)]
    rcs = [p.wait(timeout=240) for p in ps]
    sys.exit(max(rcs))


if __name__ == "__main__":
    main()
