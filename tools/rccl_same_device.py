"""Does this image's RCCL accept two ranks on one GPU?  Two processes on
cuda:0 (gloo only to pass the unique id) call sw_dist_init (ncclCommInitRank)
at world 2 and, if that succeeds, solve one instance sharded over RCCL; the
result is compared with the CPU shard engine at world 2 (oracle/shard_twin.c).
Prints one JSON line.   python tools/rccl_same_device.py"""
import json
import os
import socket
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]


def worker(rank, world, port, outdir):
    import numpy as np
    import torch.distributed as dist

    import sw_native as sn
    import sw_synth as ss

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = [sn.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    out = {"rank": rank}
    s = sn.Solver(device=0)
    try:
        s.dist_init(uid[0], rank, world)
        out["init"] = "ok"
        a = ss.synth_problem(3, 600, 128, 20, 120.0, 1e5, 5.0)
        lo, hi = sn.shard_range(a.N, world, rank)
        r = s.dist_solve(a.slice(lo, hi), lo, a.N)
        out.update(objective=r["objective"], status=r["status"], lo=lo, hi=hi)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), plan=r["plan"], cnt=r["planned_rounds"])
    except Exception as e:  # the refusal is the answer, not an error of this script
        out["init"] = out.get("init", "refused")
        out["error"] = str(e)
    s.close()
    json.dump(out, open(os.path.join(outdir, f"r{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


def main():
    import numpy as np
    import torch.multiprocessing as mp

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    d = tempfile.mkdtemp()
    mp.spawn(worker, args=(2, port, d), nprocs=2, join=True)
    rs = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    line = {"ranks": rs}
    if all(r.get("init") == "ok" and "objective" in r for r in rs):
        import ctypes

        import sw_native as sn
        import sw_synth as ss
        import test_shard as ts
        from conftest import TWIN_SO

        lib = ctypes.CDLL(TWIN_SO)
        lib.shard_twin_solve.argtypes = [ctypes.POINTER(sn.SwHostComm), ctypes.c_int32, ctypes.c_int32,
                                         ctypes.POINTER(sn.SwProblem), ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(sn.SwResult)]
        lib.shard_twin_solve.restype = ctypes.c_int
        a = ss.synth_problem(3, 600, 128, 20, 120.0, 1e5, 5.0)
        ref = ts.run_threads(lib, a, 2)
        plan = np.concatenate([np.load(os.path.join(d, f"r{r}.npz"))["plan"] for r in range(2)])
        line["twin_equal"] = bool(np.array_equal(plan, ref["plan"]) and
                                  rs[0]["objective"] == ref["objective"])
    print(json.dumps(line))


if __name__ == "__main__":
    main()
