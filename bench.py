#!/usr/bin/env python3
"""Benchmark: Shockwave plan solves/sec at 900 jobs × 30 rounds (BASELINE.json).

One "step" = one batched launch that solves --batch independent C3-shaped
plan problems (900 jobs, 30-round horizon; G=256, Δ=120 s, k=1e5, λ=5 —
SURVEY.md §8 C3, a seed sweep as in C5) end to end on the GPU: key rows,
P1 level/price search, packing, P2 placement, plan emission.  Inputs are
uploaded to HBM before the timed region.  Each rank solves its own batch
(replicas, no data-path collective; "scaling": "weak").

    python bench.py                      # N=1, defaults finish in ~1 min
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Printed on rank 0: ONE JSON line with metric/value/unit, roofline and
cpu_baseline (DESIGN.md §6 defines every figure).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "shockwave-replication_amd")
sys.path.insert(0, PKG)

import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md chip table)

# The result line is the only thing on stdout: libraries (RCCL prints its
# version banner on communicator init) write to fd 1 directly, so fd 1 is
# pointed at stderr and the JSON line goes to a saved copy of the real stdout.
_RESULT_OUT = None


def emit(line: dict):
    print(json.dumps(line), file=_RESULT_OUT or sys.stdout, flush=True)


def pass_bytes(N: int, T: int) -> int:
    """Algorithmic bytes of one pass of the plan kernel over an instance's jobs.

    Every price/level/packing pass reads each job's fp32 key row (4·T B) and
    its constants/state (32 B: rate, cap, R, d as the 8-B values a pass
    touches), per DESIGN.md §4.  The analogue of SURVEY.md §8(d)'s B_iter for
    this kernel; the working set stays on chip (VGPR/LDS).
    """
    return 4 * N * T + 32 * N


def pmc_traffic(batch: int, jobs: int, rounds: int):
    """HBM bytes per batched launch from the committed rocprofv3 PMC passes
    (profiles/*_summary.json, FETCH_SIZE ×2 per the gfx950 note + WRITE_SIZE),
    when they were collected on this exact workload; else None."""
    import glob

    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        w = d.get("workload", {})
        if w.get("instances") == batch and w.get("jobs") == jobs and w.get("rounds") == rounds:
            best = (d.get("hbm_bytes_per_launch_fetch_x2"), os.path.relpath(path, ROOT))
    return best


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192,
                    help="instances per GPU per step (32 per CU: one 512-thread workgroup fits a "
                         "CU at a time; a launch ends with its most expensive instances running "
                         "alone, ~0.75 ms, so more instances per launch amortise that tail, "
                         "DESIGN.md §6)")
    ap.add_argument("--jobs", type=int, default=900)
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--cpu-sample-jobs", type=int, default=900)
    ap.add_argument("--workload", choices=("c3", "c4"), default="c3",
                    help="c3: batched 900x30 instances per GPU (headline, replicas); "
                         "c4: one 10k x 30 instance sharded across the ranks (RCCL)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args()


def cpu_baseline(args):
    """The reference algorithm's CPU restatement (HiGHS MILP of P1 + P2,
    oracle/milp_ref.py, time_limit 15 s per MILP as scale_*gpus.json) on one
    C3 instance, timed on this host (single process)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import milp_ref as mr

    a = ss.synth_problem(10_000 + args.seed, args.cpu_sample_jobs, 256, args.rounds, 120.0, 1e5, 5.0)
    P = mr.Problem(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, list(a.bases))
    t0 = time.perf_counter()
    sol = mr.plan_solve(P, rel_gap=1e-3, time_limit=15.0)
    dt = time.perf_counter() - t0
    return {
        "value": 1.0 / dt,
        "unit": "plan-solves/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"1 plan solve (P1+P2 MILPs via scipy HiGHS, gap 1e-3, 15 s limit each) "
                   f"of a {args.cpu_sample_jobs}x{args.rounds} C3 instance: {dt:.2f} s, "
                   f"P1 status {sol.status}, P2 status {sol.p2_status}"),
        "seconds": dt,
    }


def main_c4(args, world, rank, local, dist):
    """one 10,000-job × 30-round instance, jobs sharded across
    the ranks (sw_dist_shard_range), every step's counts/maxima all-reduced and
    lane sums / placement keys all-gathered on RCCL over xGMI.  One step = one
    complete sharded plan solve; total work is fixed, so scaling is strong."""
    import torch

    c = ss.C4
    a = ss.synth_problem(args.seed + 77, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    lo, hi = sn.shard_range(a.N, world, rank)
    local_arrays = a.slice(lo, hi)
    solver = sn.Solver(device=local)
    uid = [sn.unique_id() if rank == 0 else None]
    if dist is not None:
        dist.broadcast_object_list(uid, src=0)
    solver.dist_init(uid[0], rank, world)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # inputs resident in HBM (the contract's value); the plan stays there too
    shard = sn.DeviceShard(local_arrays, f"cuda:{local}")
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        r = solver.dist_solve_dev(shard, lo, a.N)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = solver.dist_solve_dev(shard, lo, a.N)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    # the host-buffer boundary (sw_dist_plan_solve: per-job arrays up and the
    # plan down over PCIe every solve), reported beside the value
    hsteps = max(1, args.steps // 2)
    barrier()
    t1 = time.perf_counter()
    for _ in range(hsteps):
        rh = solver.dist_solve(local_arrays, lo, a.N)
    torch.cuda.synchronize()
    host_elapsed = time.perf_counter() - t1
    barrier()
    assert rh["objective"] == r["objective"] and rh["iters"] == r["iters"]
    if dist is not None:
        t = torch.tensor([elapsed, host_elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, host_elapsed = float(t[0].item()), float(t[1].item())
    if rank == 0:
        line = {
            "metric": "Shockwave plan solves/sec, 10k jobs x 30 rounds sharded (C4)",
            "value": args.steps / elapsed,
            "unit": "plan-solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded C4 instance)",
            "config": {"workload": f"C4 sharded solve: {a.N} jobs x {a.T} rounds, G={a.G}, "
                                   f"k={a.k:g}; jobs split over {world} ranks",
                       "jobs": a.N, "rounds": a.T, "parallelism": f"jobs sharded x{world}"},
            "collective_steps": r["iters"],
            "objective": r["objective"],
            "host_boundary_solves_per_s": hsteps / host_elapsed,
        }
        emit(line)
    solver.close()
    if dist is not None:
        dist.destroy_process_group()


def main():
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    if args.workload == "c4":
        return main_c4(args, world, rank, local, dist)

    solver = sn.Solver(device=local)
    batch = [ss.synth_problem(args.seed + rank * 100_000 + i, args.jobs, 256, args.rounds, 120.0,
                              1e5, 5.0) for i in range(args.batch)]
    solver.upload(batch)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        solver.run()
    results = solver.download()
    iters = np.array([r["iters"] for r in results], dtype=np.float64)

    solver.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solver.run()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    _, ms_plan, runs = solver.kernel_times()
    solver.set_timing(False)

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # single-instance latency (a scheduler's call pattern), rank 0 only
    lat_ms = None
    if rank == 0:
        one = sn.Solver(device=local)
        one.upload(batch[:1])
        one.run()
        one.download()
        t1 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            one.run()
        one.download()
        lat_ms = (time.perf_counter() - t1) / reps * 1e3
        one.close()

    total = args.steps * args.batch * world
    value = total / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    avg_kernel_s = (ms_plan / max(runs, 1)) / 1e3
    alg_bytes = float(np.sum(iters) * pass_bytes(args.jobs, args.rounds))
    achieved = alg_bytes / avg_kernel_s if avg_kernel_s > 0 else 0.0

    traffic = pmc_traffic(args.batch, args.jobs, args.rounds)
    if rank == 0:
        cpu = None
        if args.cpu_baseline:
            try:
                cpu = cpu_baseline(args)
            except Exception as e:  # reported, never silently substituted
                cpu = {"value": None, "unit": "plan-solves/s", "cores": 1, "kind": "port",
                       "sample": f"failed: {e!r}"}
        line = {
            "metric": "Shockwave plan solves/sec at 900 jobs x 30 rounds",
            "value": value,
            "unit": "plan-solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded C3-shaped instances; reference trace pickles are missing)",
            "config": {
                "workload": f"C3 plan solve: {args.jobs} jobs x {args.rounds} rounds, G=256, "
                            f"k=1e5, lambda=5; {args.batch} independent instances per GPU per step",
                "jobs": args.jobs, "rounds": args.rounds, "instances_per_gpu": args.batch,
                "parallelism": f"replicas x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved / 1e9,
                "peak": HBM_PEAK / 1e9,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK,
                "traffic": traffic[0] if traffic else None,
                "traffic_source": traffic[1] if traffic else None,
                "note": ("achieved counts the per-pass working set, which stays on chip "
                         "(VGPR/LDS); traffic is the HBM side (PMC). DESIGN.md §6"),
                "kernel": "sw_plan_kernel",
                "avg_kernel_ms": avg_kernel_s * 1e3,
                "passes_per_instance": float(np.mean(iters)),
                "bytes_per_pass": pass_bytes(args.jobs, args.rounds),
            },
            "cpu_baseline": cpu,
            "single_instance_ms": lat_ms,
            "speedup_vs_cpu": (value / cpu["value"]) if cpu and cpu.get("value") else None,
        }
        emit(line)
    solver.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
