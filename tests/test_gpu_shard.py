"""Sharded single-instance solve on the GPU engine (csrc/sw_shard.hip).

The box has one MI355X, so multi-rank runs put W handles on cuda:0 as threads
of this process with host collectives (a barrier-based allgather); the
world-1 run goes through RCCL (ncclAllReduce / ncclAllGather on the handle's
stream).  Every run must return exactly the CPU shard engine's result at the
same world size (oracle/shard_twin.c, ranks as threads: tests/test_shard.py)
for plan rows, counts and the bits of every objective — at world 1 that is
the single-instance twin's (oracle/plan_twin.c), which the batched GPU kernel
also matches; above it the share placement's.
"""
import threading

import numpy as np
import pytest

import sw_native as sn
import sw_synth as ss
from helpers import check_plan_valid
from test_shard import (CASES, ThreadGroup, assemble, assert_same_as_single, assert_share_contract, run_threads,  # noqa: F401
                        shard_lib)

pytestmark = pytest.mark.gpu


def gpu_shard_threads(a, world, peer=False):
    group = ThreadGroup(world)
    out = [None] * world
    errs = []

    def work(r):
        try:
            s = sn.Solver(device=0)
            s.dist_init_host(sn.HostComm(group.member(r)), r, world)
            if peer:  # every thread enters the peer setup at once
                s.dist_enable_peer(a.N)
            lo, hi = sn.shard_range(a.N, world, r)
            out[r] = (lo, hi, s.dist_solve(a.slice(lo, hi), lo, a.N))
            s.close()
        except Exception as e:
            errs.append(e)
            group.barrier.abort()

    ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs, errs
    return assemble(a, out)


@pytest.fixture(scope="module")
def rccl_solver():
    s = sn.Solver(device=0)
    s.dist_init(sn.unique_id(), 0, 1)
    yield s
    s.close()


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[1]}_G{c[2]}_T{c[3]}_k{c[4]:g}" for c in CASES])
def test_gpu_shard_rccl_world1(case, rccl_solver, twin):
    seed, N, G, T, k, lam = case
    a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
    r = rccl_solver.dist_solve(a, 0, a.N)
    check_plan_valid(a, r)
    assert_same_as_single(r, twin.solve(a), f"rccl W=1 {case}")


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("case", [CASES[1], CASES[4], CASES[6], CASES[7]],
                         ids=["N50", "N300_T64", "N900", "N1500"])
def test_gpu_shard_host_comm(case, world, shard_lib):
    seed, N, G, T, k, lam = case
    a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
    r = gpu_shard_threads(a, world)
    check_plan_valid(a, r)
    assert_same_as_single(r, run_threads(shard_lib, a, world), f"W={world} {case}")


def test_gpu_shard_c4_shape(rccl_solver, twin, shard_lib):
    """The 10k-job × 30-round C4 instance, whole on one rank:
    the CPU shard engine at world 1 bit for bit (its eight shares placed by
    eight workgroups, sw_share_count), and so the result of every world size."""
    c = ss.C4
    a = ss.synth_problem(11, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    r = rccl_solver.dist_solve(a, 0, a.N)
    check_plan_valid(a, r)
    assert_same_as_single(r, run_threads(shard_lib, a, 1), "C4")
    assert_share_contract(r, twin.solve(a), "C4 vs single")


@pytest.mark.parametrize("seed", [71, 73, 74, 75])
def test_gpu_shard_c4_seeds(seed, rccl_solver, shard_lib):
    """Other C4-shaped instances (tools/c4_seeds.py): 71 ends SELECT with a
    width tail (on the device at world 1, k_fast_tail), 73 and 75 strand
    rounds in a share (the host's share repair, then the rest of the device
    path: fast_solve's resume), 74 takes the common path; each the CPU shard
    engine's result bit for bit, collective steps included."""
    c = ss.C4
    a = ss.synth_problem(seed, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    r = rccl_solver.dist_solve(a, 0, a.N)
    check_plan_valid(a, r)
    ref = run_threads(shard_lib, a, 1)
    assert_same_as_single(r, ref, f"C4 seed {seed}")
    assert r["iters"] == ref["iters"], (seed, r["iters"], ref["iters"])


def test_gpu_shard_c4_world8(shard_lib):
    c = ss.C4
    a = ss.synth_problem(12, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    r = gpu_shard_threads(a, 8)
    assert_same_as_single(r, run_threads(shard_lib, a, 8), "C4 W=8")


@pytest.mark.parametrize("world", [2])
def test_gpu_shard_peer_transport_threaded_ranks(world, shard_lib):
    """sw_dist_enable_peer with ranks that are threads of ONE process,
    entering the setup concurrently: every rank must see the same process
    identity (one nonce per process, initialised once) and take the
    same-process pointer path, then one solve matches the twin.  World 2
    only: the ranks share one GPU here, and each one's exchange kernel waits
    on the device for the others, so their streams need hardware queues of
    their own (GPU_MAX_HW_QUEUES = 4 per process on the box, and this module
    already holds the RCCL handle's stream; at world 4 two ranks shared a
    queue and the exchange timed out, include/shockwave_amd.h)."""
    for case in (CASES[1], CASES[6]):
        seed, N, G, T, k, lam = case
        a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
        r = gpu_shard_threads(a, world, peer=True)
        check_plan_valid(a, r)
        assert_same_as_single(r, run_threads(shard_lib, a, world), f"peer threads W={world} {case}")


def test_gpu_shard_rejects_bad_slice(rccl_solver):
    a = ss.synth_problem(0, 100, 32, 10, 120.0, 1e5, 5.0)
    with pytest.raises(sn.NativeError):
        rccl_solver.dist_solve(a.slice(0, 50), 0, a.N)


@pytest.mark.parametrize("case", [CASES[1], CASES[6], CASES[7]], ids=["N50", "N900", "N1500"])
def test_gpu_shard_device_resident(case, rccl_solver):
    """sw_dist_plan_solve_dev (inputs and plan in HBM) returns exactly what the
    host-buffer entry point returns: plan bytes, counts, objective bits, steps."""
    import torch
    seed, N, G, T, k, lam = case
    a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
    shard = sn.DeviceShard(a, "cuda:0")
    torch.cuda.synchronize()
    rd = rccl_solver.dist_solve_dev(shard, 0, a.N)
    rh = rccl_solver.dist_solve(a, 0, a.N)
    assert np.array_equal(shard.plan.cpu().numpy(), rh["plan"])
    assert np.array_equal(shard.planned.cpu().numpy(), rh["planned_rounds"])
    for key in ("objective", "utility", "makespan", "p2_objective", "bound", "iters", "status", "rc"):
        assert rd[key] == rh[key] or (rd[key] != rd[key] and rh[key] != rh[key]), key


def test_gpu_shard_device_rejects_bad_input(rccl_solver):
    """The per-job checks run on the device for HBM-resident inputs."""
    import torch
    a = ss.synth_problem(3, 200, 32, 10, 120.0, 1e5, 5.0)
    shard = sn.DeviceShard(a, "cuda:0")
    shard.F[7] = shard.E[7] + 1  # completed epochs > total epochs
    torch.cuda.synchronize()
    with pytest.raises(sn.NativeError):
        rccl_solver.dist_solve_dev(shard, 0, a.N)
    shard.F[7] = 0
    torch.cuda.synchronize()
    r = rccl_solver.dist_solve_dev(shard, 0, a.N)  # the handle recovers
    assert r["rc"] in (0, 1)
    # ... exactly: the step results published after the refused solve (world 1:
    # by the step kernels themselves) are this solve's, as a second solve shows
    plan = shard.plan.cpu().numpy().copy()
    r2 = rccl_solver.dist_solve_dev(shard, 0, a.N)
    assert np.array_equal(shard.plan.cpu().numpy(), plan)
    for key in ("objective", "utility", "makespan", "p2_objective", "bound", "iters", "status", "rc"):
        assert r2[key] == r[key] or (r2[key] != r2[key] and r[key] != r[key]), key


def test_gpu_shard_peer_transport_two_processes(tmp_path, shard_lib):
    """sw_dist_enable_peer: two processes on cuda:0 (gloo only for the setup),
    every step's all-reduce / all-gather one k_xchg kernel writing into the
    other process's IPC-mapped exchange region; the result must be the CPU
    shard engine's at world 2, bit for bit, C4 shape included."""
    import json
    import os
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    c = ss.C4
    cases = [CASES[1], CASES[6], CASES[7], (13, c["N"], c["G"], c["T"], c["k"], c["lam"])]
    cj = tmp_path / "cases.json"
    cj.write_text(json.dumps([list(x) for x in cases]))
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "peer_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", str(port), str(tmp_path), str(cj)])
             for r in range(2)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=150))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(None)
    assert rcs == [0, 0], rcs
    for ci, case in enumerate(cases):
        seed, N, G, T, k, lam = case
        a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
        parts = []
        for r in range(2):
            z = np.load(tmp_path / f"c{ci}_r{r}.npz")
            res = {key: float(v) for key, v in zip(("objective", "utility", "makespan",
                                                      "p2_objective", "bound"), z["scal"])}
            res.update(rc=int(z["meta"][0]), status=int(z["meta"][1]), iters=int(z["meta"][2]),
                       plan=z["plan"], planned_rounds=z["cnt"])
            parts.append((int(z["lo"]), int(z["hi"]), res))
        rs = assemble(a, parts)
        check_plan_valid(a, rs)
        assert_same_as_single(rs, run_threads(shard_lib, a, 2), f"peer W=2 {case}")


def test_gpu_shard_peer_late_rank_fails_cleanly(tmp_path):
    """A rank that enters a solve after its peers' exchange timeout: both
    ranks get SW_ERR_RCCL (no hang), and the handle then stays unusable —
    the next solve on it fails at once instead of exchanging with sequence
    numbers that no longer agree (include/shockwave_amd.h, sw_dist_enable_peer)."""
    import json
    import os
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cj = tmp_path / "cases.json"
    cj.write_text(json.dumps([list(CASES[1])]))
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "peer_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", str(port), str(tmp_path), str(cj),
                               "late"]) for r in range(2)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=120))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(None)
    assert rcs == [0, 0], rcs
    for r in range(2):
        out = json.load(open(tmp_path / f"late_r{r}.json"))
        assert out[0][0] == "error" and "timed out" in out[0][1], (r, out)
        assert out[1][0] == "error" and "rebuild the handle" in out[1][1], (r, out)


def test_gpu_shard_fuzz_rccl_world1(rccl_solver, twin):
    """The sharded engine over 256 fuzz instances (tests/fuzzcases.py)."""
    from fuzzcases import fuzz_problem

    for s in range(256):
        a = fuzz_problem(s)
        r = rccl_solver.dist_solve(a, 0, a.N)
        check_plan_valid(a, r)
        assert_same_as_single(r, twin.solve(a), f"rccl W=1 fuzz seed {s}")


@pytest.mark.parametrize("world", [2, 4])
def test_gpu_shard_fuzz_host_comm(world, shard_lib):
    from fuzzcases import fuzz_problem

    for s in range(256, 256 + 48):
        a = fuzz_problem(s)
        assert_same_as_single(gpu_shard_threads(a, world), run_threads(shard_lib, a, world),
                              f"W={world} fuzz seed {s}")


@pytest.mark.parametrize("world", [1, 2])
def test_gpu_shard_pattern_placement(world, rccl_solver, twin, shard_lib):
    """The level search's branch and bound and the round-pattern placement on
    the GPU engine (frag-fuzz seeds of tests/test_shard.py): RCCL at world 1,
    host collectives at world 2, each equal to the twin bit for bit."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_frag_fuzz as mk

    for s in (50115, 50417, 50439, 50104, 50169):  # 50169: a kept raise
        a = mk.instance(s)
        r = rccl_solver.dist_solve(a, 0, a.N) if world == 1 else gpu_shard_threads(a, world)
        check_plan_valid(a, r)
        ref = twin.solve(a) if world == 1 else run_threads(shard_lib, a, world)
        assert_same_as_single(r, ref, f"W={world} frag seed {s}")


def test_gpu_shard_peer_refuses_too_many_same_device_ranks(shard_lib):
    """Four ranks of one process on one device exceed half of the process's
    hardware queues (GPU_MAX_HW_QUEUES = 4 on the box): sw_dist_enable_peer
    refuses on every rank with SW_ERR_INVALID at once (no 10 s timeout), and
    the init call's transport (host collectives) still solves, equal to the
    twin."""
    import time

    world = 4
    case = CASES[1]
    seed, N, G, T, k, lam = case
    a = ss.synth_problem(seed, N, G, T, 120.0, k, lam)
    group = ThreadGroup(world)
    codes = [None] * world
    out = [None] * world
    errs = []

    def work(r):
        try:
            s = sn.Solver(device=0)
            s.dist_init_host(sn.HostComm(group.member(r)), r, world)
            try:
                s.dist_enable_peer(a.N)
                codes[r] = 0
            except sn.NativeError as e:
                codes[r] = e.code
            lo, hi = sn.shard_range(a.N, world, r)
            out[r] = (lo, hi, s.dist_solve(a.slice(lo, hi), lo, a.N))
            s.close()
        except Exception as e:
            errs.append(e)
            group.barrier.abort()

    t0 = time.time()
    ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs, errs
    assert codes == [sn.SW_ERR_INVALID] * world, codes
    assert time.time() - t0 < 60
    assert_same_as_single(assemble(a, out), run_threads(shard_lib, a, world), "after the refusal")


def test_gpu_workspace_resolve_paths_match_twin(rccl_solver, twin, shard_lib):
    """Re-solved (SW_STATUS_P1_REPACKED) instances above 1,024 jobs: the plan
    kernel's workspace form (per-round re-optimisation with its items in the
    position slots and values in workspace rows; the pattern search's scratch
    in LDS at 1,500 jobs, in the workspace rows at 2,000) through
    sw_plan_solve, and the sharded engines' gathered k_rr at world 1 (RCCL)
    and 2 (host collectives): equal to the twin (world 1) or the CPU shard
    engine (world 2) bit for bit."""
    cases = [(0, 1500), (2, 1500), (3, 1500), (3, 2000)]
    rep = 0
    s = sn.Solver(device=0)
    for seed, N in cases:
        a = ss.synth_problem(seed, N, 12, 12, 120.0, 1.0, 5.0, width_p=(0.4, 0.3, 0.2, 0.1))
        rt = twin.solve(a)
        rep += bool(rt["status"] & sn.SW_STATUS_P1_REPACKED)
        r1 = s.solve(a)
        check_plan_valid(a, r1)
        assert_same_as_single(r1, rt, f"sw_plan_solve seed {seed} N {N}")
        assert r1["iters"] == rt["iters"]
        assert_same_as_single(rccl_solver.dist_solve(a, 0, a.N), rt, f"dist W=1 seed {seed} N {N}")
        assert_same_as_single(gpu_shard_threads(a, 2), run_threads(shard_lib, a, 2),
                              f"dist W=2 seed {seed} N {N}")
    s.close()
    assert rep >= 2, rep


def test_gpu_rccl_world2_on_one_device():
    """The RCCL transport above world 1 on a one-GPU box:
    two processes on cuda:0 call sw_dist_init at world 2.  This image's RCCL
    refuses two ranks on one device (ncclCommInitRank: invalid usage, both
    ranks, no hang — profiles/r8_rccl_two_ranks_one_gpu.json); if a build
    accepts them, the sharded solve over RCCL must equal the CPU shard engine
    at world 2 bit for bit (tools/rccl_same_device.py)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "rccl_same_device.py")],
                         capture_output=True, text=True, timeout=170)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    inits = [r["init"] for r in line["ranks"]]
    if inits == ["ok", "ok"]:
        assert line["twin_equal"], line
    else:
        assert inits == ["refused", "refused"], line
        assert all("ncclCommInitRank" in r["error"] for r in line["ranks"]), line
