"""Generate tests/golden/c4_digest.json: the CPU solves of the C4 instance that
bench.py's c4_sharded sub-record solves sharded over N GPUs — the twin
(oracle/plan_twin.c, the single-instance solve: top-level digest) and the CPU
shard engine (oracle/shard_twin.c, the specification of the GPU shard engine)
at worlds 1, 2, 4 and 8 (by_world).  The C4 instance is placed in
SW_VSHARES = 8 shares at every world size (sw_share_count), so
the four sharded digests are one and the same; it shares the single
instance's counts and P1 objective, not its plan rows.  bench.py checks its
gathered plan / counts / objective against the digest of its world size.

    python tests/golden/make_c4_digest.py
"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd")]
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

SEED = 77  # bench.py C4_SEED
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c4_digest.json")


def main():
    c = ss.C4
    a = ss.synth_problem(SEED, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libplan_twin.so"))
    sn.declare_solver_api(lib, "twin_")
    pr, res = a.c_problem(), a.c_result()
    rc = lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
    assert rc >= 0
    out = {"generator": "tests/golden/make_c4_digest.py", "seed": SEED, "N": a.N, "T": a.T,
           "G": a.G, "k": a.k,
           "plan_sha": hashlib.sha256(a.plan.tobytes()).hexdigest()[:32],
           "counts_sha": hashlib.sha256(a.planned.astype(sn.np.int32).tobytes()).hexdigest()[:32],
           "objective_hex": float(res.objective).hex(), "status": res.status, "iters": res.iters}
    sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
    import test_shard as ts  # noqa: E402

    slib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libplan_twin.so"))
    slib.shard_twin_solve.argtypes = [ctypes.POINTER(sn.SwHostComm), ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(sn.SwProblem), ctypes.c_int64, ctypes.c_int64,
                                      ctypes.POINTER(sn.SwResult)]
    slib.shard_twin_solve.restype = ctypes.c_int
    by = {}
    for W in (1, 2, 4, 8):
        r = ts.run_threads(slib, a, W)
        by[str(W)] = {"plan_sha": hashlib.sha256(sn.np.ascontiguousarray(r["plan"]).tobytes()).hexdigest()[:32],
                      "counts_sha": hashlib.sha256(sn.np.ascontiguousarray(r["planned_rounds"],
                                                                          dtype=sn.np.int32).tobytes()).hexdigest()[:32],
                      "objective_hex": float(r["objective"]).hex(),
                      "p2_objective": float(r["p2_objective"]), "status": int(r["status"])}
    assert all(by[w] == by["1"] for w in by), "the sharded C4 solve depends on the world size"
    assert by["1"]["counts_sha"] == out["counts_sha"] and by["1"]["objective_hex"] == out["objective_hex"]
    out["by_world"] = by
    json.dump(out, open(OUT, "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main()
