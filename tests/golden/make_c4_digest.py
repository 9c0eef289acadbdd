"""Generate tests/golden/c4_digest.json: the CPU twin's solve (oracle/plan_twin.c,
the bit-exact restatement of the GPU algorithm) of the C4 instance that
bench.py's c4_sharded sub-record solves sharded over N GPUs.  bench.py checks
its gathered plan / counts / objective against these digests at every N
(the sharded solve returns the single-instance result bit for bit).

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
    json.dump(out, open(OUT, "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main()
