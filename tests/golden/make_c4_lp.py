"""Generate tests/golden/c4_lp.json: the LP-relaxation bound of the reference P1
(shockwave.py:330-382, every binary relaxed to [0, 1]; oracle/milp_ref.build_p1)
on the C4 instance (10,000 jobs x 30 rounds, bench.py C4_SEED), solved once by
HiGHS in the build container.  The relaxation's optimum bounds every integer
plan from above, so (LP - J) / |J| certifies the sharded GPU solve's objective
J (tests/test_gpu_shard.py::test_gpu_shard_c4_shape).  At this size the MILP
itself does not finish in the reference's 15 s limit, but the LP does.

    python tests/golden/make_c4_lp.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "oracle")]
import milp_ref as mr  # noqa: E402
import sw_synth as ss  # noqa: E402

SEED = 77  # bench.py C4_SEED, tests/golden/c4_digest.json
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c4_lp.json")


def main():
    c = ss.C4
    a = ss.synth_problem(SEED, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])
    h = hashlib.sha256()
    for arr in (a.w, a.d, a.F, a.E, a.R, a.p):
        h.update(np.ascontiguousarray(arr).tobytes())
    P = mr.Problem(a.w, a.d, a.F, a.E, a.R, a.p, a.T, a.G, a.delta, a.k, list(a.bases))
    t0 = time.perf_counter()
    st, _x, obj, _bound, dt = mr.solve_p1(P, 1e-3, 3600.0, relax=True)
    out = {"generator": "tests/golden/make_c4_lp.py", "seed": SEED, "N": a.N, "T": a.T, "G": a.G,
           "k": a.k, "inputs_sha": h.hexdigest()[:32], "lp_status": st, "lp_bound": obj,
           "seconds": time.perf_counter() - t0}
    json.dump(out, open(OUT, "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main()
