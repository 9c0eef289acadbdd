"""Generate tests/golden/p2_cases.json: plan-solve inputs captured from the
round-loop simulator (sw_sim.py, 220-job trace, 64 and 128 GPUs, CPU twin
solver), chosen so that every P2 placement of the cascade is exercised
(DESIGN.md §3.3): density order, weight order, class-wise repack.

    python tests/golden/make_p2_cases.py

Inputs only (the expected outputs are whatever the twin / MILP oracle return
when the tests run).
"""
import contextlib
import ctypes
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd"), os.path.join(ROOT, "tools")]
import sw_sim  # noqa: E402
import sw_native as sn  # noqa: E402
from sim_parity import twin_solver  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "p2_cases.json")
TRACE = os.path.join(ROOT, "data", "traces",
                     "220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace")


def main():
    tw = twin_solver()
    cases = []
    for g in (64, 128):
        calls = []

        class Rec:
            def solve(self, a):
                r = tw.solve(a)
                calls.append((a, r["status"]))
                return r

        cfg = json.load(open(os.path.join(ROOT, "data", "configs", f"scale_{g}gpus.json")))
        with contextlib.redirect_stdout(io.StringIO()):
            sw_sim.run_trace("shockwave", TRACE, g, 120, cfg, shockwave_solver=Rec())
        picked = {}
        for i, (a, stt) in enumerate(calls):
            kind = ("classwise" if stt & sn.SW_STATUS_P2_CLASSWISE else
                    "weight" if stt & sn.SW_STATUS_P2_WEIGHT_ORDER else "density")
            if a.N >= 30 and len(picked.get(kind, [])) < 3 and i % 3 == 0:
                picked.setdefault(kind, []).append(a)
        for kind, lst in picked.items():
            for a in lst:
                cases.append({"kind": kind, "G": a.G, "T": a.T, "delta": a.delta, "k": a.k,
                              "bases": list(map(float, a.bases)), "w": a.w.tolist(),
                              "d": a.d.tolist(), "F": a.F.tolist(), "E": a.E.tolist(),
                              "R": a.R.tolist(), "p": a.p.tolist()})
    json.dump(cases, open(OUT, "w"), separators=(",", ":"))
    print(f"wrote {OUT}: {[c['kind'] for c in cases]}")


if __name__ == "__main__":
    main()
