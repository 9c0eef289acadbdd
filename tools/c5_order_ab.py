"""Launch-order A/B for the C5 sweep (bench.c5_leg's workload on one GPU):
ms per sweep for several instance orders.  Results are per instance, so the
order changes no result; only which instances share a CU and which start
first.  python tools/c5_order_ab.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))

import bench  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def cost_rank(a):
    """coarse cost class: the k = 10 instances (exchange-heavy, G = 32 / 64)
    first, then k = 1e-3 (long level search), then k = 1e5"""
    return {10.0: 0, 1e-3: 1}.get(float(a.k), 2)


def orders(probs):
    cur = bench.c5_order(probs)
    heavy_first = sorted(probs, key=lambda a: (cost_rank(a), -a.G))
    n = len(probs)
    h = n // 2
    # workgroup i and i + n/2 tend to share a CU: pair the heaviest half with
    # the lightest half, heaviest with lightest
    paired = heavy_first[:h] + heavy_first[h:][::-1]
    return {"current": cur, "k10_first": heavy_first, "paired": paired, "reversed": cur[::-1]}


def main():
    import torch

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    probs = ss.sweep_problems(bench.C5_INSTANCES, 900, seed0=bench.C5_SEED0, T_override=30)
    ref = None
    for name, ordv in orders(probs).items():
        s = sn.Solver(device=0)
        s.upload(ordv)
        for _ in range(2):
            s.run()
        res = s.download()
        key = {id(a): r for a, r in zip(ordv, res)}
        digest = [(key[id(a)]["objective"], key[id(a)]["p2_objective"]) for a in probs]
        if ref is None:
            ref = digest
        torch.cuda.synchronize()
        best = []
        for _rep in range(3):
            t0 = time.perf_counter()
            for _ in range(steps):
                s.run()
            torch.cuda.synchronize()
            best.append((time.perf_counter() - t0) / steps * 1e3)
        s.close()
        print(json.dumps({"order": name, "ms_per_sweep": best, "min_ms": min(best),
                          "plan_solves_per_s": bench.C5_INSTANCES / min(best) * 1e3,
                          "same_results": digest == ref}), flush=True)


if __name__ == "__main__":
    main()
