"""Per-cluster-size cost of the C5 sweep's instances under full load: a batch
of 256 instances of one configuration (one per CU) per launch, and the
512-instance sweep in three launch orders.

    python tools/c5_classes.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shockwave-replication_amd")]
import bench  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def timed(s, batch, reps=20):
    s.upload(batch)
    s.run()
    s.download()
    t0 = time.perf_counter()
    for _ in range(reps):
        s.run()
    s.download()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    s = sn.Solver(device=0)
    probs = ss.sweep_problems(bench.C5_INSTANCES, 900, seed0=bench.C5_SEED0, T_override=30)
    out = {}
    for G in (32, 64, 128, 256):
        cls = [p for p in probs if int(p.G) == G]
        out[f"G{G}_x{len(cls)}_ms"] = timed(s, cls)
    orders = {
        "sweep_order": probs,
        "k_then_G": sorted(probs, key=lambda a: (a.k, -a.G)),
        "k1e-3_G32_G64_G256": sorted(probs, key=lambda a: {128: 0, 32: 1, 64: 2, 256: 3}[int(a.G)]),
        "k1e-3_G256_G32_G64": sorted(probs, key=lambda a: {128: 0, 256: 1, 32: 2, 64: 3}[int(a.G)]),
    }
    for name, b in orders.items():
        out[f"sweep_{name}_ms"] = timed(s, b)
    s.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
