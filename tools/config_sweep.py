"""Plan-solve cost per cluster configuration (scale_{64,128,256}gpus.json's
k and lambda; 900 jobs x 30 rounds): single-instance latency and the batched
rate over 1024 instances, with the mean passes per instance.  A/B builds via
SW_LIB_PATH."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shockwave-replication_amd")]
import numpy as np  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

CFGS = {"64": (64, 10.0, 5.0), "128": (128, 1e-3, 15.0), "256": (256, 1e5, 5.0)}


def timed(s, batch, reps):
    s.upload(batch)
    s.run()
    r = s.download()
    t0 = time.perf_counter()
    for _ in range(reps):
        s.run()
    s.download()
    return (time.perf_counter() - t0) / reps, r


def main():
    s = sn.Solver(device=0)
    out = {}
    for name, (G, k, lam) in CFGS.items():
        batch = [ss.synth_problem(500 + i, 900, G, 30, 120.0, k, lam) for i in range(1024)]
        t1, _ = timed(s, batch[:1], 20)
        tb, r = timed(s, batch, 3)
        it = [x["iters"] for x in r] if isinstance(r, list) else None
        out[name] = {"G": G, "k": k, "lambda": lam, "single_ms": t1 * 1e3,
                     "batch_solves_per_s": len(batch) / tb,
                     "mean_passes": float(np.mean(it)) if it else None}
        print(name, json.dumps(out[name]), flush=True)
    s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
