"""Stage times of the C5 sweep (512 instances, bench.c5_leg's problems and
order): the plan stage and the P2 exchange kernel, HIP events on the
handle's stream, 20 launches; and the slowest instances' exchange activity
(status bits, P2 before / after).  python tools/c5_stages.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

probs = ss.sweep_problems(bench.C5_INSTANCES, 900, seed0=bench.C5_SEED0, T_override=30)
mine = bench.c5_order(bench.c5_share(probs, 1, 0))
s = sn.Solver(device=0)
s.upload(mine)
s.run()
res = s.download()
torch.cuda.synchronize()
s.set_timing(True)
for _ in range(20):
    s.run()
torch.cuda.synchronize()
p2x, plan, runs = s.kernel_times()
out = {"plan_ms": plan / runs, "p2x_ms": p2x / runs, "runs": runs}
by = {}
for a, r in zip(mine, res):
    d = by.setdefault(int(a.G), {"n": 0, "exchanged": 0, "slow_bits": 0})
    d["n"] += 1
    d["exchanged"] += bool(r["status"] & sn.SW_STATUS_P2_EXCHANGED)
out["by_G"] = by
print(json.dumps(out))
