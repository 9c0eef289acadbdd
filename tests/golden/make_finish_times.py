"""Generate tests/golden/finish_times.json: the plan-solve INPUTS (d_j, R_j,
FTF_j, p_j) as the REFERENCE's own code computes them over a sequence of
solves, so the drop-in ShockwaveScheduler's host side is pinned by reference
execution, not by a restatement.

    python tests/golden/make_finish_times.py

Run in the build container only (/root/reference is not on the GPU box).
What runs is reference code:
  * scheduler/job_metadata.py is imported as a module (pure numpy; it imports
    here) — every estimator call is the reference's;
  * ShockwaveScheduler._compute_finish_times and
    ._compute_interpolated_finish_time (shockwave.py:224-279) are taken from
    the AST of scheduler/shockwave.py (the module itself cannot be imported:
    cvxpy / gurobipy are absent) and executed on a plain object holding the
    scheduler's state fields (shockwave.py:13-24).  The only cvxpy call on
    that path is cp.maximum(0, R - planned_runtime) (:260-262), the makespan
    expression; it is given numpy.maximum and planned runtimes of 0.0, so the
    recorded makespans are the call-#2 remaining runtimes R_j exactly.
  * d_j follows _job_log_utility's two lines (:116-120) — the solver-side
    statements of that function build cvxpy variables and are not executed.
  * p_j = FTF_j ** lambda as the objective builds it (:368).
Between solves the generator applies throughput updates, completions,
arrivals and deletions as the simulator's hooks do (scheduler.py:435-448,
:3598-3621, :602-610, :3473).  Only inputs and outputs are stored.
"""
import ast
import json
import os
import random
import sys
import types
from collections import OrderedDict

import numpy as np

REF = "/root/reference/scheduler"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "finish_times.json")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import make_profile  # noqa: E402


def reference_methods():
    """The two methods' code objects, compiled from the reference's AST."""
    src = open(os.path.join(REF, "shockwave.py")).read()
    tree = ast.parse(src)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "ShockwaveScheduler")
    want = {"_compute_finish_times", "_compute_interpolated_finish_time"}
    fns = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in want]
    assert {f.name for f in fns} == want
    mod = ast.Module(body=fns, type_ignores=[])
    ns = {"np": np, "cp": types.SimpleNamespace(maximum=np.maximum)}
    exec(compile(mod, os.path.join(REF, "shockwave.py"), "exec"), ns)
    return ns["_compute_finish_times"], ns["_compute_interpolated_finish_time"]


class RefState:
    """The ShockwaveScheduler state fields the two methods read (shockwave.py:13-28)."""

    def __init__(self, cfg, ft, ift):
        self.num_gpus = cfg["num_gpus"]
        self.round_duration = cfg["time_per_iteration"]
        self.future_rounds = cfg["future_rounds"]
        self.priority_power = cfg["lambda"]
        self.round_index = 0
        self.job_metadata = OrderedDict()
        self.finish_time_estimates = {}
        self._ft = types.MethodType(ft, self)
        self._compute_interpolated_finish_time = types.MethodType(ift, self)

    @property
    def num_jobs(self):
        return len(self.job_metadata)


def main():
    sys.path.insert(0, REF)
    import job_metadata as ref

    ft, ift = reference_methods()
    rng = random.Random(20261016)
    scenarios = []
    for sc in range(6):
        cfg = {"num_gpus": rng.choice([4, 8, 32]), "time_per_iteration": rng.choice([60, 120]),
               "future_rounds": rng.choice([5, 10, 20]), "lambda": rng.choice([1.0, 5.0, 15.0])}
        st = RefState(cfg, ft, ift)
        profiles, events, solves = {}, [], []
        next_id = 0
        for step in range(8):
            # arrivals (scheduler.py:602-610)
            for _ in range(rng.randint(0 if step else 3, 3)):
                E = rng.choice([2, 3, 5, 8, 20, 50, 120])
                prof = make_profile(rng, E)
                jid = next_id
                next_id += 1
                profiles[jid] = prof
                md = ref.ShockwaveJobMetadata(prof, cfg["time_per_iteration"], prof["scale_factor"])
                t = float(st.round_index * cfg["time_per_iteration"])
                md.submit(t)
                st.job_metadata[jid] = md
                events.append(["add", jid, t.hex()])
            # measured rounds and progress of running jobs (scheduler.py:435-448, :3598-3621)
            for jid, md in list(st.job_metadata.items()):
                if rng.random() < 0.6:
                    tput = rng.uniform(0.5, 30.0)
                    bs = rng.choice(profiles[jid]["bs_every_epoch"])
                    md.update_throughput_schedule(st.round_index, tput, bs)
                    events.append(["tput", jid, st.round_index, tput.hex(), bs])
                if rng.random() < 0.5:
                    F = min(md.total_epochs, md.completed_epochs + rng.randint(0, 2))
                    md.complete(F)
                    events.append(["complete", jid, F])
            # a deletion now and then (scheduler.py:3469-3473)
            if len(st.job_metadata) > 3 and rng.random() < 0.3:
                jid = rng.choice(list(st.job_metadata))
                st.job_metadata.pop(jid)
                events.append(["delete", jid])
            # one plan solve's inputs: _job_log_utility's estimator lines, then
            # the reference's own _compute_finish_times
            N = st.num_jobs
            d = []
            for md in st.job_metadata.values():
                md.recompute_epoch_duration()  # shockwave.py:116
                d.append(float(np.mean(md.epoch_durations[: md.completed_epochs + 1])))  # :118-120
            makespans, ftfs = st._ft([0.0] * N)
            p = [float(f) ** cfg["lambda"] for f in ftfs]
            solves.append({"round_index": st.round_index, "ids": list(st.job_metadata),
                           "d": [x.hex() for x in d],
                           "R": [float(m).hex() for m in makespans],
                           "ftf": [float(f).hex() for f in ftfs],
                           "p": [x.hex() for x in p]})
            events.append(["solve"])
            st.round_index += rng.randint(1, cfg["future_rounds"])
            events.append(["round", st.round_index])
        scenarios.append({"config": cfg, "profiles": {str(k): v for k, v in profiles.items()},
                          "events": events, "solves": solves})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_finish_times.py",
                   "reference": "scheduler/shockwave.py:224-279 (AST-executed), "
                                "scheduler/job_metadata.py (imported)",
                   "scenarios": scenarios}, f)
    print(f"wrote {OUT}: {len(scenarios)} scenarios, "
          f"{sum(len(s['solves']) for s in scenarios)} solves")


if __name__ == "__main__":
    main()
