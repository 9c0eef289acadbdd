"""Generate tests/golden/estimators.json from the REFERENCE's own estimators.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden.py

It imports ``scheduler/job_metadata.py`` from /root/reference (pure numpy; it
imports and runs here — SURVEY.md §8c), drives seeded random profiles
through the exact call sequence the reference solver makes per plan solve
(shockwave.py:111-134 then :255-278, per job):

    #1 recompute_epoch_duration();  d = np.mean(epoch_durations[:F+1])
    #2 R_mk  = compute_remaining_runtime()
    #3 R_jct = compute_remaining_runtime()
    S = sum(epoch_durations[:F]);  #4 R_fin = compute_remaining_runtime()

interleaved with update_throughput_schedule / complete calls, and records
every returned value (as float hex, bit-exact) plus the epoch durations after
each solve.  The JSON holds only data (profiles, operations, outputs); the
reference's source is not copied.
"""
import json
import os
import random
import sys

import numpy as np

REF = "/root/reference/scheduler"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "estimators.json")


def make_profile(rng, E, max_regimes=4):
    pool = [16, 32, 64, 128, 256, 512, 1024, 2048]
    regimes = sorted(rng.sample(pool[:max(6, max_regimes)], rng.randint(1, max_regimes)))
    bs, cur = [], rng.choice(regimes)
    for _ in range(E):
        if rng.random() < 0.15:
            cur = rng.choice(regimes)
        bs.append(cur)
    base = rng.uniform(5.0, 600.0)
    dur = [max(0.2, base * (64.0 / b) ** 0.5 * rng.uniform(0.8, 1.2)) for b in bs]
    return {
        "num_epochs": E,
        "num_samples_per_epoch": rng.choice([50000, 100000, 10000, 59675, 117907]),
        "scale_factor": rng.choice([1, 1, 1, 2, 2, 4, 8]),
        "duration": sum(dur),
        "bs_every_epoch": bs,
        "mem_every_epoch": [1.0] * E,
        "util_every_epoch": [1.0] * E,
        "duration_every_epoch": dur,
    }


def run_case(ref, rng, prof, wide=False):
    """One seeded call sequence through the reference estimators."""
    E = prof["num_epochs"]
    delta = rng.choice([60, 120, 360])
    md = ref.ShockwaveJobMetadata(prof, delta, prof["scale_factor"])
    ops, outs = [], []
    rnd = 0
    for s in range(rng.randint(2, 7)):
        # a few measured rounds and progress
        for _ in range(rng.randint(0, 3)):
            rnd += rng.randint(1, 12)
            tput = rng.uniform(0.5, 30.0) if rng.random() > 0.1 else 0.0
            bs = rng.choice(prof["bs_every_epoch"])
            ops.append(["tput", rnd, tput.hex(), bs])
            md.update_throughput_schedule(rnd, tput, bs)
        if wide:
            # large jumps, F anywhere in [F, E-1]: many Dirichlet +1 steps
            # per regime, crossing binades of the prior E/#regimes
            F = rng.randint(md.completed_epochs, max(md.completed_epochs, E - 1))
            ops.append(["complete", F])
            md.complete(F)
        elif rng.random() < 0.7:
            F = min(E, md.completed_epochs + rng.randint(0, max(1, E // 3)))
            if rng.random() < 0.05:
                F = None
            ops.append(["complete", F])
            md.complete(F)
        # one plan-solve worth of estimator calls, in the reference order
        md.recompute_epoch_duration()
        d = float(np.mean(md.epoch_durations[: md.completed_epochs + 1]))
        r2 = md.compute_remaining_runtime()
        r3 = md.compute_remaining_runtime()
        sF = sum(md.epoch_durations[: md.completed_epochs])
        r4 = md.compute_remaining_runtime()
        ops.append(["solve"])
        outs.append({
            "d": float(d).hex(), "R_mk": float(r2).hex(), "R_jct": float(r3).hex(),
            "sum_done": float(sF).hex(), "R_fin": float(r4).hex(),
            "F": md.completed_epochs,
            "durations_sha": [float(x).hex() for x in md.epoch_durations[:5]]
            + [float(sum(md.epoch_durations)).hex()],
            "bs_map": {str(k): float(v).hex() for k, v in md.compute_bs_epoch_duration().items()},
        })
        # compute_bs_epoch_duration above recomputes once more (kept in the record)
    return {"profile": prof, "round_duration": delta, "ops": ops, "outs": outs}


def main():
    sys.path.insert(0, REF)
    import job_metadata as ref  # the reference module itself

    rng = random.Random(20261015)
    cases = []
    for c in range(40):
        E = rng.choice([1, 2, 3, 5, 8, 20, 50, 120, 400])
        cases.append(run_case(ref, rng, make_profile(rng, E)))
    # round 3: 1-7 regimes (6- and 7-regime jobs included), F up to E-1, so
    # the reference's one-at-a-time Dirichlet adds cross binades of the prior
    rng = random.Random(20261017)
    for c in range(80):
        E = rng.choice([13, 19, 25, 26, 38, 45, 60, 97, 250, 700, 1500, 3000])
        nreg = 6 if c % 4 == 0 else (7 if c % 4 == 1 else rng.randint(1, 7))
        prof = make_profile(rng, E, max_regimes=nreg)
        if c % 4 < 2:  # force exactly nreg regimes where E allows
            pool = sorted(set(prof["bs_every_epoch"]))
            want = sorted(rng.sample([16, 32, 64, 128, 256, 512, 1024, 2048], nreg))
            # one dominant regime first (its Dirichlet count grows to ~F),
            # the others take one or two epochs each at the end
            tail = [b for b in want[1:] for _ in range(rng.randint(1, 2))]
            prof["bs_every_epoch"] = ([want[0]] * max(0, E - len(tail)) + tail)[:E]
        cases.append(run_case(ref, rng, prof, wide=True))
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "scheduler/job_metadata.py (JitongZ/shockwave-replication)",
                   "cases": cases}, f)
    print(f"wrote {OUT}: {len(cases)} cases")


if __name__ == "__main__":
    main()
