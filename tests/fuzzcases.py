"""Seeded random plan-solve instances for the GPU ↔ twin fuzz (test data, no
product logic).

Where sw_synth draws trace-shaped inputs, these reach into the corners the
validator accepts (shockwave_amd.h, sw_validate.h): any T in 1..64, clusters
from 0 to 600 GPUs, widths up to 255 and wider than the cluster, finished jobs
(F = E), zero priorities, zero regularizer, non-default base grids, and exact
duplicate jobs, whose keys tie in every sort and price search.
"""
import numpy as np

import sw_native as sn


def _bases(rng):
    if rng.random() < 0.7:
        return (0.0, 0.2, 0.4, 0.6, 0.8, 1.0)
    nb = int(rng.integers(2, 9))
    inner = np.sort(rng.choice(np.arange(1, 100), size=nb - 2, replace=False)) / 100.0
    return tuple([0.0] + [float(x) for x in inner] + [1.0])


def fuzz_problem(seed: int, max_n: int = 1024, min_n: int = 1, off=(),
                 trace_widths: bool = False) -> sn.ProblemArrays:
    """trace_widths: widths from {1, 2, 4, 8} only (the reference traces).
    off: features to leave out ("done", "smalld", "r0", "p0", "dup", "bases"), with
    the same random draws, for narrowing down a mismatch."""
    rng = np.random.default_rng(10_000_019 + seed)
    N = int(np.exp(rng.uniform(np.log(min_n), np.log(max_n + 1)))) if rng.random() < 0.95 else int(
        rng.integers(min_n, max_n + 1))
    N = max(min_n, min(N, max_n))
    G = int(rng.choice([0, 1, 2, 3, int(rng.integers(4, 64)), int(rng.integers(64, 601))],
                       p=[0.02, 0.04, 0.04, 0.05, 0.45, 0.40]))
    T = int(rng.choice([1, 2, int(rng.integers(3, 65)), 20, 30, 64], p=[0.04, 0.04, 0.72, 0.08, 0.08, 0.04]))
    k = float(rng.choice([0.0, 10.0 ** rng.uniform(-4, 6)], p=[0.08, 0.92]))
    lam = float(rng.uniform(0.0, 20.0))
    delta = float(rng.choice([120.0, rng.uniform(10.0, 900.0)]))

    mode = rng.random()
    if trace_widths:  # the reference traces' scale factors only
        mode = 0.0
    if mode < 0.6:
        pw = rng.dirichlet(np.ones(4))
        w = rng.choice(np.array([1, 2, 4, 8]), size=N, p=pw)
    elif mode < 0.85:
        w = rng.integers(1, max(2, min(255, max(G, 1)) + 1), size=N)
    else:  # some jobs wider than the cluster: accepted, never scheduled
        w = rng.integers(1, 17, size=N)
        wide = rng.random(N) < 0.1
        w[wide] = G + rng.integers(1, 300, size=int(wide.sum()))
    w = np.where(w <= G, np.minimum(w, 255), w).astype(np.int32)

    E = rng.integers(1, 201, size=N).astype(np.int32)
    F = np.floor(rng.uniform(0.0, 1.0, size=N) * (E + 1)).astype(np.int32)
    F = np.minimum(F, E)
    done = rng.random(N) < 0.03
    F[done] = E[done]
    if "done" in off:
        F = np.minimum(F, E - 1)
    d = np.maximum(1.0, np.round(rng.uniform(1.0, 20000.0, size=N) / E))
    if rng.random() < 0.2:
        d2 = np.round(d * rng.uniform(0.01, 0.2)) + 1.0
        d = d if "smalld" in off else d2
    R = (E - F) * d * rng.uniform(0.5, 1.5, size=N)
    r0 = rng.random(N) < 0.02
    R[r0 & ("r0" not in off)] = 0.0
    ftf = np.exp(rng.normal(np.log(1.5), 0.6, size=N))
    p = ftf ** lam
    p0 = rng.random(N) < 0.03
    p[p0 & ("p0" not in off)] = 0.0

    # exact duplicates: every key of a copied job ties with its source
    if N >= 4 and rng.random() < 0.5:
        ndup = int(rng.integers(1, max(2, N // 4)))
        src = rng.integers(0, N, size=ndup)
        dst = rng.integers(0, N, size=ndup)
        if "dup" not in off:
            for arr in (w, d, F, E, R, p):
                arr[dst] = arr[src]
    bases = _bases(rng)
    if "bases" in off:
        bases = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0)
    return sn.ProblemArrays(w, d, F, E, R, p, T, G, delta, k, bases)
