"""Seeded synthetic plan-solve instances.

The reference's trace metadata pickles are missing (.MISSING_LARGE_BLOBS), so
every benchmark input is synthetic, shaped after the reference's traces and
configs:

  * scale factors w ∈ {1,2,4,8} with p = (0.6, 0.3, 0.09, 0.01) — the
    trace-name suffix of scheduler/traces/shockwave/*.trace;
  * isolated job durations 720–18,000 s split into E epochs (1–200), epoch
    durations rounded to ≥ 1 s as job_metadata.py:39 does;
  * completed epochs F ~ U[0, E), remaining runtime R within ±30 % of the
    remaining epochs' duration (the Dirichlet estimate of
    job_metadata.py:167-202 moves around the truth);
  * finish-time fairness FTF log-normal around 1.5, priority p = FTF**λ
    (shockwave.py:368);
  * (T, k, λ) per cluster size from scheduler/shockwave_replicate/
    scale_{64,128,256}gpus.json (32 GPUs uses the 64-GPU file; BASELINE.json
    overrides T to 30 for the 900-job / 256-GPU headline).
"""
from __future__ import annotations

import numpy as np

try:
    from .sw_native import ProblemArrays
except ImportError:  # flat-module use (reference-style sys.path import)
    from sw_native import ProblemArrays

BASES = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0)

# scale_{64,128,256}gpus.json: future_rounds, k, lambda (64: k=10, λ=5;
# 128: k=1e-3, λ=15; 256: k=1e5, λ=5); 32 GPUs has no JSON and uses 64's
CLUSTER_CONFIG = {
    32: dict(T=20, k=1e1, lam=5.0),
    64: dict(T=20, k=1e1, lam=5.0),
    128: dict(T=20, k=1e-3, lam=15.0),
    256: dict(T=20, k=1e5, lam=5.0),
}

# the headline configuration (BASELINE.json configs[2] / SURVEY.md §8 C3)
C3 = dict(N=900, T=30, G=256, delta=120.0, k=1e5, lam=5.0)
C4 = dict(N=10000, T=30, G=2848, delta=120.0, k=1e5, lam=5.0)


def synth_arrays(seed: int, N: int, G: int, T: int = 30, delta: float = 120.0, k: float = 1e5,
                 lam: float = 5.0, width_p=(0.6, 0.3, 0.09, 0.01)):
    """Per-job SoA inputs (w, d, F, E, R, p) of one plan solve."""
    rng = np.random.default_rng(seed)
    w = rng.choice(np.array([1, 2, 4, 8], dtype=np.int32), size=N, p=np.asarray(width_p))
    E = rng.integers(1, 201, size=N).astype(np.int32)
    duration = rng.uniform(720.0, 18000.0, size=N)
    d = np.maximum(1.0, np.round(duration / E))
    F = np.floor(rng.uniform(0.0, 1.0, size=N) * E).astype(np.int32)
    F = np.minimum(F, E - 1)
    R = (E - F) * d * rng.uniform(0.7, 1.3, size=N)
    ftf = np.exp(rng.normal(np.log(1.5), 0.45, size=N))
    p = ftf ** lam
    return w, d, F, E, R, p


def synth_problem(seed: int, N: int, G: int, T: int = 30, delta: float = 120.0, k: float = 1e5,
                  lam: float = 5.0, bases=BASES, **kw) -> ProblemArrays:
    w, d, F, E, R, p = synth_arrays(seed, N, G, T, delta, k, lam, **kw)
    return ProblemArrays(w, d, F, E, R, p, T, G, delta, k, bases)


def c3_problem(seed: int) -> ProblemArrays:
    c = C3
    return synth_problem(seed, c["N"], c["G"], c["T"], c["delta"], c["k"], c["lam"])


def sweep_problems(n_instances: int, N: int = 900, seed0: int = 0, T_override: int | None = 30):
    """C5: seeds × cluster sizes {32, 64, 128, 256}, configs from the matching JSON."""
    sizes = (32, 64, 128, 256)
    out = []
    for i in range(n_instances):
        G = sizes[i % len(sizes)]
        cfg = CLUSTER_CONFIG[G]
        T = T_override or cfg["T"]
        out.append(synth_problem(seed0 + i, N, G, T, 120.0, cfg["k"], cfg["lam"]))
    return out
