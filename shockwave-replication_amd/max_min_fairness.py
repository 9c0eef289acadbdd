"""Host mirror of the Gavel MaxMinFairness policies
(scheduler/policies/max_min_fairness.py:12-100, policy.py:14-63,
proportional.py:10-44) over the native allocation kernels.

Same names and call signature as the reference:
``policy.get_allocation(unflattened_throughputs, scale_factors,
priority_weights, cluster_spec)`` → ``{job_id: {worker_type: share}}`` (or
None when there are no jobs).  The ECOS solve (max_min_fairness.py:73-95) is
replaced by

  * one worker type: ``sw_mmf_allocate`` — the LP's level, and the analytic
    centre of its optimal face, the point ECOS converges to;
  * several worker types: ``sw_mmf_allocate_types`` — the same LP solved
    exactly by the simplex method on the GPU: the LP's optimal level, and an
    optimal vertex as the allocation (ECOS returns an interior point of the
    same optimal face, so the shares agree only where the optimum is unique).

The result is clipped to [0, 1] as ``x.value.clip(min=0.0).clip(max=1.0)``
(max_min_fairness.py:100).  A native error raises; there is no CPU fallback.

Known divergence (several worker types): where the LP's optimum is not
unique — typical for max-min LPs, and certain for the unit-throughput
``MaxMinFairnessPolicy`` with identical types — the per-job, per-type shares
are a vertex of the optimal face, not ECOS's interior point: the level t* is
the same, the split over jobs and types may differ.  The first such call
warns (``SimplexVertexWarning``); parity is unpinned (ECOS is absent here).
The simulator and every BASELINE configuration use one worker type.
"""
import warnings

import numpy as np

import sw_native


class SimplexVertexWarning(UserWarning):
    """The heterogeneous allocation is an optimal vertex, not ECOS's interior point."""


_WARNED = False


def _flatten(d, cluster_spec):
    """policy.py:28-44: jobs sorted by id, worker types sorted by name (from
    the first job), the throughput matrix and the per-type worker counts."""
    job_ids = sorted(d.keys())
    if len(job_ids) == 0:
        return None, None, None
    worker_types = sorted(d[job_ids[0]].keys())
    if len(worker_types) == 0:
        return None, None, None
    num_workers = [cluster_spec[wt] for wt in worker_types]
    m = np.array([[d[j][wt] for wt in worker_types] for j in job_ids], dtype=np.float64)
    return m, (job_ids, worker_types), num_workers


def _unflatten(x, index):
    job_ids, worker_types = index
    return {job_ids[i]: {worker_types[k]: x[i, k] for k in range(len(worker_types))}
            for i in range(len(job_ids))}


def _proportional_throughputs(throughputs, worker_types, cluster_spec):
    """ProportionalPolicy.get_throughputs (proportional.py:15-44): the cluster
    split evenly over the jobs, each row scaled to sum to at most 1."""
    m, _ = throughputs.shape
    x = np.array([[cluster_spec[wt] / m for wt in worker_types] for _ in range(m)])
    x = x / np.sum(x, axis=1).max()
    return np.sum(np.multiply(throughputs, x), axis=1).reshape((m, 1))


class MaxMinFairnessPolicyWithPerf:
    """max_min_fairness.py:37-100 (heterogeneity-aware: real throughputs)."""

    def __init__(self, solver="ECOS", native=None):
        self._name = "MaxMinFairness_Perf"
        self._solver = solver  # kept for the signature; the LP runs on the GPU
        self._native = native

    def _engine(self):
        if self._native is None:
            self._native = sw_native.Solver(device=0)
        return self._native

    def coefficients(self, unflattened_throughputs, scale_factors, unflattened_priority_weights,
                     cluster_spec):
        """The LP's coefficient matrix, in the reference's float operations
        (max_min_fairness.py:54-87): (throughputs · priority_weights) · scale
        factors, priority_weights = 1/w_j · 1/proportional throughput."""
        throughputs, index, num_workers = _flatten(unflattened_throughputs, cluster_spec)
        if throughputs is None:
            return None, None, None, None
        m, n = throughputs.shape
        job_ids, worker_types = index
        sf_array = np.array([[scale_factors[job_ids[i]]] * n for i in range(m)], dtype=np.float64)
        pw = np.array([1.0 / unflattened_priority_weights[j] for j in job_ids])
        prop = _proportional_throughputs(throughputs, worker_types, cluster_spec)
        pw = np.multiply(pw.reshape((m, 1)), 1.0 / prop.reshape((m, 1)))
        coef = np.multiply(throughputs * pw.reshape((m, 1)), sf_array)
        sf = np.array([scale_factors[j] for j in job_ids], dtype=np.int32)
        return coef, sf, index, num_workers

    def get_allocation(self, unflattened_throughputs, scale_factors, unflattened_priority_weights,
                       cluster_spec):
        coef, sf, index, num_workers = self.coefficients(
            unflattened_throughputs, scale_factors, unflattened_priority_weights, cluster_spec)
        if coef is None:
            return None
        eng = self._engine()
        if coef.shape[1] == 1 and (coef > 0.0).all():
            x, _, _ = eng.mmf_allocate(sf, coef[:, 0], int(num_workers[0]))
            x = x.reshape(-1, 1)
        else:
            global _WARNED
            if not _WARNED:
                _WARNED = True
                warnings.warn("MaxMinFairness over several worker types returns an optimal vertex of the "
                              "LP (GPU simplex); the reference's ECOS returns an interior point of the same "
                              "optimal face, so shares may differ where the optimum is not unique",
                              SimplexVertexWarning, stacklevel=2)
            x, _, _ = eng.mmf_allocate_types(num_workers, sf, coef)
        return _unflatten(x.clip(min=0.0).clip(max=1.0), index)


class MaxMinFairnessPolicy:
    """max_min_fairness.py:12-34: the WithPerf policy with every throughput 1.0
    (the Fig-9 "gavel" baseline)."""

    def __init__(self, solver="ECOS", native=None):
        self._name = "MaxMinFairness"
        self._max_min_fairness_perf_policy = MaxMinFairnessPolicyWithPerf(solver, native)

    def get_allocation(self, unflattened_throughputs, scale_factors, priority_weights, cluster_spec):
        if not unflattened_throughputs:
            return None
        ones = {j: {wt: 1.0 for wt in unflattened_throughputs[j]} for j in unflattened_throughputs}
        return self._max_min_fairness_perf_policy.get_allocation(ones, scale_factors, priority_weights,
                                                                 cluster_spec)
