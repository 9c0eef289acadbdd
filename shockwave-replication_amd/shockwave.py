"""ShockwaveScheduler — drop-in for the reference ``scheduler/shockwave.py``.

Same constructor and public methods (shockwave.py:12-91), consumed by the
reference's ``scheduler.py`` round loop in the same way:
``add_metadata`` (scheduler.py:610), ``delete_metadata`` (:3473),
``job_metadata`` read directly (:445-447, :3602-3619), ``set_recompute_flag``
(:3591), ``increment_round`` (:3621), ``current_round_schedule()``
(:1003).

What changes is the solve.  The reference builds P1 (EG / NSW MILP,
shockwave.py:330-388) and P2 (unfair-job prioritisation MILP, :281-328) in
CVXPY and hands both to Gurobi.  Here the host runs the estimators exactly
as the reference does (same call order and quirks, :111-134 and :255-278),
packs d_j, R_j, F_j, E_j, w_j and p_j = FTF_j^λ into SoA arrays and makes ONE
call through the C-ABI (include/shockwave_amd.h, sw_plan_solve) to the HIP
plan kernel on the GPU.  There is no CPU fallback: if the HIP library or the
GPU is missing, the solve raises.

Error behaviour mirrors the reference:
  * a P1 failure raises AssertionError (shockwave.py:382);
  * a P2 failure keeps the P1 placement (shockwave.py:325-326), reported by
    the library as SW_FALLBACK;
  * no planned job keeps the (empty) P1 placement (shockwave.py:319-320).
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import numpy as np

try:
    from .job_metadata import ShockwaveJobMetadata  # noqa: F401  (type of the metadata)
    from . import sw_native
except ImportError:  # reference-style flat import (directory on sys.path)
    from job_metadata import ShockwaveJobMetadata  # noqa: F401
    import sw_native


def _make_solver(config):
    device = int(config.get("device", os.environ.get("SW_DEVICE", 0)))
    return sw_native.Solver(device=device)


class ShockwaveScheduler(object):
    def __init__(self, shockwave_config: dict, solver=None):
        """shockwave.py:13-24.  ``solver`` (optional) is an object with a
        ``solve(ProblemArrays) -> dict`` method; by default a sw_native.Solver
        on the configured device, created on first use."""
        self.shockwave_config = shockwave_config
        self.num_gpus = shockwave_config["num_gpus"]
        self.round_duration = shockwave_config["time_per_iteration"]
        self.future_rounds = shockwave_config["future_rounds"]
        self.priority_power = shockwave_config["lambda"]
        self.regularizer = shockwave_config["k"]
        self.round_index = 0
        self.recompute_flag = False
        self.schedules = OrderedDict()
        self.job_metadata = OrderedDict()
        self.finish_time_estimates = {}
        self._solver = solver
        self.last_solve = None  # result dict of the last plan solve

    # ---- state API (shockwave.py:26-43) ------------------------------------
    @property
    def num_jobs(self):
        return len(self.job_metadata)

    def add_metadata(self, job_id, metadata):
        self.job_metadata[job_id] = metadata

    def delete_metadata(self, job_id):
        return self.job_metadata.pop(job_id, None)

    def increment_round(self):
        self.round_index += 1

    def set_recompute_flag(self):
        self.recompute_flag = True

    def unset_recompute_flag(self):
        self.recompute_flag = False

    # ---- the schedule call (shockwave.py:77-91) --------------------------------
    def current_round_schedule(self):
        print(f"Computing schedule in round {self.round_index} for {self.num_jobs} jobs")
        if not self.recompute_flag:
            if len(self.schedules) > 0 and self.round_index in self.schedules.keys():
                print("Using previous round schedule...")
                return self.schedules[self.round_index]
        plan = self._eisenberg_gale_program()
        self._generate_schedule(plan)
        self.unset_recompute_flag()
        return self.schedules[self.round_index]

    # ---- estimator inputs (shockwave.py:93-134, :224-279) ------------------------
    def _log_bases(self):
        return sw_native.log_bases(self.shockwave_config["log_approximation_bases"])

    def _compute_interpolated_finish_time(self, job_id, alpha=0.9):
        """History-weighted finish-time estimate (shockwave.py:224-242)."""
        history = self.finish_time_estimates[job_id]
        rounds = [r for r, _ in history]
        windows = np.diff(rounds)
        total = np.sum(windows)
        weights = np.array([1]) if total == 0 else windows / total
        times = np.array([ft for _, ft in history[: weights.size]])
        avg = np.dot(weights, times)
        return alpha * avg + (1 - alpha) * history[-1][1]

    def _gather_inputs(self):
        """Run the estimators in the reference's order and pack SoA arrays.

        Pass 1 over jobs = _job_log_utility (shockwave.py:111-134):
            call #1 recompute_epoch_duration(); d_j = mean(durations[:F+1]).
        Pass 2 over jobs = _compute_finish_times (shockwave.py:255-278):
            #2 R_mk, #3 R_jct, sum(durations[:F]) then #4 R_fin; append the
            finish-time estimate; FTF = JCT_pred / interpolated finish.
        Priority p_j = FTF_j ** λ (shockwave.py:368).
        """
        jobs = list(self.job_metadata.items())
        N = len(jobs)
        w = np.empty(N, dtype=np.int32)
        d = np.empty(N, dtype=np.float64)
        F = np.empty(N, dtype=np.int32)
        E = np.empty(N, dtype=np.int32)
        R = np.empty(N, dtype=np.float64)
        p = np.empty(N, dtype=np.float64)
        for i, (_, job) in enumerate(jobs):
            job.recompute_epoch_duration()
            d[i] = job.interpolated_epoch_duration() if hasattr(job, "interpolated_epoch_duration") \
                else float(np.mean(job.epoch_durations[: job.completed_epochs + 1]))
            w[i] = job.nworkers
            F[i] = job.completed_epochs
            E[i] = job.total_epochs
        contention = N / self.num_gpus
        round_time = (self.round_index + self.future_rounds) * self.round_duration
        ftf = np.empty(N, dtype=np.float64)
        for i, (job_id, job) in enumerate(jobs):
            R[i] = job.compute_remaining_runtime()
            remaining = job.compute_remaining_runtime()
            jct = round_time + remaining * contention
            done = job.completed_duration() if hasattr(job, "completed_duration") \
                else sum(job.epoch_durations[: job.completed_epochs])
            finish = done + job.compute_remaining_runtime()
            self.finish_time_estimates.setdefault(job_id, []).append((self.round_index, finish))
            ftf[i] = jct / self._compute_interpolated_finish_time(job_id)
        lam = self.priority_power
        for i in range(N):
            p[i] = float(ftf[i]) ** lam
        return sw_native.ProblemArrays(
            w, d, F, E, R, p, self.future_rounds, self.num_gpus, self.round_duration,
            self.regularizer, tuple(self.shockwave_config["log_approximation_bases"]))

    # ---- the solve (shockwave.py:330-388, :281-328, :400-411) ---------------------
    def _eisenberg_gale_program(self):
        """P1 + P2 on the GPU; returns the N×T 0/1 plan."""
        arrays = self._gather_inputs()
        if arrays.N == 0:
            self.last_solve = None
            return np.zeros((0, self.future_rounds), dtype=np.uint8)
        if self._solver is None:
            self._solver = _make_solver(self.shockwave_config)
        try:
            res = self._solver.solve(arrays)
        except sw_native.NativeError as e:
            raise AssertionError(f"P1 has no solution: {e}") from e  # shockwave.py:382
        if res["rc"] == sw_native.SW_FALLBACK:
            print("WARNING: Allocation returned by policy not optimal!")  # :409-410
        self.last_solve = res
        return res["plan"]

    def _generate_schedule(self, plan):
        """schedules[round_index + t] = job ids planned in round t, in
        job_metadata insertion order (shockwave.py:390-398)."""
        ids = list(self.job_metadata.keys())
        plan = np.asarray(plan)
        for t in range(self.future_rounds):
            col = plan[:, t] if plan.size else np.zeros(0, dtype=np.uint8)
            self.schedules[self.round_index + t] = [ids[j] for j in np.flatnonzero(col)]
