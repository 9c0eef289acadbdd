"""Round-loop simulator counterpart — SURVEY.md §8(f) row 1.

Restates the part of the reference's ``Scheduler.simulate()``
(scheduler/scheduler.py:1365-1796) that the Shockwave comparison runs:
trace-driven arrivals, fixed-length rounds on a homogeneous v100 cluster,
the Shockwave policy (plan solve on the GPU through ShockwaveScheduler) and
the Gavel MaxMinFairness baseline (allocation LP + deficit-based priorities),
dynamic batch-size scaling (GNS / Accordion) and the Fig-9 metrics.

What is kept from the reference, and where it lives:
  round loop, time jumps, completions heap   scheduler.py:1509-1778
  completion bookkeeping (_done_callback)    :3223-3484 (single-job ids only)
  step / finish-time model                   :1131-1212
  worker placement (strided, keep previous)  :838-890, :1017-1129
  Shockwave hooks                            :602-610, :435-448, :991-1014,
                                             :3590-3591, :3598-3621, :1731-1732
  GNS / Accordion triggers                   :1308-1363
  batch-size rescale of steps                :3488-3591
  MaxMinFairness priorities / deficits       :2589-2800, :892-989, :2351-2466
  metrics                                    :2131-2189, :3627-3655

What is not simulated (never reached by the Shockwave experiments):
job packing (pairs), throughput estimation, SLOs, spot prices, checkpoints,
the ``ideal`` mode and synthetic (non-trace) arrivals.  Job ids are plain
ints; the reference's ``JobIdPair(i, None)`` hashes and compares equal to
``i`` (job_id_pair.py), so dictionary behaviour is identical.

The policy decisions go through pluggable objects so the same loop runs with
the product solvers (HIP, default) or with the CPU oracles (tests only):
  * Shockwave: ``ShockwaveScheduler(config, solver=…)``;
  * MaxMinFairness: ``mmf_allocator(scale_factors, coefficients, G) → x``.
"""
from __future__ import annotations

import heapq
import math
from collections import OrderedDict

try:
    from . import sw_trace as st
    from .job_metadata import ShockwaveJobMetadata
    from .shockwave import ShockwaveScheduler
except ImportError:  # flat-module use
    import sw_trace as st
    from job_metadata import ShockwaveJobMetadata
    from shockwave import ShockwaveScheduler

BS_BIG = 0  # scheduler.py:61-62
BS_SMALL = 1
MAX_FAILED_ATTEMPTS = 5  # scheduler.py:49
WORKER_TYPE = "v100"  # the Shockwave hooks hard-code it (scheduler.py:1000, :3609)

POLICY_NAMES = {"shockwave": "Shockwave", "max_min_fairness": "MaxMinFairness"}


class Simulator:
    """One simulated cluster run (the reference's ``Scheduler`` with
    ``simulate=True``).

    policy:           "shockwave" or "max_min_fairness" (utils.get_policy names)
    throughputs:      {(job_type, scale_factor): v100 steps/s} (sw_trace.load_throughputs)
    profiles:         {int job id: profile dict} (the trace pickle; sw_trace.synthesize_profiles)
    shockwave_config: the JSON config + time_per_iteration + num_gpus (driver :60-70)
    shockwave_solver: solver object for ShockwaveScheduler (default: the HIP solver)
    mmf_allocator:    MaxMinFairness allocation function (default: the HIP kernel)
    """

    def __init__(self, policy, throughputs, profiles, time_per_iteration=120,
                 shockwave_config=None, shockwave_solver=None, mmf_allocator=None,
                 minimum_time_between_allocation_resets=1920, verbose=False):
        if policy not in POLICY_NAMES:
            raise ValueError(f"Unknown policy {policy!r} (supported: {sorted(POLICY_NAMES)})")
        self.policy_name = POLICY_NAMES[policy]
        self._oracle_throughputs = throughputs
        self._profiles = profiles
        self._time_per_iteration = time_per_iteration
        self._min_reset_interval = minimum_time_between_allocation_resets
        self._verbose = verbose
        self._current_timestamp = 0.0
        self._num_completed_rounds = 0
        self._job_id_counter = 0
        self._jobs = OrderedDict()
        self._throughputs = {}
        self._steps_run_so_far = {}
        self._total_steps_run = {}
        self._job_time_so_far = OrderedDict()
        self._worker_time_so_far = 0.0
        self._cumulative_worker_time_so_far = {}
        self._priorities = OrderedDict()
        self._deficits = {}
        self._allocation = {}
        self._need_to_update_allocation = False
        self._last_reset_time = 0.0
        self._per_job_start_timestamps = {}
        self._per_job_latest_timestamps = {}
        self._job_completion_times = OrderedDict()
        self._job_priority_weights = {}
        self._completed_jobs = set()
        self._running_jobs = set()
        self._num_failures_per_job = {}
        self._original_bs = {}
        self._bs_scale = {}
        self._num_jobs_in_trace = 0
        self._worker_ids = []
        self._current_worker_assignments = OrderedDict()
        self._current_round_scheduled_jobs = None
        self._gns_cache = {}
        self.num_solves = 0
        self.solve_seconds = 0.0
        if self.policy_name == "Shockwave":
            if shockwave_config is None:
                raise ValueError("the shockwave policy needs a configuration (driver :56-59)")
            self._shockwave = ShockwaveScheduler(shockwave_config, solver=shockwave_solver)
        else:
            self._shockwave = None
        self._mmf_allocator = mmf_allocator

    # ---- helpers ------------------------------------------------------------------
    def _log(self, msg):
        if self._verbose:
            print(msg)

    def _remaining_steps(self, job_id):  # scheduler.py:2834-2837
        return self._jobs[job_id].total_steps - self._total_steps_run[job_id]

    @staticmethod
    def _num_epochs(model, batch_size, num_steps):  # scheduler.py:3488-3494
        return math.ceil(num_steps / math.ceil(st.DATASET_SIZE[model] / batch_size))

    @staticmethod
    def _total_steps(model, batch_size, num_epochs):  # scheduler.py:3496-3502
        return num_epochs * math.ceil(st.DATASET_SIZE[model] / batch_size)

    # ---- jobs ---------------------------------------------------------------------
    def add_job(self, job, timestamp):
        """scheduler.py:537-619 (the fields the simulation reads)."""
        job_id = self._job_id_counter
        self._job_id_counter += 1
        job.job_id = job_id
        self._jobs[job_id] = job
        self._steps_run_so_far[job_id] = 0
        self._total_steps_run[job_id] = 0
        self._job_time_so_far[job_id] = self._time_per_iteration / 2.0
        self._throughputs[job_id] = self._oracle_throughputs[(job.job_type, job.scale_factor)]
        self._original_bs[job_id] = job.batch_size
        self._num_jobs_in_trace += 1
        self._num_failures_per_job[job_id] = 0
        self._priorities[job_id] = 0.0  # _add_to_priorities (:2640-2660)
        self._deficits[job_id] = 0.0
        self._need_to_update_allocation = True
        self._bs_scale[job_id] = None
        if self._shockwave is not None:
            md = ShockwaveJobMetadata(self._profiles[job_id], self._time_per_iteration,
                                      job.scale_factor)
            md.submit(self._current_timestamp)  # the current time, not the arrival (:607)
            self._shockwave.add_metadata(job_id, md)
        self._per_job_start_timestamps[job_id] = timestamp
        self._per_job_latest_timestamps[job_id] = None
        return job_id

    def _remove_job(self, job_id):
        """scheduler.py:627-705."""
        self._completed_jobs.add(job_id)
        duration = self._per_job_latest_timestamps[job_id] - self._per_job_start_timestamps[job_id]
        self._job_priority_weights[job_id] = self._jobs[job_id].priority_weight
        del self._jobs[job_id]
        if self._num_failures_per_job[job_id] >= MAX_FAILED_ATTEMPTS:
            self._job_completion_times[job_id] = None
        else:
            self._job_completion_times[job_id] = duration
        del self._steps_run_so_far[job_id]
        del self._job_time_so_far[job_id]
        del self._throughputs[job_id]
        del self._num_failures_per_job[job_id]
        self._priorities.pop(job_id, None)  # _remove_from_priorities (:2662-2682)
        self._deficits.pop(job_id, None)
        self._need_to_update_allocation = True

    # ---- completions ------------------------------------------------------------------
    def _done(self, job_id, num_steps, execution_time):
        """The aggregate part of _done_callback (scheduler.py:3223-3484) for one
        single-job micro-task: steps summed over its workers, time = max."""
        to_remove = []
        if job_id not in self._jobs:
            return
        succeeded = num_steps > 0 and execution_time > 0
        if not succeeded:
            self._num_failures_per_job[job_id] += 1
            if self._num_failures_per_job[job_id] >= MAX_FAILED_ATTEMPTS:
                to_remove.append(job_id)
            self._need_to_update_allocation = True
        else:
            self._num_failures_per_job[job_id] = 0
            if job_id in self._running_jobs:
                self._running_jobs.remove(job_id)
                self._steps_run_so_far[job_id] += num_steps
                self._total_steps_run[job_id] += num_steps
                if self._remaining_steps(job_id) <= 0:
                    to_remove.append(job_id)
            if job_id in self._job_time_so_far:
                self._job_time_so_far[job_id] += execution_time
                self._worker_time_so_far += execution_time
            for w in self._current_worker_assignments.get(job_id, ()):
                self._cumulative_worker_time_so_far[w] += execution_time
        # _update_throughput (:429-448): Shockwave records steps/s for this round
        if self._shockwave is not None and job_id in self._throughputs:
            tput = 0 if execution_time <= 0 else num_steps / execution_time
            md = self._shockwave.job_metadata.get(job_id)
            if md is not None:
                md.update_throughput_schedule(self._num_completed_rounds, tput,
                                              self._jobs[job_id].batch_size)
        self._scale_bs_and_iters(job_id)
        self._bs_scale[job_id] = None
        for jid in to_remove:
            self._remove_job(jid)
            if self._shockwave is not None:
                self._shockwave.delete_metadata(jid)

    def _scale_bs_and_iters(self, job_id):
        """scheduler.py:3504-3591: apply a pending batch-size change, keep the
        epoch count and the completed epochs."""
        if self._bs_scale.get(job_id) is None:
            return
        job = self._jobs[job_id]
        old_bs, model, mode = job.batch_size, job.model, job.mode
        original = self._original_bs[job_id]
        if st.MAX_BS.get(model) == original:
            self._bs_scale[job_id] = None
            return
        if mode == "gns":
            assert self._bs_scale[job_id] == BS_BIG
            new_bs = 2 * old_bs
        elif mode == "accordion":
            new_bs = st.MAX_BS[model] if self._bs_scale[job_id] == BS_BIG else original
        else:
            new_bs = old_bs
        job.update_bs(new_bs)
        key = (job.job_type, job.scale_factor)
        if key not in self._oracle_throughputs:
            self._log(f"Reverting job {job_id} bs: {new_bs} -> {old_bs}")
            self._bs_scale[job_id] = None
            job.update_bs(old_bs)
            return
        self._throughputs[job_id] = self._oracle_throughputs[key]
        total_steps = job.total_steps
        run = self._total_steps_run[job_id]
        old_epochs = self._num_epochs(model, old_bs, total_steps)
        new_total = math.ceil(total_steps * old_bs / new_bs)
        if self._num_epochs(model, new_bs, new_total) != old_epochs:
            new_total = self._total_steps(model, new_bs, old_epochs)
        job.total_steps = new_total
        done_epochs = self._num_epochs(model, old_bs, run)
        new_run = self._total_steps(model, new_bs, done_epochs)
        self._total_steps_run[job_id] = new_run
        self._steps_run_so_far[job_id] = new_run
        self._bs_scale[job_id] = None
        if self._shockwave is not None:
            self._shockwave.set_recompute_flag()

    # ---- batch-size triggers (scheduler.py:1308-1363) ---------------------------------
    def _gns_pattern(self, job, original_bs, n):
        key = (job.model, original_bs, job.scale_factor, n)
        pat = self._gns_cache.get(key)
        if pat is None:
            pat = st.gns_bs_pattern(job.job_type, original_bs, n, job.scale_factor)
            self._gns_cache[key] = pat
        return pat

    def _simulate_gns(self, job_id):
        job = self._jobs[job_id]
        bs = job.batch_size
        epoch = self._num_epochs(job.model, bs, self._total_steps_run[job_id])
        pat = self._gns_pattern(job, self._original_bs[job_id], max(760, epoch + 2))
        if pat[epoch + 1] > bs or pat[epoch] > bs:
            if st.MAX_BS.get(job.model) != bs:
                self._bs_scale[job_id] = BS_BIG

    def _simulate_accordion(self, job_id):
        job = self._jobs[job_id]
        bs, model = job.batch_size, job.model
        original = self._original_bs[job_id]
        epoch = self._num_epochs(model, bs, self._total_steps_run[job_id])
        if model == "Transformer":
            return
        critical = st.accordion_in_critical_regime(model, original, epoch)
        if bs == original and not critical:
            if st.MAX_BS.get(model) != bs:
                self._bs_scale[job_id] = BS_BIG
        elif bs != original and critical:
            if st.MIN_BS.get(model) != bs:
                self._bs_scale[job_id] = BS_SMALL

    # ---- Shockwave hooks ----------------------------------------------------------------
    def _shockwave_scheduler_update(self):
        """scheduler.py:3598-3621."""
        sw = self._shockwave
        for job_id in self._current_round_scheduled_jobs:
            if job_id in self._completed_jobs:
                if job_id in sw.job_metadata:
                    sw.job_metadata[job_id].complete()
                continue
            steps = self._steps_run_so_far.get(job_id, 0)
            if job_id in sw.job_metadata:
                job = self._jobs[job_id]
                spe = math.ceil(st.DATASET_SIZE[job.model] / job.batch_size)
                epoch = min(sw.job_metadata[job_id].total_epochs, math.floor(steps / spe))
                sw.job_metadata[job_id].complete(epoch)
        sw.increment_round()

    def _shockwave_schedule(self):
        """scheduler.py:991-1014: the cached plan's round, filtered to active jobs."""
        import time
        before = self._shockwave.last_solve
        t0 = time.perf_counter()
        self._current_round_scheduled_jobs = self._shockwave.current_round_schedule()
        dt = time.perf_counter() - t0
        if self._shockwave.last_solve is not before:
            self.num_solves += 1
            self.solve_seconds += dt
        assert self._current_round_scheduled_jobs is not None
        return [(j, self._jobs[j].scale_factor) for j in self._current_round_scheduled_jobs
                if j in self._jobs]

    # ---- MaxMinFairness (Gavel) ------------------------------------------------------------
    def _compute_allocation(self):
        """scheduler.py:2351-2466 → policies/max_min_fairness.py:14-95 for one
        worker type: MaxMinFairnessPolicy replaces every throughput by 1.0, the
        proportional throughput of each job is then 1.0 (proportional.py:27-44),
        so the LP is  max min_j c_j x_j  s.t.  Σ_j sf_j x_j ≤ G, 0 ≤ x_j ≤ 1
        with c_j = sf_j / priority_weight_j.  Jobs in sorted id order."""
        ids = sorted(self._jobs.keys())
        if not ids:
            return {}
        sf = [self._jobs[j].scale_factor for j in ids]
        coef = [self._jobs[j].scale_factor / self._jobs[j].priority_weight for j in ids]
        if self._mmf_allocator is None:
            try:
                from . import sw_native
            except ImportError:
                import sw_native
            self._mmf_allocator = sw_native.MmfAllocator()
        import time
        t0 = time.perf_counter()
        x = self._mmf_allocator(sf, coef, len(self._worker_ids))
        self.num_solves += 1
        self.solve_seconds += time.perf_counter() - t0
        return {j: min(1.0, max(0.0, float(v))) for j, v in zip(ids, x)}

    def _reset_time_run_so_far(self):
        """scheduler.py:2589-2638."""
        now = self._current_timestamp
        elapsed = now - self._last_reset_time
        half = self._time_per_iteration / 2.0
        self._worker_time_so_far = 0.0
        for job_id in self._job_time_so_far:
            received = self._job_time_so_far[job_id] - half
            should = self._allocation[job_id] * elapsed if job_id in self._allocation else 0
            self._deficits[job_id] = self._deficits.get(job_id, 0.0) + (should - received)
            self._job_time_so_far[job_id] = half
            self._worker_time_so_far += half
        self._last_reset_time = now

    def _update_priorities(self):
        """scheduler.py:2684-2800 (simulation branch)."""
        now = self._current_timestamp
        elapsed = (now - self._last_reset_time) >= self._min_reset_interval
        need = (elapsed or self._last_reset_time == 0) and self._need_to_update_allocation
        if need:
            self._reset_time_run_so_far()
            self._allocation = self._compute_allocation()
            self._need_to_update_allocation = False
        fractions = {}
        wt = self._worker_time_so_far
        for job_id in self._job_time_so_far:
            fractions[job_id] = 0.0 if wt == 0.0 else self._job_time_so_far[job_id] / wt
        for job_id in self._priorities:
            if job_id not in self._allocation:
                self._priorities[job_id] = 0.0
                continue
            a = self._allocation[job_id]
            prio = a * 1e9
            if a == 0.0:
                prio = 0.0
            elif self._throughputs[job_id] == 0:
                prio = 0
            elif fractions[job_id] > 0.0:
                prio = a / fractions[job_id]
            self._priorities[job_id] = prio

    def _mmf_schedule(self):
        """scheduler.py:892-989: greedy over (priority, deficit, allocation) desc."""
        left = len(self._worker_ids)
        entries = [(j, self._priorities[j], self._deficits[j], self._allocation.get(j, 0.0))
                   for j in self._priorities]
        entries.sort(key=lambda e: (e[1], e[2], e[3]), reverse=True)
        out = []
        for job_id, *_ in entries:
            if left == 0:
                continue
            if self._throughputs[job_id] <= 0:
                continue
            s = self._jobs[job_id].scale_factor
            if s > left:
                continue
            left -= s
            out.append((job_id, s))
        return out

    # ---- placement (scheduler.py:1017-1129, :838-890) ------------------------------------
    def _schedule_jobs_on_workers(self):
        if self._shockwave is None:
            self._update_priorities()
            scheduled = self._mmf_schedule()
        else:
            scheduled = self._shockwave_schedule()
        scheduled.sort(key=lambda x: x[1], reverse=True)
        free = list(self._worker_ids)  # one GPU per server (driver default "1:1:1")
        ptr = 0
        assigned = set()
        new = OrderedDict()
        for cur_sf in sorted({s for _, s in scheduled}, reverse=True):
            for job_id, s in scheduled:  # keep jobs on their previous workers
                if s != cur_sf or job_id not in self._current_worker_assignments:
                    continue
                prev = self._current_worker_assignments[job_id]
                if not any(w in assigned for w in prev):
                    new[job_id] = prev
                    assigned.update(prev)
            for job_id, s in scheduled:
                if s != cur_sf:
                    continue
                if self._shockwave is None and job_id not in self._allocation:
                    continue
                ids = list(new.get(job_id, ()))
                while len(ids) < s and ptr < len(free):
                    w = free[ptr]
                    if w not in assigned:
                        ids.append(w)
                        assigned.add(w)
                    ptr += 1
                if len(ids) != s:
                    raise RuntimeError(f"Could not assign workers to job {job_id}!")
                new[job_id] = tuple(ids)
                self._per_job_latest_timestamps[job_id] = self._current_timestamp
                self._running_jobs.add(job_id)
        return new

    def _steps_and_finish_time(self, job_id):
        """scheduler.py:1131-1212 for a single job."""
        tput = self._throughputs[job_id]
        steps = min(int(tput * self._time_per_iteration), self._remaining_steps(job_id))
        finish = self._current_timestamp
        if tput <= 0:
            raise RuntimeError(f"Throughput for job {job_id} should not be less than 0!")
        finish = max(finish, self._current_timestamp + steps / tput)
        self._running_jobs.add(job_id)
        return steps, finish

    # ---- the loop (scheduler.py:1365-1796, trace branch) -----------------------------------
    def simulate(self, num_gpus, arrival_times, jobs):
        """Runs the trace to completion and returns the makespan (seconds)."""
        self._worker_ids = list(range(num_gpus))
        self._cumulative_worker_time_so_far = {w: 0.0 for w in self._worker_ids}
        for i in range(1, len(arrival_times)):
            assert arrival_times[i] >= arrival_times[i - 1]
        queued = list(zip(arrival_times, jobs))
        remaining = len(jobs)
        running = []
        next_arrival = arrival_times[0] if arrival_times else 0
        round_start, round_end = 0.0, None
        self._current_timestamp = arrival_times[0] if arrival_times else 0.0
        while True:
            if remaining == 0:
                break
            if queued:
                next_arrival = queued[0][0]
            else:
                next_arrival = None
                if not running:
                    self._last_reset_time = 0
            max_ts = 0
            if running and -running[0][0] > max_ts:
                max_ts = -running[0][0]
                if round_end is not None:
                    round_start = round_end
                round_end = max_ts
            if max_ts > 0:
                self._current_timestamp = max_ts
            elif next_arrival is not None:
                self._current_timestamp = next_arrival
            while running:
                finish, job_id, workers, steps = running[0]
                finish = -finish
                if finish > self._current_timestamp:
                    break
                self._per_job_latest_timestamps[job_id] = finish
                self._done(job_id, steps, finish - round_start)
                if job_id not in self._jobs:
                    remaining -= 1
                heapq.heappop(running)
            for job_id in list(self._jobs.keys()):
                mode = self._jobs[job_id].mode
                if mode == "accordion":
                    self._simulate_accordion(job_id)
                elif mode == "gns":
                    self._simulate_gns(job_id)
            if self._shockwave is not None and self._num_completed_rounds >= 1:
                self._shockwave_scheduler_update()
            assert not running
            while queued and queued[0][0] <= self._current_timestamp:
                arrival, job = queued.pop(0)
                self.add_job(job, timestamp=arrival)
            if not self._jobs:
                break
            scheduled = self._schedule_jobs_on_workers()
            if self._shockwave is not None and len(scheduled) == 0:
                break  # scheduler.py:1731-1732
            self._current_worker_assignments = scheduled
            for job_id, workers in scheduled.items():
                steps, finish = self._steps_and_finish_time(job_id)
                heapq.heappush(running, (-finish, job_id, workers, steps))
            self._num_completed_rounds += 1
        return self._current_timestamp

    # ---- metrics -------------------------------------------------------------------------
    def get_average_jct(self):
        """scheduler.py:2131-2189."""
        jcts = [self._job_completion_times[j] for j in sorted(self._job_completion_times)
                if self._job_completion_times[j] is not None]
        return sum(jcts) / len(jcts) if jcts else None

    def get_finish_time_fairness(self):
        """scheduler.py:3627-3655: ρ = round(JCT / (isolated JCT × contention), 3),
        contention = max(1, jobs in trace / GPUs); unfair = % of ρ > 1.1."""
        if not self._job_completion_times:
            return None
        contention = max(1.0, self._num_jobs_in_trace / len(self._worker_ids))
        ftf = []
        for j in sorted(self._job_completion_times):
            jct = self._job_completion_times[j]
            if jct is None:
                continue
            iso = sum(self._profiles[j]["duration_every_epoch"])
            ftf.append(round(jct / (iso * contention), 3))
        unfair = 100 * sum(f > 1.1 for f in ftf) / len(ftf)
        return ftf, unfair

    def get_cluster_utilization(self):
        """Σ busy GPU-seconds / (GPUs × makespan)."""
        if self._current_timestamp <= 0:
            return 0.0
        busy = sum(self._cumulative_worker_time_so_far.values())
        return busy / (len(self._worker_ids) * self._current_timestamp)

    def summary(self):
        ftf, unfair = self.get_finish_time_fairness()
        return {
            "policy": self.policy_name,
            "num_gpus": len(self._worker_ids),
            "makespan": self._current_timestamp,
            "avg_jct": self.get_average_jct(),
            "worst_ftf": max(ftf),
            "unfair_fraction": unfair,
            "rounds": self._num_completed_rounds,
            "jobs_completed": len(self._job_completion_times),
            "solves": self.num_solves,
            "solve_seconds": self.solve_seconds,
            "utilization": self.get_cluster_utilization(),
            "jcts": {str(j): v for j, v in self._job_completion_times.items()},
        }


def run_trace(policy, trace_file, num_gpus, time_per_iteration=120, config=None,
              throughputs=None, shockwave_solver=None, mmf_allocator=None, max_jobs=None,
              verbose=False):
    """The driver's main() (simulate_scheduler_with_trace.py:27-133): parse the
    trace, synthesise the profiles (the missing pickle), set job durations from
    them (:37-39), simulate, and return the Fig-9 metrics."""
    tp = throughputs if throughputs is not None else st.load_throughputs()
    jobs, arrivals = st.parse_trace(trace_file)
    if max_jobs is not None:
        jobs, arrivals = jobs[:max_jobs], arrivals[:max_jobs]
    profiles = st.synthesize_profiles(jobs, tp)
    for i, j in enumerate(jobs):
        j.duration = sum(profiles[i]["duration_every_epoch"])
    sw_config = None
    if policy == "shockwave":
        sw_config = dict(config)
        sw_config["time_per_iteration"] = time_per_iteration
        sw_config["num_gpus"] = num_gpus
    sim = Simulator(policy, tp, profiles, time_per_iteration=time_per_iteration,
                    shockwave_config=sw_config, shockwave_solver=shockwave_solver,
                    mmf_allocator=mmf_allocator, verbose=verbose)
    sim.simulate(num_gpus, arrivals, jobs)
    return sim.summary()
