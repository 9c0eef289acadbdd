"""ctypes binding of the C-ABI in include/shockwave_amd.h.

This is the only way the host mirror reaches the solver: there is no Python
or CPU fallback.  If ``libshockwave_amd.so`` is missing or was built without
HIP the loader raises, so a product call can never silently run elsewhere.

The structs mirror include/shockwave_amd.h field for field.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libshockwave_amd.so"
LIB_PATH = os.path.join(_HERE, "lib", LIB_NAME)

SW_OK = 0
SW_FALLBACK = 1
SW_ERR_INVALID = -1
SW_ERR_HIP = -2
SW_ERR_CAPACITY = -3
SW_ERR_RCCL = -4
SW_ERR_NOT_BUILT = -5

SW_STATUS_P1_REPACKED = 0x1
SW_STATUS_P2_FALLBACK = 0x2
SW_STATUS_NO_PLANNED = 0x4
SW_STATUS_P2_WEIGHT_ORDER = 0x8
SW_STATUS_P2_CLASSWISE = 0x10
SW_STATUS_P2_REPAIRED = 0x20
SW_STATUS_P2_EXCHANGED = 0x40
SW_STATUS_P1_UNCERTIFIED = 0x80

SW_MAX_ROUNDS = 64
SW_MAX_BASES = 8
SW_NCCL_UNIQUE_ID_BYTES = 128

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_up = C.POINTER(C.c_uint8)


class SwProblem(C.Structure):
    _fields_ = [
        ("num_jobs", C.c_int32),
        ("future_rounds", C.c_int32),
        ("num_gpus", C.c_int32),
        ("num_bases", C.c_int32),
        ("round_duration", C.c_double),
        ("regularizer", C.c_double),
        ("bases", _dp),
        ("log_bases", _dp),
        ("nworkers", _ip),
        ("epoch_duration", _dp),
        ("completed_epochs", _ip),
        ("total_epochs", _ip),
        ("remaining_runtime", _dp),
        ("priority", _dp),
    ]


class SwResult(C.Structure):
    _fields_ = [
        ("plan", _up),
        ("planned_rounds", _ip),
        ("objective", C.c_double),
        ("utility", C.c_double),
        ("makespan", C.c_double),
        ("p2_objective", C.c_double),
        ("bound", C.c_double),
        ("iters", C.c_int32),
        ("status", C.c_int32),
        ("plan_masks", C.POINTER(C.c_uint64)),
    ]


class SwConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("max_instances", C.c_int32),
        ("max_total_jobs", C.c_int64),
        ("max_jobs_per_instance", C.c_int32),
        ("stream", C.c_void_p),
    ]


# sw_host_comm (include/shockwave_amd.h): blocking host collectives
ALLRED_I64 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_int32)
ALLRED_U64 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_int32)
ALLRED_F64 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int32)
ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)


class SwHostComm(C.Structure):
    _fields_ = [
        ("ctx", C.c_void_p),
        ("allreduce_sum_i64", ALLRED_I64),
        ("allreduce_max_u64", ALLRED_U64),
        ("allreduce_max_f64", ALLRED_F64),
        ("allgather", ALLGATHER),
    ]


class HostComm:
    """sw_host_comm backed by Python collectives.

    ``impl`` provides ``allgather_bytes(bytes) -> list[bytes]`` (rank order);
    every reduction is built from it, so any transport works: a
    torch.distributed gloo group (TorchGroupComm), or threads in tests.  The
    ctypes callbacks are kept alive by this object.
    """

    def __init__(self, impl):
        self.impl = impl
        self.error = None

        def guard(fn):
            def run(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # reported through the solve's return code
                    self.error = e
                    return -1
            return run

        def sum_i64(_ctx, buf, n):
            v = np.ctypeslib.as_array(buf, (n,))
            parts = self.impl.allgather_bytes(v.tobytes())
            v[:] = np.sum([np.frombuffer(b, np.int64) for b in parts], axis=0)

        def max_u64(_ctx, buf, n):
            v = np.ctypeslib.as_array(buf, (n,))
            parts = self.impl.allgather_bytes(v.tobytes())
            v[:] = np.max([np.frombuffer(b, np.uint64) for b in parts], axis=0)

        def max_f64(_ctx, buf, n):
            v = np.ctypeslib.as_array(buf, (n,))
            parts = self.impl.allgather_bytes(v.tobytes())
            v[:] = np.max([np.frombuffer(b, np.float64) for b in parts], axis=0)

        def gather(_ctx, send, recv, nbytes):
            mine = C.string_at(send, nbytes) if nbytes else b""
            parts = self.impl.allgather_bytes(mine)
            out = b"".join(parts)
            if out:
                C.memmove(recv, out, len(out))

        self._cbs = (ALLRED_I64(guard(sum_i64)), ALLRED_U64(guard(max_u64)),
                     ALLRED_F64(guard(max_f64)), ALLGATHER(guard(gather)))
        self.c = SwHostComm(None, *self._cbs)


class TorchGroupComm:
    """allgather_bytes over a torch.distributed process group (gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)

    def allgather_bytes(self, data: bytes):
        import torch

        t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else \
            torch.zeros(0, dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [o.numpy().tobytes() for o in out]


def shard_range(total_jobs: int, world: int, rank: int):
    """sw_dist_shard_range in Python (the same rule, for callers that slice)."""
    if world < 1 or 512 % world or not 0 <= rank < world or total_jobs < 0:
        raise ValueError("world must divide 512 and 0 <= rank < world")
    q = (total_jobs + 511) // 512
    per = (512 // world) * q
    return min(total_jobs, rank * per), min(total_jobs, (rank + 1) * per)


def log_bases(bases):
    """shockwave.py:99-105 — log(β_b), with log(0) replaced by log(1e-6)."""
    return [math.log(1e-6) if b == 0.0 else math.log(b) for b in bases]


class ProblemArrays:
    """Owns the contiguous numpy arrays behind one SwProblem (and its result).

    Fields follow include/shockwave_amd.h; see there for the reference line of
    each one.
    """

    def __init__(self, nworkers, epoch_duration, completed_epochs, total_epochs,
                 remaining_runtime, priority, future_rounds, num_gpus, round_duration,
                 regularizer, bases=(0.0, 0.2, 0.4, 0.6, 0.8, 1.0)):
        self.w = np.ascontiguousarray(nworkers, dtype=np.int32)
        self.d = np.ascontiguousarray(epoch_duration, dtype=np.float64)
        self.F = np.ascontiguousarray(completed_epochs, dtype=np.int32)
        self.E = np.ascontiguousarray(total_epochs, dtype=np.int32)
        self.R = np.ascontiguousarray(remaining_runtime, dtype=np.float64)
        self.p = np.ascontiguousarray(priority, dtype=np.float64)
        self.T = int(future_rounds)
        self.G = int(num_gpus)
        self.delta = float(round_duration)
        self.k = float(regularizer)
        self.bases = np.ascontiguousarray(bases, dtype=np.float64)
        self.ell = np.ascontiguousarray(log_bases(list(bases)), dtype=np.float64)
        n = len(self.w)
        for a in (self.d, self.F, self.E, self.R, self.p):
            if len(a) != n:
                raise ValueError("per-job arrays must have the same length")
        self.N = n
        self.plan = np.zeros((n, self.T), dtype=np.uint8)
        self.planned = np.zeros(n, dtype=np.int32)

    def c_problem(self) -> SwProblem:
        p = SwProblem()
        p.num_jobs = self.N
        p.future_rounds = self.T
        p.num_gpus = self.G
        p.num_bases = len(self.bases)
        p.round_duration = self.delta
        p.regularizer = self.k
        p.bases = self.bases.ctypes.data_as(_dp)
        p.log_bases = self.ell.ctypes.data_as(_dp)
        p.nworkers = self.w.ctypes.data_as(_ip)
        p.epoch_duration = self.d.ctypes.data_as(_dp)
        p.completed_epochs = self.F.ctypes.data_as(_ip)
        p.total_epochs = self.E.ctypes.data_as(_ip)
        p.remaining_runtime = self.R.ctypes.data_as(_dp)
        p.priority = self.p.ctypes.data_as(_dp)
        return p

    def slice(self, lo: int, hi: int) -> "ProblemArrays":
        """This instance's jobs [lo, hi) with the global scalars (a rank's shard)."""
        return ProblemArrays(self.w[lo:hi], self.d[lo:hi], self.F[lo:hi], self.E[lo:hi],
                             self.R[lo:hi], self.p[lo:hi], self.T, self.G, self.delta, self.k,
                             tuple(self.bases))

    def c_result(self) -> SwResult:
        r = SwResult()
        r.plan = self.plan.ctypes.data_as(_up)
        r.planned_rounds = self.planned.ctypes.data_as(_ip)
        return r


class DeviceShard:
    """One rank's jobs resident in HBM (torch tensors on `device`) for
    sw_dist_plan_solve_dev; plan [N, T] u8 and planned_rounds [N] i32 are
    device tensors the solve writes."""

    def __init__(self, arrays: ProblemArrays, device):
        import torch
        self.a = arrays
        dev = torch.device(device)
        self.w = torch.from_numpy(arrays.w).to(dev)
        self.d = torch.from_numpy(arrays.d).to(dev)
        self.F = torch.from_numpy(arrays.F).to(dev)
        self.E = torch.from_numpy(arrays.E).to(dev)
        self.R = torch.from_numpy(arrays.R).to(dev)
        self.p = torch.from_numpy(arrays.p).to(dev)
        self.plan = torch.zeros((arrays.N, arrays.T), dtype=torch.uint8, device=dev)
        self.planned = torch.zeros(arrays.N, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)  # the handle's stream does not order after torch's

    def c_problem(self) -> SwProblem:
        p = self.a.c_problem()  # scalars and the host bases table
        p.nworkers = C.cast(C.c_void_p(self.w.data_ptr()), _ip)
        p.epoch_duration = C.cast(C.c_void_p(self.d.data_ptr()), _dp)
        p.completed_epochs = C.cast(C.c_void_p(self.F.data_ptr()), _ip)
        p.total_epochs = C.cast(C.c_void_p(self.E.data_ptr()), _ip)
        p.remaining_runtime = C.cast(C.c_void_p(self.R.data_ptr()), _dp)
        p.priority = C.cast(C.c_void_p(self.p.data_ptr()), _dp)
        return p

    def c_result(self) -> SwResult:
        r = SwResult()
        r.plan = C.cast(C.c_void_p(self.plan.data_ptr()), _up)
        r.planned_rounds = C.cast(C.c_void_p(self.planned.data_ptr()), _ip)
        return r


def result_dict(r: SwResult, arrays: ProblemArrays, rc: int) -> dict:
    return {
        "rc": rc,
        "plan": arrays.plan.copy(),
        "planned_rounds": arrays.planned.copy(),
        "objective": r.objective,
        "utility": r.utility,
        "makespan": r.makespan,
        "p2_objective": r.p2_objective,
        "bound": r.bound,
        "iters": r.iters,
        "status": r.status,
    }


def declare_solver_api(lib, prefix: str):
    """Declare argtypes of a library exporting <prefix>plan_solve (product or twin)."""
    fn = getattr(lib, prefix + "plan_solve")
    fn.argtypes = [C.POINTER(SwProblem), C.POINTER(SwResult)] if prefix == "twin_" else \
        [C.c_void_p, C.POINTER(SwProblem), C.POINTER(SwResult)]
    fn.restype = C.c_int
    return fn


# Every symbol include/shockwave_amd.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "sw_abi_version", "sw_create", "sw_destroy", "sw_last_error", "sw_create_error",
    "sw_plan_solve", "sw_plan_solve_batch", "sw_batch_upload", "sw_batch_run",
    "sw_batch_download", "sw_stream", "sw_set_timing", "sw_kernel_times",
    "sw_dist_unique_id", "sw_dist_init", "sw_dist_plan_solve", "sw_dist_shard_range",
    "sw_dist_init_host", "sw_mmf_allocate", "sw_dist_plan_solve_dev", "sw_dist_enable_peer",
    "sw_mmf_allocate_types", "sw_batch_keep_masks",
)


class NativeError(RuntimeError):
    """A negative return code of the C-ABI; .code holds it."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


_LIB = None


def load(path: str | None = None):
    """Load libshockwave_amd.so (raises NativeError if it is absent)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # SW_LIB_PATH: an alternative in-tree build (A/B experiments, tools/)
    p = path or os.environ.get("SW_LIB_PATH") or LIB_PATH
    if not os.path.exists(p):
        raise NativeError(
            f"{p} not found: build it with `python __graft_entry__.py build` "
            "(there is no CPU fallback for the plan solver)")
    lib = C.CDLL(p)
    lib.sw_abi_version.restype = C.c_int
    lib.sw_create.argtypes = [C.POINTER(SwConfig)]
    lib.sw_create.restype = C.c_void_p
    lib.sw_destroy.argtypes = [C.c_void_p]
    lib.sw_destroy.restype = None
    lib.sw_last_error.argtypes = [C.c_void_p]
    lib.sw_last_error.restype = C.c_char_p
    lib.sw_create_error.argtypes = []
    lib.sw_create_error.restype = C.c_char_p
    lib.sw_plan_solve.argtypes = [C.c_void_p, C.POINTER(SwProblem), C.POINTER(SwResult)]
    lib.sw_plan_solve.restype = C.c_int
    lib.sw_plan_solve_batch.argtypes = [C.c_void_p, C.c_int32, C.POINTER(SwProblem),
                                        C.POINTER(SwResult)]
    lib.sw_plan_solve_batch.restype = C.c_int
    lib.sw_batch_upload.argtypes = [C.c_void_p, C.c_int32, C.POINTER(SwProblem)]
    lib.sw_batch_upload.restype = C.c_int
    lib.sw_batch_run.argtypes = [C.c_void_p]
    lib.sw_batch_run.restype = C.c_int
    lib.sw_batch_download.argtypes = [C.c_void_p, C.POINTER(SwResult)]
    lib.sw_batch_download.restype = C.c_int
    lib.sw_batch_keep_masks.argtypes = [C.c_void_p, C.c_int32]
    lib.sw_batch_keep_masks.restype = C.c_int
    lib.sw_stream.argtypes = [C.c_void_p]
    lib.sw_stream.restype = C.c_void_p
    lib.sw_set_timing.argtypes = [C.c_void_p, C.c_int32]
    lib.sw_set_timing.restype = C.c_int
    lib.sw_kernel_times.argtypes = [C.c_void_p, _dp, _dp, _ip]
    lib.sw_kernel_times.restype = C.c_int
    lib.sw_dist_unique_id.argtypes = [C.c_void_p]
    lib.sw_dist_unique_id.restype = C.c_int
    lib.sw_dist_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]
    lib.sw_dist_init.restype = C.c_int
    lib.sw_dist_plan_solve.argtypes = [C.c_void_p, C.POINTER(SwProblem), C.c_int64, C.c_int64,
                                       C.POINTER(SwResult)]
    lib.sw_dist_plan_solve.restype = C.c_int
    lib.sw_dist_plan_solve_dev.argtypes = [C.c_void_p, C.POINTER(SwProblem), C.c_int64, C.c_int64,
                                           C.POINTER(SwResult)]
    lib.sw_dist_plan_solve_dev.restype = C.c_int
    lib.sw_dist_shard_range.argtypes = [C.c_int64, C.c_int32, C.c_int32,
                                        C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.sw_dist_shard_range.restype = C.c_int
    lib.sw_dist_init_host.argtypes = [C.c_void_p, C.POINTER(SwHostComm), C.c_int32, C.c_int32]
    lib.sw_dist_init_host.restype = C.c_int
    lib.sw_dist_enable_peer.argtypes = [C.c_void_p, C.c_int64]
    lib.sw_dist_enable_peer.restype = C.c_int
    lib.sw_mmf_allocate.argtypes = [C.c_void_p, C.c_int32, C.c_int32, _ip, _dp, _dp, _dp]
    lib.sw_mmf_allocate.restype = C.c_int
    lib.sw_mmf_allocate_types.argtypes = [C.c_void_p, C.c_int32, C.c_int32, _ip, _ip, _dp, _dp, _dp]
    lib.sw_mmf_allocate_types.restype = C.c_int
    if path is None:
        _LIB = lib
    return lib


class Solver:
    """One device handle (sw_create / sw_destroy)."""

    def __init__(self, device=0, max_instances=1, max_total_jobs=0, max_jobs_per_instance=0,
                 stream=None, lib=None):
        self.lib = lib or load()
        cfg = SwConfig(int(device), int(max_instances), int(max_total_jobs),
                       int(max_jobs_per_instance), C.c_void_p(stream) if stream else None)
        h = self.lib.sw_create(C.byref(cfg))
        if not h:
            msg = self.lib.sw_create_error()
            raise NativeError("sw_create failed: " + (msg.decode() if msg else "?"))
        self.h = C.c_void_p(h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.sw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self) -> str:
        m = self.lib.sw_last_error(self.h)
        return m.decode() if m else ""

    def _check(self, rc, what):
        if rc < 0:
            raise NativeError(f"{what} failed ({rc}): {self.error()}", rc)
        return rc

    def solve(self, arrays: ProblemArrays) -> dict:
        prob = arrays.c_problem()
        res = arrays.c_result()
        rc = self._check(self.lib.sw_plan_solve(self.h, C.byref(prob), C.byref(res)),
                         "sw_plan_solve")
        return result_dict(res, arrays, rc)

    def solve_batch(self, batch: list, masks: bool = False, plan: bool = True) -> list:
        """sw_plan_solve_batch over host arrays.  masks=True also asks for the
        bit-packed plan (sw_result.plan_masks, one uint64 per job, returned as
        "plan_masks"); plan=False leaves the byte plan out (arrays.plan is not
        written)."""
        probs = (SwProblem * len(batch))(*[a.c_problem() for a in batch])
        ress = (SwResult * len(batch))(*[a.c_result() for a in batch])
        mk = []
        for i, a in enumerate(batch):
            if not plan:
                ress[i].plan = None
            if masks:
                m = np.zeros(a.N, dtype=np.uint64)
                ress[i].plan_masks = m.ctypes.data_as(C.POINTER(C.c_uint64))
                mk.append(m)
        rc = self._check(self.lib.sw_plan_solve_batch(self.h, len(batch), probs, ress),
                         "sw_plan_solve_batch")
        out = [result_dict(ress[i], a, rc) for i, a in enumerate(batch)]
        for d, m in zip(out, mk):
            d["plan_masks"] = m
        return out

    # device-resident batch (bench)
    def upload(self, batch: list):
        self._probs = (SwProblem * len(batch))(*[a.c_problem() for a in batch])
        self._batch = batch
        self._check(self.lib.sw_batch_upload(self.h, len(batch), self._probs), "sw_batch_upload")

    def run(self):
        self._check(self.lib.sw_batch_run(self.h), "sw_batch_run")

    def keep_masks(self, keep: bool):
        """sw_batch_keep_masks: whether sw_batch_run stores the bit-packed plans."""
        self._check(self.lib.sw_batch_keep_masks(self.h, 1 if keep else 0), "sw_batch_keep_masks")

    def download(self, masks: bool = False) -> list:
        """sw_batch_download; masks=True also asks for the bit-packed plans
        ("plan_masks", which the last run must have kept: keep_masks)."""
        ress = (SwResult * len(self._batch))(*[a.c_result() for a in self._batch])
        mk = []
        if masks:
            for i, a in enumerate(self._batch):
                m = np.zeros(max(a.N, 1), dtype=np.uint64)
                ress[i].plan_masks = m.ctypes.data_as(C.POINTER(C.c_uint64))
                mk.append(m)
        rc = self._check(self.lib.sw_batch_download(self.h, ress), "sw_batch_download")
        out = [result_dict(ress[i], a, rc) for i, a in enumerate(self._batch)]
        for d, m, a in zip(out, mk, self._batch):
            d["plan_masks"] = m[:a.N]
        return out

    def stream(self) -> int:
        return self.lib.sw_stream(self.h) or 0

    def set_timing(self, on: bool):
        self._check(self.lib.sw_set_timing(self.h, 1 if on else 0), "sw_set_timing")

    def kernel_times(self):
        a, b, n = C.c_double(), C.c_double(), C.c_int32()
        self._check(self.lib.sw_kernel_times(self.h, C.byref(a), C.byref(b), C.byref(n)),
                    "sw_kernel_times")
        return a.value, b.value, n.value

    # ---- Gavel MaxMinFairness allocation (include/shockwave_amd.h sw_mmf_allocate) ----
    def mmf_allocate(self, scale_factors, coefficients, num_workers: int):
        """x_j of the MaxMinFairness LP (one worker type); returns (x, t*, μ)."""
        sf = np.ascontiguousarray(scale_factors, dtype=np.int32)
        c = np.ascontiguousarray(coefficients, dtype=np.float64)
        if len(sf) != len(c):
            raise ValueError("scale_factors and coefficients must have the same length")
        x = np.zeros(len(sf), dtype=np.float64)
        lvl = np.zeros(2, dtype=np.float64)
        self._check(self.lib.sw_mmf_allocate(self.h, len(sf), int(num_workers),
                                             sf.ctypes.data_as(_ip), c.ctypes.data_as(_dp),
                                             x.ctypes.data_as(_dp), lvl.ctypes.data_as(_dp)),
                    "sw_mmf_allocate")
        return x, float(lvl[0]), float(lvl[1])

    def mmf_allocate_types(self, workers, scale_factors, coefficients):
        """x[j][k] of the heterogeneity-aware MaxMinFairness LP over worker
        types (sw_mmf_allocate_types); returns (x [m, n], t*, pivots)."""
        w = np.ascontiguousarray(workers, dtype=np.int32)
        sf = np.ascontiguousarray(scale_factors, dtype=np.int32)
        c = np.ascontiguousarray(coefficients, dtype=np.float64)
        if c.ndim != 2 or c.shape != (len(sf), len(w)):
            raise ValueError("coefficients must be [num_jobs][num_types]")
        x = np.zeros(c.shape, dtype=np.float64)
        lvl = np.zeros(2, dtype=np.float64)
        self._check(self.lib.sw_mmf_allocate_types(self.h, c.shape[0], c.shape[1], w.ctypes.data_as(_ip),
                                                   sf.ctypes.data_as(_ip), c.ctypes.data_as(_dp),
                                                   x.ctypes.data_as(_dp), lvl.ctypes.data_as(_dp)),
                    "sw_mmf_allocate_types")
        return x, float(lvl[0]), int(lvl[1])

    # ---- sharded single instance (include/shockwave_amd.h sw_dist_*) ----
    def dist_init(self, unique_id: bytes, rank: int, world: int):
        """RCCL collectives; unique_id from unique_id() on rank 0, broadcast by the caller."""
        buf = C.create_string_buffer(bytes(unique_id), SW_NCCL_UNIQUE_ID_BYTES)
        self._check(self.lib.sw_dist_init(self.h, buf, int(rank), int(world)), "sw_dist_init")

    def dist_init_host(self, comm: "HostComm", rank: int, world: int):
        """Host collectives (e.g. gloo through TorchGroupComm)."""
        self._comm = comm  # keeps the callbacks alive
        self._check(self.lib.sw_dist_init_host(self.h, C.byref(comm.c), int(rank), int(world)),
                    "sw_dist_init_host")

    def dist_enable_peer(self, max_total_jobs: int):
        """Peer-memory step transport (sw_dist_enable_peer): each step's
        collective becomes one kernel that writes into the other ranks'
        IPC-mapped exchange regions over xGMI; after dist_init or
        dist_init_host, on every rank."""
        self._check(self.lib.sw_dist_enable_peer(self.h, int(max_total_jobs)), "sw_dist_enable_peer")

    def dist_solve(self, local: ProblemArrays, job_offset: int, total_jobs: int) -> dict:
        prob = local.c_problem()
        res = local.c_result()
        rc = self.lib.sw_dist_plan_solve(self.h, C.byref(prob), int(job_offset), int(total_jobs),
                                         C.byref(res))
        comm = getattr(self, "_comm", None)
        if rc < 0 and comm is not None and comm.error is not None:
            raise NativeError(f"sw_dist_plan_solve: collective failed: {comm.error!r}")
        self._check(rc, "sw_dist_plan_solve")
        return result_dict(res, local, rc)

    def dist_solve_dev(self, shard: "DeviceShard", job_offset: int, total_jobs: int) -> dict:
        """sw_dist_plan_solve_dev: inputs and the plan stay in HBM (shard's
        tensors); only the scalar results come back."""
        prob, res = shard.c_problem(), shard.c_result()
        rc = self.lib.sw_dist_plan_solve_dev(self.h, C.byref(prob), int(job_offset),
                                             int(total_jobs), C.byref(res))
        self._check(rc, "sw_dist_plan_solve_dev")
        return {"rc": rc, "objective": res.objective, "utility": res.utility,
                "makespan": res.makespan, "p2_objective": res.p2_objective, "bound": res.bound,
                "iters": res.iters, "status": res.status}


class MmfAllocator:
    """The simulator's MaxMinFairness allocation function on the GPU:
    ``allocator(scale_factors, coefficients, num_workers) -> x``."""

    def __init__(self, device=0, solver=None):
        self.solver = solver or Solver(device=device)

    def __call__(self, scale_factors, coefficients, num_workers):
        return self.solver.mmf_allocate(scale_factors, coefficients, num_workers)[0]


def unique_id(lib=None) -> bytes:
    """sw_dist_unique_id (call on rank 0 only)."""
    lib = lib or load()
    buf = C.create_string_buffer(SW_NCCL_UNIQUE_ID_BYTES)
    rc = lib.sw_dist_unique_id(buf)
    if rc < 0:
        raise NativeError(f"sw_dist_unique_id failed ({rc})")
    return buf.raw
