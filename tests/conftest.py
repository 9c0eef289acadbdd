"""Shared test setup.

Markers: ``gpu`` tests need an MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on the CPU-only build container.

Import layout mirrors the reference: the product directory
``shockwave-replication_amd/`` is put on sys.path so its modules import as
``shockwave``, ``job_metadata`` … exactly like the reference's flat
``scheduler/`` modules.  ``oracle/`` is test infrastructure and is put on the
path only here.
"""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "shockwave-replication_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


TWIN_SO = os.environ.get("SW_TWIN_PATH") or os.path.join(ORACLE, "_build", "libplan_twin.so")


def _build_twin():
    if not os.path.exists(TWIN_SO):
        subprocess.check_call(["make", "-s", "-C", ORACLE])


@pytest.fixture(scope="session")
def twin():
    """The CPU bit-exact twin (oracle/plan_twin.c), loaded through ctypes."""
    _build_twin()
    import sw_native as sn

    lib = ctypes.CDLL(TWIN_SO)
    sn.declare_solver_api(lib, "twin_")
    lib.twin_eval_counts.argtypes = [ctypes.POINTER(sn.SwProblem), ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_double)]
    lib.twin_eval_counts.restype = ctypes.c_double

    class Twin:
        def solve(self, arrays):
            pr = arrays.c_problem()
            res = arrays.c_result()
            rc = lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))
            if rc < 0:
                raise ValueError(f"twin rejected the problem ({rc})")
            return sn.result_dict(res, arrays, rc)

        def rc(self, arrays):
            pr = arrays.c_problem()
            res = arrays.c_result()
            return lib.twin_plan_solve(ctypes.byref(pr), ctypes.byref(res))

        def eval_counts(self, arrays, counts):
            import numpy as np

            c = np.ascontiguousarray(counts, dtype=np.int32)
            mk = ctypes.c_double()
            pr = arrays.c_problem()
            obj = lib.twin_eval_counts(ctypes.byref(pr), c.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       ctypes.byref(mk))
            return obj, mk.value

    return Twin()


@pytest.fixture(scope="session")
def gpu_solver():
    """A product solver handle on cuda:0 (fails loudly if the HIP library is absent)."""
    import sw_native as sn

    s = sn.Solver(device=0)
    yield s
    s.close()
