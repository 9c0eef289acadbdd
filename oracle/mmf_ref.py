"""oracle/mmf_ref.py — TEST INFRASTRUCTURE for the MaxMinFairness allocation.

Two checkers for sw_mmf_allocate (include/shockwave_amd.h):
  * ``lp_level`` — the reference's LP (policies/max_min_fairness.py:68-93,
    policy.py:57-63, one worker type, unit throughputs) solved with scipy's
    HiGHS ``linprog``: returns the optimal min share t*.  The reference used
    ECOS through CVXPY; cvxpy/ecos are absent here, so the LP
    optimum is pinned by HiGHS on the identical model.
  * ``twin_allocate`` — oracle/mmf_twin.c, the bit-exact CPU twin of the HIP
    kernel, loaded through ctypes.
Only tests/ may import this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np
from scipy.optimize import linprog

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libmmf_twin.so")
_LIB = None


def lp_level(scale_factors, coefficients, num_workers):
    """max t s.t. t ≤ c_j x_j, Σ sf_j x_j ≤ G, 0 ≤ x_j ≤ 1 (variables [x, t])."""
    sf = np.asarray(scale_factors, dtype=np.float64)
    c = np.asarray(coefficients, dtype=np.float64)
    n = len(sf)
    obj = np.zeros(n + 1)
    obj[-1] = -1.0
    A = np.zeros((n + 1, n + 1))
    b = np.zeros(n + 1)
    A[:n, :n] = -np.diag(c)
    A[:n, n] = 1.0
    A[n, :n] = sf
    b[n] = num_workers
    bounds = [(0.0, 1.0)] * n + [(None, None)]
    r = linprog(obj, A_ub=A, b_ub=b, bounds=bounds, method="highs")
    assert r.status == 0, r.message
    return -r.fun, r.x[:n]


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = C.CDLL(_SO)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        lib.mmf_twin_allocate.argtypes = [C.c_int32, C.c_int32, ip, dp, dp, dp, dp]
        lib.mmf_twin_allocate.restype = C.c_int
        _LIB = lib
    return _LIB


def twin_allocate(scale_factors, coefficients, num_workers):
    """(x, t*, μ) from the CPU twin of the HIP kernel."""
    sf = np.ascontiguousarray(scale_factors, dtype=np.int32)
    c = np.ascontiguousarray(coefficients, dtype=np.float64)
    n = len(sf)
    x = np.zeros(n)
    lvl = np.zeros(2)
    scratch = np.zeros(max(n, 1))
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
    _lib().mmf_twin_allocate(n, int(num_workers), sf.ctypes.data_as(ip), c.ctypes.data_as(dp),
                             x.ctypes.data_as(dp), lvl.ctypes.data_as(dp),
                             scratch.ctypes.data_as(dp))
    return x, float(lvl[0]), float(lvl[1])


def twin_allocator(scale_factors, coefficients, num_workers):
    """The simulator's allocator interface backed by the twin."""
    return twin_allocate(scale_factors, coefficients, num_workers)[0]


def lp_level_types(workers, scale_factors, coefficients):
    """The heterogeneity-aware LP (policies/max_min_fairness.py:44-100 with
    policy.py:57-63), m jobs × n types, solved by HiGHS: max t s.t.
    t ≤ Σ_k coef[j][k]·x[j][k], Σ_j sf_j·x[j][k] ≤ workers[k], Σ_k x[j][k] ≤ 1,
    x ≥ 0.  Returns (t*, x[m][n])."""
    W = np.asarray(workers, dtype=np.float64)
    sf = np.asarray(scale_factors, dtype=np.float64)
    c = np.asarray(coefficients, dtype=np.float64)
    m, n = c.shape
    nv = m * n + 1
    obj = np.zeros(nv)
    obj[-1] = -1.0
    rows, b = [], []
    for j in range(m):
        r = np.zeros(nv)
        r[j * n:(j + 1) * n] = -c[j]
        r[-1] = 1.0
        rows.append(r)
        b.append(0.0)
    for k in range(n):
        r = np.zeros(nv)
        r[k:m * n:n] = sf
        rows.append(r)
        b.append(W[k])
    for j in range(m):
        r = np.zeros(nv)
        r[j * n:(j + 1) * n] = 1.0
        rows.append(r)
        b.append(1.0)
    res = linprog(obj, A_ub=np.array(rows), b_ub=np.array(b), bounds=[(0.0, None)] * nv, method="highs")
    assert res.status == 0, res.message
    return -res.fun, res.x[:m * n].reshape(m, n)


def twin_allocate_types(workers, scale_factors, coefficients):
    """(x[m][n], t*, pivots) from the CPU twin of the simplex kernel."""
    W = np.ascontiguousarray(workers, dtype=np.int32)
    sf = np.ascontiguousarray(scale_factors, dtype=np.int32)
    c = np.ascontiguousarray(coefficients, dtype=np.float64)
    m, n = c.shape
    x = np.zeros(m * n)
    lvl = np.zeros(2)
    piv = C.c_int64()
    lib = _lib()
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
    lib.mmf_twin_allocate_types.argtypes = [C.c_int32, C.c_int32, ip, ip, dp, dp, dp, C.POINTER(C.c_int64)]
    lib.mmf_twin_allocate_types.restype = C.c_int
    rc = lib.mmf_twin_allocate_types(m, n, W.ctypes.data_as(ip), sf.ctypes.data_as(ip), c.ctypes.data_as(dp),
                                     x.ctypes.data_as(dp), lvl.ctypes.data_as(dp), C.byref(piv))
    assert rc == 0, rc
    return x.reshape(m, n), float(lvl[0]), int(piv.value)
