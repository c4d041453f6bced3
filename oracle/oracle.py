"""ORACLE (test infrastructure only) -- ctypes binding of oracle/pgo_oracle.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product path (graphslam_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")


class OrcParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int), ("relative_error_tol", C.c_double),
                ("absolute_error_tol", C.c_double), ("error_tol", C.c_double),
                ("lambda_initial", C.c_double), ("lambda_factor", C.c_double),
                ("lambda_upper_bound", C.c_double), ("lambda_lower_bound", C.c_double),
                ("min_model_fidelity", C.c_double), ("use_fixed_lambda_factor", C.c_int),
                ("algorithm", C.c_int), ("max_outer", C.c_int)]


class OrcStats(C.Structure):
    _fields_ = [("status", C.c_int), ("iterations", C.c_int), ("inner_iterations", C.c_int),
                ("linearizations", C.c_int), ("initial_error", C.c_double),
                ("final_error", C.c_double), ("t_total", C.c_double), ("t_linearize", C.c_double),
                ("t_factor", C.c_double), ("t_solve", C.c_double), ("t_error", C.c_double),
                ("factor_flops", C.c_double), ("nnz_l", C.c_double), ("nsuper", C.c_int),
                ("t_symbolic", C.c_double)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.c_int, C.c_int, ip, ip, dp, dp, C.c_int, ip, dp, dp, C.POINTER(C.c_int)]
        L.orc_create_ordered.restype = C.c_void_p
        L.orc_create_ordered.argtypes = [C.c_int, C.c_int, ip, ip, dp, dp, C.c_int, ip, dp, dp, ip,
                                         C.POINTER(C.c_int)]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_default_params.argtypes = [C.POINTER(OrcParams)]
        L.orc_optimize.argtypes = [C.c_void_p, dp, C.POINTER(OrcParams), dp, C.POINTER(OrcStats), dp,
                                   C.c_int, C.POINTER(C.c_int)]
        L.orc_linearize.argtypes = [C.c_void_p, dp, dp, dp, dp, dp]
        L.orc_solve.argtypes = [C.c_void_p, dp, C.c_double, dp]
        L.orc_error.argtypes = [C.c_void_p, dp]
        L.orc_error.restype = C.c_double
        L.orc_information.argtypes = [dp, dp]
        L.orc_closest_keyframe.argtypes = [C.c_int, dp, C.c_double, C.c_double, C.c_int, dp]
        L.orc_closest_keyframe.restype = C.c_int
        _lib = L
    return _lib


def set_threads(t):
    """OpenMP threads of later oracle calls."""
    lib().orc_set_threads(int(t))


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def closest_keyframe(xy, qx, qy, skip=10):
    """graph.cpp:146-178 restated in C: (index, distance) or (-1, nan)."""
    xy = np.ascontiguousarray(xy, dtype=np.float64)
    d = C.c_double(float("nan"))
    i = lib().orc_closest_keyframe(len(xy), _dp(xy), float(qx), float(qy), int(skip), C.byref(d))
    return i, d.value


def information(cov):
    cov = np.ascontiguousarray(cov, dtype=np.float64).reshape(9)
    om = np.zeros(9)
    rc = lib().orc_information(_dp(cov), _dp(om))
    return rc, om.reshape(3, 3)


@dataclass
class OracleResult:
    poses: np.ndarray
    stats: dict
    trace: np.ndarray


class Oracle:
    """CPU restatement of LevenbergMarquardtOptimizer(graph, initial).optimize()."""

    def __init__(self, g, order=None):
        """order (optional): new -> old pose permutation for the sparse Cholesky
        (e.g. the GPU plan's nested dissection, PoseGraph.debug_ordering());
        default: the oracle's own AMD."""
        L = lib()
        ei, ej = g.edge_index()
        self._keep = dict(
            ei=np.ascontiguousarray(ei, dtype=np.int32), ej=np.ascontiguousarray(ej, dtype=np.int32),
            ez=np.ascontiguousarray(g.edge_z, dtype=np.float64),
            ec=np.ascontiguousarray(g.edge_cov, dtype=np.float64),
            pi=np.ascontiguousarray(g.prior_index(), dtype=np.int32),
            pz=np.ascontiguousarray(g.prior_pose, dtype=np.float64),
            pc=np.ascontiguousarray(g.prior_cov, dtype=np.float64))
        k = self._keep
        st = C.c_int(0)
        self.n = g.num_poses
        self.ne = g.num_edges
        if order is not None:
            k["order"] = np.ascontiguousarray(order, dtype=np.int32)
            self.h = L.orc_create_ordered(self.n, self.ne, _ip(k["ei"]), _ip(k["ej"]), _dp(k["ez"]), _dp(k["ec"]),
                                          len(k["pi"]), _ip(k["pi"]), _dp(k["pz"]), _dp(k["pc"]),
                                          _ip(k["order"]), C.byref(st))
        else:
            self.h = L.orc_create(self.n, self.ne, _ip(k["ei"]), _ip(k["ej"]), _dp(k["ez"]), _dp(k["ec"]),
                                  len(k["pi"]), _ip(k["pi"]), _dp(k["pz"]), _dp(k["pc"]), C.byref(st))
        self.status = st.value
        if not self.h:
            raise ValueError(f"oracle rejected graph: status {st.value}")
        self.initial = np.ascontiguousarray(g.initial, dtype=np.float64)

    def close(self):
        if self.h:
            lib().orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def params(**kw):
        p = OrcParams()
        lib().orc_default_params(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def optimize(self, init=None, trace_cap=4096, **kw) -> OracleResult:
        init = self.initial if init is None else np.ascontiguousarray(init, dtype=np.float64)
        out = np.zeros((self.n, 3))
        tr = np.zeros((trace_cap, 7))
        ntr = C.c_int(0)
        st = OrcStats()
        p = self.params(**kw)
        lib().orc_optimize(self.h, _dp(init), C.byref(p), _dp(out), C.byref(st), _dp(tr), trace_cap,
                           C.byref(ntr))
        stats = {f: getattr(st, f) for f, _ in OrcStats._fields_}
        return OracleResult(out, stats, tr[: ntr.value].copy())

    def linearize(self, poses=None):
        poses = self.initial if poses is None else np.ascontiguousarray(poses, dtype=np.float64)
        hd = np.zeros((self.n, 3, 3))
        ho = np.zeros((self.ne, 3, 3))
        g = np.zeros((self.n, 3))
        err = C.c_double(0)
        lib().orc_linearize(self.h, _dp(poses), _dp(hd), _dp(ho), _dp(g), C.byref(err))
        return hd, ho, g, err.value

    def solve(self, lam, poses=None):
        poses = self.initial if poses is None else np.ascontiguousarray(poses, dtype=np.float64)
        d = np.zeros((self.n, 3))
        rc = lib().orc_solve(self.h, _dp(poses), lam, _dp(d))
        return rc, d

    def error(self, poses=None):
        poses = self.initial if poses is None else np.ascontiguousarray(poses, dtype=np.float64)
        return lib().orc_error(self.h, _dp(poses))


# ---------------------------------------------------------------- scan registration
def gicp_align(src, tgt, guess=None, k=20, eps=1e-3, max_it=200, max_inner=20, max_dist=5.0,
               trans_eps=5e-4, rot_eps=2e-3):
    """C restatement of the scanner's PCL GICP (gicp_oracle.c; scanner.cpp:35-50).
    Returns (T 4x4, iterations, converged, fitness); gicp_align.last_inner holds
    the optimiser steps of the call."""
    L = lib()
    L.orc_gicp_align.argtypes = [C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_float), C.c_int, C.c_int, C.c_double,
                                 C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.POINTER(C.c_double),
                                 C.POINTER(C.c_double)]
    s = np.ascontiguousarray(src, dtype=np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(tgt, dtype=np.float32).reshape(-1, 3)
    G = np.eye(4) if guess is None else np.asarray(guess, dtype=np.float64).reshape(4, 4)
    T12 = np.ascontiguousarray(np.concatenate([G[:3, :3].reshape(9), G[:3, 3]]))
    out = np.zeros(4)
    fp = C.POINTER(C.c_float)
    rc = L.orc_gicp_align(s.ctypes.data_as(fp), len(s), t.ctypes.data_as(fp), len(t), k, eps, max_it, max_inner,
                          max_dist, trans_eps, rot_eps, _dp(T12), _dp(out))
    if rc != 0:
        raise ValueError(f"orc_gicp_align: {rc}")
    T = np.eye(4)
    T[:3, :3] = T12[:9].reshape(3, 3)
    T[:3, 3] = T12[9:]
    gicp_align.last_inner = int(out[3])
    return T, int(out[0]), bool(out[1]), float(out[2])


def gicp_covariances(points, k=20, eps=1e-3):
    """computeCovariances restated: (n, 3, 3)."""
    L = lib()
    L.orc_gicp_covariances.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_double, C.POINTER(C.c_double)]
    p = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    c = np.zeros((len(p), 6))
    if L.orc_gicp_covariances(p.ctypes.data_as(C.POINTER(C.c_float)), len(p), k, eps, _dp(c)) != 0:
        raise ValueError("orc_gicp_covariances")
    out = np.empty((len(p), 3, 3))
    for a, (i, j) in enumerate([(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]):
        out[:, i, j] = out[:, j, i] = c[:, a]
    return out


def make_delta(T):
    """scanner.hpp:55-61 on the float transform: (T(0,3), T(1,3), atan(T(1,0) / T(0,0)))."""
    Tf = np.asarray(T, dtype=np.float32)
    return float(Tf[0, 3]), float(Tf[1, 3]), float(np.arctan(np.float64(Tf[1, 0] / Tf[0, 0])))


def compute_covariance(k_dd, k_rd, k_rr, delta):
    """scanner.hpp:64-80 (off-diagonals left 0; the reference leaves them uninitialised)."""
    dl = np.sqrt(delta[0] ** 2 + delta[1] ** 2)
    Q = np.zeros((3, 3))
    Q[0, 0] = Q[1, 1] = k_dd * dl
    Q[2, 2] = k_rd * dl + k_rr * delta[2]
    return Q


def registration(src, tgt, guess=None, **kw):
    """gicp() of scanner.cpp:35-74 restated end to end: (keyframe_flag, delta, Q, T, fitness)."""
    T, it, conv, fit = gicp_align(src, tgt, guess, **kw)
    d = make_delta(T)
    return conv and fit > 0.1, d, compute_covariance(0.1, 0.1, 0.1, d), T, fit, it
