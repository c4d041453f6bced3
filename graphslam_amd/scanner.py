"""Mirror of the scanner node's scan registration.

The reference (/root/reference/src/scanner/src/scanner.cpp) turns every laser
scan into a point cloud (``scan_to_pointcloud``, scanner.cpp:13-21,
laser_geometry's ``projectLaser``), registers it to the last keyframe's cloud
with PCL's Generalized-ICP (``gicp``, scanner.cpp:35-74) and, on a keyframe,
the closest keyframe's cloud to the last keyframe's (scanner.cpp:141) for a loop
closure.  The same names here:

    scanner.cpp:13   scan_to_pointcloud(LaserScan)      -> scan_to_pointcloud(ranges, ...)
    scanner.cpp:40   pcl::GeneralizedIterativeClosestPoint -> GeneralizedIterativeClosestPoint
    scanner.cpp:35   common::Registration gicp(in_1, in_2) -> gicp(in_1, in_2) -> Registration
    scanner.hpp:55   make_Delta(T)                       -> Registration.delta
    scanner.hpp:64   compute_covariance(0.1, 0.1, 0.1, D) -> Registration.covariance

Every registration runs in libpgo.so on the GPU (pgo_gicp_align_batch, one
workgroup per registration; no CPU fallback).  ``gicp_batch`` registers many
pairs in one launch -- the shape the live system has when a keyframe is
registered against its predecessor and its loop-closure candidate, or when a
map is rebuilt.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .pose_graph import PgoError

CONVERGED_FITNESS_THRESHOLD = 0.1   # scanner.cpp:10
K_DISP_DISP = K_ROT_DISP = K_ROT_ROT = 0.1   # scanner.cpp:11
MAX_POINTS = 4096


def scan_to_pointcloud(ranges, angle_min, angle_increment, range_min, range_max):
    """laser_geometry::LaserProjection::projectLaser (scanner.cpp:13-21): beam i at
    angle_min + i * angle_increment, kept when range_min <= r < range_max, as a
    float32 (n, 3) cloud in the laser frame (z = 0).  laser_geometry is not
    vendored in the reference; its published projection is restated."""
    r = np.asarray(ranges, dtype=np.float32)
    a = angle_min + np.arange(len(r), dtype=np.float64) * angle_increment
    keep = (r >= range_min) & (r < range_max)
    out = np.zeros((int(keep.sum()), 3), dtype=np.float32)
    out[:, 0] = r[keep] * np.cos(a[keep]).astype(np.float32)
    out[:, 1] = r[keep] * np.sin(a[keep]).astype(np.float32)
    return out


@dataclass
class Registration:
    """common::Registration's registration part (scanner.cpp:54-70)."""
    keyframe_flag: bool
    delta: tuple            # make_Delta: (x, y, theta)
    covariance: np.ndarray  # compute_covariance, 3 x 3
    transform: np.ndarray   # getFinalTransformation(), 4 x 4
    fitness: float          # getFitnessScore()
    converged: bool         # hasConverged()
    iterations: int
    inner_iterations: int = 0   # optimiser steps over all rounds


def default_params(**kw) -> L.PgoGicpParams:
    p = L.PgoGicpParams()
    L.lib().pgo_gicp_default_params(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(f"pgo_gicp_params has no field {k!r}")
        setattr(p, k, v)
    return p


_RESULT_DTYPE = np.dtype({"names": [f[0] for f in L.PgoGicpResult._fields_],
                          "formats": [(np.float64, 16), np.int32, np.int32, np.float64, (np.float64, 3),
                                      (np.float64, 9), np.int32, np.int32],
                          "offsets": [getattr(L.PgoGicpResult, f[0]).offset for f in L.PgoGicpResult._fields_],
                          "itemsize": C.sizeof(L.PgoGicpResult)})


class ScanRegistrar:
    """One pgo_gicp handle (a HIP stream on `device`)."""

    def __init__(self, device: int = 0):
        self._L = L.lib()
        self._h = self._L.pgo_gicp_create(int(device))
        if not self._h:
            raise MemoryError("pgo_gicp_create")

    def close(self):
        if self._h:
            self._L.pgo_gicp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def align_batch(self, sources, targets, guesses=None, params=None, arrays=False):
        """Register sources[b] -> targets[b] for every b in one launch; returns a
        list of Registration (arrays=True: a dict of numpy arrays over the whole
        batch -- T (B, 4, 4), delta (B, 3), cov (B, 3, 3), fitness, iterations,
        inner_iterations, converged, keyframe -- without per-pair objects).
        guesses: B x 4 x 4 (None: identity)."""
        B = len(sources)
        if len(targets) != B:
            raise ValueError("sources and targets differ in length")
        src = [np.ascontiguousarray(s, dtype=np.float32).reshape(-1, 3) for s in sources]
        tgt = [np.ascontiguousarray(t, dtype=np.float32).reshape(-1, 3) for t in targets]
        sn = np.array([len(s) for s in src], dtype=np.int32)
        tn = np.array([len(t) for t in tgt], dtype=np.int32)
        S = np.ascontiguousarray(np.concatenate(src) if B else np.zeros((0, 3), np.float32))
        T = np.ascontiguousarray(np.concatenate(tgt) if B else np.zeros((0, 3), np.float32))
        g = None
        if guesses is not None:
            g = np.ascontiguousarray(np.asarray(guesses, dtype=np.float64).reshape(B, 16))
        p = params if params is not None else default_params()
        res = (L.PgoGicpResult * max(B, 1))()
        fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int)
        rc = self._L.pgo_gicp_align_batch(self._h, B, S.ctypes.data_as(fp), sn.ctypes.data_as(ip),
                                          T.ctypes.data_as(fp), tn.ctypes.data_as(ip), L.dptr(g), C.byref(p), res)
        if rc != L.PGO_OK:
            raise PgoError(rc, self._L.pgo_gicp_last_error(self._h).decode())
        if arrays:
            rec = np.frombuffer(res, dtype=_RESULT_DTYPE, count=B)
            return {k: rec[k].copy() for k in _RESULT_DTYPE.names} | {
                "T": rec["T"].reshape(B, 4, 4).copy(), "cov": rec["cov"].reshape(B, 3, 3).copy()}
        out = []
        for b in range(B):
            r = res[b]
            out.append(Registration(keyframe_flag=bool(r.keyframe), delta=tuple(r.delta),
                                    covariance=np.array(r.cov[:]).reshape(3, 3),
                                    transform=np.array(r.T[:]).reshape(4, 4), fitness=r.fitness,
                                    converged=bool(r.converged), iterations=r.iterations,
                                    inner_iterations=r.inner_iterations))
        return out

    def device_ms(self):
        ms = C.c_double()
        self._L.pgo_gicp_debug_ms(self._h, C.byref(ms))
        return ms.value


_default = None


def _registrar():
    global _default
    if _default is None:
        _default = ScanRegistrar(0)
    return _default


def gicp(input_1, input_2) -> Registration:
    """scanner.cpp:35-74: register cloud input_1 (source) to input_2 (target)."""
    return _registrar().align_batch([input_1], [input_2])[0]


def gicp_batch(pairs, guesses=None, params=None):
    """Many gicp() calls in one launch: pairs = [(input_1, input_2), ...]."""
    return _registrar().align_batch([a for a, _ in pairs], [b for _, b in pairs], guesses, params)


class GeneralizedIterativeClosestPoint:
    """pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ>, the members the
    reference uses (scanner.cpp:40-50) plus the parameter setters."""

    def __init__(self, device: int = 0):
        self._reg = ScanRegistrar(device)
        self._p = default_params()
        self._src = self._tgt = None
        self._res = None

    def setInputSource(self, cloud):
        self._src = np.asarray(cloud, dtype=np.float32).reshape(-1, 3)

    def setInputTarget(self, cloud):
        self._tgt = np.asarray(cloud, dtype=np.float32).reshape(-1, 3)

    def setMaximumIterations(self, n):
        self._p.max_iterations = int(n)

    def setMaxCorrespondenceDistance(self, d):
        self._p.max_correspondence_distance = float(d)

    def setTransformationEpsilon(self, e):
        self._p.transformation_epsilon = float(e)

    def setRotationEpsilon(self, e):
        self._p.rotation_epsilon = float(e)

    def setCorrespondenceRandomness(self, k):
        self._p.k_correspondences = int(k)

    def setMaximumOptimizerIterations(self, n):
        self._p.max_inner_iterations = int(n)

    def align(self, guess=None):
        """Returns the source cloud transformed by the final transformation."""
        if self._src is None or self._tgt is None:
            raise ValueError("setInputSource / setInputTarget first")
        g = None if guess is None else [np.asarray(guess, dtype=np.float64).reshape(4, 4)]
        self._res = self._reg.align_batch([self._src], [self._tgt], g, self._p)[0]
        T = self._res.transform
        return (self._src.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)

    def hasConverged(self):
        return bool(self._res and self._res.converged)

    def getFitnessScore(self):
        return self._res.fitness

    def getFinalTransformation(self):
        return self._res.transform.astype(np.float32)
