"""GTSAM-named mirror of the surface /root/reference/src/graph/src/graph.cpp uses.

So a caller of the reference's path can switch with the same names, argument
meaning and error behaviour:

    graph.cpp:45   noiseModel::Gaussian::Covariance(Q)   -> noiseModel.Gaussian.Covariance(Q)
    graph.cpp:57   graph.add(PriorFactor<Pose2>(k, p, n))  -> graph.add(PriorFactorPose2(k, p, n))
    graph.cpp:58   initial.insert(k, Pose2(x, y, th))     -> initial.insert(k, Pose2(x, y, th))
    graph.cpp:87   graph.add(BetweenFactor<Pose2>(...))   -> graph.add(BetweenFactorPose2(...))
    graph.cpp:119  LevenbergMarquardtOptimizer(graph, initial).optimize()
                                                          -> same
    graph.cpp:123  poses_opti.at<Pose2>(k).x()            -> poses_opti.atPose2(k).x()
    graph.cpp:60   graph.nrFactors()                      -> graph.nrFactors()

The optimisation itself runs in libpgo.so on the GPU (no CPU fallback).
"""
from __future__ import annotations

import math

import numpy as np

from .pose_graph import (BadCovariance, IndeterminantLinearSystemException, PgoError, PoseGraph,  # noqa: F401
                         ValuesKeyAlreadyExists, ValuesKeyDoesNotExist, default_params)


class Pose2:
    """gtsam::Pose2 (x, y, theta); theta reported in (-pi, pi] like Rot2::theta()."""

    __slots__ = ("_x", "_y", "_t")

    def __init__(self, x=0.0, y=0.0, theta=0.0):
        self._x, self._y, self._t = float(x), float(y), float(theta)

    def x(self):
        return self._x

    def y(self):
        return self._y

    def theta(self):
        return math.atan2(math.sin(self._t), math.cos(self._t))

    def vector(self):
        return np.array([self._x, self._y, self.theta()])

    def __repr__(self):
        return f"Pose2({self._x!r}, {self._y!r}, {self.theta()!r})"


class _Gaussian:
    def __init__(self, cov):
        self.covariance = np.array(cov, dtype=np.float64).reshape(3, 3)

    @staticmethod
    def Covariance(Q):
        return _Gaussian(Q)

    @staticmethod
    def Information(I):
        return _Gaussian(np.linalg.inv(np.asarray(I, dtype=np.float64)))


class _Diagonal:
    @staticmethod
    def Sigmas(s):
        s = np.asarray(s, dtype=np.float64)
        return _Gaussian(np.diag(s * s))

    @staticmethod
    def Variances(v):
        return _Gaussian(np.diag(np.asarray(v, dtype=np.float64)))


class noiseModel:  # noqa: N801 -- mirrors gtsam::noiseModel
    Gaussian = _Gaussian
    Diagonal = _Diagonal


class PriorFactorPose2:
    def __init__(self, key, prior: Pose2, noise: _Gaussian):
        self.key, self.prior, self.noise = int(key), prior, noise

    def keys(self):
        return [self.key]


class BetweenFactorPose2:
    def __init__(self, key1, key2, measured: Pose2, noise: _Gaussian):
        self.key1, self.key2, self.measured, self.noise = int(key1), int(key2), measured, noise

    def keys(self):
        return [self.key1, self.key2]


class NonlinearFactorGraph:
    def __init__(self):
        self.factors = []

    def add(self, factor):
        if not isinstance(factor, (PriorFactorPose2, BetweenFactorPose2)):
            raise TypeError("only PriorFactorPose2 / BetweenFactorPose2 are on this path")
        self.factors.append(factor)

    push_back = add

    def size(self):
        return len(self.factors)

    def nrFactors(self):
        return len(self.factors)

    def error(self, values: "Values") -> float:
        """0.5 * sum e' Omega e, computed on the device."""
        with _build(self, values) as pg:
            return pg.error()


class Values:
    def __init__(self):
        self._keys = []
        self._xyt = {}

    def insert(self, key, pose: Pose2):
        key = int(key)
        if key in self._xyt:
            raise ValuesKeyAlreadyExists(-2, f"key {key} already inserted")
        self._keys.append(key)
        self._xyt[key] = (pose.x(), pose.y(), pose._t)

    def update(self, key, pose: Pose2):
        key = int(key)
        if key not in self._xyt:
            raise ValuesKeyDoesNotExist(-3, f"key {key} has no value")
        self._xyt[key] = (pose.x(), pose.y(), pose._t)

    def exists(self, key):
        return int(key) in self._xyt

    def atPose2(self, key) -> Pose2:
        key = int(key)
        if key not in self._xyt:
            raise ValuesKeyDoesNotExist(-3, f"key {key} has no value")
        return Pose2(*self._xyt[key])

    at = atPose2

    def size(self):
        return len(self._keys)

    def keys(self):
        return list(self._keys)

    def as_array(self):
        return np.array([self._xyt[k] for k in self._keys], dtype=np.float64).reshape(-1, 3)


class _Handle:
    def __init__(self, pg):
        self.pg = pg

    def __enter__(self):
        return self.pg

    def __exit__(self, *a):
        self.pg.close()


def _build(graph: NonlinearFactorGraph, values: Values, device=0):
    pg = PoseGraph(device)
    keys = values.keys()
    if keys:
        pg.add_vertices(np.array(keys, dtype=np.uint64), values.as_array())
    for f in graph.factors:
        if isinstance(f, PriorFactorPose2):
            pg.add_prior(f.key, [f.prior.x(), f.prior.y(), f.prior._t], f.noise.covariance)
        else:
            pg.add_edge(f.key1, f.key2, [f.measured.x(), f.measured.y(), f.measured._t], f.noise.covariance)
    return _Handle(pg)


class Marginals:
    """``gtsam::Marginals(graph, values)`` (graph.cpp:120, commented in the reference):
    ``marginalCovariance(key)`` -> 3x3 numpy array (x, y, theta)."""

    def __init__(self, graph: NonlinearFactorGraph, values: Values, device=0):
        self.graph, self.values, self.device = graph, values, device

    def marginalCovariance(self, key):
        return self.marginalCovariances([key])[0]

    def marginalCovariances(self, keys):
        with _build(self.graph, self.values, self.device) as pg:
            return pg.marginal_covariances(keys)


class LevenbergMarquardtParams:
    """gtsam::LevenbergMarquardtParams with GTSAM 4.0 defaults (+ PCG knobs)."""

    def __init__(self):
        self._p = default_params()

    def setMaxIterations(self, v):
        self._p.max_iterations = int(v)

    def setRelativeErrorTol(self, v):
        self._p.relative_error_tol = float(v)

    def setAbsoluteErrorTol(self, v):
        self._p.absolute_error_tol = float(v)

    def setErrorTol(self, v):
        self._p.error_tol = float(v)

    def setlambdaInitial(self, v):
        self._p.lambda_initial = float(v)

    def setlambdaFactor(self, v):
        self._p.lambda_factor = float(v)

    def setlambdaUpperBound(self, v):
        self._p.lambda_upper_bound = float(v)

    def setlambdaLowerBound(self, v):
        self._p.lambda_lower_bound = float(v)

    def setUseFixedLambdaFactor(self, v):
        self._p.use_fixed_lambda_factor = int(bool(v))

    def setPcgRelativeTol(self, v):
        self._p.pcg_relative_tol = float(v)

    @property
    def raw(self):
        return self._p


class GaussNewtonParams(LevenbergMarquardtParams):
    def __init__(self):
        super().__init__()
        self._p.algorithm = 1


class LevenbergMarquardtOptimizer:
    """``LevenbergMarquardtOptimizer(graph, initial[, params]).optimize()`` (graph.cpp:119)."""

    _params_cls = LevenbergMarquardtParams

    def __init__(self, graph: NonlinearFactorGraph, initial: Values, params=None, device=0):
        self.graph, self.initial = graph, initial
        self.params = params if params is not None else self._params_cls()
        self.device = device
        self.stats = None
        self._handle = None

    def optimize(self) -> Values:
        """GTSAM keeps the optimizer's state: the graph is loaded on the first
        call, a later call continues from the values the previous one reached."""
        if self._handle is None:
            self._handle = _build(self.graph, self.initial, self.device)
        pg = self._handle.pg
        self.stats = pg.optimize(self.params.raw)
        xyt = pg.poses()
        out = Values()
        for k, p in zip(self.initial.keys(), xyt):
            out.insert(k, Pose2(*p))
        return out

    def iterations(self):
        return self.stats["iterations"] if self.stats else 0

    def error(self):
        return self.stats["final_error"] if self.stats else None


class GaussNewtonOptimizer(LevenbergMarquardtOptimizer):
    _params_cls = GaussNewtonParams
