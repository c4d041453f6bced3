"""ORACLE (test infrastructure only) -- numpy/scipy twin of the reference path.

This module is a CPU restatement of what ``src/graph/src/graph.cpp:119``
(``gtsam::LevenbergMarquardtOptimizer(graph, initial).optimize()``) computes on
the factor graph built by ``graph.cpp:27-113``.  The arithmetic lives in GTSAM,
which is NOT vendored in /root/reference, NOT installed here and NOT version
pinned (``src/graph/CMakeLists.txt:9`` has ``find_package(GTSAM REQUIRED)`` with
no version).  The semantics restated below follow GTSAM 4.0.x's
published source (tags [GTSAM] below name the upstream function):

* Pose2 = (t, Rot2(c, s)); ``Rot2::normalize`` rescales (c, s) only when
  |c^2+s^2-1| > 1e-10; ``Rot2::atan2``/``fromCosSin`` normalize, ``fromAngle``
  does not; ``theta() = atan2(s, c)``.                      [GTSAM Rot2.cpp]
* ``Pose2::between`` with its closed-form H1 and H2 = I.    [GTSAM Pose2.cpp]
* Default chart (no SLOW_BUT_CORRECT_EXPMAP): Local(p) = (x, y, theta),
  Retract(v) = p * Pose2(v0, v1, v2).                       [GTSAM Pose2.cpp]
* BetweenFactor e = Local(z, between(p1, p2)), J1 = H1, J2 = I (no Hlocal;
  SLOW_BUT_CORRECT_BETWEENFACTOR off).                      [GTSAM BetweenFactor.h]
* PriorFactor e = -Local(x, prior), H = I.                  [GTSAM PriorFactor.h]
* ``noiseModel::Gaussian::Covariance(Q)`` (graph.cpp:45,83,103): smart check --
  every off-diagonal |Q_ij| <= 1e-9 -> Diagonal::Variances(diag Q); otherwise
  Information(Q^-1) whose R = LLT(Q^-1).matrixU() reads the LOWER triangle of
  Q^-1, so Omega = R^T R = the lower triangle of Q^-1 mirrored.  [GTSAM NoiseModel.cpp]
* LM: defaults lambda0=1e-5, factor 10 (fixed), upper 1e5, lower 0,
  minModelFidelity 1e-3, diagonalDamping off -> (H + lambda I) delta = -g;
  ``tryLambda`` accept rule and ``checkConvergence`` with maxIterations=100,
  relTol=absTol=1e-5, errTol=0.   [GTSAM LevenbergMarquardtOptimizer.cpp,
  NonlinearOptimizer.cpp]
* error = sum over factors of 0.5 * e^T Omega e.

Parity status: GTSAM cannot be run here and the reference holds no tests,
fixtures or golden vectors for this path, so this twin is **parity unpinned**
against GTSAM itself; it is pinned by known-answer graphs (noise-free loops
converge to ground truth), finite-difference Jacobian checks and agreement with
the independent C restatement ``oracle/pgo_oracle.c`` (tests/test_oracle.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

NORMALIZE_TOL = 1e-10
DIAG_TOL = 1e-9


class BadCovariance(ValueError):
    pass


class Indeterminant(RuntimeError):
    pass


# ---------------------------------------------------------------- Pose2 algebra
def normalize(c, s):
    c = np.array(c, dtype=np.float64, copy=True)
    s = np.array(s, dtype=np.float64, copy=True)
    scale = c * c + s * s
    m = np.abs(scale - 1.0) > NORMALIZE_TOL
    if np.any(m):
        f = scale[m] ** -0.5
        c[m] *= f
        s[m] *= f
    return c, s


def from_xyt(xyt):
    """Pose2(x, y, theta) -> (x, y, c, s) with Rot2::fromAngle (no normalize)."""
    xyt = np.asarray(xyt, dtype=np.float64).reshape(-1, 3)
    return np.stack([xyt[:, 0], xyt[:, 1], np.cos(xyt[:, 2]), np.sin(xyt[:, 2])], axis=1)


def to_xyt(p):
    return np.stack([p[:, 0], p[:, 1], np.arctan2(p[:, 3], p[:, 2])], axis=1)


def between(a, b):
    """a^-1 * b with the rotation built by Rot2::atan2 (normalized)."""
    c1, s1, c2, s2 = a[:, 2], a[:, 3], b[:, 2], b[:, 3]
    c, s = normalize(c1 * c2 + s1 * s2, -s1 * c2 + c1 * s2)
    dx, dy = b[:, 0] - a[:, 0], b[:, 1] - a[:, 1]
    return np.stack([c1 * dx + s1 * dy, -s1 * dx + c1 * dy, c, s], axis=1)


def between_jacobian(a, b, hx):
    """H1 of Pose2::between (= -AdjointMap(between(b, a)) inlined)."""
    c, s = hx[:, 2], hx[:, 3]
    x, y = b[:, 0] - a[:, 0], b[:, 1] - a[:, 1]
    c2, s2 = b[:, 2], b[:, 3]
    n = a.shape[0]
    J = np.zeros((n, 3, 3))
    J[:, 0, 0] = -c
    J[:, 0, 1] = -s
    J[:, 0, 2] = -s2 * x + c2 * y
    J[:, 1, 0] = s
    J[:, 1, 1] = -c
    J[:, 1, 2] = -c2 * x - s2 * y
    J[:, 2, 2] = -1.0
    return J


def local(a, b):
    d = between(a, b)
    return np.stack([d[:, 0], d[:, 1], np.arctan2(d[:, 3], d[:, 2])], axis=1)


def retract(p, d):
    """p * Pose2(d0, d1, d2) (default Pose2 chart)."""
    cd, sd = np.cos(d[:, 2]), np.sin(d[:, 2])
    c, s = p[:, 2], p[:, 3]
    nc, ns = normalize(c * cd - s * sd, s * cd + c * sd)
    return np.stack([p[:, 0] + c * d[:, 0] - s * d[:, 1],
                     p[:, 1] + s * d[:, 0] + c * d[:, 1], nc, ns], axis=1)


# --------------------------------------------------------------- noise models
def information(cov):
    """Omega for noiseModel::Gaussian::Covariance(cov) (cov: [K,9] row-major)."""
    cov = np.asarray(cov, dtype=np.float64).reshape(-1, 3, 3)
    om = np.zeros_like(cov)
    for k in range(cov.shape[0]):
        q = cov[k]
        off = q - np.diag(np.diag(q))
        if np.all(np.abs(off) <= DIAG_TOL):
            v = np.diag(q)
            if np.any(~(v > 0.0)) or not np.all(np.isfinite(v)):
                raise BadCovariance(f"factor {k}: non-positive variance {v}")
            om[k] = np.diag(1.0 / v)
            continue
        try:
            inv = np.linalg.inv(q)
        except np.linalg.LinAlgError as exc:
            raise BadCovariance(f"factor {k}: singular covariance") from exc
        low = np.tril(inv)
        sym = low + np.tril(inv, -1).T
        try:
            np.linalg.cholesky(sym)
        except np.linalg.LinAlgError as exc:
            raise BadCovariance(f"factor {k}: covariance inverse not positive definite") from exc
        om[k] = sym
    return om


# --------------------------------------------------------------------- graph
@dataclass
class Problem:
    n: int
    ei: np.ndarray
    ej: np.ndarray
    ez: np.ndarray          # [E,4] (x,y,c,s)
    eom: np.ndarray         # [E,3,3]
    pi: np.ndarray
    pz: np.ndarray          # [P,4]
    pom: np.ndarray         # [P,3,3]


def problem_from_graph(g):
    ei, ej = g.edge_index()
    return Problem(n=g.num_poses, ei=np.asarray(ei), ej=np.asarray(ej), ez=from_xyt(g.edge_z),
                   eom=information(g.edge_cov), pi=g.prior_index(), pz=from_xyt(g.prior_pose),
                   pom=information(g.prior_cov))


def residuals(prob: Problem, poses):
    p1, p2 = poses[prob.ei], poses[prob.ej]
    hx = between(p1, p2)
    ee = local(prob.ez, hx)
    ep = -local(poses[prob.pi], prob.pz)
    return ee, ep, p1, p2, hx


def error(prob: Problem, poses):
    ee, ep, *_ = residuals(prob, poses)
    return 0.5 * (np.einsum("ei,eij,ej->", ee, prob.eom, ee) + np.einsum("ei,eij,ej->", ep, prob.pom, ep))


@dataclass
class Linear:
    H: sp.csc_matrix
    g: np.ndarray
    ee: np.ndarray
    ep: np.ndarray
    J1: np.ndarray
    err0: float


def linearize(prob: Problem, poses) -> Linear:
    ee, ep, p1, p2, hx = residuals(prob, poses)
    J1 = between_jacobian(p1, p2, hx)
    om = prob.eom
    B = np.einsum("eki,ekl->eil", J1, om)            # J1^T Omega   (block (i,j))
    D1 = np.einsum("eil,elj->eij", B, J1)            # J1^T Omega J1
    g1 = np.einsum("eil,el->ei", B, ee)
    g2 = np.einsum("eil,el->ei", om, ee)
    n = prob.n
    rows, cols, vals = [], [], []

    def add_block(r, c, blk):
        ii = (3 * r[:, None, None] + np.arange(3)[None, :, None]).repeat(3, axis=2)
        jj = (3 * c[:, None, None] + np.arange(3)[None, None, :]).repeat(3, axis=1)
        rows.append(ii.ravel())
        cols.append(jj.ravel())
        vals.append(blk.ravel())

    add_block(prob.ei, prob.ei, D1)
    add_block(prob.ej, prob.ej, om)
    add_block(prob.ei, prob.ej, B)
    add_block(prob.ej, prob.ei, np.transpose(B, (0, 2, 1)))
    add_block(prob.pi, prob.pi, prob.pom)
    H = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(3 * n, 3 * n)).tocsc()
    g = np.zeros((n, 3))
    np.add.at(g, prob.ei, g1)
    np.add.at(g, prob.ej, g2)
    gp = np.einsum("pij,pj->pi", prob.pom, ep)
    np.add.at(g, prob.pi, gp)
    err0 = 0.5 * (np.einsum("ei,eij,ej->", ee, om, ee) + np.einsum("ei,eij,ej->", ep, prob.pom, ep))
    return Linear(H=H, g=g.ravel(), ee=ee, ep=ep, J1=J1, err0=err0)


def linear_error(prob: Problem, lin: Linear, delta):
    """GaussianFactorGraph::error(delta) = 0.5 sum |R (J delta + e)|^2."""
    d = delta.reshape(-1, 3)
    re = lin.ee + np.einsum("eij,ej->ei", lin.J1, d[prob.ei]) + d[prob.ej]
    rp = lin.ep + d[prob.pi]
    return 0.5 * (np.einsum("ei,eij,ej->", re, prob.eom, re) + np.einsum("ei,eij,ej->", rp, prob.pom, rp))


def solve(H, rhs, lam):
    A = (H + lam * sp.identity(H.shape[0], format="csc")).tocsc() if lam else H
    try:
        lu = spla.splu(A, permc_spec="COLAMD")
    except RuntimeError as exc:          # "Factor is exactly singular"
        raise Indeterminant(str(exc)) from exc
    x = lu.solve(rhs)
    if not np.all(np.isfinite(x)):
        raise Indeterminant("non-finite solution")
    return x


# ------------------------------------------------------------------ optimizers
def marginal_covariances(prob: Problem, poses, idx):
    """gtsam::Marginals(graph, values).marginalCovariance(key) (used, commented
    out, at graph.cpp:120,126-127): the 3x3 block of H^-1 of each pose in idx, H =
    J'Omega J at `poses` (no damping).  Columns of H^-1 by a sparse LU solve."""
    import scipy.sparse.linalg as spla
    lin = linearize(prob, poses)
    lu = spla.splu(lin.H.tocsc(), permc_spec="COLAMD")
    out = np.zeros((len(idx), 3, 3))
    n3 = 3 * prob.n
    for q, i in enumerate(idx):
        E = np.zeros((n3, 3))
        E[3 * i:3 * i + 3, :] = np.eye(3)
        X = lu.solve(E)
        blk = X[3 * i:3 * i + 3, :]
        out[q] = 0.5 * (blk + blk.T)
    return out


@dataclass
class LMParams:
    max_iterations: int = 100
    relative_error_tol: float = 1e-5
    absolute_error_tol: float = 1e-5
    error_tol: float = 0.0
    lambda_initial: float = 1e-5
    lambda_factor: float = 10.0
    lambda_upper_bound: float = 1e5
    lambda_lower_bound: float = 0.0
    min_model_fidelity: float = 1e-3
    use_fixed_lambda_factor: bool = True
    max_outer: int = 0          # >0: stop after this many linearisations (truncated fixtures)


@dataclass
class Result:
    poses: np.ndarray           # [N,4] (x, y, c, s)
    error: float
    initial_error: float
    iterations: int
    inner_iterations: int
    trace: list = field(default_factory=list)

    def xyt(self):
        return to_xyt(self.poses)


def check_convergence(p: LMParams, cur, new):
    """NonlinearOptimizer.cpp checkConvergence."""
    if new <= p.error_tol:
        return True
    absd = cur - new
    reld = absd / cur
    return bool((p.relative_error_tol and reld <= p.relative_error_tol) or absd <= p.absolute_error_tol)


def levenberg_marquardt(prob: Problem, poses0, params: LMParams | None = None) -> Result:
    p = params or LMParams()
    poses = np.array(poses0, dtype=np.float64, copy=True)
    err = error(prob, poses)
    lam, factor = p.lambda_initial, p.lambda_factor
    iters = inner = 0
    trace = []
    res = Result(poses, err, err, 0, 0, trace)
    if err <= p.error_tol or iters >= p.max_iterations:
        return res
    new_err = err
    outer = 0
    while True:
        cur_err = new_err
        lin = linearize(prob, poses)
        outer += 1
        while True:                                        # tryLambda loop
            model_fidelity = 0.0
            success = stop = False
            new_e = math.inf
            lin_change = math.nan
            try:
                delta = solve(lin.H, -lin.g, lam)
                solved = True
            except Indeterminant:
                solved = False
            if solved:
                old_lin = linear_error(prob, lin, np.zeros_like(delta))
                new_lin = linear_error(prob, lin, delta)
                lin_change = old_lin - new_lin
                if lin_change >= 0:
                    cand = retract(poses, delta.reshape(-1, 3))
                    new_e = error(prob, cand)
                    cost_change = err - new_e
                    if lin_change > np.finfo(float).eps * old_lin:
                        model_fidelity = cost_change / lin_change
                        success = model_fidelity > p.min_model_fidelity
                    if abs(cost_change) < p.relative_error_tol * err:
                        stop = True
            trace.append(dict(iteration=iters, lam=lam, solved=solved, lin_change=lin_change,
                              new_error=new_e, fidelity=model_fidelity, accepted=success))
            if success:
                if p.use_fixed_lambda_factor:
                    lam /= p.lambda_factor
                else:
                    lam *= max(1.0 / 3.0, 1.0 - (2.0 * model_fidelity - 1.0) ** 3)
                    factor *= 2.0
                lam = max(p.lambda_lower_bound, lam)
                poses, err = cand, new_e
                iters += 1
                inner += 1
                break
            if not stop:
                lam *= factor
                inner += 1
                if not p.use_fixed_lambda_factor:
                    factor *= 2.0
                if lam >= p.lambda_upper_bound:
                    break
                continue
            break
        new_err = err
        if p.max_outer > 0 and outer >= p.max_outer:
            break
        if not (iters < p.max_iterations and not check_convergence(p, cur_err, new_err)
                and math.isfinite(cur_err)):
            break
    return Result(poses, err, res.initial_error, iters, inner, trace)


def gauss_newton(prob: Problem, poses0, params: LMParams | None = None) -> Result:
    """GaussNewtonOptimizer::iterate under NonlinearOptimizer::defaultOptimize."""
    p = params or LMParams()
    poses = np.array(poses0, dtype=np.float64, copy=True)
    err = error(prob, poses)
    err0 = err
    iters = 0
    trace = []
    if err <= p.error_tol:
        return Result(poses, err, err0, 0, 0, trace)
    new_err = err
    while True:
        cur_err = new_err
        lin = linearize(prob, poses)
        delta = solve(lin.H, -lin.g, 0.0)
        poses = retract(poses, delta.reshape(-1, 3))
        err = error(prob, poses)
        iters += 1
        trace.append(dict(iteration=iters, new_error=err))
        new_err = err
        if not (iters < p.max_iterations and not check_convergence(p, cur_err, new_err)
                and math.isfinite(cur_err)):
            break
    return Result(poses, err, err0, iters, iters, trace)


def optimize_graph(g, params: LMParams | None = None, algorithm="lm") -> Result:
    prob = problem_from_graph(g)
    x0 = from_xyt(g.initial)
    if algorithm == "gn":
        return gauss_newton(prob, x0, params)
    return levenberg_marquardt(prob, x0, params)
