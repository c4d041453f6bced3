"""Synthetic SE(2) pose graphs for the BASELINE.json configs (C1..C5).

The reference ships no datasets and no tests, so the inputs the
hot path is measured and checked on are generated here, following the recipe
of SURVEY.md §8(d):

* Manhattan random walk on an integer grid of side ``L`` with reflecting walls,
  1 m steps, turn left / right with p = 0.2 each (straight 0.6).
* Measurements ``z_ij = between(gt_i, gt_j) o Pose2(n)``,
  ``n ~ N(0, diag(sigma^2))``, ``sigma = (0.05 m, 0.05 m, 0.00873 rad)``;
  covariance ``diag(sigma^2)`` passed as a row-major ``float64[9]`` exactly like
  ``Pose2DWithCovariance.covariance`` (``src/common/msg/Pose2DWithCovariance.msg:2``).
* Prior on the first key: pose (0, 0, 0), covariance ``diag(0.1^2)*I``
  (``src/graph/src/graph.cpp:13-14,38-45``).  Keys start at 1
  (``graph.cpp:31,207``: ``keyframe_IDs++`` before first use).
* Initial values are the dead-reckoned composition of the odometry
  measurements (what ``new_factor`` intends with ``compose``,
  ``graph.cpp:71``; the reference's buggy ``compose`` (``graph.hpp:30-43``)
  is deliberately not reproduced).
* Odometry factors are oriented (earlier, later) like ``factor_new``
  (``scanner.cpp:123-124``); loop closures are oriented (later, earlier) like
  ``factor_loop`` (``scanner.cpp:150-151``: id_1 = last keyframe,
  id_2 = closest keyframe).

All randomness comes from one ``numpy.random.Generator(PCG64(seed))`` drawn in
a fixed order (walk, odometry noise, loop-closure choice, loop-closure noise),
so every config is bit-reproducible.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

SIGMA = np.array([0.05, 0.05, 0.00873], dtype=np.float64)
PRIOR_SIGMA = np.array([0.1, 0.1, 0.1], dtype=np.float64)   # graph.cpp:13-14
SKIP_RECENT = 10                                              # graph.cpp:15


def wrap(theta):
    """Wrap to (-pi, pi] the way Rot2::theta() = atan2(s, c) reports it."""
    return np.arctan2(np.sin(theta), np.cos(theta))


def between_xyt(a, b):
    """Pose2 a^-1 * b on (x, y, theta) arrays of shape (..., 3)."""
    ca, sa = np.cos(a[..., 2]), np.sin(a[..., 2])
    dx, dy = b[..., 0] - a[..., 0], b[..., 1] - a[..., 1]
    out = np.empty(np.broadcast(a, b).shape, dtype=np.float64)
    out[..., 0] = ca * dx + sa * dy
    out[..., 1] = -sa * dx + ca * dy
    out[..., 2] = wrap(b[..., 2] - a[..., 2])
    return out


def compose_xyt(a, b):
    """Pose2 a * b on (x, y, theta) arrays."""
    ca, sa = np.cos(a[..., 2]), np.sin(a[..., 2])
    out = np.empty(np.broadcast(a, b).shape, dtype=np.float64)
    out[..., 0] = a[..., 0] + ca * b[..., 0] - sa * b[..., 1]
    out[..., 1] = a[..., 1] + sa * b[..., 0] + ca * b[..., 1]
    out[..., 2] = wrap(a[..., 2] + b[..., 2])
    return out


@dataclass
class PoseGraph:
    """A pose graph in the C-ABI's input layout (keys + row-major covariances)."""

    name: str
    keys: np.ndarray            # uint64 [N]    key of pose index p
    initial: np.ndarray         # f64 [N,3]     (x, y, theta) initial values
    ground_truth: np.ndarray    # f64 [N,3]
    edge_k1: np.ndarray         # uint64 [E]
    edge_k2: np.ndarray         # uint64 [E]
    edge_z: np.ndarray          # f64 [E,3]     measured Pose2 (x, y, theta)
    edge_cov: np.ndarray        # f64 [E,9]     row-major covariance
    prior_keys: np.ndarray      # uint64 [P]
    prior_pose: np.ndarray      # f64 [P,3]
    prior_cov: np.ndarray       # f64 [P,9]
    meta: dict = field(default_factory=dict)

    @property
    def num_poses(self) -> int:
        return int(self.keys.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.edge_k1.shape[0])

    def edge_index(self):
        """Dense pose indices (i, j) of every between factor (keys are p + 1 here)."""
        lut = {int(k): p for p, k in enumerate(self.keys)}
        if np.array_equal(self.keys, np.arange(1, self.num_poses + 1, dtype=np.uint64)):
            return (self.edge_k1.astype(np.int64) - 1, self.edge_k2.astype(np.int64) - 1)
        return (np.array([lut[int(k)] for k in self.edge_k1]),
                np.array([lut[int(k)] for k in self.edge_k2]))

    def prior_index(self):
        lut = {int(k): p for p, k in enumerate(self.keys)}
        return np.array([lut[int(k)] for k in self.prior_keys], dtype=np.int64)


def _diag_cov(sigma, n):
    cov = np.zeros((n, 9), dtype=np.float64)
    cov[:, 0] = sigma[0] ** 2
    cov[:, 4] = sigma[1] ** 2
    cov[:, 8] = sigma[2] ** 2
    return cov


def manhattan_walk(n, side, rng):
    """Ground-truth poses of a Manhattan walk; returns (gt [n,3], cell [n] int64)."""
    u = rng.random(max(n - 1, 0))
    steps = ((1, 0), (0, 1), (-1, 0), (0, -1))
    lo = -(side // 2)
    hi = side - side // 2 - 1
    x = y = 0
    h = 0
    xs = np.empty(n, dtype=np.int64)
    ys = np.empty(n, dtype=np.int64)
    hs = np.empty(n, dtype=np.int64)
    xs[0], ys[0], hs[0] = 0, 0, 0
    for k in range(n - 1):
        r = u[k]
        if r < 0.2:
            h = (h + 1) & 3
        elif r < 0.4:
            h = (h + 3) & 3
        dx, dy = steps[h]
        if not (lo <= x + dx <= hi and lo <= y + dy <= hi):
            h = (h + 2) & 3          # reflecting wall: turn around
            dx, dy = steps[h]
        x += dx
        y += dy
        xs[k + 1], ys[k + 1], hs[k + 1] = x, y, h
    gt = np.empty((n, 3), dtype=np.float64)
    gt[:, 0] = xs
    gt[:, 1] = ys
    gt[:, 2] = wrap(hs * (np.pi / 2))
    cell = (xs - lo) * side + (ys - lo)
    return gt, cell


def _noisy_between(gt, i, j, rng):
    exact = between_xyt(gt[i], gt[j])
    noise = rng.standard_normal((len(i), 3)) * SIGMA
    return compose_xyt(exact, noise)


def _dead_reckon(z_odo, n):
    """init_0 = (0,0,0); init_{k+1} = init_k o z_k (vectorised cumulative compose)."""
    init = np.zeros((n, 3), dtype=np.float64)
    if n == 1:
        return init
    th = np.concatenate([[0.0], np.cumsum(z_odo[:, 2])])
    c, s = np.cos(th[:-1]), np.sin(th[:-1])
    dx = c * z_odo[:, 0] - s * z_odo[:, 1]
    dy = s * z_odo[:, 0] + c * z_odo[:, 1]
    init[1:, 0] = np.cumsum(dx)
    init[1:, 1] = np.cumsum(dy)
    init[:, 2] = wrap(th)
    return init


def _same_cell_pairs(cell, min_gap):
    """All (later, earlier) index pairs in the same grid cell with later-earlier > min_gap."""
    order = np.argsort(cell, kind="stable")      # within a cell: increasing index
    sc = cell[order]
    out_a, out_b = [], []
    d = 1
    n = len(order)
    while d < n:
        same = sc[d:] == sc[:-d]
        if not same.any():
            break
        a = order[d:][same]          # later
        b = order[:-d][same]         # earlier
        keep = (a - b) > min_gap
        out_a.append(a[keep])
        out_b.append(b[keep])
        d += 1
    if not out_a:
        return np.empty(0, np.int64), np.empty(0, np.int64)
    a = np.concatenate(out_a)
    b = np.concatenate(out_b)
    key = np.lexsort((b, a))
    return a[key], b[key]


def _assemble(name, seed, gt, init, i, j, z, meta):
    n = gt.shape[0]
    keys = np.arange(1, n + 1, dtype=np.uint64)
    return PoseGraph(
        name=name,
        keys=keys,
        initial=init,
        ground_truth=gt,
        edge_k1=(i + 1).astype(np.uint64),
        edge_k2=(j + 1).astype(np.uint64),
        edge_z=z,
        edge_cov=_diag_cov(SIGMA, len(i)),
        prior_keys=np.array([1], dtype=np.uint64),
        prior_pose=np.zeros((1, 3), dtype=np.float64),
        prior_cov=_diag_cov(PRIOR_SIGMA, 1),
        meta=dict(meta, seed=seed),
    )


def manhattan(n, side, num_edges, seed, name="manhattan", window=1, loop_closures=None):
    """Odometry chain (+ window edges i->i-k, 2 <= k <= window) + same-cell loop
    closures, exactly ``num_edges`` between factors: with ``loop_closures``
    None every window edge is kept and the loop closures fill up to
    ``num_edges``; otherwise that many loop closures are drawn and the window
    edges are seeded-subsampled to fill up."""
    rng = np.random.Generator(np.random.PCG64(seed))
    gt, cell = manhattan_walk(n, side, rng)
    oi = np.arange(n - 1, dtype=np.int64)
    oj = oi + 1
    z_odo = _noisy_between(gt, oi, oj, rng)
    init = _dead_reckon(z_odo, n)
    ei, ej, ez = [oi], [oj], [z_odo]
    if window > 1:
        wi = np.concatenate([np.arange(n - k, dtype=np.int64) for k in range(2, window + 1)])
        wj = wi + np.concatenate([np.full(n - k, k, dtype=np.int64) for k in range(2, window + 1)])
        if loop_closures is not None:
            keep = num_edges - (n - 1) - loop_closures
            if not 0 <= keep <= len(wi):
                raise ValueError(f"{name}: cannot fill {num_edges} edges with window {window}")
            pick = np.sort(rng.choice(len(wi), size=keep, replace=False))
            wi, wj = wi[pick], wj[pick]
        ei.append(wi)
        ej.append(wj)
        ez.append(_noisy_between(gt, wi, wj, rng))
    have = sum(len(a) for a in ei)
    need = num_edges - have
    if need < 0:
        raise ValueError(f"{name}: chain/window edges {have} exceed num_edges {num_edges}")
    la, lb = _same_cell_pairs(cell, SKIP_RECENT)
    if need > len(la):
        raise ValueError(f"{name}: only {len(la)} loop-closure candidates for {need}")
    pick = np.sort(rng.choice(len(la), size=need, replace=False)) if need else np.empty(0, np.int64)
    li, lj = la[pick], lb[pick]               # (later, earlier) like factor_loop
    ei.append(li)
    ej.append(lj)
    ez.append(_noisy_between(gt, li, lj, rng))
    meta = dict(side=side, window=window, loop_closures=int(need), lc_candidates=int(len(la)))
    return _assemble(name, seed, gt, init, np.concatenate(ei), np.concatenate(ej),
                     np.concatenate(ez), meta)


def nearest_keyframe_chain(n, side, seed, name="C1-nn"):
    """The reference's live behaviour: odometry chain plus one loop factor per
    keyframe to the closest keyframe among all but the last 10, by the current
    (initial) estimate -- ``graph.cpp:146-178`` (strict ``<`` argmin: first index
    wins ties), oriented (last, closest) as ``scanner.cpp:150-151``."""
    rng = np.random.Generator(np.random.PCG64(seed))
    gt, _ = manhattan_walk(n, side, rng)
    oi = np.arange(n - 1, dtype=np.int64)
    oj = oi + 1
    z_odo = _noisy_between(gt, oi, oj, rng)
    init = _dead_reckon(z_odo, n)
    li, lj = [], []
    for last in range(SKIP_RECENT, n):
        cand = last + 1 - SKIP_RECENT
        d = np.hypot(init[:cand, 0] - init[last, 0], init[:cand, 1] - init[last, 1])
        li.append(last)
        lj.append(int(np.argmin(d)))
    li = np.asarray(li, dtype=np.int64)
    lj = np.asarray(lj, dtype=np.int64)
    z_lc = _noisy_between(gt, li, lj, rng)
    return _assemble(name, seed, gt, init, np.concatenate([oi, li]), np.concatenate([oj, lj]),
                     np.concatenate([z_odo, z_lc]), dict(side=side, loop_closures=len(li)))


CONFIGS = {
    # name: (builder, kwargs)  -- BASELINE.json "configs" / SURVEY.md §8(d)
    "C1": dict(n=1000, side=16, num_edges=1019, seed=1001),
    "C2": dict(n=10_000, side=32, num_edges=40_000, seed=1002),
    "C3": dict(n=100_000, side=100, num_edges=500_000, seed=1003),
    # 1M poses / 5M edges, 5 % loop-closure density: 50k same-cell loop closures
    # (5 % of the poses), odometry, and window edges i->i-k (k = 2..5) subsampled
    # to 5M in total (BASELINE.json configs[4]; DESIGN.md "Configs")
    "C5": dict(n=1_000_000, side=316, num_edges=5_000_000, seed=1005, window=5, loop_closures=50_000),
}


def make(name: str) -> PoseGraph:
    """Build a named config: C1, C1-nn, C2, C3 (headline), C5."""
    if name == "C1-nn":
        return nearest_keyframe_chain(1000, 16, 1001)
    if name not in CONFIGS:
        raise KeyError(f"unknown config {name!r}; have {sorted(CONFIGS) + ['C1-nn']}")
    return manhattan(name=name, **CONFIGS[name])


def noise_free(gt, pairs, prior_index=0, name="kat"):
    """Known-answer graph: exact measurements between ground-truth poses.

    ``pairs`` is a list of (i, j); the initial values are ground truth perturbed
    deterministically so the optimiser has work to do.  The optimum is the ground
    truth exactly (chi^2 = 0)."""
    gt = np.asarray(gt, dtype=np.float64)
    n = gt.shape[0]
    i = np.array([p[0] for p in pairs], dtype=np.int64)
    j = np.array([p[1] for p in pairs], dtype=np.int64)
    z = between_xyt(gt[i], gt[j])
    k = np.arange(n)
    init = gt.copy()
    init[:, 0] += 0.05 * np.sin(1.3 * k + 0.1)
    init[:, 1] += 0.05 * np.cos(0.7 * k + 0.2)
    init[:, 2] = wrap(init[:, 2] + 0.02 * np.sin(2.1 * k))
    init[prior_index] = gt[prior_index]
    g = _assemble(name, 0, gt, init, i, j, z, {})
    g.prior_keys = np.array([prior_index + 1], dtype=np.uint64)
    g.prior_pose = gt[prior_index:prior_index + 1].copy()
    return g


def square_loop(side_poses=5, step=1.0):
    """Noise-free closed square loop: 4*side_poses poses, odometry + one closure."""
    pts = []
    x = y = 0.0
    th = 0.0
    for leg in range(4):
        for _ in range(side_poses):
            pts.append((x, y, th))
            x += step * np.cos(th)
            y += step * np.sin(th)
        th = float(wrap(th + np.pi / 2))
    gt = np.array(pts)
    n = gt.shape[0]
    pairs = [(k, k + 1) for k in range(n - 1)] + [(n - 1, 0)]
    return noise_free(gt, pairs, name="square")


def straight_chain(n=10, step=1.0):
    gt = np.zeros((n, 3))
    gt[:, 0] = step * np.arange(n)
    return noise_free(gt, [(k, k + 1) for k in range(n - 1)], name="chain")


# ---------------------------------------------------------------- laser scans (scan registration, 8f row 4)
def laser_world(seed=7, width=20.0, height=12.0, boxes=6):
    """A rectangular room with `boxes` axis-aligned boxes: (m, 4) wall segments
    (x0, y0, x1, y1) -- the kind of world the reference's Stage simulation scans."""
    rng = np.random.Generator(np.random.PCG64(seed))
    seg = [(0, 0, width, 0), (width, 0, width, height), (width, height, 0, height), (0, height, 0, 0)]
    rects = []
    for _ in range(boxes):
        w, h = rng.uniform(0.5, 2.0, size=2)
        x, y = rng.uniform(1.0, width - 3.0), rng.uniform(1.0, height - 3.0)
        rects.append((x, y, x + w, y + h))
        seg += [(x, y, x + w, y), (x + w, y, x + w, y + h), (x + w, y + h, x, y + h), (x, y + h, x, y)]
    return np.array(seg, dtype=np.float64), np.array(rects, dtype=np.float64)


def simulate_scan(segments, pose, n_beams=360, range_max=10.0, noise=0.01, rng=None):
    """sensor_msgs/LaserScan ranges of a 360-degree laser at pose (x, y, theta):
    beam i at angle_min + i * angle_increment (angle_min = -pi), the nearest wall
    hit (+ N(0, noise^2)), range_max + 1 where nothing is hit within range_max."""
    x, y, th = pose
    inc = 2 * np.pi / n_beams
    a = -np.pi + np.arange(n_beams) * inc
    d = np.stack([np.cos(th + a), np.sin(th + a)], axis=1)                  # (n, 2)
    p0, e = segments[:, :2], segments[:, 2:] - segments[:, :2]              # (m, 2)
    ap = p0 - np.array([x, y])
    den = d[:, None, 0] * e[None, :, 1] - d[:, None, 1] * e[None, :, 0]     # cross(d, e)
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (ap[None, :, 0] * e[None, :, 1] - ap[None, :, 1] * e[None, :, 0]) / den
        u = (ap[None, :, 0] * d[:, None, 1] - ap[None, :, 1] * d[:, None, 0]) / den
    ok = (np.abs(den) > 1e-12) & (t > 1e-9) & (u >= 0) & (u <= 1)
    r = np.where(ok, t, np.inf).min(axis=1)
    if rng is not None and noise > 0:
        r = r + rng.normal(0.0, noise, size=r.shape)
    r = np.where(r < range_max, r, range_max + 1.0)
    return r.astype(np.float32), -np.pi, inc, 0.05, range_max


def _xyt_to_T(p):
    c, s = np.cos(p[2]), np.sin(p[2])
    T = np.eye(4)
    T[:2, :2] = [[c, -s], [s, c]]
    T[:2, 3] = p[:2]
    return T


def scan_pairs(count, seed=11, n_beams=360, motion=(0.3, 0.1, 0.05), noise=0.01, range_max=10.0):
    """`count` registration pairs in one world: (source cloud = scan at pose B,
    target cloud = scan at pose A, true T = A^-1 B) with B = A o motion (each
    component scaled by U(0.5, 1.5) and a random sign), the scanner's
    gicp(current, keyframe) shape (scanner.cpp:115)."""
    from .scanner import scan_to_pointcloud
    segs, rects = laser_world(seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))

    def free(p):
        return not np.any((p[0] > rects[:, 0] - 0.3) & (p[0] < rects[:, 2] + 0.3) &
                          (p[1] > rects[:, 1] - 0.3) & (p[1] < rects[:, 3] + 0.3))
    out = []
    while len(out) < count:
        A = np.array([rng.uniform(1.5, 18.5), rng.uniform(1.5, 10.5), rng.uniform(-np.pi, np.pi)])
        m = np.array(motion) * rng.uniform(0.5, 1.5, size=3) * rng.choice([-1.0, 1.0], size=3)
        TB = _xyt_to_T(A) @ _xyt_to_T(m)
        B = np.array([TB[0, 3], TB[1, 3], np.arctan2(TB[1, 0], TB[0, 0])])
        if not (free(A) and free(B)):
            continue
        ca = scan_to_pointcloud(*simulate_scan(segs, A, n_beams, range_max, noise, rng))
        cb = scan_to_pointcloud(*simulate_scan(segs, B, n_beams, range_max, noise, rng))
        if len(ca) < 30 or len(cb) < 30:
            continue
        out.append((cb, ca, _xyt_to_T(m)))
    return out
