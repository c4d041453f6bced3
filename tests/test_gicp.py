"""Scan registration: the scanner node's GICP (scanner.cpp:35-74).

PARITY UNPINNED against PCL: GeneralizedIterativeClosestPoint is a third-party
dependency absent from /root/reference (ROS-era PCL, version not pinned), and
the reference holds no registration fixtures.  The C restatement
(oracle/gicp_oracle.c) is pinned by known answers instead: exact-correspondence
clouds must give back the applied motion to 1e-6, simulated laser scans of a
room the motion to a few cm (the point-to-point accuracy GICP has on planar
scans, where the plane model makes the in-plane covariance isotropic), and the
plane-regularised covariances must have eigenvalues (eps, 1, 1).  The GPU path
(pgo_gicp_align_batch) is compared with the restatement on the same clouds:
transforms within 1e-6, the same iteration counts, fitness within 1e-6
relative, and make_Delta / compute_covariance / keyframe flag (scanner.hpp:55-80,
scanner.cpp:55-58) as the host restatement forms them.
"""
import ctypes as C

import numpy as np
import pytest

from graphslam_amd.datasets import scan_pairs, simulate_scan, laser_world


def _rot(axis, a):
    c, s = np.cos(a), np.sin(a)
    R = np.eye(3)
    i, j = [(1, 2), (0, 2), (0, 1)][axis]
    R[i, i], R[i, j], R[j, i], R[j, j] = c, -s, s, c
    return R


def _exact_pair(src, R, t):
    tgt = (src.astype(np.float64) @ R.T + t).astype(np.float32)
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return tgt, T


@pytest.fixture(scope="module")
def pairs():
    return scan_pairs(16, seed=11)


# ---------------------------------------------------------------- oracle (CPU)
def test_oracle_exact_known_motion(oracle_lib, pairs):
    for b, (src, _, _) in enumerate(pairs[:6]):
        R = _rot(2, 0.03 * (b - 2))
        t = np.array([0.2 - 0.05 * b, 0.1 * (b % 3), 0.0])
        tgt, Tt = _exact_pair(src, R, t)
        T, it, conv, fit = oracle_lib.gicp_align(src, tgt)
        assert conv and it < 200
        assert np.abs(T - Tt).max() < 1e-6
        assert fit < 1e-10


def test_oracle_simulated_scans_recover_motion(oracle_lib, pairs):
    ex, eth = [], []
    for src, tgt, Tt in pairs:
        T, it, conv, fit = oracle_lib.gicp_align(src, tgt)
        d, dt = oracle_lib.make_delta(T), oracle_lib.make_delta(Tt)
        ex.append(np.hypot(d[0] - dt[0], d[1] - dt[1]))
        eth.append(abs(d[2] - dt[2]))
        assert abs(T[2, 3]) < 1e-6 and abs(T[2, 2] - 1) < 1e-9   # planar scans stay planar
    assert np.median(ex) < 0.03 and np.median(eth) < 0.01
    assert np.mean(np.array(ex) < 0.05) >= 0.75


def test_oracle_covariances_plane_model(oracle_lib, pairs):
    src = pairs[0][0]
    Cv = oracle_lib.gicp_covariances(src, k=20, eps=1e-3)
    assert np.allclose(Cv, np.transpose(Cv, (0, 2, 1)))
    w = np.linalg.eigvalsh(Cv)
    assert np.allclose(w, [1e-3, 1.0, 1.0], atol=1e-9)
    # planar cloud: the eps direction is z
    assert np.allclose(Cv[:, 2, 2], 1e-3, atol=1e-9)
    # k larger than the cloud: all points are neighbours
    Cs = oracle_lib.gicp_covariances(src[:5], k=20, eps=1e-3)
    assert np.allclose(np.linalg.eigvalsh(Cs), [1e-3, 1.0, 1.0], atol=1e-9)


def test_make_delta_and_covariance():
    from oracle.oracle import compute_covariance, make_delta
    T = np.eye(4)
    a = -0.3
    T[:2, :2] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
    T[:2, 3] = [0.3, -0.4]
    d = make_delta(T)
    assert np.allclose(d, [0.3, -0.4, a], atol=1e-6)
    Q = compute_covariance(0.1, 0.1, 0.1, d)
    assert np.isclose(Q[0, 0], 0.05, atol=1e-7) and Q[0, 0] == Q[1, 1]
    assert np.isclose(Q[2, 2], 0.05 + 0.1 * d[2])   # negative theta lowers it (reference formula)
    # atan, not atan2: a half-turn reads as ~0
    T[:2, :2] = [[-1, 0], [0, -1]]
    assert abs(make_delta(T)[2]) < 1e-12


def test_scan_to_pointcloud_range_filter():
    from graphslam_amd.scanner import scan_to_pointcloud
    r = np.array([1.0, 0.01, 2.0, 11.0, 10.0], np.float32)
    pc = scan_to_pointcloud(r, 0.0, np.pi / 2, 0.05, 10.0)
    assert pc.dtype == np.float32 and pc.shape == (2, 3)
    assert np.allclose(pc, [[1, 0, 0], [-2, 0, 0]], atol=1e-6)
    segs, _ = laser_world(7)
    ranges, amin, inc, rmin, rmax = simulate_scan(segs, (10.0, 6.0, 0.0), 360, 30.0, 0.0)
    assert np.all(ranges < rmax) and ranges.min() > 0   # a closed room: every beam hits


def test_abi_rejects_bad_arguments(pgo_lib):
    from graphslam_amd import _lib as L
    h = pgo_lib.pgo_gicp_create(0)
    try:
        p = L.PgoGicpParams()
        pgo_lib.pgo_gicp_default_params(C.byref(p))
        assert (p.max_iterations, p.k_correspondences, p.max_correspondence_distance) == (200, 20, 5.0)
        res = (L.PgoGicpResult * 1)()
        fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int)
        pts = np.zeros((5000, 3), np.float32)
        n_ok, n_big = np.array([10], np.int32), np.array([5000], np.int32)
        rc = pgo_lib.pgo_gicp_align_batch(h, 1, pts.ctypes.data_as(fp), n_big.ctypes.data_as(ip),
                                          pts.ctypes.data_as(fp), n_ok.ctypes.data_as(ip), None, C.byref(p), res)
        assert rc == L.PGO_E_ARG and b"4096" in pgo_lib.pgo_gicp_last_error(h)
        p.k_correspondences = 33
        rc = pgo_lib.pgo_gicp_align_batch(h, 1, pts.ctypes.data_as(fp), n_ok.ctypes.data_as(ip),
                                          pts.ctypes.data_as(fp), n_ok.ctypes.data_as(ip), None, C.byref(p), res)
        assert rc == L.PGO_E_ARG
        assert pgo_lib.pgo_gicp_align_batch(h, 0, None, None, None, None, None, None, res) == L.PGO_OK
        assert pgo_lib.pgo_gicp_align_batch(None, 1, None, None, None, None, None, None, res) == L.PGO_E_ARG
    finally:
        pgo_lib.pgo_gicp_destroy(h)


# ---------------------------------------------------------------- GPU
def _check_against_oracle(r, src, tgt, oracle_lib, guess=None):
    T, it, conv, fit = oracle_lib.gicp_align(src, tgt, guess)
    assert r.iterations == it and r.inner_iterations == oracle_lib.gicp_align.last_inner
    assert r.converged == conv
    assert np.abs(r.transform - T).max() < 1e-6, np.abs(r.transform - T).max()
    assert abs(r.fitness - fit) <= 1e-6 * max(fit, 1e-9) + 1e-12
    d = oracle_lib.make_delta(r.transform)
    assert np.allclose(r.delta, d, atol=1e-12, rtol=0)
    assert np.allclose(r.covariance, oracle_lib.compute_covariance(0.1, 0.1, 0.1, d), atol=1e-12)
    assert r.keyframe_flag == (r.converged and r.fitness > 0.1)


@pytest.mark.gpu
def test_gpu_matches_oracle_batch(oracle_lib, pairs):
    from graphslam_amd.scanner import ScanRegistrar
    reg = ScanRegistrar(0)
    out = reg.align_batch([s for s, _, _ in pairs], [t for _, t, _ in pairs])
    assert len(out) == len(pairs)
    for r, (src, tgt, _) in zip(out, pairs):
        _check_against_oracle(r, src, tgt, oracle_lib)
    assert any(r.keyframe_flag for r in out) and not all(r.keyframe_flag for r in out)
    arr = reg.align_batch([s for s, _, _ in pairs], [t for _, t, _ in pairs], arrays=True)
    assert np.array_equal(arr["T"], np.stack([r.transform for r in out]))
    assert np.array_equal(arr["fitness"], [r.fitness for r in out])
    assert np.array_equal(arr["keyframe"].astype(bool), [r.keyframe_flag for r in out])
    assert np.array_equal(arr["cov"], np.stack([r.covariance for r in out]))


@pytest.mark.gpu
def test_gpu_exact_known_motion_and_guess(oracle_lib, pairs):
    from graphslam_amd.scanner import ScanRegistrar
    reg = ScanRegistrar(0)
    src = pairs[3][0]
    tgt, Tt = _exact_pair(src, _rot(2, 0.08) @ _rot(0, 0.01), np.array([0.25, -0.15, 0.02]))
    r = reg.align_batch([src], [tgt])[0]
    assert np.abs(r.transform - Tt).max() < 1e-6 and r.fitness < 1e-10
    # an initial guess (align(output, guess))
    G = np.eye(4)
    G[:3, 3] = [0.2, -0.1, 0.0]
    r2 = reg.align_batch([src], [tgt], guesses=[G])[0]
    assert np.abs(r2.transform - Tt).max() < 1e-6
    _check_against_oracle(r2, src, tgt, oracle_lib, G)


@pytest.mark.gpu
def test_gpu_batch_independent_of_batch(pairs):
    """A pair's result does not depend on what else is in the launch (bitwise)."""
    from graphslam_amd.scanner import ScanRegistrar
    reg = ScanRegistrar(0)
    S, T = [s for s, _, _ in pairs], [t for _, t, _ in pairs]
    full = reg.align_batch(S, T)
    for b in (0, 5, 15):
        one = reg.align_batch([S[b]], [T[b]])[0]
        assert np.array_equal(one.transform, full[b].transform) and one.fitness == full[b].fitness
    rev = reg.align_batch(S[::-1], T[::-1])
    for a, b in zip(rev[::-1], full):
        assert np.array_equal(a.transform, b.transform)


@pytest.mark.gpu
def test_gpu_edge_sizes(oracle_lib, pairs):
    from graphslam_amd.scanner import ScanRegistrar
    reg = ScanRegistrar(0)
    rng = np.random.default_rng(3)
    big_src = rng.uniform(-20, 20, size=(4096, 3)).astype(np.float32)
    big_src[:, 2] *= 0.05
    big_tgt, Tt = _exact_pair(big_src, _rot(2, 0.02), np.array([0.1, 0.05, 0.0]))
    one = np.array([[1.0, 2.0, 0.0]], np.float32)
    S = [big_src, one, pairs[0][0][:7], pairs[1][0]]
    T = [big_tgt, one + 0.5, pairs[0][1][:9], pairs[1][1]]
    out = reg.align_batch(S, T)
    assert np.abs(out[0].transform - Tt).max() < 1e-6
    for r, s, t in zip(out, S, T):
        _check_against_oracle(r, s, t, oracle_lib)
    # a single point: fewer than 3 correspondences, the guess stays
    assert np.array_equal(out[1].transform, np.eye(4)) and out[1].iterations == 1


@pytest.mark.gpu
def test_gpu_pcl_mirror_and_gicp(pairs):
    from graphslam_amd.scanner import GeneralizedIterativeClosestPoint, gicp, gicp_batch
    src, tgt, _ = pairs[2]
    g = GeneralizedIterativeClosestPoint()
    g.setInputSource(src)
    g.setInputTarget(tgt)
    moved = g.align()
    T = g.getFinalTransformation()
    assert T.dtype == np.float32 and g.hasConverged()
    assert np.allclose(moved, src @ T[:3, :3].T.astype(np.float64) + T[:3, 3], atol=1e-4)
    r = gicp(src, tgt)
    assert np.allclose(r.transform, T, atol=1e-6) and r.fitness == g.getFitnessScore()
    rb = gicp_batch([(src, tgt), (tgt, src)])
    assert np.array_equal(rb[0].transform, r.transform)
    # max iterations 1: stops after one correspondence round, still "converged" (PCL)
    g.setMaximumIterations(1)
    g.align()
    assert g.hasConverged()


@pytest.mark.gpu
def test_gpu_ties_params_and_errors(oracle_lib, pairs):
    """Duplicate points (exact distance ties: lowest index on both sides),
    non-default parameters, a far initial guess, and non-finite input."""
    from graphslam_amd import _lib as L
    from graphslam_amd.pose_graph import PgoError
    from graphslam_amd.scanner import ScanRegistrar, default_params
    reg = ScanRegistrar(0)
    src, tgt, _ = pairs[4]
    tgt_dup = np.concatenate([tgt, tgt[::3]])            # every 3rd target point twice
    src_dup = np.concatenate([src[:50], src[:50], src])  # duplicated source points
    r = reg.align_batch([src_dup], [tgt_dup])[0]
    _check_against_oracle(r, src_dup, tgt_dup, oracle_lib)
    # non-default parameters reach the kernels
    p = default_params(max_iterations=3, k_correspondences=10, max_correspondence_distance=1.0)
    r3 = reg.align_batch([src], [tgt], params=p)[0]
    T, it, conv, fit = oracle_lib.gicp_align(src, tgt, None, k=10, max_it=3, max_dist=1.0)
    assert r3.iterations == it <= 3 and np.abs(r3.transform - T).max() < 1e-6
    # a far guess (a quarter turn): whatever the local minimum, the same as the restatement
    G = np.eye(4)
    G[:2, :2] = [[0, -1], [1, 0]]
    r4 = reg.align_batch([src], [tgt], guesses=[G])[0]
    _check_against_oracle(r4, src, tgt, oracle_lib, G)
    bad = src.copy()
    bad[7, 1] = np.nan
    with pytest.raises(PgoError) as e:
        reg.align_batch([bad], [tgt])
    assert e.value.status == L.PGO_E_NONFINITE
