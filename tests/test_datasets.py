"""Synthetic input generator: exact sizes, determinism, layout."""
import numpy as np
import pytest

from graphslam_amd import datasets


@pytest.mark.parametrize("name,n,e", [("C1", 1000, 1019), ("C1-nn", 1000, 1989), ("C2", 10_000, 40_000)])
def test_sizes(name, n, e):
    g = datasets.make(name)
    assert g.num_poses == n and g.num_edges == e
    assert g.edge_cov.shape == (e, 9) and g.edge_z.shape == (e, 3)
    assert g.keys[0] == 1 and np.all(np.diff(g.keys.astype(np.int64)) == 1)   # graph.cpp:31 ids start at 1
    assert g.prior_keys.tolist() == [1]
    assert np.allclose(g.prior_cov[0], np.diag([0.01, 0.01, 0.01]).ravel())   # graph.cpp:13-14,38-45


def test_deterministic():
    a, b = datasets.make("C2"), datasets.make("C2")
    for f in ("initial", "edge_k1", "edge_k2", "edge_z", "edge_cov"):
        assert np.array_equal(getattr(a, f), getattr(b, f))


def test_loop_closure_orientation_and_gap():
    g = datasets.make("C2")
    n = g.num_poses
    lc = slice(n - 1, None)
    k1, k2 = g.edge_k1[lc].astype(np.int64), g.edge_k2[lc].astype(np.int64)
    assert np.all(k1 - k2 > 10)      # (later, earlier), |i-j| > keyframes_to_skip_in_loop_closing
    i, j = g.edge_index()
    same_cell = np.all(np.abs(g.ground_truth[i[lc], :2] - g.ground_truth[j[lc], :2]) < 1e-9)
    assert same_cell


def test_measurements_consistent_with_ground_truth():
    g = datasets.make("C1")
    i, j = g.edge_index()
    exact = datasets.between_xyt(g.ground_truth[i], g.ground_truth[j])
    err = g.edge_z - exact
    err[:, 2] = np.angle(np.exp(1j * err[:, 2]))
    assert np.abs(err[:, :2]).max() < 0.3 and np.abs(err[:, 2]).max() < 0.05
    assert abs(err[:, 0].std() - 0.05) < 0.01


def test_dead_reckoning_is_odometry_composition():
    g = datasets.make("C1")
    x = g.initial
    for k in range(0, 999, 111):
        nxt = datasets.compose_xyt(x[k], g.edge_z[k])
        assert np.allclose(nxt[:2], x[k + 1, :2], atol=1e-9)
        assert abs(np.angle(np.exp(1j * (nxt[2] - x[k + 1, 2])))) < 1e-9


def test_nearest_keyframe_chain_matches_reference_rule():
    g = datasets.make("C1-nn")
    n = g.num_poses
    k1 = g.edge_k1[n - 1:].astype(np.int64) - 1
    k2 = g.edge_k2[n - 1:].astype(np.int64) - 1
    assert k1[0] == 10 and np.all(np.diff(k1) == 1)
    for last, closest in list(zip(k1, k2))[::97]:
        d = np.hypot(*(g.initial[:last - 9, :2] - g.initial[last, :2]).T)
        assert closest == int(np.argmin(d))


def test_kat_builders():
    sq = datasets.square_loop()
    assert sq.num_poses == 20 and sq.num_edges == 20
    i, j = sq.edge_index()
    assert np.allclose(datasets.between_xyt(sq.ground_truth[i], sq.ground_truth[j]), sq.edge_z)
