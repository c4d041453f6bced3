"""Loop-closure candidate search: the closest_keyframe service (graph.cpp:146-178).

Parity unpinned against the reference itself (it has no tests and cannot be
built here): the C restatement in oracle/pgo_oracle.c is pinned
by an independent numpy evaluation of the same formula (first index among the
smallest sqrt((x2-x1)^2 + (y2-y1)^2)), including ties.  The GPU search
(pgo_closest_keyframe / pgo_closest_keyframes) must return the oracle's index
and the bit-identical distance.
"""
import numpy as np
import pytest

from oracle import oracle

SKIP = 10  # keyframes_to_skip_in_loop_closing, graph.cpp:15


def numpy_closest(xy, q, skip=SKIP):
    n = len(xy) - skip
    if len(xy) == 0 or n <= 0:
        return -1, float("nan")
    d = np.sqrt((xy[:n, 0] - q[0]) ** 2 + (xy[:n, 1] - q[1]) ** 2)
    i = int(np.argmin(d))               # first index of the minimum, like the strict < loop
    return i, float(d[i])


@pytest.fixture(scope="module")
def orc(oracle_lib):
    return oracle_lib


def test_oracle_matches_numpy_random(orc):
    rng = np.random.default_rng(11)
    for n in (11, 12, 100, 5000):
        xy = rng.normal(scale=50, size=(n, 2))
        for _ in range(20):
            q = rng.normal(scale=50, size=2)
            assert orc.closest_keyframe(xy, q[0], q[1], SKIP) == numpy_closest(xy, q)


def test_oracle_ties_and_edges(orc):
    # identical positions: the earliest index wins
    xy = np.zeros((30, 2))
    assert orc.closest_keyframe(xy, 1.0, 1.0, SKIP) == (0, np.sqrt(2.0))
    # integer grid (Manhattan keyframes revisit cells): many exact ties
    g = np.array([[x, y] for _ in range(3) for x in range(5) for y in range(5)], float)
    for q in ([2, 2], [0.5, 0.5], [4, 0], [10, 10]):
        assert orc.closest_keyframe(g, q[0], q[1], SKIP) == numpy_closest(g, q)
    # not enough keyframes: size <= skip
    assert orc.closest_keyframe(np.zeros((10, 2)), 0, 0, SKIP)[0] == -1
    assert orc.closest_keyframe(np.zeros((11, 2)), 0, 0, SKIP)[0] == 0
    assert orc.closest_keyframe(np.zeros((0, 2)), 0, 0, 0)[0] == -1


# ---------------------------------------------------------------- GPU
def _graph_with_values(xy):
    from graphslam_amd.pose_graph import PoseGraph
    pg = PoseGraph(device=0)
    n = len(xy)
    keys = np.arange(1, n + 1, dtype=np.uint64) * 7           # non-dense keys
    pg.add_vertices(keys, np.column_stack([xy, np.zeros(n)]))
    return pg, keys


@pytest.mark.gpu
def test_gpu_closest_keyframe_random():
    rng = np.random.default_rng(5)
    for n in (11, 300, 100_000):
        xy = rng.normal(scale=100, size=(n, 2))
        pg, keys = _graph_with_values(xy)
        for _ in range(10):
            q = rng.normal(scale=100, size=2)
            i, d = oracle.closest_keyframe(xy, q[0], q[1], SKIP)
            k, dg = pg.closest_keyframe(q[0], q[1], SKIP)
            assert k == keys[i] and dg == d
        pg.close()


@pytest.mark.gpu
def test_gpu_closest_keyframe_ties_and_edges():
    from graphslam_amd.pose_graph import NotEnoughKeyframes
    g = np.array([[x, y] for _ in range(40) for x in range(5) for y in range(5)], float)   # 1000 keyframes
    pg, keys = _graph_with_values(g)
    for q in ([2, 2], [0.5, 0.5], [4, 0], [10, 10], [2.0000001, 1.9999999]):
        for skip in (0, 1, SKIP, 990):
            i, d = oracle.closest_keyframe(g, q[0], q[1], skip)
            assert pg.closest_keyframe(q[0], q[1], skip) == (keys[i], d)
    pg.close()
    pg, keys = _graph_with_values(np.zeros((10, 2)))
    with pytest.raises(NotEnoughKeyframes):
        pg.closest_keyframe(0.0, 0.0, SKIP)
    assert pg.closest_keyframe(0.0, 0.0, 9) == (keys[0], 0.0)
    pg.close()


@pytest.mark.gpu
def test_gpu_closest_keyframes_batched_on_optimised_c2():
    """Every keyframe of the optimised C2 graph re-queried as keyframes.back()."""
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    g = datasets.make("C2")
    pg = PoseGraph.from_dataset(g, device=0)
    pg.optimize()
    xy = pg.poses()[:, :2]
    keys = np.asarray(g.keys, dtype=np.uint64)
    rng = np.random.default_rng(3)
    sel = np.concatenate([np.arange(12), rng.choice(len(keys), 400, replace=False)])   # incl. too-early queries
    rng.shuffle(sel)
    got_k, got_d = pg.closest_keyframes(keys[sel], SKIP)
    from graphslam_amd import _lib
    for q, kq, dq in zip(sel, got_k, got_d):
        i, d = oracle.closest_keyframe(xy[: q + 1], xy[q, 0], xy[q, 1], SKIP)
        if i < 0:
            assert kq == _lib.PGO_NO_KEY and dq == np.inf
        else:
            assert kq == keys[i] and dq == d, (q, kq, keys[i], dq, d)
    # the single-query form agrees with the last keyframe's batched answer
    k1, d1 = pg.closest_keyframe(xy[-1, 0], xy[-1, 1], SKIP)
    kb, db = pg.closest_keyframes(keys[-1:], SKIP)
    assert (k1, d1) == (kb[0], db[0])
    pg.close()
