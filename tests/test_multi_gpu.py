"""Multi-rank speculative lambda search (include/pgo.h "multi-GPU").

CPU (gloo, world size 2): the host transport's all-gather / broadcast through
the C-ABI (pgo_comm_selftest needs no GPU with host callbacks).

GPU: two and three ranks sharing cuda:0 (RCCL refuses two ranks on one
device, so these ranks exchange through the host transport over gloo; the
library's round logic is the same for both transports) must reproduce the
one-rank run bitwise -- same accepted steps, same lambda tries, same final
values -- while solving the tries of a round in parallel.  A one-rank RCCL
communicator checks the RCCL transport's calls on the box.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

from graphslam_amd import _lib  # noqa: E402 (constants only; the library loads lazily)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _selftest_worker(rank, world, port, q):
    try:
        dist = _init(rank, world, port)
        from graphslam_amd import multi_gpu
        from graphslam_amd.pose_graph import PoseGraph
        pg = PoseGraph(device=0)
        hc = multi_gpu.attach_host(pg, dist, rank, world)
        pg.comm_selftest()
        q.put((rank, pg.comm_rank(), None))
        del hc
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def _run(world, target, args, timeout=300):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(k, world, port, q) + args) for k in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=timeout) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


def _hybrid_selftest_worker(rank, world, port, q, groups):
    try:
        dist = _init(rank, world, port)
        from graphslam_amd import multi_gpu
        from graphslam_amd.pose_graph import PoseGraph
        pg = PoseGraph(device=0)
        keep = multi_gpu.attach_hybrid(pg, dist, rank, world, groups, transport="host")
        pg.comm_selftest()
        q.put((rank, (pg.comm_rank(), pg.comm_part_rank()), None))
        del keep
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world,groups", [(4, 2), (6, 3), (4, 1), (4, 4)])
def test_hybrid_layout_gloo(world, groups):
    """PGO_MULTI_HYBRID's two communicators over gloo sub-groups (CPU, host
    transport): rank r sits at position r % (world / groups) of group
    r // (world / groups); the speculative communicator links one rank of every
    group and passes the exchange self test (all-gather + broadcast from its
    last rank, whose global rank differs from its group rank)."""
    out = _run(world, _hybrid_selftest_worker, (groups,))
    pp = world // groups
    for rank, rs, err in out:
        assert err is None, err
        assert rs == ((rank // pp, groups), (rank % pp, pp))


def test_host_comm_selftest_gloo_world2():
    out = _run(2, _selftest_worker, ())
    for rank, rs, err in out:
        assert err is None, err
        assert rs == (rank, 2)


def _partition_worker(rank, world, port, q, case):
    try:
        dist = _init(rank, world, port)
        import torch as _t
        from graphslam_amd import datasets
        from graphslam_amd.pose_graph import PoseGraph
        pg = PoseGraph.from_dataset(datasets.make(case))
        owner, rf, top = pg.debug_partition(world)
        mine = _t.from_numpy(owner.astype(np.int64))
        outs = [_t.empty_like(mine) for _ in range(world)]
        dist.all_gather(outs, mine)
        q.put((rank, [o.numpy() for o in outs], rf, top, None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))


@pytest.mark.parametrize("case", ["C1-nn", "C2"])
def test_partition_plan_gloo_world2(case):
    """PGO_MULTI_PARTITION's plan logic on CPU, two gloo ranks: both compute
    the identical subtree partition of the elimination tree (every rank plans
    for itself), every supernode is owned by exactly one rank or the
    replicated top, the top is closed under parents, each rank's subtrees are
    postorder ranges, and both ranks get work."""
    out = _run(2, _partition_worker, (case,))
    for rank, owners, rf, top, err in out:
        assert err is None, err
        assert np.array_equal(owners[0], owners[1])
    owner = out[0][1][0]
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    pg = PoseGraph.from_dataset(datasets.make(case))
    w, m, lv = pg.debug_fronts()
    assert len(owner) == len(w)
    assert set(np.unique(owner)) <= {-1, 0, 1} and (owner == 0).any() and (owner == 1).any()
    rf = out[0][2]
    assert rf.min() > 0.25 * rf.max()                      # balanced within the LPT bound


def test_partition_structure_sizes():
    """Partition invariants for 2/4/8 ranks on C2 (host only): a front's rank
    is its parent's unless the parent is top (subtrees are closed), the top is
    closed under parents (an ancestor of a top front is top)."""
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    g = datasets.make("C2")
    pg = PoseGraph.from_dataset(g)
    parent = _plan_parents(pg)
    for size in (2, 4, 8):
        owner, rf, top = pg.debug_partition(size)
        for s, p in enumerate(parent):
            if p < 0:
                continue
            if owner[p] >= 0:
                assert owner[s] == owner[p]
            if owner[s] < 0:
                assert owner[p] < 0
        assert top > 0 and len(rf) == size and (rf > 0).sum() >= min(size, 2)


def _plan_parents(pg):
    import ctypes as C
    from graphslam_amd import _lib
    L = _lib.lib()
    ns = L.pgo_debug_fronts(pg._h, None, None, None, 0)
    par = np.zeros(ns, np.int32)
    rc = L.pgo_debug_parents(pg._h, par.ctypes.data_as(C.POINTER(C.c_int)), ns)
    assert rc == ns
    return par


# ---------------------------------------------------------------- GPU
def perturbed_c2():
    """C2 with heavy heading noise on the initial values: GTSAM's LM rejects
    up to 12 lambda tries in a row on it (oracle trace)."""
    from graphslam_amd import datasets
    g = datasets.make("C2")
    init = np.array(g.initial, copy=True)
    init[:, 2] += np.random.default_rng(7).normal(0, 0.5, len(init))
    return g, init


def _graph(case):
    from graphslam_amd import datasets
    if case == "C2p":
        return perturbed_c2()
    g = datasets.make(case)
    return g, np.array(g.initial, copy=True)


def _opt_worker(rank, world, port, q, case, kw, env=None, poison=False):
    try:
        os.environ.update(env or {})
        dist = _init(rank, world, port)
        from graphslam_amd import multi_gpu
        from graphslam_amd.pose_graph import PoseGraph
        g, init = _graph(case)
        pg = PoseGraph.from_dataset(g, device=0)
        pg.set_poses(init)
        hc = multi_gpu.attach_host(pg, dist, rank, world)
        if poison:   # a first optimize makes the workspace, then every must-write element is NaN
            pg.save_values()
            pg.optimize(**kw)
            pg.debug_poison_fronts()
            pg.restore_values()
        st = pg.optimize(**kw)
        st["trace"] = pg.trace()
        q.put((rank, st, pg.poses(), None))
        del hc
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, repr(e)))


_SINGLE = {}


def _single(case, kw, lanes=1):
    """One rank; lanes=1 is GTSAM's plain sequential lambda search.  The large
    graphs' one-rank references are kept for the module (C5's is shared by six
    tests; the library is deterministic run to run, test_save_restore_and_determinism)."""
    key = (case, tuple(sorted(kw.items())), lanes)
    if key in _SINGLE:
        st, x = _SINGLE[key]
        return dict(st), x.copy()
    from graphslam_amd.pose_graph import PoseGraph
    g, init = _graph(case)
    pg = PoseGraph.from_dataset(g, device=0)
    pg.set_poses(init)
    st = pg.optimize(**dict(kw, lambda_lanes=lanes))
    x = pg.poses()
    pg.close()
    if case in ("C3", "C5"):
        _SINGLE[key] = (dict(st), x.copy())
    return st, x


def _same(st, x, st1, x1):
    for k in ("iterations", "inner_iterations", "linearizations", "status"):
        assert st[k] == st1[k], (k, st[k], st1[k])
    assert st["final_error"] == st1["final_error"]
    np.testing.assert_array_equal(x, x1)          # bitwise: the same accepted candidates
    # no factorisation was silently re-run after a lost in-launch hand-off (round 6)
    assert st["handoff_retries"] == 0 and st1["handoff_retries"] == 0, (st["handoff_retries"], st1["handoff_retries"])


@pytest.mark.gpu
@pytest.mark.parametrize("case,lanes,kw", [
    ("C2p", 2, {}),
    ("C2p", 3, {}),
    ("C2p", 2, {"use_fixed_lambda_factor": 0}),
    ("C2p", 3, {"profile_every": 3}),
    ("C2p", 2, {"use_graphs": 0}),
    ("C3", 2, {}),
    ("C3", 4, {}),
])
def test_lanes_match_sequential(case, lanes, kw):
    """Concurrent lambda tries on one GPU (pgo_params.lambda_lanes) reproduce
    the sequential search bit for bit, in no more rounds.  (Rounds are sized to
    the tries expected -- one after a first-try acceptance, two after a
    multi-try one -- so a trajectory whose multi-try linearisations all follow
    first-try ones takes as many rounds as the sequential search, each of them
    a one-lane round.)"""
    st1, x1 = _single(case, kw, lanes=1)
    st, x = _single(case, kw, lanes=lanes)
    _same(st, x, st1, x1)
    assert st["lambda_rounds"] <= st1["lambda_rounds"]
    assert st["solves"] >= st1["solves"]
    if st1["inner_iterations"] > st1["linearizations"]:
        # a multi-try linearisation: the round after it is sized to two tries,
        # so some round ran more than one lane (a regression to one-lane
        # rounds throughout would keep solves == lambda_rounds)
        assert st["solves"] > st["lambda_rounds"], (st["solves"], st["lambda_rounds"])


def _single_worker(rank, world, port, q, case, kw, lanes, env):
    """_single in a fresh process (PGO_LANES_ADAPT is read once per process)."""
    try:
        os.environ.update(env)
        st, x = _single(case, kw, lanes)
        q.put((rank, st, x, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, repr(e)))


@pytest.mark.gpu
@pytest.mark.parametrize("case,lanes", [("C2p", 3), ("C3", 3)])
def test_full_lane_rounds_save_rounds(case, lanes):
    """With every round running all its lanes (PGO_LANES_ADAPT=0) consecutive
    tries of a multi-try linearisation share a round: strictly fewer rounds
    than the sequential search's tries, and the same trajectory bit for bit."""
    st1, x1 = _single(case, {}, lanes=1)
    assert st1["inner_iterations"] > st1["linearizations"]   # some linearisation walked several tries
    (_, st, x, err), = _run(1, _single_worker, (case, {}, lanes, {"PGO_LANES_ADAPT": "0"}), timeout=600)
    assert err is None, err
    _same(st, x, st1, x1)
    assert st["lambda_rounds"] < st1["lambda_rounds"], (st["lambda_rounds"], st1["lambda_rounds"])
    assert st["solves"] > st["lambda_rounds"]


@pytest.mark.gpu
def test_lane_count_changes_on_one_handle():
    """Lanes are numeric workspaces of the one plan (grid dimension y of every
    launch): switching 2 -> 1 -> 3 -> 2 on the same handle re-allocates them and
    re-captures the graphs; every run equals the sequential search bit for bit."""
    from graphslam_amd.pose_graph import PoseGraph
    g, init = _graph("C2p")
    st1, x1 = _single("C2p", {})
    pg = PoseGraph.from_dataset(g, device=0)
    for lanes in (2, 1, 3, 2):
        pg.set_poses(init)
        st = pg.optimize(lambda_lanes=lanes)
        _same(st, pg.poses(), st1, x1)


@pytest.mark.gpu
@pytest.mark.parametrize("case,world,kw", [
    ("C2p", 2, {"lambda_lanes": 1}),
    ("C2p", 3, {"lambda_lanes": 1}),
    ("C2p", 2, {"use_fixed_lambda_factor": 0}),
    ("C2p", 2, {"lambda_lanes": 2, "profile_every": 2}),
    ("C3", 2, {}),
    ("C3", 4, {"lambda_lanes": 1}),
])
def test_speculative_lambda_matches_one_rank(case, world, kw):
    st1, x1 = _single(case, {k: v for k, v in kw.items() if k != "lambda_lanes"})
    out = _run(world, _opt_worker, (case, kw), timeout=600)
    for rank, st, x, err in out:
        assert err is None, err
        assert st["ranks"] == world and st["transport"] == _lib.PGO_TRANSPORT_HOST
        _same(st, x, st1, x1)
        # a round solves `world` x lanes tries at once: fewer rounds than sequential tries
        if st1["inner_iterations"] > st1["linearizations"] and not kw.get("profile_every"):
            assert st["lambda_rounds"] < st1["lambda_rounds"]
    assert st1["ranks"] == 1 and st1["solves"] == st1["lambda_rounds"] >= st1["inner_iterations"]


@pytest.mark.gpu
def test_speculative_lambda_oracle_trajectory():
    """The 2-rank run on the perturbed C2 graph follows the C oracle's LM
    trajectory (iterations, lambda tries, final error)."""
    from oracle.oracle import Oracle
    g, init = perturbed_c2()
    ref = Oracle(g).optimize(init=init)
    out = _run(2, _opt_worker, ("C2p", {}), timeout=600)
    st = out[0][1]
    assert st["iterations"] == ref.stats["iterations"]
    assert st["inner_iterations"] == ref.stats["inner_iterations"]
    assert abs(st["final_error"] - ref.stats["final_error"]) <= 1e-8 * ref.stats["final_error"]


@pytest.mark.gpu
@pytest.mark.parametrize("case,world,lanes,kw", [
    ("C2p", 2, 1, {}), ("C2p", 3, 1, {}), ("C2p", 4, 1, {}),
    ("C2p", 2, 2, {}), ("C2p", 4, 3, {}),                       # lambda lanes x partition
    ("C3", 2, 1, {}), ("C3", 4, 1, {}),
    ("C3", 4, 2, {"max_outer": 3}),
    ("C3", 8, 1, {"max_outer": 2}),                             # BASELINE config C4 at 8 ranks
])
def test_partitioned_factorisation_matches_one_rank(case, world, lanes, kw):
    """PGO_MULTI_PARTITION, ranks sharing cuda:0 over the host transport:
    every try's factorisation split into the ranks' subtrees + the distributed
    top (top fronts' columns dealt to the ranks, every factored panel
    broadcast by its rank), the subtree roots' Schur complements and the
    subtree solutions all-gathered -- the LM trajectory and the final values
    are bitwise those of one rank, with and without lambda lanes (every rank
    factors the same lanes).  The 8-rank C3 case stops after 2 linearisations
    (its host-staged exchanges are slow on one shared GPU), both sides."""
    st1, x1 = _single(case, kw)
    out = _run(world, _opt_worker, (case, dict(kw, multi_gpu=1, lambda_lanes=lanes)), timeout=1200)
    for rank, st, x, err in out:
        assert err is None, err
        assert st["handoff_retries"] == 0 and st["transport"] == _lib.PGO_TRANSPORT_HOST
        assert st["iterations"] == st1["iterations"]
        assert st["inner_iterations"] == st1["inner_iterations"]
        assert st["linearizations"] == st1["linearizations"]
        assert st["final_error"] == st1["final_error"]
        np.testing.assert_array_equal(x, x1)
        if lanes > 1:   # (rounds sized to the tries expected: no more than one lane's)
            assert st["lambda_rounds"] <= st1["lambda_rounds"]
            if st1["inner_iterations"] > st1["linearizations"]:
                assert st["solves"] > st["lambda_rounds"]   # some round batched tries


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["partition", "spec"])
def test_c5_two_ranks_match_one_rank(mode):
    """BASELINE config C5 (1M poses / 5M edges) with two ranks sharing cuda:0
    over the host transport, first linearisation (max_outer 1): the
    partitioned factorisation (subtrees per rank, distributed top, 2.3 TFLOP
    per factorisation) and the speculative lambda search each reproduce the
    one-rank trajectory and values bit for bit."""
    kw = {"max_outer": 1}
    st1, x1 = _single("C5", kw)
    mkw = dict(kw, multi_gpu=1, lambda_lanes=1) if mode == "partition" else dict(kw, lambda_lanes=1)
    out = _run(2, _opt_worker, ("C5", mkw), timeout=1200)
    for rank, st, x, err in out:
        assert err is None, err
        assert st["ranks"] == 2
        _same(st, x, st1, x1)


def _hybrid_worker(rank, world, port, q, case, kw, groups, env=None):
    try:
        os.environ.update(env or {})
        dist = _init(rank, world, port)
        from graphslam_amd import multi_gpu
        from graphslam_amd.pose_graph import PoseGraph
        g, init = _graph(case)
        pg = PoseGraph.from_dataset(g, device=0)
        pg.set_poses(init)
        keep = multi_gpu.attach_hybrid(pg, dist, rank, world, groups, transport="host")
        st = pg.optimize(**kw)
        st["trace"] = pg.trace()
        q.put((rank, st, pg.poses(), None))
        del keep
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, repr(e)))


@pytest.mark.gpu
@pytest.mark.parametrize("case,world,groups,lanes,kw,env", [
    ("C2p", 4, 2, 1, {}, {}),                    # 2 groups x 2-rank partitions
    ("C2p", 6, 3, 1, {}, {}),                    # 3 groups x 2
    ("C2p", 4, 2, 2, {}, {}),                    # ... with 2 lambda lanes per group
    ("C3", 4, 2, 1, {"max_outer": 3}, {}),
    ("C5", 4, 2, 1, {"max_outer": 1}, {}),       # BASELINE config C5: 2 groups x 2-rank partitions
    ("C5", 4, 2, 1, {"max_outer": 1}, {"PGO_DIST_TOP": "0"}),   # ... with the replicated top: auto's 4-rank pick
    # round 6: the 8-rank layouts -- --multi auto's picks, C3 and C5: 4
    # groups x 2-rank partitions with the replicated top (profiles/r06_partition_bounds.json);
    # C5 also 4 x 2 and 2 x 4 with the distributed top (the 2 x 4's best central estimate)
    ("C3", 8, 4, 1, {"max_outer": 2}, {"PGO_DIST_TOP": "0"}),
    ("C5", 8, 4, 1, {"max_outer": 1}, {"PGO_DIST_TOP": "0"}),
    ("C5", 8, 4, 1, {"max_outer": 1}, {}),
    ("C5", 8, 2, 1, {"max_outer": 1}, {}),
])
def test_hybrid_matches_one_rank(case, world, groups, lanes, kw, env):
    """PGO_MULTI_HYBRID, ranks sharing cuda:0 over gloo sub-groups: each group
    splits every factorisation over its ranks (subtrees + distributed top, or
    the replicated top with PGO_DIST_TOP=0) and the groups run the speculative
    lambda search (one rank of each group per exchange) -- the trajectory and
    values are bitwise the one-rank run's, and a round covers groups x lanes
    tries.  C5's first linearisation walks 10 tries, so its 4- and 2-group
    searches spread them over the groups."""
    st1, x1 = _single(case, kw)
    out = _run(world, _hybrid_worker, (case, dict(kw, multi_gpu=2, lambda_lanes=lanes), groups, env), timeout=1200)
    for rank, st, x, err in out:
        assert err is None, err
        assert st["ranks"] == world
        assert st["transport"] == st["part_transport"] == _lib.PGO_TRANSPORT_HOST
        _same(st, x, st1, x1)
        if st1["inner_iterations"] > st1["linearizations"]:   # some linearisation walked several tries:
            assert st["lambda_rounds"] < st1["lambda_rounds"]   # the groups shared them


@pytest.mark.gpu
@pytest.mark.parametrize("case,world,groups", [("C2p", 2, 1), ("C3", 2, 1), ("C2p", 4, 2), ("C3", 4, 2)])
def test_replicated_top_matches_one_rank(case, world, groups):
    """The replicated top (PGO_DIST_TOP=0: every rank factors the top fronts
    after one all-gather of the subtree roots' update matrices) -- what the
    model prices faster than the distributed top at two ranks, so what --multi
    auto runs there and inside 2-rank hybrid groups -- bitwise the one-rank
    trajectory, alone (groups 1) and in the hybrid."""
    kw = {"max_outer": 3} if case == "C3" else {}
    st1, x1 = _single(case, kw)
    env = {"PGO_DIST_TOP": "0"}
    if groups == 1:
        out = _run(world, _opt_worker, (case, dict(kw, multi_gpu=1, lambda_lanes=1), env), timeout=900)
    else:
        out = _run(world, _hybrid_worker, (case, dict(kw, multi_gpu=2, lambda_lanes=1), groups, env), timeout=900)
    for rank, st, x, err in out:
        assert err is None, err
        _same(st, x, st1, x1)


@pytest.mark.gpu
def test_c5_four_ranks_partition_matches_one_rank():
    """BASELINE config C5 partitioned over four ranks sharing cuda:0 (first
    linearisation): bitwise the one-rank trajectory and values."""
    kw = {"max_outer": 1}
    st1, x1 = _single("C5", kw)
    out = _run(4, _opt_worker, ("C5", dict(kw, multi_gpu=1, lambda_lanes=1)), timeout=1200)
    for rank, st, x, err in out:
        assert err is None, err
        assert st["ranks"] == 4
        _same(st, x, st1, x1)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"PGO_DIST_TOP": "0"}])
def test_partitioned_poisoned_workspace_bitwise(env):
    """The poisoned-workspace check of the partitioned path: after
    a first optimize every element a factorisation must write before reading --
    fronts, frontal vectors, diagonal inverses, incl. the diagonal tiles' L that
    is no longer stored -- is NaN on both ranks (pgo_debug_poison_fronts), and
    the second optimize from the same values is bitwise the one-rank run: no
    stale or unexchanged element is read by the subtrees, the distributed /
    replicated top or the panel exchange."""
    st1, x1 = _single("C2p", {})
    out = _run(2, _opt_worker, ("C2p", dict(multi_gpu=1, lambda_lanes=1), env, True), timeout=900)
    for rank, st, x, err in out:
        assert err is None, err
        _same(st, x, st1, x1)


@pytest.mark.gpu
def test_partitioned_bad_pivot_on_one_rank():
    """A non-positive pivot that only one rank sees (PGO_DEBUG_BAD_PIVOT: rank
    1's first two factorisations) is reduced over the ranks with the subtree
    solutions: every rank rejects those tries and walks the same trace to the
    same stop reason and values."""
    env = {"PGO_DEBUG_BAD_PIVOT": "1:2"}
    out = _run(2, _opt_worker, ("C2p", dict(multi_gpu=1, lambda_lanes=1), env), timeout=900)
    for rank, st, x, err in out:
        assert err is None, err
    (_, st0, x0, _), (_, st1, x1, _) = out
    np.testing.assert_array_equal(st0["trace"][:, :7], st1["trace"][:, :7])   # (column 7: wall ms)
    assert st0["stop_reason"] == st1["stop_reason"]
    np.testing.assert_array_equal(x0, x1)
    tr = st0["trace"]
    assert tr[0, 2] == 0.0 and tr[1, 2] == 0.0      # the first two tries: not solved
    assert tr[2:, 2].min() == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("force", ["0", "1"])
def test_rccl_one_rank_communicator(monkeypatch, force):
    """RCCL transport on the box: a one-rank communicator (the only RCCL
    communicator one GPU allows) loads librccl, passes the exchange self test
    and leaves the optimisation unchanged."""
    # force = 1 (PGO_COMM_FORCE_COLLECTIVES): the one-rank communicator still
    # calls ncclAllGather / ncclBroadcast (in-place slot arithmetic included)
    monkeypatch.setenv("PGO_COMM_FORCE_COLLECTIVES", force)
    from graphslam_amd import multi_gpu
    from graphslam_amd.pose_graph import PoseGraph
    g, init = perturbed_c2()
    pg = PoseGraph.from_dataset(g, device=0)
    pg.set_poses(init)
    pg.comm_init_rccl(multi_gpu.unique_id(), 0, 1)
    assert pg.comm_rank() == (0, 1)
    pg.comm_selftest()
    st = pg.optimize(lambda_lanes=1)
    if force == "1":
        assert st["ms_comm"] > 0.0           # the all-gathers / broadcasts ran through RCCL
    st1, x1 = _single("C2p", {})
    assert st["inner_iterations"] == st1["inner_iterations"]
    np.testing.assert_array_equal(pg.poses(), x1)
    pg.comm_free()


# ---------------------------------------------------------------- RCCL set-up agreement (CPU, gloo)
class _FakeHandle:
    """Stands in for a PoseGraph in multi_gpu's set-up: records the
    communicator calls; `fail` names the init that raises on this rank."""

    def __init__(self, fail=None):
        self.calls, self.fail = [], fail

    def _rec(self, name, *a):
        self.calls.append(name)
        if name == self.fail:
            raise RuntimeError(f"forced {name} failure")

    def comm_init_rccl_part(self, uid, rank, size):
        self._rec("rccl_part", uid, rank, size)

    def comm_init_rccl(self, uid, rank, size):
        self._rec("rccl", uid, rank, size)

    def comm_init_host_part(self, s):
        self._rec("host_part")

    def comm_init_host(self, s):
        self._rec("host")

    def comm_free(self):
        self.calls.append("free")


def _setup_worker(rank, world, port, q, groups, fail_rank, fail_what):
    """attach_hybrid over RCCL with one rank failing at `fail_what` ('uid': its
    unique id, or an init name), then the bench's fallback to host transport."""
    try:
        dist = _init(rank, world, port)
        from graphslam_amd import multi_gpu
        pg = _FakeHandle(fail_what if rank == fail_rank and fail_what != "uid" else None)
        orig = multi_gpu.unique_id

        def uid():
            if rank == fail_rank and fail_what == "uid":
                raise RuntimeError("forced unique id failure")
            return b"x" * 128

        multi_gpu.unique_id = uid
        outcome = "rccl"
        try:
            multi_gpu.attach_hybrid(pg, dist, rank, world, groups, transport="rccl")
        except multi_gpu.CommSetupError:
            outcome = "fallback"
            multi_gpu.attach_hybrid(pg, dist, rank, world, groups, transport="host")
        multi_gpu.unique_id = orig
        q.put((rank, (outcome, pg.calls), None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("fail_rank,fail_what", [(2, "uid"), (1, "rccl_part"), (3, "rccl"), (None, None)])
def test_rccl_setup_failure_falls_back_together(fail_rank, fail_what):
    """one rank failing at any blocking step of the hybrid's RCCL
    set-up (its group's unique id, its partition-group init, the main init)
    makes EVERY rank raise CommSetupError at the same agreement point -- no rank
    is left inside a collective -- so all fall back to the host transport
    together; without a failure all stay on RCCL.  4 gloo ranks as 2 x 2, the
    RCCL calls stubbed (CPU)."""
    out = _run(4, _setup_worker, (2, fail_rank, fail_what))
    outcomes = set()
    for rank, res, err in out:
        assert err is None, err
        outcome, calls = res
        outcomes.add(outcome)
        if outcome == "fallback":
            assert calls[-2:] == ["host_part", "host"], calls
            if fail_what == "uid":   # agreed before any init
                assert "rccl_part" not in calls and "rccl" not in calls, calls
            else:                    # agreed after the failing init: every rank freed what it made
                assert "free" in calls, calls
        else:
            assert calls == ["rccl_part", "rccl"], calls
    assert outcomes == ({"rccl"} if fail_rank is None else {"fallback"})


def _hybrid_binding_worker(rank, world, port, q, case):
    """case 'one-rank-groups': hybrid with partition groups of one rank (the
    speculative search alone); 'stale': a hybrid set-up, then the main
    communicator replaced without pgo_comm_free -- the old partition group must
    not be used (PGO_MULTI_HYBRID then reports PGO_E_ARG)."""
    try:
        dist = _init(rank, world, port)
        from graphslam_amd import multi_gpu
        from graphslam_amd.pose_graph import PoseGraph
        g, init = _graph("C2p")
        pg = PoseGraph.from_dataset(g, device=0)
        pg.set_poses(init)
        if case == "one-rank-groups":
            keep = multi_gpu.attach_hybrid(pg, dist, rank, world, world, transport="host")   # groups of 1
            st = pg.optimize(multi_gpu=2, lambda_lanes=1)
            q.put((rank, (st, pg.poses(), pg.comm_part_rank()), None))
        else:
            keep = multi_gpu.attach_hybrid(pg, dist, rank, world, 1, transport="host")       # one group of `world`
            keep.append(multi_gpu.attach_host(pg, dist, rank, world))                       # main replaced, no free
            try:
                pg.optimize(multi_gpu=2, lambda_lanes=1)
                res = "ran"
            except Exception as e:  # noqa: BLE001
                res = repr(e)
            q.put((rank, (res, pg.comm_part_rank()), None))
        del keep
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.gpu
def test_hybrid_partition_groups_of_one_rank_are_the_speculative_search():
    """PGO_MULTI_HYBRID with partition groups of one rank (groups ==
    ranks) is a valid layout -- the speculative search alone -- and reproduces
    the one-rank run bit for bit (it used to return PGO_E_ARG)."""
    st1, x1 = _single("C2p", {})
    out = _run(2, _hybrid_binding_worker, ("one-rank-groups",), timeout=600)
    for rank, res, err in out:
        assert err is None, err
        st, x, part = res
        assert part == (0, 1)
        assert st["transport"] == _lib.PGO_TRANSPORT_HOST and st["part_transport"] == _lib.PGO_TRANSPORT_NONE
        _same(st, x, st1, x1)


@pytest.mark.gpu
def test_replaced_main_communicator_drops_the_stale_partition_group():
    """a main communicator initialised again without pgo_comm_free
    frees the partition group set up before the previous one, so a hybrid
    optimize cannot run on a stale group: PGO_E_ARG, the group gone (size 1)."""
    out = _run(2, _hybrid_binding_worker, ("stale",), timeout=600)
    for rank, res, err in out:
        assert err is None, err
        msg, part = res
        assert "PGO_MULTI_HYBRID needs a partition-group communicator" in msg or "-1" in msg, msg
        assert part == (0, 1)
