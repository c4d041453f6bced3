"""The multi-GPU cost model (graphslam_amd/multi_model.py), host only."""
import numpy as np


def _pg(name="C2"):
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    return PoseGraph.from_dataset(datasets.make(name))


def test_front_flops_match_the_plan():
    """The model's per-front flops sum to the planner's factorisation flops."""
    from graphslam_amd import multi_model
    pg = _pg()
    w, m, _ = pg.debug_fronts()
    total = pg.debug_plan()["factor_flops"]
    assert abs(multi_model.front_flops(m, w).sum() - total) <= 1e-9 * total


def test_plan_levels_partition_the_flops():
    """Per level, the ranks' subtree flops plus the top's add up to the level's."""
    from graphslam_amd import multi_model
    pg = _pg()
    for P in (2, 4):
        lv = multi_model.plan_levels(pg, P)
        np.testing.assert_allclose(lv["Fr"].sum(axis=0) + lv["Ft"], lv["F"], rtol=1e-12)
        assert (lv["S"] >= lv["St"]).all() and (lv["S"][None, :] >= lv["Sr"]).all()
        assert (lv["root_doubles"] > 0).sum() >= 2


def test_estimate_and_choice():
    """Estimates are positive and finite over the whole sensitivity range; the
    auto choice is the built mode with the best worst case."""
    from graphslam_amd import multi_model
    pg = _pg()
    pd = multi_model.PlanData(pg, "C2")
    for P in (2, 4, 8):
        e = multi_model.estimate(pg, P, "C2", pd=pd)
        for k in ("est_one_gpu_s", "est_replicated_top_s", "est_distributed_top_s"):
            assert np.isfinite(e[k]) and e[k] > 0
        assert e["level_times"].startswith("modelled")   # no measured C2 spans
        assert len(e["sensitivity"]) == len(multi_model.B_RANGE) * len(multi_model.T_BCAST_RANGE)
        for row in e["sensitivity"].values():
            assert all(np.isfinite(v) and v > 0 for v in row.values())
        assert set(e["est_speedup_hybrid"]) == {str(G) for G in range(2, P) if P % G == 0}
        mode, groups, dist = multi_model.choose(e)
        lo = e["range_min"]
        best = max(v for k, v in lo.items() if k in ("spec", "partition") or (k.startswith("hybrid") and "_" not in k))
        got = lo["partition"] if mode == "partition" else lo["spec"] if mode == "spec" else lo[f"hybrid{groups}"]
        assert got == best
        # each candidate's worst case is that of ONE fixed top over the whole sweep
        for G in (G for G in range(2, P) if P % G == 0):
            top = "dist" if e["hybrid_distributed_top"][str(G)] else "rep"
            assert lo[f"hybrid{G}"] == lo[f"hybrid{G}_{top}"] == max(lo[f"hybrid{G}_dist"], lo[f"hybrid{G}_rep"])
        top = "dist" if e["partition_distributed_top"] else "rep"
        assert lo["partition"] == lo[f"partition_{top}"]
        if mode == "hybrid":
            assert dist == e["hybrid_distributed_top"][str(groups)]
        assert e["measured_on_hardware"] is False


def test_rounds_follow_the_library_sizing():
    """One GPU's rounds as pgo_optimize sizes them: one lane expected at the
    first linearisation and after a first-try acceptance, two after a
    multi-try one, the rest at all lanes (C3: 13 rounds, 26 factorisations, as
    the bench's lambda_rounds / solves)."""
    from graphslam_amd import multi_model
    r = multi_model.one_gpu_rounds([1, 1, 1, 1, 10, 2, 3, 5], lanes=3)
    assert len(r) == 13 and sum(r) == 26       # BENCH_r04: 13 lambda rounds, 26 solves
    assert r[:5] == [1, 1, 1, 1, 1]
    # spec: ceil(k / P) one-lane rounds
    _, n = multi_model.trajectory_ms([1, 1, 1, 1, 10, 2, 3, 5], {1: 1.0}, 8)
    assert n == 9
