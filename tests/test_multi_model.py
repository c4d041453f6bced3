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
    """Estimates are positive and finite; the choice follows the larger one."""
    from graphslam_amd import multi_model
    pg = _pg()
    for P in (2, 8):
        e = multi_model.estimate(pg, P, "C2")
        for k in ("est_one_gpu_s", "est_replicated_top_s", "est_distributed_top_s"):
            assert np.isfinite(e[k]) and e[k] > 0
        assert e["level_times"].startswith("modelled")   # no measured C2 spans
        mode = multi_model.choose_mode(e)
        assert mode == ("partition" if e["est_speedup"] > e["est_speedup_spec"] else "spec")
        assert multi_model.dist_top(e) == (e["est_speedup_distributed_top"] >= e["est_speedup_replicated_top"])
    assert multi_model.spec_gain(8) == 2.3 and 1.4 < multi_model.spec_gain(3) < 2.0
