"""graphslam_amd -- MI355X-native SE(2) pose-graph optimisation backend.

Drop-in for the one hot path of Sergimech/GraphSLAM: the src/graph node's
``gtsam::LevenbergMarquardtOptimizer(graph, initial).optimize()``
(/root/reference/src/graph/src/graph.cpp:119) on Pose2 prior + between factors.

* ``include/pgo.h`` / ``graphslam_amd/libpgo.so`` -- the C-ABI (HIP kernels for gfx950)
* ``graphslam_amd.PoseGraph``        -- native handle (bulk numpy in/out)
* ``graphslam_amd.gtsam``            -- GTSAM-named mirror (Pose2, Values, ...)
* ``graphslam_amd.datasets``         -- synthetic Manhattan graphs (BASELINE configs)
"""
from __future__ import annotations

__all__ = ["PoseGraph", "default_params", "gtsam", "datasets"]


def __getattr__(name):  # lazy: importing the package must not require the .so
    if name in ("PoseGraph", "default_params", "PgoError"):
        from . import pose_graph
        return getattr(pose_graph, name)
    if name in ("gtsam", "datasets"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
