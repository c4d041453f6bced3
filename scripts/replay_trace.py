"""Per-launch timeline of one factorisation replay (diagnostics): run under
rocprofv3 --kernel-trace; times `reps` replays of the captured factorisation
graph with `lanes` lambda lanes (pgo_debug_factor_time).  Summarise with
scripts/timeline_summary.py.

    rocprofv3 --kernel-trace -f csv -d OUT -o t -- python3 scripts/replay_trace.py --lanes 3 --reps 2
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--lanes", type=int, default=3)
ap.add_argument("--reps", type=int, default=2)
args = ap.parse_args()
from graphslam_amd import datasets  # noqa: E402
from graphslam_amd.pose_graph import PoseGraph  # noqa: E402

pg = PoseGraph.from_dataset(datasets.make(args.config))
print("ms per replay", pg.debug_factor_time(args.lanes, args.reps), flush=True)
