"""Bitwise A/B of a knob (diagnostics): one GTSAM-default LM optimize of a
config per process, printing the final error and a hash of the poses, so runs
under different environment knobs can be compared bit for bit.

    PGO_X=1 python scripts/bitwise_env_check.py [--config C3] [--lanes 3]
"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--lanes", type=int, default=3)
    args = ap.parse_args()
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph, default_params
    pg = PoseGraph.from_dataset(datasets.make(args.config))
    st = pg.optimize(default_params(lambda_lanes=args.lanes))
    x = pg.poses()
    h = hashlib.sha256(x.tobytes()).hexdigest()[:16]
    print(f"{args.config} lanes {args.lanes}: final {st['final_error']!r} tries {st['inner_iterations']} poses {h}")


if __name__ == "__main__":
    main()
