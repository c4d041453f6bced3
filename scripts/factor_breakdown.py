"""Graph-mode factorisation time by launch family (diagnostics, GPU box).

For each lambda-lane count, the device time of one replay of the captured
factorisation graph (pgo_debug_factor_time), in a fresh process per
PGO_ABLATE setting (families left out at capture: the factor is then wrong,
only its time is read).  The difference to the full replay is what a family
adds to the critical path.

    python scripts/factor_breakdown.py [--config C3] [--lanes 1 3] [--ablate small plain ...]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(config, lanes, reps):
    sys.path.insert(0, ROOT)
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    pg = PoseGraph.from_dataset(datasets.make(config))
    return {str(l): pg.debug_factor_time(l, reps) for l in lanes}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--lanes", nargs="+", type=int, default=[1, 3])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--ablate", nargs="*", default=["small", "plain", "assemble", "vec", "first", "step",
                                                    "step,plain"])
    ap.add_argument("--envs", nargs="*", default=None,
                    help="instead of ablations: settings to compare, each 'tag:VAR=VAL[,VAR=VAL]'")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        print(json.dumps(one(args.config, args.lanes, args.reps)), flush=True)
        return
    res = {}
    runs = []
    if args.envs is not None:
        for e in ["default:"] + args.envs:
            tag, _, kv = e.partition(":")
            runs.append((tag, dict(x.split("=", 1) for x in kv.split(",") if x)))
    else:
        runs = [("none", {})] + [(a, {"PGO_ABLATE": a}) for a in args.ablate]
    for ab, extra in runs:
        env = dict(os.environ)
        env.update(extra)
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--config", args.config, "--reps", str(args.reps),
               "--lanes"] + [str(l) for l in args.lanes]
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        res[ab] = json.loads(line[-1]) if line else {"error": out.stderr[-300:]}
        print(ab, res[ab], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
