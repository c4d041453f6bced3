"""Plan-derived bounds of the partitioned multi-GPU factorisation (host only).

For each config and rank count P: the per-rank flops of one factorisation with
the distributed top (subtrees + the rank's top columns + the top work every
rank repeats), the flop bound on the speed-up (total / busiest rank), the same
bound with the top replicated on every rank, and the distributed top's
exchanges per factorisation (broadcast rounds, bytes every rank receives).
Also graphslam_amd/multi_model.py's level-by-level time estimates of both tops
and of the speculative search (bench.py's --multi auto uses the same model).
Writes profiles/<out>.json.

    python scripts/partition_bounds.py [--configs C3 C5] [--out r06_partition_bounds]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from graphslam_amd.multi_model import PlanData, choose, estimate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C3", "C5"])
    ap.add_argument("--ranks", nargs="+", type=int, default=[2, 4, 8])
    ap.add_argument("--out", default="r06_partition_bounds")
    args = ap.parse_args()
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    res = {}
    for c in args.configs:
        g = datasets.make(c)
        pg = PoseGraph.from_dataset(g)
        pd = PlanData(pg, c)
        res[c] = {}
        for P in args.ranks:
            b = dict(pd.bound(P))
            b["rank_flops"] = [float(v) for v in b["rank_flops"]]
            b.update(estimate(pg, P, c, pd=pd))
            mode, groups, dist = choose(b)
            b["auto"] = {"mode": mode, "groups": groups, "distributed_top": dist}
            res[c][str(P)] = b
            print(c, P, json.dumps({k: v for k, v in b.items() if k not in ("rank_flops", "sensitivity")}), flush=True)
        pg.close()
    path = os.path.join(ROOT, "profiles", args.out + ".json")
    json.dump(res, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
