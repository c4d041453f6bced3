"""Model-only estimate (nothing here is built) of a subtree-to-subcube mapping of
the partitioned factorisation, against the built distributed top
(graphslam_amd/multi_model.py).

The built distributed top deals every top front's panels over all P ranks and
every rank receives every top panel (the replicated backward solve needs them),
so the bytes each rank receives grow with P.  Subtree-to-subcube instead gives
a top front only the ranks below it: the root all P, each child subtree half of
them (split by subtree flops), and so on down to one rank per subtree.  A top
front's panels are then broadcast inside its group only, and with the backward
solve distributed the same way a rank receives only the panels of the top
fronts on its path to the root.  Same constants as multi_model (t_step, t_bcast,
B, R, the measured one-lane level spans where recorded).

    python scripts/subcube_model.py [--configs C3 C5] [--out r04_subcube_model]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from graphslam_amd import multi_model as mm  # noqa: E402


def subcube_groups(parent, f, P):
    """Rank interval [lo, hi) of every front: the root all P ranks; a front's
    children split their parent's interval by subtree flops (largest first,
    greedy), down to single ranks (a whole subtree on one rank)."""
    ns = len(parent)
    kids = [[] for _ in range(ns)]
    roots = []
    for s in range(ns):
        (kids[parent[s]] if parent[s] >= 0 else roots).append(s)
    sub = f.astype(np.float64).copy()
    for s in range(ns):   # postorder: children before parents
        if parent[s] >= 0:
            sub[parent[s]] += sub[s]
    lo = np.zeros(ns, np.int64)
    hi = np.zeros(ns, np.int64)

    def split(items, a, b):
        """items (fronts) over ranks [a, b): one rank each when b - a == 1."""
        stack = [(items, a, b)]
        while stack:
            its, a, b = stack.pop()
            if not its:
                continue
            if b - a == 1 or len(its) == 1:
                for s in its:
                    lo[s], hi[s] = a, b
                    if kids[s]:
                        stack.append((kids[s], a, b))
                continue
            # two bins by flops (largest first), ranks split in proportion
            order = sorted(its, key=lambda s: -sub[s])
            bins, load = ([], []), [0.0, 0.0]
            for s in order:
                k = 0 if load[0] <= load[1] else 1
                bins[k].append(s)
                load[k] += sub[s]
            tot = load[0] + load[1]
            cut = a + int(round((b - a) * load[0] / tot)) if tot > 0 else a + (b - a) // 2
            cut = min(max(cut, a + 1), b - 1)
            stack.append((bins[0], a, cut))
            stack.append((bins[1], cut, b))

    split(roots, 0, P)
    return lo, hi


def estimate(pg, P, config):
    w, m, lv = pg.debug_fronts()
    parent = pg.debug_parents()
    f = mm.front_flops(m, w)
    lo, hi = subcube_groups(parent, f, P)
    g = (hi - lo).astype(np.float64)
    blocked = (m > 128) | (w > 32)
    steps = np.where(blocked, (w + 63) // 64, 1).astype(np.float64)
    nl = int(lv.max()) + 1
    F = np.zeros(nl)
    np.add.at(F, lv, f)
    T = mm.level_spans(config)
    measured = T is not None and len(T) == nl
    if not measured:
        S = np.zeros(nl)
        np.maximum.at(S, lv, steps)
        T = np.maximum(F / mm.R_MEASURED.get(config, mm.R_DEFAULT), S * mm.T_STEP)
    one = float(T.sum())
    # per rank and level: its share of the level's flops (a front's flops split
    # over its group), floored by the longest panel chain among its fronts
    share = np.zeros((P, nl))
    chain = np.zeros((P, nl))
    pbytes = 8.0 * (m.astype(np.float64) * w - w.astype(np.float64) * (w - 1) / 2)
    recv = np.zeros(P)
    points = np.zeros(P)
    for s in range(len(w)):
        a, b = int(lo[s]), int(hi[s])
        share[a:b, lv[s]] += f[s] / (b - a)
        chain[a:b, lv[s]] = np.maximum(chain[a:b, lv[s]], steps[s] * mm.T_STEP)
        if b - a > 1:   # a shared front: its panels broadcast inside its group
            recv[a:b] += pbytes[s] * (b - a - 1) / (b - a)
            points[a:b] += steps[s]
    t_rank = np.maximum(T[None, :] * share / np.maximum(F, 1.0)[None, :], chain).sum(axis=1)
    t_rank += points * mm.T_BCAST + recv / mm.B_XGMI
    worst = int(np.argmax(t_rank))
    return {"est_one_gpu_s": one, "est_subcube_s": float(t_rank.max()), "est_speedup_subcube": one / float(t_rank.max()),
            "recv_bytes_per_rank_max": float(recv.max()), "exchange_points_max": float(points.max()),
            "busiest_rank": worst, "level_times": "measured one-lane replay" if measured else "modelled",
            "built": False}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C3", "C5"])
    ap.add_argument("--ranks", nargs="+", type=int, default=[2, 4, 8])
    ap.add_argument("--out", default="r04_subcube_model")
    args = ap.parse_args()
    from graphslam_amd import datasets
    from graphslam_amd.pose_graph import PoseGraph
    res = {}
    for c in args.configs:
        pg = PoseGraph.from_dataset(datasets.make(c))
        res[c] = {}
        for P in args.ranks:
            res[c][str(P)] = estimate(pg, P, c)
            print(c, P, json.dumps(res[c][str(P)]), flush=True)
        pg.close()
    path = os.path.join(ROOT, "profiles", args.out + ".json")
    json.dump(res, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
