"""Cost model of the multi-GPU modes, used by bench.py's
``--multi auto`` and scripts/partition_bounds.py.

The partitioned factorisation splits the elimination tree: each rank factors
its subtrees, then the top fronts (the separators above them) are either
replicated on every rank after one all-gather of the subtree roots' update
matrices (``PGO_DIST_TOP=0``), or distributed column by column with every
factored top panel broadcast by its owner (the default distributed top).  The
one-GPU factorisation of a level is either throughput-bound (many fronts) or
chain-bound (a few big fronts whose 64-column panel steps run one after the
other), so the model works level by level:

    T_L(one GPU)        measured per-level span of a one-lane replay when
                        given (profiles/r04_level_spans.json), else
                        max(F_L / R, S_L * t_step)
    rank r at level L   max(T_L * F_rL / F_L, S_rL * t_step)   (its flop share,
                        but never below the panel chain of its longest front)
    replicated top      every rank pays the top levels' one-GPU time, plus one
                        all-gather of the roots' update matrices (bytes / B)
    distributed top     the top's flops spread over the ranks but its chains
                        not, every exchange point adds t_bcast on the chain,
                        every rank receives exchange_bytes (bytes / B)

F = flops, S = panel steps of the level's longest front.  Constants: t_step =
31.2 us (the root front's measured step cadence, one lane, r04a), t_bcast =
30 us (RCCL small-message latency over xGMI, order of magnitude), B = 50 GB/s
(one xGMI link's worth of ring bandwidth per receiving rank), R = the measured
one-GPU factorisation rate (C3 11.4, C5 26 TFLOP/s).  Only t_step and R are
measured; t_bcast and B are stated, no 8-GPU node has run this code.

The speculative lambda search (every rank solves different tries of GTSAM's
lambda sequence) is bounded by the tries per linearisation: SPEC_GAIN from the
C3 trajectory (24 tries in 8 linearisations: 1, 1, 1, 1, 10, 2, 3, 5), one
lambda lane per rank, a one-lane round about half a three-lane one
(DESIGN.md §5).
"""
from __future__ import annotations

import json
import os

import numpy as np

T_STEP = 31.2e-6
T_BCAST = 30e-6
B_XGMI = 50e9
R_MEASURED = {"C3": 11.4e12, "C5": 26e12}
R_DEFAULT = 11.4e12
SPEC_GAIN = {1: 1.0, 2: 1.4, 4: 2.0, 8: 2.3}
_SPANS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                      "r04_level_spans.json")


def spec_gain(P: int) -> float:
    ks = sorted(SPEC_GAIN)
    return float(np.interp(P, ks, [SPEC_GAIN[k] for k in ks]))


def front_flops(m, w):
    """Factorisation flops of fronts (m rows, w pivot columns), as the planner
    counts them (pgo_symbolic.cpp, CholPlan::flops)."""
    m = np.asarray(m, np.float64)
    w = np.asarray(w, np.float64)
    # sum_{k<w} 1 + r + r (r + 1), r = m - k - 1
    s1 = w
    s_r = w * (m - 1) - w * (w - 1) / 2
    s_r2 = sum_sq(m - w, m - 1)
    return s1 + 2 * s_r + s_r2


def sum_sq(a, b):
    """sum of r^2 for r = a .. b (vectorised, a <= b + 1)."""
    def cube(n):
        return n * (n + 1) * (2 * n + 1) / 6
    return cube(b) - cube(a - 1)


def level_spans(config: str, lanes: int = 1):
    """Measured one-GPU per-level spans (s) of a replay, if recorded."""
    if not os.path.exists(_SPANS):
        return None
    d = json.load(open(_SPANS)).get(config, {}).get(str(lanes))
    return None if d is None else np.asarray(d, np.float64) * 1e-6


def plan_levels(pg, P: int):
    """Per level of the one-rank plan: total flops and longest panel chain, per
    rank its subtree fronts' flops and chain, and the top fronts' (owner -1)
    flops and chain for a P-rank partition; plus the subtree roots' update
    matrix doubles per rank (the replicated top's all-gather)."""
    w, m, lv = pg.debug_fronts()
    owner = pg.debug_partition(P)[0] if P > 1 else np.zeros(len(w), np.int32)
    parent = pg.debug_parents()
    f = front_flops(m, w)
    blocked = (m > 128) | (w > 32)
    steps = np.where(blocked, (w + 63) // 64, 1).astype(np.float64)
    nl = int(lv.max()) + 1 if len(lv) else 0
    F = np.zeros(nl)
    S = np.zeros(nl)
    Fr = np.zeros((P, nl))
    Sr = np.zeros((P, nl))
    Ft = np.zeros(nl)
    St = np.zeros(nl)
    np.add.at(F, lv, f)
    np.maximum.at(S, lv, steps)
    top = owner < 0
    np.add.at(Ft, lv[top], f[top])
    np.maximum.at(St, lv[top], steps[top])
    for r in range(P):
        sel = owner == r
        np.add.at(Fr[r], lv[sel], f[sel])
        np.maximum.at(Sr[r], lv[sel], steps[sel])
    root = (owner >= 0) & ((parent < 0) | (owner[np.maximum(parent, 0)] < 0))
    u = (m - w).astype(np.float64)
    root_doubles = np.zeros(P)
    np.add.at(root_doubles, owner[root], (u * (u + 1) / 2 + u)[root])
    return dict(F=F, S=S, Fr=Fr, Sr=Sr, Ft=Ft, St=St, root_doubles=root_doubles, total_flops=float(f.sum()))


def estimate(pg, P: int, config: str | None = None, bound: dict | None = None) -> dict:
    """Model times (s) and speed-ups of the P-rank modes against one GPU.
    bound: pg.debug_partition_bound(P) (the distributed top's exchanges)."""
    lv = plan_levels(pg, P)
    R = R_MEASURED.get(config, R_DEFAULT)
    T = level_spans(config) if config else None
    measured = T is not None and len(T) == len(lv["F"])
    if not measured:
        T = np.maximum(lv["F"] / R, lv["S"] * T_STEP)
    F = np.maximum(lv["F"], 1.0)
    one = float(T.sum())
    sub = np.maximum(T * lv["Fr"] / F, lv["Sr"] * T_STEP)          # [rank, level]
    sub_t = float(sub.sum(axis=1).max())
    top_rep = float(np.maximum(T * lv["Ft"] / F, lv["St"] * T_STEP).sum())
    recv = lv["root_doubles"].sum() - lv["root_doubles"]            # doubles each rank receives
    ag = 8.0 * float(recv.max()) / B_XGMI + T_BCAST
    rep = sub_t + top_rep + ag
    b = bound or pg.debug_partition_bound(P)
    top_dist = float(np.maximum(T * lv["Ft"] / (F * P), lv["St"] * T_STEP).sum())
    dist = sub_t + top_dist + b["exchange_points"] * T_BCAST + b["exchange_bytes"] / B_XGMI
    out = {"est_one_gpu_s": one, "est_replicated_top_s": rep, "est_distributed_top_s": dist,
           "est_speedup_replicated_top": one / rep, "est_speedup_distributed_top": one / dist,
           "est_speedup_spec": spec_gain(P), "allgather_bytes_per_rank": 8.0 * float(recv.max()),
           "level_times": "measured one-lane replay" if measured else "modelled (flops / R, panel chain)",
           "model": f"t_step {T_STEP * 1e6:.1f} us, t_bcast {T_BCAST * 1e6:.0f} us per exchange point, "
                    f"B {B_XGMI / 1e9:.0f} GB/s, R {R / 1e12:.1f} TFLOP/s"}
    out["est_speedup"] = max(out["est_speedup_replicated_top"], out["est_speedup_distributed_top"])
    return out


def choose_mode(est: dict) -> str:
    """'partition' (with est['dist_top'] saying which top) when the better
    partitioned estimate beats the speculative search's, else 'spec'."""
    return "partition" if est["est_speedup"] > est["est_speedup_spec"] else "spec"


def dist_top(est: dict) -> bool:
    return est["est_speedup_distributed_top"] >= est["est_speedup_replicated_top"]
