"""Cost model of the multi-GPU modes, used by bench.py's
``--multi auto`` and scripts/partition_bounds.py.  Every number it produces is
an estimate: no 8-GPU node has run this code.

Modes (the built ones first):

* partitioned factorisation (``partition``): the elimination tree split --
  each rank factors its subtrees, then the top fronts (the separators above
  them) are either replicated on every rank after one all-gather of the
  subtree roots' update matrices (``PGO_DIST_TOP=0``), or distributed column
  by column with every factored top panel broadcast by its owner (the default
  distributed top);
* speculative lambda search (``spec``): every rank solves different tries of
  GTSAM's lambda sequence (one lane each), the outcomes are all-gathered;
* hybrid (``hybrid``, G groups): each group of P / G ranks splits every
  factorisation (the distributed or the replicated top, whichever the model
  prices faster at P / G), the G groups run the speculative search;
* subtree-to-subcube (modelled only, not built): a top front factored by the
  ranks below it, its panels broadcast inside that group.

One factorisation (one lambda lane) is priced level by level: a level of the
one-GPU factorisation is throughput-bound (many fronts) or chain-bound (a few
big fronts whose 64-column panel steps run one after the other):

    T_L(one GPU)        the measured per-level span of a one-lane replay
                        (profiles/r04_level_spans.json, C3), else
                        max(F_L / R, S_L * t_step)
    rank r at level L   max(T_L * F_rL / F_L, S_rL * t_step)
    replicated top      every rank pays the top levels' one-GPU time, plus one
                        all-gather of the roots' update matrices (bytes / B)
    distributed top     the top's flops spread over the ranks but not its
                        chains; t_bcast per exchange point on the chain; every
                        rank receives exchange_bytes (bytes / B)

The LM trajectory is priced round by round from its tries per linearisation
(measured: TRIES, bench.py's per_step / c5 lines) and the measured replay time
of a round of L lanes (ROUND_MS):

    one GPU   rounds sized as the library sizes them (1 try expected at the
              first linearisation and after a first-try acceptance, 2 after a
              multi-try one, then all 3 lanes), each round ROUND_MS[L]
    spec      P one-lane tries per round: ceil(k / P) rounds per linearisation,
              each ROUND_MS[1] + the outcome all-gather and the accepted
              values' broadcast
    hybrid    the same with G groups, each round ROUND_MS[1] / S_part(P / G)

Stated constants, swept rather than trusted: B (bytes per second a receiving
rank ingests) in B_RANGE, t_bcast (latency of one exchange point) in
T_BCAST_RANGE; measured: t_step, R, ROUND_MS, TRIES.  ``choose`` picks the
built mode whose *worst* speed-up over that range is largest.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np

T_STEP = 31.2e-6                 # root front's step cadence, one lane (r04 stamps)
B_RANGE = (50e9, 150e9, 300e9)   # xGMI ingest per receiving rank (one link ~153 GB/s, 7 links)
T_BCAST_RANGE = (10e-6, 30e-6)   # RCCL latency of one exchange point
B_CENTRAL, T_BCAST_CENTRAL = 150e9, 30e-6
R_MEASURED = {"C3": 11.9e12, "C5": 26.6e12}   # one-GPU factorisation rate (bench factorisation aggregate)
R_DEFAULT = 11.9e12
# one lambda round's device time by lanes (factorisation replay + the lanes'
# solves), ms: C3 replays 8.23 / 12.52 / 17.02 ms (profiles/r05b_lanes_C3.txt)
# + 0.56 ms per lane left over in the bench's ms_solve (profiles/r05b_bench.json);
# profiles/r05_model_inputs.json overrides these (and holds C5's)
ROUND_MS = {"C3": {1: 8.785, 2: 13.637, 3: 18.705}}
# tries per linearisation of the headline trajectories (bench per_step /
# c5 lines); C3: 24 tries in 8 linearisations
TRIES = {"C3": [1, 1, 1, 1, 10, 2, 3, 5]}
_PROF = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
_SPANS = os.path.join(_PROF, "r04_level_spans.json")
_MEASURED = os.path.join(_PROF, "r05_model_inputs.json")   # measured ROUND_MS / TRIES per config (optional)


def _measured(config):
    """ROUND_MS and TRIES for a config: the committed measurements first."""
    rm, tr = ROUND_MS.get(config), TRIES.get(config)
    if os.path.exists(_MEASURED):
        d = json.load(open(_MEASURED)).get(config, {})
        if "round_ms" in d:
            rm = {int(k): float(v) for k, v in d["round_ms"].items()}
        if "tries" in d:
            tr = [int(k) for k in d["tries"]]
    return rm, tr


def front_flops(m, w):
    """Factorisation flops of fronts (m rows, w pivot columns), as the planner
    counts them (pgo_symbolic.cpp, CholPlan::flops)."""
    m = np.asarray(m, np.float64)
    w = np.asarray(w, np.float64)
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
    if not config or not os.path.exists(_SPANS):
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


class PlanData:
    """The host-side plan facts the model needs for one graph, computed once
    per rank count (each debug_* call runs a symbolic analysis)."""

    def __init__(self, pg, config):
        self.pg, self.config = pg, config
        self._lv, self._bound = {}, {}
        self.n = int(pg.num_vertices)

    def levels(self, P):
        if P not in self._lv:
            self._lv[P] = plan_levels(self.pg, P)
        return self._lv[P]

    def bound(self, P):
        if P not in self._bound:
            self._bound[P] = self.pg.debug_partition_bound(P)
        return self._bound[P]


def _one_gpu_levels(lv, config):
    T = level_spans(config)
    measured = T is not None and len(T) == len(lv["F"])
    if not measured:
        T = np.maximum(lv["F"] / R_MEASURED.get(config, R_DEFAULT), lv["S"] * T_STEP)
    return T, measured


def partition_speedups(pd: PlanData, P: int, B: float = B_CENTRAL, t_bcast: float = T_BCAST_CENTRAL) -> dict:
    """One factorisation: the one-GPU time and the replicated / distributed
    top's P-rank times (s) at the given transport constants."""
    lv = pd.levels(max(P, 1))
    T, measured = _one_gpu_levels(lv, pd.config)
    one = float(T.sum())
    if P <= 1:
        return {"one": one, "rep": one, "dist": one, "measured": measured, "ag_bytes": 0.0,
                "exchange_points": 0.0, "exchange_bytes": 0.0}
    F = np.maximum(lv["F"], 1.0)
    sub_t = float(np.maximum(T * lv["Fr"] / F, lv["Sr"] * T_STEP).sum(axis=1).max())
    top_rep = float(np.maximum(T * lv["Ft"] / F, lv["St"] * T_STEP).sum())
    recv = lv["root_doubles"].sum() - lv["root_doubles"]
    ag = 8.0 * float(recv.max())
    rep = sub_t + top_rep + ag / B + t_bcast
    b = pd.bound(P)
    top_dist = float(np.maximum(T * lv["Ft"] / (F * P), lv["St"] * T_STEP).sum())
    dist = sub_t + top_dist + b["exchange_points"] * t_bcast + b["exchange_bytes"] / B
    return {"one": one, "rep": rep, "dist": dist, "measured": measured, "ag_bytes": ag,
            "exchange_points": float(b["exchange_points"]), "exchange_bytes": float(b["exchange_bytes"])}


def one_gpu_rounds(tries, lanes: int = 3, adapt: bool = True):
    """Lane counts of the one-GPU lambda rounds, as pgo_optimize sizes them
    (pgo_api.cpp: 1 try expected at the first linearisation and after a
    first-try acceptance, 2 after a multi-try one; the rest at all lanes)."""
    rounds, prev = [], 0
    for k in tries:
        expect = 1 if prev == 0 else min(prev, 2)
        walked = 0
        while walked < k:
            lr = lanes
            if adapt and expect > walked:
                lr = min(lr, expect - walked)
            rounds.append(lr)
            walked += lr
        prev = k
    return rounds


def _round_ms(rm, lanes):
    """Round time of `lanes` lanes from the measured ones (linear between and beyond)."""
    if lanes in rm:
        return rm[lanes]
    ks = sorted(rm)
    if len(ks) == 1:
        return rm[ks[0]] * lanes
    return float(np.interp(lanes, ks, [rm[k] for k in ks], right=None)) if lanes <= ks[-1] else \
        rm[ks[-1]] + (lanes - ks[-1]) * (rm[ks[-1]] - rm[ks[-2]]) / (ks[-1] - ks[-2])


def trajectory_ms(tries, rm, slots: int, per_round_extra_ms: float = 0.0, one_round_ms: float | None = None):
    """ms of a trajectory whose rounds hold `slots` one-lane tries (spec /
    hybrid), each round one_round_ms (default the one-lane round) + extra."""
    r1 = rm[1] if one_round_ms is None else one_round_ms
    rounds = sum(math.ceil(k / slots) for k in tries)
    return rounds * (r1 + per_round_extra_ms), rounds


def estimate(pg, P: int, config: str | None = None, pd: PlanData | None = None) -> dict:
    """Model speed-ups of every mode against one GPU at P ranks, over the
    sensitivity range of the stated constants; the central point first.
    pd: a PlanData of pg to reuse across rank counts."""
    pd = pd or PlanData(pg, config)
    rm, tries = _measured(config)
    if rm is None:   # a config without measured rounds: C3's lane scaling on the modelled factorisation
        one_f = partition_speedups(pd, 1)["one"] * 1e3
        rm = {L: one_f * ROUND_MS["C3"][L] / ROUND_MS["C3"][1] for L in ROUND_MS["C3"]}
    if tries is None:
        tries = TRIES["C3"]
    one_ms = sum(_round_ms(rm, L) for L in one_gpu_rounds(tries))
    grid = {}
    hybrid_dist = {}   # per G: the groups' partition with the distributed top (else replicated)
    groups = [G for G in range(2, P) if P % G == 0]
    for B in B_RANGE:
        for tb in T_BCAST_RANGE:
            key = f"B{B / 1e9:.0f}_t{tb * 1e6:.0f}"
            # spec / hybrid: per round an all-gather of the outcomes and a
            # broadcast of the accepted values (32 B per pose)
            extra = 1e3 * (2 * tb + 32.0 * pd.n / B)
            spec_ms, _ = trajectory_ms(tries, rm, P, extra)
            ps = partition_speedups(pd, P, B, tb)
            s_dist, s_rep = ps["one"] / ps["dist"], ps["one"] / ps["rep"]
            row = {"spec": one_ms / spec_ms, "partition_dist": s_dist, "partition_rep": s_rep}
            for G in groups:   # each group's partition with one fixed top
                qs = partition_speedups(pd, P // G, B, tb)
                for top in ("dist", "rep"):
                    h_ms, _ = trajectory_ms(tries, rm, G, extra, rm[1] * qs[top] / qs["one"])
                    row[f"hybrid{G}_{top}"] = one_ms / h_ms
            grid[key] = row
    # Only one top runs, so each candidate is priced with a fixed top over the
    # whole sweep, and its top is the one with the better worst case (ADVICE
    # r05: taking the better top per grid point overstated the worst case);
    # "partition" / "hybrid<G>" are the chosen variants' figures
    worst = lambda k: min(r[k] for r in grid.values())   # noqa: E731
    part_dist = worst("partition_dist") >= worst("partition_rep")
    for G in groups:
        hybrid_dist[G] = worst(f"hybrid{G}_dist") >= worst(f"hybrid{G}_rep")
    for row in grid.values():
        row["partition"] = row["partition_dist" if part_dist else "partition_rep"]
        for G in groups:
            row[f"hybrid{G}"] = row[f"hybrid{G}_dist" if hybrid_dist[G] else f"hybrid{G}_rep"]
    central = grid[f"B{B_CENTRAL / 1e9:.0f}_t{T_BCAST_CENTRAL * 1e6:.0f}"]
    lo = {k: min(r[k] for r in grid.values()) for k in central}
    hi = {k: max(r[k] for r in grid.values()) for k in central}
    ps = partition_speedups(pd, P)
    b = pd.bound(P) if P > 1 else {}
    out = {"est_one_gpu_s": ps["one"], "est_replicated_top_s": ps["rep"], "est_distributed_top_s": ps["dist"],
           "est_speedup_replicated_top": central["partition_rep"],
           "est_speedup_distributed_top": central["partition_dist"],
           "est_speedup_spec": central["spec"], "est_speedup": central["partition"],
           "est_speedup_hybrid": {str(G): central[f"hybrid{G}"] for G in groups},
           "partition_distributed_top": bool(part_dist),
           "hybrid_distributed_top": {str(G): bool(v) for G, v in hybrid_dist.items()},
           "range_min": lo, "range_max": hi, "sensitivity": grid,
           "allgather_bytes_per_rank": ps["ag_bytes"],
           "exchange_points": b.get("exchange_points"), "exchange_bytes": b.get("exchange_bytes"),
           "one_gpu_trajectory_ms": one_ms, "tries_per_linearization": list(tries),
           "round_ms": {str(k): v for k, v in rm.items()},
           "level_times": "measured one-lane replay" if ps["measured"] else "modelled (flops / R, panel chain)",
           "model": (f"t_step {T_STEP * 1e6:.1f} us; B {[x / 1e9 for x in B_RANGE]} GB/s, t_bcast "
                     f"{[x * 1e6 for x in T_BCAST_RANGE]} us swept (central {B_CENTRAL / 1e9:.0f} GB/s, "
                     f"{T_BCAST_CENTRAL * 1e6:.0f} us); R {R_MEASURED.get(config, R_DEFAULT) / 1e12:.1f} TFLOP/s; "
                     f"rounds priced on the measured tries and round times"),
           "measured_on_hardware": False}
    return out


def choose(est: dict) -> tuple[str, int, bool]:
    """(mode, groups, distributed top) of the built mode whose worst-case
    speed-up over the sensitivity range is largest: 'spec', 'partition' or
    'hybrid' (groups = G; the partition's top: distributed unless the
    replicated one is better in the worst case)."""
    lo = est["range_min"]
    cands = {"spec": lo["spec"], "partition": lo["partition"]}
    for k, v in lo.items():
        if k.startswith("hybrid") and "_" not in k:   # (hybrid<G>: the fixed-top variant chosen in estimate)
            cands[k] = v
    best = max(cands, key=lambda k: cands[k])
    dist = est.get("partition_distributed_top", lo["partition_dist"] >= lo["partition_rep"])
    if best.startswith("hybrid"):
        G = int(best[6:])
        return "hybrid", G, est.get("hybrid_distributed_top", {}).get(str(G), True)
    return best, 1, dist


# ---- kept for callers of the round-4 interface
def choose_mode(est: dict) -> str:
    return choose(est)[0]


def dist_top(est: dict) -> bool:
    return choose(est)[2]
