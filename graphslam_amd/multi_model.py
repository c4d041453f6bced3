"""Cost model of the multi-GPU modes, used by bench.py's
``--multi auto`` and scripts/partition_bounds.py.

Per factorisation with P ranks, the partitioned mode costs about

    max_rank_flops / R  +  exchange_points * t_x  +  exchange_bytes / B

(the busiest rank's flops at the one-GPU factorisation rate, one broadcast
round per factored top panel, every rank receiving every top panel), against
total_flops / R on one GPU.  The constants are stated, not measured on an
8-GPU node (none has run this code yet): R = 25 TFLOP/s (the C5 factorisation
rate on one MI355X, profiles/r02c_c5_bench.json), t_x = 30 us per broadcast
round (RCCL small-message latency over xGMI, order of magnitude), B = 50 GB/s
(one xGMI link's worth of broadcast bandwidth per rank).  The speculative lambda
search is bounded by tries per linearisation (C3: 24 / 8, measured rounds 13 -> 8):
its estimate is SPEC_GAIN = 1.6.
"""
from __future__ import annotations

R_FLOPS = 25e12
T_X = 30e-6
B_BCAST = 50e9
SPEC_GAIN = 1.6


def partition_estimate(b: dict) -> dict:
    """b: PoseGraph.debug_partition_bound(P).  Returns the model's times (s)
    and estimated speed-up of the partitioned factorisation."""
    one = b["total_flops"] / R_FLOPS
    part = max(b["rank_flops"]) / R_FLOPS + b["exchange_points"] * T_X + b["exchange_bytes"] / B_BCAST
    return {"est_one_gpu_s": one, "est_partition_s": part, "est_speedup": one / part,
            "model": f"R {R_FLOPS / 1e12:.0f} TFLOP/s, {T_X * 1e6:.0f} us per broadcast round, "
                     f"{B_BCAST / 1e9:.0f} GB/s broadcast"}


def choose_mode(b: dict) -> str:
    """'partition' when its estimate beats the speculative search's bound."""
    return "partition" if partition_estimate(b)["est_speedup"] > SPEC_GAIN else "spec"
