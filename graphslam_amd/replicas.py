"""One process per GPU: rank setup and the timed region of bench.py.

Used by every multi-GPU mode ("Multi-GPU"): independent replicas
(`--multi replicas`, no data-path collective), the speculative lambda search
and the partitioned solve.  torch.distributed (gloo, CPU tensors only) is used
for the barrier around the timed region and for the max-over-ranks time /
summed work -- plumbing, not the product.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass


@dataclass
class Rank:
    rank: int
    world: int
    local_rank: int
    dist: object = None

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, v: float) -> float:
        return self._reduce(v, "MAX")

    def sum(self, v: float) -> float:
        return self._reduce(v, "SUM")

    def _reduce(self, v, op):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def init_from_env() -> Rank:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return Rank(rank, world, local, dist)


def timed_steps(r: Rank, step, steps: int, warmup: int):
    """warmup untimed calls, then exactly `steps` timed calls bracketed by
    barriers; returns (max-over-ranks seconds, summed per-rank work, per-rank
    list of step results).  `step()` returns the number of work units it did
    and must not return before its device work has completed."""
    for _ in range(warmup):
        step()
    results = []
    r.barrier()
    t0 = time.perf_counter()
    units = 0.0
    for _ in range(steps):
        res = step()
        units += res[0] if isinstance(res, tuple) else res
        results.append(res)
    r.barrier()
    elapsed = time.perf_counter() - t0
    return r.max(elapsed), r.sum(units), results
