"""Multi-GPU speculative lambda search: attach a communicator to a PoseGraph.

One process per GPU, every rank holding the same graph (include/pgo.h,
"multi-GPU").  The library does the exchange itself; this module only sets the
communicator up:

* ``attach_rccl`` -- rank 0 makes an RCCL unique id (``pgo_comm_unique_id``),
  the id's 128 bytes travel over the caller's torch.distributed group (gloo,
  host), every rank calls ``pgo_comm_init_rccl`` on its own device.  The
  per-round all-gather and the accepted-values broadcast then run as RCCL
  collectives on the library's HIP stream, over xGMI.
* ``HostComm`` / ``attach_host`` -- the same exchange through host callbacks on
  a torch.distributed gloo group (tests: two ranks sharing one GPU, where RCCL
  refuses duplicate devices, or CPU-only self tests).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def unique_id() -> bytes:
    buf = C.create_string_buffer(256)
    n = L.lib().pgo_comm_unique_id(buf, 256)
    if n < 0:
        raise RuntimeError(f"pgo_comm_unique_id failed ({n}): RCCL not loadable")
    return buf.raw[:n]


class CommSetupError(RuntimeError):
    """An RCCL communicator could not be brought up.  Raised on EVERY rank
    together (the setup steps end in agreement points), so a caller can fall
    back to the host transport on all ranks without a rank left waiting in a
    collective."""


def _agree(dist, ok: bool, group=None) -> bool:
    """All-reduce(MIN) of a success flag over `group` (default: every rank,
    gloo): True only when every rank succeeded.  Every rank must call it, the
    failed ones included."""
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _try(fn, errs):
    try:
        return fn(), True
    except Exception as e:  # noqa: BLE001 -- turned into an agreed failure
        errs.append(repr(e))
        return None, False


def _rccl_setup(pg, dist, setups):
    """Bring up RCCL communicators with agreement points between the blocking
    steps: (1) every sub-group's first rank makes its ids, (2) the
    ids travel over gloo, (3) each communicator is initialised in turn -- a
    collective inside its sub-group.  After each step every rank learns whether
    all ranks succeeded; on any failure all ranks free what they made and raise
    CommSetupError together, so no rank is left inside a collective its peers
    have abandoned.  setups: [(global ranks of the sub-group, its gloo group or
    None, my position, size, init fn)]."""
    errs = []
    ids = []
    ok = True
    for ranks, grp, me, size, init in setups:            # (1) ids, made by each group's first rank
        uid, good = _try(unique_id, errs) if me == 0 else (None, True)
        ids.append(uid)
        ok = ok and good
    if not _agree(dist, ok):
        raise CommSetupError(f"RCCL unique id failed on some rank ({'; '.join(errs) or 'elsewhere'})")
    for k, (ranks, grp, me, size, init) in enumerate(setups):   # (2) ids over gloo
        if size > 1:
            obj = [ids[k]]
            _, good = _try(lambda: dist.broadcast_object_list(obj, src=ranks[0], group=grp), errs)
            ids[k] = obj[0]
            ok = ok and good and ids[k] is not None
    if not _agree(dist, ok):
        raise CommSetupError(f"RCCL id exchange failed on some rank ({'; '.join(errs) or 'elsewhere'})")
    for k, (ranks, grp, me, size, init) in enumerate(setups):   # (3) one communicator at a time
        _, good = _try(lambda: init(ids[k], me, size), errs)
        if not _agree(dist, good):
            try:
                pg.comm_free()
            except Exception:  # noqa: BLE001
                pass
            raise CommSetupError(f"RCCL communicator {k} failed on some rank ({'; '.join(errs) or 'elsewhere'})")


def attach_rccl(pg, dist, rank: int, world: int):
    """RCCL communicator over all `world` ranks of the default torch.distributed
    group; CommSetupError on every rank if any rank fails."""
    _rccl_setup(pg, dist, [(list(range(world)), None, rank, world, pg.comm_init_rccl)])


class HostComm:
    """pgo_host_comm over a torch.distributed (gloo) group, host buffers.
    `ranks`: the group's global ranks in group order (a sub-group: broadcast
    roots are given in group numbering)."""

    def __init__(self, dist, rank: int, world: int, group=None, ranks=None):
        import torch
        self._torch, self._dist, self._group = torch, dist, group
        self._ranks = list(ranks) if ranks is not None else list(range(world))
        self.rank, self.world = rank, world
        self._ag = L.ALLGATHER_FN(self._allgather)
        self._bc = L.BROADCAST_FN(self._broadcast)
        self.struct = L.PgoHostComm(None, rank, world, self._ag, self._bc)

    def _view(self, ptr, n):
        return self._torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * n).from_address(ptr)))

    def _allgather(self, ctx, src, dst, n):
        try:
            t = self._view(src, n).clone()
            outs = [self._torch.empty(n, dtype=self._torch.uint8) for _ in range(self.world)]
            self._dist.all_gather(outs, t, group=self._group)
            flat = self._torch.cat(outs).numpy()      # keep alive across the copy
            C.memmove(dst, flat.ctypes.data, n * self.world)
            return 0
        except Exception:  # noqa: BLE001 -- no exception may cross the C-ABI
            return 1

    def _broadcast(self, ctx, buf, n, root):
        try:
            self._dist.broadcast(self._view(buf, n), src=self._ranks[root], group=self._group)
            return 0
        except Exception:  # noqa: BLE001
            return 1


def attach_host(pg, dist, rank: int, world: int, group=None) -> HostComm:
    hc = HostComm(dist, rank, world, group)
    pg.comm_init_host(hc.struct)
    return hc


def hybrid_layout(world: int, groups: int):
    """PGO_MULTI_HYBRID rank layout: `groups` partition groups of world/groups
    consecutive ranks; the speculative search links the ranks at the same
    position of every group.  Returns (part_ranks, spec_ranks): for each group
    its global ranks, for each position its global ranks."""
    if groups < 1 or world % groups:
        raise ValueError(f"{world} ranks do not split into {groups} equal groups")
    pp = world // groups
    part = [list(range(g * pp, (g + 1) * pp)) for g in range(groups)]
    spec = [[g * pp + i for g in range(groups)] for i in range(pp)]
    return part, spec


def attach_hybrid(pg, dist, rank: int, world: int, groups: int, transport: str = "rccl"):
    """Both communicators of the hybrid mode: the partition group's (ranks of
    one group split every factorisation) and the speculative search's (one rank
    per group).  Every rank must call this (torch.distributed sub-groups are
    created collectively).  transport "rccl": ids made by each sub-group's
    first rank and sent over gloo; "host": gloo sub-groups as host transports
    (ranks sharing one GPU in tests).  Returns the objects to keep alive."""
    part, spec = hybrid_layout(world, groups)
    pp = world // groups
    pgroups = [dist.new_group(r) for r in part]
    sgroups = [dist.new_group(r) for r in spec]
    g, i = rank // pp, rank % pp
    keep = []
    if transport == "host":
        hp = HostComm(dist, i, pp, pgroups[g], part[g])
        pg.comm_init_host_part(hp.struct)
        hs = HostComm(dist, g, groups, sgroups[i], spec[i])
        pg.comm_init_host(hs.struct)
        keep += [hp, hs]
    else:   # partition group first, then the main communicator (pgo.h: the order binds them)
        _rccl_setup(pg, dist, [(part[g], pgroups[g], i, pp, pg.comm_init_rccl_part),
                               (spec[i], sgroups[i], g, groups, pg.comm_init_rccl)])
    return keep
