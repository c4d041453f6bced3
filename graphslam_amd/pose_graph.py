"""Native handle over libpgo.so: a device-resident pose graph.

``PoseGraph`` is the bulk, zero-copy-ish entry point (numpy arrays in, numpy
arrays out) used by the GTSAM-named mirror in ``graphslam_amd.gtsam`` and by
bench.py.  Every call goes through the C-ABI of include/pgo.h.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class PgoError(RuntimeError):
    def __init__(self, status, message):
        super().__init__(f"[{status}] {message}")
        self.status = status


class ValuesKeyAlreadyExists(PgoError, KeyError):
    """gtsam::ValuesKeyAlreadyExists (Values::insert on an existing key)."""


class ValuesKeyDoesNotExist(PgoError, KeyError):
    """gtsam::ValuesKeyDoesNotExist (Values::at / a factor on a missing key)."""


class IndeterminantLinearSystemException(PgoError):
    """gtsam::IndeterminantLinearSystemException (singular Gauss-Newton system)."""


class BadCovariance(PgoError, ValueError):
    """Covariance is not symmetric positive definite (GTSAM's LLT would fail)."""


class NotEnoughKeyframes(PgoError):
    """closest_keyframe service returning false (graph.cpp:170-171)."""


_EXC = {
    L.PGO_E_DUP_KEY: ValuesKeyAlreadyExists,
    L.PGO_E_NO_KEY: ValuesKeyDoesNotExist,
    L.PGO_E_INDETERMINANT: IndeterminantLinearSystemException,
    L.PGO_E_BAD_COV: BadCovariance,
    L.PGO_E_NOT_ENOUGH: NotEnoughKeyframes,
}

KEYFRAMES_TO_SKIP_IN_LOOP_CLOSING = 10   # graph.cpp:15


def default_params(**kw) -> L.PgoParams:
    p = L.PgoParams()
    L.lib().pgo_default_params(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(f"pgo_params has no field {k!r}")
        setattr(p, k, v)
    return p


class PoseGraph:
    """One pgo_graph handle (one HIP stream, graph + values resident in HBM)."""

    def __init__(self, device: int = 0, ordering: int = L.PGO_ORDERING_ND):
        self._L = L.lib()
        opts = L.PgoOpts()
        opts.device = device
        opts.ordering = ordering
        self._h = self._L.pgo_create(C.byref(opts))
        if not self._h:
            raise MemoryError("pgo_create failed")
        self.last_stats = None

    # ------------------------------------------------------------------ utils
    def _check(self, rc):
        if rc < 0:
            msg = self._L.pgo_last_error(self._h).decode()
            raise _EXC.get(rc, PgoError)(rc, msg)
        return rc

    def close(self):
        if getattr(self, "_h", None):
            self._L.pgo_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------ construction
    def add_vertex(self, key, x, y, theta):
        self._check(self._L.pgo_add_vertex(self._h, int(key), float(x), float(y), float(theta)))

    def add_vertices(self, keys, xyt):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
        self._check(self._L.pgo_add_vertices(self._h, len(keys), L.u64ptr(keys), L.dptr(xyt)))

    def add_prior(self, key, pose, cov):
        pose = np.ascontiguousarray(pose, dtype=np.float64).reshape(3)
        cov = np.ascontiguousarray(cov, dtype=np.float64).reshape(9)
        self._check(self._L.pgo_add_prior(self._h, int(key), L.dptr(pose), L.dptr(cov)))

    def add_edge(self, k1, k2, z, cov):
        z = np.ascontiguousarray(z, dtype=np.float64).reshape(3)
        cov = np.ascontiguousarray(cov, dtype=np.float64).reshape(9)
        self._check(self._L.pgo_add_edge(self._h, int(k1), int(k2), L.dptr(z), L.dptr(cov)))

    def add_edges(self, k1, k2, z, cov):
        k1 = np.ascontiguousarray(k1, dtype=np.uint64)
        k2 = np.ascontiguousarray(k2, dtype=np.uint64)
        z = np.ascontiguousarray(z, dtype=np.float64).reshape(-1, 3)
        cov = np.ascontiguousarray(cov, dtype=np.float64)
        stride = 0 if cov.size == 9 else 9
        if stride and cov.reshape(-1, 9).shape[0] != len(k1):
            raise ValueError("cov must be one [9] or [E,9]")
        self._check(self._L.pgo_add_edges(self._h, len(k1), L.u64ptr(k1), L.u64ptr(k2), L.dptr(z),
                                          L.dptr(cov), stride))

    @classmethod
    def from_dataset(cls, g, device=0, ordering=L.PGO_ORDERING_ND):
        """Load a graphslam_amd.datasets.PoseGraph (vertices, priors, edges)."""
        pg = cls(device, ordering)
        pg.add_vertices(g.keys, g.initial)
        for k, p, c in zip(g.prior_keys, g.prior_pose, g.prior_cov):
            pg.add_prior(int(k), p, c)
        pg.add_edges(g.edge_k1, g.edge_k2, g.edge_z, g.edge_cov)
        return pg

    # -------------------------------------------------------------- optimise
    def optimize(self, params: L.PgoParams | None = None, **kw):
        p = params if params is not None else default_params(**kw)
        st = L.PgoStats()
        rc = self._L.pgo_optimize(self._h, C.byref(p), C.byref(st))
        self.last_stats = st.as_dict()
        self._check(rc)
        return self.last_stats

    def trace(self):
        """Per-iteration record of the last optimize (pgo_get_trace): rows of
        (accepted steps, lambda, solved, model decrease, candidate error,
        fidelity, accepted, wall ms)."""
        n = self._check(self._L.pgo_get_trace(self._h, None, 0))
        out = np.zeros((n, 8))
        if n:
            self._check(self._L.pgo_get_trace(self._h, L.dptr(out), n))
        return out

    def kernel_profile(self):
        """Profiled factorisations of the last optimize (profile_every > 0):
        {family: {launches, ms, flops, bytes}} for the families that ran."""
        nf = self._check(self._L.pgo_get_kernel_profile(self._h, None, 0))
        out = np.zeros((nf, 5))
        self._check(self._L.pgo_get_kernel_profile(self._h, L.dptr(out), nf))
        res = {}
        for f in range(nf):
            if out[f, 0] > 0:
                res[self._L.pgo_kernel_family_name(f).decode()] = dict(
                    launches=int(out[f, 0]), ms=float(out[f, 1]), flops=float(out[f, 2]), bytes=float(out[f, 3]))
        return res

    def debug_partition(self, size):
        """Host-only: the PGO_MULTI_PARTITION subtree partition over `size`
        ranks: (owner per supernode, -1 = replicated top; per-rank subtree
        flops; top flops)."""
        owner, out = self._partition(size)
        return owner, out[:size].copy(), float(out[size])

    def _partition(self, size):
        ns = self._check(self._L.pgo_debug_partition(self._h, int(size), None, None, 0))
        cap = max(ns, 2 * size + 4)
        owner = np.zeros(cap, np.int32)
        out = np.zeros(cap)
        self._check(self._L.pgo_debug_partition(self._h, int(size), owner.ctypes.data_as(C.POINTER(C.c_int)),
                                                L.dptr(out), cap))
        return owner[:ns], out

    def debug_partition_bound(self, size):
        """Host-only: the partitioned factorisation's per-rank flops with the
        distributed top (top fronts' columns dealt to the ranks), the work every
        rank repeats, and the plan-derived flop bound on the speed-up
        (factorisation flops / the busiest rank's)."""
        _, out = self._partition(size)
        total = self.debug_plan()["factor_flops"]
        rank = out[size + 1:2 * size + 1].copy()
        return {"ranks": int(size), "rank_flops": rank, "replicated_flops": float(out[2 * size + 1]),
                "replicated_top_flops": float(out[size]), "total_flops": float(total),
                "bound": float(total / rank.max()),
                "bound_replicated_top": float(total / (out[size] + out[:size].max())),
                "exchange_points": int(out[2 * size + 2]), "exchange_bytes": float(8.0 * out[2 * size + 3])}

    def debug_ordering(self):
        """Host-only: the Cholesky solver's pose ordering (new -> insertion index)."""
        n = self.num_vertices
        perm = np.zeros(n, np.int32)
        self._check(self._L.pgo_debug_ordering(self._h, perm.ctypes.data_as(C.POINTER(C.c_int32)), n))
        return perm

    # ---------------------------------------------------------------- values
    @property
    def num_vertices(self):
        return int(self._L.pgo_num_vertices(self._h))

    @property
    def num_factors(self):
        return int(self._L.pgo_num_factors(self._h))

    def pose(self, key):
        out = np.zeros(3)
        self._check(self._L.pgo_get_pose(self._h, int(key), L.dptr(out)))
        return out

    def poses(self, keys=None):
        if keys is None:
            n = self.num_vertices
            out = np.zeros((n, 3))
            self._check(self._L.pgo_get_poses(self._h, n, None, L.dptr(out)))
            return out
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros((len(keys), 3))
        self._check(self._L.pgo_get_poses(self._h, len(keys), L.u64ptr(keys), L.dptr(out)))
        return out

    def marginal_covariances(self, keys):
        """3x3 covariances (x, y, theta) of the poses at the current values:
        gtsam::Marginals(graph, values).marginalCovariance(key) (graph.cpp:120,126-127)."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), dtype=np.uint64)
        out = np.zeros((len(keys), 3, 3))
        self._check(self._L.pgo_marginal_covariances(self._h, len(keys), L.u64ptr(keys), L.dptr(out)))
        return out

    def set_poses(self, xyt, keys=None):
        xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
        kp = None
        if keys is not None:
            keys = np.ascontiguousarray(keys, dtype=np.uint64)
            kp = L.u64ptr(keys)
        self._check(self._L.pgo_set_poses(self._h, xyt.shape[0], kp, L.dptr(xyt)))

    def save_values(self):
        self._check(self._L.pgo_save_values(self._h))

    def restore_values(self):
        self._check(self._L.pgo_restore_values(self._h))

    def error(self):
        e = C.c_double(0)
        self._check(self._L.pgo_error(self._h, C.byref(e)))
        return e.value

    # ------------------------------------------------------------ diagnostics
    # ------------------------------------------------- loop-closure search
    def closest_keyframe(self, x, y, skip=KEYFRAMES_TO_SKIP_IN_LOOP_CLOSING):
        """closest_keyframe service (graph.cpp:146-178): (key, distance) of the
        vertex nearest to (x, y) among all but the last `skip` inserted."""
        key, dist = C.c_uint64(), C.c_double()
        self._check(self._L.pgo_closest_keyframe(self._h, float(x), float(y), int(skip), C.byref(key),
                                                 C.byref(dist)))
        return key.value, dist.value

    def closest_keyframes(self, query_keys, skip=KEYFRAMES_TO_SKIP_IN_LOOP_CLOSING):
        """Batched service: for each query key, the answer when it was the last
        keyframe (candidates inserted before it, minus skip - 1).  Keys with no
        candidate get PGO_NO_KEY and +inf."""
        q = np.ascontiguousarray(query_keys, dtype=np.uint64)
        keys = np.zeros(len(q), np.uint64)
        dist = np.zeros(len(q))
        self._check(self._L.pgo_closest_keyframes(self._h, len(q), L.u64ptr(q), int(skip), L.u64ptr(keys),
                                                  L.dptr(dist)))
        return keys, dist

    def debug_search_ms(self):
        a, b = C.c_double(), C.c_double()
        self._check(self._L.pgo_debug_search_ms(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    # ------------------------------------------------- multi-GPU (pgo_comm_*)
    def comm_init_rccl(self, unique_id: bytes, rank: int, size: int):
        """ncclCommInitRank on this handle's device (collective over all ranks)."""
        buf = C.create_string_buffer(bytes(unique_id), len(unique_id))
        self._check(self._L.pgo_comm_init_rccl(self._h, buf, len(unique_id), rank, size))

    def comm_init_host(self, comm: L.PgoHostComm):
        """The caller's own host transport (callbacks must outlive the handle's use)."""
        self._comm_keepalive = comm
        self._check(self._L.pgo_comm_init_host(self._h, C.byref(comm)))

    def comm_init_rccl_part(self, unique_id: bytes, rank: int, size: int):
        """The hybrid mode's partition-group communicator over RCCL (collective over the group)."""
        buf = C.create_string_buffer(bytes(unique_id), len(unique_id))
        self._check(self._L.pgo_comm_init_rccl_part(self._h, buf, len(unique_id), rank, size))

    def comm_init_host_part(self, comm: L.PgoHostComm):
        """The hybrid mode's partition-group communicator over the caller's host transport."""
        self._pcomm_keepalive = comm
        self._check(self._L.pgo_comm_init_host_part(self._h, C.byref(comm)))

    def comm_part_rank(self):
        r, n = C.c_int(), C.c_int()
        self._check(self._L.pgo_comm_part_rank(self._h, C.byref(r), C.byref(n)))
        return r.value, n.value

    def comm_free(self):
        self._check(self._L.pgo_comm_free(self._h))

    def comm_rank(self):
        r, n = C.c_int(), C.c_int()
        self._check(self._L.pgo_comm_rank(self._h, C.byref(r), C.byref(n)))
        return r.value, n.value

    def comm_selftest(self):
        self._check(self._L.pgo_comm_selftest(self._h))

    def debug_linearize(self, num_edges, cholesky=False):
        """H diagonal / off-diagonal blocks, gradient and error at the current
        values; cholesky=True takes the Cholesky-mode sweep (owner blocks in
        factor order) instead of the two-slot block-CSR sweep."""
        n = self.num_vertices
        hd = np.zeros((n, 3, 3))
        ho = np.zeros((num_edges, 3, 3))
        g = np.zeros((n, 3))
        e = C.c_double(0)
        fn = self._L.pgo_debug_linearize_cholesky if cholesky else self._L.pgo_debug_linearize
        self._check(fn(self._h, L.dptr(hd), L.dptr(ho), L.dptr(g), C.byref(e)))
        return hd, ho, g, e.value

    def debug_poison_fronts(self):
        """NaN into the Cholesky workspace's written-before-read elements (tests)."""
        self._check(self._L.pgo_debug_poison_fronts(self._h))

    def debug_factor_time(self, lanes=1, reps=10):
        """Device ms of one replay of the captured factorisation graph with
        `lanes` lambda lanes (diagnostics; PGO_ABLATE applies)."""
        ms = C.c_double(0)
        self._check(self._L.pgo_debug_factor_time(self._h, int(lanes), int(reps), C.byref(ms)))
        return ms.value

    def debug_spmv(self, x, lam=0.0):
        x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, 3)
        y = np.zeros_like(x)
        self._check(self._L.pgo_debug_spmv(self._h, float(lam), L.dptr(x), L.dptr(y)))
        return y

    def debug_plan(self, cap=4096):
        """Host-only symbolic analysis summary of the supernodal Cholesky plan."""
        out = np.zeros(cap)
        self._check(self._L.pgo_debug_plan(self._h, L.dptr(out), cap))
        keys = ["supernodes", "levels", "nnz_l", "factor_flops", "syrk_flops", "front_doubles",
                "launches_factor", "launches_solve", "max_front", "trsm_tasks", "syrk_tiles", "small_fronts"]
        summary = {k: out[i] for i, k in enumerate(keys)}
        nl = int(out[1])
        lv = out[16:16 + 6 * nl].reshape(-1, 6)
        summary["levels_table"] = lv
        return summary

    def debug_fronts(self):
        """Host-only: (w, m, level) of every supernode of the Cholesky plan."""
        ns = self._L.pgo_debug_fronts(self._h, None, None, None, 0)
        if ns < 0:
            self._check(ns)
        w = np.zeros(ns, np.int32)
        m = np.zeros(ns, np.int32)
        lv = np.zeros(ns, np.int32)
        ip = C.POINTER(C.c_int)
        self._check(min(0, self._L.pgo_debug_fronts(self._h, w.ctypes.data_as(ip), m.ctypes.data_as(ip),
                                                     lv.ctypes.data_as(ip), ns)))
        return w, m, lv

    def debug_parents(self):
        """Host-only: the parent supernode of every supernode (-1: a root)."""
        ns = self._L.pgo_debug_fronts(self._h, None, None, None, 0)
        if ns < 0:
            self._check(ns)
        par = np.zeros(ns, np.int32)
        self._check(min(0, self._L.pgo_debug_parents(self._h, par.ctypes.data_as(C.POINTER(C.c_int)), ns)))
        return par

    def debug_solve(self, lam, params=None, **kw):
        p = params if params is not None else default_params(**kw)
        d = np.zeros((self.num_vertices, 3))
        it = C.c_int(0)
        self._check(self._L.pgo_debug_solve(self._h, float(lam), C.byref(p), L.dptr(d), C.byref(it)))
        return d, it.value
