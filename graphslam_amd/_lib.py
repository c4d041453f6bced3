"""ctypes binding of libpgo.so (include/pgo.h).

The library is built in-tree (graphslam_amd/libpgo.so, see csrc/Makefile).
There is no fallback: if the HIP library is missing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PGO_LIB_PATH") or os.path.join(HERE, "libpgo.so")   # override: A/B builds
HEADER = os.path.join(os.path.dirname(HERE), "include", "pgo.h")

PGO_OK = 0
PGO_E_ARG = -1
PGO_E_DUP_KEY = -2
PGO_E_NO_KEY = -3
PGO_E_BAD_COV = -4
PGO_E_INDETERMINANT = -5
PGO_E_NONFINITE = -6
PGO_E_HIP = -7
PGO_E_NO_DEVICE = -8
PGO_E_NOMEM = -9
PGO_E_BAD_EDGE = -10
PGO_E_COMM = -11
PGO_E_NOT_ENOUGH = -12
PGO_NO_KEY = (1 << 64) - 1
PGO_W_MAXITER = 1
PGO_ORDERING_ND = 0
PGO_ORDERING_AMD = 1
PGO_ALG_LM = 0
PGO_ALG_GN = 1
PGO_SOLVER_PCG = 0
PGO_SOLVER_CHOLESKY = 1
PGO_MULTI_SPECULATIVE = 0
PGO_MULTI_PARTITION = 1
PGO_MULTI_HYBRID = 2
PGO_TRANSPORT_NONE = 0
PGO_TRANSPORT_RCCL = 1
PGO_TRANSPORT_HOST = 2
TRANSPORTS = {0: "none", 1: "rccl", 2: "host"}
ABI_VERSION = 6
STOP_REASONS = {0: "converged", 1: "lambda_upper_bound", 2: "max_iterations", 3: "max_outer", 4: "small_cost_change",
                5: "error"}


class PgoOpts(C.Structure):
    _fields_ = [("device", C.c_int), ("ordering", C.c_int), ("reserved", C.c_int * 6)]


class PgoParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int), ("relative_error_tol", C.c_double),
                ("absolute_error_tol", C.c_double), ("error_tol", C.c_double),
                ("lambda_initial", C.c_double), ("lambda_factor", C.c_double),
                ("lambda_upper_bound", C.c_double), ("lambda_lower_bound", C.c_double),
                ("min_model_fidelity", C.c_double), ("use_fixed_lambda_factor", C.c_int),
                ("algorithm", C.c_int), ("linear_solver", C.c_int), ("pcg_relative_tol", C.c_double),
                ("pcg_max_iterations", C.c_int), ("pcg_check_interval", C.c_int), ("max_outer", C.c_int),
                ("profile_every", C.c_int), ("use_graphs", C.c_int), ("lambda_lanes", C.c_int),
                ("multi_gpu", C.c_int)]


class PgoStats(C.Structure):
    _fields_ = [("status", C.c_int), ("iterations", C.c_int), ("inner_iterations", C.c_int),
                ("linearizations", C.c_int), ("initial_error", C.c_double), ("final_error", C.c_double),
                ("pcg_iterations", C.c_longlong), ("ms_total", C.c_double), ("ms_upload", C.c_double),
                ("ms_linearize", C.c_double), ("ms_solve", C.c_double), ("ms_update", C.c_double),
                ("kernel_spmv_ms", C.c_double), ("kernel_spmv_count", C.c_longlong),
                ("kernel_linearize_ms", C.c_double), ("kernel_linearize_count", C.c_longlong),
                ("kernel_syrk_ms", C.c_double), ("kernel_syrk_count", C.c_longlong),
                ("syrk_flops", C.c_double), ("factor_flops", C.c_double),
                ("kernel_syrk_launches", C.c_longlong), ("lambda_rounds", C.c_int), ("ranks", C.c_int),
                ("solves", C.c_longlong), ("ms_comm", C.c_double),
                ("ms_factor_profiled", C.c_double), ("ms_solve_profiled", C.c_double), ("stop_reason", C.c_int),
                ("ms_factor_graph", C.c_double), ("factor_graph_flops", C.c_double),
                ("plan_update", C.c_int), ("ms_plan", C.c_double), ("upload_kind", C.c_int),
                ("handoff_retries", C.c_int), ("transport", C.c_int), ("part_transport", C.c_int)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
BROADCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int)


class PgoHostComm(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("rank", C.c_int), ("size", C.c_int),
                ("allgather", ALLGATHER_FN), ("broadcast", BROADCAST_FN)]


class PgoGicpParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int), ("k_correspondences", C.c_int), ("gicp_epsilon", C.c_double),
                ("max_correspondence_distance", C.c_double), ("transformation_epsilon", C.c_double),
                ("rotation_epsilon", C.c_double), ("max_inner_iterations", C.c_int)]


class PgoGicpResult(C.Structure):
    _fields_ = [("T", C.c_double * 16), ("converged", C.c_int), ("iterations", C.c_int),
                ("fitness", C.c_double), ("delta", C.c_double * 3), ("cov", C.c_double * 9),
                ("keyframe", C.c_int), ("inner_iterations", C.c_int)]



def build():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "csrc")], check=True)


def declared_symbols():
    """Every function name include/pgo.h declares."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pgo_[a-z_0-9]+)\s*\(", text)))


_lib = None


def lib():
    """Load libpgo.so; raise (never fall back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libpgo.so not built at {LIB_PATH}: run `make -C graphslam_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, dp, u64p = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)
    sig = {
        "pgo_create": (vp, [C.POINTER(PgoOpts)]),
        "pgo_destroy": (None, [vp]),
        "pgo_last_error": (C.c_char_p, [vp]),
        "pgo_status_string": (C.c_char_p, [C.c_int]),
        "pgo_abi_version": (C.c_int, []),
        "pgo_default_params": (None, [C.POINTER(PgoParams)]),
        "pgo_add_vertex": (C.c_int, [vp, C.c_uint64, C.c_double, C.c_double, C.c_double]),
        "pgo_add_vertices": (C.c_int, [vp, C.c_size_t, u64p, dp]),
        "pgo_add_prior": (C.c_int, [vp, C.c_uint64, dp, dp]),
        "pgo_add_edge": (C.c_int, [vp, C.c_uint64, C.c_uint64, dp, dp]),
        "pgo_add_edges": (C.c_int, [vp, C.c_size_t, u64p, u64p, dp, dp, C.c_int]),
        "pgo_optimize": (C.c_int, [vp, C.POINTER(PgoParams), C.POINTER(PgoStats)]),
        "pgo_get_pose": (C.c_int, [vp, C.c_uint64, dp]),
        "pgo_get_poses": (C.c_int, [vp, C.c_size_t, u64p, dp]),
        "pgo_set_poses": (C.c_int, [vp, C.c_size_t, u64p, dp]),
        "pgo_save_values": (C.c_int, [vp]),
        "pgo_restore_values": (C.c_int, [vp]),
        "pgo_num_factors": (C.c_size_t, [vp]),
        "pgo_num_vertices": (C.c_size_t, [vp]),
        "pgo_error": (C.c_int, [vp, dp]),
        "pgo_debug_linearize": (C.c_int, [vp, dp, dp, dp, dp]),
        "pgo_debug_linearize_cholesky": (C.c_int, [vp, dp, dp, dp, dp]),
        "pgo_debug_spmv": (C.c_int, [vp, C.c_double, dp, dp]),
        "pgo_debug_solve": (C.c_int, [vp, C.c_double, C.POINTER(PgoParams), dp, C.POINTER(C.c_int)]),
        "pgo_debug_factor_time": (C.c_int, [vp, C.c_int, C.c_int, dp]),
        "pgo_debug_poison_fronts": (C.c_int, [vp]),
        "pgo_debug_plan": (C.c_int, [vp, dp, C.c_int]),
        "pgo_marginal_covariances": (C.c_int, [vp, C.c_size_t, C.POINTER(C.c_uint64), dp]),
        "pgo_debug_fronts": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int]),
        "pgo_closest_keyframe": (C.c_int, [vp, C.c_double, C.c_double, C.c_int, u64p, dp]),
        "pgo_closest_keyframes": (C.c_int, [vp, C.c_size_t, u64p, C.c_int, u64p, dp]),
        "pgo_debug_search_ms": (C.c_int, [vp, dp, dp]),
        "pgo_comm_unique_id": (C.c_int, [vp, C.c_size_t]),
        "pgo_comm_init_rccl": (C.c_int, [vp, vp, C.c_size_t, C.c_int, C.c_int]),
        "pgo_comm_init_host": (C.c_int, [vp, C.POINTER(PgoHostComm)]),
        "pgo_comm_free": (C.c_int, [vp]),
        "pgo_comm_rank": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "pgo_comm_init_rccl_part": (C.c_int, [vp, vp, C.c_size_t, C.c_int, C.c_int]),
        "pgo_comm_init_host_part": (C.c_int, [vp, C.POINTER(PgoHostComm)]),
        "pgo_comm_part_rank": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "pgo_comm_selftest": (C.c_int, [vp]),
        "pgo_get_trace": (C.c_int, [vp, dp, C.c_int]),
        "pgo_get_kernel_profile": (C.c_int, [vp, dp, C.c_int]),
        "pgo_kernel_family_name": (C.c_char_p, [C.c_int]),
        "pgo_debug_ordering": (C.c_int, [vp, C.POINTER(C.c_int32), C.c_size_t]),
        "pgo_debug_partition": (C.c_int, [vp, C.c_int, C.POINTER(C.c_int), dp, C.c_int]),
        "pgo_debug_parents": (C.c_int, [vp, C.POINTER(C.c_int), C.c_int]),
        "pgo_gicp_default_params": (None, [C.POINTER(PgoGicpParams)]),
        "pgo_gicp_create": (vp, [C.c_int]),
        "pgo_gicp_destroy": (None, [vp]),
        "pgo_gicp_last_error": (C.c_char_p, [vp]),
        "pgo_gicp_align_batch": (C.c_int, [vp, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int),
                                           C.POINTER(C.c_float), C.POINTER(C.c_int), dp,
                                           C.POINTER(PgoGicpParams), C.POINTER(PgoGicpResult)]),
        "pgo_gicp_debug_ms": (C.c_int, [vp, dp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.pgo_abi_version() != ABI_VERSION:
        raise RuntimeError("libpgo.so ABI version mismatch")
    _lib = L
    return L


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def u64ptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint64)) if a is not None else None
