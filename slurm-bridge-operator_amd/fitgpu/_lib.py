"""ctypes binding of libfitgpu.so (the C-ABI in include/fitgpu.h).

This is the Python twin of the cgo binding shown in INTEGRATION.md; it only marshals pointers.
Loading fails loudly when the library is missing — there is no fallback implementation.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FITGPU_LIB: an alternative in-tree build of the same library (diagnostic / variant builds)
LIB_PATH = os.environ.get("FITGPU_LIB") or os.path.join(_HERE, "libfitgpu.so")

FIT_OK = 0
FIT_E_INVAL = -1
FIT_E_HIP = -2
FIT_E_RCCL = -3
FIT_E_OOM = -4
FIT_E_NODEV = -5
FIT_E_STATE = -6
FIT_E_PARSE = -7
FIT_E_UNLIMITED = -8
FIT_UNPLACED = -1
FIT_REJECTED = -2

# every symbol include/fitgpu.h declares (tests/test_abi.py checks the header agrees)
EXPORTS = [
    "fit_create", "fit_destroy", "fit_abi_version", "fit_strerror", "fit_last_error",
    "fit_nccl_unique_id", "fit_load_nodes", "fit_load_nodes_device", "fit_load_partitions",
    "fit_place", "fit_place_device", "fit_read_nodes", "fit_partition_free",
    "fit_parse_duration", "fit_parse_resources", "fit_parse_nodes", "fit_parse_partition",
    "fit_parse_partitions_names", "fit_extract_batch_resources", "fit_apply_spec", "fit_array_len",
    "fit_pod_request", "fit_job_demand", "fit_partition_capacity",
    "fit_load_timeline", "fit_load_timeline_device", "fit_place_tl", "fit_place_tl_device",
    "fit_read_timeline", "fit_ingest_nodes", "fit_expand_hostlist",
    "fit_admitter_create", "fit_admit", "fit_admit_group", "fit_admitter_load_nodes",
    "fit_admitter_partition_free", "fit_admitter_confirm", "fit_admitter_release", "fit_admitter_set_ttl",
    "fit_admitter_reservations", "fit_admitter_pending", "fit_admitter_destroy",
    "fit_array_tasks", "fit_pod_demand", "fit_script_with_nodelist", "fit_partition_limits",
    "fit_node_columns", "fit_node_names", "fit_admitter_load_table", "fit_admitter_generation",
    "fit_admitter_script", "fit_set_max_array_size", "fit_release_events", "fit_set_watchdog_us",
    "fit_lock_dir",
]


XCHG_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int64)
FIT_XCHG_ALLGATHER_U64, FIT_XCHG_MIN_U64, FIT_XCHG_MAX_I32, FIT_XCHG_MIN_I32 = 1, 2, 3, 4
FIT_SHARD_AUTO, FIT_SHARD_NODES, FIT_SHARD_COMPONENTS = 0, 1, 2
FIT_FLAG_COLLECTIVES = 1  # fit_opts.flags: multi-rank code path at world 1 (include/fitgpu.h)


class FitOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("rank", C.c_int32), ("world", C.c_int32),
                ("nccl_id", C.c_void_p), ("shard_mode", C.c_int32), ("window_min", C.c_int32),
                ("window_max", C.c_int32), ("flags", C.c_int32), ("exchange", XCHG_FN),
                ("exchange_user", C.c_void_p)]


class FitStats(C.Structure):
    _fields_ = [("jobs", C.c_int64), ("placed", C.c_int64), ("unplaced", C.c_int64),
                ("rejected", C.c_int64), ("rounds", C.c_int64), ("evals", C.c_int64),
                ("useful_evals", C.c_int64), ("stops_rescan", C.c_int64),
                ("stops_dirty", C.c_int64), ("ms_total", C.c_double), ("ms_scan", C.c_double),
                ("ms_commit", C.c_double), ("ms_exchange", C.c_double), ("ms_device", C.c_double),
                ("shard_mode", C.c_int32),
                ("components", C.c_int32), ("engine", C.c_int32), ("reserved", C.c_int32),
                ("ms_arb_wait", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


FIT_MAX_K = 8


class FitAdmitReq(C.Structure):
    _fields_ = [("priority", C.c_int64), ("cpu", C.c_int32), ("mem_mib", C.c_int32),
                ("gpu", C.c_int32), ("wall_min", C.c_int32), ("part", C.c_uint16),
                ("nodes_k", C.c_uint16), ("flags", C.c_uint16), ("reserved", C.c_uint16)]


FIT_REQ_ARRAY = 1  # fit_admit_req.flags: a task of an array job (never pinned)


class FitAdmitRes(C.Structure):
    _fields_ = [("node", C.c_int32 * FIT_MAX_K), ("batch", C.c_int64), ("batch_jobs", C.c_int32),
                ("order", C.c_int32), ("ticket", C.c_int64)]


FIT_TABLE_STATE = 1  # fit_node_table.flags: part_mask carries node State (include/fitgpu.h)
FIT_TABLE_PIN = 2    # pin placements on a table without State (the operator's choice)


class FitNodeTable(C.Structure):
    _fields_ = [("n", C.c_int32), ("cpu_free", C.c_void_p), ("mem_free", C.c_void_p), ("gpu_free", C.c_void_p),
                ("avail_min", C.c_void_p), ("part_mask", C.c_void_p), ("names", C.c_char_p), ("flags", C.c_int32),
                ("generation", C.c_int64)]


class FitPodLabels(C.Structure):
    _fields_ = [(n, C.c_char_p) for n in ("nodes", "cpus_per_task", "mem_per_cpu", "ntasks_per_node", "array",
                                          "ntasks")]


class FitResources(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("mem_per_node", C.c_int64), ("cpu_per_node", C.c_int64),
                ("wall_ns", C.c_int64)]


class FitNode(C.Structure):
    _fields_ = [("cpus", C.c_int64), ("memory", C.c_int64), ("gpus", C.c_int64),
                ("allo_cpus", C.c_int64), ("allo_memory", C.c_int64), ("allo_gpus", C.c_int64)]


class FitJobResources(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("cpus_per_task", C.c_int64), ("ntasks", C.c_int64),
                ("ntasks_per_node", C.c_int64), ("mem_per_cpu", C.c_int64), ("wall_ns", C.c_int64),
                ("array", C.c_char * 64)]


_lib = None


def lib() -> C.CDLL:
    """Load libfitgpu.so (built by __graft_entry__.build() / `make`); raise if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C slurm-bridge-operator_amd`")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        i32, i64, u16p = C.c_int32, C.c_int64, C.POINTER(C.c_uint16)
        L.fit_strerror.restype = C.c_char_p
        L.fit_strerror.argtypes = [C.c_int]
        L.fit_last_error.restype = C.c_char_p
        L.fit_create.argtypes = [C.POINTER(FitOpts), C.POINTER(P)]
        L.fit_destroy.argtypes = [P]
        L.fit_destroy.restype = None
        L.fit_nccl_unique_id.argtypes = [P]
        if hasattr(L, "fit_set_watchdog_us"):  # (absent from pre-round-5 variant builds, FITGPU_LIB)
            L.fit_set_watchdog_us.argtypes = [P, i64]
        if hasattr(L, "fit_lock_dir"):  # (absent from pre-round-6 variant builds, FITGPU_LIB)
            L.fit_lock_dir.argtypes = [C.c_char_p, i32]
        for name in ("fit_load_nodes", "fit_load_nodes_device"):
            getattr(L, name).argtypes = [P, i32, P, P, P, P, P]
        L.fit_load_partitions.argtypes = [P, i32, P, P, P]
        for name in ("fit_place", "fit_place_device"):
            getattr(L, name).argtypes = [P, i32, P, P, P, P, P, P, i32, P, C.POINTER(FitStats)]
        L.fit_read_nodes.argtypes = [P, P, P, P]
        L.fit_load_timeline.argtypes = [P, i32, i32, P, P, P, P, P]
        L.fit_load_timeline_device.argtypes = [P, i32, i32, P, i64, P, P, P, P]
        for name in ("fit_place_tl", "fit_place_tl_device"):
            getattr(L, name).argtypes = [P, i32, P, P, P, P, P, P, P, C.POINTER(FitStats)]
        L.fit_read_timeline.argtypes = [P, P, P, P]
        L.fit_ingest_nodes.argtypes = [C.c_char_p, C.c_char_p, i32, i32, P, P, P, P, P, C.c_char_p, i32]
        L.fit_expand_hostlist.argtypes = [C.c_char_p, C.c_char_p, i32]
        L.fit_partition_free.argtypes = [P, i32, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
        L.fit_admitter_create.argtypes = [P, i32, i32, C.POINTER(P)]
        L.fit_admit.argtypes = [P, C.POINTER(FitAdmitReq), C.POINTER(FitAdmitRes)]
        L.fit_admitter_load_nodes.argtypes = [P, i32, P, P, P, P, P]
        L.fit_admitter_partition_free.argtypes = [P, i32, C.POINTER(i64), C.POINTER(i64),
                                                  C.POINTER(i64)]
        L.fit_admit_group.argtypes = [P, C.POINTER(FitAdmitReq), i32, C.POINTER(FitAdmitRes)]
        for name in ("fit_admitter_confirm", "fit_admitter_release"):
            getattr(L, name).argtypes = [P, i64]
        L.fit_admitter_set_ttl.argtypes = [P, i32]
        L.fit_admitter_reservations.argtypes = [P]
        L.fit_admitter_pending.argtypes = [P]
        L.fit_admitter_destroy.argtypes = [P]
        L.fit_admitter_destroy.restype = None
        L.fit_array_tasks.argtypes = [C.c_char_p, C.POINTER(i64), C.POINTER(i64)]
        L.fit_pod_demand.argtypes = [C.POINTER(FitPodLabels), C.c_char_p, C.c_uint16, i64, C.POINTER(FitAdmitReq),
                                     i32]
        L.fit_script_with_nodelist.argtypes = [C.c_char_p, C.c_char_p, i32, C.POINTER(i32), i32, C.c_char_p, i32]
        L.fit_partition_limits.argtypes = [i64, i64, i64, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
        L.fit_node_columns.argtypes = [C.POINTER(FitNode), i32, C.c_uint32, P, P, P, P, P]
        L.fit_node_names.argtypes = [C.c_char_p, i32, C.c_char_p, i32]
        L.fit_admitter_load_table.argtypes = [P, C.POINTER(FitNodeTable)]
        L.fit_admitter_generation.argtypes = [P]
        L.fit_admitter_generation.restype = i64
        L.fit_admitter_script.argtypes = [P, C.POINTER(i64), i32, C.c_char_p, C.c_char_p, i32, C.POINTER(i32)]
        L.fit_set_max_array_size.argtypes = [i32]
        L.fit_set_max_array_size.restype = i32
        L.fit_release_events.argtypes = [i32, i32, P, P, P, P, P, P, i32, i32, P, P, P, P, P, i32]
        L.fit_parse_duration.argtypes = [C.c_char_p, C.POINTER(i64)]
        L.fit_parse_resources.argtypes = [C.c_char_p, C.POINTER(FitResources)]
        L.fit_parse_nodes.argtypes = [C.c_char_p, C.POINTER(FitNode), i32]
        L.fit_parse_partition.argtypes = [C.c_char_p, C.c_char_p, i32]
        L.fit_parse_partitions_names.argtypes = [C.c_char_p, C.c_char_p, i32]
        L.fit_extract_batch_resources.argtypes = [C.c_char_p, C.POINTER(FitJobResources)]
        L.fit_apply_spec.argtypes = [C.POINTER(FitJobResources), i64, i64, i64, i64, C.c_char_p, i64]
        L.fit_apply_spec.restype = None
        L.fit_array_len.argtypes = [C.c_char_p]
        L.fit_array_len.restype = i64
        L.fit_pod_request.argtypes = [C.POINTER(FitJobResources), C.POINTER(i64), C.POINTER(i64)]
        L.fit_pod_request.restype = None
        L.fit_job_demand.argtypes = [C.POINTER(FitJobResources), C.POINTER(i32), C.POINTER(i32),
                                     C.POINTER(i32), u16p]
        L.fit_partition_capacity.argtypes = [C.POINTER(FitNode), i32, C.POINTER(i64),
                                             C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
        L.fit_partition_capacity.restype = None
        _lib = L
    return _lib


class FitError(RuntimeError):
    def __init__(self, code: int, where: str):
        L = lib()
        msg = L.fit_strerror(code).decode()
        detail = (L.fit_last_error() or b"").decode()
        super().__init__(f"{where}: {msg} ({code}): {detail}")
        self.code = code


def check(rc: int, where: str) -> int:
    if rc < 0:
        raise FitError(rc, where)
    return rc
