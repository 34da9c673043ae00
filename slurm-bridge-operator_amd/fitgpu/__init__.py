"""fitgpu — MI355X-native batched job→node placement for slurm-bridge-operator.

Python face of libfitgpu.so (C-ABI: include/fitgpu.h).  The names mirror the reference's Go
functions on the resource-fit path so the tests read like the reference's own:

    ParseDuration                 pkg/slurm-agent/parse.go:36-109
    parse_resources               parse.go:111-190          (parseResources)
    parse_nodes                   slurm.go:343-364 + parse.go:291-308 (Client.Nodes/parseNode)
    parse_partition               parse.go:278-289          (parsePartition)
    parse_partitions_names        parse.go:192-210          (parsePartitionsNames)
    extract_batch_resources       pkg/slurm-bridge-operator/parse.go:30-69
    apply_spec                    pod.go:70-107             (setRequireResourceBySpec + defaults)
    parse_array_len               parse.go:126-135          (parseArrayLen)
    gen_resource_list_for_pod     pod.go:143-162            (genResourceListForPod)
    get_partition_capacity        pkg/slurm-virtual-kubelet/node.go:169-199
    Engine.place                  the fit decision the reference leaves to kube-scheduler/slurmctld

Every compute call goes through the HIP library; nothing here computes a placement.
"""
from __future__ import annotations

import ctypes as C
import threading
import weakref
from dataclasses import dataclass

import numpy as np

from ._lib import (FIT_E_PARSE, FIT_E_STATE, FIT_FLAG_COLLECTIVES, FIT_E_UNLIMITED, FIT_REJECTED, FIT_REQ_ARRAY,
                   FIT_SHARD_AUTO,
                   FIT_SHARD_COMPONENTS, FIT_SHARD_NODES, FIT_TABLE_PIN, FIT_TABLE_STATE, FIT_UNPLACED, FIT_XCHG_ALLGATHER_U64,
                   FIT_XCHG_MAX_I32, FIT_XCHG_MIN_I32, FIT_XCHG_MIN_U64, XCHG_FN, FitAdmitReq, FitAdmitRes, FitError,
                   FitJobResources, FitNode, FitNodeTable, FitOpts, FitPodLabels, FitResources, FitStats, check, lib)

__all__ = [
    "Engine", "FitError", "ErrDurationIsUnlimited", "ParseDuration", "parse_resources", "parse_nodes",
    "parse_partition", "parse_partitions_names", "extract_batch_resources", "apply_spec",
    "parse_array_len", "gen_resource_list_for_pod", "job_demand", "get_partition_capacity",
    "FIT_UNPLACED", "FIT_REJECTED", "Resources", "Node", "JobResources", "TorchHostExchange",
    "FIT_SHARD_AUTO", "FIT_SHARD_NODES", "FIT_SHARD_COMPONENTS", "expand_hostlist", "ingest_nodes",
    "FIT_FLAG_COLLECTIVES", "Admitter", "array_tasks", "pod_demand", "script_with_nodelist",
    "partition_limits", "node_columns", "POD_LABEL_KEYS", "node_names", "set_max_array_size", "FIT_TABLE_STATE",
    "FIT_TABLE_PIN",
]


class ErrDurationIsUnlimited(Exception):
    """pkg/slurm-agent/slurm.go:49 — the duration field has value UNLIMITED (or is empty)."""


def _ptr(a) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data) if isinstance(a, np.ndarray) else C.c_void_p(a.data_ptr())


# ------------------------------------------------------------------------------- ingest
def ParseDuration(s: str) -> int:
    """Duration in nanoseconds; raises ErrDurationIsUnlimited / ValueError like the Go errors."""
    ns = C.c_int64()
    rc = lib().fit_parse_duration(s.encode(), C.byref(ns))
    if rc == FIT_E_UNLIMITED:
        raise ErrDurationIsUnlimited(s)
    if rc == FIT_E_PARSE:
        raise ValueError(f"invalid duration {s!r}")
    check(rc, "fit_parse_duration")
    return ns.value


@dataclass
class Resources:  # pkg/slurm-agent/slurm.go:104-110 (Features unused on this path)
    Nodes: int
    MemPerNode: int
    CPUPerNode: int
    WallTime: int  # ns, -1 = UNLIMITED


def parse_resources(text: str) -> Resources:
    r = FitResources()
    rc = lib().fit_parse_resources(text.encode(), C.byref(r))
    if rc == FIT_E_PARSE:
        raise ValueError("could not parse partition resources")
    check(rc, "fit_parse_resources")
    return Resources(r.nodes, r.mem_per_node, r.cpu_per_node, r.wall_ns)


@dataclass
class Node:  # pkg/slurm-agent/slurm.go:113-121
    Cpus: int
    Memory: int
    Gpus: int
    AlloCpus: int
    AlloMemory: int
    AlloGpus: int


def parse_nodes(text: str, cap: int | None = None) -> list[Node]:
    cap = cap if cap is not None else text.count("\n\n") + 2
    arr = (FitNode * max(cap, 1))()
    n = check(lib().fit_parse_nodes(text.encode(), arr, cap), "fit_parse_nodes")
    return [Node(a.cpus, a.memory, a.gpus, a.allo_cpus, a.allo_memory, a.allo_gpus) for a in arr[:n]]


def _names(fn, text: str) -> list[str]:
    buflen = len(text.encode()) * 2 + 64
    buf = C.create_string_buffer(buflen)
    n = check(fn(text.encode(), buf, buflen), fn.__name__)
    return [s.decode() for s in buf.raw.split(b"\0")[:n]]


def parse_partition(text: str) -> list[str]:
    return _names(lib().fit_parse_partition, text)


def parse_partitions_names(text: str) -> list[str]:
    return _names(lib().fit_parse_partitions_names, text)


def expand_hostlist(expr: str) -> list[str]:
    """Slurm hostlist expansion (fixes parsePartition's split, parse.go:278-289)."""
    buflen = 1 << 16
    while True:
        buf = C.create_string_buffer(buflen)
        n = lib().fit_expand_hostlist(expr.encode(), buf, buflen)
        if n == FIT_E_PARSE:
            raise ValueError(f"malformed hostlist {expr!r}")
        if n >= 0:
            return [x.decode() for x in buf.raw.split(b"\0")[:n]]
        if buflen > 1 << 28:
            check(n, "fit_expand_hostlist")
        buflen *= 16


def node_names(entries: list[str]) -> list[str]:
    """The Partition RPC's node list (parsePartition's comma split, parse.go:278-289) → the expanded
    node names to send to the Nodes RPC, one engine row each (fit_node_names)."""
    blob = b"".join(e.encode() + b"\0" for e in entries)
    buflen = 1 << 16
    while True:
        buf = C.create_string_buffer(buflen)
        n = lib().fit_node_names(blob, len(entries), buf, buflen)
        if n == FIT_E_PARSE:
            raise ValueError(f"malformed hostlist or a node name listed twice: {entries!r}")
        if n >= 0:
            return [x.decode() for x in buf.raw.split(b"\0")[:n]]
        if buflen > 1 << 28:
            check(n, "fit_node_names")
        buflen *= 16


def release_events(n: int, jobs: list, slots: int, slot_min: int):
    """Release events for Engine.load_timeline from running jobs (fit_release_events): ``jobs`` is a
    list of (node rows, minutes left, cpu, mem MiB, gpus); returns a synth.Timeline."""
    from .synth import Timeline
    m = len(jobs)
    off = np.zeros(m + 1, np.int32)
    for i, j in enumerate(jobs):
        off[i + 1] = off[i] + len(j[0])
    nodes = np.array([x for j in jobs for x in j[0]], np.int32)
    rem = np.array([j[1] for j in jobs], np.int64)
    cols = [np.array([j[k] for j in jobs], np.int32) for k in (2, 3, 4)]
    e = int(off[-1])
    out = [np.zeros(n + 1, np.int32)] + [np.zeros(max(e, 1), np.int32) for _ in range(4)]
    r = lib().fit_release_events(n, m, _ptr(off), _ptr(nodes) if e else None, _ptr(rem), *[_ptr(c) for c in cols],
                                 slots, slot_min, *[_ptr(o) for o in out], e)
    check(r, "fit_release_events")
    return Timeline(slots=slots, slot_min=slot_min, off=out[0], slot=out[1][:r], cpu=out[2][:r],
                    mem=out[3][:r], gpu=out[4][:r])


def ingest_nodes(text: str, partitions: list[str]):
    """`scontrol show nodes` text → (synth.Nodes columns for Engine.load_nodes, node names)
    (Client.Nodes + parseNode, slurm.go:354-363 / parse.go:291-308, plus Gres,
    GresUsed, State, Partitions, NodeName)."""
    from .synth import Nodes
    cap = text.count("\n\n") + 2
    cols = [np.empty(cap, np.int32) for _ in range(4)] + [np.empty(cap, np.uint32)]
    blob = b"".join(p.encode() + b"\0" for p in partitions)
    names_len = len(text.encode()) + 64
    names = C.create_string_buffer(names_len)
    n = lib().fit_ingest_nodes(text.encode(), blob, len(partitions), cap, *[_ptr(c) for c in cols], names,
                               names_len)
    if n == FIT_E_PARSE:
        raise ValueError("malformed Gres count")
    check(n, "fit_ingest_nodes")
    nodes = Nodes(*(c[:n].copy() for c in cols))
    return nodes, [x.decode() for x in names.raw.split(b"\0")[:n]]


@dataclass
class JobResources:  # apis/kubecluster.org/v1alpha1/affinity.go:40-48
    Nodes: int = 0
    CpusPerTask: int = 0
    Ntasks: int = 0
    NtasksPerNode: int = 0
    MemPerCpu: int = 0
    WallTime: int = 0
    Array: str = ""

    def _c(self) -> FitJobResources:
        r = FitJobResources()
        r.nodes, r.cpus_per_task, r.ntasks = self.Nodes, self.CpusPerTask, self.Ntasks
        r.ntasks_per_node, r.mem_per_cpu, r.wall_ns = self.NtasksPerNode, self.MemPerCpu, self.WallTime
        r.array = self.Array.encode()[:63]
        return r

    @staticmethod
    def _py(r: FitJobResources) -> "JobResources":
        return JobResources(r.nodes, r.cpus_per_task, r.ntasks, r.ntasks_per_node, r.mem_per_cpu,
                            r.wall_ns, r.array.decode())


def extract_batch_resources(script: str) -> JobResources:
    r = FitJobResources()
    rc = lib().fit_extract_batch_resources(script.encode(), C.byref(r))
    if rc == FIT_E_PARSE:
        raise ValueError("could not extract required resources")
    check(rc, "fit_extract_batch_resources")
    return JobResources._py(r)


def apply_spec(res: JobResources, nodes=0, cpus_per_task=0, mem_per_cpu=0, ntasks_per_node=0,
               array="", ntasks=0) -> JobResources:
    r = res._c()
    lib().fit_apply_spec(C.byref(r), nodes, cpus_per_task, mem_per_cpu, ntasks_per_node,
                         array.encode(), ntasks)
    return JobResources._py(r)


def parse_array_len(array: str) -> int:
    return lib().fit_array_len(array.encode())


def gen_resource_list_for_pod(res: JobResources) -> dict:
    cpu, mem = C.c_int64(), C.c_int64()
    lib().fit_pod_request(C.byref(res._c()), C.byref(cpu), C.byref(mem))
    return {"cpu": cpu.value, "memory": mem.value}


def job_demand(res: JobResources) -> tuple[int, int, int, int]:
    """(cpus per node, MiB per node, walltime minutes, nodes) — DESIGN.md §2 demand rule."""
    cpu, mem, wall, k = C.c_int32(), C.c_int32(), C.c_int32(), C.c_uint16()
    check(lib().fit_job_demand(C.byref(res._c()), C.byref(cpu), C.byref(mem), C.byref(wall),
                               C.byref(k)), "fit_job_demand")
    return cpu.value, mem.value, wall.value, k.value


def get_partition_capacity(nodes: list[Node]) -> dict:
    arr = (FitNode * max(len(nodes), 1))()
    for i, n in enumerate(nodes):
        arr[i] = FitNode(n.Cpus, n.Memory, n.Gpus, n.AlloCpus, n.AlloMemory, n.AlloGpus)
    cpu, mem, gpu, pods = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    lib().fit_partition_capacity(arr, len(nodes), C.byref(cpu), C.byref(mem), C.byref(gpu), C.byref(pods))
    out = {"cpu": cpu.value, "memory": mem.value, "pods": pods.value}
    if gpu.value > 0:
        out["nvidia.com/gpu"] = gpu.value
    return out


# ---------------------------------------------------------------- CreatePod call site
# pkg/common/labels.go:9-14, the keys newSubmitRequestForPod reads (provider.go:74-123)
POD_LABEL_KEYS = {"nodes": "sbo.kubecluster.org/nodes", "cpus_per_task": "sbo.kubecluster.org/cpus-per-task",
                  "mem_per_cpu": "sbo.kubecluster.org/mem-per-cpu",
                  "ntasks_per_node": "sbo.kubecluster.org/ntasks-per-node",
                  "array": "sbo.kubecluster.org/array", "ntasks": "sbo.kubecluster.org/ntask"}


def array_tasks(array: str) -> tuple[int, int]:
    """(distinct task ids, tasks that may run at once) of a Slurm --array expression."""
    n, r = C.c_int64(), C.c_int64()
    rc = lib().fit_array_tasks(array.encode(), C.byref(n), C.byref(r))
    if rc == FIT_E_PARSE:
        raise ValueError(f"malformed array {array!r}")
    check(rc, "fit_array_tasks")
    return n.value, r.value


def set_max_array_size(n: int) -> int:
    """Slurm's MaxArraySize for pod_demand (process-wide; default 1001); returns the previous one."""
    return check(lib().fit_set_max_array_size(n), "fit_set_max_array_size")


def pod_demand(labels: dict, script: str | None, part: int = 0, priority: int = 0) -> list[tuple]:
    """A pod's admission requests from its labels (keys of POD_LABEL_KEYS' values) and script:
    [(priority, cpu, mem_mib, gpu, wall_min, part, nodes_k, flags)] — one per array task that
    may run at once (include/fitgpu.h fit_pod_demand); flags FIT_REQ_ARRAY marks an array job's
    tasks (never pinned by Admitter.script)."""
    byname = {v: k for k, v in POD_LABEL_KEYS.items()}
    vals = {byname[k]: str(v).encode() for k, v in labels.items() if k in byname}
    lab = FitPodLabels(*(vals.get(k) for k in ("nodes", "cpus_per_task", "mem_per_cpu", "ntasks_per_node",
                                               "array", "ntasks")))
    scr = script.encode() if script is not None else None
    n = lib().fit_pod_demand(C.byref(lab), scr, part, priority, None, 0)
    if n == FIT_E_PARSE:
        raise ValueError("malformed #SBATCH header or array expression")
    check(n, "fit_pod_demand")
    out = (FitAdmitReq * n)()
    check(lib().fit_pod_demand(C.byref(lab), scr, part, priority, out, n), "fit_pod_demand")
    return [(r.priority, r.cpu, r.mem_mib, r.gpu, r.wall_min, r.part, r.nodes_k, r.flags) for r in out]


def script_with_nodelist(script: str, names: list[str], nodes: list[int]) -> str:
    """The script with `#SBATCH --nodelist=` for the engine's nodes (fit_script_with_nodelist)."""
    blob = b"".join(x.encode() + b"\0" for x in names)
    outlen = len(script.encode()) + 32 + len(blob) + 1
    buf = C.create_string_buffer(outlen)
    ids = (C.c_int32 * len(nodes))(*nodes)
    n = check(lib().fit_script_with_nodelist(script.encode(), blob, len(names), ids, len(nodes), buf, outlen),
              "fit_script_with_nodelist")
    return buf.raw[:n].decode()


def partition_limits(wall_time_s: int, cpu_per_node: int, mem_per_node: int) -> tuple[int, int, int]:
    """ResourcesResponse fields → (max_time_min, max_cpus_per_node, max_mem_per_node), -1 = none."""
    a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
    check(lib().fit_partition_limits(wall_time_s, cpu_per_node, mem_per_node, C.byref(a), C.byref(b), C.byref(c)),
          "fit_partition_limits")
    return a.value, b.value, c.value


def node_columns(nodes: list[Node], part_mask: int = 1):
    """NodesResponse rows → synth.Nodes columns (free = total − alloc) for load_nodes."""
    from .synth import Nodes
    n = len(nodes)
    arr = (FitNode * max(n, 1))()
    for i, x in enumerate(nodes):
        arr[i] = FitNode(x.Cpus, x.Memory, x.Gpus, x.AlloCpus, x.AlloMemory, x.AlloGpus)
    cols = [np.empty(max(n, 1), np.int32) for _ in range(4)] + [np.empty(max(n, 1), np.uint32)]
    check(lib().fit_node_columns(arr, n, part_mask, *[_ptr(c) for c in cols]), "fit_node_columns")
    return Nodes(*(c[:n].copy() for c in cols))


# ------------------------------------------------------------------------------- engine
def lock_dir() -> tuple[str, bool]:
    """fit_lock_dir: the directory of the per-GPU launch lock file and whether it is the shared
    one (FIT_LOCK_DIR, or the /var/run/fitgpu host path) rather than the /tmp fallback."""
    buf = C.create_string_buffer(4096)
    rc = lib().fit_lock_dir(buf, len(buf))
    check(rc, "fit_lock_dir")
    return buf.value.decode(), rc == 0


def nccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    check(lib().fit_nccl_unique_id(buf), "fit_nccl_unique_id")
    return buf.raw


class TorchHostExchange:
    """Host-side exchange over torch.distributed (e.g. gloo) for the engine's collectives.

    Lets several ranks share one GPU in tests, exercising exactly the multi-rank engine code that
    RCCL drives in production (fit_opts.exchange, include/fitgpu.h)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.fn = XCHG_FN(self._call)

    def _call(self, user, op, buf, count):
        import torch
        try:
            d = self.dist
            if op in (FIT_XCHG_ALLGATHER_U64, FIT_XCHG_MIN_U64):
                n = count * (self.world if op == FIT_XCHG_ALLGATHER_U64 else 1)
                arr = np.ctypeslib.as_array(C.cast(buf, C.POINTER(C.c_int64)), shape=(n,))
                mine = arr[self.rank * count:(self.rank + 1) * count] if op == FIT_XCHG_ALLGATHER_U64 else arr
                parts = [torch.empty(count, dtype=torch.int64) for _ in range(self.world)]
                d.all_gather(parts, torch.from_numpy(mine.copy()), group=self.group)
                if op == FIT_XCHG_ALLGATHER_U64:
                    arr[:] = torch.cat(parts).numpy()
                else:
                    arr[:] = np.minimum.reduce([p.numpy().view(np.uint64) for p in parts]).view(np.int64)
            else:
                arr = np.ctypeslib.as_array(C.cast(buf, C.POINTER(C.c_int32)), shape=(count,))
                t = torch.from_numpy(arr.copy())
                d.all_reduce(t, op=d.ReduceOp.MAX if op == FIT_XCHG_MAX_I32 else d.ReduceOp.MIN, group=self.group)
                arr[:] = t.numpy()
            return 0
        except Exception:  # never let a Python exception cross the C boundary
            return -1


class Engine:
    """One placement context on one GPU (optionally one rank of a multi-GPU group)."""

    def __init__(self, device: int = -1, rank: int = 0, world: int = 1, nccl_id: bytes | None = None,
                 window_min: int = 0, window_max: int = 0, shard_mode: int = 0,
                 exchange: "TorchHostExchange | None" = None, flags: int = 0):
        self._idbuf = C.create_string_buffer(nccl_id, 128) if nccl_id else None
        self._xchg = exchange
        o = FitOpts(device, rank, world, C.cast(self._idbuf, C.c_void_p) if self._idbuf else None,
                    shard_mode, window_min, window_max, flags, exchange.fn if exchange else XCHG_FN(), None)
        h = C.c_void_p()
        check(lib().fit_create(C.byref(o), C.byref(h)), "fit_create")
        self._h = h
        self.n = 0
        self._admitters = weakref.WeakSet()  # closed before the context goes (Admitter holds it)

    def close(self):
        for a in list(getattr(self, "_admitters", ())):
            a.close()
        if getattr(self, "_h", None):
            lib().fit_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load_nodes(self, nodes):
        cols = [np.ascontiguousarray(nodes.cpu_free, np.int32), np.ascontiguousarray(nodes.mem_free, np.int32),
                np.ascontiguousarray(nodes.gpu_free, np.int32), np.ascontiguousarray(nodes.avail_min, np.int32),
                np.ascontiguousarray(nodes.part_mask, np.uint32)]
        n = len(cols[0])
        check(lib().fit_load_nodes(self._h, n, *[_ptr(c) for c in cols]), "fit_load_nodes")
        self.n = n

    def load_nodes_device(self, cpu, mem, gpu, avail, mask):
        """torch tensors on this context's GPU (int32 / int32 / int32 / int32 / int32-viewed uint32)."""
        n = int(cpu.numel())
        check(lib().fit_load_nodes_device(self._h, n, *[_ptr(t) for t in (cpu, mem, gpu, avail, mask)]),
              "fit_load_nodes_device")
        self.n = n

    def set_watchdog_us(self, us: int):
        """Deadline of every device-side wait of the persistent engines (fit_set_watchdog_us);
        us <= 0 restores the default (10 s)."""
        check(lib().fit_set_watchdog_us(self._h, int(us)), "fit_set_watchdog_us")

    def load_partitions(self, parts):
        cols = [np.ascontiguousarray(a, np.int32) for a in (parts.max_time_min, parts.max_cpus_per_node,
                                                            parts.max_mem_per_node)]
        check(lib().fit_load_partitions(self._h, len(cols[0]), *[_ptr(c) for c in cols]),
              "fit_load_partitions")

    def place(self, jobs, kmax: int = 1, out=None):
        """Host arrays in, placements out[J, kmax] (an int32 array the caller may pass, e.g. pinned)."""
        cols = [np.ascontiguousarray(a, np.int32) for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)]
        part = np.ascontiguousarray(jobs.part, np.uint16)
        k = np.ascontiguousarray(jobs.nodes_k, np.uint16)
        j = len(part)
        if out is None:
            out = np.empty((j, kmax), np.int32)
        elif out.dtype != np.int32 or out.size != j * kmax or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous int32 array of J * kmax entries")
        st = FitStats()
        check(lib().fit_place(self._h, j, *[_ptr(c) for c in cols], _ptr(part), _ptr(k), kmax, _ptr(out),
                              C.byref(st)), "fit_place")
        return out, st.as_dict()

    def place_device(self, cpu, mem, gpu, wall, part, nodes_k, out, kmax: int = 1):
        """All arguments torch tensors resident on this GPU; writes out[J*kmax]."""
        st = FitStats()
        check(lib().fit_place_device(self._h, int(cpu.numel()), _ptr(cpu), _ptr(mem), _ptr(gpu), _ptr(wall),
                                     _ptr(part), _ptr(nodes_k) if nodes_k is not None else None, kmax,
                                     _ptr(out), C.byref(st)), "fit_place_device")
        return st.as_dict()

    # ---- time-windowed backfill ------------------------------------------
    def load_timeline(self, tline):
        """Release events (synth.Timeline) over a horizon of tline.slots slots of tline.slot_min
        minutes, on top of the node table of the last load_nodes."""
        cols = [np.ascontiguousarray(a, np.int32) for a in (tline.off, tline.slot, tline.cpu, tline.mem,
                                                            tline.gpu)]
        check(lib().fit_load_timeline(self._h, int(tline.slots), int(tline.slot_min), *[_ptr(c) for c in cols]),
              "fit_load_timeline")
        self.slots = int(tline.slots)

    def load_timeline_device(self, slots, slot_min, off, slot, cpu, mem, gpu):
        """torch int32 tensors on this GPU (off has n + 1 entries)."""
        check(lib().fit_load_timeline_device(self._h, int(slots), int(slot_min), _ptr(off), int(slot.numel()),
                                             *[_ptr(t) for t in (slot, cpu, mem, gpu)]), "fit_load_timeline_device")
        self.slots = int(slots)

    def place_tl(self, jobs, node=None, start=None):
        """Returns (node[J], start_slot[J], stats); node / start may be caller int32 arrays."""
        cols = [np.ascontiguousarray(a, np.int32) for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)]
        part = np.ascontiguousarray(jobs.part, np.uint16)
        j = len(part)
        node = np.empty(j, np.int32) if node is None else node
        start = np.empty(j, np.int32) if start is None else start
        for a in (node, start):
            if a.dtype != np.int32 or a.size != j or not a.flags.c_contiguous:
                raise ValueError("node / start must be contiguous int32 arrays of J entries")
        st = FitStats()
        check(lib().fit_place_tl(self._h, j, *[_ptr(c) for c in cols], _ptr(part), _ptr(node), _ptr(start),
                                 C.byref(st)), "fit_place_tl")
        return node, start, st.as_dict()

    def place_tl_device(self, cpu, mem, gpu, wall, part, out_node, out_start):
        st = FitStats()
        check(lib().fit_place_tl_device(self._h, int(cpu.numel()), *[_ptr(t) for t in (cpu, mem, gpu, wall, part)],
                                        _ptr(out_node), _ptr(out_start), C.byref(st)), "fit_place_tl_device")
        return st.as_dict()

    def read_timeline(self):
        """Dense [n, slots, 3] int32 (cpu, mem, gpu)."""
        c, m, g = (np.empty((self.n, self.slots), np.int32) for _ in range(3))
        check(lib().fit_read_timeline(self._h, _ptr(c), _ptr(m), _ptr(g)), "fit_read_timeline")
        return np.stack([c, m, g], axis=2)

    def read_nodes(self):
        c, m, g = (np.empty(self.n, np.int32) for _ in range(3))
        check(lib().fit_read_nodes(self._h, _ptr(c), _ptr(m), _ptr(g)), "fit_read_nodes")
        return c, m, g

    def partition_free(self, p: int):
        c, m, g = C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().fit_partition_free(self._h, p, C.byref(c), C.byref(m), C.byref(g)), "fit_partition_free")
        return {"cpu": c.value, "mem_mib": m.value, "gpu": g.value}


class Admitter:
    """Batched admission over one Engine (include/fitgpu.h "batched admission"; the CreatePod
    call site of pkg/slurm-virtual-kubelet/provider.go:35-60).  `admit` blocks the calling thread
    until its batch is placed (ctypes releases the GIL, so threads admit concurrently, as the 10
    PodSyncWorkers do) and returns (nodes, batch, batch_jobs, order, ticket); nodes[0] is
    FIT_UNPLACED / FIT_REJECTED when the pod cannot be placed now.

    Lifetime: close() (also Engine.close()) stops new calls, waits for the calls already inside
    (their batches are still placed), then destroys the native admitter — a caller can never hold
    a handle that is being freed."""

    def __init__(self, engine: Engine, max_batch: int = 1024, max_wait_us: int = 2000):
        self._engine = engine  # keeps the context alive
        h = C.c_void_p()
        check(lib().fit_admitter_create(engine._h, max_batch, max_wait_us, C.byref(h)), "fit_admitter_create")
        self._h = h
        self._cv = threading.Condition()
        self._users = 0
        engine._admitters.add(self)

    def _enter(self):
        with self._cv:
            if not self._h:
                raise FitError(FIT_E_STATE, "Admitter closed")
            self._users += 1
            return self._h

    def _leave(self):
        with self._cv:
            self._users -= 1
            self._cv.notify_all()

    def _call(self, fn, *args):
        h = self._enter()
        try:
            return fn(h, *args)
        finally:
            self._leave()

    @staticmethod
    def _res(r, nodes_k):
        k = max(nodes_k, 1)
        nodes = [r.node[i] for i in range(k)] if r.node[0] >= 0 else [r.node[0]]
        return nodes, r.batch, r.batch_jobs, r.order, r.ticket

    def admit(self, priority: int, cpu: int, mem_mib: int, gpu: int = 0, wall_min: int = 0,
              part: int = 0, nodes_k: int = 1):
        q = FitAdmitReq(priority, cpu, mem_mib, gpu, wall_min, part, nodes_k)
        r = FitAdmitRes()
        check(self._call(lambda h: lib().fit_admit(h, C.byref(q), C.byref(r))), "fit_admit")
        return self._res(r, nodes_k)

    def admit_group(self, reqs: list[tuple]):
        """All-or-nothing admission of (priority, cpu, mem, gpu, wall, part, k) requests (the
        tasks of one array job, pod_demand's output); one result per request."""
        n = len(reqs)
        q = (FitAdmitReq * n)(*[FitAdmitReq(*r) for r in reqs])
        r = (FitAdmitRes * n)()
        check(self._call(lambda h: lib().fit_admit_group(h, q, n, r)), "fit_admit_group")
        return [self._res(r[i], reqs[i][6]) for i in range(n)]

    def load_nodes(self, nodes):
        cols = [np.ascontiguousarray(nodes.cpu_free, np.int32), np.ascontiguousarray(nodes.mem_free, np.int32),
                np.ascontiguousarray(nodes.gpu_free, np.int32), np.ascontiguousarray(nodes.avail_min, np.int32),
                np.ascontiguousarray(nodes.part_mask, np.uint32)]
        check(self._call(lambda h: lib().fit_admitter_load_nodes(h, len(cols[0]), *[_ptr(c) for c in cols])),
              "fit_admitter_load_nodes")
        self._engine.n = len(cols[0])

    def load_table(self, nodes, names: list[str] | None = None, state: bool = False, pin: bool = False,
                   generation: int = 0):
        """fit_admitter_load_table: the node table with its names (reservations follow nodes by
        name; pinning needs them), whether part_mask carries node State (FIT_TABLE_STATE: pinned)
        and whether to pin without State (FIT_TABLE_PIN)."""
        cols = [np.ascontiguousarray(nodes.cpu_free, np.int32), np.ascontiguousarray(nodes.mem_free, np.int32),
                np.ascontiguousarray(nodes.gpu_free, np.int32), np.ascontiguousarray(nodes.avail_min, np.int32),
                np.ascontiguousarray(nodes.part_mask, np.uint32)]
        blob = b"".join(x.encode() + b"\0" for x in names) if names is not None else None
        t = FitNodeTable(len(cols[0]), *[c.ctypes.data for c in cols], blob,
                         (FIT_TABLE_STATE if state else 0) | (FIT_TABLE_PIN if pin else 0), generation)
        check(self._call(lambda h: lib().fit_admitter_load_table(h, C.byref(t))), "fit_admitter_load_table")
        self._engine.n = len(cols[0])

    def generation(self) -> int:
        return check(self._call(lambda h: lib().fit_admitter_generation(h)), "fit_admitter_generation")

    def script(self, tickets: list[int], script: str) -> tuple[str, bool]:
        """(script to submit, pinned): fit_admitter_script."""
        t = (C.c_int64 * len(tickets))(*tickets)
        outlen = len(script.encode()) + 64 + 4096 * 8
        buf = C.create_string_buffer(outlen)
        pinned = C.c_int32()
        n = check(self._call(lambda h: lib().fit_admitter_script(h, t, len(tickets), script.encode(), buf, outlen,
                                                                 C.byref(pinned))), "fit_admitter_script")
        return buf.raw[:n].decode(), bool(pinned.value)

    def partition_free(self, p: int):
        c, m, g = C.c_int64(), C.c_int64(), C.c_int64()
        check(self._call(lambda h: lib().fit_admitter_partition_free(h, p, C.byref(c), C.byref(m), C.byref(g))),
              "fit_admitter_partition_free")
        return {"cpu": c.value, "mem_mib": m.value, "gpu": g.value}

    def confirm(self, ticket: int):
        check(self._call(lambda h: lib().fit_admitter_confirm(h, ticket)), "fit_admitter_confirm")

    def release(self, ticket: int):
        check(self._call(lambda h: lib().fit_admitter_release(h, ticket)), "fit_admitter_release")

    def set_ttl(self, loads: int):
        check(self._call(lambda h: lib().fit_admitter_set_ttl(h, loads)), "fit_admitter_set_ttl")

    def reservations(self) -> int:
        return check(self._call(lambda h: lib().fit_admitter_reservations(h)), "fit_admitter_reservations")

    def pending(self) -> int:
        return check(self._call(lambda h: lib().fit_admitter_pending(h)), "fit_admitter_pending")

    def close(self):
        cv = getattr(self, "_cv", None)
        if cv is None:
            return
        with cv:
            h, self._h = self._h, None  # no new calls
            while self._users:
                cv.wait()  # calls already inside finish (their batches are placed)
        if h:
            lib().fit_admitter_destroy(h)

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
