"""Deterministic synthetic cluster / job-stream generator (integer-only, counter-based splitmix64).

The reference has no benchmark inputs; BASELINE.json names five configurations and
SURVEY.md §8(d) fixes their distributions.  Every value here is a pure function of
(seed, stream, index), so any slice of the stream can be generated independently (numpy here,
a C twin of ``rnd``, ``ref_rnd`` in ``oracle/fitref.c:563``, that must agree bit-for-bit — ``tests/test_synth.py``).

    rnd(seed, stream, i) = mix64(seed + GOLDEN * (i * 64 + stream + 1))      (mod 2**64)
    uni(r, m)            = ((r >> 32) * m) >> 32                              in [0, m)

Units (SPEC): cpus, MiB, GPU count, minutes.  ``avail_min`` INT32_MAX = no horizon.
Partition limits use -1 for UNLIMITED, like ``parseResources`` (pkg/slurm-agent/parse.go:139-168).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
INT32_MAX = 2**31 - 1

SEEDS = {"c1": 0x5EED0001, "c2": 0x5EED0002, "c3": 0x5EED0003, "c4": 0x5EED0004, "c5": 0x5EED0005}

# stream ids (never reuse one across fields)
S_NCLASS, S_NMEM, S_NGPU, S_ACPU, S_AMEM, S_AGPU, S_NPART, S_AVF, S_AVV = range(0, 9)
S_RN, S_RS = 9, 10  # C5: running jobs per node, their release slots
S_JCPU, S_JMEM, S_JGPUF, S_JGPUV, S_JWO, S_JWV, S_JPART, S_JK = range(16, 24)
S_PTIME = 32
S_JALL = 24  # c3o: job targets the all-nodes partition
S_ARUN = 25  # array-expanded streams: tasks per array job

NODE_CPUS = np.array([32, 64, 96, 128, 192, 256], dtype=np.int64)
NODE_MEMMUL = np.array([2048, 4096, 8192], dtype=np.int64)
JOB_CPUS = np.array([1, 2, 4, 8, 16, 32, 64], dtype=np.int64)
JOB_CPU_W = np.cumsum([64, 32, 16, 8, 4, 2, 1])  # p ∝ 1/cpus, total 127
JOB_MEMMUL = np.array([500, 1024, 2048, 4096], dtype=np.int64)
JOB_GPUS = np.array([1, 2, 4, 8], dtype=np.int64)
JOB_K = np.array([1, 2, 4, 8], dtype=np.int64)
PART_TIME = np.array([60, 240, 720, 1440, 2880, -1], dtype=np.int64)


def mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def rnd(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        ctr = idx.astype(np.uint64) * np.uint64(64) + np.uint64(stream + 1)
        return mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + GOLDEN * ctr)


def uni(r: np.ndarray, m) -> np.ndarray:
    """Integer in [0, m) from the high 32 bits (no rejection: deterministic, tiny bias)."""
    m = np.asarray(m, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return (((r >> np.uint64(32)) * m) >> np.uint64(32)).astype(np.int64)


@dataclass
class Nodes:
    cpu_free: np.ndarray  # int32
    mem_free: np.ndarray  # int32, MiB
    gpu_free: np.ndarray  # int32
    avail_min: np.ndarray  # int32 minutes, INT32_MAX = unlimited
    part_mask: np.ndarray  # uint32, bit p = member of partition p

    @property
    def n(self) -> int:
        return int(self.cpu_free.shape[0])


@dataclass
class Jobs:
    cpu: np.ndarray  # int32 per-node demand
    mem: np.ndarray  # int32 MiB per node
    gpu: np.ndarray  # int32 per node
    wall: np.ndarray  # int32 minutes
    part: np.ndarray  # uint16 partition index
    nodes_k: np.ndarray  # uint16 nodes per job (>= 1)

    @property
    def j(self) -> int:
        return int(self.cpu.shape[0])


@dataclass
class Timeline:
    """C5 reservation horizon: ``slots`` slots of ``slot_min`` minutes, plus the
    release events of the jobs already running on each node, CSR by node id: events of node x are
    [off[x], off[x+1]), slots non-decreasing; at slot ``slot[e]`` the node gets back
    (cpu[e], mem[e], gpu[e])."""
    slots: int
    slot_min: int
    off: np.ndarray  # int32 [n + 1]
    slot: np.ndarray  # int32 [E]
    cpu: np.ndarray  # int32 [E]
    mem: np.ndarray  # int32 [E], MiB
    gpu: np.ndarray  # int32 [E]


@dataclass
class Partitions:
    max_time_min: np.ndarray  # int32, -1 unlimited
    max_cpus_per_node: np.ndarray  # int32, -1 unlimited
    max_mem_per_node: np.ndarray  # int32, -1 unlimited

    @property
    def p(self) -> int:
        return int(self.max_time_min.shape[0])


def gen_nodes(seed: int, n: int, parts: int, gpu_heavy: bool = False, start: int = 0) -> Nodes:
    i = np.arange(start, start + n, dtype=np.uint64)
    cpus = NODE_CPUS[uni(rnd(seed, S_NCLASS, i), 6)]
    mem = cpus * NODE_MEMMUL[uni(rnd(seed, S_NMEM, i), 3)]
    if gpu_heavy:
        gpus = np.full(n, 8, dtype=np.int64)
    else:
        u = uni(rnd(seed, S_NGPU, i), 100)
        gpus = np.where(u < 70, 0, np.where(u < 85, 4, 8)).astype(np.int64)
    acpu = cpus * uni(rnd(seed, S_ACPU, i), 51) // 100
    amem = mem * uni(rnd(seed, S_AMEM, i), 51) // 100
    agpu = gpus * uni(rnd(seed, S_AGPU, i), 51) // 100
    part = uni(rnd(seed, S_NPART, i), parts)
    avf = uni(rnd(seed, S_AVF, i), 100)
    avv = 60 + uni(rnd(seed, S_AVV, i), 2821)
    avail = np.where(avf < 90, INT32_MAX, avv)
    return Nodes(
        cpu_free=(cpus - acpu).astype(np.int32),
        mem_free=(mem - amem).astype(np.int32),
        gpu_free=(gpus - agpu).astype(np.int32),
        avail_min=avail.astype(np.int32),
        part_mask=(np.uint32(1) << part.astype(np.uint32)).astype(np.uint32),
    )


def gen_releases(seed: int, n: int, slots: int = 1024, slot_min: int = 5, gpu_heavy: bool = False,
                 start: int = 0) -> Timeline:
    """Release events of the allocation gen_nodes() subtracts: node x runs R = 1..4 jobs (uniform)
    that hold the allocated (cpu, mem, gpu) in R near-equal integer parts, each released at a
    uniform slot in [1, slots)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    cpus = NODE_CPUS[uni(rnd(seed, S_NCLASS, i), 6)]
    mem = cpus * NODE_MEMMUL[uni(rnd(seed, S_NMEM, i), 3)]
    if gpu_heavy:
        gpus = np.full(n, 8, dtype=np.int64)
    else:
        u = uni(rnd(seed, S_NGPU, i), 100)
        gpus = np.where(u < 70, 0, np.where(u < 85, 4, 8)).astype(np.int64)
    alloc = np.stack([cpus * uni(rnd(seed, S_ACPU, i), 51) // 100, mem * uni(rnd(seed, S_AMEM, i), 51) // 100,
                      gpus * uni(rnd(seed, S_AGPU, i), 51) // 100], axis=1)  # [n, 3]
    r = 1 + uni(rnd(seed, S_RN, i), 4)  # [n]
    rr = np.arange(4, dtype=np.int64)
    idx = (i[:, None] * np.uint64(4) + rr[None, :].astype(np.uint64))
    rs = 1 + uni(rnd(seed, S_RS, idx), slots - 1)  # [n, 4]
    rs = np.where(rr[None, :] < r[:, None], rs, np.iinfo(np.int64).max)
    rs.sort(axis=1)
    # part k of R: alloc*(k+1)//R - alloc*k//R
    k = rr[None, :, None]
    part = alloc[:, None, :] * (k + 1) // r[:, None, None] - alloc[:, None, :] * k // r[:, None, None]
    valid = rr[None, :] < r[:, None]
    counts = valid.sum(axis=1)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(counts)
    return Timeline(slots=slots, slot_min=slot_min, off=off.astype(np.int32),
                    slot=rs[valid].astype(np.int32), cpu=part[..., 0][valid].astype(np.int32),
                    mem=part[..., 1][valid].astype(np.int32), gpu=part[..., 2][valid].astype(np.int32))


def gen_jobs(seed: int, j: int, parts: int, multi_node: bool = False, start: int = 0) -> Jobs:
    i = np.arange(start, start + j, dtype=np.uint64)
    u = uni(rnd(seed, S_JCPU, i), 127)
    cpus = JOB_CPUS[np.searchsorted(JOB_CPU_W, u, side="right")]
    mem = cpus * JOB_MEMMUL[uni(rnd(seed, S_JMEM, i), 4)]
    gf = uni(rnd(seed, S_JGPUF, i), 100)
    gpus = np.where(gf < 80, 0, JOB_GPUS[uni(rnd(seed, S_JGPUV, i), 4)])
    octave = uni(rnd(seed, S_JWO, i), 10)
    lo = np.int64(5) << octave
    hi = np.minimum(np.int64(10) << octave, 2880)
    wall = lo + uni(rnd(seed, S_JWV, i), (hi - lo + 1).astype(np.uint64))
    part = uni(rnd(seed, S_JPART, i), parts)
    if multi_node:
        k = JOB_K[uni(rnd(seed, S_JK, i), 4)]
    else:
        k = np.ones(j, dtype=np.int64)
    return Jobs(
        cpu=cpus.astype(np.int32),
        mem=mem.astype(np.int32),
        gpu=gpus.astype(np.int32),
        wall=wall.astype(np.int32),
        part=part.astype(np.uint16),
        nodes_k=k.astype(np.uint16),
    )


def gen_partitions(seed: int, parts: int) -> Partitions:
    i = np.arange(parts, dtype=np.uint64)
    t = PART_TIME[uni(rnd(seed, S_PTIME, i), 6)]
    neg = np.full(parts, -1, dtype=np.int32)
    return Partitions(max_time_min=t.astype(np.int32), max_cpus_per_node=neg.copy(), max_mem_per_node=neg.copy())


# ---- BASELINE.json configs -------------------------------------------------------------------
CONFIGS = {
    # name: (nodes, jobs, partitions, gpu_heavy, multi_node)
    "c2": (4096, 65536, 1, False, False),
    "c3": (100_000, 1_000_000, 16, False, False),
    "c4": (100_000, 1_000_000, 16, True, True),
    "c5": (100_000, 1_000_000, 16, False, False),  # + 1,024-slot horizon (make_c5)
    # C3 with overlapping partitions: every node also belongs to an all-nodes
    # partition 16 that ~10 % of the jobs target, so the 16 partitions union into ONE component
    "c3o": (100_000, 1_000_000, 16, False, False),
}
C3O_ALL_PCT = 10
C5_SLOTS, C5_SLOT_MIN = 1024, 5  # 1,024 slots × 5 min = 85.3 h ≥ the longest walltime (2,880 min)


def make_config(name: str, nodes: int | None = None, jobs: int | None = None, shard: int = 0):
    """Synthetic cluster for BASELINE.json config ``name`` (optionally truncated for tests).
    ``shard`` s > 0 draws the s-th disjoint slice of the same streams (nodes [s*n, (s+1)*n), jobs
    [s*j, (s+1)*j)): an independent cluster of the same shape, for weak-scaling runs."""
    n, j, p, gh, mn = CONFIGS[name]
    seed = SEEDS["c3" if name == "c3o" else name]
    n = n if nodes is None else nodes
    j = j if jobs is None else jobs
    nd, jb = gen_nodes(seed, n, p, gh, start=shard * n), gen_jobs(seed, j, p, mn, start=shard * j)
    if name != "c3o":
        return nd, jb, gen_partitions(seed, p)
    # c3o: C3's cluster and stream, plus partition p (all nodes) for C3O_ALL_PCT % of the jobs
    nd.part_mask = nd.part_mask | np.uint32(1 << p)
    i = np.arange(shard * j, shard * j + j, dtype=np.uint64)
    jb.part = np.where(uni(rnd(seed, S_JALL, i), 100) < C3O_ALL_PCT, p, jb.part).astype(np.uint16)
    return nd, jb, gen_partitions(seed, p + 1)


# Array-expanded streams: `--array=1-N` turns one SlurmBridgeJob into N
# identical pods (fit_array_tasks; reference pkg/slurm-bridge-operator/parse.go array handling), so
# the pending queue holds runs of identical demands.  Tasks per array job from ARRAY_RUNS.
ARRAY_RUNS = np.array([1, 1, 2, 4, 8, 8, 16, 32], dtype=np.int64)


def expand_arrays(seed: int, jobs: Jobs, j: int | None = None) -> Jobs:
    """The first ``j`` (default: as many as ``jobs``) pods of the stream in which job i of ``jobs``
    is an array job of ARRAY_RUNS[u] identical tasks, each task its own pending pod in priority
    order (mean 9 tasks per array job)."""
    j = jobs.j if j is None else j
    runs = ARRAY_RUNS[uni(rnd(seed, S_ARUN, np.arange(jobs.j, dtype=np.uint64)), len(ARRAY_RUNS))]
    src = np.repeat(np.arange(jobs.j), runs)[:j]
    if len(src) < j:
        raise ValueError(f"expand_arrays: {jobs.j} array jobs give {len(src)} < {j} pods")
    return Jobs(cpu=jobs.cpu[src], mem=jobs.mem[src], gpu=jobs.gpu[src], wall=jobs.wall[src],
                part=jobs.part[src], nodes_k=jobs.nodes_k[src])


def make_array_config(name: str, nodes: int | None = None, jobs: int | None = None):
    """``name`` in c2a / c3a / c5a: config c2 / c3 / c5's cluster with an array-expanded pending
    queue of the same length.  Returns make_config's (or make_c5's) tuple."""
    base = name[:-1]
    n, j, _p, _gh, _mn = CONFIGS[base]
    j = j if jobs is None else jobs
    seed = SEEDS[base]
    if base == "c5":
        nd, tl, jb, pt = make_c5(nodes, j // 4 + 64)
        return nd, tl, expand_arrays(seed, jb, j), pt
    nd, jb, pt = make_config(base, nodes, j // 4 + 64)
    return nd, expand_arrays(seed, jb, j), pt


def make_c5(nodes: int | None = None, jobs: int | None = None, shard: int = 0):
    """C5 (BASELINE.json config 5): C3's cluster shape plus the release timeline of the running
    jobs over a 1,024-slot horizon.  Returns (nodes, timeline, jobs, partitions)."""
    n, j, p, gh, mn = CONFIGS["c5"]
    seed = SEEDS["c5"]
    n = n if nodes is None else nodes
    j = j if jobs is None else jobs
    return (gen_nodes(seed, n, p, gh, start=shard * n),
            gen_releases(seed, n, C5_SLOTS, C5_SLOT_MIN, gh, start=shard * n),
            gen_jobs(seed, j, p, mn, start=shard * j), gen_partitions(seed, p))


def make_c1():
    """C1: 8 nodes × 100 copies of manifests/samples/kubecluster.org_v1alpha1_slurmbridgejob.yaml.

    The sample (yaml lines 12-25) has nodes=1, ntasks=3, cpusPerTask=1, memPerCpu=500 → per-node demand
    cpu=3, mem=1500 MiB (SPEC demand rule, pkg/slurm-bridge-operator/pod.go:143-162).  Nodes come from
    the synthetic ``scontrol show nodes`` fixture (64 CPUs / 256 GiB each, idle).
    """
    n = 8
    nodes = Nodes(
        cpu_free=np.full(n, 64, np.int32),
        mem_free=np.full(n, 262144, np.int32),
        gpu_free=np.zeros(n, np.int32),
        avail_min=np.full(n, INT32_MAX, np.int32),
        part_mask=np.ones(n, np.uint32),
    )
    j = 100
    jobs = Jobs(
        cpu=np.full(j, 3, np.int32),
        mem=np.full(j, 1500, np.int32),
        gpu=np.zeros(j, np.int32),
        wall=np.zeros(j, np.int32),
        part=np.zeros(j, np.uint16),
        nodes_k=np.ones(j, np.uint16),
    )
    parts = Partitions(np.full(1, -1, np.int32), np.full(1, -1, np.int32), np.full(1, -1, np.int32))
    return nodes, jobs, parts
