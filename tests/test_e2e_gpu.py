"""End-to-end and boundary-contract tests on the GPU (VERDICT r1 missing 3/4).

* C1 end to end (BASELINE config 1): `scontrol show nodes` / `show partition` text →
  fit_ingest_nodes / fit_parse_resources (pkg/slurm-agent/parse.go:111-190, :291-308), the sample
  SlurmBridgeJob (manifests/samples/kubecluster.org_v1alpha1_slurmbridgejob.yaml:12-25) →
  fit_extract_batch_resources → fit_apply_spec → fit_job_demand (pkg/slurm-bridge-operator/
  parse.go:30-69, pod.go:70-162), × 100 → fit_place, against the oracle on the same columns.
* fit_partition_free (the allocation-aware replacement of GetPartitionCapacity's sum,
  pkg/slurm-virtual-kubelet/node.go:183-190) against the oracle's final columns.
* Context-state contracts: a failed load leaves no usable node table; a read-only query does not
  change what fit_load_timeline builds from.
* The RCCL branch of the exchange on one GPU (FIT_FLAG_COLLECTIVES: one-rank communicator).
"""
import ctypes as C
import os

import numpy as np
import pytest

import fitgpu
from fitgpu import (FIT_FLAG_COLLECTIVES, FIT_SHARD_COMPONENTS, FIT_SHARD_NODES, Engine, FitError,
                    synth)
from fitgpu import _lib
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SAMPLE_SCRIPT = "#!/bin/sh\n#SBATCH --nodes=1\nsrun hostname\nhostname\npwd\nfor i in {1..5};do echo $i && sleep 15;done\n"
MIN_NS = 60 * 10**9


def _limit_min(ns):
    return -1 if ns < 0 else -(-ns // MIN_NS)


def _c1_inputs():
    nodes, names = fitgpu.ingest_nodes(open(os.path.join(GOLD, "c1_scontrol_show_nodes.txt")).read(), ["debug"])
    res = fitgpu.parse_resources(open(os.path.join(GOLD, "c1_scontrol_show_partition.txt")).read())
    parts = synth.Partitions(np.array([_limit_min(res.WallTime)], np.int32), np.array([res.CPUPerNode], np.int32),
                             np.array([res.MemPerNode], np.int32))
    r = fitgpu.apply_spec(fitgpu.extract_batch_resources(SAMPLE_SCRIPT), ntasks=3, mem_per_cpu=500,
                          cpus_per_task=1)  # spec fields of the sample (yaml:20-25)
    cpu, mem, wall, k = fitgpu.job_demand(r)
    j = 100
    jobs = synth.Jobs(np.full(j, cpu, np.int32), np.full(j, mem, np.int32), np.zeros(j, np.int32),
                      np.full(j, wall, np.int32), np.zeros(j, np.uint16), np.full(j, k, np.uint16))
    return nodes, names, jobs, parts


def test_c1_end_to_end():
    nodes, names, jobs, parts = _c1_inputs()
    assert names == [f"node{i}" for i in range(1, 9)]
    # the C1 fixture is the cluster synth.make_c1 describes
    n1, j1, p1 = synth.make_c1()
    for a, b in zip((nodes.cpu_free, nodes.mem_free, nodes.gpu_free, nodes.avail_min, nodes.part_mask),
                    (n1.cpu_free, n1.mem_free, n1.gpu_free, n1.avail_min, n1.part_mask)):
        assert np.array_equal(a, b)
    assert (jobs.cpu[0], jobs.mem[0], jobs.nodes_k[0]) == (3, 1500, 1)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs)
        fin = e.read_nodes()
        free = e.partition_free(0)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    assert np.array_equal(out, ref)
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert st["placed"] == 100
    # best fit packs node 0 first: 21 jobs of 3 cpus fill 63 of its 64, then node 1, ...
    assert out[:21, 0].tolist() == [0] * 21 and out[21, 0] == 1
    assert free == {"cpu": 8 * 64 - 300, "mem_mib": 8 * 262144 - 150000, "gpu": 0}


def test_mixed_fixture_end_to_end():
    """The 5-node fixture (GPU node, DOWN* and DRAIN nodes, two partitions) with a job mix."""
    text = open(os.path.join(GOLD, "scontrol_show_nodes.txt")).read()
    nodes, _ = fitgpu.ingest_nodes(text, ["debug", "gpu"])
    rng = np.random.default_rng(3)
    j = 400
    jobs = synth.Jobs(rng.integers(0, 9, j).astype(np.int32), rng.integers(0, 9000, j).astype(np.int32),
                      rng.integers(0, 2, j).astype(np.int32), np.zeros(j, np.int32),
                      rng.integers(0, 2, j).astype(np.uint16), np.ones(j, np.uint16))
    parts = synth.Partitions(np.full(2, -1, np.int32), np.full(2, -1, np.int32), np.full(2, -1, np.int32))
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, _ = e.place(jobs)
        fin = e.read_nodes()
    ref, _, rfin = po.ref_place(nodes, jobs, parts)
    assert np.array_equal(out, ref)
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert not np.isin(out[:, 0], [2, 3]).any()  # DOWN* / DRAIN nodes never take work


@pytest.mark.parametrize("name", ["c3", "c3o"])
def test_partition_free(name):
    nodes, jobs, parts = synth.make_config(name, 8000, 40000)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.place(jobs)
        got = [e.partition_free(p) for p in range(parts.p)]
    _, _, (fc, fm, fg) = po.ref_place(nodes, jobs, parts)
    for p in range(parts.p):
        member = ((nodes.part_mask >> np.uint32(p)) & 1).astype(bool)
        want = {"cpu": int(np.maximum(fc[member], 0).sum()), "mem_mib": int(np.maximum(fm[member], 0).sum()),
                "gpu": int(np.maximum(fg[member], 0).sum())}
        assert got[p] == want, p


def test_failed_load_leaves_no_node_table():
    nodes, jobs, parts = synth.make_config("c2", 512, 4096)
    big = (1 << 20) + 1  # one partition component above MAX_COMPONENT_NODES: FIT_E_INVAL late in the load
    col, mask = np.ones(big, np.int32), np.ones(big, np.uint32)  # kept alive across the call
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        rc = _lib.lib().fit_load_nodes(e._h, big, *(fitgpu._ptr(col) for _ in range(4)), fitgpu._ptr(mask))
        assert rc == _lib.FIT_E_INVAL, _lib.lib().fit_last_error()
        with pytest.raises(FitError) as ei:
            e.place(jobs)
        assert ei.value.code == _lib.FIT_E_STATE
        e.load_nodes(nodes)  # a good load makes the context usable again
        out, _ = e.place(jobs)
    ref, _, _ = po.ref_place(nodes, jobs, parts)
    assert np.array_equal(out, ref)


def test_read_nodes_does_not_change_timeline_source():
    nodes, tline, jobs, parts = synth.make_c5(512, 4096)

    def run(query):
        with Engine() as e:
            e.load_nodes(nodes)
            e.load_partitions(parts)
            e.place(jobs)  # plain fit consumes resources in the node rows
            if query:
                e.read_nodes()
                e.partition_free(0)
            e.load_timeline(tline)  # slot 0 = the table of the last fit_load_nodes
            return e.place_tl(jobs)[:2]

    a, b = run(False), run(True)
    rn, rs, _, _ = po.ref_place_tl(nodes, tline, jobs, parts)
    for x in (a, b):
        assert np.array_equal(x[0], rn) and np.array_equal(x[1], rs)


def test_partition_count_limit():
    with Engine() as e:
        t = np.full(33, -1, np.int32)
        assert _lib.lib().fit_load_partitions(e._h, 33, *(fitgpu._ptr(t) for _ in range(3))) == _lib.FIT_E_INVAL
        t = np.full(32, -1, np.int32)
        assert _lib.lib().fit_load_partitions(e._h, 32, *(fitgpu._ptr(t) for _ in range(3))) == 0


@pytest.mark.parametrize("mode", [FIT_SHARD_NODES, FIT_SHARD_COMPONENTS])
def test_rccl_exchange_one_rank(mode):
    """The RCCL calls of the sharded path (ncclAllGather, ncclAllReduce ncclMin/ncclMax) on real
    device buffers, through a one-rank communicator: placements identical to the oracle's."""
    nodes, jobs, parts = synth.make_config("c3", 4000, 20000)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    with Engine(flags=FIT_FLAG_COLLECTIVES, shard_mode=mode) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs)
        fin = e.read_nodes()
    assert st["shard_mode"] == mode
    assert np.array_equal(out, ref)
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))


def test_rccl_exchange_one_rank_backfill():
    nodes, tline, jobs, parts = synth.make_c5(1024, 4096)
    rn, rs, _, _ = po.ref_place_tl(nodes, tline, jobs, parts)
    with Engine(flags=FIT_FLAG_COLLECTIVES) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tline)
        node, start, st = e.place_tl(jobs)
    assert st["shard_mode"] == FIT_SHARD_NODES
    assert np.array_equal(node, rn) and np.array_equal(start, rs)
