"""The reference's own test tables, carried through the GPU placement (the
reference-pinned checks lived only in CPU tests, which the `-m gpu` run deselects).

* Test_parseResources (pkg/slurm-agent/parse_test.go:224-258): each `scontrol show partition`
  text of the table goes through the product's fit_parse_resources; the parsed limits (MaxTime,
  MaxCPUsPerNode, MaxMemPerNode — the table's expected values, asserted first) become the
  partition row of a GPU placement whose jobs straddle every limit.  Placement and rejections are
  compared with the oracle, and each rejection with the reference's own limit values.
* TestParseDuration (parse_test.go:26-122): every duration the table accepts becomes a job's
  walltime (minutes, rounded up like fit_job_demand); the table's "unlimited" cases become an
  unlimited partition.  Jobs longer than the 30-minute MaxTime of the first table entry must be
  FIT_REJECTED, the others placed or unplaced exactly as the oracle says.
"""
import json
import os

import numpy as np
import pytest

import fitgpu
from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))
MIN_NS = 60 * 10**9


def _limit_min(ns):
    return -1 if ns < 0 else -(-ns // MIN_NS)


def _nodes(n, seed=7):
    rng = np.random.default_rng(seed)
    return synth.Nodes(cpu_free=rng.integers(0, 9, n).astype(np.int32),
                       mem_free=rng.integers(0, 2049, n).astype(np.int32),
                       gpu_free=rng.integers(0, 3, n).astype(np.int32),
                       avail_min=np.where(rng.random(n) < 0.8, 2**31 - 1, rng.integers(1, 200, n)).astype(np.int32),
                       part_mask=np.ones(n, np.uint32))


def _place_both(nodes, jobs, parts):
    with Engine(device=0) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, _ = e.place(jobs)
        fin = e.read_nodes()
    ref, _, rfin = po.ref_place(nodes, jobs, parts)
    assert np.array_equal(out, ref), "placements differ from the oracle"
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin)), "node state differs from the oracle"
    return np.asarray(out).reshape(jobs.j, -1)[:, 0]  # kmax 1: the node of each job


@pytest.mark.parametrize("i", range(len(GOLD["parse_resources"])))
def test_parse_resources_table_through_placement(i):
    case = GOLD["parse_resources"][i]
    r = fitgpu.parse_resources(case["in"])
    w = case["want"]
    assert (r.Nodes, r.MemPerNode, r.CPUPerNode, r.WallTime) == (w["nodes"], w["mem_per_node"],
                                                                 w["cpu_per_node"], w["wall_ns"])
    tmax, cmax, mmax = _limit_min(r.WallTime), r.CPUPerNode, r.MemPerNode
    parts = synth.Partitions(np.array([tmax], np.int32), np.array([cmax], np.int32), np.array([mmax], np.int32))
    # jobs at, just under and just over each limit (unlimited limits: a large value instead)
    rng = np.random.default_rng(100 + i)
    n = 2048
    edge = lambda lim, big: np.array([lim - 1, lim, lim + 1] if lim >= 0 else [big // 2, big, 2 * big])
    cpu = rng.choice(np.maximum(edge(cmax, 4), 0), n)
    mem = rng.choice(np.maximum(edge(mmax, 1024), 0), n)
    wall = rng.choice(np.maximum(edge(tmax, 120), 1), n)
    jobs = synth.Jobs(cpu=cpu.astype(np.int32), mem=mem.astype(np.int32), gpu=rng.integers(0, 2, n).astype(np.int32),
                      wall=wall.astype(np.int32), part=np.zeros(n, np.uint16), nodes_k=np.ones(n, np.uint16))
    out = _place_both(_nodes(256), jobs, parts)
    over = ((tmax >= 0) & (jobs.wall > tmax)) | ((cmax >= 0) & (jobs.cpu > cmax)) | ((mmax >= 0) & (jobs.mem > mmax))
    assert np.array_equal(out == -2, over), "rejections differ from the reference's limits"
    assert (out >= 0).any()


def test_parse_duration_table_through_placement():
    # the first Test_parseResources entry: MaxTime=30 (minutes)
    r = fitgpu.parse_resources(GOLD["parse_resources"][0]["in"])
    tmax = _limit_min(r.WallTime)
    assert tmax == 30
    walls, unlimited = [], 0
    for case in GOLD["parse_duration"]:
        if case["ns"] is None:
            exc = fitgpu.ErrDurationIsUnlimited if case["unlimited"] else ValueError
            with pytest.raises(exc):
                fitgpu.ParseDuration(case["in"])
            unlimited += case["unlimited"]
            continue
        ns = fitgpu.ParseDuration(case["in"])
        assert ns == case["ns"]
        walls.append(_limit_min(ns))  # minutes, rounded up (fit_job_demand)
    assert unlimited == 2 and len(walls) == sum(c["ns"] is not None for c in GOLD["parse_duration"]) == 6
    n = 64 * len(walls)
    wall = np.tile(np.array(walls, np.int32), 64)
    # two partitions: MaxTime from the table (0) and unlimited (1, the "UNLIMITED" / "" cases)
    parts = synth.Partitions(np.array([tmax, -1], np.int32), np.array([-1, -1], np.int32), np.array([-1, -1], np.int32))
    part = (np.arange(n) % 2).astype(np.uint16)
    jobs = synth.Jobs(cpu=np.ones(n, np.int32), mem=np.full(n, 100, np.int32), gpu=np.zeros(n, np.int32),
                      wall=wall, part=part, nodes_k=np.ones(n, np.uint16))
    nodes = _nodes(128, seed=11)
    nodes.part_mask[:] = 3
    nodes.avail_min[:] = 2**31 - 1
    out = _place_both(nodes, jobs, parts)
    assert np.array_equal(out == -2, (part == 0) & (wall > tmax))
    assert ((out >= 0) | (out == -1))[part == 1].all()
