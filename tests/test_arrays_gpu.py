"""Array-expanded pending queues on the GPU ("add a workload with array-expanded
streams").  `--array=1-N` turns one SlurmBridgeJob into N identical pods (fit_array_tasks), so the
queue holds runs of identical demands (synth.expand_arrays: 1-32 tasks, mean 9).  Identical jobs
in a row are the case where the winner of job t is again the winner of job t + 1 while it still
fits, and where a window's jobs share every candidate list — placements, start slots and final
node state must still equal the oracle's (oracle/fitref.c ref_place, oracle/fitref_tl.c
ref_place_tl) bit for bit.  Full-size c3a / c4a / c5a digests: tests/golden/placements_big.json
(tools/make_golden_big.py, the same oracles)."""
import hashlib
import json
import os

import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "placements_big.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _place(nodes, jobs, parts, kmax=1):
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs, kmax=kmax)
        return out, st, e.read_nodes()


@pytest.mark.parametrize("name,nn,jj,kmax", [("c2a", None, None, 1), ("c3a", 20000, 100000, 1),
                                             ("c4a", 8192, 30000, 8)])
def test_array_stream_vs_oracle(name, nn, jj, kmax):
    nodes, jobs, parts = synth.make_array_config(name, nn, jj)
    out, st, fin = _place(nodes, jobs, parts, kmax)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    assert np.array_equal(out, ref)
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])


def test_array_stream_backfill_vs_oracle():
    nodes, tline, jobs, parts = synth.make_array_config("c5a", 4096, 16384)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tline)
        node, start, st = e.place_tl(jobs)
        tl = e.read_timeline()
    rn, rs, rst, rtl = po.ref_place_tl(nodes, tline, jobs, parts)
    assert np.array_equal(node, rn) and np.array_equal(start, rs)
    assert np.array_equal(tl, rtl)
    assert st["placed"] == rst["placed"]


@pytest.mark.parametrize("name", ["c3a", "c4a"])
def test_array_full_digest(name):
    key = f"{name}:100000x1000000"
    if key not in GOLD:
        pytest.skip(f"{key}: digest not generated (tools/make_golden_big.py {name})")
    g = GOLD[key]
    nodes, jobs, parts = synth.make_array_config(name)
    out, st, fin = _place(nodes, jobs, parts, g["kmax"])
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])
    assert sha(out) == g["placements_sha256"]
    assert [sha(x) for x in fin] == [g["final_cpu_sha256"], g["final_mem_sha256"], g["final_gpu_sha256"]]


def test_array_full_digest_backfill():
    key = "c5a:100000x1000000"
    if key not in GOLD:
        pytest.skip(f"{key}: digest not generated (tools/make_golden_big.py c5a)")
    g = GOLD[key]
    nodes, tline, jobs, parts = synth.make_array_config("c5a")
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tline)
        node, start, st = e.place_tl(jobs)
        tl = e.read_timeline()
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])
    assert sha(node) == g["node_sha256"] and sha(start) == g["start_sha256"]
    assert [sha(tl[..., i]) for i in range(3)] == [g["final_cpu_sha256"], g["final_mem_sha256"],
                                                   g["final_gpu_sha256"]]


def test_wide_first_tile_cuts_rounds():
    """A run of identical jobs drains a 4-key first tile's bound within a few jobs (a rescan inside
    the first tile); k_engine then scans the next rounds' first tiles with FIT_K0W keys (DESIGN.md
    §3.6). c2a: 79 rounds without it, 47 with it (profiles/r04_arrays_firsttile_ab.txt) — and the
    placements stay the oracle's."""
    nodes, jobs, parts = synth.make_array_config("c2a")
    out, st, _ = _place(nodes, jobs, parts)
    assert st["rounds"] <= 60, st
    ref, _, _ = po.ref_place(nodes, jobs, parts)
    assert np.array_equal(out, ref)
