"""The demand-class engine (k_class, csrc/fit_class.hip) — bit-exact against the
oracle (oracle/fitref.c ref_place) and the committed full-size digests.

FIT_ENGINE=class runs it at every size whenever the node table qualifies (one partition per
component, rows within one workgroup's LDS, <= 192 demand classes per component); otherwise the
placement goes to the persistent engine, which `engine` in the stats tells apart (3 = class)."""
import hashlib
import json
import os

import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
INT32_MAX = 2**31 - 1
HERE = os.path.dirname(__file__)
GOLD = json.load(open(os.path.join(HERE, "golden", "placements.json")))
GOLD_BIG = json.load(open(os.path.join(HERE, "golden", "placements_big.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _place(nodes, jobs, parts, kmax=1, **kw):
    with Engine(**kw) as e:
        e.load_partitions(parts)
        e.load_nodes(nodes)
        out, st = e.place(jobs, kmax=kmax)
        fin = e.read_nodes()
    return out, st, fin


def _check(nodes, jobs, parts, kmax=1, engine_id=3):
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    out, st, fin = _place(nodes, jobs, parts, kmax)
    assert st["engine"] == engine_id, st
    bad = np.flatnonzero((out != ref).any(axis=1))
    assert bad.size == 0, f"first mismatch at job {bad[0]}: {out[bad[0]]} vs {ref[bad[0]]}"
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])
    return st


@pytest.mark.parametrize("name,nn,jj,kmax", [("c3", 20000, 100000, 1), ("c2", 4096, 65536, 1),
                                              ("c4", 8192, 40000, 8), ("c3", 2000, 50000, 1),
                                              ("c4", 100000, 30000, 8)])
def test_class_matches_oracle(name, nn, jj, kmax, monkeypatch):
    monkeypatch.setenv("FIT_ENGINE", "class")
    nodes, jobs, parts = synth.make_config(name, nn, jj)
    _check(nodes, jobs, parts, kmax)


@pytest.mark.parametrize("name", ["c3a", "c2a"])
def test_class_arrays(name, monkeypatch):
    """Runs of identical pods (array jobs): consecutive jobs of one class."""
    monkeypatch.setenv("FIT_ENGINE", "class")
    nodes, jobs, parts = synth.make_array_config(name, 20000 if name == "c3a" else None, 60000)
    _check(nodes, jobs, parts)


@pytest.mark.parametrize("key", ["c2:4096x65536", "c3:100000x1000000"])
def test_class_golden(key, monkeypatch):
    monkeypatch.setenv("FIT_ENGINE", "class")
    name, size = key.split(":")
    nn, jj = (int(x) for x in size.split("x"))
    nodes, jobs, parts = synth.make_config(name, nn, jj)
    out, st, fin = _place(nodes, jobs, parts)
    g = GOLD[key]
    assert st["engine"] == 3
    assert sha(out[:, 0]) == g["placements_sha256"]
    assert sha(fin[0]) == g["final_cpu_sha256"]
    assert sha(fin[1]) == g["final_mem_sha256"]
    assert sha(fin[2]) == g["final_gpu_sha256"]
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])


@pytest.mark.parametrize("key", ["c4:100000x1000000", "c4a:100000x1000000", "c3a:100000x1000000"])
def test_class_golden_big(key, monkeypatch):
    monkeypatch.setenv("FIT_ENGINE", "class")
    g = GOLD_BIG[key]
    name = key.split(":")[0]
    if name.endswith("a"):
        nodes, jobs, parts = synth.make_array_config(name)
    else:
        nodes, jobs, parts = synth.make_config(name)
    kmax = g.get("kmax", 1)
    out, st, fin = _place(nodes, jobs, parts, kmax=kmax)
    assert st["engine"] == 3
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])
    assert sha(out if kmax > 1 else out[:, 0]) == g["placements_sha256"]
    assert sha(fin[0]) == g["final_cpu_sha256"]
    assert sha(fin[1]) == g["final_mem_sha256"]
    assert sha(fin[2]) == g["final_gpu_sha256"]


def random_case(seed):
    """Disjoint partitions (every node in at most one: the class engine's domain), few or many
    demand classes, finite availability on some nodes, zero and oversized demands, limits,
    multi-node jobs."""
    r = np.random.default_rng(seed)
    n = int(r.integers(1, 300 if r.random() < 0.4 else 8000))
    j = int(r.integers(1, 8000))
    p = int(r.integers(1, 6))
    cls = r.integers(0, 4, n)
    cpu = np.array([8, 32, 64, 128], np.int32)[cls] - r.integers(0, 8, n).astype(np.int32)
    mem = (np.array([16, 64, 256, 512], np.int32)[cls] * 1024 - r.integers(0, 4096, n)).astype(np.int32)
    gpu = np.where(r.random(n) < 0.3, r.integers(0, 9, n), 0).astype(np.int32)
    avail = np.where(r.random(n) < 0.2, r.integers(0, 3000, n), INT32_MAX).astype(np.int32)
    mask = (np.uint32(1) << r.integers(0, p, n).astype(np.uint32)).astype(np.uint32)
    mask[r.random(n) < 0.05] = 0
    nodes = synth.Nodes(cpu, mem, gpu, avail, mask)
    lim = lambda lo, hi: np.where(r.random(p) < 0.5, -1, r.integers(lo, hi, p)).astype(np.int32)  # noqa: E731
    parts = synth.Partitions(lim(30, 3000), lim(4, 100), lim(4096, 300000))
    kmax = int(r.choice([1, 2, 4, 8]))
    few = r.random() < 0.6  # a handful of shapes (labels), or many
    if few:
        shapes = np.stack([r.integers(0, 40, 12), r.integers(0, 64 * 1024, 12),
                           np.where(r.random(12) < 0.3, r.integers(0, 5, 12), 0)], axis=1)
        pick = shapes[r.integers(0, 12, j)]
        jc, jm, jg = (pick[:, i].astype(np.int32) for i in range(3))
    else:
        jc = r.integers(0, 40, j).astype(np.int32)
        jm = r.integers(0, 64 * 1024, j).astype(np.int32)
        jg = np.where(r.random(j) < 0.2, r.integers(0, 5, j), 0).astype(np.int32)
    jobs = synth.Jobs(jc, jm, jg, r.integers(0, 2880, j).astype(np.int32), r.integers(0, p, j).astype(np.uint16),
                      r.integers(1, kmax + 1, j).astype(np.uint16))
    return nodes, jobs, parts, kmax


@pytest.mark.parametrize("seed", range(48))
def test_class_fuzz(seed, monkeypatch):
    monkeypatch.setenv("FIT_ENGINE", "class")
    nodes, jobs, parts, kmax = random_case(5000 + seed)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    out, st, fin = _place(nodes, jobs, parts, kmax)
    bad = np.flatnonzero((out != ref).any(axis=1))
    assert bad.size == 0, f"seed {seed} engine {st['engine']}: first mismatch at job {bad[0]}: " \
                          f"{out[bad[0]]} vs {ref[bad[0]]}"
    for a, b in zip(fin, rfin):
        assert np.array_equal(a, b)
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])


@pytest.mark.auto_engine
def test_class_is_the_production_choice(monkeypatch):
    """FIT_CLASS=1, FIT_ENGINE unset: a large placement on single-partition components runs the
    class engine; overlapping partitions (c3o: one component) keep the persistent engine; without
    FIT_CLASS (automatic) a k = 1 queue runs the persistent engine; a small one stays on the
    rounds."""
    monkeypatch.delenv("FIT_ENGINE", raising=False)
    monkeypatch.setenv("FIT_CLASS", "1")
    nodes, jobs, parts = synth.make_config("c3", 20000, 40000)
    _check(nodes, jobs, parts, engine_id=3)
    nodes, jobs, parts = synth.make_config("c3o", 8000, 40000)
    _check(nodes, jobs, parts, engine_id=1)
    nodes, jobs, parts = synth.make_config("c3", 20000, 1500)
    _check(nodes, jobs, parts, engine_id=0)
    monkeypatch.delenv("FIT_CLASS", raising=False)
    nodes, jobs, parts = synth.make_config("c3", 20000, 40000)
    _check(nodes, jobs, parts, engine_id=1)


@pytest.mark.auto_engine
def test_class_is_the_default_for_multi_node_queues(monkeypatch):
    """FIT_CLASS and FIT_ENGINE unset: a large placement whose live jobs are mostly multi-node (C4:
    75 %) runs the class engine (its all-picks-at-once commit beats the single-wave commit there);
    FIT_CLASS=0 keeps the persistent engine; a k = 1 queue keeps it too (previous test)."""
    monkeypatch.delenv("FIT_ENGINE", raising=False)
    monkeypatch.delenv("FIT_CLASS", raising=False)
    nodes, jobs, parts = synth.make_config("c4", 8192, 30000)
    _check(nodes, jobs, parts, kmax=8, engine_id=3)
    monkeypatch.setenv("FIT_CLASS", "0")
    _check(nodes, jobs, parts, kmax=8, engine_id=1)


def test_class_consecutive_placements(monkeypatch):
    """Two placements on one context: the second sees the first's table (classes re-counted)."""
    monkeypatch.setenv("FIT_ENGINE", "class")
    nodes, jobs, parts = synth.make_config("c3", 20000, 80000)
    ref, _, rfin = po.ref_place(nodes, jobs, parts)
    with Engine() as e:
        e.load_partitions(parts)
        e.load_nodes(nodes)
        a = synth.Jobs(*(x[:30000] for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, jobs.nodes_k)))
        b = synth.Jobs(*(x[30000:] for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, jobs.nodes_k)))
        o1, s1 = e.place(a)
        o2, s2 = e.place(b)
        fin = e.read_nodes()
    assert s1["engine"] == 3 and s2["engine"] == 3
    assert np.array_equal(np.concatenate([o1, o2]), ref)
    assert all(np.array_equal(x, y) for x, y in zip(fin, rfin))
