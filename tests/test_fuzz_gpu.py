"""Randomised GPU parity: small clusters with random shapes the synthetic configurations do not
produce — overlapping and empty partition masks, nodes in no partition, zero and oversized
demands, partition limits, multi-node jobs up to kmax, tiny windows, timelines with random release
events — placed by the HIP engines and compared bit-exactly with the oracle (placements, start
slots, final node state / timelines).  Seeds are fixed, so a failure names its case.  Engines by seed: the persistent engine at every
size (conftest), the host-driven rounds (seed % 4 == 1), the direct small placement k_small at
every size (seed % 8 == 2), the production choice by size (seed % 4 == 3)."""
import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
INT32_MAX = 2**31 - 1


def random_case(seed, timeline=False):
    r = np.random.default_rng(seed)
    n = int(r.integers(1, 300 if r.random() < 0.5 else 3000))  # half the cases heavily contended
    j = int(r.integers(1, 6000))
    p = int(r.integers(1, 7))
    cls = r.integers(0, 4, n)
    cpu = np.array([8, 32, 64, 128], np.int32)[cls] - r.integers(0, 8, n).astype(np.int32)
    mem = (np.array([16, 64, 256, 512], np.int32)[cls] * 1024 - r.integers(0, 4096, n)).astype(np.int32)
    gpu = np.where(r.random(n) < 0.3, r.integers(0, 9, n), 0).astype(np.int32)
    avail = np.where(r.random(n) < 0.2, r.integers(0, 3000, n), INT32_MAX).astype(np.int32)
    mask = r.integers(0, 1 << p, n).astype(np.uint32)           # overlapping, some empty
    mask[r.random(n) < 0.05] = 0
    nodes = synth.Nodes(cpu, mem, gpu, avail, mask)
    lim = lambda lo, hi: np.where(r.random(p) < 0.5, -1, r.integers(lo, hi, p)).astype(np.int32)  # noqa: E731
    parts = synth.Partitions(lim(30, 3000), lim(4, 100), lim(4096, 300000))
    kmax = 1 if timeline else int(r.choice([1, 2, 4, 8]))
    jobs = synth.Jobs(r.integers(0, 40, j).astype(np.int32), r.integers(0, 64 * 1024, j).astype(np.int32),
                      np.where(r.random(j) < 0.2, r.integers(0, 5, j), 0).astype(np.int32),
                      r.integers(0, 2880, j).astype(np.int32), r.integers(0, p, j).astype(np.uint16),
                      r.integers(1, kmax + 1, j).astype(np.uint16))
    if not timeline:
        return nodes, jobs, parts, kmax
    slots, slot_min = int(r.choice([16, 64, 256, 1024])), int(r.choice([1, 5, 30]))
    ev = r.integers(0, 4, n)
    off = np.zeros(n + 1, np.int32)
    off[1:] = np.cumsum(ev)
    e = int(off[-1])
    slot = np.concatenate([np.sort(r.integers(-2, slots + 4, k)) for k in ev]).astype(np.int32) if e else \
        np.zeros(0, np.int32)
    tl = synth.Timeline(slots, slot_min, off, slot, r.integers(0, 16, e).astype(np.int32),
                        r.integers(0, 8192, e).astype(np.int32), r.integers(0, 2, e).astype(np.int32))
    jobs.nodes_k[:] = 1
    return nodes, tl, jobs, parts


@pytest.mark.parametrize("seed", range(64))
def test_fuzz_place(seed, monkeypatch):
    if seed % 4 == 1:  # the host-driven round loop (node-sharded multi-GPU's engine)
        monkeypatch.setenv("FIT_ENGINE", "rounds")
    elif seed % 8 == 2:  # k_small, the admission batches' one-launch placement, at every size
        monkeypatch.setenv("FIT_ENGINE", "direct")
    elif seed % 4 == 3:  # the production choice by size (direct / rounds / persistent)
        monkeypatch.delenv("FIT_ENGINE", raising=False)
    nodes, jobs, parts, kmax = random_case(seed)
    r = np.random.default_rng(1000 + seed)
    kw = {} if seed % 3 else {"window_min": int(r.integers(1, 64)), "window_max": int(r.integers(64, 2048))}
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    with Engine(**kw) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs, kmax=kmax)
        fin = e.read_nodes()
    bad = np.flatnonzero((out != ref).any(axis=1))
    assert bad.size == 0, f"seed {seed}: first mismatch at job {bad[0]}: {out[bad[0]]} vs {ref[bad[0]]}"
    for a, b in zip(fin, rfin):
        assert np.array_equal(a, b)
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])


@pytest.mark.parametrize("seed", range(32))
def test_fuzz_backfill(seed, monkeypatch):
    if seed % 4 == 1:
        monkeypatch.setenv("FIT_ENGINE", "rounds")
    elif seed % 4 == 3:
        monkeypatch.delenv("FIT_ENGINE", raising=False)
    nodes, tl, jobs, parts = random_case(100 + seed, timeline=True)
    rn, rs, rst, rfin = po.ref_place_tl(nodes, tl, jobs, parts)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tl)
        node, start, st = e.place_tl(jobs)
        fin = e.read_timeline()
    bad = np.flatnonzero((node != rn) | (start != rs))
    assert bad.size == 0, f"seed {seed}: first mismatch at job {bad[0]}: ({node[bad[0]]}, {start[bad[0]]}) " \
                          f"vs ({rn[bad[0]]}, {rs[bad[0]]})"
    live = nodes.part_mask != 0
    assert np.array_equal(fin[live], rfin[live])
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])
