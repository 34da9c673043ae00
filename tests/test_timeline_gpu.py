"""GPU parity for SPEC §2b (time-windowed backfill, BASELINE config C5): the HIP engine
(k_scan_tl / k_commit_tl) vs the dense-timeline oracle (oracle/fitref_tl.c) — bit-exact node,
start slot and final timelines at sizes the oracle runs in seconds; full C5 (100k nodes × 1M jobs)
through size-independent properties (the oracle needs ~1.5 h there)."""
import numpy as np
import pytest

from _tl_cases import EXPECT_NODE, EXPECT_START, hand_case
from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def run_tl(nodes, tline, jobs, parts, **kw):
    with Engine(**kw) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tline)
        node, start, st = e.place_tl(jobs)
        fin = e.read_timeline()
    return node, start, st, fin


def check_tl(nodes, tline, jobs, parts, **kw):
    rn, rs, rst, rfin = po.ref_place_tl(nodes, tline, jobs, parts)
    node, start, st, fin = run_tl(nodes, tline, jobs, parts, **kw)
    bad = np.flatnonzero((node != rn) | (start != rs))
    assert bad.size == 0, f"first mismatch at job {bad[0]}: gpu ({node[bad[0]]}, {start[bad[0]]}) " \
                          f"oracle ({rn[bad[0]]}, {rs[bad[0]]})"
    live = nodes.part_mask != 0  # rows outside every partition are not on the device
    assert np.array_equal(fin[live], rfin[live])
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])
    return st


def test_hand_case():
    node, start, st, fin = run_tl(*hand_case())
    assert np.array_equal(node, EXPECT_NODE) and np.array_equal(start, EXPECT_START)
    check_tl(*hand_case())


@pytest.mark.parametrize("engine", ["persistent", "rounds"])
@pytest.mark.parametrize("nn,jj", [(64, 1024), (256, 4096), (1024, 16384), (4096, 16384)])
def test_c5(nn, jj, engine, monkeypatch):
    """persistent: one k_engine_tl launch; rounds: host-driven k_scan_tl / k_commit_tl."""
    monkeypatch.setenv("FIT_ENGINE", engine)
    nodes, tline, jobs, parts = synth.make_c5(nn, jj)
    check_tl(nodes, tline, jobs, parts)


@pytest.mark.parametrize("engine", ["persistent", "rounds"])
@pytest.mark.parametrize("wmin,wmax", [(1, 1), (1, 8), (64, 64), (512, 65536)])
def test_c5_window_policies(wmin, wmax, engine, monkeypatch):
    monkeypatch.setenv("FIT_ENGINE", engine)
    nodes, tline, jobs, parts = synth.make_c5(256, 4096)
    check_tl(nodes, tline, jobs, parts, window_min=wmin, window_max=wmax)


@pytest.mark.parametrize("engine", ["persistent", "rounds"])
def test_c5_full_nodes_prefix(engine, monkeypatch):
    """All 100k nodes, the first 2,000 jobs (a prefix is exact: later jobs never affect earlier)."""
    monkeypatch.setenv("FIT_ENGINE", engine)
    nodes, tline, jobs, parts = synth.make_c5(None, 2000)
    check_tl(nodes, tline, jobs, parts)


@pytest.mark.parametrize("nn,jj", [(256, 4096), (4096, 16384), (None, 2000)])
def test_c5_split_launch(nn, jj, monkeypatch):
    """FIT_TL_SPLIT: committers and scan workers as two concurrent launches (host waits for the
    committers' residency flag before launching the workers) — same placements as the oracle."""
    monkeypatch.setenv("FIT_ENGINE", "persistent")
    monkeypatch.setenv("FIT_TL_SPLIT", "1")
    nodes, tline, jobs, parts = synth.make_c5(nn, jj)
    check_tl(nodes, tline, jobs, parts)


def test_gpu_contention_future_starts():
    """GPU-heavy jobs on few GPU nodes: most starts are in the future (the backfill path)."""
    nodes, tline, jobs, parts = synth.make_c5(128, 4096)
    jobs.gpu[:] = np.where(np.arange(jobs.j) % 3 == 0, 1 + np.arange(jobs.j) % 4, 0).astype(np.int32)
    st = check_tl(nodes, tline, jobs, parts)
    assert st["placed"] > 0


def test_edge_cases():
    nodes, tline, jobs, parts = synth.make_c5(96, 2048)
    nodes.part_mask[::7] = 0                       # nodes outside every partition
    nodes.cpu_free[::11] = -5                      # over-allocated now (clamped to -1)
    nodes.avail_min[::5] = np.arange(0, 600, 30)[: len(nodes.avail_min[::5])]  # short availability
    jobs.cpu[::13] = 0
    jobs.mem[::13] = 0                             # zero-demand jobs
    jobs.wall[::17] = 0                            # zero walltime: one slot
    jobs.wall[::19] = 5121                         # 1,025 slots > horizon: unplaced
    check_tl(nodes, tline, jobs, parts)


def test_no_releases_and_empty_jobs():
    nodes, tline, jobs, parts = synth.make_c5(64, 512)
    empty = synth.Timeline(tline.slots, tline.slot_min, np.zeros(nodes.n + 1, np.int32),
                           *(np.zeros(0, np.int32) for _ in range(4)))
    check_tl(nodes, empty, jobs, parts)
    none = synth.Jobs(*(a[:0] for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, jobs.nodes_k)))
    node, start, st, fin = run_tl(nodes, empty, none, parts)
    assert node.size == 0 and st["placed"] == 0


def test_c5_full_properties():
    """Full C5, 100k nodes × 1M jobs: every reservation lies inside its node's availability and
    partition, the final timelines equal the initial ones minus the reservations (conservation),
    and no slot of a used node goes below zero."""
    nodes, tline, jobs, parts = synth.make_c5()
    node, start, st, fin = run_tl(nodes, tline, jobs, parts)
    ok = node >= 0
    assert st["placed"] == int(ok.sum()) and st["placed"] > 0.6 * jobs.j
    assert np.all((nodes.part_mask[node[ok]] >> jobs.part[ok].astype(np.uint32)) & 1)
    d = np.maximum(1, -(-jobs.wall.astype(np.int64) // tline.slot_min))
    assert np.all(start[ok] + d[ok] <= tline.slots)
    # conservation, through a difference array over (node, slot)
    init = po.ref_build_timeline(nodes, tline).astype(np.int64)
    delta = np.zeros((nodes.n, tline.slots + 1, 3), np.int64)
    dem = np.stack([jobs.cpu, jobs.mem, jobs.gpu], axis=1).astype(np.int64)
    np.add.at(delta, (node[ok], start[ok]), dem[ok])
    np.add.at(delta, (node[ok], start[ok] + d[ok]), -dem[ok])
    used = np.cumsum(delta, axis=1)[:, :-1]
    live = nodes.part_mask != 0
    assert np.array_equal(fin[live].astype(np.int64), (init - used)[live])
    assert (fin[used.any(axis=2)] >= 0).all()
