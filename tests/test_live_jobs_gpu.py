"""The commit's live-job walk (DESIGN.md §3.7 "Live jobs only"): jobs that no node fits at their
round's start are skipped through the scan's per-tile feasibility masks, records index the
window's live jobs, and a record whose job index is the window size ends the window.  These
cases put the skip's edges on the GPU against the oracle (bit-exact placements and node state):
windows with no live job at all (the end record at index 0), whole job tiles skipped by the
cursor, live jobs only in a window's last tile, alternating live / dead jobs, and jobs that die
during the round (not skippable: the normal path resolves them)."""
import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def _nodes(n, seed):
    rng = np.random.default_rng(seed)
    return synth.Nodes(cpu_free=rng.integers(4, 33, n).astype(np.int32),
                       mem_free=rng.integers(4096, 65537, n).astype(np.int32),
                       gpu_free=rng.integers(0, 5, n).astype(np.int32),
                       avail_min=np.full(n, 2**31 - 1, np.int32),
                       part_mask=np.where(np.arange(n) % 5 == 0, 3, 1).astype(np.uint32))


def _jobs(live_mask, seed, part=None):
    """live_mask[j]: the job fits somewhere at the start (small demand) or never (cpu 10,000)."""
    rng = np.random.default_rng(seed)
    j = live_mask.size
    cpu = np.where(live_mask, rng.integers(1, 9, j), 10_000)
    return synth.Jobs(cpu=cpu.astype(np.int32), mem=rng.integers(100, 4000, j).astype(np.int32),
                      gpu=np.where(rng.random(j) < 0.2, 1, 0).astype(np.int32),
                      wall=rng.integers(1, 500, j).astype(np.int32),
                      part=(np.zeros(j, np.uint16) if part is None else part),
                      nodes_k=np.ones(j, np.uint16))


def _check(nodes, jobs, **kw):
    parts = synth.Partitions(np.array([-1, -1], np.int32), np.array([-1, -1], np.int32),
                             np.array([-1, -1], np.int32))
    with Engine(device=0, **kw) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs)
        fin = e.read_nodes()
    ref, _, rfin = po.ref_place(nodes, jobs, parts)
    assert np.array_equal(out, ref), "placements differ from the oracle"
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin)), "node state differs from the oracle"
    return np.asarray(out).reshape(jobs.j, -1)[:, 0], st


WINDOWS = [dict(), dict(window_min=64, window_max=64), dict(window_min=256, window_max=256),
           dict(window_min=1, window_max=8)]


@pytest.mark.parametrize("kw", WINDOWS)
def test_no_live_job(kw):
    """Every job is dead at every round start: the end record comes first in every window."""
    live = np.zeros(3000, bool)
    out, st = _check(_nodes(512, 1), _jobs(live, 2), **kw)
    assert (out == -1).all() and st["unplaced"] == 3000


@pytest.mark.parametrize("kw", WINDOWS)
def test_dead_tiles_between_live_runs(kw):
    """Runs of dead jobs spanning whole 64-job tiles between short live runs, and a live run only
    in a window's last tile."""
    live = np.zeros(5000, bool)
    for a, b in [(0, 3), (200, 260), (777, 778), (1500, 1563), (4990, 5000)]:
        live[a:b] = True
    out, _ = _check(_nodes(1024, 3), _jobs(live, 4), **kw)
    assert (out[~live] == -1).all() and (out[live] >= 0).any()


@pytest.mark.parametrize("kw", WINDOWS)
def test_alternating_live_dead(kw):
    live = (np.arange(4096) % 2) == 1
    _check(_nodes(256, 5), _jobs(live, 6), **kw)


@pytest.mark.parametrize("kw", WINDOWS[:2])
def test_jobs_dying_inside_the_round(kw):
    """Small cluster, many live jobs: most die during a round (not at its start) and are resolved
    by the decider; some are dead from the start and skipped."""
    rng = np.random.default_rng(7)
    live = rng.random(6000) < 0.9
    part = np.where(rng.random(6000) < 0.3, 1, 0).astype(np.uint16)
    out, st = _check(_nodes(64, 8), _jobs(live, 9, part), **kw)
    assert st["unplaced"] > (~live).sum()  # jobs that died during their round too
