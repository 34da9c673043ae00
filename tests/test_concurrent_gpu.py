"""Several placement contexts on ONE GPU at the same time.

The f4 deployment runs one virtual kubelet — and so one engine context — per Slurm partition
(pkg/configurator/configurator.go:151-171); on a shared GPU their placements may overlap.  Each
persistent launch (k_engine / k_engine_tl) sizes its grid to the whole chip and relies on its own
committer blocks being resident while its workers spin, so two or three of them side by side
must neither deadlock (the watchdog would trip: FIT_E_HIP) nor change any placement.  Contexts
place from separate threads (ctypes drops the GIL), every result bit-exact vs the oracle of record
(oracle/fitref.c ref_place, oracle/fitref_tl.c ref_place_tl: 6.6 s / 2.3 s of CPU for these
sizes)."""
import threading

import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def _place_many(workloads, rounds):
    """Each workload on its own context and thread, `rounds` placements each, all threads released
    together; returns per workload the list of (out, final columns) or the exception."""
    res = [[] for _ in workloads]
    bar = threading.Barrier(len(workloads))

    def run(i):
        kind, args = workloads[i]
        try:
            with Engine(device=0) as e:
                if kind == "fit":
                    nodes, jobs, parts = args
                    e.load_partitions(parts)
                    for _ in range(rounds):
                        e.load_nodes(nodes)
                        bar.wait(timeout=120)
                        out, _ = e.place(jobs)
                        res[i].append((out[:, 0].copy(), e.read_nodes()))
                else:
                    nodes, tline, jobs, parts = args
                    e.load_partitions(parts)
                    for _ in range(rounds):
                        e.load_nodes(nodes)
                        e.load_timeline(tline)
                        bar.wait(timeout=120)
                        node, start, _ = e.place_tl(jobs)
                        res[i].append((node.copy(), start.copy()))
        except Exception as x:  # surfaced below
            res[i].append(x)
            bar.abort()

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(workloads))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a placement thread hung"
    for r in res:
        for x in r:
            if isinstance(x, Exception):
                raise x
    return res


@pytest.mark.parametrize("contexts", [2, 3])
def test_concurrent_contexts_c3_prefix(contexts):
    """`contexts` C3-prefix placements (different seeds' shards, 16 components each) at once."""
    wl, refs = [], []
    for s in range(contexts):
        nodes, jobs, parts = synth.make_config("c3", 20000, 60000, shard=s)
        wl.append(("fit", (nodes, jobs, parts)))
        ref, _, fin = po.ref_place(nodes, jobs, parts)
        ref = ref[:, 0]
        refs.append((ref, fin))
    res = _place_many(wl, rounds=3)
    for (ref, fin), runs in zip(refs, res):
        assert len(runs) == 3
        for out, got in runs:
            assert np.array_equal(out, ref)
            assert all(np.array_equal(a, b) for a, b in zip(got, fin))


def test_concurrent_contexts_mixed_fit_and_backfill():
    """A plain placement and a backfill placement on the same GPU at once (k_engine beside
    k_engine_tl), plus a one-component C3o prefix (its one committer beside the others')."""
    n1, j1, p1 = synth.make_config("c3", 20000, 60000, shard=1)
    n2, t2, j2, p2 = synth.make_c5(4096, 16384)
    n3, j3, p3 = synth.make_config("c3o", 8192, 30000)
    r1 = po.ref_place(n1, j1, p1)[0][:, 0]
    r2n, r2s, _, _ = po.ref_place_tl(n2, t2, j2, p2)
    r3 = po.ref_place(n3, j3, p3)[0][:, 0]
    res = _place_many([("fit", (n1, j1, p1)), ("tl", (n2, t2, j2, p2)), ("fit", (n3, j3, p3))], rounds=2)
    for out, _ in res[0]:
        assert np.array_equal(out, r1)
    for node, start in res[1]:
        assert np.array_equal(node, r2n) and np.array_equal(start, r2s)
    for out, _ in res[2]:
        assert np.array_equal(out, r3)
