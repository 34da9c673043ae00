"""Array-expanded pending queues (synth.expand_arrays) on the CPU: the generator's shape, and the
CPU paths the bench times (oracle/cpu_baseline.c, oracle/cpu_fast.c) against oracle/fitref.c on
such a queue (runs of identical demands)."""
import numpy as np

from fitgpu import synth
from oracle import pyoracle as po


def _runs(jobs):
    c = np.stack([jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part.astype(np.int32),
                  jobs.nodes_k.astype(np.int32)]).T
    cut = np.flatnonzero(np.any(c[1:] != c[:-1], axis=1)) + 1
    return np.diff(np.concatenate([[0], cut, [len(c)]]))


def test_expand_arrays_shape():
    nodes, jobs, parts = synth.make_array_config("c2a")
    assert (nodes.n, jobs.j) == (4096, 65536)
    r = _runs(jobs)
    assert r.max() <= 32 and 6 < r.mean() < 12  # tasks per array job 1..32, mean 9 (adjacent equal
    # array jobs merge into one run, so a run may exceed 32 only by chance: checked not to here)
    a, b = synth.make_array_config("c2a"), synth.make_array_config("c2a")
    assert all(np.array_equal(x, y) for x, y in zip(a[1].__dict__.values(), b[1].__dict__.values()))
    # prefix property: a shorter queue is the first jobs of a longer one
    _, j2, _ = synth.make_array_config("c3a", 1000, 5000)
    _, j3, _ = synth.make_array_config("c3a", 1000, 20000)
    assert np.array_equal(j2.cpu, j3.cpu[:5000]) and np.array_equal(j2.part, j3.part[:5000])


def test_cpu_paths_on_array_stream():
    nodes, jobs, parts = synth.make_array_config("c3a", 2000, 12000)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    out, st, fin = po.cpu_place(nodes, jobs, parts, threads=4)
    assert np.array_equal(np.asarray(out).reshape(-1), ref[:, 0])
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))


def test_cpu_backfill_on_array_stream():
    nodes, tline, jobs, parts = synth.make_array_config("c5a", 1024, 3000)
    rn, rs, _, rtl = po.ref_place_tl(nodes, tline, jobs, parts)
    n, s, _, tl = po.cpu_place_tl(nodes, tline, jobs, parts, threads=4, rle=True)
    assert np.array_equal(n, rn) and np.array_equal(s, rs)
