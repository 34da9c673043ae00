"""fit_release_events (include/fitgpu.h): release events for fit_load_timeline from the running
jobs a caller knows (the virtual kubelet's own pods: JobInfo.end_time / node_list,
workload.proto:252-292, and their demand).  Checked against a plain-Python restatement of the
header's rule on random inputs, plus the edge cases it names (CPU only)."""
import ctypes as C

import numpy as np
import pytest

import fitgpu
from fitgpu import _lib


def restated(n, jobs, slots, slot_min):
    """The header's rule, one event per (job, node), ordered by node, slot, job order."""
    ev = []
    for i, (nodes, rem, cpu, mem, gpu) in enumerate(jobs):
        s = 1 if rem <= 0 else -(-rem // slot_min)
        s = min(max(s, 1), slots)
        ev += [(x, s, i, cpu, mem, gpu) for x in nodes]
    ev.sort(key=lambda v: (v[0], v[1], v[2]))
    off = np.zeros(n + 1, np.int32)
    for v in ev:
        off[v[0] + 1] += 1
    return np.cumsum(off).astype(np.int32), [np.array([v[k] for v in ev], np.int32) for k in (1, 3, 4, 5)]


@pytest.mark.parametrize("seed", range(40))
def test_matches_restatement(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 40))
    slots, slot_min = int(rng.integers(1, 300)), int(rng.integers(1, 30))
    jobs = []
    for _ in range(int(rng.integers(0, 30))):
        k = int(rng.integers(1, min(n, 5) + 1))
        nodes = [int(x) for x in rng.choice(n, k, replace=False)]
        rem = int(rng.integers(-100, slots * slot_min + 500))
        jobs.append((nodes, rem, int(rng.integers(0, 64)), int(rng.integers(0, 1 << 20)), int(rng.integers(0, 9))))
    tl = fitgpu.release_events(n, jobs, slots, slot_min)
    off, cols = restated(n, jobs, slots, slot_min)
    assert np.array_equal(tl.off, off)
    for got, want in zip((tl.slot, tl.cpu, tl.mem, tl.gpu), cols):
        assert np.array_equal(got, want)
    assert (np.diff(tl.slot) >= 0)[np.repeat(np.arange(n), np.diff(tl.off))[1:] ==
                                    np.repeat(np.arange(n), np.diff(tl.off))[:-1]].all()


def test_edges():
    # past its end time: still held until the next slot; at / past the horizon: the horizon slot
    tl = fitgpu.release_events(3, [([0], 0, 1, 2, 3), ([0, 2], -5, 4, 5, 6), ([1], 10 ** 9, 7, 8, 9),
                                   ([2], 11, 1, 1, 0)], slots=8, slot_min=5)
    assert tl.off.tolist() == [0, 2, 3, 5]
    assert tl.slot.tolist() == [1, 1, 8, 1, 3]
    assert tl.cpu.tolist() == [1, 4, 7, 4, 1]
    empty = fitgpu.release_events(4, [], slots=4, slot_min=1)
    assert empty.off.tolist() == [0, 0, 0, 0, 0] and len(empty.slot) == 0


def _raw(n, off, nodes, rem, cpu, slots=4, slot_min=1, cap=None):
    m = len(off) - 1
    arr = lambda v, t=np.int32: np.array(v, t)
    off, nodes, rem, cpu = arr(off), arr(nodes if nodes else [0]), arr(rem, np.int64), arr(cpu)
    out = [np.zeros(n + 1, np.int32)] + [np.zeros(16, np.int32) for _ in range(4)]
    p = lambda a: C.c_void_p(a.ctypes.data)
    return _lib.lib().fit_release_events(n, m, p(off), p(nodes), p(rem), p(cpu), p(cpu), p(cpu), slots, slot_min,
                                         *[p(o) for o in out], 16 if cap is None else cap)


def test_invalid_inputs():
    assert _raw(2, [0, 1], [1], [3], [1]) == 1
    assert _raw(2, [0, 1], [2], [3], [1]) == _lib.FIT_E_INVAL       # node id out of range
    assert _raw(2, [0, 1], [-1], [3], [1]) == _lib.FIT_E_INVAL      # negative node id
    assert _raw(2, [0, 1], [0], [3], [-1]) == _lib.FIT_E_INVAL      # negative demand
    assert _raw(2, [1, 1], [0], [3], [1]) == _lib.FIT_E_INVAL       # job_off not starting at 0
    assert _raw(2, [0, 2, 1], [0, 1], [3, 3], [1, 1]) == _lib.FIT_E_INVAL  # decreasing job_off
    assert _raw(2, [0, 2], [0, 1], [3], [1], cap=1) == _lib.FIT_E_INVAL   # cap too small
    assert _raw(2, [0, 1], [0], [3], [1], slots=0) == _lib.FIT_E_INVAL
    assert _raw(2, [0, 1], [0], [3], [1], slot_min=0) == _lib.FIT_E_INVAL
