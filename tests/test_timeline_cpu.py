"""SPEC §2b oracle (oracle/fitref_tl.c) on CPU: the hand-worked case, the timeline build, and the
C5 generator.  The reference has no backfill: parity unpinned vs the reference,
pinned here by the hand-computed placements and an independent pure-Python slot walk."""
import numpy as np

from _tl_cases import EXPECT_NODE, EXPECT_START, hand_case
from fitgpu import synth
from oracle import pyoracle as po


def test_hand_case():
    node, start, st, fin = po.ref_place_tl(*hand_case())
    assert np.array_equal(node, EXPECT_NODE) and np.array_equal(start, EXPECT_START)
    assert (st["placed"], st["unplaced"], st["rejected"]) == (4, 2, 1)
    assert fin[0, :, 0].tolist() == [0, 0, 0, 4, 4, 4, 8, 8]
    assert fin[1, :, 0].tolist() == [0, 0, 0, 1, 2, -1, -1, -1]


def py_place_tl(nodes, tline, jobs, parts):
    """Independent pure-Python restatement (small cases): numpy windows, no shared code."""
    tl = po.ref_build_timeline(nodes, tline).astype(np.int64)
    H, L = tline.slots, tline.slot_min
    out_n, out_s = [], []
    for q in range(jobs.j):
        p = int(jobs.part[q])
        mt = int(parts.max_time_min[p]) if p < parts.p else 0
        if p >= parts.p or (mt >= 0 and jobs.wall[q] > mt):
            out_n.append(-2)
            out_s.append(-1)
            continue
        d = max(1, -(-int(jobs.wall[q]) // L))
        dem = np.array([jobs.cpu[q], jobs.mem[q], jobs.gpu[q]], np.int64)
        best = None
        for x in range(nodes.n):
            if not (int(nodes.part_mask[x]) >> p) & 1 or d > H:
                continue
            ok = (tl[x] >= dem).all(axis=1)
            for s in range(H - d + 1):
                if ok[s:s + d].all():
                    w = tl[x, s:s + d].min(axis=0) - dem
                    sc = (min(w[2], 255) << 24) | (min(w[0], 4095) << 12) | min(w[1] >> 10, 4095)
                    k = (s, sc, x)
                    best = k if best is None or k < best else best
                    break
        if best is None:
            out_n.append(-1)
            out_s.append(-1)
            continue
        s, _, x = best
        tl[x, s:s + d] -= dem
        out_n.append(x)
        out_s.append(s)
    return np.array(out_n, np.int32), np.array(out_s, np.int32), tl


def test_oracle_matches_python_restatement():
    nodes, tline, jobs, parts = synth.make_c5(24, 300)
    tline.slots = 64  # keep the Python walk small; releases past the horizon are ignored
    jobs.wall[:] = np.minimum(jobs.wall, 200)
    node, start, _, fin = po.ref_place_tl(nodes, tline, jobs, parts)
    pn, ps, pfin = py_place_tl(nodes, tline, jobs, parts)
    assert np.array_equal(node, pn) and np.array_equal(start, ps)
    assert np.array_equal(fin, pfin)


def test_build_timeline_matches_events():
    nodes, tline, jobs, parts = synth.make_c5(50, 1)
    tl = po.ref_build_timeline(nodes, tline)
    for x in range(nodes.n):
        u = min(tline.slots, int(nodes.avail_min[x]) // tline.slot_min)
        ev = slice(tline.off[x], tline.off[x + 1])
        for t in (0, 1, 300, 1023):
            want = np.array([nodes.cpu_free[x], nodes.mem_free[x], nodes.gpu_free[x]], np.int64)
            m = tline.slot[ev] <= t
            want += np.array([tline.cpu[ev][m].sum(), tline.mem[ev][m].sum(), tline.gpu[ev][m].sum()])
            want = np.clip(want, -1, 2**31 - 1) if t < u else np.full(3, -1)
            assert tl[x, t].tolist() == want.tolist()


def test_c5_generator_shape():
    nodes, tline, jobs, parts = synth.make_c5(1000, 10)
    assert tline.off[0] == 0 and tline.off[-1] == len(tline.slot) and np.all(np.diff(tline.off) >= 1)
    for x in range(0, 1000, 37):
        s = tline.slot[tline.off[x]:tline.off[x + 1]]
        assert np.all(np.diff(s) >= 0) and np.all((s >= 1) & (s < tline.slots))
    # the releases add back exactly the allocation gen_nodes subtracted: at the end of the horizon
    # every (always available) node is whole again
    tl = po.ref_build_timeline(nodes, tline)
    full = nodes.avail_min == 2**31 - 1
    cpus = tl[full, -1, 0]
    assert set(np.unique(cpus)) <= set(synth.NODE_CPUS.tolist())


def test_invalid_releases_rejected():
    nodes, tline, jobs, parts = hand_case()
    bad = synth.Timeline(8, 10, np.array([0, 2, 2, 2], np.int32), np.array([5, 3], np.int32),
                         np.array([1, 1], np.int32), np.zeros(2, np.int32), np.zeros(2, np.int32))
    try:
        po.ref_build_timeline(nodes, bad)
    except ValueError:
        return
    raise AssertionError("unsorted release slots must be rejected")
