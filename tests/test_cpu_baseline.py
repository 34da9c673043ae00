"""The fair CPU baselines bench.py times (oracle/cpu_baseline.c: component-aware scan, components
on several threads) give exactly the oracle's results (oracle/fitref.c:ref_place,
oracle/fitref_tl.c:ref_place_tl) — so their throughput is a like-for-like baseline."""
import numpy as np
import pytest

from fitgpu import synth
from oracle import pyoracle as po


@pytest.mark.parametrize("name,nn,jj", [("c2", 1024, 16384), ("c3", 8000, 40000), ("c3o", 8000, 40000)])
@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_place_matches_oracle(name, nn, jj, threads):
    nodes, jobs, parts = synth.make_config(name, nn, jj)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    out, st, fin = po.cpu_place(nodes, jobs, parts, threads=threads)
    assert np.array_equal(out, ref[:, 0])
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert {k: st[k] for k in ("placed", "unplaced", "rejected")} == \
        {k: rst[k] for k in ("placed", "unplaced", "rejected")}


@pytest.mark.parametrize("threads", [1, 3])
def test_cpu_place_tl_matches_oracle(threads):
    nodes, tline, jobs, parts = synth.make_c5(1024, 3000)
    rn, rs, rst, rtl = po.ref_place_tl(nodes, tline, jobs, parts)
    n, s, st, tl = po.cpu_place_tl(nodes, tline, jobs, parts, threads=threads)
    assert np.array_equal(n, rn) and np.array_equal(s, rs) and np.array_equal(tl, rtl)
    assert st["placed"] == rst["placed"] and st["rejected"] == rst["rejected"]
