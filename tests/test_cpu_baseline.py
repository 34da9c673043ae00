"""The CPU baselines bench.py times give exactly the oracle's results (oracle/fitref.c:ref_place,
oracle/fitref_tl.c:ref_place_tl) — so their throughput is a like-for-like baseline:

  component   oracle/cpu_baseline.c: each job scans its component's nodes, components on threads
  split       oracle/cpu_fast.c: every job's argmin split over the threads (BASELINE.md:22)
  rounds      oracle/cpu_fast.c: the GPU's candidate-list + dirty-set round algorithm on the CPU
  rle         oracle/cpu_fast.c: SPEC §2b on run-length timelines (the GPU's layout)
  k           oracle/cpu_baseline.c cpu_place_k: multi-node jobs (config C4), components on threads"""
import numpy as np
import pytest

from fitgpu import synth
from oracle import pyoracle as po


@pytest.mark.parametrize("variant", ["component", "split", "rounds"])
@pytest.mark.parametrize("name,nn,jj", [("c2", 1024, 16384), ("c3", 8000, 40000), ("c3o", 8000, 40000),
                                        ("c4", 512, 4000)])
@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_place_matches_oracle(name, nn, jj, threads, variant):
    nodes, jobs, parts = synth.make_config(name, nn, jj)
    if name == "c4":  # multi-node jobs are not the CPU variants' case: k = 1 here
        jobs = synth.Jobs(jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, np.ones_like(jobs.nodes_k))
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    out, st, fin = po.cpu_place(nodes, jobs, parts, threads=threads, variant=variant)
    assert np.array_equal(out, ref[:, 0])
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert {k: st[k] for k in ("placed", "unplaced", "rejected")} == \
        {k: rst[k] for k in ("placed", "unplaced", "rejected")}


@pytest.mark.parametrize("rle", [False, True])
@pytest.mark.parametrize("threads", [1, 3])
def test_cpu_place_tl_matches_oracle(threads, rle):
    nodes, tline, jobs, parts = synth.make_c5(1024, 3000)
    rn, rs, rst, rtl = po.ref_place_tl(nodes, tline, jobs, parts)
    n, s, st, tl = po.cpu_place_tl(nodes, tline, jobs, parts, threads=threads, rle=rle)
    assert np.array_equal(n, rn) and np.array_equal(s, rs) and np.array_equal(tl, rtl)
    assert st["placed"] == rst["placed"] and st["rejected"] == rst["rejected"]


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("nn,jj", [(512, 4000), (4096, 20000)])
def test_cpu_place_k_matches_oracle(nn, jj, threads):
    """config C4 (--nodes=k up to 8): the k smallest distinct keys, all or nothing, as ref_place."""
    nodes, jobs, parts = synth.make_config("c4", nn, jj)
    assert jobs.nodes_k.max() > 1
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=8)
    out, st, fin = po.cpu_place_k(nodes, jobs, parts, 8, threads)
    assert np.array_equal(out, ref)
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert {k: st[k] for k in ("placed", "unplaced", "rejected")} == \
        {k: rst[k] for k in ("placed", "unplaced", "rejected")}
