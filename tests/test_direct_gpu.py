"""k_small — the direct small placement (one launch, jobs one at a time against every node of their
component) that admission batches run on — bit-exact against the oracle
(oracle/fitref.c ref_place) at sizes far beyond its production range (FIT_ENGINE=direct forces it
at every size): the C3 prefix (16 components), one large component (c3o), multi-node jobs up to
kmax 8 (c4), components past the VGPR-resident size, and the automatic choice at its threshold
(FIT_SMALL_DIRECT)."""
import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def _check(nodes, jobs, parts, kmax=1, engine_id=2):
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    with Engine(device=0) as e:
        e.load_partitions(parts)
        e.load_nodes(nodes)
        out, st = e.place(jobs, kmax=kmax)
        fin = e.read_nodes()
    assert st["engine"] == engine_id
    bad = np.flatnonzero((out != ref).any(axis=1))
    assert bad.size == 0, f"first mismatch at job {bad[0]}: {out[bad[0]]} vs {ref[bad[0]]}"
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))
    assert (st["placed"], st["unplaced"], st["rejected"]) == (rst["placed"], rst["unplaced"], rst["rejected"])
    return st


# components up to 8,192 rows keep them in VGPRs (SMALL_RPT); c3o 12k and c2 10k are one larger
# component each: a pass over the rows per extraction
@pytest.mark.parametrize("name,nn,jj,kmax", [("c3", 20000, 60000, 1), ("c3o", 8192, 20000, 1),
                                              ("c4", 4096, 20000, 8), ("c2", 512, 8192, 1),
                                              ("c3o", 12000, 6000, 1), ("c2", 10000, 5000, 1),
                                              ("c4", 9000, 3000, 8)])
def test_direct_matches_oracle(name, nn, jj, kmax, monkeypatch):
    monkeypatch.setenv("FIT_ENGINE", "direct")
    nodes, jobs, parts = synth.make_config(name, nn, jj)
    _check(nodes, jobs, parts, kmax)


@pytest.mark.parametrize("j,want", [(1, 2), (128, 2), (129, 0)])
def test_direct_threshold(j, want, monkeypatch):
    """Unset FIT_ENGINE: up to 128 jobs run k_small (engine 2), more the host-driven rounds (0)."""
    monkeypatch.delenv("FIT_ENGINE", raising=False)
    nodes, jobs, parts = synth.make_config("c4", 4096, j)
    _check(nodes, jobs, parts, kmax=8, engine_id=want)


def test_direct_consecutive_batches(monkeypatch):
    """Admission-sized batches one after the other on one context: each sees the table the
    previous ones left (the oracle places the concatenated queue)."""
    monkeypatch.delenv("FIT_ENGINE", raising=False)
    nodes, jobs, parts = synth.make_config("c3", 20000, 640)
    ref, _, rfin = po.ref_place(nodes, jobs, parts)
    got = []
    with Engine(device=0) as e:
        e.load_partitions(parts)
        e.load_nodes(nodes)
        for b in range(0, 640, 10):
            sub = synth.Jobs(*(x[b:b + 10] for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part,
                                                     jobs.nodes_k)))
            out, st = e.place(sub)
            assert st["engine"] == 2
            got.append(out)
        fin = e.read_nodes()
    assert np.array_equal(np.concatenate(got), ref)
    assert all(np.array_equal(a, b) for a, b in zip(fin, rfin))


@pytest.mark.parametrize("engine", ["", "direct", "rounds"])
@pytest.mark.parametrize("bad", ["negative", "kmax"])
def test_invalid_job_fails_without_consuming(engine, bad, monkeypatch):
    """a batch of <= 128 jobs with one invalid job (a negative demand, or
    nodes_k > kmax) fails with FIT_E_INVAL and leaves the node table as it was — every k_small block
    runs the prefilter over the whole batch before it commits anything, as the rounds path checks
    the job-list kernel's flag on the host."""
    import fitgpu
    from fitgpu import _lib
    if engine:
        monkeypatch.setenv("FIT_ENGINE", engine)
    else:
        monkeypatch.delenv("FIT_ENGINE", raising=False)
    nodes, jobs, parts = synth.make_config("c4", 4096, 40)
    jobs.nodes_k = np.minimum(jobs.nodes_k, 4).astype(np.uint16)
    if bad == "negative":
        jobs.cpu[17] = -1
    else:
        jobs.nodes_k[17] = 8
    with Engine(device=0) as e:
        e.load_partitions(parts)
        e.load_nodes(nodes)
        before = e.read_nodes()
        with pytest.raises(fitgpu.FitError) as ei:
            e.place(jobs, kmax=4)
        assert ei.value.code == _lib.FIT_E_INVAL
        after = e.read_nodes()
        assert all(np.array_equal(a, b) for a, b in zip(before, after))
        # the context still places: the valid prefix, bit-exact vs the oracle
        ok = synth.Jobs(*(x[:17] for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, jobs.nodes_k)))
        out, _ = e.place(ok, kmax=4)
    ref, _, _ = po.ref_place(nodes, ok, parts, kmax=4)
    assert np.array_equal(out, ref)
