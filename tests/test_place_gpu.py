"""GPU parity: the HIP engine vs the sequential best-fit oracle (bit-exact placements + node state).

Sizes are ones the oracle finishes in seconds; BASELINE.json's full C3 size is covered by the
golden hashes in tests/golden (test_golden_gpu.py) and by size-independent properties."""
import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def run_engine(nodes, jobs, parts, **kw):
    with Engine(**kw) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs)
        fin = e.read_nodes()
    return out, st, fin


def check_parity(nodes, jobs, parts, **kw):
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    out, st, fin = run_engine(nodes, jobs, parts, **kw)
    assert np.array_equal(out, ref), f"first mismatch at job {int(np.argmax(out[:, 0] != ref[:, 0]))}"
    for a, b in zip(fin, rfin):
        assert np.array_equal(a, b)
    assert st["placed"] == rst["placed"] and st["rejected"] == rst["rejected"]
    assert st["unplaced"] == rst["unplaced"]
    return st


def test_c1_sample_job():
    nodes, jobs, parts = synth.make_c1()
    st = check_parity(nodes, jobs, parts)
    assert st["placed"] == 100


@pytest.mark.parametrize("nn,jj", [(64, 1024), (256, 4096), (4096, 65536)])
def test_c2(nn, jj):
    nodes, jobs, parts = synth.make_config("c2", nn, jj)
    check_parity(nodes, jobs, parts)


def test_c3_prefix():
    nodes, jobs, parts = synth.make_config("c3", 20000, 100000)
    check_parity(nodes, jobs, parts)


@pytest.mark.parametrize("wmin,wmax", [(1, 1), (1, 8), (64, 64), (512, 65536)])
def test_window_policies_c2(wmin, wmax):
    nodes, jobs, parts = synth.make_config("c2", 512, 8192)
    check_parity(nodes, jobs, parts, window_min=wmin, window_max=wmax)
