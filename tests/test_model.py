"""The speculative-prefix round algorithm (CPU model of the HIP kernels, oracle/round_model.c)
reproduces the sequential oracle bit-exactly for any window / candidate / dirty-cap settings,
including adversarial inputs (ties, zero demands, overlapping partitions, negative capacities)."""
import numpy as np
import pytest

from fitgpu import synth
from oracle import pyoracle as po


def same(nodes, jobs, parts, **kw):
    ref, _, rfin = po.ref_place(nodes, jobs, parts)
    out, st, fin = po.model_place(nodes, jobs, parts, **kw)
    assert np.array_equal(out, ref[:, 0])
    for a, b in zip(fin, rfin):
        assert np.array_equal(a, b)
    return st


PARAMS = [dict(slice=2048, ks=16, km=64, ucap=256, wmin=256, wmax=8192),
          dict(slice=64, ks=1, km=1, ucap=1, wmin=1, wmax=4),
          dict(slice=7, ks=2, km=8, ucap=3, wmin=3, wmax=50),
          dict(slice=100, ks=4, km=16, ucap=16, wmin=64, wmax=64)]


@pytest.mark.parametrize("prm", PARAMS)
def test_model_c2_small(prm):
    same(*synth.make_config("c2", 300, 5000), **prm)


@pytest.mark.parametrize("prm", PARAMS)
def test_model_c3_small(prm):
    same(*synth.make_config("c3", 2000, 20000), **prm)


def _nodes(n, cpu, mem, gpu=0, avail=synth.INT32_MAX, mask=1):
    f = lambda v: np.full(n, v, np.int32) if np.isscalar(v) else np.asarray(v, np.int32)  # noqa: E731
    return synth.Nodes(f(cpu), f(mem), f(gpu), f(avail), np.asarray(np.full(n, mask) if np.isscalar(mask) else mask,
                                                                    np.uint32))


def _jobs(j, cpu, mem, gpu=0, wall=0, part=0):
    f = lambda v, t=np.int32: np.full(j, v, t) if np.isscalar(v) else np.asarray(v, t)  # noqa: E731
    return synth.Jobs(f(cpu), f(mem), f(gpu), f(wall), f(part, np.uint16), np.ones(j, np.uint16))


P1 = synth.Partitions(np.full(4, -1, np.int32), np.full(4, -1, np.int32), np.full(4, -1, np.int32))


@pytest.mark.parametrize("prm", PARAMS)
def test_identical_nodes_one_job_each(prm):
    # worst case for speculation: every job wants the same lowest-id node
    same(_nodes(200, 4, 4096), _jobs(300, 4, 4096), P1, **prm)


@pytest.mark.parametrize("prm", PARAMS)
def test_zero_demand_and_ties(prm):
    rng = np.random.default_rng(1)
    n = _nodes(50, rng.integers(0, 3, 50), rng.integers(0, 3000, 50))
    j = _jobs(400, rng.integers(0, 2, 400), rng.integers(0, 1500, 400))
    same(n, j, P1, **prm)


@pytest.mark.parametrize("prm", PARAMS)
def test_overlapping_partitions_and_negative_capacity(prm):
    rng = np.random.default_rng(2)
    masks = rng.choice([1, 2, 3, 4, 12, 0], 120)
    n = _nodes(120, rng.integers(-3, 40, 120), rng.integers(-100, 80000, 120), rng.integers(-1, 9, 120),
               rng.choice([synth.INT32_MAX, 100, 2000, -5], 120), masks)
    j = _jobs(1500, rng.integers(0, 9, 1500), rng.integers(0, 9000, 1500), rng.integers(0, 3, 1500),
              rng.integers(0, 3000, 1500), rng.integers(0, 4, 1500))
    parts = synth.Partitions(np.array([-1, 1000, -1, 60], np.int32), np.array([-1, -1, 4, -1], np.int32),
                             np.array([-1, -1, -1, 5000], np.int32))
    same(n, j, parts, **prm)


def test_capped_scores():
    # residuals beyond the score fields' caps (gpu 255, cpu 4095, mem 4 TiB) tie on the cap
    n = _nodes(40, np.arange(4090, 4130), np.full(40, 2**31 - 1), np.arange(250, 290))
    j = _jobs(300, 1, 1024, 1)
    for prm in PARAMS:
        same(n, j, P1, **prm)
