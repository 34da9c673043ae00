"""The numpy generator and its C twin (oracle/fitref.c:ref_rnd) agree bit-for-bit."""
import numpy as np

from fitgpu import synth
from oracle import pyoracle as po


def test_rnd_twins_agree():
    L = po.lib()
    idx = np.array([0, 1, 2, 63, 64, 12345, 999_999, 2**33 + 7], dtype=np.uint64)
    for seed in (0, synth.SEEDS["c3"], 2**63 + 5):
        for stream in (0, 5, 17, 32):
            py = synth.rnd(seed, stream, idx)
            c = [L.ref_rnd(seed, stream, int(i)) for i in idx]
            assert [int(v) for v in py] == c


def test_generator_is_slice_consistent():
    a = synth.gen_jobs(synth.SEEDS["c3"], 1000, 16)
    b = synth.gen_jobs(synth.SEEDS["c3"], 500, 16, start=500)
    assert np.array_equal(a.cpu[500:], b.cpu) and np.array_equal(a.wall[500:], b.wall)


def test_distributions_match_spec():
    n = synth.gen_nodes(synth.SEEDS["c3"], 100_000, 16)
    j = synth.gen_jobs(synth.SEEDS["c3"], 100_000, 16)
    assert set(np.unique(j.cpu)) == {1, 2, 4, 8, 16, 32, 64}
    assert abs((j.gpu == 0).mean() - 0.8) < 0.01
    assert abs((n.avail_min == synth.INT32_MAX).mean() - 0.9) < 0.01
    assert j.wall.min() >= 5 and j.wall.max() <= 2880
    assert (n.cpu_free >= 16).all() and set(np.unique(n.part_mask)) == {1 << p for p in range(16)}
