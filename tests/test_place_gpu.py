"""GPU parity: the HIP engine vs the sequential best-fit oracle (bit-exact placements + node state).

Sizes are ones the oracle finishes in seconds; BASELINE.json's full C3 size is covered by the
golden hashes in tests/golden (test_golden_gpu.py) and by size-independent properties."""
import numpy as np
import pytest

from fitgpu import Engine, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def run_engine(nodes, jobs, parts, kmax=1, **kw):
    with Engine(**kw) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs, kmax=kmax)
        fin = e.read_nodes()
    return out, st, fin


def check_parity(nodes, jobs, parts, kmax=1, **kw):
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    out, st, fin = run_engine(nodes, jobs, parts, kmax=kmax, **kw)
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


@pytest.mark.parametrize("engine", ["persistent", "rounds"])
def test_c3o_overlapping_partitions_prefix(engine, monkeypatch):
    """C3 plus an all-nodes partition (~10 % of the jobs): the 17 partitions union into ONE
    component, so a single serial chain decides every job."""
    if engine == "rounds":
        monkeypatch.setenv("FIT_ENGINE", "rounds")
    nodes, jobs, parts = synth.make_config("c3o", 20000, 100000)
    st = check_parity(nodes, jobs, parts)
    assert st["components"] == 1


@pytest.mark.parametrize("ks_min", ["8", "4", "2"])
def test_fewer_keys_per_slice(ks_min, monkeypatch):
    """A large component keeps fewer keys per block-slice over more slices (engine.cpp: KS 16 →
    8 → 4 while a wave's sub-slice exceeds FIT_SUB_TARGET nodes); forced down to KS 8 / 4 / 2 on
    one 20,000-node component for single-node jobs (decider / helper commit), and for C4's
    multi-node jobs (single-wave commit), where the engine keeps KS >= kmax (8) so that every
    round's first job stays resolvable."""
    monkeypatch.setenv("FIT_SUB_TARGET", "64")
    monkeypatch.setenv("FIT_KS_MIN", ks_min)
    nodes, jobs, parts = synth.make_config("c3o", 20000, 50000)
    check_parity(nodes, jobs, parts)
    nodes, jobs, parts = synth.make_config("c4", 20000, 20000)
    nodes.part_mask = nodes.part_mask | np.uint32(1 << 16)  # one component
    jobs.part = np.where(np.arange(jobs.j) % 10 == 3, 16, jobs.part).astype(np.uint16)
    parts = synth.gen_partitions(synth.SEEDS["c4"], 17)
    st = check_parity(nodes, jobs, parts, kmax=8)
    assert st["components"] == 1


@pytest.mark.parametrize("wmin,wmax", [(1, 1), (1, 8), (64, 64), (512, 65536)])
def test_window_policies_c2(wmin, wmax):
    nodes, jobs, parts = synth.make_config("c2", 512, 8192)
    check_parity(nodes, jobs, parts, window_min=wmin, window_max=wmax)


# ---- multi-node jobs (SPEC k > 1, config C4: GPU-heavy nodes, nodes_k in {1, 2, 4, 8}) ----------
@pytest.mark.parametrize("engine", ["persistent", "rounds"])
@pytest.mark.parametrize("nn,jj", [(64, 1024), (512, 8192), (4096, 65536)])
def test_c4_multi_node(nn, jj, engine, monkeypatch):
    if engine == "rounds":
        monkeypatch.setenv("FIT_ENGINE", "rounds")
    nodes, jobs, parts = synth.make_config("c4", nn, jj)
    assert jobs.nodes_k.max() > 1
    st = check_parity(nodes, jobs, parts, kmax=8)
    assert st["placed"] > 0


def test_c4_prefix():
    nodes, jobs, parts = synth.make_config("c4", 20000, 100000)
    check_parity(nodes, jobs, parts, kmax=8)


def test_c4_window_policies():
    nodes, jobs, parts = synth.make_config("c4", 512, 8192)
    for wmin, wmax in [(1, 1), (1, 8), (64, 64)]:
        check_parity(nodes, jobs, parts, kmax=8, window_min=wmin, window_max=wmax)


def test_multi_node_edge_cases():
    # 8 identical 64-cpu nodes; jobs needing k nodes of 20 cpus: three k=8 jobs fill the cluster,
    # k=1 jobs keep flowing; all-or-nothing (no partial allocation)
    nodes, _, parts = synth.make_c1()
    k = np.array([8, 8, 1, 2, 1, 4, 8, 1] * 8, np.uint16)
    n = len(k)
    jobs = synth.Jobs(np.full(n, 20, np.int32), np.full(n, 1000, np.int32), np.zeros(n, np.int32),
                      np.full(n, 60, np.int32), np.zeros(n, np.uint16), k)
    st = check_parity(nodes, jobs, parts, kmax=8)
    assert st["unplaced"] > 0
    # kmax larger than any k: unused columns stay -1
    check_parity(nodes, jobs, parts, kmax=8)


def test_nodes_k_above_kmax_is_rejected():
    nodes, jobs, parts = synth.make_config("c4", 64, 256)
    from fitgpu import FitError
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        with pytest.raises(FitError):
            e.place(jobs, kmax=2)


# ---- commit hand-off patterns (decider / recorder / helpers) ----------------------
def _uniform(n, j, cpu_node, cpu_job, mem_job=100, seed=0):
    """n identical nodes, j jobs of cpu_job cpus (one partition): best fit packs one node at a time."""
    rng = np.random.default_rng(seed)
    nodes = synth.Nodes(np.full(n, cpu_node, np.int32), np.full(n, 1 << 20, np.int32),
                        np.zeros(n, np.int32), np.full(n, synth.INT32_MAX, np.int32),
                        np.ones(n, np.uint32))
    cpu = np.asarray(cpu_job, np.int32) if np.ndim(cpu_job) else np.full(j, cpu_job, np.int32)
    if cpu.size != j:
        cpu = rng.choice(cpu, j).astype(np.int32)
    jobs = synth.Jobs(cpu, np.full(j, mem_job, np.int32), np.zeros(j, np.int32),
                      np.full(j, 60, np.int32), np.zeros(j, np.uint16), np.ones(j, np.uint16))
    parts = synth.Partitions(np.full(1, -1, np.int32), np.full(1, -1, np.int32),
                             np.full(1, -1, np.int32))
    return nodes, jobs, parts


@pytest.mark.parametrize("n,j,cpu_node,cpu_job", [
    (64, 16384, 64, 1),          # every job lands on the node the previous one dirtied (ring winners)
    (4096, 8192, 32, 32),        # every job fills a fresh node: dirty set full every 256 jobs
    (1024, 20000, 96, [1, 2, 3, 5, 8, 13]),  # mixed sizes: items, ring entries and fresh nodes
    (512, 20000, 64, [7, 64, 1]),  # cluster fills up: long tail of unplaced jobs
])
def test_commit_hand_off_patterns(n, j, cpu_node, cpu_job):
    nodes, jobs, parts = _uniform(n, j, cpu_node, cpu_job)
    check_parity(nodes, jobs, parts)


def test_node_count_limit():
    # commit keys tag positions as pos << 3 (FIT_MAX_NODES = 2^29 rows): larger tables are refused
    from fitgpu import _lib
    with Engine() as e:
        assert _lib.lib().fit_load_nodes(e._h, (1 << 29) + 1, None, None, None, None, None) == \
            _lib.FIT_E_INVAL
