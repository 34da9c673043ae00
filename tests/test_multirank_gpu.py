"""Multi-rank placement on one GPU: 2 ranks share cuda:0 and exchange through the host callback
(gloo), running exactly the engine code RCCL drives on an 8-GPU node (node-sharded: per-round
allgather of candidates + 64-bit min of bounds; component-sharded: one merge at the end).
Both ranks must return the oracle's placements and node state."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from fitgpu import FIT_SHARD_COMPONENTS, FIT_SHARD_NODES, synth
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode,config,nn,jj", [(FIT_SHARD_NODES, "c3", 20000, 100000),
                                               (FIT_SHARD_COMPONENTS, "c3", 20000, 100000),
                                               (FIT_SHARD_NODES, "c2", 4096, 65536)])
def test_two_ranks_match_oracle(tmp_path, mode, config, nn, jj):
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_multirank_worker.py"), "--rank", str(r),
                               "--world", "2", "--port", str(port), "--mode", str(mode), "--config", config,
                               "--nodes", str(nn), "--jobs", str(jj), "--out", str(tmp_path / f"r{r}.npz")])
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    nodes, jobs, parts = synth.make_config(config, nn, jj)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts)
    for r in range(2):
        d = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(d["out"], ref)
        for k, col in zip(("cpu", "mem", "gpu"), rfin):
            assert np.array_equal(d[k], col)
        assert list(d["stats"][:3]) == [rst["placed"], rst["unplaced"], rst["rejected"]]
        assert d["stats"][3] == mode


def test_two_ranks_multi_node_class_engine(tmp_path):
    """C4-shaped (75 % multi-node jobs, kmax 8) with the library's own engine choice — the
    demand-class engine — component-sharded over 2 ranks: each rank places its components, the
    merge gives both ranks the oracle's placements and node state."""
    port = free_port()
    nn, jj = 8192, 30000
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_multirank_worker.py"), "--rank", str(r),
                               "--world", "2", "--port", str(port), "--mode", str(FIT_SHARD_COMPONENTS),
                               "--config", "c4", "--nodes", str(nn), "--jobs", str(jj), "--kmax", "8",
                               "--auto-engine", "--out", str(tmp_path / f"r{r}.npz")])
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    nodes, jobs, parts = synth.make_config("c4", nn, jj)
    ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=8)
    for r in range(2):
        d = np.load(tmp_path / f"r{r}.npz")
        assert d["stats"][4] == 3  # the class engine ran
        assert np.array_equal(d["out"], ref)
        for k, col in zip(("cpu", "mem", "gpu"), rfin):
            assert np.array_equal(d[k], col)
        assert list(d["stats"][:3]) == [rst["placed"], rst["unplaced"], rst["rejected"]]


def test_two_ranks_backfill_match_oracle(tmp_path):
    """C5 (SPEC §2b) node-sharded over 2 ranks: each scans half of every component, candidates and
    bounds are exchanged every round, the commit runs replicated; both ranks equal the oracle."""
    port = free_port()
    nn, jj = 2048, 16384
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_multirank_worker.py"), "--rank", str(r),
                               "--world", "2", "--port", str(port), "--mode", str(FIT_SHARD_NODES),
                               "--config", "c5", "--nodes", str(nn), "--jobs", str(jj),
                               "--out", str(tmp_path / f"r{r}.npz")])
             for r in range(2)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    nodes, tline, jobs, parts = synth.make_c5(nn, jj)
    rn, rs, rst, rfin = po.ref_place_tl(nodes, tline, jobs, parts)
    live = nodes.part_mask != 0
    for r in range(2):
        d = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(d["node"], rn) and np.array_equal(d["start"], rs)
        assert np.array_equal(d["fin"][live], rfin[live])
        assert list(d["stats"][:3]) == [rst["placed"], rst["unplaced"], rst["rejected"]]
        assert d["stats"][3] == FIT_SHARD_NODES
