"""Full-size parity for BASELINE configs C4 and C5: the HIP engine reproduces the oracle's SHA-256
digests at 100k nodes × 1M jobs (tests/golden/placements_big.json, made offline in the dev container
by tools/make_golden_big.py — C5 took the oracle 3,441 s, C4 281 s).

C4: GPU-heavy cluster (8 GPUs per node), multi-node jobs (nodes_k ∈ {1, 2, 4, 8}), kmax 8 —
    placements of every job's k nodes and the final free columns.
C5: 1,024-slot backfill horizon — node and start slot per job and the final dense timelines."""
import hashlib
import json
import os

import numpy as np
import pytest

from fitgpu import Engine, synth

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "placements_big.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_c4_full_digest():
    g = GOLD["c4:100000x1000000"]
    nodes, jobs, parts = synth.make_config("c4")
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs, kmax=g["kmax"])
        fin = e.read_nodes()
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])
    assert sha(out) == g["placements_sha256"]
    assert sha(fin[0]) == g["final_cpu_sha256"]
    assert sha(fin[1]) == g["final_mem_sha256"]
    assert sha(fin[2]) == g["final_gpu_sha256"]


def test_c5_full_digest():
    g = GOLD["c5:100000x1000000"]
    nodes, tline, jobs, parts = synth.make_c5()
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tline)
        node, start, st = e.place_tl(jobs)
        tl = e.read_timeline()
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])
    assert sha(node) == g["node_sha256"]
    assert sha(start) == g["start_sha256"]
    assert sha(tl[..., 0]) == g["final_cpu_sha256"]
    assert sha(tl[..., 1]) == g["final_mem_sha256"]
    assert sha(tl[..., 2]) == g["final_gpu_sha256"]
