"""Node-table ingest: `scontrol show nodes` → engine columns, and Slurm hostlist
expansion.  The reference parses only CPUTot/CPUAlloc/RealMemory/AllocMem (parse.go:291-308) —
those fields must equal its mirror (fit_parse_nodes, pinned to the reference's parseNode); the
added fields (Gres/GresUsed/State/Partitions/NodeName) are checked against the build-authored
fixture tests/golden/scontrol_show_nodes.txt (parity unpinned vs the reference, which drops them)."""
import os

import numpy as np
import pytest

from fitgpu import expand_hostlist, ingest_nodes, parse_nodes, parse_partition

FIX = open(os.path.join(os.path.dirname(__file__), "golden", "scontrol_show_nodes.txt")).read()
INT32_MAX = 2**31 - 1


def test_fixture_columns():
    nodes, names = ingest_nodes(FIX, ["debug", "gpu", "batch"])
    assert names == ["node01", "node02", "node03", "node04", "gpu05"]
    assert nodes.cpu_free.tolist() == [48, 32, 32, 28, 0]
    assert nodes.mem_free.tolist() == [257000 - 65536, 128000, 128000, 120000, 24000]
    assert nodes.gpu_free.tolist() == [2, 0, 0, 0, 0]
    # debug = bit 0, gpu = bit 1; DOWN* and DRAIN nodes are never placed (mask 0)
    assert nodes.part_mask.tolist() == [0b11, 0b01, 0, 0, 0b10]
    assert (nodes.avail_min == INT32_MAX).all()


def test_reference_fields_match_parse_node_mirror():
    nodes, _ = ingest_nodes(FIX, [])
    ref = parse_nodes(FIX)  # Client.Nodes + parseNode as the reference has them
    assert nodes.cpu_free.tolist() == [r.Cpus - r.AlloCpus for r in ref]
    assert nodes.mem_free.tolist() == [r.Memory - r.AlloMemory for r in ref]
    assert all(r.Gpus == 0 for r in ref)  # the reference never sets Gpus
    assert nodes.part_mask.tolist() == [0] * 5  # no partitions asked for


def test_gres_forms():
    def one(gres, used="(null)"):
        t = f"NodeName=n CPUTot=4 CPUAlloc=0 RealMemory=10 AllocMem=0 Gres={gres} GresUsed={used} " \
            f"State=IDLE Partitions=p"
        nodes, _ = ingest_nodes(t, ["p"])
        return int(nodes.gpu_free[0])
    assert one("gpu:4") == 4
    assert one("gpu:h100:8(S:0-1)", "gpu:h100:3(IDX:0-2)") == 5
    assert one("gpu:a100:2,gpu:v100:2") == 4
    assert one("mps:400,gpu:2(S:0,1)") == 2
    assert one("gpu") == 1
    assert one("(null)") == 0
    assert one("gpu:2K") == 2048
    with pytest.raises(ValueError):
        one("gpu:a:b:x")


@pytest.mark.parametrize("state,ok", [("IDLE", True), ("MIXED", True), ("ALLOCATED", True),
                                      ("IDLE+CLOUD", True), ("COMPLETING", True), ("DOWN", False),
                                      ("IDLE*", False), ("IDLE+DRAIN", False), ("DRAINED", False),
                                      ("ALLOCATED+DRAINING", False), ("MAINT", False),
                                      ("IDLE+POWERED_DOWN", False), ("FUTURE", False), ("IDLE~", False),
                                      ("IDLE%", False), ("IDLE+POWERING_DOWN", False), ("MIXED#", True),
                                      ("IDLE+POWERING_UP", True), ("IDLE$", False), ("MIXED@", False),
                                      ("IDLE-", True)])
def test_state(state, ok):
    t = f"NodeName=n CPUTot=4 CPUAlloc=0 RealMemory=10 AllocMem=0 State={state} Partitions=p"
    nodes, _ = ingest_nodes(t, ["p"])
    assert bool(nodes.part_mask[0]) == ok


def test_cap_and_empty():
    nodes, names = ingest_nodes("", ["p"])
    assert nodes.n == 0 and names == []


@pytest.mark.parametrize("expr,want", [
    ("node[1-3,5]", ["node1", "node2", "node3", "node5"]),
    ("node[01-03]", ["node01", "node02", "node03"]),
    ("node[08-11]", ["node08", "node09", "node10", "node11"]),
    ("a,b[1-2],c", ["a", "b1", "b2", "c"]),
    ("rack[1-2]-n[1-2]", ["rack1-n1", "rack1-n2", "rack2-n1", "rack2-n2"]),
    ("gpu[1-2]-ib", ["gpu1-ib", "gpu2-ib"]),
    ("single", ["single"]),
    ("", []),
])
def test_hostlist(expr, want):
    assert expand_hostlist(expr) == want


def test_hostlist_fixes_parse_partition_split():
    text = "PartitionName=debug Nodes=node[1-3,5] Default=YES"
    assert parse_partition(text) == ["node[1-3", "5]"]  # the reference's split
    assert expand_hostlist(",".join(parse_partition(text))) == ["node1", "node2", "node3", "node5"]


@pytest.mark.parametrize("bad", ["node[3-1]", "node[1-", "node[a-b]", "node[-1]"])
def test_hostlist_malformed(bad):
    with pytest.raises(ValueError):
        expand_hostlist(bad)


def test_hostlist_large():
    names = expand_hostlist("n[000001-100000]")
    assert len(names) == 100000 and names[0] == "n000001" and names[-1] == "n100000"


def test_ingest_to_engine_columns_roundtrip():
    """A synthetic 2,000-node `scontrol show nodes` dump round-trips into the same columns."""
    rng = np.random.default_rng(7)
    n = 2000
    cpus = rng.choice([32, 64, 128], n)
    alloc = rng.integers(0, 32, n)
    mem = cpus * 4096
    amem = rng.integers(0, 100000, n)
    gpus = rng.choice([0, 4, 8], n)
    used = np.minimum(gpus, rng.integers(0, 5, n))
    parts = ["p0", "p1", "p2"]
    recs = []
    for i in range(n):
        g = f"gpu:mi355x:{gpus[i]}(S:0-1)" if gpus[i] else "(null)"
        u = f"gpu:mi355x:{used[i]}(IDX:0-{max(used[i] - 1, 0)})" if gpus[i] else "(null)"
        recs.append(f"NodeName=n{i:05d} Arch=x86_64\n   CPUAlloc={alloc[i]} CPUTot={cpus[i]}\n   Gres={g}\n"
                    f"   RealMemory={mem[i]} AllocMem={amem[i]}\n   State=MIXED\n   Partitions={parts[i % 3]}\n"
                    f"   GresUsed={u}")
    nodes, names = ingest_nodes("\n\n".join(recs), parts)
    assert names == [f"n{i:05d}" for i in range(n)]
    assert np.array_equal(nodes.cpu_free, cpus - alloc)
    assert np.array_equal(nodes.mem_free, mem - amem)
    assert np.array_equal(nodes.gpu_free, gpus - used)
    assert np.array_equal(nodes.part_mask, 1 << (np.arange(n) % 3))
