"""The CreatePod call site on the GPU: what
pkg/slurm-virtual-kubelet/fit_admission.go does, through the C-ABI, against the oracle.

* Node names (a10 / f4): the Partition RPC's list (parsePartition, pkg/slurm-agent/parse.go:278-289,
  which leaves C1's `Nodes=node[1-8]` as ONE entry) → fit_node_names → the names the Nodes RPC is
  asked for (slurm.go:343-364) → one engine row per record; every forwarded `--nodelist=` names the
  NodeName of the record the oracle chose (cross-checked with fit_ingest_nodes).
* Pinning policy (f4): a table with node State (fit_ingest_nodes) never offers a DRAIN node and
  pins; the gRPC table (no State in workload.proto:165-174) gates capacity without pinning unless
  the operator asks for FIT_TABLE_PIN.
* Array groups inside a shared batch are oracle-equal: a group that does not fit entirely takes
  nothing, and every later request of the batch sees the table without it.
* Reservations: give-backs on an oversubscribed node (unclamped host table), a partial group on a
  table loaded directly into the engine, confirmations racing a refresh (generations), and
  reservations that follow their node by name across a reload that reorders the partition.
"""
import os
import threading

import numpy as np
import pytest

import fitgpu
from fitgpu import FIT_REJECTED, FIT_UNPLACED, Admitter, Engine, FitError, synth
from fitgpu import _lib
from oracle import pyoracle as po

pytestmark = [pytest.mark.gpu, pytest.mark.auto_engine]
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SCRIPT = "#!/bin/sh\n#SBATCH --nodes=1\nsrun hostname\nhostname\npwd\n"
NODES_TEXT = open(os.path.join(GOLD, "c1_scontrol_show_nodes.txt")).read()
PART_TEXT = open(os.path.join(GOLD, "c1_scontrol_show_partition.txt")).read()
UNLIMITED = synth.Partitions(np.full(1, -1, np.int32), np.full(1, -1, np.int32), np.full(1, -1, np.int32))


def _jobs(reqs):
    cols = ((1, np.int32), (2, np.int32), (3, np.int32), (4, np.int32), (5, np.uint16), (6, np.uint16))
    return synth.Jobs(*(np.array([r[i] for r in reqs], dt) for i, dt in cols))


def _grpc_table(text):
    """What Refresh builds from the gRPC API: Partition RPC → fit_node_names → Nodes RPC rows
    (parseNode: no State, no NodeName) → fit_node_columns."""
    names = fitgpu.node_names(fitgpu.parse_partition(PART_TEXT.strip()))
    rows = fitgpu.parse_nodes(text)
    assert len(rows) == len(names)  # Refresh refuses a count mismatch
    return fitgpu.node_columns(rows, part_mask=1), names


def _nodelist(script):
    lines = [ln for ln in script.split("\n") if ln.startswith("#SBATCH --nodelist=")]
    assert len(lines) <= 1
    return lines[0][len("#SBATCH --nodelist="):].split(",") if lines else None


def _pod(cpus_per_task, prio):
    labels = {fitgpu.POD_LABEL_KEYS["ntasks"]: "1", fitgpu.POD_LABEL_KEYS["mem_per_cpu"]: "500",
              fitgpu.POD_LABEL_KEYS["cpus_per_task"]: str(cpus_per_task)}
    return fitgpu.pod_demand(labels, SCRIPT, 0, prio)


@pytest.mark.parametrize("source", ["grpc+pin", "ingest"])
def test_c1_nodelist_names_the_oracle_node(source):
    """C1's partition (`Nodes=node[1-8]`) through the parsePartition mirror and
    fit_node_names, C1's nodes as the Nodes RPC returns them; pods admitted until all 8 nodes are
    used; every --nodelist is the NodeName of the record the oracle placed the pod on."""
    ingest_cols, ingest_names = fitgpu.ingest_nodes(NODES_TEXT, ["debug"])
    if source == "ingest":
        cols, names = ingest_cols, ingest_names
    else:
        cols, names = _grpc_table(NODES_TEXT)
        assert names == ingest_names  # record i of `scontrol show nodes <names>` is name i
    pods = [_pod(20, i) for i in range(25)]  # 3 per 64-cpu node, the 25th does not fit
    with Engine() as e:
        e.load_partitions(UNLIMITED)
        with Admitter(e, max_batch=16, max_wait_us=100) as adm:
            adm.load_table(cols, names, state=source == "ingest", pin=source != "ingest")
            got = [adm.admit_group(p) for p in pods]
            scripts = [adm.script([g[0][4]], SCRIPT) if g[0][4] else None for g in got]
    ref, _, _ = po.ref_place(cols, _jobs([p[0] for p in pods]), UNLIMITED)
    assert [g[0][0][0] for g in got] == ref[:, 0].tolist()
    assert sorted(set(ref[:24, 0].tolist())) == list(range(8)) and ref[24, 0] == FIT_UNPLACED
    for i, s in enumerate(scripts[:24]):
        text, pinned = s
        assert pinned and _nodelist(text) == [ingest_names[ref[i, 0]]], (i, text)
        assert text.replace(f"#SBATCH --nodelist={ingest_names[ref[i, 0]]}\n", "") == SCRIPT
    assert scripts[24] is None


def test_drain_node_policy():
    """a DRAIN node with free capacity.  State-aware ingest keeps it out of
    every partition, so the engine never picks it and the scripts are pinned; the gRPC table cannot
    see State — the engine may pick it, so the scripts stay unpinned (capacity gate only) unless
    the operator asks for pinning (FIT_TABLE_PIN), which then names it."""
    recs = NODES_TEXT.strip().split("\n\n")
    recs[2] = recs[2].replace("State=IDLE ", "State=IDLE+DRAIN ")   # node3
    recs[5] = recs[5].replace("State=IDLE ", "State=DRAIN ")        # node6
    text = "\n\n".join(recs) + "\n"
    ingest_cols, names = fitgpu.ingest_nodes(text, ["debug"])
    assert ingest_cols.part_mask.tolist() == [1, 1, 0, 1, 1, 0, 1, 1]
    pods = [_pod(60, i) for i in range(10)]  # one per node
    out = {}
    for mode in ("ingest", "grpc", "grpc+pin"):
        cols = ingest_cols if mode == "ingest" else _grpc_table(text)[0]
        with Engine() as e:
            e.load_partitions(UNLIMITED)
            with Admitter(e, max_batch=16, max_wait_us=100) as adm:
                adm.load_table(cols, names, state=mode == "ingest", pin=mode == "grpc+pin")
                got = [adm.admit_group(p)[0] for p in pods]
                out[mode] = [(g[0][0], adm.script([g[4]], SCRIPT) if g[4] else None) for g in got]
        ref, _, _ = po.ref_place(cols, _jobs([p[0] for p in pods]), UNLIMITED)
        assert [n for n, _ in out[mode]] == ref[:, 0].tolist(), mode
    placed = [n for n, _ in out["ingest"] if n >= 0]
    assert sorted(placed) == [0, 1, 3, 4, 6, 7]
    assert all(s[1] and _nodelist(s[0])[0] not in ("node3", "node6") for n, s in out["ingest"] if n >= 0)
    grpc = [(n, s) for n, s in out["grpc"] if n >= 0]
    assert sorted(n for n, _ in grpc) == list(range(8))  # the gRPC table offers the drained nodes
    assert all(s == (SCRIPT, False) for _, s in grpc)     # ... so nothing is pinned
    pinned = {_nodelist(s[0])[0] for n, s in out["grpc+pin"] if n >= 0}
    assert {"node3", "node6"} <= pinned                    # the operator's choice, documented risk


def test_array_task_never_pinned():
    """an array job whose demand is ONE request (`--array=0-9%1`: one task at
    a time, or `--array=5`) is still an array — its one sbatch runs every task, so a --nodelist
    would pin all of them to the node reserved for one.  On a pinnable table (ingest State, and the
    gRPC table with FIT_TABLE_PIN) such a pod keeps its script; a plain pod is pinned.  The array
    comes from the label or from the script's own #SBATCH --array."""
    cols, names = fitgpu.ingest_nodes(NODES_TEXT, ["debug"])
    base = {fitgpu.POD_LABEL_KEYS["ntasks"]: "1", fitgpu.POD_LABEL_KEYS["mem_per_cpu"]: "500",
            fitgpu.POD_LABEL_KEYS["cpus_per_task"]: "4"}
    arr_script = SCRIPT.replace("--nodes=1\n", "--nodes=1\n#SBATCH --array=0-3%1\n")
    cases = [(dict(base, **{fitgpu.POD_LABEL_KEYS["array"]: "0-9%1"}), SCRIPT, False),
             (dict(base, **{fitgpu.POD_LABEL_KEYS["array"]: "5"}), SCRIPT, False),
             (base, arr_script, False),
             (base, SCRIPT, True)]
    for state, pin in ((True, False), (False, True)):
        with Engine() as e:
            e.load_partitions(UNLIMITED)
            with Admitter(e, max_batch=16, max_wait_us=100) as adm:
                adm.load_table(cols, names, state=state, pin=pin)
                for labels, script, want in cases:
                    reqs = fitgpu.pod_demand(labels, script, 0, 0)
                    assert len(reqs) == 1 and reqs[0][7] == (0 if want else fitgpu.FIT_REQ_ARRAY)
                    g = adm.admit_group(reqs)
                    assert g[0][0][0] >= 0 and g[0][4] > 0
                    text, pinned = adm.script([g[0][4]], script)
                    assert pinned == want, (labels, script)
                    assert (text == script) != want
                    if want:
                        assert _nodelist(text) == [names[g[0][0][0]]]


def _oracle_units(nodes, parts, units, kmax=8):
    """Sequential admission of units (lists of requests) in order; a unit takes its nodes only
    when every request of it is placed (fit_admit_group's all or nothing)."""
    cur = synth.Nodes(nodes.cpu_free.copy(), nodes.mem_free.copy(), nodes.gpu_free.copy(), nodes.avail_min,
                      nodes.part_mask)
    res = []
    for u in units:
        ref, _, fin = po.ref_place(cur, _jobs(u), parts, kmax=kmax)
        if (ref[:, 0] >= 0).all():
            res.append([[int(x) for x in ref[i, :max(u[i][6], 1)]] for i in range(len(u))])
            cur = synth.Nodes(fin[0], fin[1], fin[2], nodes.avail_min, nodes.part_mask)
        else:
            code = FIT_REJECTED if (ref[:, 0] == FIT_REJECTED).any() else FIT_UNPLACED
            res.append([[code]] * len(u))
    return res, cur


def test_groups_in_one_batch_match_oracle():
    """failing --array groups and single pods in ONE batch; every result equals
    the oracle's sequential all-or-nothing admission in the batch's order, and so do the free
    columns after it (the dropped groups took nothing, the pods behind them used that room)."""
    nodes, _, _ = synth.make_c1()
    parts = synth.Partitions(np.full(1, 600, np.int32), np.full(1, -1, np.int32), np.full(1, -1, np.int32))

    def req(prio, cpu, wall=10, n=1, k=1):
        return [(prio, cpu, 1000, 0, wall, 0, k)] * n

    units = [req(0, 40), req(1, 60, n=10),      # 7 of the 10 tasks would fit: dropped
             req(2, 30), req(3, 20, n=3), req(4, 64), req(5, 100, n=2),   # too big: unplaced, not partial
             req(6, 50, n=5), req(7, 10), req(8, 14, n=6),                # 4 of 5 would fit: dropped
             req(9, 14), req(10, 5, wall=700, n=2),                       # MaxTime 600: rejected
             req(11, 8, k=2), req(12, 2, n=4, k=2), req(13, 3)]
    total = sum(len(u) for u in units)
    res = [None] * len(units)
    with Engine() as e:
        e.load_partitions(parts)
        with Admitter(e, max_batch=total, max_wait_us=30_000_000) as adm:  # closes when all are queued
            adm.load_nodes(nodes)
            go = threading.Barrier(len(units))

            def caller(i):
                go.wait()
                res[i] = adm.admit_group(units[i])

            th = [threading.Thread(target=caller, args=(i,)) for i in range(len(units))]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            free = adm.partition_free(0)
            assert adm.reservations() == sum(len(u) for u, r in zip(units, res) if r[0][0][0] >= 0)
    assert len({r[0][1] for r in res}) == 1 and res[0][0][2] == total  # one batch
    want, fin = _oracle_units(nodes, parts, units)
    assert [[g[0] for g in r] for r in res] == want
    # the scenario exercises the drop: units 1 and 6 would be placed in part on the table they
    # meet (so a single fit_place gives them nodes), yet take nothing; unit 5 fits nowhere at all
    partial = []
    cur = synth.Nodes(nodes.cpu_free.copy(), nodes.mem_free.copy(), nodes.gpu_free.copy(), nodes.avail_min,
                      nodes.part_mask)
    for u, w in zip(units, want):
        ref, _, f = po.ref_place(cur, _jobs(u), parts, kmax=8)
        partial.append(0 < int((ref[:, 0] >= 0).sum()) < len(u))
        if w[0][0] >= 0:
            cur = synth.Nodes(f[0], f[1], f[2], nodes.avail_min, nodes.part_mask)
    assert [i for i, x in enumerate(partial) if x] == [1, 6]
    assert want[1] == [[FIT_UNPLACED]] * 10 and want[6] == [[FIT_UNPLACED]] * 5
    assert want[5] == [[FIT_UNPLACED]] * 2 and want[10] == [[FIT_REJECTED]] * 2
    assert want[2] == [[1]]  # the 30-cpu pod behind the dropped group uses the room it left
    assert free == {"cpu": int(np.maximum(fin.cpu_free, 0).sum()), "mem_mib": int(np.maximum(fin.mem_free, 0).sum()),
                    "gpu": 0}
    # order: each request's index in the batch's priority order
    assert [r[0][3] for r in res] == [sum(len(u) for u in units[:i]) for i in range(len(units))]


def test_giveback_on_oversubscribed_node():
    """Slurm's refresh leaves less room than the open reservations hold; the
    engine clamps the node at -1, the admitter keeps the true -5; a release of 2 cpus leaves it at
    -3, so nothing fits there (the clamped copy would have shown +1 and over-committed)."""
    one = synth.Nodes(np.array([10], np.int32), np.array([10000], np.int32), np.zeros(1, np.int32),
                      np.full(1, np.iinfo(np.int32).max, np.int32), np.ones(1, np.uint32))
    with Engine() as e:
        e.load_partitions(UNLIMITED)
        with Admitter(e, max_batch=8, max_wait_us=100) as adm:
            adm.load_nodes(one)
            a = adm.admit(0, 8, 100)
            b = adm.admit(1, 2, 100)
            assert a[0] == [0] and b[0] == [0] and adm.partition_free(0)["cpu"] == 0
            slurm = synth.Nodes(np.array([5], np.int32), one.mem_free, one.gpu_free, one.avail_min, one.part_mask)
            adm.load_nodes(slurm)  # another job took 5 cpus; a and b still reserved: 5 - 10 = -5
            assert adm.partition_free(0)["cpu"] == 0
            adm.release(b[4])      # -3
            assert adm.admit(2, 1, 10)[0] == [FIT_UNPLACED]
            assert adm.partition_free(0)["cpu"] == 0
            adm.release(a[4])      # 5
            assert adm.partition_free(0)["cpu"] == 5
            assert adm.admit(3, 5, 10)[0] == [0] and adm.admit(4, 1, 10)[0] == [FIT_UNPLACED]


def test_partial_group_on_engine_loaded_table():
    """a partial group on a table loaded with fit_load_nodes directly (not
    through the admitter) takes nothing and does not wedge the admitter; later batches match the
    oracle."""
    nodes, _, _ = synth.make_c1()
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(UNLIMITED)
        with Admitter(e, max_batch=64, max_wait_us=100) as adm:
            g = adm.admit_group([(0, 64, 100, 0, 0, 0, 1)] * 9)  # 8 fit, the 9th does not
            assert [x[0] for x in g] == [[FIT_UNPLACED]] * 9 and adm.reservations() == 0
            singles = [adm.admit(i + 1, 50, 100) for i in range(9)]
            adm.release(singles[0][4])
            assert adm.partition_free(0)["cpu"] == 8 * 64 - 7 * 50
    ref, _, _ = po.ref_place(nodes, _jobs([(0, 50, 100, 0, 0, 0, 1)] * 9), UNLIMITED)
    assert [s[0][0] for s in singles] == ref[:, 0].tolist()


def test_confirm_racing_a_refresh():
    """a table fetched BEFORE a confirmation still lacks the job, so loading it
    must keep the reservation; only a table fetched after the confirmation drops it.  A table
    older than the one already loaded is refused."""
    nodes, _, _ = synth.make_c1()
    with Engine() as e:
        e.load_partitions(UNLIMITED)
        with Admitter(e, max_batch=8, max_wait_us=100) as adm:
            adm.load_nodes(nodes)
            a = adm.admit(0, 60, 1000)
            g1 = adm.generation()      # the ticker starts its Nodes RPC ...
            adm.confirm(a[4])          # ... the status poll sees the job running ...
            adm.load_table(nodes, generation=g1)  # ... the RPC's answer (without the job) arrives
            assert adm.partition_free(0)["cpu"] == 8 * 64 - 60
            g2 = adm.generation()
            slurm = synth.Nodes(nodes.cpu_free.copy(), nodes.mem_free.copy(), nodes.gpu_free, nodes.avail_min,
                                nodes.part_mask)
            slurm.cpu_free[a[0][0]] -= 60
            slurm.mem_free[a[0][0]] -= 1000
            adm.load_table(slurm, generation=g2)  # fetched after the confirm: carries the job itself
            assert adm.partition_free(0)["cpu"] == 8 * 64 - 60
            with pytest.raises(FitError) as ei:
                adm.load_table(nodes, generation=g1)  # stale
            assert ei.value.code == _lib.FIT_E_STATE
            with pytest.raises(FitError):
                adm.load_table(nodes, generation=10**9)  # never issued


def test_reservations_follow_node_names():
    """A refresh that drops a node from the partition and reorders the rest carries every open
    reservation to its node by name; the pinned script names the same node before and after."""
    nodes, _, _ = synth.make_c1()
    names = [f"node{i}" for i in range(1, 9)]
    with Engine() as e:
        e.load_partitions(UNLIMITED)
        with Admitter(e, max_batch=8, max_wait_us=100) as adm:
            adm.load_table(nodes, names, state=True)
            a = adm.admit(0, 64, 1000)  # fills node1 (id 0)
            b = adm.admit(1, 60, 1000)  # node2 (id 1)
            assert (a[0], b[0]) == ([0], [1])
            assert _nodelist(adm.script([b[4]], SCRIPT)[0]) == ["node2"]
            order = [7, 6, 5, 4, 3, 1, 0]  # node8 .. node4, node2, node1 (node3 left the partition)
            sub = synth.Nodes(*(np.ascontiguousarray(c[order]) for c in (nodes.cpu_free, nodes.mem_free,
                                                                          nodes.gpu_free, nodes.avail_min,
                                                                          nodes.part_mask)))
            adm.load_table(sub, [names[i] for i in order], state=True)
            assert _nodelist(adm.script([b[4]], SCRIPT)[0]) == ["node2"]
            assert _nodelist(adm.script([a[4]], SCRIPT)[0]) == ["node1"]
            assert adm.partition_free(0)["cpu"] == 7 * 64 - 124
            c = adm.admit(2, 5, 10)  # best fit: node2's 4 free cpus do not hold 5; node1 is full
            assert c[0] == [0]        # node8 (id 0 now)
            assert adm.admit(3, 4, 10)[0] == [5]  # exactly node2's remaining 4 cpus


def test_backfill_from_running_pods():
    """What's-missing r03 #2 (f2 had no caller): the call site's running pods — JobInfo.node_list
    (a hostlist, expanded and mapped to engine rows through the names table) and JobInfo.end_time
    (minutes left), workload.proto:252-292, with each pod's demand — become release events
    (fit_release_events) for fit_load_timeline; backfill of new pods against that timeline is
    bit-exact vs the oracle, and some of them start in the future."""
    cols, names = fitgpu.ingest_nodes(NODES_TEXT, ["debug"])
    row = {nm: i for i, nm in enumerate(names)}
    running = [("node[1-3]", 45, 48, 64000, 0), ("node4", 200, 60, 100000, 0), ("node[5,7-8]", 12, 40, 20000, 0),
               ("node6", -3, 64, 1000, 0), ("node[2,6]", 90, 8, 50000, 0)]
    jobs = [([row[x] for x in fitgpu.expand_hostlist(nl)], rem, c, m, g) for nl, rem, c, m, g in running]
    held = np.zeros((3, len(names)), np.int64)  # what Slurm's CPUAlloc / AllocMem count for them
    for nodes, _, c, m, g in jobs:
        for x in nodes:
            held[:, x] += (c, m, g)
    table = synth.Nodes((cols.cpu_free - held[0]).astype(np.int32), (cols.mem_free - held[1]).astype(np.int32),
                        (cols.gpu_free - held[2]).astype(np.int32), cols.avail_min, cols.part_mask)
    tl = fitgpu.release_events(len(names), jobs, slots=96, slot_min=5)
    assert tl.off.tolist() == [0, 1, 3, 4, 5, 6, 8, 9, 10]
    rng = np.random.default_rng(7)
    j = 200
    new = synth.Jobs(rng.integers(1, 48, j).astype(np.int32), rng.integers(100, 90000, j).astype(np.int32),
                     np.zeros(j, np.int32), rng.integers(5, 240, j).astype(np.int32), np.zeros(j, np.uint16),
                     np.ones(j, np.uint16))
    rn, rs, rst, _ = po.ref_place_tl(table, tl, new, UNLIMITED)
    with Engine() as e:
        e.load_nodes(table)
        e.load_partitions(UNLIMITED)
        e.load_timeline(tl)
        node, start, st = e.place_tl(new)
    assert np.array_equal(node, rn) and np.array_equal(start, rs)
    assert (st["placed"], st["unplaced"]) == (rst["placed"], rst["unplaced"])
    assert (start > 0).any() and (start == 0).any()
