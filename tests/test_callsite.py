"""CreatePod call-site helpers (host code in libfitgpu.so, no GPU needed) against the oracle's
independent restatement (oracle/fitref.c ref_pod_demand / ref_array_tasks / ref_job_demand):

  fit_pod_demand          labels (pkg/common/labels.go:9-14, read by newSubmitRequestForPod,
                          provider.go:74-123) + the pod's #SBATCH script (parse.go:30-69) →
                          array-expanded admission requests
  fit_array_tasks         Slurm --array task count (the fix of parseArrayLen, parse.go:126-135)
  fit_script_with_nodelist the engine's decision forwarded in SubmitJobRequest.script
  fit_partition_limits    ResourcesResponse (api/slurm.go:297-341) → fit_load_partitions limits
  fit_node_columns        NodesResponse rows (workload.proto:165-174) → fit_load_nodes columns
"""
import ctypes as C

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

import fitgpu
from fitgpu import POD_LABEL_KEYS
from oracle import pyoracle as po

KEYS = ["nodes", "cpus_per_task", "mem_per_cpu", "ntasks_per_node", "array", "ntasks"]

SBATCH = st.lists(st.sampled_from([
    "#!/bin/sh", "", "#SBATCH --nodes=2", "#SBATCH -N 3", "#SBATCH --nodes=2-4", "#SBATCH --time=1:00:00",
    "#SBATCH -t 30", "#SBATCH --time=UNLIMITED", "#SBATCH --time=2-00:00:00", "#SBATCH --mem-per-cpu=500",
    "#SBATCH --cpus-per-task=4", "#SBATCH -c 2", "#SBATCH --ntasks-per-node=8", "#SBATCH --exclusive --nodes=2",
    "#SBATCH --exclusive", "#SBATCH --time=foo", "srun hostname", "#SBATCH --ntasks=3", "#SBATCH --nodes=20",
    "#SBATCH --mem-per-cpu 2048", "#SBATCH --time=0:90"]), max_size=7).map("\n".join)
INTS = st.one_of(st.none(), st.integers(-3, 40).map(str), st.sampled_from(["x", "", "9223372036854775808", "+4",
                                                                           "4096", "3000000000"]))
ARRAYS = st.one_of(st.none(), st.sampled_from([
    "", "1-4", "0-15", "1,3,5-7", "0-15:4", "1-100%10", "1-10%2", "5", "1-3,5", "x-y", "1-", "-3", "4-1",
    "1-10:0", "0-4194303%3", "0-4194304", "1%", "%2", "1,,2", "7:2", " 1-3 ", "1-3,2-4", "0-1000%4", "1000",
    "1001", "0-1001%2", "5-2000:500"]))


def script_has_array(script: str) -> bool:
    """sbatch's --array / -a among its #SBATCH directives: the pod is an array job
    (fit_admit_req.flags FIT_REQ_ARRAY), whatever the demand count.  sbatch reads directives up to
    the first line that is neither blank nor a comment (a plain comment line does not
    end them, unlike parse.go:36-46's header rule, which the demand itself follows)."""
    for line in script.split("\n"):
        body = line.lstrip(" \t\v\f\r")
        if body == "":
            continue
        if not body.startswith("#"):
            break
        if not line.startswith("#SBATCH"):
            continue
        if any(t == "--array" or t.startswith("--array=") or t.startswith("-a") for t in line[7:].split()):
            return True
    return False


def oracle_pod_demand(labels: dict, script, max_array_size: int = 1001):
    raw = [None if labels.get(k) is None else str(labels[k]).encode() for k in KEYS]
    arr = (C.c_char_p * 6)(*raw)
    out = np.zeros(4 * 64, np.int32)
    n = po.lib().ref_pod_demand(arr, None if script is None else script.encode(), C.c_int64(max_array_size),
                                out.ctypes.data_as(C.POINTER(C.c_int32)), 64)
    return n, out.reshape(64, 4)


@settings(max_examples=3000, deadline=None)
@given(SBATCH, INTS, INTS, INTS, INTS, ARRAYS, INTS, st.integers(0, 31), st.integers(-5, 1 << 40))
def test_pod_demand_matches_oracle(script, nodes, cpt, mpc, tpn, array, ntasks, part, prio):
    labels = {k: v for k, v in zip(KEYS, (nodes, cpt, mpc, tpn, array, ntasks)) if v is not None}
    n, ref = oracle_pod_demand(labels, script)
    try:
        got = fitgpu.pod_demand({POD_LABEL_KEYS[k]: v for k, v in labels.items()}, script, part, prio)
        rc = 0
    except ValueError:
        rc = -1  # FIT_E_PARSE
    except fitgpu.FitError:
        rc = -2  # FIT_E_INVAL
    if n < 0:
        assert rc == n, (labels, script)
        return
    assert rc == 0 and len(got) == n, (labels, script, got, n)
    arr = bool(labels.get("array")) or (script is not None and script_has_array(script))
    for i, g in enumerate(got[:64]):
        assert g == (prio, int(ref[i, 0]), int(ref[i, 1]), 0, int(ref[i, 2]), part, int(ref[i, 3]), int(arr))


def test_array_flag_after_a_comment_line():
    """sbatch keeps reading #SBATCH lines past plain comments, so an --array after
    one still makes the pod an array job (never pinned); a command line ends the directives."""
    base = "#!/bin/sh\n#SBATCH --nodes=1\n"
    flags = lambda sc: [r[7] for r in fitgpu.pod_demand({}, sc)]
    assert flags(base + "# stage the inputs\n#SBATCH --array=0-3%1\nsrun a\n") == [fitgpu.FIT_REQ_ARRAY]
    assert flags(base + "\n   \n#SBATCH -a 5\nsrun a\n") == [fitgpu.FIT_REQ_ARRAY]
    assert flags(base + "srun a\n#SBATCH --array=0-3\n") == [0]
    assert flags(base + "# only a comment\nsrun a\n") == [0]


def test_pod_demand_sample_manifest():
    """manifests/samples/kubecluster.org_v1alpha1_slurmbridgejob.yaml → the operator's labels
    (getResourceRequestLabelsForPod, pod.go:164-190) + its script: C1's demand (3 cpus, 1,500 MiB)."""
    script = "#!/bin/sh\n#SBATCH --nodes=1\nsrun hostname\nhostname\npwd\n"
    labels = {POD_LABEL_KEYS["ntasks"]: "3", POD_LABEL_KEYS["mem_per_cpu"]: "500",
              POD_LABEL_KEYS["cpus_per_task"]: "1"}
    assert fitgpu.pod_demand(labels, script, 0, 5) == [(5, 3, 1500, 0, 0, 0, 1, 0)]
    # --time in the script → walltime minutes (rounded up); an array label → one request per task
    script2 = script.replace("--nodes=1\n", "--nodes=1\n#SBATCH --time=1:30:30\n")
    labels[POD_LABEL_KEYS["array"]] = "1-4"
    assert fitgpu.pod_demand(labels, script2, 2, 9) == [(9, 3, 1500, 0, 91, 2, 1, 1)] * 4
    # a label overrides the script (a command-line flag beats an #SBATCH line, slurm.go:189-229)
    labels[POD_LABEL_KEYS["nodes"]] = "2"
    labels[POD_LABEL_KEYS["array"]] = "0-9%3"
    assert fitgpu.pod_demand(labels, script2) == [(0, 2, 1000, 0, 91, 0, 2, 1)] * 3  # ceil(3/2) tasks/node
    # a label strconv.ParseInt rejects is skipped (provider.go logs and goes on)
    assert fitgpu.pod_demand({POD_LABEL_KEYS["ntasks"]: "three"}, None) == [(0, 1, 1024, 0, 0, 0, 1, 0)]
    with pytest.raises(ValueError):
        fitgpu.pod_demand({POD_LABEL_KEYS["array"]: "1-10:x"}, None)
    with pytest.raises(ValueError):  # the reference panics on a bare last flag (parse.go:58-60)
        fitgpu.pod_demand({}, "#SBATCH --exclusive\n")
    with pytest.raises(fitgpu.FitError):  # more nodes than a job may take (FIT_MAX_K)
        fitgpu.pod_demand({POD_LABEL_KEYS["nodes"]: "9"}, None)


@pytest.mark.parametrize("expr,want", [("1-4", (4, 4)), ("0-15", (16, 16)), ("1,3,5-7", (5, 5)),
                                        ("0-15:4", (4, 4)), ("1-100%10", (100, 10)), ("1-10%2", (10, 2)),
                                        ("1-3,5", (4, 4)), ("1-3,2-4", (4, 4)), ("7", (1, 1)),
                                        ("1-10%20", (10, 10))])
def test_array_tasks(expr, want):
    assert fitgpu.array_tasks(expr) == want
    t, r = C.c_int64(), C.c_int64()
    assert po.lib().ref_array_tasks(expr.encode(), C.byref(t), C.byref(r)) == 0 and (t.value, r.value) == want
    # parseArrayLen (the reference) gets the %-limited and mixed forms wrong: 0 for "1-10%2"
    if expr in ("1-10%2", "1-3,5"):
        assert fitgpu.parse_array_len(expr) == 0


@pytest.mark.parametrize("expr", ["", "x", "1-", "4-1", "1-10:0", "0-4194304", "%2", "1%", "1,,2", "7:2", "1-3%0"])
def test_array_tasks_malformed(expr):
    with pytest.raises(ValueError):
        fitgpu.array_tasks(expr)
    t, r = C.c_int64(), C.c_int64()
    assert po.lib().ref_array_tasks(expr.encode(), C.byref(t), C.byref(r)) == -1


def test_pod_demand_max_array_size():
    """an array label is capped by Slurm's MaxArraySize (ids 0 .. MaxArraySize - 1,
    default 1001), as sbatch refuses it: one label can no longer become millions of requests."""
    big = {POD_LABEL_KEYS["array"]: "0-4194303%3"}
    with pytest.raises(fitgpu.FitError) as ei:
        fitgpu.pod_demand(big, None)
    assert ei.value.code == fitgpu._lib.FIT_E_INVAL and oracle_pod_demand({"array": "0-4194303%3"}, None)[0] == -2
    assert len(fitgpu.pod_demand({POD_LABEL_KEYS["array"]: "0-1000"}, None)) == 1001
    # a stepped range is bounded by the last id it reaches (0-1001:3 ends at 999)
    assert len(fitgpu.pod_demand({POD_LABEL_KEYS["array"]: "0-1001:3"}, None)) == 334
    assert oracle_pod_demand({"array": "0-1001:3"}, None)[0] == 334
    with pytest.raises(fitgpu.FitError):  # ... and 0-1002:3 reaches 1002
        fitgpu.pod_demand({POD_LABEL_KEYS["array"]: "0-1002:3"}, None)
    prev = fitgpu.set_max_array_size(4 << 20)
    try:
        assert prev == 1001
        assert len(fitgpu.pod_demand(big, None)) == 3
        assert oracle_pod_demand({"array": "0-4194303%3"}, None, 4 << 20)[0] == 3
        with pytest.raises(fitgpu.FitError):
            fitgpu.set_max_array_size(0)
    finally:
        fitgpu.set_max_array_size(prev)


@pytest.mark.parametrize("entries,want", [
    (["node[1-8]"], [f"node{i}" for i in range(1, 9)]),           # C1's Nodes= (the a3 case)
    (["node[1-3", "5]"], ["node1", "node2", "node3", "node5"]),   # parsePartition's split of node[1-3,5]
    (["gpu[01-02]-ib", "cpu7", "x[1-2][3-4]"], ["gpu01-ib", "gpu02-ib", "cpu7", "x13", "x14", "x23", "x24"]),
    ([], []),
])
def test_node_names(entries, want):
    """the engine's node-name table comes from the Partition RPC's list, expanded
    (fit_node_names), in the order `scontrol show nodes` is asked for them."""
    assert fitgpu.node_names(entries) == want


def test_node_names_errors():
    # a repeated name (no 1:1 record match) is FIT_E_PARSE — not the buffer-too-small FIT_E_INVAL
    # callers retry on with a larger buffer
    assert fitgpu.lib().fit_node_names(b"a\0a\0", 2, fitgpu.C.create_string_buffer(64), 64) == fitgpu._lib.FIT_E_PARSE
    assert fitgpu.lib().fit_node_names(b"a\0b\0", 2, fitgpu.C.create_string_buffer(2), 2) == fitgpu._lib.FIT_E_INVAL
    with pytest.raises(ValueError):
        fitgpu.node_names(["a", "a"])
    with pytest.raises(ValueError):
        fitgpu.node_names(["n[1-3]", "n2"])
    with pytest.raises(ValueError):
        fitgpu.node_names(["n[1-"])


def test_node_names_match_c1_records():
    """The C1 fixtures: Partition RPC → fit_node_names gives exactly the NodeName of every record
    of `scontrol show nodes`, in record order (cross-checked with fit_ingest_nodes)."""
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    part = open(os.path.join(g, "c1_scontrol_show_partition.txt")).read()
    nodes = open(os.path.join(g, "c1_scontrol_show_nodes.txt")).read()
    entries = fitgpu.parse_partition(part.strip())
    assert entries == ["node[1-8]"]
    names = fitgpu.node_names(entries)
    _, ingest_names = fitgpu.ingest_nodes(nodes, ["debug"])
    assert names == ingest_names and len(fitgpu.parse_nodes(nodes)) == len(names) == 8


NAMES = ["node01", "node02", "gpu-a", "gpu-b"]


@settings(max_examples=800, deadline=None)
@given(SBATCH, st.lists(st.integers(0, 3), min_size=1, max_size=4, unique=True))
def test_script_with_nodelist_keeps_the_header(script, nodes):
    """The directive lands at the end of the #SBATCH header: the header stays one block, so
    extractBatchResourcesFromScript reads the same resources (it ignores --nodelist), and the
    script after the header is untouched."""
    out = fitgpu.script_with_nodelist(script, NAMES, nodes)
    want = "#SBATCH --nodelist=" + ",".join(NAMES[i] for i in nodes)
    lines = out.split("\n")
    assert want in lines
    assert out.replace(want + "\n", "", 1) == script or out.replace("\n" + want + "\n", "\n", 1) == script or \
        out.replace(want + "\n", "", 1) == script + "\n"
    try:
        before = fitgpu.extract_batch_resources(script)
    except ValueError:
        return
    assert fitgpu.extract_batch_resources(out) == before
    # every line above the directive is a header line, the one after is not a #SBATCH line
    at = lines.index(want)
    assert all(ln == "" or ln.startswith("#!") or ln.startswith("#SBATCH") for ln in lines[:at])
    assert at + 1 >= len(lines) or not lines[at + 1].startswith("#SBATCH")


def test_script_with_nodelist_cases():
    s = "#!/bin/sh\n#SBATCH --nodes=2\n#SBATCH -w other\nsrun hostname\n"
    assert fitgpu.script_with_nodelist(s, NAMES, [2, 0]) == (
        "#!/bin/sh\n#SBATCH --nodes=2\n#SBATCH -w other\n#SBATCH --nodelist=gpu-a,node01\nsrun hostname\n")
    assert fitgpu.script_with_nodelist("srun x", NAMES, [1]) == "#SBATCH --nodelist=node02\nsrun x"
    assert fitgpu.script_with_nodelist("#!/bin/bash", NAMES, [3]) == "#!/bin/bash\n#SBATCH --nodelist=gpu-b\n"
    with pytest.raises(fitgpu.FitError):
        fitgpu.script_with_nodelist("x", NAMES, [4])  # node id outside the table


def test_partition_limits():
    # UNLIMITED walltime arrives as 0 s (a -1 ns Duration's Seconds(), api/slurm.go:309), -1 / 0 = none
    assert fitgpu.partition_limits(0, -1, 0) == (-1, -1, -1)
    assert fitgpu.partition_limits(1800, 64, 262144) == (30, 64, 262144)
    assert fitgpu.partition_limits(90, 1, 1) == (2, 1, 1)  # minutes rounded up like a job's --time


def test_node_columns():
    ns = [fitgpu.Node(64, 262144, 8, 12, 40960, 3), fitgpu.Node(32, 131072, 0, 40, 0, 0)]
    cols = fitgpu.node_columns(ns, part_mask=5)
    assert cols.cpu_free.tolist() == [52, -8] and cols.mem_free.tolist() == [221184, 131072]
    assert cols.gpu_free.tolist() == [5, 0] and cols.part_mask.tolist() == [5, 5]
    assert (cols.avail_min == np.iinfo(np.int32).max).all()
