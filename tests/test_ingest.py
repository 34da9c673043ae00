"""Product ingest / demand / capacity helpers (host code in libfitgpu.so, no GPU needed) against
(1) the reference's own test tables and (2) the oracle restatement on fuzzed inputs."""
import ctypes as C
import json
import os

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

import fitgpu
from fitgpu import _lib
from oracle import pyoracle as po

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))


@pytest.mark.parametrize("case", GOLD["parse_duration"], ids=lambda c: repr(c["in"]))
def test_parse_duration_reference_table(case):
    if case["ns"] is None:
        exc = fitgpu.ErrDurationIsUnlimited if case["unlimited"] else ValueError
        with pytest.raises(exc):
            fitgpu.ParseDuration(case["in"])
    else:
        assert fitgpu.ParseDuration(case["in"]) == case["ns"]


@pytest.mark.parametrize("i", range(len(GOLD["parse_resources"])))
def test_parse_resources_reference_table(i):
    case = GOLD["parse_resources"][i]
    r = fitgpu.parse_resources(case["in"])
    w = case["want"]
    assert (r.Nodes, r.MemPerNode, r.CPUPerNode, r.WallTime) == (w["nodes"], w["mem_per_node"],
                                                                 w["cpu_per_node"], w["wall_ns"])


def test_parse_partitions_names_reference_table():
    for case in GOLD["parse_partitions_names"]:
        assert fitgpu.parse_partitions_names(case["in"]) == case["want"]


DUR_ALPHABET = st.text(alphabet="0123456789:-+ UNLIMTEDfoab", max_size=14)


def _ref_dur(s):
    ns = C.c_int64()
    rc = po.lib().ref_parse_duration(s.encode(), C.byref(ns))
    return rc, ns.value


@settings(max_examples=3000, deadline=None)
@given(DUR_ALPHABET)
def test_parse_duration_matches_oracle(s):
    rc, ns = _ref_dur(s)
    mine = C.c_int64()
    prc = _lib.lib().fit_parse_duration(s.encode(), C.byref(mine))
    expect = {0: 0, 1: _lib.FIT_E_UNLIMITED, -1: _lib.FIT_E_PARSE}[rc]
    assert prc == expect
    if rc == 0:
        assert mine.value == ns


FIELD = st.sampled_from(["MaxTime", "MaxCPUsPerNode", "TotalCPUs", "MaxMemPerNode", "MaxNodes",
                         "TotalNodes", "Nodes", "PartitionName", "CPUTot", "CPUAlloc", "RealMemory",
                         "AllocMem", "Other"])
VALUE = st.one_of(st.sampled_from(["UNLIMITED", "", "00:30:00", "1-00:00:00", "512", "-1", "abc", "7,8",
                                   "99999999999999999999", "3-5", "x=y"]),
                  st.integers(-5, 10**6).map(str))
TEXT = st.lists(st.tuples(FIELD, VALUE, st.sampled_from([" ", "\n   ", "\t", "\n\n"])), max_size=12).map(
    lambda fs: "".join(f"{k}={v}{sep}" for k, v, sep in fs))


class RefRes(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("mem_per_node", C.c_int64), ("cpu_per_node", C.c_int64),
                ("wall_ns", C.c_int64)]


class RefNode(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("cpus", "memory", "gpus", "allo_cpus", "allo_memory", "allo_gpus")]


@settings(max_examples=1500, deadline=None)
@given(TEXT)
def test_parse_resources_matches_oracle(text):
    r = RefRes()
    rc = po.lib().ref_parse_resources(text.encode(), C.byref(r))
    m = _lib.FitResources()
    prc = _lib.lib().fit_parse_resources(text.encode(), C.byref(m))
    assert (prc == 0) == (rc == 0)
    if rc == 0:
        assert (m.nodes, m.mem_per_node, m.cpu_per_node, m.wall_ns) == (r.nodes, r.mem_per_node,
                                                                         r.cpu_per_node, r.wall_ns)


@settings(max_examples=1500, deadline=None)
@given(TEXT)
def test_parse_nodes_matches_oracle(text):
    cap = 64
    ref = (RefNode * cap)()
    n = po.lib().ref_parse_nodes(text.encode(), ref, cap)
    mine = fitgpu.parse_nodes(text, cap)
    assert len(mine) == n
    for a, b in zip(mine, ref[:n]):
        assert (a.Cpus, a.Memory, a.Gpus, a.AlloCpus, a.AlloMemory) == (b.cpus, b.memory, b.gpus, b.allo_cpus,
                                                                        b.allo_memory)
    buf = C.create_string_buffer(8192)
    rn = po.lib().ref_parse_partition(text.encode(), buf, 8192)
    assert fitgpu.parse_partition(text) == [s.decode() for s in buf.raw.split(b"\0")[:rn]]
    rn = po.lib().ref_parse_partitions_names(text.encode(), buf, 8192)
    assert fitgpu.parse_partitions_names(text) == [s.decode() for s in buf.raw.split(b"\0")[:rn]]


SHOW_NODES = """NodeName=node1 Arch=x86_64 CoresPerSocket=16
   CPUAlloc=12 CPUTot=64 CPULoad=0.50
   AvailableFeatures=(null)
   Gres=gpu:4 GresUsed=gpu:1
   NodeAddr=node1 NodeHostName=node1
   RealMemory=262144 AllocMem=40960 FreeMem=200000 Sockets=2 Boards=1
   State=MIXED ThreadsPerCore=1 TmpDisk=0 Weight=1 Owner=N/A
   Partitions=debug
   CfgTRES=cpu=64,mem=256G,billing=64,gres/gpu=4

NodeName=node2 Arch=x86_64 CoresPerSocket=16
   CPUAlloc=0 CPUTot=32 CPULoad=0.00
   RealMemory=131072 AllocMem=0 FreeMem=130000 Sockets=2 Boards=1
   State=IDLE ThreadsPerCore=1 TmpDisk=0 Weight=1 Owner=N/A
   Partitions=debug
"""


def test_parse_nodes_fixture():
    """Build-authored `scontrol show nodes` fixture (the reference has none): Gres is not parsed
    and keys with a second '=' (CfgTRES=cpu=...) are skipped, as in parse.go:291-308."""
    ns = fitgpu.parse_nodes(SHOW_NODES)
    assert [(n.Cpus, n.AlloCpus, n.Memory, n.AlloMemory, n.Gpus) for n in ns] == [
        (64, 12, 262144, 40960, 0), (32, 0, 131072, 0, 0)]
    cap = fitgpu.get_partition_capacity(ns)  # node.go:169-199 arithmetic, MiB × 2048 quirk kept
    assert cap == {"cpu": 96, "memory": (262144 + 131072) * 2048, "pods": 96}


SBATCH_LINES = st.lists(st.sampled_from([
    "#SBATCH --nodes=2", "#SBATCH -N 3", "#SBATCH --nodes=2-4", "#SBATCH --time=1:00:00", "#SBATCH -t 30",
    "#SBATCH --time=UNLIMITED", "#SBATCH --mem-per-cpu=500", "#SBATCH --cpus-per-task=4", "#SBATCH -c 2",
    "#SBATCH --ntasks-per-node=8", "#SBATCH --exclusive --nodes=2", "#SBATCH --exclusive", "#SBATCH --time=foo",
    "#!/bin/sh", "", "srun hostname", "#SBATCH --ntasks=3", "#SBATCH --mem-per-cpu 2048"]), max_size=8).map(
    "\n".join)


class RefJob(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("nodes", "cpus_per_task", "ntasks", "ntasks_per_node", "mem_per_cpu",
                                         "wall_ns")] + [("array", C.c_char * 64)]


@settings(max_examples=2000, deadline=None)
@given(SBATCH_LINES, st.integers(0, 4), st.integers(0, 8), st.integers(0, 4096), st.integers(0, 16),
       st.sampled_from(["", "1-10", "1,2,3", "1-10%2", "0-0", "x-y", "5"]), st.integers(0, 32))
def test_demand_derivation_matches_oracle(script, nodes, cpt, mpc, tpn, array, ntasks):
    ref = RefJob()
    rc = po.lib().ref_extract_batch_resources(script.encode(), C.byref(ref))
    try:
        mine = fitgpu.extract_batch_resources(script)
        prc = 0
    except ValueError:
        prc = -1
    # reference errors (-1) and reference panics (-3) both surface as FIT_E_PARSE
    assert (prc == 0) == (rc == 0)
    if rc != 0:
        return
    assert (mine.Nodes, mine.CpusPerTask, mine.Ntasks, mine.NtasksPerNode, mine.MemPerCpu, mine.WallTime) == (
        ref.nodes, ref.cpus_per_task, ref.ntasks, ref.ntasks_per_node, ref.mem_per_cpu, ref.wall_ns)
    po.lib().ref_apply_spec_and_defaults(C.byref(ref), C.c_int64(nodes), C.c_int64(cpt), C.c_int64(mpc),
                                         C.c_int64(tpn), array.encode(), C.c_int64(ntasks))
    mine = fitgpu.apply_spec(mine, nodes, cpt, mpc, tpn, array, ntasks)
    assert (mine.Nodes, mine.CpusPerTask, mine.MemPerCpu, mine.NtasksPerNode, mine.Ntasks, mine.Array) == (
        ref.nodes, ref.cpus_per_task, ref.mem_per_cpu, ref.ntasks_per_node, ref.ntasks, ref.array.decode())
    rc_cpu, rc_mem = C.c_int64(), C.c_int64()
    po.lib().ref_pod_request(C.byref(ref), C.byref(rc_cpu), C.byref(rc_mem))
    req = fitgpu.gen_resource_list_for_pod(mine)
    assert (req["cpu"], req["memory"]) == (rc_cpu.value, rc_mem.value)
    if array:
        assert fitgpu.parse_array_len(array) == po.lib().ref_parse_array_len(array.encode())


def test_sample_job_demand():
    """manifests/samples/kubecluster.org_v1alpha1_slurmbridgejob.yaml:12-25 → C1's per-node demand."""
    script = "#!/bin/sh\n#SBATCH --nodes=1\nsrun hostname\nhostname\npwd\n"
    r = fitgpu.apply_spec(fitgpu.extract_batch_resources(script), ntasks=3, mem_per_cpu=500, cpus_per_task=1)
    assert fitgpu.gen_resource_list_for_pod(r) == {"cpu": 3, "memory": 3 * 500 * 1024}  # pod.go:143-162
    assert fitgpu.job_demand(r) == (3, 1500, 0, 1)


def test_bare_last_flag_is_an_error_not_a_crash():
    # the reference indexes params[j+1] out of range here (parse.go:58-60) and panics
    with pytest.raises(ValueError):
        fitgpu.extract_batch_resources("#SBATCH --exclusive\n")
    ref = RefJob()
    assert po.lib().ref_extract_batch_resources(b"#SBATCH --exclusive\n", C.byref(ref)) == -3


def test_parse_array_len_quirks():
    assert fitgpu.parse_array_len("1-10") == 10
    assert fitgpu.parse_array_len("1,2,3") == 3
    assert fitgpu.parse_array_len("1-10%2") == 0  # Atoi("10%2") fails → 0 - 1 + 1 (parse.go:126-135)
