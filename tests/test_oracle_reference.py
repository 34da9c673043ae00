"""The oracle is pinned by the reference's own Go test tables (tests/golden/reference_vectors.json,
transcribed from pkg/slurm-agent/parse_test.go by tools/make_golden.py)."""
import ctypes as C
import json
import os

import pytest

from oracle import pyoracle as po

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))


class RefRes(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("mem_per_node", C.c_int64), ("cpu_per_node", C.c_int64),
                ("wall_ns", C.c_int64)]


@pytest.mark.parametrize("case", GOLD["parse_duration"], ids=lambda c: repr(c["in"]))
def test_oracle_parse_duration(case):  # TestParseDuration, parse_test.go:26-122
    ns = C.c_int64()
    rc = po.lib().ref_parse_duration(case["in"].encode(), C.byref(ns))
    if case["ns"] is None:
        assert rc != 0
        assert (rc == 1) == case["unlimited"]
    else:
        assert rc == 0 and ns.value == case["ns"]


@pytest.mark.parametrize("i", range(len(GOLD["parse_resources"])))
def test_oracle_parse_resources(i):  # Test_parseResources, parse_test.go:224-258
    case = GOLD["parse_resources"][i]
    r = RefRes()
    assert po.lib().ref_parse_resources(case["in"].encode(), C.byref(r)) == 0
    assert {k: getattr(r, k) for k, _ in RefRes._fields_} == case["want"]


def test_oracle_parse_partitions_names():  # Test_parsePartitionsNames, parse_test.go:296-314
    for case in GOLD["parse_partitions_names"]:
        buf = C.create_string_buffer(4096)
        n = po.lib().ref_parse_partitions_names(case["in"].encode(), buf, 4096)
        assert [s.decode() for s in buf.raw.split(b"\0")[:n]] == case["want"]
