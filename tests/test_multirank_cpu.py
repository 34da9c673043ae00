"""N>1 path on CPU: (1) node sharding keeps the round algorithm exact (CPU model with shards);
(2) the host exchange ops the engine calls, over a real world-size-2 gloo group."""
import ctypes as C
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from fitgpu import synth
from oracle import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_node_sharding_is_exact_in_model(shards):
    nodes, jobs, parts = synth.make_config("c3", 3000, 30000)
    ref, _, _ = po.ref_place(nodes, jobs, parts)
    out, st, _ = po.model_place(nodes, jobs, parts, slice=64, ks=16, km=64, shards=shards)
    assert np.array_equal(out, ref[:, 0])


WORKER = r'''
import ctypes as C, os, sys
import numpy as np
sys.path[:0] = [sys.argv[3], os.path.join(sys.argv[3], "slurm-bridge-operator_amd")]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
import torch.distributed as dist
rank = int(sys.argv[1]); dist.init_process_group("gloo", rank=rank, world_size=2)
from fitgpu import TorchHostExchange
from fitgpu._lib import FIT_XCHG_ALLGATHER_U64, FIT_XCHG_MIN_U64, FIT_XCHG_MAX_I32, FIT_XCHG_MIN_I32
x = TorchHostExchange()
INF = np.uint64(2**64 - 1)
g = np.zeros(6, np.uint64); g[rank * 3:(rank + 1) * 3] = [rank + 1, INF, 7 + rank]
assert x.fn(None, FIT_XCHG_ALLGATHER_U64, g.ctypes.data, 3) == 0
assert g.tolist() == [1, 2**64 - 1, 7, 2, 2**64 - 1, 8], g
m = np.array([INF, 5 + rank, 2**63 + rank], np.uint64)
assert x.fn(None, FIT_XCHG_MIN_U64, m.ctypes.data, 3) == 0
assert m.tolist() == [2**64 - 1, 5, 2**63], m
a = np.array([-1, -2, rank * 10 - 1], np.int32)
assert x.fn(None, FIT_XCHG_MAX_I32, a.ctypes.data, 3) == 0 and a.tolist() == [-1, -2, 9]
b = np.array([rank, 100 - rank], np.int32)
assert x.fn(None, FIT_XCHG_MIN_I32, b.ctypes.data, 2) == 0 and b.tolist() == [0, 99]
dist.destroy_process_group()
'''


def test_host_exchange_ops_gloo_world2(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    w = tmp_path / "w.py"
    w.write_text(WORKER)
    root = os.path.dirname(HERE)
    ps = [subprocess.Popen([sys.executable, str(w), str(r), str(port), root]) for r in range(2)]
    assert [p.wait(timeout=120) for p in ps] == [0, 0]
