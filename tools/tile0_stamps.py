"""Diagnostic: where a round's staged first scan tile spends its time (FIT_TILE0_STAMPS build)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libfitgpu_tile0.so")
from fitgpu import Engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
nodes, jobs, parts = synth.make_config(name)
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    e.place(jobs)
    buf = (C.c_ulonglong * 8)()
    assert _lib.lib().fit_debug_tile0(buf) == 0
n = max(buf[7], 1)
names = ["job rows loaded", "rows staged in LDS", "wave 0's rows scanned", "merge tree"]
print(f"{name}: {n} staged first tiles; per tile (us): " +
      ", ".join(f"{k} {buf[i] / n / 100:.2f}" for i, k in enumerate(names)))
