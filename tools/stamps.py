"""Diagnostic: per-segment cycle shares of k_commit from the FIT_STAMPS build (dev tool)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libfitgpu_stamps.so")
from fitgpu import Engine, synth  # noqa: E402

nodes, jobs, parts = synth.make_config("c3", None, int(sys.argv[1]) if len(sys.argv) > 1 else 100000)
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    e.place(jobs)  # last round's commit leaves its stamps
    buf = (C.c_ulonglong * (64 * 10))()
    assert _lib.lib().fit_debug_commit_stamps(buf) == 0
names = ["prefetch-issue", "clean-check", "dirty-eval", "reduction", "decide+update", "rotate+loop"]
tot = [0] * 6
jobs_n = 0
for c in range(64):
    row = buf[c * 10:(c + 1) * 10]
    jobs_n += row[6]
    for i in range(6):
        tot[i] += row[i]
s = sum(tot)
clk = [buf[c * 8 + 7] / 2**24 * 100 for c in range(64) if buf[c * 8 + 6]]
print(f"jobs {jobs_n}  cycles/job {s / max(jobs_n, 1):.0f}  in-kernel clock {sum(clk) / max(len(clk), 1):.0f} MHz")
for n, v in zip(names, tot):
    print(f"  {n:15s} {100 * v / max(s, 1):5.1f}%  {v / max(jobs_n, 1):7.1f} cyc/job")
