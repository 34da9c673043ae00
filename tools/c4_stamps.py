"""Diagnostic: per-segment cycles of the single-wave commit (commit_window, fit_common.h) for
config C4's multi-node windows, from the FIT_STAMPS build (`make stamps`).  The persistent engine
commits a window holding a multi-node job on wave 0 alone; the stamps of each component's last
round are read back (fit_debug_commit_stamps)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libfitgpu_stamps.so")
from fitgpu import Engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c4"
nodes, jobs, parts = synth.make_config(name, None, int(sys.argv[2]) if len(sys.argv) > 2 else None)
os.environ["FIT_ENGINE"] = "rounds"  # the host-driven k_commit: its stamps are the ones read back
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    _, st = e.place(jobs, kmax=8 if name == "c4" else 1)
    buf = (C.c_ulonglong * (64 * 8))()
    assert _lib.lib().fit_debug_commit_stamps(buf) == 0
print({k: st[k] for k in ("placed", "unplaced", "rounds", "stops_rescan", "stops_dirty", "ms_device", "ms_commit")})
names = ["prefetch-issue", "clean-check", "candidate-min", "dirty-eval", "select/decide+update", "rotate+loop"]
tot = [0] * 6
jobs_n = 0
for c in range(64):
    row = buf[c * 8:(c + 1) * 8]
    jobs_n += row[6]
    for i in range(6):
        tot[i] += row[i]
s = sum(tot)
print(f"last-round jobs {jobs_n}  cycles/job {s / max(jobs_n, 1):.0f}")
for n, v in zip(names, tot):
    print(f"  {n:22s} {v / max(jobs_n, 1):8.0f} cycles/job  {100 * v / max(s, 1):5.1f} %")
