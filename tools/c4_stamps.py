"""Diagnostic: per-segment cycles of the single-wave commit (commit_window, fit_common.h) for
config C4's multi-node windows, from the FIT_STAMPS build (`make stamps`), summed over the run.  The persistent engine
commits a window holding a multi-node job on wave 0 alone; argv[3] picks the engine whose
stamps are read (rounds: k_commit; persistent: engine_commit_single)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libfitgpu_stamps.so")
from fitgpu import Engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c4"
nodes, jobs, parts = synth.make_config(name, None, int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] else None)
eng = sys.argv[3] if len(sys.argv) > 3 else "rounds"
os.environ["FIT_ENGINE"] = eng  # rounds: k_commit's stamps; persistent: engine_commit_single's
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    kmax = 8 if name == "c4" else 1
    out, st = e.place(jobs, kmax=kmax)
    buf = (C.c_ulonglong * (64 * 10))()
    rd = _lib.lib().fit_debug_commit_stamps_pe if eng == "persistent" else _lib.lib().fit_debug_commit_stamps
    assert rd(buf) == 0
print({k: st[k] for k in ("placed", "unplaced", "rounds", "stops_rescan", "stops_dirty", "ms_device", "ms_commit")})
# segments between STAMP(i-1) and STAMP(i) of FIT_COMMIT_STEP (fit_common.h): key loads issued +
# clean flags of the next job; candidate minimum; dirty-row keys; k = 1: the wave minimum / k > 1:
# select_k; the decision's bookkeeping (k > 1: the picks' updates); the ring rotation
names = ["loads+clean-flags", "candidate-min", "dirty-eval", "wave-min | select_k", "decide+update"]
tot = [0] * 6
jobs_n = 0
below = [0, 0]
for c in range(64):
    row = buf[c * 10:(c + 1) * 10]
    jobs_n += row[6]
    below[0] += row[8]
    below[1] += row[9]
    for i in range(6):
        tot[i] += row[i]
# [5]: not cycles — the multi-node jobs' picks that were dirty rows (STAMP_CNT)
dpk = tot[5]
tot[5] = 0
s = sum(tot)
import numpy as np  # noqa: E402
o = np.asarray(out).reshape(-1, kmax)
k = np.asarray(jobs.nodes_k).astype(np.int64)
multi = (k > 1) & (o[:, 0] >= 0)
picks = int(k[multi].sum())
print(f"multi-node jobs placed {int(multi.sum())}, picks {picks}, dirty-row picks {dpk} "
      f"({100 * dpk / max(picks, 1):.1f} %); jobs with k..16 fitting dirty rows {below[0]}, and of "
      f"them all k picks dirty {below[1]}")
print(f"{eng}: jobs {jobs_n}  cycles/job {s / max(jobs_n, 1):.0f}")
for n, v in zip(names, tot):
    print(f"  {n:22s} {v / max(jobs_n, 1):8.0f} cycles/job  {100 * v / max(s, 1):5.1f} %")
