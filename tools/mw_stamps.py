"""Diagnostic: decider / helper cycle split of the multi-wave commit (FIT_STAMPS build; dev tool)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu",
                             sys.argv[2] if len(sys.argv) > 2 else "libfitgpu_stamps.so")
if len(sys.argv) > 2 and os.path.sep in sys.argv[2]:  # a variant build elsewhere in the tree
    _lib.LIB_PATH = os.path.join(ROOT, sys.argv[2])
from fitgpu import Engine, synth  # noqa: E402

W = 24  # stamps per component (MW_NSTAMP)
name = sys.argv[1] if len(sys.argv) > 1 else "c3"
nodes, jobs, parts = synth.make_array_config(name) if name.endswith("a") else synth.make_config(name)
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    out, st = e.place(jobs)
    buf = (C.c_ulonglong * (64 * W))()
    assert _lib.lib().fit_debug_mw_stamps(buf) == 0
print({k: st[k] for k in ("ms_total", "ms_commit", "ms_device", "rounds")})
tot = [sum(buf[c * W + i] for c in range(64)) for i in range(W)]
dj, hj = max(tot[2], 1), max(tot[5], 1)
print(f"decider: {tot[0] / dj:.0f} cyc/job, waiting for records (slow path) {tot[1] / dj:.0f} cyc/job")
t0n = max(sum(buf[c * W + 11] for c in range(64)), 1)
print(f"round's first tile: pickup delay {sum(buf[c * W + 10] for c in range(64)) / t0n / 100:.1f} us, "
      f"scan {sum(buf[c * W + 12] for c in range(64)) / t0n / 100:.1f} us (per task, {t0n} tasks)")
print(f"helpers: tile waits {tot[13] / hj:.0f} cyc/job, snapshot -> record {tot[14] / hj:.0f} cyc/job "
      f"(of which snapshot -> extraction start {tot[15] / hj:.0f})")
rn = max(tot[18], 1)
print(f"round start: round end -> tiles published {tot[16] / rn:.0f} cyc, decider start -> record 0 "
      f"{tot[17] / rn:.0f} cyc (per round, {tot[18]} rounds over all components)")
print(f"helpers: {tot[3] / hj:.0f} cyc/job (per helper), waiting for snapshot {tot[4] / hj:.0f}, "
      f"items/job {tot[6] / hj:.2f}")
for c in range(64):
    r = buf[c * W:(c + 1) * W]
    if r[2]:
        print(f"  comp {c:2d} jobs {r[2]:6d} dec {r[0] / r[2]:6.0f} wait {r[1] / r[2]:6.0f} | "
              f"help {r[3] / max(r[5], 1):6.0f} wait {r[4] / max(r[5], 1):6.0f}")
