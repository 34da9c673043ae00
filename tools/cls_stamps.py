"""Diagnostic: the class engine's decider (k_class, csrc/fit_class.hip) cycles by segment from the
FIT_STAMPS build (`make stamps`), for the longest component and summed over all.

    python tools/cls_stamps.py c3 [jobs]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libfitgpu_stamps.so")
from fitgpu import Engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
jj = int(sys.argv[2]) if len(sys.argv) > 2 else None
os.environ["FIT_ENGINE"] = "class"
if name.endswith("a"):
    nodes, jobs, parts = synth.make_array_config(name, None, jj)
else:
    nodes, jobs, parts = synth.make_config(name, None, jj)
kmax = 8 if name.startswith("c4") else 1
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    out, st = e.place(jobs, kmax=kmax)
    buf = (C.c_ulonglong * (2 * 32 * 8))()
    assert _lib.lib().fit_debug_class_stamps(buf) == 0
print(name, {k: st[k] for k in ("engine", "placed", "unplaced", "rounds", "stops_rescan", "ms_device", "ms_commit")})
names = ["extract+certify", "head: key (rows of B)", "refill / pick", "A issue + ring", "commit", "  (of refill: drain)"]
rows = [list(buf[c * 8:(c + 1) * 8]) for c in range(32)]
rows = [r for r in rows if r[6]]
longest = max(rows, key=lambda r: sum(r[:5]))  # [5] is a part of [2]
for label, r in (("longest component", longest), ("all components", [sum(x) for x in zip(*rows)])):
    jobs_n, commits = r[6], r[7]
    tot = sum(r[:5])
    print(f"{label}: jobs {jobs_n}, commits {commits}, {tot / max(jobs_n, 1):.0f} cycles/job "
          f"({tot / 2.4e6 / (1 if label.startswith('longest') else len(rows)):.2f} ms at 2.4 GHz)")
    for n, v in zip(names, r[:6]):
        print(f"  {n:16s} {v / max(jobs_n, 1):8.0f} cycles/job  {100 * v / max(tot, 1):5.1f} %")
op = [sum(buf[32 * 8 + c * 8 + i] for c in range(32)) for i in range(8)]
nref = max(op[5], 1)
print(f"refills (all components): {op[5]}, cycles per refill seen by the decider wave: "
      + ", ".join(f"{n} {v / nref:.0f}" for n, v in zip(["to barrier A", "scan + B1", "pool + B2", "set build", "barrier C"], op[:5])))
