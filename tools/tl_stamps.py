"""Diagnostic: cycle split of k_commit_tl (FIT_STAMPS build of the C5 commit; dev tool)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import _lib  # noqa: E402
_lib.LIB_PATH = os.environ.get("FITGPU_STAMPS_LIB") or os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libfitgpu_stamps.so")
from fitgpu import Engine, synth  # noqa: E402

nn = int(sys.argv[1]) if len(sys.argv) > 1 else None
jj = int(sys.argv[2]) if len(sys.argv) > 2 else None
nodes, tline, jobs, parts = synth.make_c5(nn, jj)
buf = (C.c_ulonglong * (64 * 12 + 8))()
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    e.load_timeline(tline)
    assert _lib.lib().fit_debug_tl_stamps(buf, 1) == 0
    node, start, st = e.place_tl(jobs)
    assert _lib.lib().fit_debug_tl_stamps(buf, 0) == 0
print({k: st[k] for k in ("ms_total", "ms_scan", "ms_commit", "rounds", "stops_rescan", "stops_dirty", "placed")})
tot = [sum(buf[c * 12 + i] for c in range(64)) for i in range(12)]
j = max(tot[5], 1)
if tot[11] and tot[4] == 0:  # decider / helper commit, coarse stamps
    print(f"decider: loop {tot[1] / j:.0f} cycles/job, first-record wait {tot[0] / max(tot[8], 1):.0f} cycles/round "
          f"({tot[8]} rounds), new dirty per job {tot[6] / j:.2f}, jobs that walked {tot[9] / j:.3f}, "
          f"round-end write-back {tot[7] / j:.0f} cycles/job; helpers: snapshot -> record "
          f"{tot[10] / max(tot[11], 1):.0f} cycles over {tot[11]} records")
    for c in range(64):
        r = buf[c * 12:(c + 1) * 12]
        if r[5]:
            print(f"  comp {c:2d} jobs {r[5]:6d} rounds {r[8]:4d} loop/job {r[1] / r[5]:6.0f} "
                  f"first-record wait/round {r[0] / max(r[8], 1):7.0f}  total {(r[0] + r[1]) / 2.4e6:6.1f} ms @2.4GHz")
elif tot[11]:  # decider / helper commit, fine stamps (FIT_STAMPS_FINE)
    apply_other = tot[8] - tot[3] - tot[4]
    print("decider cycles/job: " + ", ".join(f"{n} {v / j:.0f}" for n, v in (
        ("record wait", tot[0]), ("decision", tot[1]), ("exception (walks, global lists)", tot[2]),
        ("new-dirty copy", tot[3]), ("reservation", tot[4]), ("bookkeeping", apply_other))) +
          f"; sum {(tot[0] + tot[1] + tot[2] + tot[8]) / j:.0f}; jobs {tot[5]}")
    print(f"new dirty per job {tot[6] / j:.2f}; jobs that walked {tot[9] / j:.3f}; "
          f"round-end write-back {tot[7] / j:.0f} cycles/job; helpers: snapshot -> record "
          f"{tot[10] / max(tot[11], 1):.0f} cycles over {tot[11]} records")
else:  # single-wave commit
    names = ["clean", "dirty-eval", "new-dirty", "reserve", "tail"]
    print("cycles/job: " + ", ".join(f"{n} {tot[i] / j:.0f}" for i, n in enumerate(names)) +
          f"; new dirty per job {tot[6] / j:.2f}; write-back per job {tot[7] / j:.0f}; jobs {tot[5]}")
    print(f"new-dirty: header/runs wait + LDS copy + prefix minima {tot[11] / max(tot[6], 1):.0f} cycles per new dirty node")
    print(f"dirty-eval split: fast {tot[8] / j:.0f}, walk {tot[9] / j:.0f} (walks per job {tot[10] / j:.2f}), "
          f"reduce {(tot[1] - tot[8] - tot[9]) / j:.0f}")
sc = buf[64 * 12:64 * 12 + 8]
if sc[7]:
    print(f"round's first tile: pickup delay {sc[5] / sc[7] / 100:.1f} us, scan {sc[6] / sc[7] / 100:.1f} us "
          f"(per task, {sc[7]} tasks)")
print(f"scan: waves {sc[4]}, nodes/wave {sc[1] / max(sc[4], 1):.0f}, cycles/node {sc[0] / max(sc[1], 1):.0f}, "
      f"long-walk batches/node {sc[2] / max(sc[1], 1):.2f}, nodes with > 4 runs {sc[3] / max(sc[1], 1):.2%}")
