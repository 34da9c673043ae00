"""Diagnostic: intrinsic cycles/job of the decider loop alone (no helpers; dev tool)."""
import ctypes as C
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys
name = sys.argv[1] if len(sys.argv) > 1 else "libdecbench.so"
lib = C.CDLL(os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", name))
for w in (1000, 8000):
    buf = (C.c_ulonglong * 12)()
    assert lib.dec_bench(w, buf) == 0
    print(f"{name} w={w}: {buf[0] / max(buf[1], 1):.0f} cycles/job  (done {buf[1]}, placed {buf[2]}, "
          f"dirty {buf[3]})")
    if any(buf[4:12]):
        print("  segments (cycles/job, incl. ~40/stamp):", [round(buf[4 + i] / max(buf[1], 1)) for i in range(8)])
