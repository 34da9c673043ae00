"""Diagnostic: intrinsic cycles/job of the decider loop alone (no helpers; dev tool)."""
import ctypes as C
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "libdecbench.so"))
for w in (1000, 8000):
    buf = (C.c_ulonglong * 4)()
    assert lib.dec_bench(w, buf) == 0
    print(f"w={w}: {buf[0] / max(buf[1], 1):.0f} cycles/job  (done {buf[1]}, placed {buf[2]}, dirty {buf[3]})")
