"""Quick engine probe: one placement of a BASELINE config, stats printed as JSON (dev tool)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
if os.environ.get("FIT_LIB"):  # a variant build of the library (dev experiments)
    from fitgpu import _lib  # noqa: E402
    _lib.LIB_PATH = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", os.environ["FIT_LIB"])
from fitgpu import Engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nodes, jobs, parts = synth.make_config(name)
for r in range(reps):
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        t = time.perf_counter()
        out, st = e.place(jobs)
        dt = time.perf_counter() - t
    st["wall_s"] = dt
    st["placements_per_s"] = jobs.j / dt
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}), flush=True)
