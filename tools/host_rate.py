"""Placements/s through the host-buffer boundary (fit_load_nodes + fit_place with host arrays,
i.e. what a cgo caller pays, PCIe copies included) — reported in DESIGN.md §5, never as bench
`value` (which has inputs resident in HBM)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import Engine, synth  # noqa: E402

res = {}
for wl in ("c3", "c5"):
    if wl == "c5":
        nodes, tline, jobs, parts = synth.make_c5()
    else:
        nodes, jobs, parts = synth.make_config("c3")
    with Engine() as e:
        e.load_partitions(parts)

        def step():
            e.load_nodes(nodes)
            if wl == "c5":
                e.load_timeline(tline)
                return e.place_tl(jobs)
            return e.place(jobs)
        step()
        t = time.perf_counter()
        for _ in range(3):
            step()
        el = (time.perf_counter() - t) / 3
    res[wl] = {"placements_per_s": round(jobs.j / el, 1), "ms_per_step": round(el * 1e3, 2)}
print(json.dumps(res))
