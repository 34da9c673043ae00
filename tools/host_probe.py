"""Diagnostic: where the host-buffer step's time goes (fit_load_nodes / fit_place with pinned host
arrays vs their HBM-resident twins), min / median over repetitions.  Dev tool, not a test."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import Engine, synth  # noqa: E402


def pinned(keep, a):
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint16): np.int16, np.dtype(np.uint32): np.int32}.get(a.dtype)
    t = torch.from_numpy(a.view(view) if view else a).pin_memory()
    keep.append(t)
    out = t.numpy()
    return out.view(a.dtype) if view else out


if "--bind" in sys.argv:  # host thread on the CPUs local to GPU 0 (intersected with what we may use)
    import glob
    allowed = os.sched_getaffinity(0)
    for f in sorted(glob.glob("/sys/class/drm/card*/device/local_cpulist")):
        txt = open(f).read().strip()
        cpus = set()
        for part in txt.split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        print(f, txt, "allowed", len(allowed), "local&allowed", len(cpus & allowed))
        if cpus & allowed:
            os.sched_setaffinity(0, cpus & allowed)
            break
nodes, jobs, parts = synth.make_config("c3")
keep = []
hn = synth.Nodes(*(pinned(keep, x) for x in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free, nodes.avail_min, nodes.part_mask)))
hj = synth.Jobs(*(pinned(keep, x) for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, jobs.nodes_k)))
ho = pinned(keep, np.zeros(jobs.j, np.int32))
dev = torch.device("cuda", 0)
T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
dn = [T(nodes.cpu_free), T(nodes.mem_free), T(nodes.gpu_free), T(nodes.avail_min), T(nodes.part_mask.view(np.int32))]
dj = [T(jobs.cpu), T(jobs.mem), T(jobs.gpu), T(jobs.wall), T(jobs.part.view(np.int16)), T(jobs.nodes_k.view(np.int16))]
do = torch.empty(jobs.j, dtype=torch.int32, device=dev)
with Engine() as e:
    e.load_partitions(parts)
    res = {}
    for name, fn in (("load_nodes_host", lambda: e.load_nodes(hn)),
                     ("place_host", lambda: e.place(hj, kmax=1, out=ho)),
                     ("load_nodes_dev", lambda: e.load_nodes_device(*dn)),
                     ("place_dev", lambda: e.place_device(*dj, do, kmax=1))):
        ts = []
        for r in range(12):
            if name.startswith("place"):
                e.load_nodes(hn)
            torch.cuda.synchronize()
            t = time.perf_counter()
            st = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        ts = sorted(ts[2:])
        res[name] = (round(ts[0], 3), round(ts[len(ts) // 2], 3))
        if name.startswith("place"):
            s = st[1] if isinstance(st, tuple) else st
            res[name + "_ms_device"] = round(s.get("ms_device", 0.0), 3) if isinstance(s, dict) else None
    print(res)
