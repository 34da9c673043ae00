"""Diagnostic: distribution of run-list lengths after a full C5 placement (dev tool)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import Engine, synth  # noqa: E402

nodes, tline, jobs, parts = synth.make_c5()
with Engine() as e:
    e.load_nodes(nodes)
    e.load_partitions(parts)
    e.load_timeline(tline)
    node, start, st = e.place_tl(jobs)
    fin = e.read_timeline()
runs = 1 + (fin[:, 1:, :] != fin[:, :-1, :]).any(axis=2).sum(axis=1)
print("placed", st["placed"], "future starts", int((start > 0).sum()))
print("runs per node: mean %.1f p50 %d p90 %d p99 %d max %d; > 32: %.2f%%, > 64: %.2f%%" % (
    runs.mean(), np.percentile(runs, 50), np.percentile(runs, 90), np.percentile(runs, 99), runs.max(),
    100 * (runs > 32).mean(), 100 * (runs > 64).mean()))
