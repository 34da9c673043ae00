"""Dev tool: place the C5 backfill workload a few times with the default library (profiling target)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import Engine, synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nodes, tline, jobs, parts = synth.make_c5()
with Engine() as e:
    for _ in range(reps):
        e.load_nodes(nodes)
        e.load_partitions(parts)
        e.load_timeline(tline)
        _, _, st = e.place_tl(jobs)
        print({k: st[k] for k in ("ms_total", "ms_commit", "rounds", "placed")}, flush=True)
