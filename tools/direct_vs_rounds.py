"""Where k_small (the direct placement) stops beating the host-driven rounds: fit_place of a
B-job batch on the C3 table and on one VK's one-partition table, each engine forced
(FIT_ENGINE=direct / rounds), library clock (ms_total) median over repeats.  Sets the default
of FIT_SMALL_DIRECT (engine.cpp small_direct)."""
import json
import os
import sys

import numpy as np

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slurm-bridge-operator_amd")]
from fitgpu import Engine, synth  # noqa: E402


def tables():
    nodes, jobs, parts = synth.make_config("c3")
    sel = (nodes.part_mask & 1) != 0
    n1 = synth.Nodes(*(np.ascontiguousarray(x[sel]) for x in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free,
                                                               nodes.avail_min)), np.ones(int(sel.sum()), np.uint32))
    js = jobs.part == 0
    j1 = synth.Jobs(*(np.ascontiguousarray(x[js]) for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)),
                    np.zeros(int(js.sum()), np.uint16), np.ascontiguousarray(jobs.nodes_k[js]))
    p1 = synth.Partitions(*(np.ascontiguousarray(x[:1]) for x in (parts.max_time_min, parts.max_cpus_per_node,
                                                                   parts.max_mem_per_node)))
    return {"c3_table": (nodes, jobs, parts), "one_partition": (n1, j1, p1)}


def main():
    res = {}
    for tname, (tn, tj, tp) in tables().items():
        for eng in ("direct", "rounds"):
            os.environ["FIT_ENGINE"] = eng
            e = Engine(device=0)
            e.load_partitions(tp)
            for bs in (16, 64, 128, 256, 512, 1024, 2048):
                tot = []
                for rep in range(12):
                    e.load_nodes(tn)
                    sub = synth.Jobs(*(np.ascontiguousarray(x[rep * bs:(rep + 1) * bs])
                                       for x in (tj.cpu, tj.mem, tj.gpu, tj.wall, tj.part, tj.nodes_k)))
                    _, st = e.place(sub)
                    if rep >= 2:
                        tot.append(st["ms_total"])
                res.setdefault(tname, {}).setdefault(str(bs), {})[eng] = round(1e3 * float(np.median(tot)), 1)
            e.close()
            print(tname, eng, {b: v[eng] for b, v in res[tname].items()}, flush=True)
    print(json.dumps({"call_us_p50": res}))


if __name__ == "__main__":
    main()
