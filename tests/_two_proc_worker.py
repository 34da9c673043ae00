"""Child process of tests/test_watchdog_gpu.py::test_two_processes_mixed_fit_and_backfill: one
virtual kubelet's engine (its own process and context on GPU 0) placing the same workload several
times, starting at a shared wall-clock instant so that its persistent launches overlap the other
process's.  Writes every result to an .npz for the parent, which checks them against the oracle."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

from fitgpu import Engine, synth  # noqa: E402


def main(kind: str, start_at: float, rounds: int, out_path: str) -> None:
    if kind == "fit":
        nodes, jobs, parts = synth.make_config("c3", 20000, 60000, shard=1)
    elif kind == "c3o":
        nodes, jobs, parts = synth.make_config("c3o", 8192, 30000)
    else:
        nodes, tline, jobs, parts = synth.make_c5(4096, 16384)
    res, waits, engines = [], [], []
    with Engine(device=0) as e:
        e.load_partitions(parts)
        time.sleep(max(0.0, start_at - time.time()))
        for _ in range(rounds):
            e.load_nodes(nodes)
            if kind == "tl":
                e.load_timeline(tline)
                node, start, st = e.place_tl(jobs)
                res.append(np.stack([node, start]))
            else:
                out, st = e.place(jobs)
                res.append(out[:, 0].copy())
            waits.append(st["ms_arb_wait"])
            engines.append(st["engine"])
    np.savez(out_path, res=np.stack(res), waits=np.array(waits), engines=np.array(engines))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
