"""One-off wide fuzz sweep (not part of the suite): tests/test_fuzz_gpu.py's random cases for seeds
[lo, hi), each placed by every engine (persistent, rounds, direct, class — the class engine where the table
qualifies, else its fallback) and compared bit-exactly with
the oracle (placements, final node state, counters); and the backfill cases of the same seeds
(persistent and rounds engines: nodes, start slots, final timelines, counters).  Prints one line per 50 seeds and a summary;
exits non-zero at the first mismatch, naming seed and engine.

    python tools/fuzz_sweep.py 1000 1500 > gpurun_out/<tag>_fuzz_sweep.txt
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from fitgpu import Engine  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from test_fuzz_gpu import random_case  # noqa: E402


def main(lo: int, hi: int) -> int:
    t0 = time.time()
    cases = jobs_total = multi = 0
    for seed in range(lo, hi):
        nodes, jobs, parts, kmax = random_case(seed)
        ref, rst, rfin = po.ref_place(nodes, jobs, parts, kmax=kmax)
        for eng in ("persistent", "rounds", "direct", "class"):
            os.environ["FIT_ENGINE"] = eng
            with Engine() as e:
                e.load_nodes(nodes)
                e.load_partitions(parts)
                out, st = e.place(jobs, kmax=kmax)
                fin = e.read_nodes()
            bad = np.flatnonzero((out != ref).any(axis=1))
            if bad.size or any(not np.array_equal(a, b) for a, b in zip(fin, rfin)) or \
                    (st["placed"], st["unplaced"], st["rejected"]) != (rst["placed"], rst["unplaced"], rst["rejected"]):
                where = f"job {bad[0]}: {out[bad[0]]} vs {ref[bad[0]]}" if bad.size else "node state / counters"
                print(f"MISMATCH seed {seed} engine {eng} kmax {kmax}: {where}", flush=True)
                return 1
            cases += 1
        nodes, tl, tjobs, parts = random_case(seed, timeline=True)
        rn, rs, rst, rfin = po.ref_place_tl(nodes, tl, tjobs, parts)
        live = nodes.part_mask != 0
        for eng in ("persistent", "rounds"):
            os.environ["FIT_ENGINE"] = eng
            with Engine() as e:
                e.load_nodes(nodes)
                e.load_partitions(parts)
                e.load_timeline(tl)
                node, start, st = e.place_tl(tjobs)
                fin = e.read_timeline()
            bad = np.flatnonzero((node != rn) | (start != rs))
            if bad.size or not np.array_equal(fin[live], rfin[live]) or \
                    (st["placed"], st["unplaced"], st["rejected"]) != (rst["placed"], rst["unplaced"], rst["rejected"]):
                where = f"job {bad[0]}" if bad.size else "timelines / counters"
                print(f"MISMATCH backfill seed {seed} engine {eng}: {where}", flush=True)
                return 1
            cases += 1
        jobs_total += len(jobs.cpu)
        multi += int((np.asarray(jobs.nodes_k) > 1).sum())
        if (seed - lo + 1) % 50 == 0:
            print(f"seeds {lo}..{seed}: ok ({cases} placements, {time.time() - t0:.0f} s)", flush=True)
    print(f"all ok: {hi - lo} seeds x (4 placement + 2 backfill engines) = {cases} runs, {jobs_total} jobs "
          f"({multi} multi-node), {time.time() - t0:.0f} s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]), int(sys.argv[2])))
