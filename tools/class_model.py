"""Driver of tools/class_model.c (diagnostic): a commit chain on persistent
demand-class candidate lists, modelled on one component of a BASELINE config before any kernel is
built.  Prints the class count, list exhaustions per 1k jobs, classes re-evaluated and changed per
commit, and a VALU / LDS estimate of the chain's step (cost model in the header below).

    gcc -O2 -shared -fPIC -o tools/libclass_model.so tools/class_model.c
    python tools/class_model.py c3 16 [nodes jobs] [--check]

Step cost model (one wave owns the classes, ceil(C / 64) per lane; gfx950 lone-wave figures from
DESIGN.md §3.7: a VALU op ≈ 4.7 cycles, an LDS round trip 48–64, a branch 25–30):
  per commit, every class:    16 VALU per class slot   (old and new key: 2 × (3 subs, sign test,
                                                         mask test, 3 mins, 2 packs) shared subs,
                                                         membership test vs L, insert test)
  per changed list:           18 VALU + 1 LDS round trip (wave-parallel sorted update of one list:
                                                         ballot for the old / new position, two DPP
                                                         row shifts, write back)
  per query:                  12 VALU + 1 LDS round trip (read the class list, first entries with
                                                         avail >= wall by ballot, readlane)
  per exhaustion:             a component scan (N / 64 × 16 VALU) + the refill (the same again)
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
from fitgpu import synth  # noqa: E402

FIELDS = ["jobs", "placed", "unplaced", "dead_fast", "commits", "evals_commit", "affected", "affected_max",
          "inserts", "moves", "drops", "evicts", "query_entries", "exhaust", "refills", "mismatches",
          "first_mismatch", "lim_pick", "skipped_wall"]


class Stats(C.Structure):
    _fields_ = [(f, C.c_int64) for f in FIELDS]


VALU_CYC, LDS_CYC = 4.7, 56.0


def component0(name, nn, jj):
    nodes, jobs, parts = synth.make_config(name, nn, jj)
    sel = (nodes.part_mask & 1) != 0  # partition 0's component (C2 / C3 / C4: partition 0 alone)
    mt, mc, mm = parts.max_time_min[0], parts.max_cpus_per_node[0], parts.max_mem_per_node[0]
    js = (jobs.part == 0) & ~((mt >= 0) & (jobs.wall > mt)) & ~((mc >= 0) & (jobs.cpu > mc)) & \
        ~((mm >= 0) & (jobs.mem > mm))
    cols = [np.ascontiguousarray(a[sel], np.int32) for a in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free,
                                                            nodes.avail_min)]
    mk = np.ascontiguousarray(nodes.part_mask[sel], np.uint32)
    shape = np.stack([jobs.part[js].astype(np.int64), jobs.cpu[js], jobs.mem[js], jobs.gpu[js]], axis=1)
    uniq, cls = np.unique(shape, axis=0, return_inverse=True)
    return cols, mk, cls.astype(np.int32).ravel(), np.ascontiguousarray(jobs.wall[js], np.int32), \
        np.ascontiguousarray(jobs.nodes_k[js], np.uint16), uniq


def run(name, K, nn=None, jj=None, check=False, lazy=False, evict_max=False):
    L = C.CDLL(os.path.join(ROOT, "tools", "libclass_model.so"))
    (cf, mf, gf, av), mk, cls, wall, kk, uniq = component0(name, nn, jj)
    n, j, nc = len(cf), len(cls), len(uniq)
    ccpu, cmem, cgpu = (np.ascontiguousarray(uniq[:, i], np.int32) for i in (1, 2, 3))
    cpart = np.ascontiguousarray(uniq[:, 0], np.uint16)
    out = np.full(j * 8, -1, np.int32)
    S = Stats()
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    t0 = time.time()
    if lazy:
        L.class_chain_lazy(n, P(cf), P(mf), P(gf), P(av), P(mk), j, P(cls), P(wall), P(kk), nc, P(ccpu), P(cmem),
                           P(cgpu), P(cpart), K, int(check), int(evict_max), P(out), C.byref(S))
    else:
        L.class_chain(n, P(cf), P(mf), P(gf), P(av), P(mk), j, P(cls), P(wall), P(kk), nc, P(ccpu), P(cmem),
                      P(cgpu), P(cpart), K, int(check), P(out), C.byref(S))
    s = {f: getattr(S, f) for f in FIELDS}
    slots = -(-nc // 64)
    if lazy:
        return report_lazy(name, n, j, nc, slots, K, s, check, evict_max, t0)
    per_job = {
        "commit_valu": s["commits"] * slots * 16 / j,
        "list_valu": s["affected"] * 18 / j, "list_lds": s["affected"] / j,
        "query_valu": 12.0, "query_lds": 1.0,
        "exhaust_valu": s["exhaust"] * 2 * (n / 64) * 16 / j,
    }
    valu = per_job["commit_valu"] + per_job["list_valu"] + per_job["query_valu"] + per_job["exhaust_valu"]
    lds = per_job["list_lds"] + per_job["query_lds"]
    cyc = valu * VALU_CYC + lds * LDS_CYC
    print(f"{name} component 0: {n} nodes, {j} jobs, {nc} classes ({slots} per lane), K={K}: "
          f"placed {s['placed']}, unplaced {s['unplaced']} ({s['dead_fast']} with an empty list), "
          f"mismatches {s['mismatches'] if check else 'unchecked'} | per 1k jobs: exhaustions "
          f"{1000 * s['exhaust'] / j:.1f} | per commit: {s['affected'] / max(s['commits'], 1):.2f} lists changed "
          f"(max {s['affected_max']}; inserts {s['inserts']}, moves {s['moves']}, drops {s['drops']}, evicts "
          f"{s['evicts']}) | per query: {s['query_entries'] / j:.2f} entries, {s['skipped_wall'] / j:.3f} skipped by "
          f"walltime | commits per job {s['commits'] / j:.2f} | est. per job: {valu:.0f} VALU + {lds:.2f} LDS "
          f"≈ {cyc:.0f} cycles (commit {per_job['commit_valu']:.0f}, lists {per_job['list_valu']:.0f}, "
          f"exhaust {per_job['exhaust_valu']:.0f}) | {time.time() - t0:.1f}s", flush=True)
    return s, cyc


def report_lazy(name, n, j, nc, slots, K, s, check, evict_max, t0):
    """Lazy sets: per commit every class slot evaluates the node (14 VALU) after one LDS read of the
    node's class-membership mask (2 VALU per slot); a changed set is an exec-masked LDS write (6
    VALU); a query gathers the set's rows (1 LDS round trip per 64 entries), evaluates them (16
    VALU per 64), takes a DPP wave minimum (14 VALU) and compares with L (4); an exhaustion is a
    component scan and a refill (2 × N / 64 × 16 VALU); a full-set eviction check evaluates the set
    (16 VALU per 64 entries + 14 for its maximum)."""
    per64 = -(-K // 64)
    commit_valu = s["commits"] * slots * 16 / j
    aff_valu = s["affected"] * 6 / j
    evict_valu = s["moves"] * (16 * per64 + 14) / j
    query_valu = 16 * per64 + 18
    exhaust_valu = s["exhaust"] * 2 * (n / 64) * 16 / j
    valu = commit_valu + aff_valu + evict_valu + query_valu + exhaust_valu
    lds = s["commits"] / j + per64
    cyc = valu * VALU_CYC + lds * LDS_CYC
    print(f"{name} component 0 LAZY{' evict-max' if evict_max else ''}: {n} nodes, {j} jobs, {nc} classes "
          f"({slots} per lane), K={K}: placed {s['placed']}, unplaced {s['unplaced']}, mismatches "
          f"{s['mismatches'] if check else 'unchecked'} | per 1k jobs: exhaustions {1000 * s['exhaust'] / j:.1f} | "
          f"per commit: {s['affected'] / max(s['commits'], 1):.2f} sets touched (inserts {s['inserts']}, bound "
          f"drops {s['evicts']}, full-set checks {s['moves']}) | entry drops {s['drops']} | per query "
          f"{s['query_entries'] / j:.1f} entries | commits per job {s['commits'] / j:.2f} | est. per job: "
          f"{valu:.0f} VALU + {lds:.2f} LDS ≈ {cyc:.0f} cycles (commit {commit_valu:.0f}, query {query_valu:.0f}, "
          f"exhaust {exhaust_valu:.0f}, evict {evict_valu:.0f}) | {time.time() - t0:.1f}s", flush=True)
    return s, cyc


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    name, K = args[0], int(args[1])
    nn = int(args[2]) if len(args) > 2 else None
    jj = int(args[3]) if len(args) > 3 else None
    run(name, K, nn, jj, "--check" in sys.argv, "--lazy" in sys.argv, "--evict-max" in sys.argv)
