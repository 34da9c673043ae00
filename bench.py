#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X: placements/sec (+ job×node fit evals/sec)
at 100k nodes × 1M jobs (config C3, 16 partitions).

A "step" is one complete placement of the 1M-job stream against a freshly loaded 100k-node table,
timed under BASELINE.md's rule — inputs already in HOST memory (pinned buffers, as a cgo caller
would hand them over), wall time of fit_load_nodes + fit_place end to end (H2D, the placement,
D2H of the placements).  That rate is `value`.  The same placement from HBM-resident inputs
(fit_load_nodes_device + fit_place_device) is reported as `kernel_path_value`.

N > 1 (default --scaling weak; SURVEY §8 e): the placement partitions into
independent units (partition components), so every rank places its own 100k × 1M cluster shard
(a disjoint slice of the generator's streams) with no collective in the data path; `value` is the
placements of all ranks ÷ the slowest rank's time.  --scaling strong splits ONE 100k × 1M
placement over the ranks instead: --shard-mode auto (default) gives each rank whole partition
components (C3: 16 components, 2 per rank at N = 8), then one RCCL merge; --shard-mode nodes splits
every component's nodes (north_star's layout: RCCL allgather of the candidate lists + u64
min-allreduce of the bounds per round, host-driven rounds).  Either way a strong step is bounded
by the longest component's serial commit chain, so strong scaling is flat (DESIGN.md §3.5 gives
the predicted curves); a strong N > 1 run also reports the weak rate as the extra key
`weak_scaling` (--no-weak-extra skips it).

    python bench.py [--gpus N --steps K --warmup W] [--workload c3|c3o|c2|c5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` is live: per-launch kernel time from the engine's HIP
events (on the engine's stream), algorithmic work from DESIGN.md §5; `traffic` comes from the
committed PMC profile named in `traffic_source`.  `cpu_baseline` times the CPU restatements
(oracle/: naive port, component-aware, multicore) on bounded samples of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]

import numpy as np  # noqa: E402

PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # int32 lane-ops/s: 256 CU × 4 SIMD32 × 2.4 GHz
PEAK_HBM_GBS = 8000.0
SCAN_OPS_PER_EVAL = 12    # algorithmic int32 ops per (job, node) fit eval
SCAN_BYTES_PER_EVAL = 20  # algorithmic node-row bytes per eval (pre-reuse)
# The GPU box's CPU share for one GPU: the lease runs one GPU's command on 16 cores (OMP_NUM_THREADS
# is set to 16 there), while nproc / os.cpu_count() count the whole machine's CPUs — so "all host
# cores" (BASELINE.md:22) is this share, not nproc; cpu_baseline's host object states both.
CPU_THREADS = int(os.environ.get("OMP_NUM_THREADS") or 16)


def commit_bytes_per_job(entries: int) -> int:
    return entries * 8 + 32 + 8 + 4  # candidate keys + job row + bound + placement


def kernel_table(agg, stats, steps, world, evals_local, names=("k_scan", "k_commit"), engine="k_engine"):
    """Per-kernel live timings (engine HIP events) and their rooflines.

    Persistent engine (engine == 1): ONE k_engine launch per step; its duration is ms_device.  The
    scan work it contains is VALU-bound (12 int32 ops per performed eval); the serial commit chain
    inside it is latency-bound and reported as ns per committed job.
    Host-driven rounds (engine == 0): one k_scan + one k_commit launch per round."""
    rounds = max(agg["rounds"], 1)
    jobs_resolved = agg["placed"] + agg["unplaced"]
    if all(s.get("engine", 0) == 3 for s in stats):
        # demand-class engine: ONE k_class launch per step, one workgroup per
        # component; its work is the serial chain (queries of <= 64 set candidates, commits
        # evaluated against every class, set refills), VALU-issue-bound in one wave per component
        ms = agg["ms_device"] / steps
        ops = evals_local / steps * SCAN_OPS_PER_EVAL
        tops = ops / (ms * 1e-3) / 1e12
        return {"k_class": {
            "ms_per_launch": round(ms, 4), "launches": steps, "bound": "valu",
            "achieved": round(tops, 4), "peak": round(PEAK_VALU_TOPS, 1), "unit": "Tops/s",
            "frac": round(tops / PEAK_VALU_TOPS, 5),
            "hbm_gbs_algorithmic": round(evals_local / steps * SCAN_BYTES_PER_EVAL / (ms * 1e-3) / 1e9, 1),
            "commit_chain_ms": round(agg["ms_commit"] / steps, 3),
            "commit_ns_per_job": round(agg["ms_commit"] * 1e6 / max(jobs_resolved, 1), 1),
            "set_refills_longest_component": agg["rounds"] / steps}}
    if all(s.get("engine", 0) == 1 for s in stats):
        ms = agg["ms_device"] / steps
        ops = evals_local / steps * SCAN_OPS_PER_EVAL
        tops = ops / (ms * 1e-3) / 1e12
        return {engine: {
            "ms_per_launch": round(ms, 4), "launches": steps, "bound": "valu",
            "achieved": round(tops, 3), "peak": round(PEAK_VALU_TOPS, 1), "unit": "Tops/s",
            "frac": round(tops / PEAK_VALU_TOPS, 4),
            "hbm_gbs_algorithmic": round(evals_local / steps * SCAN_BYTES_PER_EVAL / (ms * 1e-3) / 1e9, 1),
            "scan_worker_busy_ms": round(agg["ms_scan"] / steps, 3),
            "commit_chain_ms": round(agg["ms_commit"] / steps, 3),
            "commit_ns_per_job": round(agg["ms_commit"] * 1e6 / max(jobs_resolved, 1), 1),
            "rounds_longest_component": agg["rounds"] / steps}}
    scan_ms = agg["ms_scan"] / rounds
    commit_ms = agg["ms_commit"] / rounds
    evals_per_launch = evals_local / rounds
    scan_tops = evals_per_launch * SCAN_OPS_PER_EVAL / (scan_ms * 1e-3) / 1e12
    entries = 64 * (world if stats[-1]["shard_mode"] == 1 else 1)
    commit_gbs = jobs_resolved / rounds * commit_bytes_per_job(entries) / (commit_ms * 1e-3) / 1e9
    return {
        names[0]: {"ms_per_launch": round(scan_ms, 4), "launches": rounds, "bound": "valu",
                   "achieved": round(scan_tops, 3), "peak": round(PEAK_VALU_TOPS, 1), "unit": "Tops/s",
                   "frac": round(scan_tops / PEAK_VALU_TOPS, 4),
                   "hbm_gbs_algorithmic": round(evals_per_launch * SCAN_BYTES_PER_EVAL / (scan_ms * 1e-3) / 1e9, 1)},
        names[1]: {"ms_per_launch": round(commit_ms, 4), "launches": rounds, "bound": "latency",
                   "achieved": round(commit_gbs, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(commit_gbs / PEAK_HBM_GBS, 5)},
    }


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c3o", "c4", "c5", "c2a", "c3a", "c5a", "admit"],
                    help="c3: BASELINE headline (100k x 1M); c3o: c3 + an all-nodes partition (one "
                         "component); c4: GPU-heavy nodes (8 GPUs) with multi-node jobs (--nodes=k, "
                         "k in {1,2,4,8}, kmax 8); c5: c3 with a 1,024-slot backfill horizon; admit: CreatePod "
                         "admission latency (10 concurrent callers against the c3 node table); c2a / c3a / "
                         "c5a: the same clusters with an array-expanded pending queue (runs of identical "
                         "pods, synth.expand_arrays) — not a BASELINE config")
    ap.add_argument("--repeats", type=int, default=3,
                    help="timed runs of --steps steps each; value = their median (BASELINE.md:26)")
    ap.add_argument("--no-shard-price", action="store_true",
                    help="skip the one-GPU price of north_star's node-sharded layout (c3 / c3o)")
    ap.add_argument("--admit-pods", type=int, default=300, help="admit: pods per caller thread")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="skip the in-run rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) that measure "
                         "roofline.traffic; the committed --pmc-json profile is used instead")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-scale", type=float, default=1.0, help="scale the CPU-baseline samples (tests)")
    ap.add_argument("--no-device-path", action="store_true", help="skip the HBM-resident rate")
    ap.add_argument("--rehearse", action="store_true",
                    help="test only: every rank on cuda:0 with gloo (rehearse N>1 on a 1-GPU box)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC summary (tools/gpu_pmc.sh + tools/pmc_json.py) with HBM bytes/launch")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N>1: strong = one 100k x 1M placement split over the ranks (--shard-mode); "
                         "weak = every rank places its own 100k x 1M cluster shard (no data-path collective)")
    ap.add_argument("--no-weak-extra", action="store_true",
                    help="N>1 strong: skip the extra weak-scaling leg (the `weak_scaling` key)")
    ap.add_argument("--shard-mode", default="auto", choices=["auto", "nodes", "components"],
                    help="strong scaling split: auto = partition components when there are >= N "
                         "of them (C3), else nodes (north_star's node sharding)")
    return ap.parse_args()


def _pinned(keep, a):
    """Copy of numpy array `a` in page-locked host memory (what a caller would hand the C-ABI)."""
    import torch
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint16): np.int16, np.dtype(np.uint32): np.int32}.get(a.dtype)
    t = torch.from_numpy(a.view(view) if view else a).pin_memory()
    keep.append(t)
    out = t.numpy()
    return out.view(a.dtype) if view else out


def main():
    a = parse_args()
    if a.workload == "admit":
        import torch
        torch.cuda.set_device(0)
        return admission(a)
    import torch
    import torch.distributed as dist

    from fitgpu import (FIT_SHARD_AUTO, FIT_SHARD_COMPONENTS, FIT_SHARD_NODES, Engine, TorchHostExchange,
                        nccl_unique_id, synth)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world == 1 and a.gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    if a.rehearse:  # test only: all ranks on cuda:0, gloo; strong runs exchange through the host
        local = 0
    torch.cuda.set_device(local)
    weak = world > 1 and a.scaling == "weak"
    nid = None
    if world > 1:
        if a.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if not weak and not a.rehearse:
            obj = [nccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            nid = obj[0]
    shard = rank if weak else 0  # weak: this rank's own cluster shard (disjoint generator slice)

    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    tl = a.workload in ("c5", "c5a")
    if a.workload.endswith("a"):
        if shard:
            raise SystemExit("array-expanded workloads: strong scaling or one GPU only")
        cfg = synth.make_array_config(a.workload)
        nodes, tline, jobs, parts = cfg if tl else (cfg[0], None, cfg[1], cfg[2])
    elif tl:
        nodes, tline, jobs, parts = synth.make_c5(shard=shard)
    else:
        nodes, jobs, parts = synth.make_config(a.workload, shard=shard)
    kmax = 8 if a.workload == "c4" else 1  # C4: --nodes=k up to 8 (FIT_MAX_K)

    mode = {"auto": FIT_SHARD_AUTO, "nodes": FIT_SHARD_NODES, "components": FIT_SHARD_COMPONENTS}[a.shard_mode]
    if weak:
        eng = Engine(device=local)  # independent shard: no collective in the data path
    elif a.rehearse:
        eng = Engine(device=local, rank=rank, world=world, shard_mode=mode, exchange=TorchHostExchange())
    else:
        eng = Engine(device=local, rank=rank, world=world, nccl_id=nid, shard_mode=mode)
    eng.load_partitions(parts)

    # ---- host-memory path (BASELINE.md timing rule): pinned inputs, H2D ... D2H per step ------------
    keep = []
    h_nodes = synth.Nodes(*(_pinned(keep, x) for x in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free,
                                                        nodes.avail_min, nodes.part_mask)))
    h_jobs = synth.Jobs(*(_pinned(keep, x) for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part,
                                                      jobs.nodes_k)))
    h_out = _pinned(keep, np.zeros(jobs.j * kmax, np.int32))
    if tl:
        h_tline = synth.Timeline(tline.slots, tline.slot_min,
                                 *(_pinned(keep, x) for x in (tline.off, tline.slot, tline.cpu, tline.mem, tline.gpu)))
        h_start = _pinned(keep, np.zeros(jobs.j, np.int32))

    def step_host():
        eng.load_nodes(h_nodes)
        if tl:
            eng.load_timeline(h_tline)
            return eng.place_tl(h_jobs, node=h_out, start=h_start)[2]
        return eng.place(h_jobs, kmax=kmax, out=h_out)[1]

    # ---- HBM-resident path (kernel_path_value) --------------------------------------------------
    dev = torch.device("cuda", local)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    d_nodes = [T(nodes.cpu_free), T(nodes.mem_free), T(nodes.gpu_free), T(nodes.avail_min),
               T(nodes.part_mask.view(np.int32))]
    d_jobs = [T(jobs.cpu), T(jobs.mem), T(jobs.gpu), T(jobs.wall), T(jobs.part.view(np.int16)),
              T(jobs.nodes_k.view(np.int16))]
    d_out = torch.empty(jobs.j * kmax, dtype=torch.int32, device=dev)
    if tl:
        d_rel = [T(x) for x in (tline.off, tline.slot, tline.cpu, tline.mem, tline.gpu)]
        d_start = torch.empty(jobs.j, dtype=torch.int32, device=dev)

    def step_dev():
        eng.load_nodes_device(*d_nodes)
        if tl:
            eng.load_timeline_device(tline.slots, tline.slot_min, *d_rel)
            return eng.place_tl_device(*d_jobs[:5], d_out, d_start)
        return eng.place_device(*d_jobs, d_out, kmax=kmax)

    cdev = torch.device("cpu") if a.rehearse else dev  # gloo reduces CPU tensors

    def timed_once(step, steps):
        stats = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            stats.append(step())
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, stats

    def timed(step, repeats=None):
        """W warmup steps, then `repeats` timed runs of exactly K steps each (barrier +
        synchronize on both sides, max over ranks); returns the median run's time, its stats and
        every run's time (BASELINE.md:26: median of 3)."""
        for _ in range(a.warmup):
            step()
        runs = [timed_once(step, a.steps) for _ in range(max(1, repeats or a.repeats))]
        order = sorted(range(len(runs)), key=lambda i: runs[i][0])
        el, stats = runs[order[len(runs) // 2]]
        return el, stats, [r[0] for r in runs]

    el, stats_host, runs_host = timed(step_host)
    s0 = stats_host[-1]
    assert s0["placed"] + s0["unplaced"] + s0["rejected"] == jobs.j  # output sanity every run
    mult = world if weak else 1
    value = jobs.j * a.steps / el * mult
    el_dev, stats, runs_dev = (None, stats_host, None) if a.no_device_path else timed(step_dev)

    agg = {k: sum(s[k] for s in stats) for k in ("rounds", "evals", "useful_evals", "ms_scan", "ms_commit",
                                                  "ms_exchange", "ms_device", "placed", "unplaced")}
    evals_local = agg["evals"]
    if world > 1:  # performed / useful evaluations summed over ranks
        t = torch.tensor([float(agg["evals"]), float(agg["useful_evals"])], dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        agg["evals"], agg["useful_evals"] = int(t[0].item()), int(t[1].item())
    el_k = el_dev if el_dev is not None else el
    used_mode = {0: "1 GPU", 1: f"node-sharded x{world} (RCCL allgather + u64 min-allreduce per round)",
                 2: f"partition-component-sharded x{world} (one RCCL merge)"}[stats[-1]["shard_mode"]]
    if weak:
        used_mode = f"{world} independent cluster shards (one per GPU, no data-path collective)"
    kernels = kernel_table(agg, stats, a.steps, world, evals_local,
                           ("k_scan_tl", "k_commit_tl") if tl else ("k_scan", "k_commit"),
                           "k_engine_tl" if tl else "k_engine")
    dominant = max(kernels, key=lambda k: kernels[k]["ms_per_launch"] * kernels[k]["launches"])
    k = kernels[dominant]
    traffic, traffic_src = None, None
    if world == 1 and not a.no_live_pmc:
        traffic, traffic_src = live_traffic(a.workload, dominant)
    if traffic is None and a.pmc_json and os.path.exists(a.pmc_json):
        pmc = json.load(open(a.pmc_json))
        traffic = pmc.get(dominant, {}).get("hbm_bytes_per_launch")
        traffic_src = f"{os.path.relpath(a.pmc_json, ROOT)} ({pmc.get('source', '?')})" if traffic else None
    roofline = {"kernel": dominant, "bound": k["bound"], "achieved": k["achieved"], "peak": k["peak"],
                "unit": k["unit"], "frac": k["frac"], "traffic": traffic, "traffic_source": traffic_src}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(a.workload, nodes, jobs, parts, tline if tl else None, a.cpu_scale, kmax)

    resolved = s0["placed"] + s0["unplaced"]
    line = {
        "metric": base["metric"], "value": round(value, 1), "unit": "placements/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak" if (weak or world == 1) else "strong", "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (splitmix64 generator, fitgpu/synth.py; DESIGN.md §5); inputs in pinned host "
                "memory, timed H2D..D2H (BASELINE.md timing rule)",
        "config": {"workload": a.workload, "nodes": nodes.n * mult, "jobs": jobs.j * mult,
                   "partitions": parts.p * mult, "per_gpu": {"nodes": nodes.n, "jobs": jobs.j} if weak else None,
                   **({"slots": tline.slots, "slot_min": tline.slot_min} if tl else {}),
                   "parallelism": used_mode, "components": stats[-1]["components"]},
        "timing": {"repeats": len(runs_host), "statistic": "median (BASELINE.md:26)",
                   "value_runs": [round(jobs.j * a.steps / r * mult, 1) for r in runs_host],
                   "kernel_path_value_runs": [round(jobs.j * a.steps / r * mult, 1) for r in runs_dev] if runs_dev
                   else None},
        "kernel_path_value": round(jobs.j * a.steps / el_dev * mult, 1) if el_dev else None,
        "kernel_path_ms_per_step": round(el_dev / a.steps * 1e3, 3) if el_dev else None,
        "placed_plus_unplaced_per_s": round(resolved * a.steps / el * mult, 1),
        "jobs": {"placed": s0["placed"], "unplaced": s0["unplaced"], "rejected_by_prefilter": s0["rejected"]},
        "fit_evals_per_s": {"useful": round(agg["useful_evals"] / el_k, 1),
                            "performed": round(agg["evals"] / el_k, 1)},
        "rounds_per_step": agg["rounds"] / a.steps,
        "round_stops_per_step": {"rescan": stats[-1]["stops_rescan"], "dirty_full": stats[-1]["stops_dirty"]},
        "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
    }
    if cpu:
        line["speedup_vs_cpu"] = {v["kind"]: round(value / v["value"], 1) for v in cpu["variants"]}
    if world == 1 and not tl and a.workload in ("c3", "c3o") and not a.no_shard_price:
        line["node_sharding_1gpu"] = shard_price(Engine, FIT_SHARD_NODES, parts, h_nodes, h_jobs, h_out,
                                                 kmax, el / a.steps * 1e3)
    if world > 1 and not weak and not a.no_weak_extra:
        # extra key: the same ranks, each placing its own 100k x 1M cluster shard (disjoint generator
        # slice, its own partitions; no collective in the data path), aggregate rate, host path
        eng.close()
        if tl:
            wn, wt, wj, wp = synth.make_c5(shard=rank)
        else:
            wn, wj, wp = synth.make_config(a.workload, shard=rank)
        weng = Engine(device=local)
        weng.load_partitions(wp)
        wkeep = []
        wh_nodes = synth.Nodes(*(_pinned(wkeep, x) for x in (wn.cpu_free, wn.mem_free, wn.gpu_free,
                                                              wn.avail_min, wn.part_mask)))
        wh_jobs = synth.Jobs(*(_pinned(wkeep, x) for x in (wj.cpu, wj.mem, wj.gpu, wj.wall, wj.part,
                                                            wj.nodes_k)))
        wh_out = _pinned(wkeep, np.zeros(wj.j * kmax, np.int32))
        if tl:
            wh_tl = synth.Timeline(wt.slots, wt.slot_min,
                                   *(_pinned(wkeep, x) for x in (wt.off, wt.slot, wt.cpu, wt.mem, wt.gpu)))
            wh_start = _pinned(wkeep, np.zeros(wj.j, np.int32))

        def step_weak():
            weng.load_nodes(wh_nodes)
            if tl:
                weng.load_timeline(wh_tl)
                return weng.place_tl(wh_jobs, node=wh_out, start=wh_start)[2]
            return weng.place(wh_jobs, kmax=kmax, out=wh_out)[1]

        wel, _, _ = timed(step_weak)
        weng.close()
        line["weak_scaling"] = {"value": round(wj.j * a.steps / wel * world, 1), "unit": "placements/s",
                                "ms_per_step": round(wel / a.steps * 1e3, 3), "scaling": "weak",
                                "per_gpu": {"nodes": wn.n, "jobs": wj.j},
                                "parallelism": f"{world} independent cluster shards (one per GPU, no "
                                               "data-path collective)"}
    else:
        eng.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def live_traffic(workload, kernel, timeout=240):
    """HBM bytes per launch of `kernel`, measured now: two rocprofv3 --pmc passes (FETCH_SIZE,
    WRITE_SIZE: separate runs, MI355X_MICROARCH.md HBM section) over a one-step child run of this
    bench (the program directly after `--`), FETCH_SIZE doubled per the guide's gfx950 correction
    (tools/pmc_json.py).  (None, None) when rocprofv3 is not usable here."""
    import csv
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None, None
    vals = {}
    base = tempfile.mkdtemp(prefix="fitgpu_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(base, ctr)
            cmd = ["rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                   sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--steps", "1",
                   "--warmup", "1", "--repeats", "1", "--no-cpu", "--no-device-path", "--no-shard-price",
                   "--no-live-pmc"]
            r = subprocess.run(cmd, timeout=timeout, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            if r.returncode != 0:
                return None, None
            per = {}
            for path in __import__("glob").glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(path)):
                    if row["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0] == kernel:
                        key = row["Dispatch_Id"]
                        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
            if not per:
                return None, None
            vals[ctr] = sum(per.values()) / len(per)
    except (subprocess.TimeoutExpired, OSError, KeyError, ValueError):
        return None, None
    finally:
        shutil.rmtree(base, ignore_errors=True)
    b = int(vals["FETCH_SIZE"] * 1024 * 2 + vals["WRITE_SIZE"] * 1024)
    return b, ("live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over a 1-step child run of this bench "
               "(KiB; FETCH_SIZE x2 gfx950 correction; MALL hits included)")


def shard_price(Engine, FIT_SHARD_NODES, parts, h_nodes, h_jobs, h_out, kmax, ms_default, steps=3):
    """North_star's node-sharded layout priced on one GPU: the same
    placement through the multi-rank code path at world 1 (FIT_FLAG_COLLECTIVES: a one-rank RCCL
    communicator; per round the candidate allgather + u64 min-allreduce of the bounds, host-driven
    rounds) against the default persistent engine."""
    from fitgpu import FIT_FLAG_COLLECTIVES
    # RCCL prints its version banner on stdout when the communicator comes up: keep this process'
    # stdout to the one JSON line (fd-level, the banner is written by the native library)
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return _shard_price(Engine, FIT_SHARD_NODES, FIT_FLAG_COLLECTIVES, parts, h_nodes, h_jobs, h_out, kmax,
                            ms_default, steps)
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def _shard_price(Engine, FIT_SHARD_NODES, FIT_FLAG_COLLECTIVES, parts, h_nodes, h_jobs, h_out, kmax, ms_default,
                 steps):
    e = Engine(device=0, shard_mode=FIT_SHARD_NODES, flags=FIT_FLAG_COLLECTIVES)
    e.load_partitions(parts)
    e.load_nodes(h_nodes)
    e.place(h_jobs, kmax=kmax, out=h_out)  # warmup
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = None
    for _ in range(steps):
        e.load_nodes(h_nodes)
        st = e.place(h_jobs, kmax=kmax, out=h_out)[1]
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    e.close()
    return {"ms_per_step": round(ms, 3), "vs_default": round(ms / ms_default, 2), "steps": steps,
            "rounds": st["rounds"], "ms_exchange": round(st["ms_exchange"], 3),
            "path": "FIT_SHARD_NODES via FIT_FLAG_COLLECTIVES at world 1: host-driven rounds, RCCL allgather of "
                    "the candidate sections + ncclMin of the bounds every round"}


def admission(a):
    """CreatePod admission latency: 10 threads — the virtual kubelet's
    PodSyncWorkers (options/options.go:107), one pod per CreatePod (provider.go:35-60) — call
    fit_admit against the 100k-node C3 table; per-pod latency (call to return) p50 / p99 and pods/s,
    for the default coalescer (max_batch 1024, max_wait 2 ms: the Go call site's setting) and a
    zero-wait one (a batch is whatever is queued when the coalescer wakes)."""
    import threading

    from fitgpu import Admitter, Engine, synth
    nodes, jobs, parts = synth.make_config("c3")
    # what ONE virtual kubelet's engine holds (fit_admission.go: one partition per VK,
    # configurator.go:151-171): partition 0's ~6,250 nodes, its jobs, one partition
    sel = (nodes.part_mask & 1) != 0
    n1 = synth.Nodes(*(np.ascontiguousarray(x[sel]) for x in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free,
                                                               nodes.avail_min)),
                     np.ones(int(sel.sum()), np.uint32))
    js = jobs.part == 0
    j1 = synth.Jobs(*(np.ascontiguousarray(x[js]) for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)),
                    np.zeros(int(js.sum()), np.uint16), np.ascontiguousarray(jobs.nodes_k[js]))
    p1 = synth.Partitions(*(np.ascontiguousarray(x[:1]) for x in (parts.max_time_min, parts.max_cpus_per_node,
                                                                   parts.max_mem_per_node)))
    callers, per = 10, a.admit_pods
    out = {}
    for name, mb, mw, (pn, pj, pp) in (("max_wait_2ms", 1024, 2000, (nodes, jobs, parts)),
                                       ("max_wait_0", 1024, 0, (nodes, jobs, parts)),
                                       ("one_partition_max_wait_0", 1024, 0, (n1, j1, p1))):
        e = Engine(device=0)
        e.load_partitions(pp)
        adm = Admitter(e, max_batch=mb, max_wait_us=mw)
        adm.load_nodes(pn)
        for i in range(20):  # warmup (first launches)
            adm.admit(i, int(pj.cpu[i]), int(pj.mem[i]), int(pj.gpu[i]), int(pj.wall[i]), int(pj.part[i]))
        adm.load_nodes(pn)
        lat = [[] for _ in range(callers)]
        batches = set()
        bar = threading.Barrier(callers)

        def worker(w):
            bar.wait()
            for i in range(per):
                q = w * per + i
                t = time.perf_counter()
                r = adm.admit(q, int(pj.cpu[q]), int(pj.mem[q]), int(pj.gpu[q]), int(pj.wall[q]),
                              int(pj.part[q]))
                lat[w].append(time.perf_counter() - t)
                batches.add(r[1])

        th = [threading.Thread(target=worker, args=(w,)) for w in range(callers)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        el = time.perf_counter() - t0
        adm.close()
        e.close()
        us = np.sort(np.concatenate([np.array(x) for x in lat])) * 1e6
        out[name] = {"pods_per_s": round(callers * per / el, 1), "p50_us": round(float(np.percentile(us, 50)), 1),
                     "p99_us": round(float(np.percentile(us, 99)), 1), "max_us": round(float(us[-1]), 1),
                     "batches": len(batches), "pods_per_batch": round(callers * per / max(len(batches), 1), 2),
                     "nodes": pn.n, "partitions": pp.p}
    # the same load from native threads (tools/admit_load.cpp, built by the Makefile): the Go call
    # site's PodSyncWorkers are goroutines on OS threads, while the ten Python callers above share
    # one interpreter lock, which sets their arrival pattern (batches of 1.7-4.9 pods, box to box)
    native = {}
    exe = os.path.join(ROOT, "slurm-bridge-operator_amd", "fitgpu", "admit_load")
    if os.path.exists(exe):
        import subprocess
        import tempfile
        for name, mb, mw, (pn, pj, pp) in (("max_wait_2ms", 1024, 2000, (nodes, jobs, parts)),
                                           ("max_wait_0", 1024, 0, (nodes, jobs, parts)),
                                           ("one_partition_max_wait_0", 1024, 0, (n1, j1, p1))):
            with tempfile.TemporaryDirectory() as d:
                np.stack([pn.cpu_free, pn.mem_free, pn.gpu_free, pn.avail_min, pn.part_mask.view(np.int32)],
                         axis=1).astype(np.int32).tofile(os.path.join(d, "nodes.i32"))
                np.stack([pp.max_time_min, pp.max_cpus_per_node, pp.max_mem_per_node],
                         axis=1).astype(np.int32).tofile(os.path.join(d, "parts.i32"))
                m = callers * per + 20
                np.stack([pj.cpu[:m], pj.mem[:m], pj.gpu[:m], pj.wall[:m], pj.part[:m].astype(np.int32),
                          pj.nodes_k[:m].astype(np.int32)], axis=1).astype(np.int32).tofile(os.path.join(d, "jobs.i32"))
                r = subprocess.run([exe, d, str(callers), str(per), str(mb), str(mw)], capture_output=True,
                                   text=True, timeout=120)
            if r.returncode != 0:
                raise RuntimeError(f"admit_load {name}: {r.stderr.strip()}")
            native[name] = json.loads(r.stdout.strip().splitlines()[-1])
    # where one batch's time goes: fit_place of an admission-sized batch on the
    # same tables, host wall time of the call (ms_total) against the kernel time on the engine's
    # stream (ms_device: k_small, HIP events); the rest is the one packed H2D copy of the job
    # columns, the launch of k_small, the one D2H copy (placements + stats) and the synchronisation
    split = {}
    for tname, (tn, tj, tp) in (("c3_table", synth.make_config("c3")), ("one_partition", (n1, j1, p1))):
        e = Engine(device=0)
        e.load_partitions(tp)
        rows = {}
        for bs in (1, 4, 10, 64):
            tot, dev = [], []
            for rep in range(60):
                e.load_nodes(tn)
                sub = synth.Jobs(*(np.ascontiguousarray(x[rep * bs:(rep + 1) * bs])
                                   for x in (tj.cpu, tj.mem, tj.gpu, tj.wall, tj.part, tj.nodes_k)))
                _, st = e.place(sub)
                if rep >= 10:
                    tot.append(st["ms_total"])  # the library's own clock around fit_place
                    dev.append(st["ms_device"])
            rows[str(bs)] = {"engine": st["engine"], "call_us_p50": round(1e3 * float(np.median(tot)), 1),
                             "kernel_us_p50": round(1e3 * float(np.median(dev)), 1),
                             "host_copies_launch_sync_us_p50": round(1e3 * float(np.median(np.array(tot) - np.array(dev))), 1)}
        e.close()
        split[tname] = rows
    best = native.get("max_wait_0", out["max_wait_0"])
    line = {"metric": "CreatePod admission: pods/s and per-pod latency, 10 concurrent callers, 100k-node table",
            "value": best["pods_per_s"], "unit": "pods/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "int32", "data": "synthetic c3 node table and job stream (fitgpu/synth.py)",
            "config": {"workload": "admit", "nodes": nodes.n, "callers": callers, "pods": callers * per,
                       "partitions": parts.p},
            "callers": "native threads (tools/admit_load.cpp)" if native else "Python threads",
            "policies": native or out, "policies_python_callers": out, "batch_split": split,
            "reference": "one SubmitJob per CreatePod on 10 PodSyncWorkers, no capacity check "
                         "(provider.go:35-60, options/options.go:107)"}
    print(json.dumps(line), flush=True)


def cpu_baseline(workload, nodes, jobs, parts, tline, scale=1.0, kmax=1):
    """The CPU paths on this host (rank 0, N = 1), each on a bounded sample of the same workload
    (per-job cost is flat in J, so each sample's rate stands for the whole stream):
      naive-port                oracle/fitref*.c, every node per job, 1 thread (the SPEC as stated)
      component-aware           oracle/cpu_baseline.c, own component's nodes, vectorised, 1 thread
      same-algorithm            oracle/cpu_fast.c, the GPU's candidate-list + dirty-set rounds, 1 thread
      split-argmin              BASELINE.md:22: each job's argmin over CPU_THREADS threads, serial commit
      same-algorithm-multicore  the GPU's algorithm on CPU_THREADS threads
      multicore                 component-aware, components on CPU_THREADS threads
    backfill (c5): naive-port, component-aware (dense slot walk), run-length (the GPU's run lists,
    1 thread) and multicore (run lists, components on threads).  Multi-node jobs (c4, kmax 8):
    naive-port, component-aware and multicore (oracle/cpu_baseline.c cpu_place_k: the k smallest
    keys per job, components on threads).  The line's cpu_baseline object is the fastest variant."""
    from fitgpu import synth
    from oracle import pyoracle as po
    threads = max(1, min(CPU_THREADS, os.cpu_count() or 1))

    def prefix(m):
        m = max(1, min(int(m * scale), jobs.j))
        return m, synth.Jobs(*(x[:m] for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part, jobs.nodes_k)))

    # samples sized by an evaluation budget (each variant ~2-6 s on the box): a job costs one
    # evaluation per node it scans — every node (naive) or its component's (the others)
    ncomp = _components(nodes.part_mask)
    per_comp = nodes.n / max(ncomp, 1)
    par = min(threads, ncomp)
    if tline is not None:  # a timeline evaluation walks runs of slots: ~20x a plain fit eval
        m_naive, m_comp, m_rle = 1e8 / nodes.n, 1.5e7 / per_comp, 3e8 / per_comp
    else:
        m_naive, m_comp = 2e9 / nodes.n, 6e9 / per_comp
    m_mc = m_comp * par
    if tline is not None:
        runs = [("naive-port", 1, m_naive, lambda s: po.ref_place_tl(nodes, tline, s, parts)[2],
                 "oracle/fitref_tl.c ref_place_tl (SPEC §2b, dense timelines, every node per job)"),
                ("component-aware", 1, m_comp, lambda s: po.cpu_place_tl(nodes, tline, s, parts, 1)[2],
                 "oracle/cpu_baseline.c cpu_place_tl (own component's nodes only, dense slot walk)"),
                ("run-length", 1, m_rle, lambda s: po.cpu_place_tl(nodes, tline, s, parts, 1, rle=True)[2],
                 "oracle/cpu_fast.c cpu_place_tl_rle (run-length timelines, the GPU's layout; 1 thread)"),
                ("multicore", threads, m_rle * par,
                 lambda s: po.cpu_place_tl(nodes, tline, s, parts, threads, rle=True)[2],
                 f"oracle/cpu_fast.c cpu_place_tl_rle, {ncomp} components on {threads} threads")]
    elif kmax > 1:
        runs = [("naive-port", 1, m_naive, lambda s: po.ref_place(nodes, s, parts, kmax=kmax)[1],
                 "oracle/fitref.c ref_place (C restatement of the scalar sequential path, every node per job, "
                 "k smallest keys)"),
                ("component-aware", 1, m_comp / 2, lambda s: po.cpu_place_k(nodes, s, parts, kmax, 1)[1],
                 "oracle/cpu_baseline.c cpu_place_k (own component's nodes only, vectorised keys, top-k)"),
                ("multicore", threads, m_comp / 2 * par, lambda s: po.cpu_place_k(nodes, s, parts, kmax, threads)[1],
                 f"oracle/cpu_baseline.c cpu_place_k, {ncomp} components on {threads} threads")]
    else:
        # split-argmin: every job's scan split over the threads, one barrier per job
        m_split = 3e9 / per_comp * max(1, min(threads, 4))
        runs = [("naive-port", 1, m_naive, lambda s: po.ref_place(nodes, s, parts)[1],
                 "oracle/fitref.c ref_place (C restatement of the scalar sequential path, every node per job)"),
                ("component-aware", 1, m_comp, lambda s: po.cpu_place(nodes, s, parts, 1)[1],
                 "oracle/cpu_baseline.c cpu_place (own component's nodes only, vectorised scan)"),
                ("same-algorithm", 1, m_comp / 4, lambda s: po.cpu_place(nodes, s, parts, 1, "rounds")[1],
                 "oracle/cpu_fast.c cpu_place_rounds (the GPU's candidate-list + dirty-set rounds, 1 thread)"),
                ("split-argmin", threads, m_split, lambda s: po.cpu_place(nodes, s, parts, threads, "split")[1],
                 f"oracle/cpu_fast.c cpu_place_split (BASELINE.md:22: each job's argmin over {threads} threads, "
                 "serial commit)"),
                ("same-algorithm-multicore", threads, m_comp * min(threads, 4),
                 lambda s: po.cpu_place(nodes, s, parts, threads, "rounds")[1],
                 f"oracle/cpu_fast.c cpu_place_rounds on {threads} threads ("
                 + ("components on threads" if ncomp >= threads else "each window's scan over the threads") + ")"),
                ("multicore", threads, m_mc, lambda s: po.cpu_place(nodes, s, parts, threads)[1],
                 f"oracle/cpu_baseline.c cpu_place, {ncomp} components on {threads} threads")]
    variants = []
    for kind, cores, m, fn, what in runs:
        m, sub = prefix(m)
        t = time.perf_counter()
        st = fn(sub)
        ct = time.perf_counter() - t
        variants.append({"kind": kind, "value": round(m / ct, 1), "unit": "placements/s", "cores": cores,
                         "evals_per_s": round(st["evals"] / ct, 1),
                         "sample": f"first {m} jobs of {workload} vs all {nodes.n} nodes, {what}, {ct:.2f}s"})
    best = max(variants, key=lambda v: v["value"])
    return {"value": best["value"], "unit": "placements/s", "cores": best["cores"], "kind": "port",
            "variant": best["kind"], "sample": best["sample"], "host_cpu": _cpu_model(),
            "host": _host_info(threads), "variants": variants}


def _components(mask) -> int:
    """Partition components (partitions joined by nodes in several of them), as the engine forms them."""
    par = list(range(32))

    def find(x):
        while par[x] != x:
            par[x] = par[par[x]]
            x = par[x]
        return x
    used = set()
    for m in np.unique(mask):
        bits = [b for b in range(32) if (int(m) >> b) & 1]
        used.update(bits)
        for b in bits[1:]:
            ra, rb = find(bits[0]), find(b)
            par[max(ra, rb)] = min(ra, rb)
    return len({find(b) for b in used})


def _host_info(threads: int) -> dict:
    """BASELINE.md:23: nproc, the clock, the threads the multi-core variants used and why."""
    mhz = []
    try:
        mhz = [float(ln.split(":", 1)[1]) for ln in open("/proc/cpuinfo") if ln.startswith("cpu MHz")]
    except (OSError, ValueError):
        pass
    fmax = None
    try:
        fmax = int(open("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq").read()) / 1000.0
    except (OSError, ValueError):
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": affinity,
            "cpu_mhz_now_median": round(float(np.median(mhz)), 1) if mhz else None, "cpu_mhz_max": fmax,
            "threads_used": threads, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "why_threads": "the lease's CPU share for one GPU (OMP_NUM_THREADS on the GPU box); nproc and "
                           "the affinity mask count the whole machine, whose other cores belong to other "
                           "GPUs' jobs"}


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
