#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X: placements/sec (+ job×node fit evals/sec)
at 100k nodes × 1M jobs (config C3, 16 partitions) per GPU.

N > 1 (default --scaling weak, SURVEY §8 e / DESIGN §3.5): the placement path partitions into
independent partition components, so each rank places its own 100k × 1M cluster shard (a
disjoint slice of the generator streams) with no collective in the data path; `value` is the
aggregate placements/s of all ranks.  --scaling strong splits ONE 100k × 1M placement over the
ranks instead (--shard-mode components | nodes: RCCL allgather + u64 min-allreduce per round).

A "step" is one complete placement of the 1M-job stream against a freshly loaded 100k-node table:
fit_load_nodes_device (from HBM-resident columns) + fit_place_device.  Inputs are synthetic
(splitmix64 generator, fitgpu/synth.py) and already resident in HBM when the timed region starts.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` is live: per-launch kernel time from the engine's HIP
events (on the engine's stream), algorithmic work from DESIGN.md §5.  `cpu_baseline` times the
oracle (C restatement of the scalar path, 1 thread) on a bounded prefix of the same workload.
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c5"],
                    help="c3: BASELINE headline (100k x 1M); c5: the same with a 1,024-slot backfill horizon")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="jobs in the CPU baseline sample (default 40,000; c5: 3,000)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--rehearse", action="store_true",
                    help="test only: every rank on cuda:0 with gloo (rehearse N>1 on a 1-GPU box)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC summary (tools/gpu_pmc.sh + tools/pmc_json.py) with HBM bytes/launch")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N>1: weak = every rank places its own 100k x 1M cluster shard (independent "
                         "partition components, no data-path collective); strong = one 100k x 1M "
                         "placement split over the ranks (--shard-mode)")
    ap.add_argument("--shard-mode", default="auto", choices=["auto", "nodes", "components"],
                    help="strong scaling split: auto = partition components when there are >= N of them")
    return ap.parse_args()


def main():
    a = parse_args()
    import torch
    import torch.distributed as dist

    from fitgpu import (FIT_SHARD_AUTO, FIT_SHARD_COMPONENTS, FIT_SHARD_NODES, Engine, nccl_unique_id,
                        synth)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    if a.rehearse:
        local = 0
        if a.scaling != "weak":
            raise SystemExit("--rehearse supports --scaling weak only")
    torch.cuda.set_device(local)
    weak = world > 1 and a.scaling == "weak"
    nid = None
    if world > 1:
        if a.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if not weak:
            obj = [nccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            nid = obj[0]
    shard = rank if weak else 0  # weak: this rank's own cluster shard (disjoint generator slice)

    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    tl = a.workload == "c5"
    if tl:
        nodes, tline, jobs, parts = synth.make_c5(shard=shard)
    else:
        nodes, jobs, parts = synth.make_config(a.workload, shard=shard)
    dev = torch.device("cuda", local)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    d_nodes = [T(nodes.cpu_free), T(nodes.mem_free), T(nodes.gpu_free), T(nodes.avail_min),
               T(nodes.part_mask.view(np.int32))]
    d_jobs = [T(jobs.cpu), T(jobs.mem), T(jobs.gpu), T(jobs.wall), T(jobs.part.view(np.int16)),
              T(jobs.nodes_k.view(np.int16))]
    d_out = torch.empty(jobs.j, dtype=torch.int32, device=dev)
    if tl:
        d_rel = [T(x) for x in (tline.off, tline.slot, tline.cpu, tline.mem, tline.gpu)]
        d_start = torch.empty(jobs.j, dtype=torch.int32, device=dev)

    mode = {"auto": FIT_SHARD_AUTO, "nodes": FIT_SHARD_NODES, "components": FIT_SHARD_COMPONENTS}[a.shard_mode]
    if weak:
        eng = Engine(device=local)  # independent shard: no collective in the data path
    else:
        eng = Engine(device=local, rank=rank, world=world, nccl_id=nid, shard_mode=mode)
    eng.load_partitions(parts)

    def step():
        eng.load_nodes_device(*d_nodes)
        if tl:
            eng.load_timeline_device(tline.slots, tline.slot_min, *d_rel)
            return eng.place_tl_device(*d_jobs[:5], d_out, d_start)
        return eng.place_device(*d_jobs, d_out, kmax=1)

    for _ in range(a.warmup):
        step()
    stats = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        stats.append(step())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    cdev = torch.device("cpu") if a.rehearse else dev  # gloo reduces CPU tensors
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # output sanity every run: the engine's counts are internally consistent
    s0 = stats[-1]
    assert s0["placed"] + s0["unplaced"] + s0["rejected"] == jobs.j

    value = jobs.j * a.steps / el * (world if weak else 1)
    agg = {k: sum(s[k] for s in stats) for k in ("rounds", "evals", "useful_evals", "ms_scan", "ms_commit",
                                                  "ms_exchange", "ms_device", "placed", "unplaced")}
    evals_local = agg["evals"]
    if world > 1:  # performed / useful evaluations summed over ranks
        t = torch.tensor([float(agg["evals"]), float(agg["useful_evals"])], dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        agg["evals"], agg["useful_evals"] = int(t[0].item()), int(t[1].item())
    used_mode = {0: "1 GPU", 1: f"node-sharded x{world} (RCCL allgather + u64 min-allreduce per round)",
                 2: f"partition-component-sharded x{world} (one RCCL merge)"}[stats[-1]["shard_mode"]]
    if weak:
        used_mode = f"{world} independent cluster shards (one per GPU, no data-path collective)"
    kernels = kernel_table(agg, stats, a.steps, world, evals_local,
                           ("k_scan_tl", "k_commit_tl") if tl else ("k_scan", "k_commit"),
                           "k_engine_tl" if tl else "k_engine")
    dominant = max(kernels, key=lambda k: kernels[k]["ms_per_launch"] * kernels[k]["launches"])
    k = kernels[dominant]
    traffic = None
    if a.pmc_json and os.path.exists(a.pmc_json):
        traffic = json.load(open(a.pmc_json)).get(dominant, {}).get("hbm_bytes_per_launch")
    roofline = {"kernel": dominant, "bound": k["bound"], "achieved": k["achieved"], "peak": k["peak"],
                "unit": k["unit"], "frac": k["frac"], "traffic": traffic}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        from oracle import pyoracle as po
        sample = min(a.cpu_sample or (3000 if tl else 40000), jobs.j)
        sub = synth.Jobs(*(x[:sample] for x in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall, jobs.part,
                                                  jobs.nodes_k)))
        t = time.perf_counter()
        if tl:
            _, _, cst, _ = po.ref_place_tl(nodes, tline, sub, parts)
            what = "oracle/fitref_tl.c ref_place_tl (C restatement of SPEC §2b, dense timelines)"
        else:
            _, cst, _ = po.ref_place(nodes, sub, parts)
            what = "oracle/fitref.c ref_place (C restatement of the scalar sequential path)"
        ct = time.perf_counter() - t
        cpu = {"value": round(sample / ct, 2), "unit": "placements/s", "cores": 1, "kind": "port",
               "evals_per_s": round(cst["evals"] / ct, 1),
               "sample": f"first {sample} jobs of {a.workload} vs all {nodes.n} nodes, {what}, 1 thread, "
                         f"{ct:.1f}s",
               "host_cpu": _cpu_model()}

    line = {
        "metric": base["metric"], "value": round(value, 1), "unit": "placements/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak" if (weak or world == 1) else "strong", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (splitmix64 generator, fitgpu/synth.py; DESIGN.md §5)",
        "config": {"workload": a.workload, "nodes": nodes.n * (world if weak else 1),
                   "jobs": jobs.j * (world if weak else 1), "partitions": parts.p * (world if weak else 1),
                   "per_gpu": {"nodes": nodes.n, "jobs": jobs.j} if weak else None,
                   **({"slots": tline.slots, "slot_min": tline.slot_min} if tl else {}),
                   "parallelism": used_mode, "components": stats[-1]["components"]},
        "fit_evals_per_s": {"useful": round(agg["useful_evals"] / el, 1), "performed": round(agg["evals"] / el, 1)},
        "rounds_per_step": agg["rounds"] / a.steps,
        "round_stops_per_step": {"rescan": stats[-1]["stops_rescan"], "dirty_full": stats[-1]["stops_dirty"]},
        "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
    }
    if cpu:
        line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


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
