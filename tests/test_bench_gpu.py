"""bench.py keeps the driver's contract: one JSON line with the required keys, the roofline and
CPU-baseline objects, for the C3 headline, the C5 and c3o workloads; N>1 rehearsed with two ranks on
one GPU (gloo for the timing collectives; the strong split exchanges through the host)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.auto_engine]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def run(args, env=None, timeout=240):
    r = subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env={**os.environ, **(env or {})})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


PLAIN = {"naive-port", "component-aware", "same-algorithm", "split-argmin", "same-algorithm-multicore", "multicore"}
BACKFILL = {"naive-port", "component-aware", "run-length", "multicore"}


@pytest.mark.parametrize("workload", ["c3", "c5", "c3o"])
def test_bench_line(workload):
    d = run(["bench.py", "--workload", workload, "--steps", "1", "--warmup", "1", "--cpu-scale", "0.01",
             "--no-live-pmc"])
    assert KEYS <= set(d) and d["n_gpus"] == 1 and d["value"] > 0 and d["kernel_path_value"] > 0
    assert set(d["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac", "traffic"}
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and {v["kind"] for v in cb["variants"]} == (BACKFILL if workload == "c5" else PLAIN)
    assert d["config"]["workload"] == workload and d["config"]["jobs"] == 1_000_000
    assert d["placed_plus_unplaced_per_s"] <= d["value"]
    # BASELINE.md:26: the median of 3 timed runs
    assert d["timing"]["repeats"] == 3 and sorted(d["timing"]["value_runs"])[1] == d["value"]
    if workload != "c5":  # north_star's node-sharded layout priced on one GPU
        assert d["node_sharding_1gpu"]["ms_per_step"] > 0


def test_bench_live_traffic():
    """roofline.traffic measured in the run: two rocprofv3 --pmc passes over a child bench run."""
    d = run(["bench.py", "--workload", "c2", "--steps", "2", "--warmup", "1", "--no-cpu", "--repeats", "1",
             "--no-shard-price"], timeout=600)
    assert d["roofline"]["traffic"] > 0 and d["roofline"]["traffic_source"].startswith("live")


def test_bench_admission_latency():
    d = run(["bench.py", "--workload", "admit", "--admit-pods", "20"])
    assert d["config"]["pods"] == 200 and d["value"] > 0
    for pol in d["policies"].values():
        assert 0 < pol["p50_us"] <= pol["p99_us"] <= pol["max_us"] and pol["batches"] >= 1


def test_bench_two_rank_rehearsal():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    d = run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
             "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--rehearse", "--scaling", "weak",
             "--repeats", "1"])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["jobs"] == 2_000_000 and d["config"]["per_gpu"]["jobs"] == 1_000_000


@pytest.mark.parametrize("shard_mode,workload", [("auto", "c3"), ("nodes", "c2")])
def test_bench_two_rank_strong_rehearsal(shard_mode, workload):
    """N > 1 default (strong: ONE C3 placement split over the ranks) rehearsed with two ranks on
    one GPU (host exchange over gloo instead of RCCL), plus the extra `weak_scaling` leg."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    d = run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
             "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--rehearse",
             "--scaling", "strong", "--shard-mode", shard_mode, "--workload", workload, "--no-device-path",
             "--repeats", "1"])
    jobs = 1_000_000 if workload == "c3" else 65_536
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["jobs"] == jobs
    assert ("component" in d["config"]["parallelism"]) == (shard_mode == "auto")
    w = d["weak_scaling"]
    assert w["scaling"] == "weak" and w["value"] > 0 and w["per_gpu"]["jobs"] == jobs



@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_four_rank_rehearsal(scaling):
    """the driver's first multi-GPU run can be checked against a number — four
    ranks rehearsed on one GPU (gloo timing collectives; the strong split exchanges through the
    host).  Weak (the default): four 100k x 1M shards, aggregate; strong: one C3 placement over
    four ranks (four components each), plus the weak leg.  Predictions: DESIGN.md §3.5."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    args = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
            "--master-port", str(port), "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "1", "--rehearse",
            "--repeats", "1", "--no-device-path", "--scaling", scaling]
    if scaling == "strong":
        args.append("--no-weak-extra")
    d = run(args, timeout=400)
    assert d["n_gpus"] == 4 and d["scaling"] == scaling and d["value"] > 0
    assert d["config"]["jobs"] == (4_000_000 if scaling == "weak" else 1_000_000)
    if scaling == "strong":
        assert "component" in d["config"]["parallelism"]
