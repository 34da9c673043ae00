"""Worker for tests/test_multirank*.py: one rank of a multi-rank placement (launched as a child)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int)
    ap.add_argument("--world", type=int)
    ap.add_argument("--port", type=int)
    ap.add_argument("--mode", type=int)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--nodes", type=int, default=20000)
    ap.add_argument("--jobs", type=int, default=100000)
    ap.add_argument("--out")
    ap.add_argument("--kmax", type=int, default=1)
    ap.add_argument("--auto-engine", action="store_true", help="the library's own engine choice")
    a = ap.parse_args()
    if a.auto_engine:
        os.environ.pop("FIT_ENGINE", None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    from fitgpu import Engine, TorchHostExchange, synth
    x = TorchHostExchange()
    if a.config == "c5":  # backfill: node-sharded rounds over replicated run lists
        nodes, tline, jobs, parts = synth.make_c5(a.nodes, a.jobs)
        with Engine(device=0, rank=a.rank, world=a.world, exchange=x, shard_mode=a.mode) as e:
            e.load_nodes(nodes)
            e.load_partitions(parts)
            e.load_timeline(tline)
            node, start, st = e.place_tl(jobs)
            fin = e.read_timeline()
        np.savez(a.out, node=node, start=start, fin=fin,
                 stats=np.array([st["placed"], st["unplaced"], st["rejected"], st["shard_mode"]]))
        dist.barrier()
        dist.destroy_process_group()
        return
    nodes, jobs, parts = synth.make_config(a.config, a.nodes, a.jobs)
    with Engine(device=0, rank=a.rank, world=a.world, exchange=x, shard_mode=a.mode) as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        out, st = e.place(jobs, kmax=a.kmax)
        fin = e.read_nodes()
    np.savez(a.out, out=out, cpu=fin[0], mem=fin[1], gpu=fin[2],
             stats=np.array([st["placed"], st["unplaced"], st["rejected"], st["shard_mode"], st["engine"]]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
