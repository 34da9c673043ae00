"""Hand-built SPEC §2b (time-windowed backfill) case shared by the CPU oracle test and the GPU test.

Horizon 8 slots × 10 min.  Expected placements worked out by hand in the comments:
  j0 (2 cpu, 1024 MiB, 30 min = 3 slots): n0 fits at 0 (score cpu 2, mem 3); n1 fits at 0 with the
     tighter score (cpu 0, mem 1) → n1 @ 0.
  j1 (4 cpu, 4096, 60 min = 6 slots): n0 at 0 (slots 0-5 hold >= 4 cpus); n1 has 5 usable slots → n0 @ 0.
  j2 (1 cpu, 512, 1 slot): n0 is full on slots 0-2 (score at 3: cpu 3, mem 3); n1 is full on 0-2
     (score at 3: cpu 1, mem 1) → n1 @ 3.
  j3 (partition 1): only n2 → n2 @ 0.
  j4 (16 cpus): nothing that large → unplaced.   j5 (100 min = 10 slots > 8): unplaced.
  j6 (partition 5 of 2): rejected.
"""
import numpy as np

from fitgpu import synth

INT32_MAX = 2**31 - 1


def hand_case():
    nodes = synth.Nodes(
        cpu_free=np.array([4, 2, 8], np.int32), mem_free=np.array([4096, 2048, 8192], np.int32),
        gpu_free=np.array([0, 0, 2], np.int32), avail_min=np.array([INT32_MAX, 50, INT32_MAX], np.int32),
        part_mask=np.array([1, 1, 2], np.uint32))
    tline = synth.Timeline(slots=8, slot_min=10, off=np.array([0, 1, 1, 1], np.int32),
                           slot=np.array([3], np.int32), cpu=np.array([4], np.int32),
                           mem=np.array([4096], np.int32), gpu=np.array([0], np.int32))
    jobs = synth.Jobs(cpu=np.array([2, 4, 1, 1, 16, 1, 1], np.int32),
                      mem=np.array([1024, 4096, 512, 512, 1, 1, 1], np.int32),
                      gpu=np.zeros(7, np.int32), wall=np.array([30, 60, 10, 20, 10, 100, 10], np.int32),
                      part=np.array([0, 0, 0, 1, 0, 0, 5], np.uint16), nodes_k=np.ones(7, np.uint16))
    parts = synth.Partitions(np.full(2, -1, np.int32), np.full(2, -1, np.int32), np.full(2, -1, np.int32))
    return nodes, tline, jobs, parts


EXPECT_NODE = np.array([1, 0, 1, 2, -1, -1, -2], np.int32)
EXPECT_START = np.array([0, 0, 3, 0, -1, -1, -1], np.int32)
