"""Full-size golden digests for BASELINE configs C4 and C5 (run offline in the dev container), and
for their array-expanded streams c3a / c4a / c5a (synth.make_array_config).

C5 (100k nodes x 1M jobs, 1,024-slot horizon) takes the oracle (oracle/fitref_tl.c:ref_place_tl,
dense timelines, one thread) about 1.5 h; C4 (100k GPU-heavy nodes x 1M multi-node jobs, kmax 8)
runs oracle/fitref.c:ref_place.  The digests land in tests/golden/placements_big.json and are
checked by tests/test_golden_big_gpu.py.

    python tools/make_golden_big.py c4|c5|c3a|c4a|c5a
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slurm-bridge-operator_amd")]
import numpy as np  # noqa: E402

PATH = os.path.join(ROOT, "tests", "golden", "placements_big.json")


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def save(key, rec):
    # read-modify-write: the two configs may run concurrently in separate processes
    doc = json.load(open(PATH)) if os.path.exists(PATH) else {}
    doc[key] = rec
    tmp = PATH + f".tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(doc, f, indent=1)
    os.replace(tmp, PATH)
    print(key, rec, flush=True)


def c5(name="c5"):
    from fitgpu import synth
    from oracle import pyoracle as po
    nodes, tline, jobs, parts = synth.make_c5() if name == "c5" else synth.make_array_config(name)
    t = time.time()
    node, start, st, tl = po.ref_place_tl(nodes, tline, jobs, parts)
    save(f"{name}:{nodes.n}x{jobs.j}", {
        "node_sha256": sha(node), "start_sha256": sha(start),
        "final_cpu_sha256": sha(tl[..., 0]), "final_mem_sha256": sha(tl[..., 1]),
        "final_gpu_sha256": sha(tl[..., 2]), **st, "oracle_seconds": round(time.time() - t, 1)})


def c4(name="c4"):
    from fitgpu import synth
    from oracle import pyoracle as po
    nodes, jobs, parts = synth.make_config(name) if name in ("c3", "c4") else synth.make_array_config(name)
    kmax = 8 if name.startswith("c4") else 1
    t = time.time()
    out, st, fin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    save(f"{name}:{nodes.n}x{jobs.j}", {
        "kmax": kmax, "placements_sha256": sha(out), "final_cpu_sha256": sha(fin[0]),
        "final_mem_sha256": sha(fin[1]), "final_gpu_sha256": sha(fin[2]), **st,
        "oracle_seconds": round(time.time() - t, 1)})


if __name__ == "__main__":
    n = sys.argv[1]
    (c5 if n.startswith("c5") else c4)(n)
