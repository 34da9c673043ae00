"""Driver of tools/spec_model.c (diagnostic): the jobs-per-step distribution of a
multi-job decider step under the speculative-prefix rule, on component 0 of a BASELINE config.

    gcc -O2 -shared -fPIC -o tools/libspec_model.so tools/spec_model.c
    python tools/spec_model.py c3 8"""
import os, sys, ctypes as C, numpy as np, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'slurm-bridge-operator_amd')]
from fitgpu import synth
L = C.CDLL(os.path.join(ROOT, 'tools', 'libspec_model.so')); L.spec_steps.restype = C.c_int64
name = sys.argv[1]; mstep = int(sys.argv[2]); nn = int(sys.argv[3]) if len(sys.argv) > 3 else None; jj = int(sys.argv[4]) if len(sys.argv) > 4 else None
nodes, jobs, parts = synth.make_config(name, nn, jj)
p0 = 0
sel = (nodes.part_mask & 1) != 0
idn = np.flatnonzero(sel).astype(np.int32)
cf, mf, gf = (np.ascontiguousarray(a[sel], np.int32) for a in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free))
av = np.ascontiguousarray(nodes.avail_min[sel], np.int32); mk = np.ascontiguousarray(nodes.part_mask[sel], np.uint32)
mt, mc, mm = parts.max_time_min[0], parts.max_cpus_per_node[0], parts.max_mem_per_node[0]
js = (jobs.part == 0) & ~((mt >= 0) & (jobs.wall > mt)) & ~((mc >= 0) & (jobs.cpu > mc)) & ~((mm >= 0) & (jobs.mem > mm))
jc, jm, jg, jw = (np.ascontiguousarray(a[js], np.int32) for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall))
jp = np.ascontiguousarray(jobs.part[js], np.uint16)
P = lambda a, t: a.ctypes.data_as(C.POINTER(t))
hist = np.zeros(65, np.int64)
cause = np.zeros(2, np.int64)
t0 = time.time()
st = L.spec_steps(len(idn), P(cf, C.c_int32), P(mf, C.c_int32), P(gf, C.c_int32), P(av, C.c_int32), P(mk, C.c_uint32), P(idn, C.c_int32),
                  len(jc), P(jc, C.c_int32), P(jm, C.c_int32), P(jg, C.c_int32), P(jw, C.c_int32), P(jp, C.c_uint16), mstep, P(hist, C.c_int64), 1, P(cause, C.c_int64))
tot = (hist * np.arange(65)).sum()
print(f"{name} partition 0: {len(idn)} nodes, {len(jc)} jobs, m={mstep}: {st} steps for {tot} live jobs -> {tot/st:.2f} jobs/step; hist", {i: int(h) for i, h in enumerate(hist) if h}, f"{time.time()-t0:.1f}s", f"| steps cut by: same node {int(cause[0])}, a taken node now tighter {int(cause[1])}")
