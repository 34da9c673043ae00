"""ctypes front-end of liboracle.so (TEST INFRASTRUCTURE ONLY — the checker, never the product).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Builds the library on
first use when a compiler is present (the GPU box gets the prebuilt .so with the snapshot).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        srcs = [os.path.join(_HERE, f) for f in ("fitref.c", "fitref_tl.c", "round_model.c", "cpu_baseline.c",
                                                 "cpu_fast.c", "fitref.h", "Makefile")]
        if not os.path.exists(path) or any(os.path.getmtime(s) > os.path.getmtime(path) for s in srcs):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _LIB = C.CDLL(path)
        _LIB.ref_rnd.restype = C.c_uint64
        _LIB.ref_rnd.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64]
        _LIB.ref_key.restype = C.c_uint64
        _LIB.ref_parse_array_len.restype = C.c_int64
        _LIB.ref_key_tl.restype = C.c_uint64
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class ModelParams(C.Structure):
    _fields_ = [("slice", C.c_int32), ("ks", C.c_int32), ("km", C.c_int32), ("ucap", C.c_int32),
                ("wmin", C.c_int32), ("wmax", C.c_int32), ("shards", C.c_int32)]


def _prep(nodes, jobs, parts):
    cf = np.ascontiguousarray(nodes.cpu_free, np.int32).copy()
    mf = np.ascontiguousarray(nodes.mem_free, np.int32).copy()
    gf = np.ascontiguousarray(nodes.gpu_free, np.int32).copy()
    av = np.ascontiguousarray(nodes.avail_min, np.int32)
    mk = np.ascontiguousarray(nodes.part_mask, np.uint32)
    pt = [np.ascontiguousarray(a, np.int32) for a in (parts.max_time_min, parts.max_cpus_per_node,
                                                      parts.max_mem_per_node)]
    jb = [np.ascontiguousarray(a, np.int32) for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)]
    jp = np.ascontiguousarray(jobs.part, np.uint16)
    jk = np.ascontiguousarray(jobs.nodes_k, np.uint16)
    return cf, mf, gf, av, mk, pt, jb, jp, jk


def ref_place(nodes, jobs, parts, kmax: int = 1):
    """SPEC sequential best fit. Returns (out[J, kmax] int32, stats dict, final (cpu, mem, gpu))."""
    cf, mf, gf, av, mk, pt, jb, jp, jk = _prep(nodes, jobs, parts)
    j = jobs.j
    out = np.empty((j, kmax), np.int32)
    st = np.zeros(4, np.int64)
    I32, U32, U16 = C.c_int32, C.c_uint32, C.c_uint16
    rc = lib().ref_place(
        I32(nodes.n), _p(cf, I32), _p(mf, I32), _p(gf, I32), _p(av, I32), _p(mk, U32),
        I32(parts.p), _p(pt[0], I32), _p(pt[1], I32), _p(pt[2], I32),
        I32(j), _p(jb[0], I32), _p(jb[1], I32), _p(jb[2], I32), _p(jb[3], I32), _p(jp, U16),
        _p(jk, U16), I32(kmax), _p(out, I32), _p(st, C.c_int64))
    if rc != 0:
        raise ValueError("ref_place: invalid input")
    stats = dict(placed=int(st[0]), unplaced=int(st[1]), rejected=int(st[2]), evals=int(st[3]))
    return out, stats, (cf, mf, gf)


def model_place(nodes, jobs, parts, slice=2048, ks=8, km=32, ucap=256, wmin=256, wmax=65536, shards=1):
    """CPU model of the GPU round algorithm (k = 1 jobs)."""
    cf, mf, gf, av, mk, pt, jb, jp, _ = _prep(nodes, jobs, parts)
    j = jobs.j
    out = np.empty(j, np.int32)
    st = np.zeros(8, np.int64)
    prm = ModelParams(slice, ks, km, ucap, wmin, wmax, shards)
    I32, U32, U16 = C.c_int32, C.c_uint32, C.c_uint16
    rc = lib().model_place(
        I32(nodes.n), _p(cf, I32), _p(mf, I32), _p(gf, I32), _p(av, I32), _p(mk, U32),
        I32(parts.p), _p(pt[0], I32), _p(pt[1], I32), _p(pt[2], I32),
        I32(j), _p(jb[0], I32), _p(jb[1], I32), _p(jb[2], I32), _p(jb[3], I32), _p(jp, U16),
        C.byref(prm), _p(out, I32), _p(st, C.c_int64))
    if rc != 0:
        raise ValueError("model_place: invalid parameters")
    keys = ["rounds", "scan_evals", "dirty_evals", "stops_rescan", "stops_ucap", "commits",
            "max_window", "placed"]
    return out, {k: int(v) for k, v in zip(keys, st)}, (cf, mf, gf)


# ---- SPEC §2b time-windowed backfill (oracle/fitref_tl.c) ----------------------------------------
def ref_build_timeline(nodes, tline):
    """Dense [n, H, 3] int32 timeline (cpu, mem, gpu) of DESIGN.md §2b."""
    n, H = nodes.n, tline.slots
    tl = np.empty((n, H, 3), np.int32)
    I32 = C.c_int32
    cols = [np.ascontiguousarray(a, np.int32) for a in (nodes.cpu_free, nodes.mem_free, nodes.gpu_free,
                                                        nodes.avail_min)]
    rel = [np.ascontiguousarray(a, np.int32) for a in (tline.off, tline.slot, tline.cpu, tline.mem, tline.gpu)]
    rc = lib().ref_build_timeline(I32(n), I32(H), I32(tline.slot_min), *(_p(a, I32) for a in cols),
                                  *(_p(a, I32) for a in rel), _p(tl, I32))
    if rc != 0:
        raise ValueError("ref_build_timeline: invalid input")
    return tl


def ref_place_tl(nodes, tline, jobs, parts, tl=None):
    """SPEC §2b sequential backfill.  Returns (node[J], start[J], stats dict, final dense timeline)."""
    tl = ref_build_timeline(nodes, tline) if tl is None else np.ascontiguousarray(tl, np.int32).copy()
    I32, U32, U16 = C.c_int32, C.c_uint32, C.c_uint16
    mk = np.ascontiguousarray(nodes.part_mask, np.uint32)
    pt = [np.ascontiguousarray(a, np.int32) for a in (parts.max_time_min, parts.max_cpus_per_node,
                                                      parts.max_mem_per_node)]
    jb = [np.ascontiguousarray(a, np.int32) for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)]
    jp = np.ascontiguousarray(jobs.part, np.uint16)
    node = np.empty(jobs.j, np.int32)
    start = np.empty(jobs.j, np.int32)
    st = np.zeros(4, np.int64)
    rc = lib().ref_place_tl(I32(nodes.n), I32(tline.slots), I32(tline.slot_min), _p(tl, I32), _p(mk, U32),
                            I32(parts.p), *(_p(a, I32) for a in pt), I32(jobs.j), *(_p(a, I32) for a in jb),
                            _p(jp, U16), _p(node, I32), _p(start, I32), _p(st, C.c_int64))
    if rc != 0:
        raise ValueError("ref_place_tl: invalid input")
    stats = dict(placed=int(st[0]), unplaced=int(st[1]), rejected=int(st[2]), evals=int(st[3]))
    return node, start, stats, tl


# ---- fair CPU baselines (oracle/cpu_baseline.c; bench.py cpu_baseline leg) -----------------------
def cpu_place(nodes, jobs, parts, threads: int = 1, variant: str = "component"):
    """Sequential best fit (k = 1) on the CPU, same result as ref_place.  variant: "component"
    (oracle/cpu_baseline.c: components on `threads` threads), "split" (every job's argmin split over
    the threads, BASELINE.md:22) or "rounds" (the GPU's candidate-list + dirty-set algorithm,
    oracle/cpu_fast.c).  Returns (out[J] int32, stats dict, final (cpu, mem, gpu))."""
    cf, mf, gf, av, mk, pt, jb, jp, _ = _prep(nodes, jobs, parts)
    out = np.empty(jobs.j, np.int32)
    st = np.zeros(4, np.int64)
    I32, U32, U16 = C.c_int32, C.c_uint32, C.c_uint16
    fn = {"component": lib().cpu_place, "split": lib().cpu_place_split, "rounds": lib().cpu_place_rounds}[variant]
    rc = fn(
        I32(nodes.n), _p(cf, I32), _p(mf, I32), _p(gf, I32), _p(av, I32), _p(mk, U32),
        I32(parts.p), _p(pt[0], I32), _p(pt[1], I32), _p(pt[2], I32),
        I32(jobs.j), _p(jb[0], I32), _p(jb[1], I32), _p(jb[2], I32), _p(jb[3], I32), _p(jp, U16),
        _p(out, I32), _p(st, C.c_int64), I32(threads))
    if rc != 0:
        raise ValueError("cpu_place: invalid input")
    return out, dict(placed=int(st[0]), unplaced=int(st[1]), rejected=int(st[2]), evals=int(st[3])), (cf, mf, gf)


def cpu_place_k(nodes, jobs, parts, kmax: int, threads: int = 1):
    """Component-aware best fit with multi-node jobs (config C4; oracle/cpu_baseline.c cpu_place_k,
    components on `threads` threads): same result as ref_place(..., kmax).  Returns (out[J, kmax],
    stats dict, final (cpu, mem, gpu))."""
    cf, mf, gf, av, mk, pt, jb, jp, jk = _prep(nodes, jobs, parts)
    out = np.empty((jobs.j, kmax), np.int32)
    st = np.zeros(4, np.int64)
    I32, U32, U16 = C.c_int32, C.c_uint32, C.c_uint16
    rc = lib().cpu_place_k(
        I32(nodes.n), _p(cf, I32), _p(mf, I32), _p(gf, I32), _p(av, I32), _p(mk, U32),
        I32(parts.p), _p(pt[0], I32), _p(pt[1], I32), _p(pt[2], I32),
        I32(jobs.j), _p(jb[0], I32), _p(jb[1], I32), _p(jb[2], I32), _p(jb[3], I32), _p(jp, U16),
        _p(jk, U16), I32(kmax), _p(out, I32), _p(st, C.c_int64), I32(threads))
    if rc != 0:
        raise ValueError("cpu_place_k: invalid input")
    return out, dict(placed=int(st[0]), unplaced=int(st[1]), rejected=int(st[2]), evals=int(st[3])), (cf, mf, gf)


def cpu_place_tl(nodes, tline, jobs, parts, threads: int = 1, tl=None, rle: bool = False):
    """Component-aware SPEC §2b backfill on `threads` threads (dense slot walk, or run-length
    timelines with rle=True: oracle/cpu_fast.c).  Same result as ref_place_tl."""
    tl = ref_build_timeline(nodes, tline) if tl is None else np.ascontiguousarray(tl, np.int32).copy()
    I32, U32, U16 = C.c_int32, C.c_uint32, C.c_uint16
    mk = np.ascontiguousarray(nodes.part_mask, np.uint32)
    pt = [np.ascontiguousarray(a, np.int32) for a in (parts.max_time_min, parts.max_cpus_per_node,
                                                      parts.max_mem_per_node)]
    jb = [np.ascontiguousarray(a, np.int32) for a in (jobs.cpu, jobs.mem, jobs.gpu, jobs.wall)]
    jp = np.ascontiguousarray(jobs.part, np.uint16)
    node = np.empty(jobs.j, np.int32)
    start = np.empty(jobs.j, np.int32)
    st = np.zeros(4, np.int64)
    rc = (lib().cpu_place_tl_rle if rle else lib().cpu_place_tl)(I32(nodes.n), I32(tline.slots), I32(tline.slot_min), _p(tl, I32), _p(mk, U32),
                            I32(parts.p), *(_p(a, I32) for a in pt), I32(jobs.j), *(_p(a, I32) for a in jb),
                            _p(jp, U16), _p(node, I32), _p(start, I32), _p(st, C.c_int64), I32(threads))
    if rc != 0:
        raise ValueError("cpu_place_tl: invalid input")
    return node, start, dict(placed=int(st[0]), unplaced=int(st[1]), rejected=int(st[2]), evals=int(st[3])), tl
