"""Batched admission (include/fitgpu.h fit_admitter): concurrent
CreatePod-style callers (the virtual kubelet's 10 PodSyncWorkers, options/options.go:107) block in
fit_admit, a coalescer places each batch with one fit_place in (priority, arrival) order.

Parity: the placements every caller received, taken in the order the admitter placed them (batch,
then position in the batch), equal the oracle's sequential best fit of the same jobs in that
order from the same node table — bit-exact, including the final free columns per partition."""
import threading

import numpy as np
import pytest

from fitgpu import FIT_UNPLACED, Admitter, Engine, FitError, synth
from fitgpu import _lib
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def _run_workers(adm, reqs, workers=10):
    """reqs: list of (priority, cpu, mem, gpu, wall, part, k); returns results by request index."""
    out = [None] * len(reqs)
    start = threading.Barrier(workers)

    def worker(w):
        start.wait()
        for i in range(w, len(reqs), workers):
            out[i] = adm.admit(*reqs[i])

    th = [threading.Thread(target=worker, args=(w,)) for w in range(workers)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert all(r is not None for r in out)
    return out


def _oracle_in_admitted_order(nodes, parts, reqs, res, kmax):
    order = sorted(range(len(reqs)), key=lambda i: (res[i][1], res[i][3]))
    q = [reqs[i] for i in order]
    jobs = synth.Jobs(np.array([r[1] for r in q], np.int32), np.array([r[2] for r in q], np.int32),
                      np.array([r[3] for r in q], np.int32), np.array([r[4] for r in q], np.int32),
                      np.array([r[5] for r in q], np.uint16), np.array([r[6] for r in q], np.uint16))
    ref, _, fin = po.ref_place(nodes, jobs, parts, kmax=kmax)
    return order, ref, fin


@pytest.mark.parametrize("max_batch,max_wait_us", [(1024, 20000), (7, 5000), (1, 0)])
def test_concurrent_admission_matches_sequential_oracle(max_batch, max_wait_us):
    nodes, jobs, parts = synth.make_config("c4", 256, 400)
    reqs = [(int(p), int(jobs.cpu[i]), int(jobs.mem[i]), int(jobs.gpu[i]), int(jobs.wall[i]),
             int(jobs.part[i]), int(jobs.nodes_k[i]))
            for i, p in enumerate(np.random.default_rng(7).integers(0, 1 << 40, jobs.j))]
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        adm = Admitter(e, max_batch=max_batch, max_wait_us=max_wait_us)
        try:
            res = _run_workers(adm, reqs)
            free = [adm.partition_free(p) for p in range(parts.p)]
        finally:
            adm.close()
    order, ref, fin = _oracle_in_admitted_order(nodes, parts, reqs, res, kmax=8)
    for row, i in enumerate(order):
        k = max(reqs[i][6], 1)
        got = res[i][0]
        want = [int(x) for x in ref[row, :k]] if ref[row, 0] >= 0 else [int(ref[row, 0])]
        assert got == want, (i, row, got, want)
    # each batch is placed in priority order, and never holds more than max_batch requests
    by_batch = {}
    for i, r in enumerate(res):
        by_batch.setdefault(r[1], []).append((r[3], reqs[i][0]))
    for b, lst in by_batch.items():
        lst.sort()
        assert [p for _, p in lst] == sorted(p for _, p in lst)
        assert len(lst) == res[[i for i, r in enumerate(res) if r[1] == b][0]][2] <= max_batch
    if max_batch > 1 and max_wait_us >= 5000:
        assert len(by_batch) < len(reqs)  # concurrent callers really were coalesced
    # post-placement free capacity per partition = the oracle's final columns summed
    for p, f in enumerate(free):
        sel = ((nodes.part_mask >> np.uint32(p)) & np.uint32(1)).astype(bool)
        assert f == {"cpu": int(np.maximum(fin[0][sel], 0).sum()),
                     "mem_mib": int(np.maximum(fin[1][sel], 0).sum()),
                     "gpu": int(np.maximum(fin[2][sel], 0).sum())}, p


def test_reload_and_invalid_requests():
    nodes, _, parts = synth.make_c1()
    with Engine() as e:
        e.load_partitions(parts)
        adm = Admitter(e, max_batch=64, max_wait_us=1000)
        try:
            with pytest.raises(FitError) as ei:  # no node table yet: the batch fails, caller sees it
                adm.admit(0, 1, 1)
            assert ei.value.code == _lib.FIT_E_STATE
            adm.load_nodes(nodes)
            n0, *_ = adm.admit(0, 20, 1000)
            assert n0[0] >= 0
            with pytest.raises(FitError) as ei:
                adm.admit(1, -1, 10)
            assert ei.value.code == _lib.FIT_E_INVAL
            with pytest.raises(FitError):
                adm.admit(1, 1, 10, nodes_k=9)
            # fill the cluster: 8 nodes x 64 cpus; 64-cpu jobs take whole nodes
            got = [adm.admit(10 + i, 64, 1000)[0][0] for i in range(10)]
            assert sum(g >= 0 for g in got) <= 8 and got[-1] == FIT_UNPLACED
            # a fresh node table makes room again
            adm.load_nodes(nodes)
            assert adm.admit(100, 64, 1000)[0][0] >= 0
        finally:
            adm.close()


def test_destroy_releases_waiting_callers():
    nodes, jobs, parts = synth.make_config("c2", 64, 256)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        adm = Admitter(e, max_batch=1 << 20, max_wait_us=5_000_000)  # batches close only at destroy
        errs = []

        def caller(i):
            try:
                adm.admit(i, 1, 10)
            except FitError as x:
                errs.append(x.code)

        th = [threading.Thread(target=caller, args=(i,)) for i in range(8)]
        for t in th:
            t.start()
        import time
        time.sleep(0.2)
        adm.close()  # queued requests fail with FIT_E_STATE; close returns once they have left
        for t in th:
            t.join(timeout=30)
        assert errs == [_lib.FIT_E_STATE] * 8
