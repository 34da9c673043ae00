"""Batched admission (include/fitgpu.h fit_admitter): concurrent
CreatePod-style callers (the virtual kubelet's 10 PodSyncWorkers, options/options.go:107) block in
fit_admit, a coalescer places each batch with one fit_place in (priority, arrival) order.

Parity: the placements every caller received, taken in the order the admitter placed them (batch,
then position in the batch), equal the oracle's sequential best fit of the same jobs in that
order from the same node table — bit-exact, including the final free columns per partition."""
import threading

import numpy as np
import pytest

import fitgpu
from fitgpu import FIT_UNPLACED, Admitter, Engine, FitError, synth
from fitgpu import _lib
from oracle import pyoracle as po

pytestmark = [pytest.mark.gpu, pytest.mark.auto_engine]


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
            res = [adm.admit(10 + i, 64, 1000) for i in range(10)]
            got = [r[0][0] for r in res]
            assert sum(g >= 0 for g in got) <= 8 and got[-1] == FIT_UNPLACED
            # reloading Slurm's unchanged table keeps the admitted pods' reservations
            adm.load_nodes(nodes)
            assert adm.admit(99, 64, 1000)[0][0] == FIT_UNPLACED
            # once Slurm counts (then frees) those jobs, a fresh table makes room again
            for r in res:
                if r[4]:
                    adm.confirm(r[4])
            adm.load_nodes(nodes)
            assert adm.admit(100, 64, 1000)[0][0] >= 0
        finally:
            adm.close()


def test_destroy_releases_waiting_callers():
    """fit_admitter_destroy with callers queued inside fit_admit: they return FIT_E_STATE and
    destroy returns once they have left.  Raw C calls, so the test owns the handle's lifetime; it
    waits until all 8 requests are queued (fit_admitter_pending) before destroying."""
    import ctypes as C
    import time
    from fitgpu._lib import FitAdmitReq, FitAdmitRes, lib
    nodes, jobs, parts = synth.make_config("c2", 64, 256)
    with Engine() as e:
        e.load_nodes(nodes)
        e.load_partitions(parts)
        h = C.c_void_p()
        assert lib().fit_admitter_create(e._h, 1 << 20, 60_000_000, C.byref(h)) == 0  # closes only at destroy
        rcs = []

        def caller(i):
            q, r = FitAdmitReq(i, 1, 10, 0, 0, 0, 1), FitAdmitRes()
            rcs.append(lib().fit_admit(h, C.byref(q), C.byref(r)))

        th = [threading.Thread(target=caller, args=(i,)) for i in range(8)]
        for t in th:
            t.start()
        t0 = time.monotonic()
        while lib().fit_admitter_pending(h) < 8:
            assert time.monotonic() - t0 < 60, "callers never queued"
            time.sleep(0.005)
        lib().fit_admitter_destroy(h)
        for t in th:
            t.join(timeout=30)
        assert rcs == [_lib.FIT_E_STATE] * 8


def test_admitter_lifetime_with_engine_close():
    """Engine.close() closes its admitters first; an admit after that raises FIT_E_STATE instead of
    reaching a freed context (Admitter kept the Engine, close() did not know)."""
    nodes, _, parts = synth.make_c1()
    e = Engine()
    e.load_nodes(nodes)
    e.load_partitions(parts)
    adm = Admitter(e, max_batch=8, max_wait_us=100)
    assert adm.admit(0, 3, 1500)[0][0] >= 0
    e.close()
    with pytest.raises(FitError) as ei:
        adm.admit(1, 3, 1500)
    assert ei.value.code == _lib.FIT_E_STATE
    adm.close()  # idempotent


def _c1_with_limits(max_time):
    nodes, _, parts = synth.make_c1()
    parts = synth.Partitions(np.full(1, max_time, np.int32), np.full(1, -1, np.int32), np.full(1, -1, np.int32))
    return nodes, parts


SAMPLE_SCRIPT = "#!/bin/sh\n#SBATCH --nodes=1\n#SBATCH --time={t}\nsrun hostname\nhostname\npwd\n"
SAMPLE_LABELS = {fitgpu.POD_LABEL_KEYS["ntasks"]: "3", fitgpu.POD_LABEL_KEYS["mem_per_cpu"]: "500",
                 fitgpu.POD_LABEL_KEYS["cpus_per_task"]: "1"}


def test_pod_demand_array_and_maxtime_through_admission():
    """the reference's label set (the sample manifest's, pod.go:164-190) plus a
    script with --time and an --array label → fit_pod_demand → fit_admit_group → bit-exact vs the
    oracle's sequential best fit of the expanded tasks; a --time above the partition's MaxTime is
    FIT_REJECTED (parseResources MaxTime, pkg/slurm-agent/parse.go:128-138); a group that does not
    fit takes nothing."""
    nodes, parts = _c1_with_limits(60)
    labels = dict(SAMPLE_LABELS, **{fitgpu.POD_LABEL_KEYS["array"]: "1-4"})
    pods = [(labels, SAMPLE_SCRIPT.format(t="0:30:00")),               # 4 tasks x (3 cpu, 1500 MiB, 30 min)
            (dict(SAMPLE_LABELS), SAMPLE_SCRIPT.format(t="2:00:00")),   # 120 min > MaxTime 60: rejected
            (dict(labels, **{fitgpu.POD_LABEL_KEYS["cpus_per_task"]: "20",
                             fitgpu.POD_LABEL_KEYS["array"]: "1-40"}), SAMPLE_SCRIPT.format(t="10")),  # too big
            (dict(labels, **{fitgpu.POD_LABEL_KEYS["array"]: "0-9%3"}), SAMPLE_SCRIPT.format(t="1:00:00"))]
    reqs = [fitgpu.pod_demand(l, s, 0, prio) for prio, (l, s) in enumerate(pods)]
    assert [len(r) for r in reqs] == [4, 1, 40, 3]
    assert reqs[0][0] == (0, 3, 1500, 0, 30, 0, 1, fitgpu.FIT_REQ_ARRAY) and reqs[1][0][4] == 120
    with Engine() as e:
        e.load_partitions(parts)
        with Admitter(e, max_batch=64, max_wait_us=1000) as adm:
            adm.load_nodes(nodes)
            got = [adm.admit_group(r) for r in reqs]  # one pod after the other (own batches)
            free = adm.partition_free(0)
            assert adm.reservations() == 4 + 3
    assert all(g[0][0] >= 0 and g[4] > 0 for g in got[0]) and all(g[0][0] >= 0 for g in got[3])
    assert [g[0] for g in got[1]] == [[fitgpu.FIT_REJECTED]] and got[1][0][4] == 0
    assert all(g[0] == [FIT_UNPLACED] and g[4] == 0 for g in got[2])
    # oracle: the admitted tasks in order (the rejected pod and the failed group take nothing)
    q = reqs[0] + reqs[3]
    jobs = synth.Jobs(*(np.array([r[i] for r in q], dt) for i, dt in
                        ((1, np.int32), (2, np.int32), (3, np.int32), (4, np.int32), (5, np.uint16), (6, np.uint16))))
    ref, _, fin = po.ref_place(nodes, jobs, parts)
    assert [g[0][0] for g in got[0] + got[3]] == ref[:, 0].tolist()
    assert free == {"cpu": int(fin[0].sum()), "mem_mib": int(fin[1].sum()), "gpu": int(fin[2].sum())}
    # the rejected pod against the oracle too
    one = synth.Jobs(*(np.array([reqs[1][0][i]], dt) for i, dt in
                       ((1, np.int32), (2, np.int32), (3, np.int32), (4, np.int32), (5, np.uint16), (6, np.uint16))))
    assert po.ref_place(nodes, one, parts)[0][0, 0] == fitgpu.FIT_REJECTED


def test_reservations_survive_refresh():
    """admitted-but-unallocated pods keep their capacity across a node-table
    reload (the ticker's Refresh re-reads Slurm, which does not count them yet); confirm drops a
    reservation at the next load (Slurm counts the job now), release gives it back at once."""
    nodes, parts = _c1_with_limits(-1)
    total = {"cpu": 8 * 64, "mem_mib": 8 * 262144, "gpu": 0}
    with Engine() as e:
        e.load_partitions(parts)
        with Admitter(e, max_batch=64, max_wait_us=500) as adm:
            adm.load_nodes(nodes)
            a = adm.admit(0, 60, 1000)
            b = adm.admit(1, 60, 2000)
            c = adm.admit(2, 4, 100)
            assert all(x[0][0] >= 0 and x[4] > 0 for x in (a, b, c))
            taken = {"cpu": 124, "mem_mib": 3100, "gpu": 0}
            left = {k: total[k] - taken[k] for k in total}
            assert adm.partition_free(0) == left
            adm.load_nodes(nodes)  # Slurm's view: nothing allocated yet → all three re-applied
            assert adm.partition_free(0) == left and adm.reservations() == 3
            # the new table is placed against with the reservations in it: a 64-cpu job cannot
            # land on a's or b's node
            d = adm.admit(3, 64, 10)
            assert d[0][0] not in (a[0][0], b[0][0])
            adm.confirm(a[4])  # a is running now: the next Slurm table carries it
            adm.release(b[4])  # b's pod was deleted before it ran
            assert adm.partition_free(0)["cpu"] == left["cpu"] + 60 - 64
            alloc = synth.Nodes(nodes.cpu_free.copy(), nodes.mem_free.copy(), nodes.gpu_free.copy(),
                                nodes.avail_min, nodes.part_mask)
            alloc.cpu_free[a[0][0]] -= 60  # what Slurm reports once a runs
            alloc.mem_free[a[0][0]] -= 1000
            adm.load_nodes(alloc)
            assert adm.reservations() == 2  # c and d
            assert adm.partition_free(0) == {"cpu": total["cpu"] - 60 - 4 - 64, "mem_mib": total["mem_mib"] - 1110,
                                             "gpu": 0}
            with pytest.raises(FitError):
                adm.release(b[4])  # already gone
            adm.set_ttl(1)  # c and d have each been re-applied by at least one load: they expire now
            adm.load_nodes(alloc)
            assert adm.reservations() == 0 and adm.partition_free(0)["cpu"] == total["cpu"] - 60
