// admit.cpp — batched admission for the virtual kubelet's CreatePod (include/fitgpu.h
// "batched admission").
//
// The reference admits pods one at a time: CreatePod (pkg/slurm-virtual-kubelet/provider.go:35-60)
// runs on 10 PodSyncWorker goroutines (options/options.go:107) and goes straight to SubmitJob with
// no capacity check.  Here each CreatePod calls fit_admit (or fit_admit_group for the tasks of an
// array job), which blocks while a coalescer thread gathers the concurrent requests into one
// batch, orders it by (priority, arrival), places it with ONE fit_place (sequential best-fit over
// the whole batch) and hands every caller its own result — one engine launch per
// batch instead of one decision per pod, and the priority order of the batch decides who gets a
// contended node, not goroutine timing.
//
// Every placed request holds a reservation (ticket) until the caller confirms it (Slurm now
// counts the job) or releases it (the job will not run).  A node-table reload re-applies the open
// reservations, so a refresh from Slurm — which does not yet count admitted-but-unallocated jobs —
// never hands their capacity out twice; a release gives the demand back to the current table.
//
// Threads: callers enqueue under `m` and wait on their own unit's `done` flag (cv `cv_done`);
// the coalescer thread owns the fit_ctx for the duration of a batch; fit_admitter_load_nodes,
// fit_admitter_partition_free and the reservation calls take `ctx_m`, so they never interleave
// with a placement.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fitgpu.h"

namespace fitgpu {
void set_last_error(const char* msg);  // engine.cpp (thread-local fit_last_error)
}

namespace {

using Clock = std::chrono::steady_clock;

// One caller's requests: 1 (fit_admit) or a whole array job (fit_admit_group), never split
// across batches.
struct Unit {
    const fit_admit_req* q;
    fit_admit_res* res;
    int32_t n;
    int64_t seq;      // arrival order (tie-break of equal priorities)
    Clock::time_point t_in;
    bool done = false;
    int rc = FIT_OK;
    std::string err;  // fit_last_error of the batch, for the caller's thread
};

struct Resv {
    int32_t node[FIT_MAX_K];
    int32_t k;
    int32_t cpu, mem, gpu;
    int32_t loads;    // node-table loads that re-applied it
    bool confirmed;
};

}  // namespace

struct fit_admitter {
    fit_ctx* ctx;
    int32_t max_batch;
    std::chrono::microseconds max_wait;

    std::mutex m;                       // queue, stop flag, unit completion
    std::condition_variable cv_work;    // coalescer: a request arrived / stop
    std::condition_variable cv_done;    // callers: a batch finished
    std::deque<Unit*> pending;
    int32_t pending_jobs = 0;
    bool stop = false;
    int64_t next_seq = 0;
    int64_t batches = 0;
    int inside = 0;                     // callers inside fit_admit* (destroy waits for them)

    std::mutex ctx_m;                   // the fit_ctx, reservations, the loaded table copy
    std::thread worker;
    std::map<int64_t, Resv> resv;       // open reservations by ticket
    int64_t next_ticket = 1;
    int32_t ttl = 0;
    std::vector<Resv> giveback;         // released demand not yet returned to the table
    // the last table loaded through the admitter (avail / mask do not change with placements;
    // a give-back reloads the current free columns with them)
    int32_t n = -1;
    std::vector<int32_t> avail;
    std::vector<uint32_t> mask;

    // batch arrays, reused
    std::vector<int32_t> cpu, mem, gpu, wall, out;
    std::vector<uint16_t> part, nk;

    void run();
    void place_batch(std::vector<Unit*>& b);
    int apply_giveback();  // under ctx_m
};

int fit_admitter::apply_giveback() {
    if (giveback.empty()) return FIT_OK;
    if (n < 0) return FIT_E_STATE;
    std::vector<int32_t> c((size_t)std::max(n, 1)), me((size_t)std::max(n, 1)), g((size_t)std::max(n, 1));
    int rc = fit_read_nodes(ctx, c.data(), me.data(), g.data());
    if (rc) return rc;
    for (const Resv& r : giveback)
        for (int i = 0; i < r.k; ++i) {
            const int32_t x = r.node[i];
            if (x < 0 || x >= n) continue;
            c[x] = (int32_t)std::min<int64_t>((int64_t)c[x] + r.cpu, INT32_MAX);
            me[x] = (int32_t)std::min<int64_t>((int64_t)me[x] + r.mem, INT32_MAX);
            g[x] = (int32_t)std::min<int64_t>((int64_t)g[x] + r.gpu, INT32_MAX);
        }
    rc = fit_load_nodes(ctx, n, c.data(), me.data(), g.data(), avail.data(), mask.data());
    if (rc == FIT_OK) giveback.clear();
    return rc;
}

void fit_admitter::place_batch(std::vector<Unit*>& b) {
    // priority order; arrival order among equal priorities (stable); a unit stays contiguous
    std::sort(b.begin(), b.end(), [](const Unit* x, const Unit* y) {
        return x->q[0].priority != y->q[0].priority ? x->q[0].priority < y->q[0].priority
                                                    : x->seq < y->seq;
    });
    int32_t j = 0, kmax = 1;
    for (const Unit* u : b) {
        j += u->n;
        for (int32_t i = 0; i < u->n; ++i)
            kmax = std::max<int32_t>(kmax, std::max<int32_t>(u->q[i].nodes_k, 1));
    }
    cpu.resize(j), mem.resize(j), gpu.resize(j), wall.resize(j), part.resize(j), nk.resize(j);
    out.assign((size_t)j * kmax, -1);
    int32_t row = 0;
    for (const Unit* u : b)
        for (int32_t i = 0; i < u->n; ++i, ++row) {
            const fit_admit_req& q = u->q[i];
            cpu[row] = q.cpu;
            mem[row] = q.mem_mib;
            gpu[row] = q.gpu;
            wall[row] = q.wall_min;
            part[row] = q.part;
            nk[row] = q.nodes_k;
        }
    int rc;
    std::string err;
    const int64_t batch = batches++;
    std::lock_guard<std::mutex> g(ctx_m);
    rc = apply_giveback();
    if (rc == FIT_OK) {
        fit_stats st;
        rc = fit_place(ctx, j, cpu.data(), mem.data(), gpu.data(), wall.data(), part.data(),
                       nk.data(), kmax, out.data(), &st);
    }
    if (rc != FIT_OK) err = fit_last_error();
    row = 0;
    for (Unit* u : b) {
        u->rc = rc;
        u->err = err;
        if (rc != FIT_OK) {
            row += u->n;
            continue;
        }
        // all or nothing: a unit is admitted only if every one of its requests got its nodes
        bool all = true, rejected = false;
        for (int32_t i = 0; i < u->n; ++i) {
            const int32_t v = out[(size_t)(row + i) * kmax];
            all = all && v >= 0;
            rejected = rejected || v == FIT_REJECTED;
        }
        for (int32_t i = 0; i < u->n; ++i, ++row) {
            fit_admit_res& o = u->res[i];
            const fit_admit_req& q = u->q[i];
            const int k = std::max<int>(q.nodes_k, 1);
            Resv r{};
            r.k = k;
            r.cpu = q.cpu;
            r.mem = q.mem_mib;
            r.gpu = q.gpu;
            for (int x = 0; x < FIT_MAX_K; ++x) {
                o.node[x] = x < kmax ? out[(size_t)row * kmax + x] : -1;
                r.node[x] = x < k ? o.node[x] : -1;
            }
            o.batch = batch;
            o.batch_jobs = j;
            o.order = row;
            o.ticket = 0;
            if (all) {
                o.ticket = next_ticket++;
                resv.emplace(o.ticket, r);
            } else {
                if (o.node[0] >= 0) giveback.push_back(r);  // a partial group: undo its part
                for (int x = 0; x < FIT_MAX_K; ++x) o.node[x] = -1;
                o.node[0] = rejected ? FIT_REJECTED : FIT_UNPLACED;
            }
        }
    }
}

void fit_admitter::run() {
    std::vector<Unit*> b;
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
        cv_work.wait(lk, [&] { return stop || !pending.empty(); });
        if (stop) break;
        // the batch stays open max_wait after its first request, or until it is full
        const Clock::time_point close = pending.front()->t_in + max_wait;
        cv_work.wait_until(lk, close, [&] { return stop || pending_jobs >= max_batch; });
        if (stop) break;
        b.clear();
        int32_t jobs = 0;
        // whole units up to max_batch requests (a unit larger than max_batch goes alone)
        while (!pending.empty() && (b.empty() || jobs + pending.front()->n <= max_batch)) {
            jobs += pending.front()->n;
            pending_jobs -= pending.front()->n;
            b.push_back(pending.front());
            pending.pop_front();
        }
        lk.unlock();  // new requests queue for the next batch meanwhile
        place_batch(b);
        lk.lock();
        for (Unit* u : b) u->done = true;
        cv_done.notify_all();
    }
    for (Unit* u : pending) {  // shutting down: nothing more is placed
        u->rc = FIT_E_STATE;
        u->err = "admitter destroyed while the request was queued";
        u->done = true;
    }
    pending.clear();
    pending_jobs = 0;
    cv_done.notify_all();
}

namespace {

int enqueue_and_wait(fit_admitter* a, const fit_admit_req* reqs, int32_t n, fit_admit_res* res) {
    for (int32_t i = 0; i < n; ++i) {
        const fit_admit_req& q = reqs[i];
        if (q.cpu < 0 || q.mem_mib < 0 || q.gpu < 0 || q.wall_min < 0 || q.nodes_k > FIT_MAX_K) {
            fitgpu::set_last_error("fit_admit: negative demand or nodes_k > FIT_MAX_K");
            return FIT_E_INVAL;
        }
    }
    Unit u;
    u.q = reqs;
    u.res = res;
    u.n = n;
    u.t_in = Clock::now();
    std::unique_lock<std::mutex> lk(a->m);
    if (a->stop) {
        fitgpu::set_last_error("fit_admit: admitter is shutting down");
        return FIT_E_STATE;
    }
    u.seq = a->next_seq++;
    ++a->inside;
    a->pending.push_back(&u);
    a->pending_jobs += n;
    a->cv_work.notify_one();
    a->cv_done.wait(lk, [&] { return u.done; });
    if (--a->inside == 0 && a->stop) a->cv_done.notify_all();  // destroy may be waiting
    if (u.rc != FIT_OK) fitgpu::set_last_error(u.err.c_str());
    return u.rc;
}

}  // namespace

extern "C" {

int fit_admitter_create(fit_ctx* ctx, int32_t max_batch, int32_t max_wait_us, fit_admitter** out) {
    if (!ctx || !out || max_batch < 1 || max_wait_us < 0) {
        fitgpu::set_last_error("fit_admitter_create: ctx/out NULL, max_batch < 1 or max_wait_us < 0");
        return FIT_E_INVAL;
    }
    fit_admitter* a = new (std::nothrow) fit_admitter;
    if (!a) return FIT_E_OOM;
    a->ctx = ctx;
    a->max_batch = max_batch;
    a->max_wait = std::chrono::microseconds(max_wait_us);
    try {
        a->worker = std::thread([a] { a->run(); });
    } catch (...) {
        delete a;
        fitgpu::set_last_error("fit_admitter_create: cannot start the coalescer thread");
        return FIT_E_OOM;
    }
    *out = a;
    return FIT_OK;
}

int fit_admit(fit_admitter* a, const fit_admit_req* req, fit_admit_res* res) {
    if (!a || !req || !res) return FIT_E_INVAL;
    return enqueue_and_wait(a, req, 1, res);
}

int fit_admit_group(fit_admitter* a, const fit_admit_req* reqs, int32_t n, fit_admit_res* res) {
    if (!a || !reqs || !res || n < 1) return FIT_E_INVAL;
    return enqueue_and_wait(a, reqs, n, res);
}

int fit_admitter_load_nodes(fit_admitter* a, int32_t n, const int32_t* cpu_free,
                            const int32_t* mem_free, const int32_t* gpu_free,
                            const int32_t* avail_min, const uint32_t* part_mask) {
    if (!a || n < 0 || (n > 0 && (!cpu_free || !mem_free || !gpu_free || !avail_min || !part_mask)))
        return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    // re-apply the open reservations to the new table (Slurm does not count them yet); confirmed
    // ones are in Slurm's allocation now, expired ones are dropped
    std::vector<int32_t> c(cpu_free, cpu_free + n), me(mem_free, mem_free + n), gp(gpu_free, gpu_free + n);
    for (auto it = a->resv.begin(); it != a->resv.end();) {
        Resv& r = it->second;
        if (r.confirmed || (a->ttl > 0 && r.loads >= a->ttl)) {
            it = a->resv.erase(it);
            continue;
        }
        ++r.loads;
        for (int i = 0; i < r.k; ++i) {
            const int32_t x = r.node[i];
            if (x < 0 || x >= n) continue;  // the node left the table
            c[x] = (int32_t)std::max<int64_t>((int64_t)c[x] - r.cpu, INT32_MIN);
            me[x] = (int32_t)std::max<int64_t>((int64_t)me[x] - r.mem, INT32_MIN);
            gp[x] = (int32_t)std::max<int64_t>((int64_t)gp[x] - r.gpu, INT32_MIN);
        }
        ++it;
    }
    a->giveback.clear();  // the new table supersedes the old one
    const int rc = fit_load_nodes(a->ctx, n, c.data(), me.data(), gp.data(), avail_min, part_mask);
    if (rc == FIT_OK) {
        a->n = n;
        a->avail.assign(avail_min, avail_min + n);
        a->mask.assign(part_mask, part_mask + n);
    } else {
        a->n = -1;
    }
    return rc;
}

int fit_admitter_partition_free(fit_admitter* a, int32_t p, int64_t* cpu, int64_t* mem_mib,
                                int64_t* gpu) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    const int rc = a->apply_giveback();
    if (rc) return rc;
    return fit_partition_free(a->ctx, p, cpu, mem_mib, gpu);
}

int fit_admitter_confirm(fit_admitter* a, int64_t ticket) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    auto it = a->resv.find(ticket);
    if (it == a->resv.end()) {
        fitgpu::set_last_error("fit_admitter_confirm: unknown ticket");
        return FIT_E_INVAL;
    }
    it->second.confirmed = true;
    return FIT_OK;
}

int fit_admitter_release(fit_admitter* a, int64_t ticket) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    auto it = a->resv.find(ticket);
    if (it == a->resv.end()) {
        fitgpu::set_last_error("fit_admitter_release: unknown ticket");
        return FIT_E_INVAL;
    }
    if (!it->second.confirmed) {
        if (a->n < 0) {
            fitgpu::set_last_error("fit_admitter_release: no node table loaded through the admitter");
            return FIT_E_STATE;
        }
        a->giveback.push_back(it->second);
    }
    a->resv.erase(it);
    return FIT_OK;
}

int fit_admitter_set_ttl(fit_admitter* a, int32_t loads) {
    if (!a || loads < 0) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    a->ttl = loads;
    return FIT_OK;
}

int fit_admitter_reservations(fit_admitter* a) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    int n = 0;
    for (const auto& kv : a->resv) n += !kv.second.confirmed;
    return n;
}

int fit_admitter_pending(fit_admitter* a) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->m);
    return a->pending_jobs;
}

void fit_admitter_destroy(fit_admitter* a) {
    if (!a) return;
    {
        std::lock_guard<std::mutex> g(a->m);
        a->stop = true;
    }
    a->cv_work.notify_all();
    if (a->worker.joinable()) a->worker.join();
    {  // every queued request is done now; let their callers leave before the memory goes
        std::unique_lock<std::mutex> lk(a->m);
        a->cv_done.wait(lk, [&] { return a->inside == 0; });
    }
    delete a;
}

}  // extern "C"
