// admit.cpp — batched admission for the virtual kubelet's CreatePod (include/fitgpu.h
// "batched admission").
//
// The reference admits pods one at a time: CreatePod (pkg/slurm-virtual-kubelet/provider.go:35-60)
// runs on 10 PodSyncWorker goroutines (options/options.go:107) and goes straight to SubmitJob with
// no capacity check.  Here each CreatePod calls fit_admit, which blocks while a coalescer thread
// gathers the concurrent requests into one batch, orders it by (priority, arrival), places it with
// ONE fit_place (sequential best-fit over the whole batch) and hands every caller
// its own result — one engine launch per batch instead of one decision per pod, and the priority
// order of the batch decides who gets a contended node, not goroutine timing.
//
// Threads: callers enqueue under `m` and wait on their own request's `done` flag (cv `cv_done`);
// the coalescer thread owns the fit_ctx for the duration of a batch; fit_admitter_load_nodes and
// fit_admitter_partition_free take `ctx_m`, so they never interleave with a placement.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
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

struct Request {
    fit_admit_req q;
    fit_admit_res* res;
    int64_t seq;      // arrival order (tie-break of equal priorities)
    Clock::time_point t_in;
    bool done = false;
    int rc = FIT_OK;
    std::string err;  // fit_last_error of the batch, for the caller's thread
};

}  // namespace

struct fit_admitter {
    fit_ctx* ctx;
    int32_t max_batch;
    std::chrono::microseconds max_wait;

    std::mutex m;                       // queue, stop flag, request completion
    std::condition_variable cv_work;    // coalescer: a request arrived / stop
    std::condition_variable cv_done;    // callers: a batch finished
    std::deque<Request*> pending;
    bool stop = false;
    int64_t next_seq = 0;
    int64_t batches = 0;
    int inside = 0;                     // callers inside fit_admit (destroy waits for them)

    std::mutex ctx_m;                   // the fit_ctx (placements vs node reloads / queries)
    std::thread worker;

    // batch arrays, reused
    std::vector<int32_t> cpu, mem, gpu, wall, out;
    std::vector<uint16_t> part, nk;

    void run();
    void place_batch(std::vector<Request*>& b);
};

void fit_admitter::place_batch(std::vector<Request*>& b) {
    // priority order; arrival order among equal priorities (stable)
    std::sort(b.begin(), b.end(), [](const Request* x, const Request* y) {
        return x->q.priority != y->q.priority ? x->q.priority < y->q.priority : x->seq < y->seq;
    });
    const int32_t j = (int32_t)b.size();
    int32_t kmax = 1;
    for (const Request* r : b) kmax = std::max<int32_t>(kmax, std::max<int32_t>(r->q.nodes_k, 1));
    cpu.resize(j), mem.resize(j), gpu.resize(j), wall.resize(j), part.resize(j), nk.resize(j);
    out.assign((size_t)j * kmax, -1);
    for (int32_t i = 0; i < j; ++i) {
        const fit_admit_req& q = b[i]->q;
        cpu[i] = q.cpu;
        mem[i] = q.mem_mib;
        gpu[i] = q.gpu;
        wall[i] = q.wall_min;
        part[i] = q.part;
        nk[i] = q.nodes_k;
    }
    int rc;
    std::string err;
    {
        std::lock_guard<std::mutex> g(ctx_m);
        fit_stats st;
        rc = fit_place(ctx, j, cpu.data(), mem.data(), gpu.data(), wall.data(), part.data(),
                       nk.data(), kmax, out.data(), &st);
        if (rc != FIT_OK) err = fit_last_error();
    }
    const int64_t batch = batches++;
    for (int32_t i = 0; i < j; ++i) {
        Request* r = b[i];
        r->rc = rc;
        r->err = err;
        if (rc == FIT_OK) {
            fit_admit_res& o = *r->res;
            for (int k = 0; k < FIT_MAX_K; ++k) o.node[k] = k < kmax ? out[(size_t)i * kmax + k] : -1;
            o.batch = batch;
            o.batch_jobs = j;
            o.order = i;
        }
    }
}

void fit_admitter::run() {
    std::vector<Request*> b;
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
        cv_work.wait(lk, [&] { return stop || !pending.empty(); });
        if (stop) break;
        // the batch stays open max_wait after its first request, or until it is full
        const Clock::time_point close = pending.front()->t_in + max_wait;
        cv_work.wait_until(lk, close, [&] { return stop || (int32_t)pending.size() >= max_batch; });
        if (stop) break;
        b.clear();
        while (!pending.empty() && (int32_t)b.size() < max_batch) {
            b.push_back(pending.front());
            pending.pop_front();
        }
        lk.unlock();  // new requests queue for the next batch meanwhile
        place_batch(b);
        lk.lock();
        for (Request* r : b) r->done = true;
        cv_done.notify_all();
    }
    for (Request* r : pending) {  // shutting down: nothing more is placed
        r->rc = FIT_E_STATE;
        r->err = "admitter destroyed while the request was queued";
        r->done = true;
    }
    pending.clear();
    cv_done.notify_all();
}

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
    if (req->cpu < 0 || req->mem_mib < 0 || req->gpu < 0 || req->wall_min < 0 ||
        req->nodes_k > FIT_MAX_K) {
        fitgpu::set_last_error("fit_admit: negative demand or nodes_k > FIT_MAX_K");
        return FIT_E_INVAL;
    }
    Request r;
    r.q = *req;
    r.res = res;
    r.t_in = Clock::now();
    std::unique_lock<std::mutex> lk(a->m);
    if (a->stop) {
        fitgpu::set_last_error("fit_admit: admitter is shutting down");
        return FIT_E_STATE;
    }
    r.seq = a->next_seq++;
    ++a->inside;
    a->pending.push_back(&r);
    a->cv_work.notify_one();
    a->cv_done.wait(lk, [&] { return r.done; });
    if (--a->inside == 0 && a->stop) a->cv_done.notify_all();  // destroy may be waiting
    if (r.rc != FIT_OK) fitgpu::set_last_error(r.err.c_str());
    return r.rc;
}

int fit_admitter_load_nodes(fit_admitter* a, int32_t n, const int32_t* cpu_free,
                            const int32_t* mem_free, const int32_t* gpu_free,
                            const int32_t* avail_min, const uint32_t* part_mask) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    return fit_load_nodes(a->ctx, n, cpu_free, mem_free, gpu_free, avail_min, part_mask);
}

int fit_admitter_partition_free(fit_admitter* a, int32_t p, int64_t* cpu, int64_t* mem_mib,
                                int64_t* gpu) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    return fit_partition_free(a->ctx, p, cpu, mem_mib, gpu);
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
