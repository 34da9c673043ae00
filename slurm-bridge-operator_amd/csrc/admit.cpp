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
// reservations (by node name when both tables are named), so a refresh from Slurm — which does
// not yet count admitted-but-unallocated jobs — never hands their capacity out twice; a release
// gives the demand back.
//
// The admitter keeps the node table on the host as it really is — the loaded free columns minus
// every placement, unclamped int64 — and the engine's copy is reloaded from it whenever they
// differ (a release, a group that has to be re-placed).  The engine clamps free values at -1
// (k_gather_nodes), which is exact for placement but cannot be added back to.
//
// Threads: callers enqueue under `m` and wait on their own unit's `done` flag — spinning for up to
// kSpinCaller first (yielding the core after kSpinHot, so ten waiting callers do not starve the
// coalescer on a busy host) (a batch takes a few tens of µs; a futex wake-up costs as much again, twice
// per pod: the coalescer's and the caller's), then on cv `cv_done`; the coalescer likewise spins
// for up to kSpinCoalescer on the queue after a batch before it blocks;
// the coalescer thread owns the fit_ctx for the duration of a batch; table loads, queries and the
// reservation calls take `ctx_m`, so they never interleave with a placement.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/fitgpu.h"

namespace fitgpu {
void set_last_error(const char* msg);  // engine.cpp (thread-local fit_last_error)
int64_t ctx_load_count(const fit_ctx* c);
int ctx_table(fit_ctx* c, std::vector<int32_t>& cpu, std::vector<int32_t>& mem,
              std::vector<int32_t>& gpu, std::vector<int32_t>& avail, std::vector<uint32_t>& mask);
int script_with_names(const char* script, const std::vector<std::string_view>& names, char* out,
                      int32_t outlen);  // ingest.cpp
}  // namespace fitgpu

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
    std::atomic<bool> done{false};  // set under `m` (release); callers spin on it without `m`
    int rc = FIT_OK;
    std::string err;  // fit_last_error of the batch, for the caller's thread
};

// Names of one loaded table (shared by the reservations that live in it).
struct Names {
    std::vector<std::string> name;
    std::unordered_map<std::string_view, int32_t> id;
    bool pinnable = false;  // FIT_TABLE_STATE (the engine never chose a node Slurm would refuse)
                            // or FIT_TABLE_PIN (the operator pins without State)
};

struct Resv {
    int32_t node[FIT_MAX_K];  // ids in the CURRENT table (remapped at every load), -1 = gone
    int32_t k;
    int32_t cpu, mem, gpu;
    int32_t loads;            // node-table loads that re-applied it
    bool confirmed;
    bool array;               // a task of an array job (FIT_REQ_ARRAY): never pinned
    int64_t confirm_gen;      // latest table generation handed out when it was confirmed
    std::shared_ptr<const Names> names;
};

int32_t sat32(int64_t v) { return v > INT32_MAX ? INT32_MAX : v < INT32_MIN ? INT32_MIN : (int32_t)v; }

}  // namespace

// spin budgets before blocking (see the Threads note at the top)
constexpr std::chrono::microseconds kSpinCaller{200};
constexpr std::chrono::microseconds kSpinHot{30};  // callers: pause-spin this long, then yield
constexpr std::chrono::microseconds kSpinCoalescer{50};

inline void cpu_relax() { __builtin_ia32_pause(); }

struct fit_admitter {
    fit_ctx* ctx;
    int32_t max_batch;
    std::chrono::microseconds max_wait;

    std::mutex m;                       // queue, stop flag, unit completion
    std::condition_variable cv_work;    // coalescer: a request arrived / stop
    std::condition_variable cv_done;    // callers: a batch finished
    std::deque<Unit*> pending;
    std::atomic<int32_t> queued{0};     // pending.size(), for the coalescer's spin outside `m`
    int32_t pending_jobs = 0;
    bool stop = false;
    int64_t next_seq = 0;
    int64_t batches = 0;
    int inside = 0;                     // callers inside fit_admit* (destroy waits for them)

    std::mutex ctx_m;                   // everything below
    std::thread worker;
    std::map<int64_t, Resv> resv;       // reservations by ticket
    int64_t next_ticket = 1;
    int32_t ttl = 0;
    int64_t gen_issued = 0, gen_loaded = 0;
    // the table as it really is: loaded free columns minus open reservations and placements
    int32_t n = -1;                     // -1: not taken over from the context yet
    std::vector<int64_t> hc, hm, hg;
    std::vector<int32_t> avail;
    std::vector<uint32_t> mask;
    std::shared_ptr<const Names> names;
    bool engine_stale = false;          // the engine's table differs from the host copy
    int64_t ctx_loads_seen = -1;        // fitgpu::ctx_load_count after our own last load

    // batch arrays, reused
    std::vector<int32_t> cpu, mem, gpu, wall, out, cols;
    std::vector<uint16_t> part, nk;

    void run();
    void place_batch(std::vector<Unit*>& b);
    // under ctx_m:
    int take_over();      // host copy from the context when it was loaded behind our back
    int push_engine();    // reload the engine from the host copy when they differ
};

int fit_admitter::take_over() {
    const int64_t lc = fitgpu::ctx_load_count(ctx);
    if (n >= 0 && lc == ctx_loads_seen) return FIT_OK;
    std::vector<int32_t> c, me, g;
    const int rc = fitgpu::ctx_table(ctx, c, me, g, avail, mask);
    if (rc) return rc;
    n = (int32_t)c.size();
    hc.assign(c.begin(), c.end());
    hm.assign(me.begin(), me.end());
    hg.assign(g.begin(), g.end());
    names.reset();  // a table loaded directly has no names
    engine_stale = false;
    ctx_loads_seen = lc;
    return FIT_OK;
}

int fit_admitter::push_engine() {
    if (!engine_stale) return FIT_OK;
    cols.resize((size_t)std::max(n, 1) * 3);
    int32_t* c = cols.data();
    int32_t* me = c + std::max(n, 1);
    int32_t* g = me + std::max(n, 1);
    for (int32_t x = 0; x < n; ++x) c[x] = sat32(hc[x]), me[x] = sat32(hm[x]), g[x] = sat32(hg[x]);
    const int rc = fit_load_nodes(ctx, n, c, me, g, avail.data(), mask.data());
    if (rc) return rc;
    engine_stale = false;
    ctx_loads_seen = fitgpu::ctx_load_count(ctx);
    return FIT_OK;
}

void fit_admitter::place_batch(std::vector<Unit*>& b) {
    // priority order; arrival order among equal priorities (stable); a unit stays contiguous
    std::sort(b.begin(), b.end(), [](const Unit* x, const Unit* y) {
        return x->q[0].priority != y->q[0].priority ? x->q[0].priority < y->q[0].priority
                                                    : x->seq < y->seq;
    });
    const size_t nu = b.size();
    std::vector<int32_t> first(nu);  // a unit's index in the batch's full placement order
    int32_t j_all = 0, kmax = 1;
    for (size_t u = 0; u < nu; ++u) {
        first[u] = j_all;
        j_all += b[u]->n;
        for (int32_t i = 0; i < b[u]->n; ++i)
            kmax = std::max<int32_t>(kmax, std::max<int32_t>(b[u]->q[i].nodes_k, 1));
    }
    int rc;
    std::string err;
    const int64_t batch = batches++;
    std::lock_guard<std::mutex> g(ctx_m);
    // A group (array job) is all or nothing: when one of its tasks is not placed, the group takes
    // nothing, and every later request of the batch must see the table without it — exactly the
    // sequential semantics of placing the units one after the other.  So such a group is dropped
    // and the batch placed again from the pre-batch table; units before it are unchanged by the
    // drop, so the next pass can only find a partial group further down (at most one extra pass
    // per failing group, and none in the common case).
    std::vector<char> dropped(nu, 0), rejected(nu, 0);
    std::vector<int32_t> row_of(nu, -1);  // first row of a unit in the last pass, -1 = dropped
    rc = take_over();
    for (;;) {
        if (rc == FIT_OK) rc = push_engine();
        if (rc != FIT_OK) break;
        int32_t j = 0;
        for (size_t u = 0; u < nu; ++u) {
            row_of[u] = dropped[u] ? -1 : j;
            if (!dropped[u]) j += b[u]->n;
        }
        cpu.resize(j), mem.resize(j), gpu.resize(j), wall.resize(j), part.resize(j), nk.resize(j);
        out.assign((size_t)std::max(j, 1) * kmax, -1);
        for (size_t u = 0; u < nu; ++u) {
            if (row_of[u] < 0) continue;
            for (int32_t i = 0; i < b[u]->n; ++i) {
                const fit_admit_req& q = b[u]->q[i];
                const int32_t r = row_of[u] + i;
                cpu[r] = q.cpu, mem[r] = q.mem_mib, gpu[r] = q.gpu, wall[r] = q.wall_min;
                part[r] = q.part, nk[r] = q.nodes_k;
            }
        }
        fit_stats st;
        rc = fit_place(ctx, j, cpu.data(), mem.data(), gpu.data(), wall.data(), part.data(),
                       nk.data(), kmax, out.data(), &st);
        if (rc != FIT_OK) {
            engine_stale = true;  // the engine's table is unknown now
            break;
        }
        bool again = false;
        for (size_t u = 0; u < nu && !again; ++u) {
            if (row_of[u] < 0 || b[u]->n < 2) continue;
            int32_t placed = 0;
            bool rej = false;
            for (int32_t i = 0; i < b[u]->n; ++i) {
                const int32_t v = out[(size_t)(row_of[u] + i) * kmax];
                placed += v >= 0;
                rej = rej || v == FIT_REJECTED;
            }
            if (placed > 0 && placed < b[u]->n) {
                dropped[u] = 1;
                rejected[u] = rej;
                engine_stale = true;  // back to the pre-batch table for the next pass
                again = true;
            }
        }
        if (!again) break;
    }
    if (rc != FIT_OK) err = fit_last_error();
    for (size_t u = 0; u < nu; ++u) {
        Unit* un = b[u];
        un->rc = rc;
        un->err = err;
        if (rc != FIT_OK) continue;
        // all or nothing: a unit is admitted only if every one of its requests got its nodes
        bool all = row_of[u] >= 0, rej = rejected[u] != 0;
        for (int32_t i = 0; row_of[u] >= 0 && i < un->n; ++i) {
            const int32_t v = out[(size_t)(row_of[u] + i) * kmax];
            all = all && v >= 0;
            rej = rej || v == FIT_REJECTED;
        }
        for (int32_t i = 0; i < un->n; ++i) {
            fit_admit_res& o = un->res[i];
            const fit_admit_req& q = un->q[i];
            const int k = std::max<int>(q.nodes_k, 1);
            for (int x = 0; x < FIT_MAX_K; ++x)
                o.node[x] = row_of[u] >= 0 && x < kmax ? out[(size_t)(row_of[u] + i) * kmax + x] : -1;
            o.batch = batch;
            o.batch_jobs = j_all;
            o.order = first[u] + i;
            o.ticket = 0;
            if (all) {
                Resv r{};
                r.k = k;
                r.cpu = q.cpu, r.mem = q.mem_mib, r.gpu = q.gpu;
                r.array = (q.flags & FIT_REQ_ARRAY) != 0;
                r.names = names;
                for (int x = 0; x < FIT_MAX_K; ++x) r.node[x] = x < k ? o.node[x] : -1;
                for (int x = 0; x < k; ++x) {  // the engine took it: so does the host copy
                    const int32_t nd = r.node[x];
                    hc[nd] -= q.cpu, hm[nd] -= q.mem_mib, hg[nd] -= q.gpu;
                }
                o.ticket = next_ticket++;
                resv.emplace(o.ticket, r);
            } else {
                // a single request that did not fit took nothing; a group that did not fit
                // entirely was dropped above and took nothing either
                for (int x = 0; x < FIT_MAX_K; ++x) o.node[x] = -1;
                o.node[0] = rej ? FIT_REJECTED : FIT_UNPLACED;
            }
        }
    }
}

void fit_admitter::run() {
    std::vector<Unit*> b;
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
        if (pending.empty() && !stop) {  // a short spin before blocking: the next pod is likely close
            lk.unlock();
            const Clock::time_point until = Clock::now() + kSpinCoalescer;
            while (queued.load(std::memory_order_relaxed) == 0 && Clock::now() < until) cpu_relax();
            lk.lock();
        }
        cv_work.wait(lk, [&] { return stop || !pending.empty(); });
        if (stop) break;
        // the batch stays open max_wait after its first request, or until it is full
        if (max_wait.count() > 0) {
            const Clock::time_point close = pending.front()->t_in + max_wait;
            cv_work.wait_until(lk, close, [&] { return stop || pending_jobs >= max_batch; });
            if (stop) break;
        }
        b.clear();
        int32_t jobs = 0;
        // whole units up to max_batch requests (a unit larger than max_batch goes alone)
        while (!pending.empty() && (b.empty() || jobs + pending.front()->n <= max_batch)) {
            jobs += pending.front()->n;
            pending_jobs -= pending.front()->n;
            b.push_back(pending.front());
            pending.pop_front();
            queued.fetch_sub(1, std::memory_order_relaxed);
        }
        lk.unlock();  // new requests queue for the next batch meanwhile
        place_batch(b);
        lk.lock();
        for (Unit* u : b) u->done.store(true, std::memory_order_release);
        cv_done.notify_all();
    }
    for (Unit* u : pending) {  // shutting down: nothing more is placed
        u->rc = FIT_E_STATE;
        u->err = "admitter destroyed while the request was queued";
        u->done.store(true, std::memory_order_release);
    }
    pending.clear();
    queued.store(0, std::memory_order_relaxed);
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
    a->queued.fetch_add(1, std::memory_order_relaxed);
    a->pending_jobs += n;
    a->cv_work.notify_one();
    lk.unlock();
    const Clock::time_point t0 = Clock::now(), until = t0 + kSpinCaller, hot = t0 + kSpinHot;
    while (!u.done.load(std::memory_order_acquire)) {
        const Clock::time_point now = Clock::now();
        if (now >= until) break;
        if (now < hot) cpu_relax();
        else std::this_thread::yield();  // past the hot phase: leave the core to the coalescer
    }
    lk.lock();
    a->cv_done.wait(lk, [&] { return u.done.load(std::memory_order_acquire); });
    if (--a->inside == 0 && a->stop) a->cv_done.notify_all();  // destroy may be waiting
    if (u.rc != FIT_OK) fitgpu::set_last_error(u.err.c_str());
    return u.rc;
}

int fail(int code, const char* msg) {
    fitgpu::set_last_error(msg);
    return code;
}

}  // namespace

extern "C" {

int fit_admitter_create(fit_ctx* ctx, int32_t max_batch, int32_t max_wait_us, fit_admitter** out) {
    if (!ctx || !out || max_batch < 1 || max_wait_us < 0)
        return fail(FIT_E_INVAL, "fit_admitter_create: ctx/out NULL, max_batch < 1 or max_wait_us < 0");
    fit_admitter* a = new (std::nothrow) fit_admitter;
    if (!a) return FIT_E_OOM;
    a->ctx = ctx;
    a->max_batch = max_batch;
    a->max_wait = std::chrono::microseconds(max_wait_us);
    try {
        a->worker = std::thread([a] { a->run(); });
    } catch (...) {
        delete a;
        return fail(FIT_E_OOM, "fit_admitter_create: cannot start the coalescer thread");
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

int64_t fit_admitter_generation(fit_admitter* a) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    return ++a->gen_issued;
}

int fit_admitter_load_table(fit_admitter* a, const fit_node_table* t) {
    if (!a || !t || t->n < 0 || t->n > FIT_MAX_NODES ||
        (t->n > 0 && (!t->cpu_free || !t->mem_free || !t->gpu_free || !t->avail_min || !t->part_mask)))
        return fail(FIT_E_INVAL, "fit_admitter_load_table: bad table");
    const int32_t n = t->n;
    auto nm = std::make_shared<Names>();
    if (t->names) {
        nm->name.reserve((size_t)n);
        const char* p = t->names;
        for (int32_t i = 0; i < n; ++i, p += strlen(p) + 1) nm->name.emplace_back(p);
        for (int32_t i = 0; i < n; ++i)
            if (nm->name[i].empty() || !nm->id.emplace(nm->name[i], i).second)
                return fail(FIT_E_INVAL, "fit_admitter_load_table: empty or repeated node name");
        nm->pinnable = (t->flags & (FIT_TABLE_STATE | FIT_TABLE_PIN)) != 0;
    }
    std::lock_guard<std::mutex> g(a->ctx_m);
    if (t->generation < 0 || t->generation > a->gen_issued)
        return fail(FIT_E_INVAL, "fit_admitter_load_table: generation not issued by fit_admitter_generation");
    if (t->generation != 0 && t->generation < a->gen_loaded)
        return fail(FIT_E_STATE, "fit_admitter_load_table: older than the table already loaded");
    const int64_t gen = t->generation ? t->generation : ++a->gen_issued;
    std::vector<int64_t> c(t->cpu_free, t->cpu_free + n), me(t->mem_free, t->mem_free + n),
        gp(t->gpu_free, t->gpu_free + n);
    // carry the reservations over: a confirmed one is in the new table if it was fetched after the
    // confirmation; every other one is taken from it again (Slurm does not count it yet)
    for (auto it = a->resv.begin(); it != a->resv.end();) {
        Resv& r = it->second;
        if ((r.confirmed && gen > r.confirm_gen) || (a->ttl > 0 && r.loads >= a->ttl)) {
            it = a->resv.erase(it);
            continue;
        }
        ++r.loads;
        const bool by_name = r.names && t->names;
        for (int i = 0; i < r.k; ++i) {
            int32_t& x = r.node[i];
            if (x < 0) continue;
            if (by_name) {
                auto f = nm->id.find(r.names->name[(size_t)x]);
                x = f == nm->id.end() ? -1 : f->second;  // the node left the partition
            } else if (x >= n) {
                x = -1;
            }
            if (x < 0) continue;
            c[x] -= r.cpu, me[x] -= r.mem, gp[x] -= r.gpu;
        }
        r.names = t->names ? nm : nullptr;
        ++it;
    }
    a->hc.swap(c), a->hm.swap(me), a->hg.swap(gp);
    a->avail.assign(t->avail_min, t->avail_min + n);
    a->mask.assign(t->part_mask, t->part_mask + n);
    a->n = n;
    a->names = t->names ? std::shared_ptr<const Names>(nm) : nullptr;
    a->gen_loaded = gen;
    a->engine_stale = true;
    const int rc = a->push_engine();
    if (rc != FIT_OK) a->n = -1;  // the context has no valid table: take it over again later
    return rc;
}

int fit_admitter_load_nodes(fit_admitter* a, int32_t n, const int32_t* cpu_free,
                            const int32_t* mem_free, const int32_t* gpu_free,
                            const int32_t* avail_min, const uint32_t* part_mask) {
    const fit_node_table t{n, cpu_free, mem_free, gpu_free, avail_min, part_mask, nullptr, 0, 0};
    return fit_admitter_load_table(a, &t);
}

int fit_admitter_partition_free(fit_admitter* a, int32_t p, int64_t* cpu, int64_t* mem_mib,
                                int64_t* gpu) {
    if (!a || p < 0 || p >= FIT_MAX_PARTITIONS || !cpu || !mem_mib || !gpu) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    const int rc = a->take_over();
    if (rc) return rc;
    int64_t sc = 0, sm = 0, sg = 0;  // fit_partition_free's sum, over the exact host copy
    for (int32_t x = 0; x < a->n; ++x)
        if ((a->mask[x] >> p) & 1u) {
            sc += std::max<int64_t>(a->hc[x], 0);
            sm += std::max<int64_t>(a->hm[x], 0);
            sg += std::max<int64_t>(a->hg[x], 0);
        }
    *cpu = sc, *mem_mib = sm, *gpu = sg;
    return FIT_OK;
}

int fit_admitter_confirm(fit_admitter* a, int64_t ticket) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    auto it = a->resv.find(ticket);
    if (it == a->resv.end()) return fail(FIT_E_INVAL, "fit_admitter_confirm: unknown ticket");
    if (!it->second.confirmed) {  // a repeated confirm keeps the first one's generation
        it->second.confirmed = true;
        it->second.confirm_gen = a->gen_issued;
    }
    return FIT_OK;
}

int fit_admitter_release(fit_admitter* a, int64_t ticket) {
    if (!a) return FIT_E_INVAL;
    std::lock_guard<std::mutex> g(a->ctx_m);
    auto it = a->resv.find(ticket);
    if (it == a->resv.end()) return fail(FIT_E_INVAL, "fit_admitter_release: unknown ticket");
    const Resv& r = it->second;
    if (!r.confirmed) {  // the job will not run: its demand goes back now
        const int rc = a->take_over();
        if (rc) return rc;
        for (int i = 0; i < r.k; ++i) {
            const int32_t x = r.node[i];
            if (x < 0 || x >= a->n) continue;
            a->hc[x] += r.cpu, a->hm[x] += r.mem, a->hg[x] += r.gpu;
        }
        a->engine_stale = true;
    }
    a->resv.erase(it);
    return FIT_OK;
}

int fit_admitter_script(fit_admitter* a, const int64_t* tickets, int32_t n, const char* script,
                        char* out, int32_t outlen, int32_t* pinned) {
    if (!a || !script || !out || outlen < 1 || n < 1 || !tickets)
        return fail(FIT_E_INVAL, "fit_admitter_script: bad arguments");
    if (pinned) *pinned = 0;
    std::vector<std::string_view> nm;
    std::lock_guard<std::mutex> g(a->ctx_m);
    for (int32_t i = 0; i < n; ++i)
        if (!a->resv.count(tickets[i])) return fail(FIT_E_INVAL, "fit_admitter_script: unknown ticket");
    const Resv& r = a->resv.at(tickets[0]);
    // one request of a job that is not an array job (an array's tasks share one sbatch, and a
    // single request can still be one task of `--array=0-9%1`: --nodelist would pin every task)
    bool pin = n == 1 && !r.array && r.names && r.names->pinnable;
    for (int i = 0; pin && i < r.k; ++i) {
        if (r.node[i] < 0) pin = false;  // a node left the partition since the admission
        else nm.emplace_back(r.names->name[(size_t)r.node[i]]);
    }
    if (!pin) {
        const size_t len = strlen(script);
        if ((int64_t)len + 1 > outlen) return fail(FIT_E_INVAL, "fit_admitter_script: out too small");
        memcpy(out, script, len + 1);
        return (int)len;
    }
    const int len = fitgpu::script_with_names(script, nm, out, outlen);
    if (len < 0) return fail(len, "fit_admitter_script: out too small");
    if (pinned) *pinned = 1;
    return len;
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
