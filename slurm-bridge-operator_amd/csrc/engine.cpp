// engine.cpp — host runtime of libfitgpu.so: context, node-table ingest into HBM, the
// speculative round loop, node sharding over RCCL.  DESIGN.md §3.
//
// Boundary: include/fitgpu.h.  Everything here is plain C++ over the HIP runtime; the compute
// is in fit_kernels.hip.  There is no CPU placement path: without a gfx950 device fit_create
// fails with FIT_E_NODEV.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#include <rccl/rccl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/fitgpu.h"
#include "fit_device.h"

namespace fitgpu {
hipError_t launch_scan(int blocks, hipStream_t st, const NodeRec* rec, const int32_t* jl,
                       const int32_t* jcpu, const int32_t* jmem, const int32_t* jgpu,
                       const int32_t* jwall, const uint16_t* jpart, const uint16_t* jk,
                       const CompPlan* plan, int ncomp, uint64_t* cand, uint64_t* bnd,
                       JobRec* wjob);
hipError_t launch_commit(int ncomp, int epl, size_t lds_bytes, hipStream_t st, NodeRec* rec,
                         const CompPlan* plan, const uint64_t* cand, int64_t rank_stride,
                         int nranks, const uint64_t* bnd, const JobRec* wjob, int32_t* out,
                         int kmax, CommitResult* res);
hipError_t launch_prefilter(hipStream_t st, const int32_t* jcpu, const int32_t* jmem,
                            const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart, const uint16_t* jk,
                            int32_t nj, int32_t kmax, const int32_t* ptab, int32_t np,
                            int32_t* out, int8_t* jcomp);
size_t joblists_scratch_ints(int32_t nj);
hipError_t launch_joblists(hipStream_t st, const int8_t* jcomp, int32_t nj, int ncomp,
                           int32_t* scratch, int32_t* g, int32_t* jb, int32_t* mb, int32_t* jl,
                           int32_t* jpk);
hipError_t launch_small_args(hipStream_t st, int ncomp, NodeRec* rec, const SmallComps& C, const int32_t* ptab,
                             int32_t np, const SmallBatch& B, bool has_nk, int32_t nj, int32_t kmax, int32_t* out,
                             int32_t* stat);
hipError_t launch_small(hipStream_t st, int ncomp, NodeRec* rec, const SmallComps& C,
                        const int32_t* ptab, int32_t np, const int32_t* jcpu, const int32_t* jmem,
                        const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart,
                        const uint16_t* jk, int32_t nj, int32_t kmax, int32_t* out, int32_t* stat);
hipError_t launch_gather_nodes(hipStream_t st, const int32_t* cpu, const int32_t* mem,
                               const int32_t* gpu, const int32_t* av, const uint32_t* mask,
                               const int32_t* perm, int32_t nn, NodeRec* rec);
hipError_t launch_scatter_nodes(hipStream_t st, const NodeRec* rec, int32_t nn, int32_t* cpu,
                                int32_t* mem, int32_t* gpu);
size_t engine_lds_bytes(int32_t max_component_nodes);
// demand-class engine (fit_class.hip)
size_t class_lds_bytes(int32_t max_component_nodes);
int class_max();
int class_table_slots();
size_t class_slot_bytes();
int class_max_nodes();
hipError_t launch_classify(hipStream_t st, const int8_t* jcomp, const int32_t* jcpu, const int32_t* jmem,
                           const int32_t* jgpu, const uint16_t* jpart, int32_t nj, void* tab, int4* dem,
                           int32_t* ncls, int16_t* jcls);
hipError_t launch_class(hipStream_t st, int ncomp, size_t lds, NodeRec* rec, const int32_t* nbv, uint32_t owned,
                        const int32_t* jb, const int32_t* jl, const int32_t* jwall, const uint16_t* jk,
                        const int16_t* jcls, const int4* dem, const int32_t* ncls, int32_t kmax, int32_t* out,
                        CompOut* co, unsigned* err);
hipError_t launch_class_out(hipStream_t st, int32_t* out, int64_t n, const NodeRec* rec);
size_t engine_ctl_bytes();
size_t engine_ctl_error_offset();
size_t engine_ctl_trip_offset();
size_t engine_ring_bytes();
size_t engine_ring_tasks();
int engine_ring_groups();
// components sharing the fullest task ring (fit_engine_ctl.h: component c goes to ring
// c % min(groups, nc))
inline int64_t ring_comps(int nc) {
    const int g = std::max(1, std::min(engine_ring_groups(), nc));
    return (nc + g - 1) / g;
}
int engine_blocks_per_cu(size_t lds);
hipError_t launch_engine(int blocks, size_t lds, hipStream_t st, void* ctl, void* ring,
                         const void* cs, void* co, CompPlan* plans, int ncomp, NodeRec* rec,
                         const int32_t* jl, const int32_t* jcpu, const int32_t* jmem,
                         const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart,
                         const uint16_t* jk, uint64_t* cand, uint64_t* bnd, JobRec* wjob,
                         int32_t* out, int kmax, int64_t* wbusy, const int32_t* jpk, unsigned wd);
// time-windowed backfill (fit_timeline.hip)
hipError_t launch_build_tl(hipStream_t st, const int32_t* cpu, const int32_t* mem,
                           const int32_t* gpu, const int32_t* av, const uint32_t* mask,
                           const int32_t* perm, int32_t nn, int32_t H, int32_t slot_min,
                           const int32_t* off, const int32_t* rs, const int32_t* rc,
                           const int32_t* rm, const int32_t* rg, Seg* slab, TlHdr* hdr,
                           uint32_t* err);
hipError_t launch_scan_tl(int blocks, hipStream_t st, const Seg* slab, const TlHdr* hdr,
                          const int32_t* jl, const int32_t* jcpu, const int32_t* jmem,
                          const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart,
                          const CompPlan* plan, int ncomp, uint64_t* cand, uint64_t* bnd,
                          JobRec* wjob, int32_t H, int32_t slot_min);
size_t commit_tl_lds_bytes(int32_t max_component_nodes);
int commit_tl_runs(int32_t max_component_nodes);
hipError_t launch_commit_tl(int ncomp, int epl, size_t lds, hipStream_t st, Seg* slab,
                            TlHdr* hdr, const CompPlan* plan, const uint64_t* cand,
                            int64_t rank_stride, int nranks, const uint64_t* bnd,
                            const JobRec* wjob, const int32_t* perm, int32_t* out, int32_t* outs,
                            CommitResult* res, int32_t H, int32_t R);
int engine_tl_runs(int32_t max_component_nodes);
size_t engine_tl_lds_bytes(int32_t max_component_nodes);
int engine_tl_blocks_per_cu(size_t lds, int mode);
size_t engine_tl_scan_lds_bytes();
hipError_t launch_engine_tl(int blocks, size_t lds, hipStream_t st, void* ctl, void* ring,
                            const void* cs, void* co, CompPlan* plans, int ncomp, Seg* slab,
                            TlHdr* hdr, const int32_t* jl, const int32_t* jcpu,
                            const int32_t* jmem, const int32_t* jgpu, const int32_t* jwall,
                            const uint16_t* jpart, uint64_t* cand, uint64_t* bnd, JobRec* wjob,
                            const int32_t* perm, int32_t* out, int32_t* outs, int32_t H,
                            int32_t slot_min, int32_t R, int64_t* wbusy, int mode,
                            unsigned* resident, unsigned wd);
hipError_t launch_expand_tl(hipStream_t st, const int32_t* perm, const Seg* slab,
                            const TlHdr* hdr, int32_t nn, int32_t H, int32_t* oc, int32_t* om,
                            int32_t* og);
}  // namespace fitgpu

using namespace fitgpu;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(FIT_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                        __FILE__, __LINE__);                                                \
    } while (0)

#define NCCL_TRY(expr)                                                                      \
    do {                                                                                    \
        ncclResult_t r_ = (expr);                                                           \
        if (r_ != ncclSuccess)                                                              \
            return fail(FIT_E_RCCL, "%s failed: %s", #expr, ncclGetErrorString(r_));        \
    } while (0)

// device buffer that only grows
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 64);
        if (hipMalloc(&p, want * sizeof(T)) != hipSuccess) {
            p = nullptr;
            return fail(FIT_E_OOM, "hipMalloc(%zu bytes) failed", want * sizeof(T));
        }
        cap = want;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

template <class T>
struct HBuf {  // pinned host buffer
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 64);
        if (hipHostMalloc(&p, want * sizeof(T), hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return fail(FIT_E_OOM, "hipHostMalloc(%zu bytes) failed", want * sizeof(T));
        }
        cap = want;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

int find_root(int* par, int x) {
    while (par[x] != x) x = par[x] = par[par[x]];
    return x;
}

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// ---- per-device arbitration of persistent launches (round 5) --------------------------------
// A persistent launch (k_engine / k_engine_tl) needs its committer blocks resident while its scan
// workers spin on the task ring.  Alone on the GPU every block of its grid is resident (the grid
// is sized by occupancy).  Two side by side are not: the dispatcher hands each grid's blocks to
// the 8 XCDs in block order, so launch A's committer on XCD k can queue behind launch B's blocks
// while A's workers fill the other XCDs waiting for it — and B's committer waits behind A's
// workers (GPUTEST_r04: the watchdog tripped with three contexts on one GPU).  One virtual kubelet
// per partition (pkg/configurator/configurator.go:151-171) means several contexts per GPU, in
// several processes, so every persistent launch on a device is serialised: a process-wide mutex
// per device, then an exclusive flock on <FIT_LOCK_DIR or /tmp>/fitgpu-<PCI bus id>.lock for the
// other processes (flock: released by the kernel if the holder dies).  Held from the launch to
// the stream synchronisation that ends it.  The host-driven rounds (k_scan / k_commit, no
// cross-block waits) need no arbitration.
struct DevArb {
    std::mutex mu;
    int fd = -1;
    std::string path;
};

// The lock directory.  The lock only serialises launches whose processes see the same file, and
// the configurator runs every virtual kubelet as its own pod (configurator.go:188-293) with a
// private /tmp, so the default is a HOST path the VK pod template mounts:
//   FIT_LOCK_DIR if set (an explicit choice: used as given, a failure to open the file is an error);
//   else FIT_LOCK_DIR_DEFAULT when it is a directory (the hostPath volume, DirectoryOrCreate);
//   else /tmp — shared only inside one pod: returned as 1 so the caller can warn (fit_lock_dir).
constexpr const char* FIT_LOCK_DIR_DEFAULT = "/var/run/fitgpu";
int resolve_lock_dir(std::string& dir) {
    const char* e = getenv("FIT_LOCK_DIR");
    if (e && *e) {
        dir = e;
        return 0;
    }
    struct stat sb;
    if (stat(FIT_LOCK_DIR_DEFAULT, &sb) == 0 && S_ISDIR(sb.st_mode)) {
        dir = FIT_LOCK_DIR_DEFAULT;
        return 0;
    }
    dir = "/tmp";
    return 1;
}

DevArb* dev_arb(int device, std::string& err) {
    static std::mutex m;
    static std::map<int, DevArb*> tab;
    std::lock_guard<std::mutex> g(m);
    DevArb*& a = tab[device];
    if (!a) a = new DevArb();  // one per device for the process lifetime
    if (a->fd < 0) {
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) snprintf(bus, sizeof bus, "dev%d", device);
        for (char* q = bus; *q; ++q)
            if (*q == ':' || *q == '/') *q = '_';
        std::string dir;
        (void)resolve_lock_dir(dir);
        a->path = dir + "/fitgpu-" + bus + ".lock";
        // every user's engines share the file: created 0666 (fchmod, not the process-wide umask);
        // an existing file of another user in a sticky /tmp may refuse an O_CREAT open
        // (fs.protected_regular), so it is then opened read-only — flock needs no write access
        a->fd = open(a->path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
        if (a->fd >= 0) (void)fchmod(a->fd, 0666);  // fails harmlessly on another user's file
        else a->fd = open(a->path.c_str(), O_RDONLY | O_CLOEXEC);
        if (a->fd < 0) {
            err = a->path + ": " + strerror(errno);
            return nullptr;
        }
    }
    return a;
}

struct ArbGuard {
    DevArb* a = nullptr;
    double waited_ms = 0;
    int take(int device) {
        const double t0 = now_ms();
        std::string err;
        DevArb* d = dev_arb(device, err);
        if (!d) return fail(FIT_E_STATE, "device lock %s (set FIT_LOCK_DIR to a writable directory)", err.c_str());
        d->mu.lock();
        int r;
        do r = flock(d->fd, LOCK_EX);
        while (r != 0 && errno == EINTR);
        if (r != 0) {
            d->mu.unlock();
            return fail(FIT_E_STATE, "flock %s: %s", d->path.c_str(), strerror(errno));
        }
        a = d;
        waited_ms = now_ms() - t0;
        return 0;
    }
    ~ArbGuard() {
        if (!a) return;
        (void)flock(a->fd, LOCK_UN);
        a->mu.unlock();
    }
};

}  // namespace

struct fit_ctx {
    int device = 0;
    int rank = 0, world = 1;
    int shard_mode = FIT_SHARD_AUTO;
    ncclComm_t comm = nullptr;
    fit_exchange_fn xchg = nullptr;  // host exchange instead of RCCL (tests, custom transport)
    void* xchg_user = nullptr;
    HBuf<uint8_t> h_x;               // staging for the host exchange
    DBuf<uint64_t> xcount;           // per-rank counters (component-sharded stats)
    bool force_coll = false;         // FIT_FLAG_COLLECTIVES: sharded path + exchange at world 1
    bool collective() const { return world > 1 || force_coll; }
    bool persistent = true;          // one-launch work-queue engine (FIT_ENGINE=rounds: host loop)
    // placements of at most this many jobs (after the partition-limit prefilter) run the
    // host-driven rounds instead of a whole-chip persistent grid: an admission batch of a few
    // hundred pods is one or two rounds of a few tiles (FIT_SMALL_BATCH)
    int32_t small_batch = 2048;
    // placements of at most this many jobs run k_small: one launch, the jobs one at a time against
    // every node of their component, no rounds and one host synchronisation (FIT_SMALL_DIRECT)
    // 128: where k_small stops beating the host-driven rounds on one VK's one-partition table
    // (tools/direct_vs_rounds.py, profiles/r06q_direct_vs_rounds.txt: 184 vs 178 µs at 128 jobs;
    // the 16-component C3 table breaks even near 1,024)
    int32_t small_direct = 128;
    // a batch of <= SMALL_ARGJ jobs from host memory rides in k_small's kernel arguments (no copy to
    // the device), and the call spins on the batch's completion event instead of sleeping in a
    // stream synchronisation (FIT_SMALL_ARGS=0 / FIT_SYNC_SPIN=0: A/B switches)
    bool small_args = true, sync_spin = true;
    // the demand-class engine (fit_class.hip): 0 off (FIT_CLASS=0, and FIT_ENGINE=persistent|rounds|
    // direct), 1 for placements the persistent engine would run (FIT_CLASS=1), 2 at every size
    // (FIT_ENGINE=class), 3 (the default) for those of them whose live jobs are at least half
    // multi-node; used when every component is one partition, fits LDS and has <= class_max()
    // demand classes
    int cls_mode = 3;
    int32_t last_multi = 0;          // multi-node jobs of the last job lists (build_job_lists)
    bool cls_nodes_ok = false;       // node table: single-partition components that fit LDS
    int32_t cls_maxn = 0;            // largest component (nodes)
    DBuf<int16_t> jcls;
    DBuf<uint8_t> cls_tab;
    DBuf<int4> cls_dem;
    DBuf<int32_t> cls_n;
    DBuf<unsigned> cls_err;
    HBuf<int32_t> h_cls_n;
    HBuf<unsigned> h_cls_err;
    DBuf<int32_t> small_placed;
    HBuf<int32_t> h_small;
    DBuf<uint8_t> jpack;    // fit_place's job columns of a small batch, packed: one H2D copy
    HBuf<uint8_t> h_jpack;
    int cus = 256;
    DBuf<uint8_t> ectl, ering;
    DBuf<CompState> ecs;
    DBuf<CompOut> eco;
    DBuf<int64_t> ebusy;
    HBuf<CompState> h_ecs;
    HBuf<CompOut> h_eco;
    HBuf<int64_t> h_ebusy;
    HBuf<uint32_t> h_err;
    HBuf<TripRec> h_trip;
    DBuf<NodeRec> rec_bak;           // node rows before a persistent launch (restored on a trip)
    unsigned wd_ticks = 1000000000u; // watchdog: realtime ticks (10 ns) a wait may last (10 s)
    HBuf<uint64_t> h_count;
    hipStream_t st = nullptr;
    hipEvent_t ev[6] = {};
    // FIT_TL_SPLIT: the backfill engine's scan workers as a second, concurrent launch
    hipStream_t st2 = nullptr;
    hipEvent_t ev_join = nullptr;
    unsigned* resident = nullptr;  // host-mapped: committer blocks running
    int wmin = 256, wmax = 8192;

    // node table
    int32_t n = 0;           // rows in caller order
    int32_t nn = 0;          // rows in components (mask != 0)
    int ncomp = 0;
    int comp_of_part[32];
    std::vector<int32_t> nb;  // ncomp + 1 component offsets (positions)
    DBuf<NodeRec> rec;
    DBuf<int32_t> col_cpu, col_mem, col_gpu, col_av, perm;
    DBuf<uint32_t> col_mask;
    DBuf<int32_t> rb_cpu, rb_mem, rb_gpu;  // fit_read_nodes scratch (col_* stay the loaded table)
    std::vector<uint32_t> h_mask;
    bool have_nodes = false;
    int64_t loads = 0;        // successful node-table loads (admit.cpp notices a direct load)

    // partitions: [max_time | max_cpus | max_mem | comp] × 32
    int32_t np = 0;
    int32_t ptab[128];
    DBuf<int32_t> d_ptab;

    // per-call scratch
    DBuf<int32_t> jcpu, jmem, jgpu, jwall, out, jl, jpk;
    DBuf<uint16_t> jpart, jk;
    DBuf<int8_t> jcomp;
    DBuf<uint64_t> cand, bnd;
    DBuf<JobRec> wjob;
    DBuf<CompPlan> plan;
    DBuf<CommitResult> res;
    HBuf<CompPlan> h_plan;
    HBuf<CommitResult> h_res;
    DBuf<int32_t> jls;    // device job-list scratch (block counts, counters, offsets)
    HBuf<int32_t> h_jls;

    // time-windowed backfill: per-node run lists, built from the node
    // table + release events by fit_load_timeline
    int32_t tl_slots = 0, tl_slot_min = 0;
    bool have_tl = false;
    DBuf<Seg> slab;
    DBuf<TlHdr> tlhdr;
    DBuf<int32_t> outs, rel_off, rel_slot, rel_cpu, rel_mem, rel_gpu;
    DBuf<uint32_t> tl_err;
    HBuf<uint32_t> h_tl_err;

    ~fit_ctx() {
        for (auto* b : {&col_cpu, &col_mem, &col_gpu, &col_av, &perm, &jcpu, &jmem, &jgpu,
                        &jwall, &out, &jl, &jpk, &rb_cpu, &rb_mem, &rb_gpu})
            b->release();
        rec.release();
        tlhdr.release();
        for (auto* b : {&outs, &rel_off, &rel_slot, &rel_cpu, &rel_mem, &rel_gpu})
            b->release();
        slab.release();
        tl_err.release();
        h_tl_err.release();
        col_mask.release();
        d_ptab.release();
        jpart.release();
        jk.release();
        jcomp.release();
        cand.release();
        bnd.release();
        wjob.release();
        plan.release();
        res.release();
        h_plan.release();
        h_res.release();
        jls.release();
        h_jls.release();
        jcls.release();
        cls_tab.release();
        cls_dem.release();
        cls_n.release();
        cls_err.release();
        h_cls_n.release();
        h_cls_err.release();
        small_placed.release();
        h_small.release();
        jpack.release();
        h_jpack.release();
        h_x.release();
        xcount.release();
        h_count.release();
        ectl.release();
        ering.release();
        ecs.release();
        eco.release();
        ebusy.release();
        h_ecs.release();
        h_eco.release();
        h_ebusy.release();
        h_err.release();
        h_trip.release();
        rec_bak.release();
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (resident) (void)hipHostFree(resident);
        if (st2) (void)hipStreamDestroy(st2);
        if (st) (void)hipStreamDestroy(st);
        if (comm) (void)ncclCommDestroy(comm);
    }
};

namespace {

int build_ptab(fit_ctx* c) {
    for (int p = 0; p < 32; ++p) c->ptab[96 + p] = c->comp_of_part[p];
    if (c->d_ptab.ensure(128)) return FIT_E_OOM;
    HIP_TRY(hipMemcpyAsync(c->d_ptab.p, c->ptab, sizeof c->ptab, hipMemcpyHostToDevice, c->st));
    return 0;
}

// Components = partitions connected through nodes that belong to several of them; jobs of
// different components never compete for a node, so each is an independent sequence
// (DESIGN.md §3.1).  Nodes are laid out component by component, in id order inside each.
int load_nodes_common(fit_ctx* c, int32_t n) {
    int par[32];
    for (int i = 0; i < 32; ++i) par[i] = i;
    bool used[32] = {false};
    for (int32_t x = 0; x < n; ++x) {
        uint32_t m = c->h_mask[x];
        if (!m) continue;
        int lo = __builtin_ctz(m);
        for (uint32_t r = m; r; r &= r - 1) {
            int b = __builtin_ctz(r);
            used[b] = true;
            int ra = find_root(par, lo), rb = find_root(par, b);
            if (ra != rb) par[std::max(ra, rb)] = std::min(ra, rb);
        }
    }
    int root_comp[32];
    for (int i = 0; i < 32; ++i) root_comp[i] = -1;
    c->ncomp = 0;
    for (int p = 0; p < 32; ++p) {
        c->comp_of_part[p] = -1;
        if (!used[p]) continue;
        int r = find_root(par, p);
        if (root_comp[r] < 0) root_comp[r] = c->ncomp++;
        c->comp_of_part[p] = root_comp[r];
    }
    c->nb.assign(c->ncomp + 1, 0);
    for (int32_t x = 0; x < n; ++x)
        if (c->h_mask[x]) c->nb[c->comp_of_part[__builtin_ctz(c->h_mask[x])] + 1]++;
    for (int k = 0; k < c->ncomp; ++k) {
        if (c->nb[k + 1] > MAX_COMPONENT_NODES)
            return fail(FIT_E_INVAL, "partition component %d has %d nodes (limit %d)", k,
                        c->nb[k + 1], MAX_COMPONENT_NODES);
        c->nb[k + 1] += c->nb[k];
    }
    c->nn = c->nb[c->ncomp];
    {  // the class engine: one partition per component (the part test is then always true) and
       // the component's rows in one workgroup's LDS
        int parts_of[32] = {0};
        for (int p = 0; p < 32; ++p)
            if (c->comp_of_part[p] >= 0) ++parts_of[c->comp_of_part[p]];
        c->cls_nodes_ok = c->ncomp > 0 && c->ncomp <= 32;
        c->cls_maxn = 0;
        for (int k = 0; k < c->ncomp; ++k) {
            const int32_t nk = c->nb[k + 1] - c->nb[k];
            c->cls_maxn = std::max(c->cls_maxn, nk);
            if (parts_of[k] != 1) c->cls_nodes_ok = false;
        }
        if (c->cls_maxn > class_max_nodes() || class_lds_bytes(c->cls_maxn) > 160 * 1024)
            c->cls_nodes_ok = false;
    }
    std::vector<int32_t> fill(c->nb.begin(), c->nb.end() - 1), perm(std::max(c->nn, 1));
    for (int32_t x = 0; x < n; ++x)
        if (c->h_mask[x]) perm[fill[c->comp_of_part[__builtin_ctz(c->h_mask[x])]]++] = x;
    if (c->perm.ensure(std::max(c->nn, 1)) || c->rec.ensure(std::max(c->nn, 1))) return FIT_E_OOM;
    HIP_TRY(hipMemcpyAsync(c->perm.p, perm.data(), sizeof(int32_t) * c->nn, hipMemcpyHostToDevice,
                           c->st));
    HIP_TRY(launch_gather_nodes(c->st, c->col_cpu.p, c->col_mem.p, c->col_gpu.p, c->col_av.p,
                                c->col_mask.p, c->perm.p, c->nn, c->rec.p));
    int rc = build_ptab(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->st));
    c->n = n;
    c->have_nodes = true;
    c->have_tl = false;  // a timeline belongs to the node table it was built from
    ++c->loads;
    return 0;
}

int alloc_cols(fit_ctx* c, int32_t n) {
    size_t m = std::max<int32_t>(n, 1);
    if (c->col_cpu.ensure(m) || c->col_mem.ensure(m) || c->col_gpu.ensure(m) ||
        c->col_av.ensure(m) || c->col_mask.ensure(m))
        return FIT_E_OOM;
    return 0;
}

// ------------------------------------------------------------------------ exchange
// In-place collectives on device buffers: RCCL over xGMI, or the caller's host exchange.
int xchg(fit_ctx* c, int op, void* dbuf, int64_t count) {
    if (!c->collective() || count == 0) return 0;
    if (!c->xchg) {
        switch (op) {
            case FIT_XCHG_ALLGATHER_U64: {
                uint64_t* b = static_cast<uint64_t*>(dbuf);
                NCCL_TRY(ncclAllGather(b + (size_t)c->rank * count, b, count, ncclUint64, c->comm,
                                       c->st));
                return 0;
            }
            case FIT_XCHG_MIN_U64:
                NCCL_TRY(ncclAllReduce(dbuf, dbuf, count, ncclUint64, ncclMin, c->comm, c->st));
                return 0;
            case FIT_XCHG_MAX_I32:
                NCCL_TRY(ncclAllReduce(dbuf, dbuf, count, ncclInt32, ncclMax, c->comm, c->st));
                return 0;
            case FIT_XCHG_MIN_I32:
                NCCL_TRY(ncclAllReduce(dbuf, dbuf, count, ncclInt32, ncclMin, c->comm, c->st));
                return 0;
        }
        return fail(FIT_E_INVAL, "exchange op %d", op);
    }
    const size_t elem = (op == FIT_XCHG_ALLGATHER_U64 || op == FIT_XCHG_MIN_U64) ? 8 : 4;
    const size_t bytes = elem * (size_t)count * (op == FIT_XCHG_ALLGATHER_U64 ? c->world : 1);
    if (c->h_x.ensure(bytes)) return FIT_E_OOM;
    HIP_TRY(hipMemcpyAsync(c->h_x.p, dbuf, bytes, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    if (c->xchg(c->xchg_user, op, c->h_x.p, count) != 0)
        return fail(FIT_E_RCCL, "host exchange op %d failed", op);
    HIP_TRY(hipMemcpyAsync(dbuf, c->h_x.p, bytes, hipMemcpyHostToDevice, c->st));
    return 0;
}

// ------------------------------------------------------------- persistent engine path
const char* trip_site_name(unsigned s) {
    switch (s) {
        case TRIP_WORKER_RING: return "scan worker waiting for a task";
        case TRIP_ROUND_START: return "committer waiting for the round before last";
        case TRIP_HELPER_TILE: return "commit helper waiting for a scan tile";
        case TRIP_HELPER_SNAP: return "commit helper waiting for the decider";
        case TRIP_DECIDER_REC: return "decider waiting for a helper record";
        case TRIP_SINGLE_TILE: return "single-wave commit waiting for a scan tile";
        case TRIP_NO_PROGRESS: return "round resolved no job";
        case TRIP_NO_KERNEL: return "no scan kernel for the key count";
        default: return "unknown";
    }
}

// The launch's error word and first trip record (read back with it): FIT_E_HIP with every field.
int trip_error(fit_ctx* c, const char* engine) {
    const TripRec& t = *c->h_trip.p;
    return fail(FIT_E_HIP,
                "%s watchdog tripped (code %u): site %u (%s), component %u, round %u, arg %u, "
                "block %u, q_head %u, q_tail %u, pubt %u, tdone %u / need %u, waited %.3f ms, "
                "%.3f ms into the launch (deadline %.3f ms)",
                engine, c->h_err.p[0], t.site, trip_site_name(t.site), t.comp, t.round, t.arg,
                t.block, t.q_head, t.q_tail, t.pubt, t.tdone, t.need, t.waited / 1e5, t.when / 1e5,
                c->wd_ticks / 1e5);
}
// All rounds of all owned components in one launch (fit_persistent.hip).
int run_persistent(fit_ctx* c, const std::vector<int32_t>& jb, const std::vector<char>& owned,
                   const int32_t* cpu, const int32_t* mem, const int32_t* gpu, const int32_t* wall,
                   const uint16_t* part, const uint16_t* nk, int32_t* out, int32_t kmax,
                   fit_stats& S) {
    const int C = c->ncomp;
    hipStream_t st = c->st;
    std::vector<int> comps;
    int32_t maxnodes = 0;
    for (int k = 0; k < C; ++k)
        if (owned[k] && jb[k + 1] > jb[k]) {
            comps.push_back(k);
            maxnodes = std::max(maxnodes, c->nb[k + 1] - c->nb[k]);
        }
    const int nc = (int)comps.size();
    if (nc == 0) return 0;
    const int64_t wcap = std::min(c->wmax, 8192);  // k_engine's per-tile counters: 128 job tiles
    const int64_t per_comp_cand = wcap * MAX_SLICES * KS;
    // keys per block-slice: KS, halved (slices doubled, the same MAX_SLICES * KS candidates per
    // job) while a wave's sub-slice would exceed sub_target nodes — a round's first job tile, which
    // the commit waits for, then spreads over more blocks.  C3o (one 100k-node component): KS 16
    // 552 ms, 8 471 ms, 4 441 ms, 2 480 ms (the bound B, a minimum over more slices of fewer keys,
    // turns tight: 891 rescans); C3 / C2 components stay at KS (sub-slices of 98 / 64 nodes).
    int sub_target = 256, ks_min = 4;
    if (const char* e = getenv("FIT_SUB_TARGET")) sub_target = std::max(MIN_SUB, atoi(e));
    if (const char* e = getenv("FIT_KS_MIN")) ks_min = std::max(2, std::min(KS, atoi(e)));
    // a multi-node job needs k keys <= B on one slice: the slice that sets B has ks of them, all
    // clean when the job opens a round, so ks >= kmax keeps every round's first job resolvable
    while (ks_min < kmax) ks_min *= 2;
    // two sets of per-round buffers (plans, candidates, bounds, job rows) by round parity
    // (fit_engine_ctl.h): a round starts while the previous round's last tiles are still scanned
    if (c->ecs.ensure(nc) || c->eco.ensure(nc) || c->h_ecs.ensure(nc) || c->h_eco.ensure(nc) ||
        c->plan.ensure(2 * nc) ||
        c->cand.ensure((size_t)2 * nc * per_comp_cand + (size_t)2 * nc * PAIR_AREA) ||
        c->bnd.ensure((size_t)2 * nc * wcap) || c->wjob.ensure((size_t)2 * nc * wcap) ||
        c->ectl.ensure(engine_ctl_bytes()) || c->ering.ensure(engine_ring_bytes()) ||
        c->h_err.ensure(4))
        return FIT_E_OOM;
    if ((int64_t)2 * nc * per_comp_cand + (int64_t)2 * nc * PAIR_AREA > INT32_MAX)
        return fail(FIT_E_INVAL, "candidate buffer exceeds 2^31 entries (%d components)", nc);
    for (int i = 0; i < nc; ++i) {
        const int k = comps[i];
        CompState& s = c->h_ecs.p[i];
        s.nb = s.sb = c->nb[k];
        s.ne = s.se = c->nb[k + 1];
        const int32_t len = s.ne - s.nb;
        for (s.ks = KS;; s.ks /= 2) {
            const int slices = MAX_SLICES * KS / s.ks;
            s.sub = std::max(MIN_SUB, (len + SCAN_WAVES * slices - 1) / (SCAN_WAVES * slices));
            s.nslice = std::max(1, (len + SCAN_WAVES * s.sub - 1) / (SCAN_WAVES * s.sub));
            if (s.sub <= sub_target || s.ks / 2 < ks_min) break;
        }
        s.jstart = jb[k];
        s.jend = jb[k + 1];
        s.cand_off = (int64_t)i * per_comp_cand;
        s.slot0 = (int32_t)(i * wcap);
        s.cand_alt = (int64_t)(nc + i) * per_comp_cand;
        s.slot_alt = (int32_t)((nc + i) * wcap);
        s.pair_off = (int32_t)(2 * nc * per_comp_cand + (int64_t)2 * i * PAIR_AREA);
        s.wmin = std::min(c->wmin, (int)wcap);
        s.wmax = (int32_t)wcap;
    }
    // task ring: a committer publishes a round only after all tiles of the round before last are
    // done, so at most 2 * nc * job tiles * slices tiles are outstanding; the ring must hold them
    // all (a granule overwritten before its worker read it would be lost)
    int32_t max_slices = 1;
    for (int i = 0; i < nc; ++i) max_slices = std::max(max_slices, c->h_ecs.p[i].nslice);
    // (+ one tile: a round's first tile may be scanned as twice the slices, K_T0PAIR)
    if ((int64_t)2 * ring_comps(nc) * ((wcap + SCAN_JOBS - 1) / SCAN_JOBS + 1) * max_slices >
        (int64_t)engine_ring_tasks())
        return fail(FIT_E_INVAL, "task ring too small: %d components x %lld tiles x %d slices",
                    nc, (long long)((wcap + SCAN_JOBS - 1) / SCAN_JOBS), max_slices);
    size_t lds = engine_lds_bytes(maxnodes);
    // experiment knob: a larger LDS request caps the blocks per CU (e.g. > 80 KB: one per CU)
    if (const char* e = getenv("FIT_ENGINE_LDS_MIN")) lds = std::max(lds, (size_t)atol(e));
    int per_cu = engine_blocks_per_cu(lds);
    if (per_cu <= 0) return fail(FIT_E_HIP, "k_engine does not fit on a CU (lds %zu)", lds);
    // Only the committers (blocks [0, nc), dispatched first) must be co-resident: a worker block
    // that is not yet resident has claimed no task, so nobody waits on it.  One block per CU:
    // the scan workers are mostly idle already, and a second block on a committer's CU slows
    // the serial commit chain (measured: 2/CU → commit +3%, no scan gain).
    int workers = std::max(8, std::max(1, per_cu - 1) * c->cus - nc);
    if (const char* e = getenv("FIT_WORKERS")) workers = std::max(1, atoi(e));
    if (c->ebusy.ensure(2 * workers) || c->h_ebusy.ensure(2 * workers) || c->h_trip.ensure(1) ||
        c->rec_bak.ensure(std::max(c->nn, 1)))
        return FIT_E_OOM;
    HIP_TRY(hipMemcpyAsync(c->ecs.p, c->h_ecs.p, sizeof(CompState) * nc, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(c->ectl.p, 0, engine_ctl_bytes(), st));
    HIP_TRY(hipMemsetAsync(c->ering.p, 0, engine_ring_bytes(), st));
    // every bound KEY_INF: a round resets only the bounds its buffer set's last round used
    HIP_TRY(hipMemsetAsync(c->bnd.p, 0xff, sizeof(uint64_t) * 2 * nc * wcap, st));
    // the node rows as they were: a trip leaves them partly committed, and the context must stay
    // usable after FIT_E_HIP (restored below)
    static const bool no_backup = getenv("FIT_REC_BACKUP") && atoi(getenv("FIT_REC_BACKUP")) == 0;  // A/B only
    if (!no_backup)
        HIP_TRY(hipMemcpyAsync(c->rec_bak.p, c->rec.p, sizeof(NodeRec) * c->nn, hipMemcpyDeviceToDevice, st));
    {
        ArbGuard arb;  // one persistent launch per device at a time (see DevArb)
        int rc = arb.take(c->device);
        if (rc) return rc;
        S.ms_arb_wait = arb.waited_ms;
        HIP_TRY(hipEventRecord(c->ev[0], st));
        HIP_TRY(launch_engine(nc + workers, lds, st, c->ectl.p, c->ering.p, c->ecs.p, c->eco.p,
                              c->plan.p, nc, c->rec.p, c->jl.p, cpu, mem, gpu, wall, part, nk,
                              c->cand.p, c->bnd.p, c->wjob.p, out, kmax, c->ebusy.p, c->jpk.p,
                              c->wd_ticks));
        HIP_TRY(hipEventRecord(c->ev[1], st));
        HIP_TRY(hipMemcpyAsync(c->h_eco.p, c->eco.p, sizeof(CompOut) * nc, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(c->h_ebusy.p, c->ebusy.p, sizeof(int64_t) * 2 * workers,
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(c->h_err.p, c->ectl.p + engine_ctl_error_offset(), 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(c->h_trip.p, c->ectl.p + engine_ctl_trip_offset(), sizeof(TripRec),
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (c->h_err.p[0]) {
        const int rc = trip_error(c, "placement engine");
        if (no_backup) {  // no copy was taken: the rows are partly committed, drop the table
            c->have_nodes = c->have_tl = false;
            return rc;
        }
        HIP_TRY(hipMemcpyAsync(c->rec.p, c->rec_bak.p, sizeof(NodeRec) * c->nn, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        return rc;
    }
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    S.ms_device += ms;
    int64_t busy = 0;
    // per worker {busy ticks, evaluations scanned}: tiles of a finished round are dropped, so
    // the performed evaluations are counted where they happen
    for (int i = 0; i < workers; ++i) {
        busy += c->h_ebusy.p[2 * i];
        S.evals += c->h_ebusy.p[2 * i + 1];
    }
    S.ms_scan += busy / 1e5 / workers;  // average worker busy time (100 MHz ticks)
    double commit_max = 0;
    for (int i = 0; i < nc; ++i) {
        const CompOut& o = c->h_eco.p[i];
        const int k = comps[i];
        if (o.done_jobs != jb[k + 1] - jb[k])
            return fail(FIT_E_HIP, "component %d resolved %lld of %d jobs", k, (long long)o.done_jobs,
                        jb[k + 1] - jb[k]);
        S.placed += o.placed;
        S.rounds = std::max<int64_t>(S.rounds, o.rounds);
        S.stops_rescan += o.stops_rescan;
        S.stops_dirty += o.stops_dirty;
        commit_max = std::max(commit_max, o.t_commit / 1e5);
    }
    S.ms_commit += commit_max;
    return 0;
}

// The demand-class engine (fit_class.hip): one workgroup per component, no
// cross-block waits (so no launch arbitration), then the positions it wrote become node ids.
int run_class(fit_ctx* c, int32_t J, const std::vector<int32_t>& jb, const std::vector<char>& owned,
              const int32_t* wall, const uint16_t* nk, int32_t* out, int32_t kmax, fit_stats& S) {
    const int C = c->ncomp;
    hipStream_t st = c->st;
    if (c->eco.ensure(C) || c->h_eco.ensure(C) || c->cls_err.ensure(1) || c->h_cls_err.ensure(1) ||
        c->rec_bak.ensure(std::max(c->nn, 1)))
        return FIT_E_OOM;
    int32_t* jbd = c->jls.p + joblists_scratch_ints(J) + 2;
    HIP_TRY(hipMemsetAsync(c->cls_err.p, 0, sizeof(unsigned), st));
    HIP_TRY(hipMemcpyAsync(c->rec_bak.p, c->rec.p, sizeof(NodeRec) * c->nn, hipMemcpyDeviceToDevice, st));
    const size_t lds = class_lds_bytes(c->cls_maxn);
    HIP_TRY(hipEventRecord(c->ev[0], st));
    uint32_t own = 0;  // components this rank places (component sharding; all at world 1)
    for (int k = 0; k < C; ++k)
        if (owned[k]) own |= 1u << k;
    HIP_TRY(launch_class(st, C, lds, c->rec.p, c->nb.data(), own, jbd, c->jl.p, wall, nk, c->jcls.p,
                         c->cls_dem.p, c->cls_n.p, kmax, out, c->eco.p, c->cls_err.p));
    HIP_TRY(hipEventRecord(c->ev[1], st));
    HIP_TRY(launch_class_out(st, out, (int64_t)J * kmax, c->rec.p));
    HIP_TRY(hipMemcpyAsync(c->h_eco.p, c->eco.p, sizeof(CompOut) * C, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_cls_err.p, c->cls_err.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c->h_cls_err.p[0]) {
        HIP_TRY(hipMemcpyAsync(c->rec.p, c->rec_bak.p, sizeof(NodeRec) * c->nn, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        return fail(FIT_E_HIP, "class engine: an in-block wait exceeded its bound (error %u)", c->h_cls_err.p[0]);
    }
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    S.ms_device += ms;
    double commit_max = 0;
    for (int k = 0; k < C; ++k) {
        if (!owned[k]) continue;
        const CompOut& o = c->h_eco.p[k];
        if (o.done_jobs != jb[k + 1] - jb[k])
            return fail(FIT_E_HIP, "component %d resolved %lld of %d jobs", k, (long long)o.done_jobs,
                        jb[k + 1] - jb[k]);
        S.placed += o.placed;
        S.evals += o.evals;
        S.rounds = std::max<int64_t>(S.rounds, o.rounds);   // set refills (longest component)
        S.stops_rescan += o.stops_rescan;                   // exact-scan resolutions
        S.stops_dirty += o.stops_dirty;
        commit_max = std::max(commit_max, o.t_commit / 1e5);
    }
    S.ms_commit += commit_max;
    S.engine = 3;
    return 0;
}

// Per-component job lists in priority order (stable), built on the device from the prefilter's
// component ids (launch_joblists: counting sort by component); only the component offsets and
// two counters come back to the host.  jb[k] .. jb[k+1] = component k's list range.
// With `classify` the demand classes of every component's jobs are counted in the same
// synchronisation (k_classify, fit_class.hip); *cls_ok says whether every component has at most
// class_max() of them.
int build_job_lists(fit_ctx* c, int32_t J, fit_stats& S, std::vector<int32_t>& jb,
                    const int32_t* cpu = nullptr, const int32_t* mem = nullptr, const int32_t* gpu = nullptr,
                    const uint16_t* part = nullptr, bool classify = false, bool* cls_ok = nullptr) {
    const int C = c->ncomp;
    hipStream_t st = c->st;
    if (c->jl.ensure(std::max(J, 1)) || c->jpk.ensure(J + 1) ||
        c->jls.ensure(std::max<size_t>(joblists_scratch_ints(J), 1) + 2 * (C + 1) + 2) ||
        c->h_jls.ensure(2 * (C + 1) + 2))
        return FIT_E_OOM;
    int32_t* g = c->jls.p + joblists_scratch_ints(J);
    int32_t* jbd = g + 2;
    int32_t* mbd = jbd + C + 1;
    HIP_TRY(launch_joblists(st, c->jcomp.p, J, C, c->jls.p, g, jbd, mbd, c->jl.p, c->jpk.p));
    // the counters, the component offsets and the multi-node offsets (mbd[C]: multi-node jobs)
    HIP_TRY(hipMemcpyAsync(c->h_jls.p, g, sizeof(int32_t) * (2 * (C + 1) + 2), hipMemcpyDeviceToHost, st));
    if (classify) {
        const size_t ts = (size_t)C * class_table_slots() * class_slot_bytes();
        if (c->jcls.ensure(std::max(J, 1)) || c->cls_tab.ensure(ts) ||
            c->cls_dem.ensure((size_t)C * class_max()) || c->cls_n.ensure(C) || c->h_cls_n.ensure(C))
            return FIT_E_OOM;
        HIP_TRY(hipMemsetAsync(c->cls_tab.p, 0, ts, st));
        HIP_TRY(hipMemsetAsync(c->cls_n.p, 0, sizeof(int32_t) * C, st));
        HIP_TRY(launch_classify(st, c->jcomp.p, cpu, mem, gpu, part, J, c->cls_tab.p, c->cls_dem.p, c->cls_n.p,
                                c->jcls.p));
        HIP_TRY(hipMemcpyAsync(c->h_cls_n.p, c->cls_n.p, sizeof(int32_t) * C, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (c->h_jls.p[1]) return fail(FIT_E_INVAL, "a job has a negative demand or nodes_k > kmax");
    if (cls_ok) {
        *cls_ok = classify;
        for (int k = 0; classify && k < C; ++k)
            if (c->h_cls_n.p[k] > class_max()) *cls_ok = false;
    }
    S.rejected = c->h_jls.p[0];
    jb.assign(c->h_jls.p + 2, c->h_jls.p + 2 + C + 1);
    c->last_multi = c->h_jls.p[2 + C + 1 + C];
    for (int k = 0; k < C; ++k) S.useful_evals += (int64_t)(jb[k + 1] - jb[k]) * c->n;
    return 0;
}

// The demand classes of every component's jobs on their own (after build_job_lists, which counted
// the multi-node jobs the automatic choice needs): k_classify and one synchronisation.
int classify_jobs(fit_ctx* c, int32_t J, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
                  const uint16_t* part, bool* cls_ok) {
    const int C = c->ncomp;
    hipStream_t st = c->st;
    const size_t ts = (size_t)C * class_table_slots() * class_slot_bytes();
    if (c->jcls.ensure(std::max(J, 1)) || c->cls_tab.ensure(ts) || c->cls_dem.ensure((size_t)C * class_max()) ||
        c->cls_n.ensure(C) || c->h_cls_n.ensure(C))
        return FIT_E_OOM;
    HIP_TRY(hipMemsetAsync(c->cls_tab.p, 0, ts, st));
    HIP_TRY(hipMemsetAsync(c->cls_n.p, 0, sizeof(int32_t) * C, st));
    HIP_TRY(launch_classify(st, c->jcomp.p, cpu, mem, gpu, part, J, c->cls_tab.p, c->cls_dem.p, c->cls_n.p,
                            c->jcls.p));
    HIP_TRY(hipMemcpyAsync(c->h_cls_n.p, c->cls_n.p, sizeof(int32_t) * C, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *cls_ok = true;
    for (int k = 0; k < C; ++k)
        if (c->h_cls_n.p[k] > class_max()) *cls_ok = false;
    return 0;
}

// ------------------------------------------------------------------------ placement
// A small placement in one launch (k_small, fit_kernels.hip: prefilter, per-component job order
// and placement in one kernel) and ONE device-to-host copy: with host memory for the placements
// (h_out) the stats ride at the tail of the out buffer (fit_place sizes it), so placements and
// stats come back together into pinned memory.
// Wait for the stream's work up to now: a short spin on an event (a small placement takes tens of
// µs, the wake-up of a blocking synchronisation costs about as much), then the blocking wait.
hipError_t sync_small(fit_ctx* c) {
    if (c->sync_spin) {
        hipError_t e = hipEventRecord(c->ev[2], c->st);
        if (e != hipSuccess) return e;
        const double t0 = now_ms();
        while ((e = hipEventQuery(c->ev[2])) == hipErrorNotReady && now_ms() - t0 < 2.0) {
        }
        if (e != hipErrorNotReady) return e;
    }
    return hipStreamSynchronize(c->st);
}

int place_direct(fit_ctx* c, int32_t J, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
                 const int32_t* wall, const uint16_t* part, const uint16_t* nk, int32_t kmax,
                 int32_t* out, int32_t* h_out, fit_stats& S, const SmallBatch* hb = nullptr) {
    const int C = c->ncomp;
    const int G = std::max(C, 1);  // blocks (block 0 also when the table is empty)
    hipStream_t st = c->st;
    const size_t rows = (size_t)J * kmax;
    const size_t nback = (h_out ? rows : 0) + 2 + G;
    if (c->small_placed.ensure(2 + G) || c->h_small.ensure(nback)) return FIT_E_OOM;
    int32_t* stat = h_out ? out + rows : c->small_placed.p;
    SmallComps sc;
    for (int k = 0; k <= 32; ++k) sc.nb[k] = c->nb[std::min(k, C)];
    HIP_TRY(hipEventRecord(c->ev[0], st));
    if (hb)
        HIP_TRY(launch_small_args(st, C, c->rec.p, sc, c->d_ptab.p, c->np, *hb, nk != nullptr, J, kmax, out, stat));
    else
        HIP_TRY(launch_small(st, C, c->rec.p, sc, c->d_ptab.p, c->np, cpu, mem, gpu, wall, part, nk, J, kmax,
                             out, stat));
    HIP_TRY(hipEventRecord(c->ev[1], st));
    HIP_TRY(hipMemcpyAsync(c->h_small.p, h_out ? out : stat, sizeof(int32_t) * nback, hipMemcpyDeviceToHost,
                           st));
    HIP_TRY(sync_small(c));
    const int32_t* hs = c->h_small.p + (h_out ? rows : 0);
    if (hs[1]) return fail(FIT_E_INVAL, "a job has a negative demand or nodes_k > kmax");
    if (h_out) memcpy(h_out, c->h_small.p, sizeof(int32_t) * rows);
    S.rejected = hs[0];
    for (int k = 0; k < C; ++k) S.placed += hs[2 + k];
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    S.ms_device = S.ms_commit = ms;
    S.rounds = C > 0 && J > S.rejected ? 1 : 0;
    S.components = C;
    S.engine = 2;
    return 0;
}

int place_impl(fit_ctx* c, int32_t J, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
               const int32_t* wall, const uint16_t* part, const uint16_t* nk, int32_t kmax,
               int32_t* out, fit_stats* stats, int32_t* h_out = nullptr, bool* h_out_done = nullptr,
               const SmallBatch* hb = nullptr) {
    const double t0 = now_ms();
    fit_stats S;
    memset(&S, 0, sizeof S);
    S.jobs = J;
    hipStream_t st = c->st;
    if (J <= c->small_direct && !c->collective()) {  // a few jobs: one launch, one synchronisation
        const int rc = place_direct(c, J, cpu, mem, gpu, wall, part, nk, kmax, out, h_out, S, hb);
        if (rc) return rc;
        if (h_out_done) *h_out_done = h_out != nullptr;
        S.unplaced = J - S.placed - S.rejected;
        S.ms_total = now_ms() - t0;
        if (stats) *stats = S;
        return 0;
    }
    // 1. prefilter: out[] init, FIT_REJECTED, component per job
    if (c->jcomp.ensure(std::max(J, 1))) return FIT_E_OOM;
    HIP_TRY(launch_prefilter(st, cpu, mem, gpu, wall, part, nk, J, kmax, c->d_ptab.p, c->np, out,
                             c->jcomp.p));
    // 2. per-component job lists in priority order (stable)
    const int C = c->ncomp;
    std::vector<int32_t> jb;
    // the demand-class engine needs the class count of every component: counted in the job
    // lists' synchronisation when the node table qualifies (world > 1: component sharding only —
    // the node-sharded layout keeps the host-driven rounds)
    const int pre_mode = !c->collective() ? 0
                         : (c->shard_mode == FIT_SHARD_AUTO ? (C >= c->world ? FIT_SHARD_COMPONENTS : FIT_SHARD_NODES)
                                                            : c->shard_mode);
    const bool cls_able = c->cls_nodes_ok && pre_mode != FIT_SHARD_NODES;
    const bool try_cls = (c->cls_mode == 1 || c->cls_mode == 2) && cls_able && (c->cls_mode == 2 || J > c->small_batch);
    bool cls_ok = false;
    int rc0 = build_job_lists(c, J, S, jb, cpu, mem, gpu, part, try_cls, &cls_ok);
    if (rc0) return rc0;
    // automatic (cls_mode 3, the default): a large placement whose live jobs are mostly multi-node
    // (C4) runs the class engine — its all-picks-at-once commit beats the persistent engine's
    // single-wave commit there; k = 1 queues keep the persistent engine
    const int32_t live = J - S.rejected;
    if (c->cls_mode == 3 && cls_able && live > c->small_batch && 2 * (int64_t)c->last_multi >= live) {
        rc0 = classify_jobs(c, J, cpu, mem, gpu, part, &cls_ok);
        if (rc0) return rc0;
    }
    const bool use_cls = cls_ok && (c->cls_mode == 2 || live > c->small_batch);

    // world > 1: split by components (each rank owns whole components, no per-round exchange)
    // or by nodes (north_star: every rank scans 1/world of every component, RCCL each round)
    int mode = 0;
    std::vector<char> owned(C, 1);
    if (c->collective()) {
        mode = c->shard_mode;
        if (mode == FIT_SHARD_AUTO) mode = C >= c->world ? FIT_SHARD_COMPONENTS : FIT_SHARD_NODES;
        if (mode == FIT_SHARD_COMPONENTS) {
            // LPT by work (jobs × nodes); identical on every rank (same inputs, same order)
            std::vector<int> order(C);
            for (int k = 0; k < C; ++k) order[k] = k;
            auto work = [&](int k) { return (int64_t)(jb[k + 1] - jb[k]) * (c->nb[k + 1] - c->nb[k]); };
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return work(a) > work(b); });
            std::vector<int64_t> load(c->world, 0);
            for (int k : order) {
                int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                load[r] += work(k) + 1;
                owned[k] = r == c->rank;
            }
        }
    }
    S.shard_mode = mode;
    S.components = C;
    const bool node_sharded = mode == FIT_SHARD_NODES;
    const int shards = node_sharded ? c->world : 1;
    const int srank = node_sharded ? c->rank : 0;

    // 3. speculative rounds: one persistent launch, or the host-driven loop (node sharding
    // exchanges candidates over RCCL every round, so it keeps the host loop; a small batch is
    // cheaper as a round or two of k_scan / k_commit than as a whole-chip persistent grid)
    const bool small = J - S.rejected <= c->small_batch;
    if (use_cls) {
        int rc = run_class(c, J, jb, owned, wall, nk, out, kmax, S);
        if (rc) return rc;
    } else if (c->persistent && !node_sharded && !small) {
        int rc = run_persistent(c, jb, owned, cpu, mem, gpu, wall, part, nk, out, kmax, S);
        if (rc) return rc;
        S.engine = 1;
    } else {
    std::vector<int32_t> cur(jb.begin(), jb.end() - 1), win(C, c->wmin);
    if (c->plan.ensure(C + 1) || c->res.ensure(C + 1) || c->h_plan.ensure(C + 1) ||
        c->h_res.ensure(C + 1))
        return FIT_E_OOM;
    float ms;
    for (;;) {
        int64_t blocks = 0, slots = 0, cand_n = 0, evals = 0;
        int epl = 1;
        size_t lds = 0;
        bool any = false;
        for (int k = 0; k < C; ++k) {
            CompPlan& P = c->h_plan.p[k];
            P.k0 = 0;
            memset(&P, 0, sizeof P);
            P.nb = c->nb[k];
            P.ne = c->nb[k + 1];
            const int32_t len = P.ne - P.nb;
            const int32_t per = (len + shards - 1) / shards;
            P.sb = std::min(P.ne, P.nb + per * srank);
            P.se = std::min(P.ne, P.sb + per);
            // sub-slices of >= MIN_SUB nodes, at most MAX_SLICES block-slices per job per rank
            P.ks = KS;
            P.sub = std::max(MIN_SUB, (per + SCAN_WAVES * MAX_SLICES - 1) / (SCAN_WAVES * MAX_SLICES));
            P.nslice = std::max(1, (per + SCAN_WAVES * P.sub - 1) / (SCAN_WAVES * P.sub));
            epl = std::max(epl, (shards * P.nslice * KS + 63) / 64);
            P.jbase = cur[k];
            P.w = owned[k] ? std::min(win[k], jb[k + 1] - cur[k]) : 0;
            P.blk0 = (int32_t)blocks;
            P.cand_off = cand_n;
            P.slot0 = (int32_t)slots;
            if (P.w > 0) {
                any = true;
                blocks += (int64_t)((P.w + SCAN_JOBS - 1) / SCAN_JOBS) * P.nslice;
                cand_n += (int64_t)P.w * P.nslice * KS;
                slots += P.w;
                evals += (int64_t)P.w * (P.se - P.sb);
                lds = std::max(lds, (size_t)((len + 31) / 32) * 4);
            }
        }
        if (!any) break;
        S.rounds++;
        S.evals += evals;
        if (c->cand.ensure((size_t)cand_n * shards) || c->bnd.ensure(slots) ||
            c->wjob.ensure(slots))
            return FIT_E_OOM;
        HIP_TRY(hipMemcpyAsync(c->plan.p, c->h_plan.p, sizeof(CompPlan) * C, hipMemcpyHostToDevice,
                               st));
        HIP_TRY(hipMemsetAsync(c->bnd.p, 0xff, sizeof(uint64_t) * slots, st));
        HIP_TRY(hipEventRecord(c->ev[0], st));
        HIP_TRY(launch_scan((int)blocks, st, c->rec.p, c->jl.p, cpu, mem, gpu, wall, part, nk,
                            c->plan.p, C, c->cand.p + (size_t)srank * cand_n, c->bnd.p,
                            c->wjob.p));
        HIP_TRY(hipEventRecord(c->ev[1], st));
        if (node_sharded) {
            // every rank scanned its node shard: gather all candidate sections, min the bounds
            int rc = xchg(c, FIT_XCHG_ALLGATHER_U64, c->cand.p, cand_n);
            if (!rc) rc = xchg(c, FIT_XCHG_MIN_U64, c->bnd.p, slots);
            if (rc) return rc;
        }
        HIP_TRY(hipEventRecord(c->ev[2], st));
        HIP_TRY(launch_commit(C, epl, lds, st, c->rec.p, c->plan.p, c->cand.p, cand_n, shards,
                              c->bnd.p, c->wjob.p, out, kmax, c->res.p));
        HIP_TRY(hipEventRecord(c->ev[3], st));
        HIP_TRY(hipMemcpyAsync(c->h_res.p, c->res.p, sizeof(CommitResult) * C,
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        S.ms_scan += ms;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
        S.ms_exchange += ms;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
        S.ms_commit += ms;
        for (int k = 0; k < C; ++k) {
            const CompPlan& P = c->h_plan.p[k];
            if (P.w == 0) continue;
            const CommitResult& R = c->h_res.p[k];
            if (R.done < 0 || R.done > P.w)
                return fail(FIT_E_HIP, "commit returned %d of window %d", R.done, P.w);
            cur[k] += R.done;
            S.placed += R.placed;
            if (R.stop == 1) S.stops_rescan++;
            if (R.stop == 2) S.stops_dirty++;
            int32_t nw = R.stop ? 2 * R.done : 2 * P.w;
            win[k] = std::max(c->wmin, std::min(c->wmax, nw));
        }
    }
    S.ms_device = S.ms_scan + S.ms_exchange + S.ms_commit;
    }  // host-driven rounds
    if (mode == FIT_SHARD_COMPONENTS) {
        // each rank placed only its components: combine placements (owner's >= -1 beats -1;
        // rejections are identical everywhere) and node rows (only owners lowered them)
        int rc = xchg(c, FIT_XCHG_MAX_I32, out, (int64_t)J * kmax);
        if (!rc) rc = xchg(c, FIT_XCHG_MIN_I32, c->rec.p, (int64_t)c->nn * 8);
        if (rc) return rc;
        // global placed count: allgather one u64 per rank, sum on the host
        if (c->xcount.ensure(c->world) || c->h_count.ensure(c->world)) return FIT_E_OOM;
        c->h_count.p[c->rank] = (uint64_t)S.placed;
        HIP_TRY(hipMemcpyAsync(c->xcount.p + c->rank, c->h_count.p + c->rank, 8,
                               hipMemcpyHostToDevice, st));
        rc = xchg(c, FIT_XCHG_ALLGATHER_U64, c->xcount.p, 1);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(c->h_count.p, c->xcount.p, 8 * c->world, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        S.placed = 0;
        for (int r = 0; r < c->world; ++r) S.placed += (int64_t)c->h_count.p[r];
    }
    // jobs of partitions without nodes are FIT_UNPLACED like jobs nothing fits
    S.unplaced = J - S.placed - S.rejected;
    S.ms_total = now_ms() - t0;
    if (stats) *stats = S;
    return 0;
}

// ----------------------------------------------------------- time-windowed backfill
// SPEC §2b: the same speculative rounds as the plain fit (host-driven loop), with run-list
// scans / commits (fit_timeline.hip).  world > 1 always splits by nodes: every rank scans its
// share of each component, the candidate sections are exchanged each round and the identical
// deterministic commit runs on every rank over replicated run lists.
// Persistent single-launch backfill (k_engine_tl): the placement's rounds for
// every component in one launch, no host round trips (world == 1).
int run_persistent_tl(fit_ctx* c, const std::vector<int32_t>& jb, const int32_t* cpu,
                      const int32_t* mem, const int32_t* gpu, const int32_t* wall,
                      const uint16_t* part, int32_t* out, int32_t* outs, fit_stats& S) {
    const int C = c->ncomp;
    hipStream_t st = c->st;
    std::vector<int> comps;
    int32_t maxnodes = 0;
    for (int k = 0; k < C; ++k)
        if (jb[k + 1] > jb[k]) {
            comps.push_back(k);
            maxnodes = std::max(maxnodes, c->nb[k + 1] - c->nb[k]);
        }
    const int nc = (int)comps.size();
    if (nc == 0) return 0;
    const int R = engine_tl_runs(maxnodes);
    if (R < 1) return fail(FIT_E_INVAL, "partition component of %d nodes is too large for the "
                                        "timeline engine's LDS", maxnodes);
    const int64_t wcap = std::min(c->wmax, 8192);
    int slices = TL_SLICES, tl_min_sub = TL_MIN_SUB;
    if (const char* e = getenv("FIT_TL_SLICES")) slices = std::max(1, std::min(atoi(e), TL_SLICES));
    if (const char* e = getenv("FIT_TL_MINSUB")) tl_min_sub = std::max(1, atoi(e));
    const int64_t per_comp_cand = wcap * slices * TL_KS;
    // two sets of per-round buffers by round parity (see run_persistent)
    if (c->ecs.ensure(nc) || c->eco.ensure(nc) || c->h_ecs.ensure(nc) || c->h_eco.ensure(nc) ||
        c->plan.ensure(2 * nc) ||
        c->cand.ensure((size_t)2 * nc * per_comp_cand + (size_t)2 * nc * PAIR_AREA) ||
        c->bnd.ensure((size_t)2 * nc * wcap) || c->wjob.ensure((size_t)2 * nc * wcap) ||
        c->ectl.ensure(engine_ctl_bytes()) || c->ering.ensure(engine_ring_bytes()) ||
        c->h_err.ensure(4))
        return FIT_E_OOM;
    if ((int64_t)2 * nc * per_comp_cand + (int64_t)2 * nc * PAIR_AREA > INT32_MAX)
        return fail(FIT_E_INVAL, "candidate buffer exceeds 2^31 entries (%d components)", nc);
    for (int i = 0; i < nc; ++i) {
        const int k = comps[i];
        CompState& s = c->h_ecs.p[i];
        s.nb = s.sb = c->nb[k];
        s.ne = s.se = c->nb[k + 1];
        const int32_t len = s.ne - s.nb;
        s.ks = TL_KS;
        s.sub = std::max(tl_min_sub, (len + SCAN_WAVES * slices - 1) / (SCAN_WAVES * slices));
        s.nslice = std::max(1, (len + SCAN_WAVES * s.sub - 1) / (SCAN_WAVES * s.sub));
        s.jstart = jb[k];
        s.jend = jb[k + 1];
        s.cand_off = (int64_t)i * per_comp_cand;
        s.slot0 = (int32_t)(i * wcap);
        s.cand_alt = (int64_t)(nc + i) * per_comp_cand;
        s.slot_alt = (int32_t)((nc + i) * wcap);
        s.pair_off = (int32_t)(2 * nc * per_comp_cand + (int64_t)2 * i * PAIR_AREA);
        s.wmin = std::min(c->wmin, (int)wcap);
        s.wmax = (int32_t)wcap;
    }
    {  // task ring capacity (see run_persistent)
        int32_t max_slices = 1;
        for (int i = 0; i < nc; ++i) max_slices = std::max(max_slices, c->h_ecs.p[i].nslice);
        // (+ one tile: a round's first tile may be scanned as twice the slices, TL_T0PAIR)
        if ((int64_t)2 * ring_comps(nc) * ((wcap + SCAN_JOBS - 1) / SCAN_JOBS + 1) * max_slices >
            (int64_t)engine_ring_tasks())
            return fail(FIT_E_INVAL, "task ring too small: %d components x %lld tiles x %d slices",
                        nc, (long long)((wcap + SCAN_JOBS - 1) / SCAN_JOBS), max_slices);
    }
    const size_t lds = engine_tl_lds_bytes(maxnodes);
    // FIT_TL_SPLIT: committers and scan workers as two concurrent launches (fit_timeline.hip
    // k_engine_tl_t): the workers' launch carries only the scan's registers and LDS, so several
    // worker blocks share a CU instead of one block per CU for everything
    bool split = FIT_TL_SPLIT_DEF != 0;
    if (const char* e = getenv("FIT_TL_SPLIT")) split = atoi(e) != 0;
    const size_t lds_w = split ? engine_tl_scan_lds_bytes() : lds;
    const int per_cu = engine_tl_blocks_per_cu(lds, split ? 1 : 0);
    if (per_cu <= 0) return fail(FIT_E_HIP, "k_engine_tl does not fit on a CU (lds %zu)", lds);
    const int per_cu_w = split ? engine_tl_blocks_per_cu(lds_w, 2) : per_cu;
    if (per_cu_w <= 0) return fail(FIT_E_HIP, "k_engine_tl workers do not fit on a CU");
    int workers = split ? std::max(8, per_cu_w * std::max(1, c->cus - nc)) : std::max(8, per_cu * c->cus - nc);
    if (const char* e = getenv("FIT_WORKERS")) workers = std::max(1, atoi(e));
    if (split && !c->st2) {
        if (hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
            hipHostMalloc(&c->resident, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return fail(FIT_E_HIP, "split launch: stream / event / mapped flag");
    }
    if (c->ebusy.ensure(2 * workers) || c->h_ebusy.ensure(2 * workers) || c->h_trip.ensure(1))
        return FIT_E_OOM;
    HIP_TRY(hipMemcpyAsync(c->ecs.p, c->h_ecs.p, sizeof(CompState) * nc, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(c->ectl.p, 0, engine_ctl_bytes(), st));
    HIP_TRY(hipMemsetAsync(c->ering.p, 0, engine_ring_bytes(), st));
    // every bound KEY_INF: a round resets only the bounds its buffer set's last round used
    HIP_TRY(hipMemsetAsync(c->bnd.p, 0xff, sizeof(uint64_t) * 2 * nc * wcap, st));
    ArbGuard arb;  // one persistent launch per device at a time (see DevArb); to the sync below
    {
        int rc = arb.take(c->device);
        if (rc) return rc;
        S.ms_arb_wait = arb.waited_ms;
    }
    HIP_TRY(hipEventRecord(c->ev[0], st));
    bool resident_late = false;
    if (!split) {
        HIP_TRY(launch_engine_tl(nc + workers, lds, st, c->ectl.p, c->ering.p, c->ecs.p, c->eco.p,
                                 c->plan.p, nc, c->slab.p, c->tlhdr.p, c->jl.p, cpu, mem, gpu, wall,
                                 part, c->cand.p, c->bnd.p, c->wjob.p, c->perm.p, out, outs,
                                 c->tl_slots, c->tl_slot_min, R, c->ebusy.p, 0, nullptr, c->wd_ticks));
    } else {
        __atomic_store_n(c->resident, 0u, __ATOMIC_RELEASE);
        unsigned* dres = nullptr;
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&dres), c->resident, 0));
        HIP_TRY(launch_engine_tl(nc, lds, st, c->ectl.p, c->ering.p, c->ecs.p, c->eco.p, c->plan.p,
                                 nc, c->slab.p, c->tlhdr.p, c->jl.p, cpu, mem, gpu, wall, part,
                                 c->cand.p, c->bnd.p, c->wjob.p, c->perm.p, out, outs, c->tl_slots,
                                 c->tl_slot_min, R, c->ebusy.p, 1, dres, c->wd_ticks));
        // the workers go in once every committer block holds its CU (a worker block on a CU
        // would leave a committer no room, and the committers' rounds wait for workers)
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(c->resident, __ATOMIC_ACQUIRE) < (unsigned)nc) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                resident_late = true;  // launched anyway: the kernels' own watchdogs end it
                break;
            }
        }
        HIP_TRY(hipStreamWaitEvent(c->st2, c->ev[0], 0));  // after the control-block resets
        HIP_TRY(launch_engine_tl(workers, lds_w, c->st2, c->ectl.p, c->ering.p, c->ecs.p, c->eco.p,
                                 c->plan.p, nc, c->slab.p, c->tlhdr.p, c->jl.p, cpu, mem, gpu, wall,
                                 part, c->cand.p, c->bnd.p, c->wjob.p, c->perm.p, out, outs,
                                 c->tl_slots, c->tl_slot_min, R, c->ebusy.p, 2, nullptr, c->wd_ticks));
        HIP_TRY(hipEventRecord(c->ev_join, c->st2));
        HIP_TRY(hipStreamWaitEvent(st, c->ev_join, 0));
    }
    HIP_TRY(hipEventRecord(c->ev[1], st));
    HIP_TRY(hipMemcpyAsync(c->h_eco.p, c->eco.p, sizeof(CompOut) * nc, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_ebusy.p, c->ebusy.p, sizeof(int64_t) * 2 * workers,
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_err.p, c->ectl.p + engine_ctl_error_offset(), 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_trip.p, c->ectl.p + engine_ctl_trip_offset(), sizeof(TripRec),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // a trip leaves the run lists partly reserved: the timeline must be loaded again (a copy of
    // the slab per placement would cost more than the rare reload); the node table is untouched
    if (c->h_err.p[0]) {
        c->have_tl = false;
        return trip_error(c, "timeline engine");
    }
    if (resident_late) {
        c->have_tl = false;
        return fail(FIT_E_HIP, "timeline engine: committer blocks not resident after 10 s");
    }
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    S.ms_device += ms;
    int64_t busy = 0;
    // per worker {busy ticks, evaluations scanned}: tiles of a finished round are dropped, so
    // the performed evaluations are counted where they happen
    for (int i = 0; i < workers; ++i) {
        busy += c->h_ebusy.p[2 * i];
        S.evals += c->h_ebusy.p[2 * i + 1];
    }
    S.ms_scan += busy / 1e5 / workers;
    double commit_max = 0;
    for (int i = 0; i < nc; ++i) {
        const CompOut& o = c->h_eco.p[i];
        const int k = comps[i];
        if (o.done_jobs != jb[k + 1] - jb[k])
            return fail(FIT_E_HIP, "component %d resolved %lld of %d jobs", k, (long long)o.done_jobs,
                        jb[k + 1] - jb[k]);
        S.placed += o.placed;
        S.rounds = std::max<int64_t>(S.rounds, o.rounds);
        S.stops_rescan += o.stops_rescan;
        S.stops_dirty += o.stops_dirty;
        commit_max = std::max(commit_max, o.t_commit / 1e5);
    }
    S.ms_commit += commit_max;
    S.engine = 1;
    return 0;
}

int place_tl_impl(fit_ctx* c, int32_t J, const int32_t* cpu, const int32_t* mem,
                  const int32_t* gpu, const int32_t* wall, const uint16_t* part, int32_t* out,
                  int32_t* outs, fit_stats* stats) {
    const double t0 = now_ms();
    fit_stats S;
    memset(&S, 0, sizeof S);
    S.jobs = J;
    hipStream_t st = c->st;
    if (c->jcomp.ensure(std::max(J, 1))) return FIT_E_OOM;
    HIP_TRY(launch_prefilter(st, cpu, mem, gpu, wall, part, nullptr, J, 1, c->d_ptab.p, c->np, out,
                             c->jcomp.p));
    if (J > 0) HIP_TRY(hipMemsetAsync(outs, 0xff, sizeof(int32_t) * J, st));
    const int C = c->ncomp;
    std::vector<int32_t> jb;
    int rc = build_job_lists(c, J, S, jb);
    if (rc) return rc;
    const bool node_sharded = c->collective();
    const int shards = c->world, srank = c->rank;
    S.shard_mode = node_sharded ? FIT_SHARD_NODES : 0;
    S.components = C;
    if (c->persistent && !node_sharded && J - S.rejected > c->small_batch) {
        rc = run_persistent_tl(c, jb, cpu, mem, gpu, wall, part, out, outs, S);
        if (rc) return rc;
        S.unplaced = J - S.placed - S.rejected;
        S.ms_total = now_ms() - t0;
        if (stats) *stats = S;
        return 0;
    }
    std::vector<int32_t> cur(jb.begin(), jb.end() - 1), win(C, c->wmin);
    if (c->plan.ensure(C + 1) || c->res.ensure(C + 1) || c->h_plan.ensure(C + 1) ||
        c->h_res.ensure(C + 1))
        return FIT_E_OOM;
    int32_t maxlen = 1;
    for (int k = 0; k < C; ++k) maxlen = std::max(maxlen, c->nb[k + 1] - c->nb[k]);
    const size_t lds = commit_tl_lds_bytes(maxlen);
    const int runs = commit_tl_runs(maxlen);
    int slices = std::max(1, TL_SLICES / shards), tl_min_sub = TL_MIN_SUB;
    if (const char* e = getenv("FIT_TL_SLICES")) slices = std::max(1, std::min(atoi(e), 512 / (TL_KS * shards)));
    if (const char* e = getenv("FIT_TL_MINSUB")) tl_min_sub = std::max(1, atoi(e));
    if (runs < 1)
        return fail(FIT_E_INVAL, "partition component of %d nodes is too large for the timeline "
                                 "commit's LDS", maxlen);
    float ms;
    for (;;) {
        int64_t blocks = 0, slots = 0, cand_n = 0, evals = 0;
        int epl = 1;
        bool any = false;
        for (int k = 0; k < C; ++k) {
            CompPlan& P = c->h_plan.p[k];
            P.k0 = 0;
            memset(&P, 0, sizeof P);
            P.nb = c->nb[k];
            P.ne = c->nb[k + 1];
            const int32_t len = P.ne - P.nb;
            const int32_t per = (len + shards - 1) / shards;
            P.sb = std::min(P.ne, P.nb + per * srank);
            P.se = std::min(P.ne, P.sb + per);
            // more, shorter block-slices than the plain fit: a run walk costs more per node, so
            // the scan wants more waves in flight; candidate entries per job stay <= 256
            P.ks = TL_KS;
            P.sub = std::max(tl_min_sub, (per + SCAN_WAVES * slices - 1) / (SCAN_WAVES * slices));
            P.nslice = std::max(1, (per + SCAN_WAVES * P.sub - 1) / (SCAN_WAVES * P.sub));
            epl = std::max(epl, (shards * P.nslice * TL_KS + 63) / 64);
            P.jbase = cur[k];
            P.w = std::min(win[k], jb[k + 1] - cur[k]);
            P.blk0 = (int32_t)blocks;
            P.cand_off = cand_n;
            P.slot0 = (int32_t)slots;
            if (P.w > 0) {
                any = true;
                blocks += (int64_t)((P.w + SCAN_JOBS - 1) / SCAN_JOBS) * P.nslice;
                cand_n += (int64_t)P.w * P.nslice * TL_KS;
                slots += P.w;
                evals += (int64_t)P.w * (P.se - P.sb);
            }
        }
        if (!any) break;
        S.rounds++;
        S.evals += evals;
        if (c->cand.ensure((size_t)cand_n * shards) || c->bnd.ensure(slots) ||
            c->wjob.ensure(slots))
            return FIT_E_OOM;
        HIP_TRY(hipMemcpyAsync(c->plan.p, c->h_plan.p, sizeof(CompPlan) * C, hipMemcpyHostToDevice,
                               st));
        HIP_TRY(hipMemsetAsync(c->bnd.p, 0xff, sizeof(uint64_t) * slots, st));
        HIP_TRY(hipEventRecord(c->ev[0], st));
        HIP_TRY(launch_scan_tl((int)blocks, st, c->slab.p, c->tlhdr.p, c->jl.p, cpu, mem,
                               gpu, wall, part, c->plan.p, C, c->cand.p + (size_t)srank * cand_n,
                               c->bnd.p, c->wjob.p, c->tl_slots, c->tl_slot_min));
        HIP_TRY(hipEventRecord(c->ev[1], st));
        if (node_sharded) {
            rc = xchg(c, FIT_XCHG_ALLGATHER_U64, c->cand.p, cand_n);
            if (!rc) rc = xchg(c, FIT_XCHG_MIN_U64, c->bnd.p, slots);
            if (rc) return rc;
        }
        HIP_TRY(hipEventRecord(c->ev[2], st));
        HIP_TRY(launch_commit_tl(C, epl, lds, st, c->slab.p, c->tlhdr.p, c->plan.p, c->cand.p,
                                 cand_n, shards, c->bnd.p, c->wjob.p, c->perm.p, out, outs,
                                 c->res.p, c->tl_slots, runs));
        HIP_TRY(hipEventRecord(c->ev[3], st));
        HIP_TRY(hipMemcpyAsync(c->h_res.p, c->res.p, sizeof(CommitResult) * C,
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        S.ms_scan += ms;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
        S.ms_exchange += ms;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
        S.ms_commit += ms;
        for (int k = 0; k < C; ++k) {
            const CompPlan& P = c->h_plan.p[k];
            if (P.w == 0) continue;
            const CommitResult& R = c->h_res.p[k];
            if (R.done < 0 || R.done > P.w)
                return fail(FIT_E_HIP, "commit returned %d of window %d", R.done, P.w);
            cur[k] += R.done;
            S.placed += R.placed;
            if (R.stop == 1) S.stops_rescan++;
            if (R.stop == 2) S.stops_dirty++;
            const int32_t nw = R.stop ? 2 * R.done : 2 * P.w;
            win[k] = std::max(c->wmin, std::min(c->wmax, nw));
        }
    }
    S.ms_device = S.ms_scan + S.ms_exchange + S.ms_commit;
    S.unplaced = J - S.placed - S.rejected;
    S.ms_total = now_ms() - t0;
    if (stats) *stats = S;
    return 0;
}

int load_timeline_impl(fit_ctx* c, int32_t slots, int32_t slot_min, int64_t ne) {
    if (c->tlhdr.ensure(std::max(c->nn, 1)) ||
        c->slab.ensure((size_t)std::max(c->nn, 1) * TL_MAX_SLOTS) || c->tl_err.ensure(1) ||
        c->h_tl_err.ensure(1))
        return FIT_E_OOM;
    HIP_TRY(hipMemsetAsync(c->tl_err.p, 0, 4, c->st));
    HIP_TRY(launch_build_tl(c->st, c->col_cpu.p, c->col_mem.p, c->col_gpu.p, c->col_av.p,
                            c->col_mask.p, c->perm.p, c->nn, slots, slot_min, ne >= 0 ? c->rel_off.p : nullptr,
                            c->rel_slot.p, c->rel_cpu.p, c->rel_mem.p, c->rel_gpu.p, c->slab.p,
                            c->tlhdr.p, c->tl_err.p));
    HIP_TRY(hipMemcpyAsync(c->h_tl_err.p, c->tl_err.p, 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    if (c->h_tl_err.p[0])
        return fail(FIT_E_INVAL, "release events: slots must be non-decreasing per node and "
                                 "amounts >= 0");
    c->tl_slots = slots;
    c->tl_slot_min = slot_min;
    c->have_tl = true;
    return 0;
}

int check_timeline_args(fit_ctx* c, int32_t slots, int32_t slot_min) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (!c->have_nodes) return fail(FIT_E_STATE, "fit_load_nodes not called");
    if (slots < 1 || slots > TL_MAX_SLOTS || slot_min < 1)
        return fail(FIT_E_INVAL, "horizon of %d slots x %d min (1..%d slots)", slots, slot_min,
                    TL_MAX_SLOTS);
    if (c->nn > (int32_t)TL_POS_MASK + 1)
        return fail(FIT_E_INVAL, "%d nodes exceed the timeline key's %d-bit position", c->nn,
                    TL_POS_BITS);
    return 0;
}

}  // namespace

// ============================================================================ C-ABI
extern "C" {

int fit_abi_version(void) { return FITGPU_ABI_VERSION; }

int fit_lock_dir(char* buf, int32_t buflen) {
    std::string dir;
    const int shared = resolve_lock_dir(dir);
    if (!buf || buflen <= (int32_t)dir.size()) return fail(FIT_E_INVAL, "fit_lock_dir: buffer too small");
    memcpy(buf, dir.c_str(), dir.size() + 1);
    return shared;
}

const char* fit_strerror(int code) {
    switch (code) {
        case FIT_OK: return "ok";
        case FIT_E_INVAL: return "invalid argument";
        case FIT_E_HIP: return "HIP runtime error";
        case FIT_E_RCCL: return "RCCL error";
        case FIT_E_OOM: return "out of memory";
        case FIT_E_NODEV: return "no usable gfx950 device";
        case FIT_E_STATE: return "call out of order";
        case FIT_E_PARSE: return "parse error";
        case FIT_E_UNLIMITED: return "duration is unlimited";
        default: return "unknown error";
    }
}

const char* fit_last_error(void) { return g_last_error.c_str(); }

int fit_nccl_unique_id(void* out128) {
    if (!out128) return fail(FIT_E_INVAL, "null id buffer");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(out128, &id, sizeof id);
    return 0;
}

int fit_create(const fit_opts* opts, fit_ctx** out_ctx) {
    if (!out_ctx) return fail(FIT_E_INVAL, "null out_ctx");
    *out_ctx = nullptr;
    fit_opts o;
    memset(&o, 0, sizeof o);
    o.device = -1;
    o.world = 1;
    if (opts) o = *opts;
    if (o.world < 1 || o.rank < 0 || o.rank >= o.world)
        return fail(FIT_E_INVAL, "rank %d / world %d", o.rank, o.world);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(FIT_E_NODEV, "no HIP device visible");
    int dev = o.device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev >= ndev) return fail(FIT_E_INVAL, "device %d of %d", dev, ndev);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(FIT_E_NODEV, "device %d is %s, this build targets gfx950", dev,
                    prop.gcnArchName);
    HIP_TRY(hipSetDevice(dev));
    fit_ctx* c = new (std::nothrow) fit_ctx();
    if (!c) return fail(FIT_E_OOM, "context allocation");
    c->device = dev;
    c->cus = prop.multiProcessorCount;
    if (const char* ev = getenv("FIT_WATCHDOG_MS"))
        c->wd_ticks = (unsigned)std::min<double>(4.29e9, std::max(1.0, atof(ev) * 1e5));
    // unset FIT_ENGINE: k_small up to small_direct jobs, the host-driven rounds up to small_batch
    // live jobs, the persistent engine above (FIT_SMALL_DIRECT, FIT_SMALL_BATCH)
    if (const char* ev = getenv("FIT_SMALL_BATCH")) c->small_batch = atoi(ev);
    if (const char* ev = getenv("FIT_SMALL_DIRECT")) c->small_direct = atoi(ev);
    if (const char* ev = getenv("FIT_SMALL_ARGS")) c->small_args = atoi(ev) != 0;
    if (const char* ev = getenv("FIT_SYNC_SPIN")) c->sync_spin = atoi(ev) != 0;
    // FIT_ENGINE forces one engine at every size: "rounds", "persistent" or "direct" (k_small)
    if (const char* ev = getenv("FIT_CLASS")) c->cls_mode = atoi(ev) ? 1 : 0;  // unset: automatic (3)
    if (const char* ev = getenv("FIT_ENGINE")) {
        c->persistent = strcmp(ev, "rounds") != 0;
        if (strcmp(ev, "persistent") == 0 || strcmp(ev, "class") == 0) c->small_batch = -1;
        c->small_direct = strcmp(ev, "direct") == 0 ? INT32_MAX : -1;
        c->cls_mode = strcmp(ev, "class") == 0 ? 2 : 0;
    }
    c->rank = o.rank;
    c->world = o.world;
    c->force_coll = (o.flags & FIT_FLAG_COLLECTIVES) != 0;
    c->shard_mode = o.shard_mode;
    c->xchg = o.exchange;
    c->xchg_user = o.exchange_user;
    if (o.window_min > 0) c->wmin = o.window_min;
    if (o.window_max > 0) c->wmax = std::max(o.window_max, c->wmin);
    for (int p = 0; p < 32; ++p) {
        c->comp_of_part[p] = -1;
        c->ptab[p] = c->ptab[32 + p] = c->ptab[64 + p] = -1;
        c->ptab[96 + p] = -1;
    }
    int rc = 0;
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) rc = FIT_E_HIP;
    for (auto& e : c->ev)
        if (!rc && hipEventCreate(&e) != hipSuccess) rc = FIT_E_HIP;
    if (!rc && c->world == 1 && c->force_coll && !c->xchg) {
        // FIT_FLAG_COLLECTIVES: a one-rank RCCL communicator, so the sharded code path and its
        // RCCL calls run on one GPU exactly as they do in a multi-GPU group
        ncclUniqueId id;
        ncclResult_t r = ncclGetUniqueId(&id);
        if (r == ncclSuccess) r = ncclCommInitRank(&c->comm, 1, id, 0);
        if (r != ncclSuccess) rc = fail(FIT_E_RCCL, "ncclCommInitRank(1 rank): %s", ncclGetErrorString(r));
    } else if (!rc && c->world > 1 && !c->xchg) {
        if (!o.nccl_id) {
            rc = fail(FIT_E_INVAL, "world > 1 needs nccl_id");
        } else {
            ncclUniqueId id;
            memcpy(&id, o.nccl_id, sizeof id);
            ncclResult_t r = ncclCommInitRank(&c->comm, c->world, id, c->rank);
            if (r != ncclSuccess)
                rc = fail(FIT_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
        }
    } else if (rc) {
        fail(rc, "stream/event creation failed");
    }
    if (rc) {
        delete c;
        return rc;
    }
    *out_ctx = c;
    return 0;
}

int fit_set_watchdog_us(fit_ctx* c, int64_t us) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (us <= 0) {
        c->wd_ticks = 1000000000u;
        if (const char* ev = getenv("FIT_WATCHDOG_MS"))
            c->wd_ticks = (unsigned)std::min<double>(4.29e9, std::max(1.0, atof(ev) * 1e5));
        return 0;
    }
    // 100 realtime ticks per microsecond; the ticks are a 32-bit kernel argument (<= 42.9 s)
    c->wd_ticks = (unsigned)std::min<int64_t>(us * 100, 4290000000ll);
    return 0;
}

void fit_destroy(fit_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->st);
    delete ctx;
}

int fit_load_nodes(fit_ctx* c, int32_t n, const int32_t* cpu, const int32_t* mem,
                   const int32_t* gpu, const int32_t* av, const uint32_t* mask) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (n < 0 || n > FIT_MAX_NODES || (n > 0 && (!cpu || !mem || !gpu || !av || !mask)))
        return fail(FIT_E_INVAL, "bad node arrays");
    // the columns are overwritten below: until the load succeeds there is no valid node table
    // (a failed load must not leave new offsets paired with old node rows)
    c->have_nodes = c->have_tl = false;
    HIP_TRY(hipSetDevice(c->device));
    if (alloc_cols(c, n)) return FIT_E_OOM;
    const size_t b = sizeof(int32_t) * n;
    HIP_TRY(hipMemcpyAsync(c->col_cpu.p, cpu, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_mem.p, mem, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_gpu.p, gpu, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_av.p, av, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_mask.p, mask, b, hipMemcpyHostToDevice, c->st));
    c->h_mask.assign(mask, mask + n);
    return load_nodes_common(c, n);
}

int fit_load_nodes_device(fit_ctx* c, int32_t n, const int32_t* cpu, const int32_t* mem,
                          const int32_t* gpu, const int32_t* av, const uint32_t* mask) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (n < 0 || n > FIT_MAX_NODES || (n > 0 && (!cpu || !mem || !gpu || !av || !mask)))
        return fail(FIT_E_INVAL, "bad node arrays");
    c->have_nodes = c->have_tl = false;  // see fit_load_nodes
    HIP_TRY(hipSetDevice(c->device));
    if (alloc_cols(c, n)) return FIT_E_OOM;
    const size_t b = sizeof(int32_t) * n;
    HIP_TRY(hipMemcpyAsync(c->col_cpu.p, cpu, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_mem.p, mem, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_gpu.p, gpu, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_av.p, av, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->col_mask.p, mask, b, hipMemcpyDeviceToDevice, c->st));
    c->h_mask.resize(n);
    HIP_TRY(hipMemcpyAsync(c->h_mask.data(), mask, b, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return load_nodes_common(c, n);
}

int fit_load_partitions(fit_ctx* c, int32_t p, const int32_t* max_time,
                        const int32_t* max_cpus, const int32_t* max_mem) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (p < 0 || p > FIT_MAX_PARTITIONS || (p > 0 && (!max_time || !max_cpus || !max_mem)))
        return fail(FIT_E_INVAL, "bad partition table (p=%d)", p);
    HIP_TRY(hipSetDevice(c->device));
    c->np = p;
    for (int i = 0; i < 32; ++i) {
        c->ptab[i] = i < p ? max_time[i] : -1;
        c->ptab[32 + i] = i < p ? max_cpus[i] : -1;
        c->ptab[64 + i] = i < p ? max_mem[i] : -1;
    }
    int rc = build_ptab(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->st));
    return 0;
}

static int check_place_args(fit_ctx* c, int32_t j, const void* a, const void* b, const void* d,
                            const void* e, const void* f, int32_t kmax, const void* out) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (!c->have_nodes) return fail(FIT_E_STATE, "fit_load_nodes not called");
    if (j < 0 || (j > 0 && (!a || !b || !d || !e || !f || !out)))
        return fail(FIT_E_INVAL, "bad job arrays");
    if (kmax < 1 || kmax > FIT_MAX_K)
        return fail(FIT_E_INVAL, "kmax=%d outside [1, %d]", kmax, FIT_MAX_K);
    return 0;
}

// fit_place copies a batch of at most this many jobs as one packed transfer
constexpr int32_t kPackJobs = 16384;

int fit_place(fit_ctx* c, int32_t j, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
              const int32_t* wall, const uint16_t* part, const uint16_t* nk, int32_t kmax,
              int32_t* out, fit_stats* stats) {
    int rc = check_place_args(c, j, cpu, mem, gpu, wall, part, kmax, out);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    // demands >= 0 and nodes_k <= kmax are checked on the device (k_prefilter): FIT_E_INVAL
    size_t m = std::max(j, 1);
    // the out buffer's tail holds the direct placement's stats (place_direct: one copy back)
    if (c->out.ensure(m * kmax + 2 + FIT_MAX_PARTITIONS + 1)) return FIT_E_OOM;
    if (c->small_args && j <= SMALL_ARGJ && j <= c->small_direct && !c->collective()) {
        // the batch in k_small's kernel arguments: no copy to the device at all
        SmallBatch hb;
        memcpy(hb.cpu, cpu, sizeof(int32_t) * j);
        memcpy(hb.mem, mem, sizeof(int32_t) * j);
        memcpy(hb.gpu, gpu, sizeof(int32_t) * j);
        memcpy(hb.wall, wall, sizeof(int32_t) * j);
        memcpy(hb.part, part, sizeof(uint16_t) * j);
        if (nk) memcpy(hb.nk, nk, sizeof(uint16_t) * j);
        bool done = false;
        rc = place_impl(c, j, nullptr, nullptr, nullptr, nullptr, nullptr, nk, kmax, c->out.p, stats, out, &done,
                        &hb);
        if (rc) return rc;
        if (!done) return fail(FIT_E_HIP, "direct placement did not return its placements");
        return 0;
    }
    const int32_t *dcpu, *dmem, *dgpu, *dwall;
    const uint16_t *dpart, *dk = nullptr;
    const size_t b = sizeof(int32_t) * j, bh = sizeof(uint16_t) * j;
    if (j <= kPackJobs) {
        // a small batch (admission): the columns packed in pinned memory, ONE copy to the device
        // (the previous call's copy is complete: every fit_place ends with a synchronisation)
        const size_t bh4 = (bh + 3) & ~(size_t)3;
        const size_t tot = 4 * b + 2 * bh4;
        if (c->jpack.ensure(tot) || c->h_jpack.ensure(tot)) return FIT_E_OOM;
        uint8_t* h = c->h_jpack.p;
        memcpy(h, cpu, b);
        memcpy(h + b, mem, b);
        memcpy(h + 2 * b, gpu, b);
        memcpy(h + 3 * b, wall, b);
        memcpy(h + 4 * b, part, bh);
        if (nk) memcpy(h + 4 * b + bh4, nk, bh);
        HIP_TRY(hipMemcpyAsync(c->jpack.p, h, nk ? tot : 4 * b + bh4, hipMemcpyHostToDevice, c->st));
        uint8_t* d = c->jpack.p;
        dcpu = (const int32_t*)d;
        dmem = (const int32_t*)(d + b);
        dgpu = (const int32_t*)(d + 2 * b);
        dwall = (const int32_t*)(d + 3 * b);
        dpart = (const uint16_t*)(d + 4 * b);
        if (nk) dk = (const uint16_t*)(d + 4 * b + bh4);
    } else {
        if (c->jcpu.ensure(m) || c->jmem.ensure(m) || c->jgpu.ensure(m) || c->jwall.ensure(m) ||
            c->jpart.ensure(m) || c->jk.ensure(m))
            return FIT_E_OOM;
        HIP_TRY(hipMemcpyAsync(c->jcpu.p, cpu, b, hipMemcpyHostToDevice, c->st));
        HIP_TRY(hipMemcpyAsync(c->jmem.p, mem, b, hipMemcpyHostToDevice, c->st));
        HIP_TRY(hipMemcpyAsync(c->jgpu.p, gpu, b, hipMemcpyHostToDevice, c->st));
        HIP_TRY(hipMemcpyAsync(c->jwall.p, wall, b, hipMemcpyHostToDevice, c->st));
        HIP_TRY(hipMemcpyAsync(c->jpart.p, part, bh, hipMemcpyHostToDevice, c->st));
        if (nk) HIP_TRY(hipMemcpyAsync(c->jk.p, nk, bh, hipMemcpyHostToDevice, c->st));
        dcpu = c->jcpu.p;
        dmem = c->jmem.p;
        dgpu = c->jgpu.p;
        dwall = c->jwall.p;
        dpart = c->jpart.p;
        if (nk) dk = c->jk.p;
    }
    bool done = false;
    rc = place_impl(c, j, dcpu, dmem, dgpu, dwall, dpart, dk, kmax, c->out.p, stats, out, &done);
    if (rc) return rc;
    if (done) return 0;  // the direct small placement copied the placements back with its stats
    HIP_TRY(hipMemcpyAsync(out, c->out.p, sizeof(int32_t) * j * kmax, hipMemcpyDeviceToHost,
                           c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return 0;
}

int fit_place_device(fit_ctx* c, int32_t j, const int32_t* cpu, const int32_t* mem,
                     const int32_t* gpu, const int32_t* wall, const uint16_t* part,
                     const uint16_t* nk, int32_t kmax, int32_t* out, fit_stats* stats) {
    int rc = check_place_args(c, j, cpu, mem, gpu, wall, part, kmax, out);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    rc = place_impl(c, j, cpu, mem, gpu, wall, part, nk, kmax, out, stats);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->st));
    return 0;
}

int fit_read_nodes(fit_ctx* c, int32_t* cpu, int32_t* mem, int32_t* gpu) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (!c->have_nodes) return fail(FIT_E_STATE, "fit_load_nodes not called");
    if (c->n > 0 && (!cpu || !mem || !gpu)) return fail(FIT_E_INVAL, "null output");
    HIP_TRY(hipSetDevice(c->device));
    // scatter into scratch columns seeded with the loaded table: col_* must keep the table of
    // the last fit_load_nodes (fit_load_timeline builds slot 0 from it), whatever was queried
    const size_t b = sizeof(int32_t) * c->n;
    const size_t m = std::max<int32_t>(c->n, 1);
    if (c->rb_cpu.ensure(m) || c->rb_mem.ensure(m) || c->rb_gpu.ensure(m)) return FIT_E_OOM;
    HIP_TRY(hipMemcpyAsync(c->rb_cpu.p, c->col_cpu.p, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->rb_mem.p, c->col_mem.p, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->rb_gpu.p, c->col_gpu.p, b, hipMemcpyDeviceToDevice, c->st));
    HIP_TRY(launch_scatter_nodes(c->st, c->rec.p, c->nn, c->rb_cpu.p, c->rb_mem.p, c->rb_gpu.p));
    HIP_TRY(hipMemcpyAsync(cpu, c->rb_cpu.p, b, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipMemcpyAsync(mem, c->rb_mem.p, b, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipMemcpyAsync(gpu, c->rb_gpu.p, b, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return 0;
}

int fit_partition_free(fit_ctx* c, int32_t p, int64_t* cpu, int64_t* mem, int64_t* gpu) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (p < 0 || p >= 32 || !cpu || !mem || !gpu) return fail(FIT_E_INVAL, "bad partition");
    std::vector<int32_t> hc(c->n), hm(c->n), hg(c->n);
    int rc = fit_read_nodes(c, hc.data(), hm.data(), hg.data());
    if (rc) return rc;
    int64_t sc = 0, sm = 0, sg = 0;
    for (int32_t x = 0; x < c->n; ++x)
        if ((c->h_mask[x] >> p) & 1u) {
            sc += std::max(hc[x], 0);
            sm += std::max(hm[x], 0);
            sg += std::max(hg[x], 0);
        }
    *cpu = sc;
    *mem = sm;
    *gpu = sg;
    return 0;
}

int fit_load_timeline(fit_ctx* c, int32_t slots, int32_t slot_min, const int32_t* rel_off,
                      const int32_t* rel_slot, const int32_t* rel_cpu, const int32_t* rel_mem,
                      const int32_t* rel_gpu) {
    int rc = check_timeline_args(c, slots, slot_min);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    int64_t ne = 0;
    if (rel_off) {
        if (rel_off[0] != 0) return fail(FIT_E_INVAL, "rel_off[0] must be 0");
        for (int32_t x = 0; x < c->n; ++x)
            if (rel_off[x + 1] < rel_off[x]) return fail(FIT_E_INVAL, "rel_off decreases at %d", x);
        ne = rel_off[c->n];
        if (ne > 0 && (!rel_slot || !rel_cpu || !rel_mem || !rel_gpu))
            return fail(FIT_E_INVAL, "null release arrays");
    }
    if (c->rel_off.ensure(c->n + 1) || c->rel_slot.ensure(std::max<int64_t>(ne, 1)) ||
        c->rel_cpu.ensure(std::max<int64_t>(ne, 1)) || c->rel_mem.ensure(std::max<int64_t>(ne, 1)) ||
        c->rel_gpu.ensure(std::max<int64_t>(ne, 1)))
        return FIT_E_OOM;
    if (rel_off) {
        HIP_TRY(hipMemcpyAsync(c->rel_off.p, rel_off, sizeof(int32_t) * (c->n + 1),
                               hipMemcpyHostToDevice, c->st));
        if (ne > 0) {
            const size_t b = sizeof(int32_t) * ne;
            HIP_TRY(hipMemcpyAsync(c->rel_slot.p, rel_slot, b, hipMemcpyHostToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->rel_cpu.p, rel_cpu, b, hipMemcpyHostToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->rel_mem.p, rel_mem, b, hipMemcpyHostToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->rel_gpu.p, rel_gpu, b, hipMemcpyHostToDevice, c->st));
        }
    }
    return load_timeline_impl(c, slots, slot_min, rel_off ? ne : -1);
}

int fit_load_timeline_device(fit_ctx* c, int32_t slots, int32_t slot_min, const int32_t* rel_off,
                             int64_t n_rel, const int32_t* rel_slot, const int32_t* rel_cpu,
                             const int32_t* rel_mem, const int32_t* rel_gpu) {
    int rc = check_timeline_args(c, slots, slot_min);
    if (rc) return rc;
    if (n_rel < 0 || (n_rel > 0 && (!rel_off || !rel_slot || !rel_cpu || !rel_mem || !rel_gpu)))
        return fail(FIT_E_INVAL, "bad release arrays");
    HIP_TRY(hipSetDevice(c->device));
    if (c->rel_off.ensure(c->n + 1) || c->rel_slot.ensure(std::max<int64_t>(n_rel, 1)) ||
        c->rel_cpu.ensure(std::max<int64_t>(n_rel, 1)) ||
        c->rel_mem.ensure(std::max<int64_t>(n_rel, 1)) || c->rel_gpu.ensure(std::max<int64_t>(n_rel, 1)))
        return FIT_E_OOM;
    if (rel_off) {
        HIP_TRY(hipMemcpyAsync(c->rel_off.p, rel_off, sizeof(int32_t) * (c->n + 1),
                               hipMemcpyDeviceToDevice, c->st));
        if (n_rel > 0) {
            const size_t b = sizeof(int32_t) * n_rel;
            HIP_TRY(hipMemcpyAsync(c->rel_slot.p, rel_slot, b, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->rel_cpu.p, rel_cpu, b, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->rel_mem.p, rel_mem, b, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(c->rel_gpu.p, rel_gpu, b, hipMemcpyDeviceToDevice, c->st));
        }
    }
    return load_timeline_impl(c, slots, slot_min, rel_off ? n_rel : -1);
}

static int check_place_tl_args(fit_ctx* c, int32_t j, const void* a, const void* b,
                               const void* d, const void* e, const void* f, const void* out,
                               const void* outs) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (!c->have_nodes) return fail(FIT_E_STATE, "fit_load_nodes not called");
    if (!c->have_tl) return fail(FIT_E_STATE, "fit_load_timeline not called");
    if (j < 0 || (j > 0 && (!a || !b || !d || !e || !f || !out || !outs)))
        return fail(FIT_E_INVAL, "bad job arrays");
    return 0;
}

int fit_place_tl(fit_ctx* c, int32_t j, const int32_t* cpu, const int32_t* mem,
                 const int32_t* gpu, const int32_t* wall, const uint16_t* part, int32_t* out_node,
                 int32_t* out_start, fit_stats* stats) {
    int rc = check_place_tl_args(c, j, cpu, mem, gpu, wall, part, out_node, out_start);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    // demands >= 0 are checked on the device (k_prefilter): FIT_E_INVAL
    size_t m = std::max(j, 1);
    if (c->jcpu.ensure(m) || c->jmem.ensure(m) || c->jgpu.ensure(m) || c->jwall.ensure(m) ||
        c->jpart.ensure(m) || c->out.ensure(m) || c->outs.ensure(m))
        return FIT_E_OOM;
    const size_t b = sizeof(int32_t) * j;
    HIP_TRY(hipMemcpyAsync(c->jcpu.p, cpu, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->jmem.p, mem, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->jgpu.p, gpu, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->jwall.p, wall, b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipMemcpyAsync(c->jpart.p, part, sizeof(uint16_t) * j, hipMemcpyHostToDevice, c->st));
    rc = place_tl_impl(c, j, c->jcpu.p, c->jmem.p, c->jgpu.p, c->jwall.p, c->jpart.p, c->out.p,
                       c->outs.p, stats);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out_node, c->out.p, b, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipMemcpyAsync(out_start, c->outs.p, b, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return 0;
}

int fit_place_tl_device(fit_ctx* c, int32_t j, const int32_t* cpu, const int32_t* mem,
                        const int32_t* gpu, const int32_t* wall, const uint16_t* part,
                        int32_t* out_node, int32_t* out_start, fit_stats* stats) {
    int rc = check_place_tl_args(c, j, cpu, mem, gpu, wall, part, out_node, out_start);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    rc = place_tl_impl(c, j, cpu, mem, gpu, wall, part, out_node, out_start, stats);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->st));
    return 0;
}

int fit_read_timeline(fit_ctx* c, int32_t* cpu, int32_t* mem, int32_t* gpu) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (!c->have_tl) return fail(FIT_E_STATE, "fit_load_timeline not called");
    if (c->n > 0 && (!cpu || !mem || !gpu)) return fail(FIT_E_INVAL, "null output");
    HIP_TRY(hipSetDevice(c->device));
    const size_t cells = (size_t)c->n * c->tl_slots;
    DBuf<int32_t> d[3];
    for (auto& x : d)
        if (x.ensure(std::max<size_t>(cells, 1))) {
            for (auto& y : d) y.release();
            return FIT_E_OOM;
        }
    // rows of nodes outside every partition (mask 0) are not on the device: -1, like unusable
    int rc = 0;
    for (auto& x : d)
        if (hipMemsetAsync(x.p, 0xff, sizeof(int32_t) * cells, c->st) != hipSuccess) rc = FIT_E_HIP;
    if (rc || launch_expand_tl(c->st, c->perm.p, c->slab.p, c->tlhdr.p, c->nn, c->tl_slots, d[0].p,
                         d[1].p, d[2].p) != hipSuccess ||
        hipMemcpyAsync(cpu, d[0].p, sizeof(int32_t) * cells, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipMemcpyAsync(mem, d[1].p, sizeof(int32_t) * cells, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipMemcpyAsync(gpu, d[2].p, sizeof(int32_t) * cells, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess)
        rc = fail(FIT_E_HIP, "timeline read-back failed");
    for (auto& x : d) x.release();
    return rc;
}

}  // extern "C"

namespace fitgpu {
void set_last_error(const char* msg) { g_last_error = msg; }  // admit.cpp: the batch's error

// admit.cpp: the context's table as the admitter's host copy starts from it (a table loaded with
// fit_load_nodes directly, before the admitter manages it).  Free columns as fit_read_nodes
// gives them (current, after placements); avail / mask as loaded.
int64_t ctx_load_count(const fit_ctx* c) { return c && c->have_nodes ? c->loads : 0; }
int ctx_table(fit_ctx* c, std::vector<int32_t>& cpu, std::vector<int32_t>& mem,
              std::vector<int32_t>& gpu, std::vector<int32_t>& avail, std::vector<uint32_t>& mask) {
    if (!c) return fail(FIT_E_INVAL, "null ctx");
    if (!c->have_nodes) return fail(FIT_E_STATE, "no node table loaded");
    const size_t m = std::max<int32_t>(c->n, 1);
    cpu.resize(m), mem.resize(m), gpu.resize(m), avail.resize(m);
    const int rc = fit_read_nodes(c, cpu.data(), mem.data(), gpu.data());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(avail.data(), c->col_av.p, sizeof(int32_t) * c->n, hipMemcpyDeviceToHost));
    cpu.resize(c->n), mem.resize(c->n), gpu.resize(c->n), avail.resize(c->n);
    mask = c->h_mask;
    return 0;
}
}  // namespace fitgpu
