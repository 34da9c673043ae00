// fit_commit_mw.h — the commit of one component's window by a whole 8-wave workgroup
// (DESIGN.md §3.7): one DECIDER wave walks the jobs in priority order; seven HELPER waves
// pre-resolve the jobs ahead of it against a slightly stale snapshot of the dirty state.
//
// Why it is exact.  Let the decider have resolved jobs [0, v) when a helper snapshots the
// state for job t (v >= t - (MW_M - 1), enforced by the helper).  The helper records the MW_M
// smallest keys <= B among (clean candidates of t) ∪ (dirty rows), each item tagged clean (with
// its node row) or dirty (its slot).  When the decider reaches t, only the nodes written by jobs
// [v, t) — at most MW_M - 1 of them, the decider's own last decisions — can differ from the
// snapshot.  It drops every listed item whose node is among them (a clean node since marked in
// the bitmap, a dirty slot whose version is >= v) and re-evaluates those nodes at their current
// state.  If the list held MW_M items, at least one survives and every unlisted node has a key
// above it; if it held fewer, it held every candidate <= B.  Either way
//     best = min(surviving items, re-evaluated nodes)
// is the sequential answer restricted to keys <= B, and the SPEC stop rule reduces to
// "best > B with B finite" (a clean candidate is always <= B).  No fallback path exists.
//
// LDS protocol (one workgroup): DS instructions of a wave execute in issue order, so plain
// stores followed by a flag store are seen in that order by a wave that read the flag first;
// the fences below are compiler barriers only.
#pragma once
#include "fit_common.h"

namespace fitgpu {

#ifndef MW_ITEMS
#define MW_ITEMS 8
#endif
constexpr int MW_M = MW_ITEMS;          // items per pre-resolved record (> snapshot lag)
constexpr int MW_R = 8;                 // record ring; slot t & 7 frees once job t-8 is decided
constexpr int MW_WAVES = SCAN_WAVES;    // 1 decider [+ 1 recorder] + MW_H helpers
// MW_RECORDER: wave 1 is the RECORDER — it takes the decider's decisions from a small LDS queue
// and does their bookkeeping (dirty row, bitmap, placement, the {decided, nu} publish), which
// leaves the decider's serial chain with the decision itself.  0: the decider does both.
#ifndef MW_RECORDER
#ifdef MW_DECIDER_BENCH
#define MW_RECORDER 0
#else
#define MW_RECORDER 1
#endif
#endif
#ifndef MW_HELPERS
#define MW_HELPERS (MW_RECORDER ? 6 : 7)
#endif
constexpr int MW_H = MW_HELPERS;  // waves 1 + MW_RECORDER .. MW_RECORDER + MW_H
static_assert(MW_H + 1 + MW_RECORDER <= MW_WAVES, "one wave per role");
constexpr int MW_DQ = 16;         // decision queue (decider -> recorder)

constexpr unsigned MW_SPIN_LIMIT = 1u << 24;
#ifndef MW_HSLEEP
#define MW_HSLEEP 2
#endif
constexpr int MW_EPL = (MAX_SLICES * KS + 63) / 64;  // candidate entries per helper lane
static_assert(MW_EPL <= 2, "at most two candidate entries per lane");
static_assert(MW_R >= MW_M, "record slot reuse relies on the lag bound");

struct alignas(16) MwRow {  // dirty row, current state
    int32_t cpu, mem, gpu, avail;
    uint32_t mask, pos;
    int32_t orig, ver;  // ver: last job (window index) that created or changed it
};

struct alignas(16) MwItem {
    uint64_t key;
    int32_t tag;   // >= 0 dirty slot; -1 clean candidate (row below)
    int32_t orig;
    int32_t cpu, mem, gpu, avail;
    uint32_t mask, pad0, pad1, pad2;
};

struct alignas(16) MwHdr {
    uint32_t ready;  // t + 1 once the record of job t is complete
    int32_t v, n, q;
    int32_t cpu, mem, gpu, wall;
    uint32_t pbit, pad;
    uint64_t B;
};

struct alignas(16) MwRec {
    MwHdr h;
    MwItem it[MW_M];
};

struct alignas(16) MwShared {
    uint32_t decided;  // jobs resolved by the decider
    uint32_t nu;       // dirty rows (stored together with decided)
    uint32_t halt;     // decider stopped early
    uint32_t fail;     // helper / decider watchdog
    int32_t res[4];    // CommitResult of the window
    uint32_t pad[8];
    MwRec rec[MW_R];
    uint4 dq[MW_DQ];  // decision of job t in dq[t % MW_DQ]: {t + 1, winner, slot, 0}
    MwRow rows[UCAP];
    uint32_t bitmap[1];  // (ne - nb + 31) / 32 words, dirty membership by position
};

__host__ __device__ constexpr size_t mw_lds_bytes(int32_t max_component_nodes) {
    return sizeof(MwShared) + (size_t)((max_component_nodes + 31) / 32) * 4;
}

#ifdef FIT_STAMPS
// [comp][0] decider cycles, [1] decider wait-for-record, [2] decided jobs,
// [3] helper cycles (sum), [4] helper wait-for-snapshot, [5] helper jobs, [6] items written,
// [7] decider check+reduce, [8] decider decide+publish, [9] waits of each round's first jobs,
// [10..12] first-tile scan (workers), [13] helper tile waits, [14] helper snapshot → record,
// [15] helper snapshot → extraction start, [16] decider: records not ready at the first read,
// [17] recorder cycles, [18] recorder waiting for decisions, [19] recorder jobs
constexpr int MW_NSTAMP = 24;
__device__ unsigned long long g_mw[64][MW_NSTAMP];
#define MW_CLK(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define MW_DECL(v) unsigned long long v = 0
#define MW_ACC(v, x) v += (x)
#define MW_ADD(I_, V_) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_mw[blockIdx.x & 63][I_], (unsigned long long)(V_)); } while (0)
#else
#define MW_CLK(v)
#define MW_DECL(v)
#define MW_ACC(v, x)
#define MW_ADD(I_, V_)
#endif

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cbar() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); }

// Tile readiness: the window's scan tiles complete while the window is being
// committed; a helper waits for the (job tile)'s per-tile counter to reach nslice before reading
// that tile's candidates, bound and job row; an agent-scope acquire when a tile turns ready drops
// the CU's L1 (it may hold stale lines of these reused buffers), so the reads stay plain loads.
// tdone == nullptr: the whole window was acquired before the commit (no waits).
struct MwTiles {
    const unsigned* tdone;  // per-tile completed slice counts of this component's window
    unsigned need;          // nslice
};

// global address-space views of the helper's buffers: a plain (generic) pointer in a non-inlined
// function compiles to flat loads, which also count in lgkmcnt — every LDS wait would then drain
// the prefetched job stream
#define GAS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ const GAS T* gview(const T* p) {
    return (const GAS T*)p;
}

typedef int32_t v4i32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ NodeRec ld_node(const GAS NodeRec* p) {
    const GAS v4i32* q = (const GAS v4i32*)p;
    const v4i32 a = q[0], b = q[1];
    NodeRec r;
    r.cpu = a.x;
    r.mem = a.y;
    r.gpu = a.z;
    r.avail = a.w;
    r.mask = (uint32_t)b.x;
    r.orig = b.y;
    r.pad0 = b.z;
    r.pad1 = b.w;
    return r;
}

__device__ __forceinline__ JobRec ld_job(const GAS JobRec* p) {
    const GAS v4i32* q = (const GAS v4i32*)p;
    const v4i32 a = q[0], b = q[1];
    JobRec r;
    r.q = a.x;
    r.cpu = a.y;
    r.mem = a.z;
    r.gpu = a.w;
    r.wall = b.x;
    r.pbit = (uint32_t)b.y;
    r.k = b.z;
    r.pad = b.w;
    return r;
}

// a VGPR zero the compiler cannot see through: keeps uniform loads of data written by other
// workgroups in this launch on the vector path (vmcnt, in order) instead of the scalar cache
__device__ __forceinline__ int opaque_zero() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

// A dynamic-LDS pointer the compiler cannot re-derive: in an out-of-line function the constant
// shared base is otherwise rematerialised from the dynlds offset table (an s_load + lgkmcnt(0)
// wait) on every loop iteration; laundered through an SGPR it is computed once.  The round trip
// through address space 3 keeps every access a ds_* instruction.
template <class T>
__device__ __forceinline__ T* lds_opaque(T* p) {
    uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p;
    asm volatile("" : "+s"(a));
    return (T*)(__attribute__((address_space(3))) T*)(uintptr_t)a;
}

// The plan copied into SGPRs: an out-of-line function receives it through a generic pointer, and
// fields loaded that way sit in VGPRs, so the compiler cannot prove the job loop uniform (it
// would run it under exec masks with its counter in a VGPR).
__device__ __forceinline__ int32_t rfl(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ CompPlan plan_sgpr(const CompPlan& q) {
    CompPlan p;
    p.nb = rfl(q.nb);
    p.ne = rfl(q.ne);
    p.sb = rfl(q.sb);
    p.se = rfl(q.se);
    p.nslice = rfl(q.nslice);
    p.sub = rfl(q.sub);
    p.jbase = rfl(q.jbase);
    p.w = rfl(q.w);
    p.blk0 = rfl(q.blk0);
    p.cand_off = (int64_t)(((uint64_t)(uint32_t)rfl((int32_t)(q.cand_off >> 32)) << 32) |
                           (uint32_t)rfl((int32_t)q.cand_off));
    p.slot0 = rfl(q.slot0);
    return p;
}

__device__ __forceinline__ uint64_t mw_key(int32_t cf, int32_t mf, int32_t gf, int32_t av,
                                           uint32_t mask, uint32_t pos, int32_t jc, int32_t jm,
                                           int32_t jg, int32_t jw, uint32_t jp) {
    const int32_t dc = cf - jc, dm = mf - jm, dg = gf - jg, da = av - jw;
    const bool ok = (dc | dm | dg | da) >= 0 && (mask & jp);
    const uint32_t sc = (min((uint32_t)dg, 255u) << 24) | (min((uint32_t)dc, 4095u) << 12) |
                        min((uint32_t)dm >> 10, 4095u);
    return ok ? (((uint64_t)sc << 32) | pos) : KEY_INF;
}

// Helper entry lists: MW_EPL clean candidates + UPL dirty rows per lane, each key tagged with
// its entry index in the low bits (positions < 2^29, FIT_MAX_NODES), INF stays INF.
constexpr int MW_NE = MW_EPL + UPL;
static_assert(MW_NE <= 8, "entry index takes 3 bits (and 4 bits of item index each in 32)");
static_assert(MW_M <= 15, "item index + 1 fits 4 bits");
__device__ __forceinline__ uint64_t mw_tag(uint64_t k, int e) {
    return k == KEY_INF ? KEY_INF
                        : (k & 0xffffffff00000000ull) | (uint32_t)(((uint32_t)k << 3) | (uint32_t)e);
}
__device__ __forceinline__ void mw_cas(uint64_t& a, uint64_t& b) {
    const uint64_t lo = umin64(a, b), hi = umax64(a, b);
    a = lo;
    b = hi;
}
// ascending sort of a lane's entries (static indices only): the 12-comparator network for 6,
// odd-even transposition otherwise
template <int N>
__device__ __forceinline__ void mw_sort(uint64_t (&q)[N]) {
    if constexpr (N == 6) {
        mw_cas(q[0], q[5]); mw_cas(q[1], q[3]); mw_cas(q[2], q[4]);
        mw_cas(q[1], q[2]); mw_cas(q[3], q[4]);
        mw_cas(q[0], q[3]); mw_cas(q[2], q[5]);
        mw_cas(q[0], q[1]); mw_cas(q[2], q[3]); mw_cas(q[4], q[5]);
        mw_cas(q[1], q[2]); mw_cas(q[3], q[4]);
    } else {
#pragma unroll
        for (int r = 0; r < N; ++r)
#pragma unroll
            for (int i = r & 1; i + 1 < N; i += 2) mw_cas(q[i], q[i + 1]);
    }
}

// Wait until job tt's scan tile is complete (uniform; `ready` = tiles known complete, they finish
// roughly in order).  false: the decider halted / a watchdog tripped.
__device__ __forceinline__ bool mw_tile_ready(const MwTiles& T, int tt, int& ready, MwShared* S) {
    if (!T.tdone) return true;
    const int tile = __builtin_amdgcn_readfirstlane(tt) / SCAN_JOBS;
    if (tile < ready) return true;
    for (unsigned sp = 0;; ++sp) {
        if (__hip_atomic_load(gview(T.tdone) + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
            T.need)
            break;
        if (lds_ld(&S->halt) | lds_ld(&S->fail)) return false;
        if (sp > MW_SPIN_LIMIT) {
            lds_st(&S->fail, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ready = tile + 1;
    return true;
}

// ------------------------------------------------------------------------------- helper
// Helper h (1..MW_H) pre-resolves jobs t = h-1, h-1+MW_H, ...  Loads run two jobs ahead (keys,
// job row, bound) and one job ahead (the node rows of the candidates); the three register sets
// are indexed by literal constants only (3-way unrolled loop).
#define MW_HSTEP(A, B_, C)                                                                     \
    {                                                                                          \
        if (t >= P.w) goto hdone;                                                              \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) { /* job t+H's candidates' rows */ \
            const uint64_t k_ = kk[B_][e];                                                     \
            const uint32_t p_ = k_ != KEY_INF ? (uint32_t)k_ : (uint32_t)P.nb;                 \
            const NodeRec r_ = ld_node(rec + p_);                                              \
            rc[B_][e] = r_.cpu;                                                                \
            rm[B_][e] = r_.mem;                                                                \
            rg[B_][e] = r_.gpu;                                                                \
            ra[B_][e] = r_.avail;                                                              \
            rk[B_][e] = r_.mask;                                                               \
            ro[B_][e] = r_.orig;                                                               \
        }                                                                                      \
        {                                                                                      \
            const int tt_ = min(t + 2 * MW_H, wlast) + z;                                      \
            MW_CLK(tw0_);                                                                      \
            if (!mw_tile_ready(T, tt_, ready, S)) goto hdone;                                  \
            {                                                                                  \
                MW_CLK(tw1_);                                                                  \
                MW_ACC(a_ht, tw1_ - tw0_);                                                     \
            }                                                                                  \
            _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e)                                  \
                kk[C][e] = has[e] ? cand[eoff[e] + (int64_t)tt_ * E] : KEY_INF;                \
            jr[C] = ld_job(wjob + P.slot0 + tt_);                                              \
            jbd[C] = bnd[P.slot0 + tt_];                                                       \
        }                                                                                      \
        /* snapshot: the decider has resolved at least t - (MW_M - 1) jobs */                  \
        uint32_t v_;                                                                           \
        MW_CLK(hw0_);                                                                          \
        for (unsigned sp_ = 0;; ++sp_) {                                                       \
            v_ = lds_ld(&S->decided);                                                          \
            if ((int)v_ + (MW_M - 1) >= t) break;                                              \
            if (lds_ld(&S->halt) | lds_ld(&S->fail)) goto hdone;                               \
            if (sp_ > MW_SPIN_LIMIT) {                                                         \
                lds_st(&S->fail, 1u);                                                          \
                goto hdone;                                                                    \
            }                                                                                  \
            __builtin_amdgcn_s_sleep(MW_HSLEEP); /* keep the LDS free for the decider */       \
        }                                                                                      \
        /* the snapshot's row / bitmap reads are issued after the flag read that admitted it */ \
        asm volatile("" ::: "memory");                                                         \
        {                                                                                      \
            MW_CLK(hw1_);                                                                      \
            MW_ACC(a_hw, hw1_ - hw0_);                                                         \
            MW_ACC(a_hp, -(long long)hw1_);                                                    \
            MW_ACC(a_hx, -(long long)hw1_);                                                    \
        }                                                                                      \
        const int nu_ = (int)lds_ld(&S->nu);                                                   \
        const JobRec& J_ = jr[A];                                                              \
        const uint64_t Bd_ = jbd[A];                                                           \
        uint64_t x0[MW_EPL];                                                                   \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) {                                   \
            const uint64_t k_ = kk[A][e];                                                      \
            const bool ok_ = k_ <= Bd_ && k_ != KEY_INF;                                       \
            const uint32_t rel_ = ok_ ? (uint32_t)k_ - (uint32_t)P.nb : 0u;                    \
            const bool dirty_ = (S->bitmap[rel_ >> 5] >> (rel_ & 31)) & 1u;                    \
            x0[e] = ok_ && !dirty_ ? k_ : KEY_INF;                                             \
        }                                                                                      \
        uint64_t xd[UPL];                                                                      \
        MwRow wr_[UPL];                                                                        \
        _Pragma("unroll") for (int i = 0; i < UPL; ++i) {                                      \
            xd[i] = KEY_INF;                                                                   \
            const int u_ = i * 64 + lane;                                                      \
            if (i * 64 < nu_) {                                                                \
                wr_[i] = S->rows[u_ < nu_ ? u_ : 0];                                           \
                const uint64_t y_ = mw_key(wr_[i].cpu, wr_[i].mem, wr_[i].gpu, wr_[i].avail,   \
                                           wr_[i].mask, wr_[i].pos, J_.cpu, J_.mem, J_.gpu,    \
                                           J_.wall, J_.pbit);                                  \
                xd[i] = u_ < nu_ && y_ <= Bd_ ? y_ : KEY_INF;                                  \
            }                                                                                  \
        }                                                                                      \
        MwRec* R_ = &S->rec[t & (MW_R - 1)];                                                   \
        int n_ = 0;                                                                            \
        {                                                                                      \
            MW_CLK(hx_);                                                                       \
            MW_ACC(a_hx, hx_);                                                                 \
        }                                                                                      \
        /* every entry tagged with its index (pos << 3 | e keeps the order of distinct nodes) and\
           sorted per lane once; each extraction is then one wave minimum over the lane heads  \
           plus a predicated shift in the winning lane, and the items are written in one pass */\
        uint64_t q_[MW_NE];                                                                    \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) q_[e] = mw_tag(x0[e], e);           \
        _Pragma("unroll") for (int i = 0; i < UPL; ++i) q_[MW_EPL + i] = mw_tag(xd[i], MW_EPL + i);\
        mw_sort(q_);                                                                           \
        /* item index + 1 of each entry, 4 bits per entry (0: not taken) */                    \
        uint32_t sel_ = 0u;                                                                    \
        /* at most t - v nodes can change before job t is decided: t - v + 1 items suffice */  \
        const int nmax_ = rfl(min(MW_M, t - (int)v_ + 1));                                     \
        for (; n_ < nmax_; ++n_) {                                                             \
            int wl_;                                                                           \
            const uint64_t best_ = wave_min_key_lane(q_[0], wl_);                              \
            if (best_ == KEY_INF) break;                                                       \
            const bool me_ = lane == wl_;                                                      \
            const uint32_t sv_ = (uint32_t)(n_ + 1) << (4u * ((uint32_t)best_ & 7u));          \
            sel_ = me_ ? sel_ | sv_ : sel_;                                                    \
            _Pragma("unroll") for (int e = 0; e + 1 < MW_NE; ++e)                              \
                q_[e] = me_ ? q_[e + 1] : q_[e];                                               \
            q_[MW_NE - 1] = me_ ? KEY_INF : q_[MW_NE - 1];                                     \
        }                                                                                      \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) if ((sel_ >> (4 * e)) & 15u)        \
            R_->it[((sel_ >> (4 * e)) & 15u) - 1u] = MwItem{x0[e], -1, ro[A][e], rc[A][e], rm[A][e], rg[A][e], ra[A][e],\
                                     rk[A][e], 0, 0, 0};                                       \
        _Pragma("unroll") for (int i = 0; i < UPL; ++i) if ((sel_ >> (4 * (MW_EPL + i))) & 15u) \
            R_->it[((sel_ >> (4 * (MW_EPL + i))) & 15u) - 1u] = MwItem{xd[i], i * 64 + lane, wr_[i].orig, wr_[i].cpu,   \
                                              wr_[i].mem, wr_[i].gpu, wr_[i].avail, wr_[i].mask,\
                                              0, 0, 0};                                        \
        if (lane == 0) {                                                                       \
            R_->h.cpu = J_.cpu;                                                                \
            R_->h.mem = J_.mem;                                                                \
            R_->h.gpu = J_.gpu;                                                                \
            R_->h.wall = J_.wall;                                                              \
            R_->h.pbit = J_.pbit;                                                              \
            R_->h.B = Bd_;                                                                     \
            cbar();                                                                            \
            /* {ready, v, n, q}: one 16-byte store, after everything else of the record */     \
            *reinterpret_cast<uint4*>(&R_->h) =                                                \
                make_uint4((uint32_t)t + 1u, v_, (uint32_t)n_, (uint32_t)J_.q);                 \
        }                                                                                      \
        {                                                                                      \
            MW_CLK(hp1_);                                                                      \
            MW_ACC(a_hp, hp1_);                                                                \
        }                                                                                      \
        MW_ACC(a_hn, 1);                                                                       \
        MW_ACC(a_hi, n_);                                                                      \
        t += MW_H;                                                                             \
    }

__device__ __noinline__ void mw_helper(const CompPlan& Pref, MwShared* Sin,
                                          const NodeRec* __restrict__ rec_,
                                          const uint64_t* __restrict__ cand_,
                                          const uint64_t* __restrict__ bnd_,
                                          const JobRec* __restrict__ wjob_, int h, MwTiles T) {
    const GAS NodeRec* const rec = gview(rec_);
    const GAS uint64_t* const cand = gview(cand_);
    const GAS uint64_t* const bnd = gview(bnd_);
    const GAS JobRec* const wjob = gview(wjob_);
    // by value: a reference into the caller's stack is re-read (flat load + full vmcnt wait) after
    // every LDS store, which would drain the job-stream prefetch each step
    const CompPlan P = plan_sgpr(Pref);
    MwShared* const S = lds_opaque(Sin);
    const int lane = threadIdx.x & 63;
    const int E = P.nslice * KS;
    bool has[MW_EPL];       // candidate entry lane + 64 e of the job's E entries
    int64_t eoff[MW_EPL];
#pragma unroll
    for (int e = 0; e < MW_EPL; ++e) {
        has[e] = lane + 64 * e < E;
        eoff[e] = P.cand_off + (has[e] ? lane + 64 * e : 0);
    }
    const int wlast = P.w - 1;
    const int z = opaque_zero();
    int t = h - 1;

    uint64_t kk[3][MW_EPL], jbd[3];
    JobRec jr[3];
    int32_t rc[3][MW_EPL], rm[3][MW_EPL], rg[3][MW_EPL], ra[3][MW_EPL], ro[3][MW_EPL];
    uint32_t rk[3][MW_EPL];
    int ready = 0;  // scan tiles known complete
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // jobs t and t + H
        const int tt = min(t + s * MW_H, wlast) + z;
        if (!mw_tile_ready(T, tt, ready, S)) return;  // halted / watchdog
#pragma unroll
        for (int e = 0; e < MW_EPL; ++e)
            kk[s][e] = has[e] ? cand[eoff[e] + (int64_t)tt * E] : KEY_INF;
        jr[s] = ld_job(wjob + P.slot0 + tt);
        jbd[s] = bnd[P.slot0 + tt];
    }
#pragma unroll
    for (int e = 0; e < MW_EPL; ++e) {
        const uint32_t p = kk[0][e] != KEY_INF ? (uint32_t)kk[0][e] : (uint32_t)P.nb;
        const NodeRec r = ld_node(rec + p);
        rc[0][e] = r.cpu;
        rm[0][e] = r.mem;
        rg[0][e] = r.gpu;
        ra[0][e] = r.avail;
        rk[0][e] = r.mask;
        ro[0][e] = r.orig;
    }
    MW_DECL(a_hw);
    MW_DECL(a_hn);
    MW_DECL(a_hi);
    MW_DECL(a_ht);  // waiting for scan tiles (prefetch of job t + 2H)
    MW_DECL(a_hp);  // snapshot → record published
    MW_DECL(a_hx);  // snapshot → extraction start (dirty rows read, candidates filtered)
    MW_CLK(h0);
    for (;;) {
        MW_HSTEP(0, 1, 2)
        MW_HSTEP(1, 2, 0)
        MW_HSTEP(2, 0, 1)
    }
hdone:;
    MW_CLK(h1);
    MW_ADD(3, h1 - h0);
    MW_ADD(4, a_hw);
    MW_ADD(5, a_hn);
    MW_ADD(6, a_hi);
    MW_ADD(13, a_ht);
    MW_ADD(14, a_hp);
    MW_ADD(15, a_hx);
}
#undef MW_HSTEP

// ------------------------------------------------------------------------------ decider
// The "written ring": lane l (and every lane l + 8k) holds the row the decider wrote for the
// last job j ≡ l (mod 8): job index, slot and the row's current fields.  For job t an entry is
// live iff its job >= v (the record's snapshot); live entries are exactly the nodes that may
// differ from the snapshot, so they are re-evaluated and every record item on one of their
// positions is dropped.  When a slot is written again its older entry dies (job = -1), so a live
// entry always holds the slot's current row.  All decision work is VALU on lanes 0..7; the only
// LDS round trip per job is the record read.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_rot(uint32_t v) {  // within a 16-lane row, all valid
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_min8(uint32_t v) { return min(v, dpp_rot<CTRL>(v)); }

// min over lanes 0..7 (valid in every one of them): quad swaps, then half-row mirror
__device__ __forceinline__ uint32_t min8_u32(uint32_t v) {
    v = dpp_min8<0xb1>(v);   // quad_perm [1,0,3,2]
    v = dpp_min8<0x4e>(v);   // quad_perm [2,3,0,1]
    v = dpp_min8<0x141>(v);  // row_half_mirror
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
}

// v_writelane_b32: lane `l` of `old` := SGPR `x` (no clang builtin on this toolchain).  The lane
// select goes through M0 (one SGPR operand per VALU instruction on gfx9).
__device__ __forceinline__ int32_t writelane(int32_t x, int l, int32_t old) {
    int32_t r;
    // readfirstlane: a value the compiler believes divergent would otherwise get a VGPR here
    asm("v_writelane_b32 %0, %1, m0"
        : "=v"(r)
        : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(l), "0"(old));
    return r;
}
__device__ __forceinline__ uint32_t writelane(uint32_t x, int l, uint32_t old) {
    return (uint32_t)writelane((int32_t)x, l, (int32_t)old);
}

// bit 8i of the result is set iff byte i of m is nonzero
__device__ __forceinline__ uint64_t any_in_byte(uint64_t m) {
    m |= m >> 4;
    m |= m >> 2;
    m |= m >> 1;
    return m & 0x0101010101010101ull;
}

// one lane's view of a record: the header (every lane) and item i8 (lanes 8 i8 + r)
__device__ __forceinline__ void mw_read_rec(const MwRec* R, int i8, uint4& h0, uint4& h1,
                                            uint4& h2, uint4& i0, uint4& i1, uint4& i2) {
    // {ready, v, n, q} is one 16-byte LDS store on the helper side (its last); read first
    const uint4* hp = reinterpret_cast<const uint4*>(&R->h);
    const uint4* ip = reinterpret_cast<const uint4*>(&R->it[i8]);
    h0 = hp[0];
    // plain LDS loads may be issued in any order: keep the flag word's read first (the wave's
    // DS instructions then execute in issue order, after the helper's record stores it saw)
    asm volatile("" ::: "memory");
    h1 = hp[1];
    h2 = hp[2];
    i0 = ip[0];
    i1 = ip[1];
    i2 = ip[2];
}

constexpr uint32_t MW_DQ_END = 0xfffffffeu;  // queue entry kind: the decider stopped here

// Wait until the recorder has published job t - MW_DQ (queue entry t % MW_DQ is free).
// false: the watchdog tripped (the failure flag is set).
__device__ __forceinline__ bool mw_dq_space(MwShared* S, int t, int& dseen) {
    for (unsigned sp = 0;; ++sp) {
        dseen = rfl((int)lds_ld(&S->decided));
        if (t < dseen + MW_DQ) return true;
        if (sp > MW_SPIN_LIMIT || rfl((int)lds_ld(&S->fail))) {
            lds_st(&S->fail, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(0);
    }
}

// Out of line (as is mw_helper): called once per round, each gets its own register allocation
// instead of sharing the persistent kernel's (which otherwise spills SGPRs in this loop).
__device__ __noinline__ CommitResult mw_decider(const CompPlan& Pref, MwShared* Sin,
                                                int32_t* __restrict__ out, int kmax) {
    const CompPlan P = plan_sgpr(Pref);  // by value (see mw_helper)
    MwShared* const S = lds_opaque(Sin);
    const int lane = threadIdx.x & 63;
    const int r8 = lane & 7;   // ring entry this lane holds (full row in lanes 0..7 only)
    const int i8 = lane >> 3;  // record item this lane reads: lane 8i + r tests item i vs entry r
    const uint32_t nb = (uint32_t)P.nb;
#ifndef MW_NO_SETPRIO
    __builtin_amdgcn_s_setprio(3);  // shares its SIMD with helper wave 4
#endif
    int nu = 0, placed = 0, stop = 0, t = 0;
    int32_t wj = -1, ws = -1, wc = 0, wm = 0, wg = 0, wa = 0, wo = -1;  // written ring
    uint32_t wk = 0, wp = ~0u;
    int32_t oq = -1, ov = -1;  // placement of job t parked in lane t & 63, stored 64 at a time
    int dseen = 0;             // jobs the recorder has published (last seen)
    MW_DECL(a_nr);
    MW_DECL(a_dw);
    MW_DECL(a_d0);  // waits of the round's first MW_R jobs (pipeline fill)
    MW_DECL(a_dc);
    MW_DECL(a_dd);
    MW_CLK(d0);
    for (; t < P.w; ++t) {
        MW_CLK(dw0);
        uint4 h0, h1, h2, i0, i1, i2;
        for (unsigned sp = 0;; ++sp) {  // speculative: header and items in one round trip
            mw_read_rec(&S->rec[t & (MW_R - 1)], i8, h0, h1, h2, i0, i1, i2);
#ifdef MW_DECIDER_BENCH
            if (true) break;  // diagnostic: records pre-filled, no helpers
#endif
            if ((uint32_t)rfl((int32_t)h0.x) == (uint32_t)t + 1u) break;
            if (sp > MW_SPIN_LIMIT || rfl((int32_t)lds_ld(&S->fail))) {  // uniform exit
                lds_st(&S->fail, 1u);
                stop = 3;
                break;
            }
            MW_ACC(a_nr, sp == 0);
            __builtin_amdgcn_s_sleep(0);
        }
        const MwHdr h{h0.x, (int32_t)h0.y, (int32_t)h0.z, (int32_t)h0.w, (int32_t)h1.x,
                      (int32_t)h1.y, (int32_t)h1.z, (int32_t)h1.w, h2.x, h2.y,
                      ((uint64_t)h2.w << 32) | h2.z};
        const MwItem it{((uint64_t)i0.y << 32) | i0.x, (int32_t)i0.z, (int32_t)i0.w,
                        (int32_t)i1.x, (int32_t)i1.y, (int32_t)i1.z, (int32_t)i1.w,
                        i2.x, i2.y, i2.z, i2.w};
        if (stop) break;
        MW_CLK(dw1);
        MW_ACC(a_dw, dw1 - dw0);
        MW_ACC(a_d0, t < MW_R ? dw1 - dw0 : 0);
        const int v = __builtin_amdgcn_readfirstlane(h.v);
        const int n = __builtin_amdgcn_readfirstlane(h.n);
        const bool live = wj >= v;
        // first record item whose node no live ring entry touches (items are sorted by key)
        const uint64_t tm = __ballot(live && (uint32_t)it.key == wp);
        const uint64_t valid = n >= 8 ? ~0ull : (1ull << (8 * n)) - 1ull;
        const uint64_t un = valid & 0x0101010101010101ull & ~any_in_byte(tm);
        const int il = un ? __builtin_ctzll(un) : 0;  // its lane (8 i*)
        uint64_t best = KEY_INF;
        if (un)
            best = ((uint64_t)__builtin_amdgcn_readlane((int)(it.key >> 32), il) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)it.key, il);
        // live ring rows at their current state: any better than that item?
        const uint64_t wk0 = mw_key(wc, wm, wg, wa, wk, wp, h.cpu, h.mem, h.gpu, h.wall, h.pbit);
        const uint64_t wkey = live ? wk0 : KEY_INF;
        const uint64_t bet = __ballot(wkey < best) & 0xffull;
        int rl = -1;  // winning ring lane, -1: the item
        if (bet) {
            if (__popcll(bet) == 1) {
                rl = __builtin_ctzll(bet);
            } else {
                const uint32_t mh = min8_u32((uint32_t)(wkey >> 32));
                const uint32_t ml = min8_u32((uint32_t)(wkey >> 32) == mh ? (uint32_t)wkey : ~0u);
                rl = __builtin_ctzll(__ballot((uint32_t)(wkey >> 32) == mh &&
                                              (uint32_t)wkey == ml) & 0xffull);
            }
            best = ((uint64_t)__builtin_amdgcn_readlane((int)(wkey >> 32), rl) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wkey, rl);
        }
        MW_CLK(dw2);
        MW_ACC(a_dc, dw2 - dw1);
        if (__ballot(h.B != KEY_INF && best > h.B)) {  // uniform
            stop = 1;  // candidate list exhausted: rescan next round
            break;
        }
        int32_t node = -1;
        int32_t dkind = -1, dslot = -1;  // winner for the recorder: item 0..7, 8 ring, -1 none
        if (best != KEY_INF) {
            int32_t sc, sm, sg, sa, slot;
            uint32_t sk;
            if (rl >= 0) {
                sc = __builtin_amdgcn_readlane(wc, rl);
                sm = __builtin_amdgcn_readlane(wm, rl);
                sg = __builtin_amdgcn_readlane(wg, rl);
                sa = __builtin_amdgcn_readlane(wa, rl);
                sk = __builtin_amdgcn_readlane(wk, rl);
                node = __builtin_amdgcn_readlane(wo, rl);
                slot = __builtin_amdgcn_readlane(ws, rl);
            } else {
                sc = __builtin_amdgcn_readlane(it.cpu, il);
                sm = __builtin_amdgcn_readlane(it.mem, il);
                sg = __builtin_amdgcn_readlane(it.gpu, il);
                sa = __builtin_amdgcn_readlane(it.avail, il);
                sk = __builtin_amdgcn_readlane(it.mask, il);
                node = __builtin_amdgcn_readlane(it.orig, il);
                slot = __builtin_amdgcn_readlane(it.tag, il);
            }
            const bool fresh = slot < 0;  // a clean node becomes dirty row nu
            if (fresh && nu == UCAP) {
                stop = 2;  // dirty set full
                break;
            }
            if (fresh) slot = nu++;
            const int32_t nc = sc - __builtin_amdgcn_readfirstlane(h.cpu);
            const int32_t nm = sm - __builtin_amdgcn_readfirstlane(h.mem);
            const int32_t ng = sg - __builtin_amdgcn_readfirstlane(h.gpu);
            const uint32_t pos = (uint32_t)best;
            dkind = rl >= 0 ? 8 : il >> 3;
            dslot = slot;
            if (!MW_RECORDER && lane == 0) {
                S->rows[slot] = MwRow{nc, nm, ng, sa, sk, pos, node, t};
                if (fresh) {
                    const uint32_t rel = pos - nb;
                    __hip_atomic_fetch_or(&S->bitmap[rel >> 5], 1u << (rel & 31),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            // ring entry t & 7 (job, slot, pos in every lane; the row in lane t & 7 only); an
            // older entry of the same slot dies
            const int e = t & 7;
            const bool me = r8 == e;
            wj = me ? t : (ws == slot ? -1 : wj);
            ws = me ? slot : ws;
            wp = me ? pos : wp;
            wc = writelane(nc, e, wc);
            wm = writelane(nm, e, wm);
            wg = writelane(ng, e, wg);
            wa = writelane(sa, e, wa);
            wk = writelane(sk, e, wk);
            wo = writelane(node, e, wo);
            ++placed;
        }
        if (MW_RECORDER) {
            // queue entry t % MW_DQ is free once the recorder has published job t - MW_DQ
            if (t >= dseen + MW_DQ && !mw_dq_space(S, t, dseen)) {
                stop = 3;
                break;
            }
            if (lane == 0)  // one 16-byte store: the recorder reads it with one load
                *reinterpret_cast<uint4*>(&S->dq[t & (MW_DQ - 1)]) =
                    make_uint4((uint32_t)t + 1u, (uint32_t)dkind, (uint32_t)dslot, 0u);
        } else {
            oq = writelane(__builtin_amdgcn_readfirstlane(h.q), t & 63, oq);
            ov = writelane(node, t & 63, ov);
            if ((t & 63) == 63) {  // uniform: flush 64 placements
                if (oq >= 0) ((GAS int32_t*)out)[(int64_t)oq * kmax] = ov;  // global: vmcnt only
                oq = -1;
            }
            cbar();
            if (lane == 0)  // {decided, nu} in one 8-byte LDS store
                __hip_atomic_store(reinterpret_cast<uint64_t*>(&S->decided),
                                   ((uint64_t)(uint32_t)nu << 32) | (uint32_t)(t + 1),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        MW_CLK(dw3);
        MW_ACC(a_dd, dw3 - dw2);
    }
    if (MW_RECORDER) {  // end marker: the recorder finishes job t - 1 and reports `stop`
        if (stop == 3 || t < dseen + MW_DQ || mw_dq_space(S, t, dseen)) {
            if (lane == 0)
                *reinterpret_cast<uint4*>(&S->dq[t & (MW_DQ - 1)]) =
                    make_uint4((uint32_t)t + 1u, (uint32_t)MW_DQ_END, (uint32_t)stop, 0u);
        }
    } else if (oq >= 0 && lane < (t & 63)) {
        ((GAS int32_t*)out)[(int64_t)oq * kmax] = ov;  // last group
    }
    if (stop) lds_st(&S->halt, 1u);
    MW_CLK(d1);
    MW_ADD(0, d1 - d0);
    MW_ADD(2, t);
    MW_ADD(1, a_dw);
    MW_ADD(9, a_d0);
    MW_ADD(7, a_dc);
    MW_ADD(8, a_dd);
    MW_ADD(16, a_nr);
    return CommitResult{t, stop, nu, placed};
}

// ------------------------------------------------------------------------------ recorder
// Takes the decisions in job order and does what the helpers and the output need: the dirty row
// (current state, version t), the dirty bitmap bit of a fresh node, the placement (parked in lane
// t & 63, stored 64 at a time), then {decided, nu} — the helpers' snapshot — in one 8-byte store
// after the rest (DS order).  The winner's previous state comes from the record the decider used
// (an item: its node did not change since the snapshot, or the decider would have dropped it) or
// from the dirty row of a ring winner (this wave wrote it).  Record slot t % MW_R is reused only
// for job t + MW_R, whose helper waits for decided >= t + 1: it is intact here.
__device__ __noinline__ CommitResult mw_recorder(const CompPlan& Pref, MwShared* Sin,
                                                 int32_t* __restrict__ out, int kmax) {
    const CompPlan P = plan_sgpr(Pref);
    MwShared* const S = lds_opaque(Sin);
    const int lane = threadIdx.x & 63;
    const uint32_t nb = (uint32_t)P.nb;
    int nu = 0, placed = 0, stop = 0, t = 0;
    int32_t oq = -1, ov = -1;
    MW_DECL(a_rw);
    MW_CLK(r0);
    for (;; ++t) {
        uint4 d;
        MW_CLK(rw0);
        for (unsigned sp = 0;; ++sp) {
            asm volatile("" ::: "memory");  // a fresh LDS read every spin
            d = *reinterpret_cast<const uint4*>(&S->dq[t & (MW_DQ - 1)]);
            if ((uint32_t)rfl((int32_t)d.x) == (uint32_t)t + 1u) break;
            if (sp > MW_SPIN_LIMIT || rfl((int32_t)lds_ld(&S->fail))) {
                lds_st(&S->fail, 1u);
                stop = 3;
                break;
            }
            __builtin_amdgcn_s_sleep(0);
        }
        if (stop) break;
        {
            MW_CLK(rw1);
            MW_ACC(a_rw, rw1 - rw0);
        }
        const uint32_t kind = (uint32_t)rfl((int32_t)d.y);
        if (kind == MW_DQ_END) {
            stop = rfl((int32_t)d.z);
            break;
        }
        asm volatile("" ::: "memory");  // record / row reads after the queue entry's read
        const MwRec* R = &S->rec[t & (MW_R - 1)];
        const uint4 hq = reinterpret_cast<const uint4*>(&R->h)[0];  // {ready, v, n, q}
        int32_t node = -1;
        if (kind != 0xffffffffu) {
            const uint4 hd = reinterpret_cast<const uint4*>(&R->h)[1];  // {cpu, mem, gpu, wall}
            const int slot = rfl((int32_t)d.z);
            uint4 a, b;
            bool fresh = false;
            if (kind < 8u) {  // record item: {key, tag, orig, cpu, mem, gpu, avail, mask, ...}
                const uint4* ip = reinterpret_cast<const uint4*>(&R->it[kind]);
                const uint4 i0 = ip[0], i1 = ip[1], i2 = ip[2];
                fresh = rfl((int32_t)i0.z) < 0;
                a = make_uint4(i1.x, i1.y, i1.z, i1.w);       // cpu, mem, gpu, avail
                b = make_uint4(i2.x, i0.x, i0.w, (uint32_t)t);  // mask, pos, orig, version
            } else {  // dirty row of a ring winner
                const uint4* rp = reinterpret_cast<const uint4*>(&S->rows[slot]);
                a = rp[0];
                const uint4 r1 = rp[1];
                b = make_uint4(r1.x, r1.y, r1.z, (uint32_t)t);
            }
            a.x = (uint32_t)((int32_t)a.x - (int32_t)hd.x);
            a.y = (uint32_t)((int32_t)a.y - (int32_t)hd.y);
            a.z = (uint32_t)((int32_t)a.z - (int32_t)hd.z);
            node = rfl((int32_t)b.z);
            if (lane == 0) {
                uint4* rp = reinterpret_cast<uint4*>(&S->rows[slot]);
                rp[0] = a;
                rp[1] = b;
                if (fresh) {
                    const uint32_t rel = (uint32_t)rfl((int32_t)b.y) - nb;
                    __hip_atomic_fetch_or(&S->bitmap[rel >> 5], 1u << (rel & 31),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            if (fresh) nu = slot + 1;
            ++placed;
        }
        oq = writelane(rfl((int32_t)hq.w), t & 63, oq);
        ov = writelane(node, t & 63, ov);
        if ((t & 63) == 63) {  // uniform: flush 64 placements
            if (oq >= 0) ((GAS int32_t*)out)[(int64_t)oq * kmax] = ov;
            oq = -1;
        }
        cbar();
        if (lane == 0)  // {decided, nu} in one 8-byte LDS store, after the row and bitmap
            __hip_atomic_store(reinterpret_cast<uint64_t*>(&S->decided),
                               ((uint64_t)(uint32_t)nu << 32) | (uint32_t)(t + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (oq >= 0 && lane < (t & 63)) ((GAS int32_t*)out)[(int64_t)oq * kmax] = ov;  // last group
    if (stop) lds_st(&S->halt, 1u);
    MW_CLK(r1);
    MW_ADD(17, r1 - r0);
    MW_ADD(18, a_rw);
    MW_ADD(19, t);
    return CommitResult{t, stop, nu, placed};
}

// All MW_WAVES waves of the block call this; returns the same result in every wave.
__device__ __forceinline__ CommitResult commit_window_mw(const CompPlan& P, MwShared* S,
                                                         NodeRec* __restrict__ rec,
                                                         const uint64_t* __restrict__ cand,
                                                         const uint64_t* __restrict__ bnd,
                                                         const JobRec* __restrict__ wjob,
                                                         int32_t* __restrict__ out, int kmax,
                                                         MwTiles T = MwTiles{nullptr, 0u}) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = threadIdx.x; i < nwords; i += MW_WAVES * 64) S->bitmap[i] = 0u;
    if (threadIdx.x < MW_R) S->rec[threadIdx.x].h.ready = 0u;
    if (threadIdx.x < MW_DQ) S->dq[threadIdx.x].x = 0u;
    if (threadIdx.x == 0) {
        S->decided = 0u;
        S->halt = 0u;
        S->nu = 0u;
        S->fail = 0u;
    }
    __syncthreads();
    if (wave == 0 || (MW_RECORDER && wave == 1)) {
        const CommitResult r = wave == 0 ? mw_decider(P, S, out, kmax)
                                         : mw_recorder(P, S, out, kmax);
        if (threadIdx.x == 64 * MW_RECORDER) {  // the recorder's result when it runs
            S->res[0] = r.done;
            S->res[1] = r.stop;
            S->res[2] = r.dirty;
            S->res[3] = r.placed;
        }
    } else if (MW_RECORDER) {
        mw_helper(P, S, rec, cand, bnd, wjob, wave - 1, T);  // waves 2.. : helpers 1..MW_H
    } else if (MW_H == MW_WAVES - 1) {
        mw_helper(P, S, rec, cand, bnd, wjob, wave, T);
    } else if (wave != 4) {
        mw_helper(P, S, rec, cand, bnd, wjob, wave < 4 ? wave : wave - 1, T);
    }
    __syncthreads();
    const CommitResult r{S->res[0], S->res[1], S->res[2], S->res[3]};
    // write the dirty rows back for the next round's scan
    for (int u = threadIdx.x; u < r.dirty; u += MW_WAVES * 64) {
        const MwRow w = S->rows[u];
        NodeRec* d = rec + w.pos;
        d->cpu = w.cpu;
        d->mem = w.mem;
        d->gpu = w.gpu;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
    __syncthreads();
    return r;
}

}  // namespace fitgpu
