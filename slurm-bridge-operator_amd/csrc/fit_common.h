// fit_common.h — device building blocks shared by the host-driven kernels (fit_kernels.hip)
// and the persistent work-queue engine (fit_persistent.hip).  DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fit_device.h"

namespace fitgpu {

__device__ __forceinline__ uint64_t fit_key(int32_t cf, int32_t mf, int32_t gf, int32_t av,
                                            uint32_t mask, uint32_t pos, const JobRec& J) {
    const int32_t dc = cf - J.cpu, dm = mf - J.mem, dg = gf - J.gpu, da = av - J.wall;
    const bool ok = (dc | dm | dg | da) >= 0 && (mask & J.pbit);
    const uint32_t sc = (min((uint32_t)dg, 255u) << 24) | (min((uint32_t)dc, 4095u) << 12) |
                        min((uint32_t)dm >> 10, 4095u);
    return ok ? (((uint64_t)sc << 32) | pos) : KEY_INF;
}

// ---- wave-wide reductions (DPP; call with a full EXEC mask) ---------------------------
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_min(uint32_t v) {
    return min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, CTRL, ROWMASK,
                                                        0xf, false));
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = dpp_min<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_min<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_min<0x124, 0xf>(v);  // row_ror:4
    v = dpp_min<0x128, 0xf>(v);  // row_ror:8
    v = dpp_min<0x142, 0xa>(v);  // row_bcast:15
    v = dpp_min<0x143, 0xc>(v);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// min over the wave of a packed (score << 32 | position) key: 32-bit min of the scores, then of
// the positions among the lanes holding that score (usually one lane: a readlane).
__device__ __forceinline__ uint64_t wave_min_key(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const uint32_t mh = wave_min_u32(hi);
    const uint64_t eq = __ballot(hi == mh);
    uint32_t ml;
    if (__popcll(eq) == 1)
        ml = (uint32_t)__builtin_amdgcn_readlane((int)lo, __builtin_ctzll(eq));
    else
        ml = wave_min_u32(hi == mh ? lo : 0xffffffffu);
    return ((uint64_t)mh << 32) | ml;
}

// wave_min_key plus the lane holding the minimum (the lowest such lane)
__device__ __forceinline__ uint64_t wave_min_key_lane(uint64_t v, int& lane) {
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const uint32_t mh = wave_min_u32(hi);
    const uint64_t eq = __ballot(hi == mh);
    uint32_t ml;
    if (__popcll(eq) == 1) {
        lane = __builtin_ctzll(eq);
        ml = (uint32_t)__builtin_amdgcn_readlane((int)lo, lane);
    } else {
        ml = wave_min_u32(hi == mh ? lo : 0xffffffffu);
        lane = __builtin_ctzll(__ballot(hi == mh && lo == ml));
    }
    return ((uint64_t)mh << 32) | ml;
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a < b ? b : a; }

// sorted ascending insert of x (< KEY_INF) into key[0..K) dropping the largest (static indices
// only).  Entry i becomes key[i-1] if x < key[i-1], x if key[i-1] <= x < key[i], else key[i]:
// with the K compares c[i] = x < key[i] issued first (independent, so no compare → select
// hazard stalls), the high word is the clamp max(hi[i-1], min(hi[i], x.hi)) — exact because the
// list is sorted; one v_med3_u32 — and only the low word needs the two selects: 4 VALU per entry
// instead of two 64-bit min/max (2 compares + 4 selects + 2 hazard nops through one SGPR pair).
template <int K>
__device__ __forceinline__ void topk_insert(uint64_t (&key)[K], uint64_t x) {
    const uint32_t xh = (uint32_t)(x >> 32), xl = (uint32_t)x;
    bool c[K];
#pragma unroll
    for (int i = 0; i < K; ++i) c[i] = x < key[i];
    uint64_t n[K];
    n[0] = c[0] ? x : key[0];
#pragma unroll
    for (int i = 1; i < K; ++i) {
        const uint32_t a = (uint32_t)(key[i - 1] >> 32), b = (uint32_t)(key[i] >> 32);
        const uint32_t h = max(min(a, b), min(max(a, b), xh));  // med3 (= the clamp: a <= b)
        const uint32_t l = c[i - 1] ? (uint32_t)key[i - 1] : (c[i] ? xl : (uint32_t)key[i]);
        n[i] = ((uint64_t)h << 32) | l;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) key[i] = n[i];
}

// (list, bound) pairs: every node of the covered range that is not in the sorted list has a
// key > bound, and every list entry is <= bound (bound = last entry, INF when not full).
// Merge two such pairs over disjoint ranges into the pair for the union (bitonic, registers).
template <int K>
__device__ __forceinline__ void merge_lists(uint64_t (&a)[K], const uint64_t (&b)[K]) {
    const uint64_t bb = umin64(a[K - 1], b[K - 1]);
    uint64_t c[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint64_t x = a[i] > bb ? KEY_INF : a[i];
        const uint64_t y = b[K - 1 - i] > bb ? KEY_INF : b[K - 1 - i];
        c[i] = umin64(x, y);  // bitonic sequence holding the K smallest of the union
    }
#pragma unroll
    for (int st = K / 2; st >= 1; st >>= 1)
#pragma unroll
        for (int i = 0; i < K; ++i)
            if ((i & st) == 0) {
                const uint64_t lo = umin64(c[i], c[i + st]), hi = umax64(c[i], c[i + st]);
                c[i] = lo;
                c[i + st] = hi;
            }
#pragma unroll
    for (int i = 0; i < K; ++i) a[i] = c[i];
    // The bound stays "last entry": if bb is finite, the list achieving it is full with all its
    // K entries <= bb, so the merged list is full and c[K-1] <= bb is the new bound.
}

__device__ __forceinline__ int find_comp(const CompPlan* __restrict__ plan, int ncomp, int b) {
    int c = 0;
    for (int i = 1; i < ncomp; ++i)
        if (plan[i].blk0 <= b) c = i;
    return c;
}

// One (job-lane, node-row) evaluation.  Node fields are clamped to >= -1 when the table is built
// (k_gather_nodes) and demands are >= 0, so every difference below is exact in int32; the pair
// is feasible iff no difference is negative and the partition bit is set.
template <int K>
__device__ __forceinline__ void scan_row(const NodeRec& r, int x, const JobRec& J,
                                         uint64_t (&key)[K], uint32_t& lim) {
    const int32_t dc = r.cpu - J.cpu, dm = r.mem - J.mem, dg = r.gpu - J.gpu;
    const int32_t da = r.avail - J.wall;
    const int32_t dp = (int32_t)((r.mask & J.pbit) - 1u);  // -1: not a member (or idle lane)
    const int32_t bad = dc | dm | dg | da | dp;
    const uint32_t sc = (min((uint32_t)dg, 255u) << 24) | (min((uint32_t)dc, 4095u) << 12) |
                        min((uint32_t)dm >> 10, 4095u);
    if (bad >= 0 && sc <= lim) {
        topk_insert(key, ((uint64_t)sc << 32) | (uint32_t)x);
        const uint64_t last = key[K - 1];
        lim = last == KEY_INF ? 0xffffffffu : (uint32_t)(last >> 32) - 1u;
    }
}

// A window job row for the commit: written through (four 8-B agent-scope stores, sc1) when the
// commit runs in the same launch (see scan_tile), a plain store otherwise.
template <bool THROUGH>
__device__ __forceinline__ void store_job(JobRec* dst, const JobRec& J) {
    if constexpr (THROUGH) {
        uint64_t* d = reinterpret_cast<uint64_t*>(dst);
        const uint64_t w0 = (uint64_t)(uint32_t)J.q | ((uint64_t)(uint32_t)J.cpu << 32);
        const uint64_t w1 = (uint64_t)(uint32_t)J.mem | ((uint64_t)(uint32_t)J.gpu << 32);
        const uint64_t w2 = (uint64_t)(uint32_t)J.wall | ((uint64_t)J.pbit << 32);
        const uint64_t w3 = (uint64_t)(uint32_t)J.k | ((uint64_t)(uint32_t)J.pad << 32);
        __hip_atomic_store(d + 0, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d + 1, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d + 2, w2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d + 3, w3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *dst = J;
    }
}

// The persistent engines' candidate lists, written through with the whole block: wave 0 (lane =
// job) puts its KW keys into LDS (`buf`, KW * 64 u64), then thread i stores 16 B of job i / (KW/2)
// with one sc1 dwordx4 store, so 8 (KW = 16) or 2 (KW = 4) consecutive lanes write a job's
// contiguous list — whole 64-B lines instead of KW separate 8-B partial writes per lane (the
// fabric counts each partial write: C3 wrote 3.7 GB per launch that way).  Every thread of the
// block calls it (one barrier inside); each storing wave drains its stores before the caller's
// tile count, as before.
#ifndef FIT_COALESCED_LISTS
#define FIT_COALESCED_LISTS 1
#endif
template <int KW>
__device__ __forceinline__ void store_lists_through(uint64_t* __restrict__ buf, bool wave0, int lane,
                                                    const uint64_t* key, int nkey, uint64_t* base,
                                                    int64_t job_stride, int nactive) {
    static_assert(KW % 2 == 0, "16-B chunks");
    if (wave0) {
#pragma unroll
        for (int i = 0; i < KW; ++i) buf[lane * KW + i] = i < nkey ? key[i] : KEY_INF;
    }
    __syncthreads();
    constexpr int CPJ = KW / 2;  // 16-B chunks per job
    for (int i = threadIdx.x; i < 64 * CPJ; i += SCAN_WAVES * 64) {
        const int j = i / CPJ, c = i - j * CPJ;
        if (j >= nactive) break;  // i only grows
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        const v4 v = *reinterpret_cast<const v4*>(buf + j * KW + 2 * c);
        uint64_t* dst = base + j * job_stride + 2 * c;
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
    }
}

// -------------------------------------------------------------------------------- k_scan
// Block = SCAN_JOBS jobs (lanes) × one block-slice of SCAN_WAVES sub-slices (one per wave).
// Each wave keeps the exact top-K of its sub-slice; the 8 lists are merged through LDS in a
// bitonic tree, giving the exact top-K (and bound) of the block-slice.  K = P.ks (KS, or fewer
// keys over more block-slices for a large component: the same candidates per job, but a round's
// first job tile — which the commit waits for — is spread over more blocks).
// KW > K (the persistent engine's first job tile of a round, FIT_K0): keep only the top-K per
// block-slice but write the plan's KW-entry layout, padded with KEY_INF — an exact (list, bound)
// pair of K entries, whose insertion network is KW / K times cheaper than the full list's: the
// tile the commit waits for at every round start arrives sooner.
//
// STAGE (the persistent engine's first job tile of a round, whose scan the commit waits for): the
// block first copies its block-slice's node rows into LDS (`stage`, SCAN_WAVES * P.sub rows) with
// vector loads from all 512 lanes — one memory round trip — and the waves then read the rows from
// LDS.  The plain path's scalar loads, four rows per wait, pay one round trip per four rows: after
// the acquire that opens every task the rows come from MALL / HBM, and a lone first tile (nothing
// else runs on its CU to hide the latency) spent most of its ~19 us waiting (C3).
#ifdef FIT_TILE0_STAMPS  // diagnostic build only: where a staged first tile's time goes
__device__ unsigned long long g_tile0[8];
#define T0_MARK(i)                                                                              \
    do {                                                                                        \
        if (STAGE) {                                                                            \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                         \
            const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();                   \
            if (threadIdx.x == 0 && (i) > 0) atomicAdd(&g_tile0[(i) - 1], now_ - t0m_);         \
            if ((i) == 0 && threadIdx.x == 0) atomicAdd(&g_tile0[7], 1ull);                     \
            t0m_ = now_;                                                                        \
        }                                                                                       \
    } while (0)
#else
#define T0_MARK(i)
#endif
// PAIR (k_engine's round-first tile, K_T0PAIR; P here has half-size sub-slices over twice the
// block-slices): as scan_tile_tl's (fit_timeline.hip) — half-slices 2p and 2p+1 each keep their
// top K, the second to finish merges the first's list (stored through, counted in pairs[p]) into
// slot p and sets the bound.  Returns whether the task completes its tile's block-slice (wave 0).
template <bool PERSISTENT, int K, int KW = K, bool STAGE = false, bool PAIR = false>
__device__ __forceinline__ bool scan_tile(
    const CompPlan& P, int tile, int s, const NodeRec* __restrict__ rec,
    const int32_t* __restrict__ jl, const int32_t* __restrict__ jcpu,
    const int32_t* __restrict__ jmem, const int32_t* __restrict__ jgpu,
    const int32_t* __restrict__ jwall, const uint16_t* __restrict__ jpart,
    const uint16_t* __restrict__ jk, uint64_t* __restrict__ cand, uint64_t* __restrict__ bnd,
    JobRec* __restrict__ wjob, uint64_t (*xk)[K][64],
    unsigned long long* __restrict__ feas = nullptr, NodeRec* __restrict__ stage = nullptr,
    unsigned* __restrict__ pairs = nullptr) {
    static_assert(!PAIR || (PERSISTENT && K <= 4), "pair scratch: 4 keys per (job, pair)");
    if (tile * SCAN_JOBS >= P.w) return true;  // block-uniform
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int t = tile * SCAN_JOBS + lane;
    const bool active = t < P.w;
#ifdef FIT_TILE0_STAMPS
    unsigned long long t0m_ = 0;
#endif
    T0_MARK(0);

    JobRec J;
    J.q = active ? jl[P.jbase + t] : 0;
    J.cpu = active ? jcpu[J.q] : 0;
    J.mem = active ? jmem[J.q] : 0;
    J.gpu = active ? jgpu[J.q] : 0;
    J.wall = active ? jwall[J.q] : 0;
    J.pbit = active ? (1u << jpart[J.q]) : 0u;  // 0 → nothing feasible
    J.k = active ? (jk ? max((int)jk[J.q], 1) : 1) : 1;
    J.pad = 0;

    uint64_t key[K];
#pragma unroll
    for (int i = 0; i < K; ++i) key[i] = KEY_INF;
    // candidate test: score <= lim, lim = (K-th score - 1) once the list is full.  An equal
    // score never beats the K-th entry (positions only grow); a spurious insert when the K-th
    // score is 0 is dropped by the 64-bit insertion network, so the list stays exact.
    uint32_t lim = 0xffffffffu;
    const int n0 = P.sb + (s * SCAN_WAVES + wave) * P.sub;
    const int n1 = min(P.se, n0 + P.sub);
    if constexpr (STAGE) {
        // the block-slice's rows [a, b) into LDS, 16 B per lane per load, all loads in flight
        const int a = P.sb + s * SCAN_WAVES * P.sub, b = min(P.se, a + SCAN_WAVES * P.sub);
        typedef int32_t v4 __attribute__((ext_vector_type(4)));
        const v4* src = reinterpret_cast<const v4*>(rec + a);
        v4* dst = reinterpret_cast<v4*>(stage);
        const int nv = 2 * max(b - a, 0);  // two 16-B halves per 32-B row
        T0_MARK(1);
        for (int i = threadIdx.x; i < nv; i += SCAN_WAVES * 64) dst[i] = src[i];
        __syncthreads();
        T0_MARK(2);
        int x = n0;
        for (; x + 4 <= n1; x += 4) {
            NodeRec r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = stage[x - a + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) scan_row(r[u], x + u, J, key, lim);
        }
        for (; x < n1; ++x) scan_row(stage[x - a], x, J, key, lim);
        T0_MARK(3);
    } else {
        int x = n0;
        for (; x + 4 <= n1; x += 4) {  // 4 rows per batch: four scalar row loads per wait
            NodeRec r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = rec[x + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) scan_row(r[u], x + u, J, key, lim);
        }
        for (; x < n1; ++x) scan_row(rec[x], x, J, key, lim);
    }

    // merge tree: waves [h, 2h) hand their lists to waves [0, h)
#pragma unroll
    for (int h = SCAN_WAVES / 2; h >= 1; h >>= 1) {
        if (wave >= h && wave < 2 * h) {
#pragma unroll
            for (int i = 0; i < K; ++i) xk[wave - h][i][lane] = key[i];
        }
        __syncthreads();
        if (wave < h) {
            uint64_t o[K];
#pragma unroll
            for (int i = 0; i < K; ++i) o[i] = xk[wave][i][lane];
            merge_lists(key, o);
        }
        __syncthreads();
    }
    T0_MARK(4);
    if (feas != nullptr && wave == 0) {  // the tile's jobs with a fitting node in this block-slice
        const uint64_t fm = __ballot(active && key[0] != KEY_INF);
        if (lane == 0 && fm != 0ull) atomicOr(feas, (unsigned long long)fm);
    }
    if constexpr (PERSISTENT && !PAIR && FIT_COALESCED_LISTS) {
        // every thread: the lists through LDS (the merge buffer, free again) and out coalesced
        const int na = max(0, min(SCAN_JOBS, P.w - tile * SCAN_JOBS));
        store_lists_through<KW>(reinterpret_cast<uint64_t*>(xk), wave == 0, lane, key, K,
                                cand + P.cand_off + ((int64_t)(tile * SCAN_JOBS) * P.nslice + s) * KW,
                                (int64_t)P.nslice * KW, na);
        if (wave != 0 || !active) return true;
        if (key[K - 1] != KEY_INF)
            atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                      (unsigned long long)key[K - 1]);
        if (s == 0) store_job<PERSISTENT>(wjob + P.slot0 + t, J);
        return true;
    }
    if (wave != 0) return true;  // (no barrier follows inside scan_tile)
    if constexpr (PAIR) {
        const int ns = P.nslice >> 1, pr = s >> 1;
        uint64_t* const fin = cand + P.cand_off + ((int64_t)t * ns + pr) * KW;
        uint64_t* const tmp = cand + P.pair_off + ((int64_t)lane * 32 + pr) * 4;  // tile 0: t = lane
        if (active) {
            if (s & 1) {
#pragma unroll
                for (int i = 0; i < K; ++i)
                    __hip_atomic_store(tmp + i, key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
#pragma unroll
                for (int i = 0; i < KW; ++i)
                    __hip_atomic_store(fin + i, i < K ? key[i] : KEY_INF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (s == 0) store_job<true>(wjob + P.slot0 + t, J);
        }
        // R1: the list (and the live-job bits above) stored and drained before the pair count
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned prev = 0u;
        if (lane == 0) prev = __hip_atomic_fetch_add(pairs + pr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_readfirstlane((int)prev) == 0) return false;  // the partner merges
        if (active) {
            const uint64_t* const other = (s & 1) ? fin : tmp;
            uint64_t o[K];
#pragma unroll
            for (int i = 0; i < K; ++i)
                o[i] = __hip_atomic_load(const_cast<uint64_t*>(other + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            merge_lists(key, o);
#pragma unroll
            for (int i = 0; i < K; ++i)
                __hip_atomic_store(fin + i, key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (key[K - 1] != KEY_INF)
                atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                          (unsigned long long)key[K - 1]);
        }
        return true;
    }
    if (!active) return true;
    uint64_t* dst = cand + P.cand_off + ((int64_t)t * P.nslice + s) * KW;
    if constexpr (PERSISTENT) {
        // the commit of the same launch reads these: written through (sc1 stores, agent-scope
        // atomics) so the worker needs no release fence before it counts the tile done — the
        // fence's write-back of the XCD's L2 cost every task a few us (MI355X_MICROARCH.md,
        // fence table; cdna_hip_programming.md §6 Guideline 16 R1)
#pragma unroll
        for (int i = 0; i < KW; ++i)
            __hip_atomic_store(dst + i, i < K ? key[i] : KEY_INF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
#pragma unroll
        for (int i = 0; i < KW; i += 2) {
            ulonglong2 v;
            v.x = i < K ? key[i] : KEY_INF;
            v.y = i + 1 < K ? key[i + 1] : KEY_INF;
            *reinterpret_cast<ulonglong2*>(dst + i) = v;
        }
    }
    if (key[K - 1] != KEY_INF)
        atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                  (unsigned long long)key[K - 1]);
    if (s == 0) store_job<PERSISTENT>(wjob + P.slot0 + t, J);
    return true;
}

// ------------------------------------------------------------------------------ k_commit
// One wave per component walks the window in priority order.  For job t it needs
//   clean best  = min over its candidate entries <= B whose node is not dirty (LDS bitmap),
//   dirty best  = min over the dirty rows (held in VGPRs, UPL per lane) at their current state,
// then commits min(clean, dirty) or stops the round.  The candidate keys, job
// row and bound are loaded two jobs ahead and the candidates' node rows one job ahead, so the
// serial chain per job is LDS + VALU + one wave reduction.
constexpr int UPL = UCAP / 64;  // dirty slots per lane

// ---- diagnostic in-kernel stamps (only in the FIT_STAMPS build; never in the shipped kernel)
#ifdef FIT_STAMPS
__device__ unsigned long long g_stamps[64][10];  // [8], [9]: STAMP_CNT2 counters
#define STAMP_DECL unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long st_prev = 0; \
    const unsigned long long st_t0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
#define STAMP(i)                                                                          \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        unsigned long long now_;                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now_)::"memory");      \
        __builtin_amdgcn_sched_barrier(0);                                                \
        if (i > 0) st_acc[(i) > 0 ? (i) - 1 : 0] += now_ - st_prev;                                     \
        st_prev = now_;                                                                   \
    } while (0)
#define STAMP_CNT(x) (st_acc[5] += (x))  // multi-node jobs: dirty-row picks
#define STAMP_CNT2(a, b) (st_acc[6] += (a), st_acc[7] += (b))
#define STAMP_FLUSH(c, n)                                                                 \
    {                                                                                     \
        const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                      \
        const unsigned long long r1_ = __builtin_amdgcn_s_memrealtime();                  \
        if (threadIdx.x == 0) {                                                           \
            for (int i_ = 0; i_ < 6; ++i_) g_stamps[c][i_] += st_acc[i_]; /* whole run */ \
            g_stamps[c][6] += n;                                                          \
            g_stamps[c][8] += st_acc[6];                                                  \
            g_stamps[c][9] += st_acc[7];                                                  \
            g_stamps[c][7] = ((t1_ - st_t0) << 24) / max(r1_ - st_r0, 1ull); /* cyc/10ns << 24 */ \
        }                                                                                 \
    }
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_CNT(x)
#define STAMP_CNT2(a, b)
#define STAMP_FLUSH(c, n)
#endif

// Multi-node jobs (SPEC k > 1): the K smallest keys among the lane's clean candidate entries and
// dirty-row keys, ascending.  seld[i]: sel[i] is a dirty row; drank[i]: the pick index of this
// lane's dirty entry i (-1: not picked).  kth = the K-th key (INF when fewer
// than K exist).  Returns how many were found.  Each lane sorts its entries once; then every
// extraction is a wave minimum of the lane heads — the 32-bit minimum of the scores, then of the
// positions among the lanes holding it, each as four fused DPP minima and the permlane16 / 32 swaps
// of gfx950 (in every lane, no readlane, no branch) — and the lane that held it pops its head.
// Round 5: the previous form (a 64-bit wave minimum over every entry, with a readlane and a tie
// branch, and a pass clearing the taken key) cost ≈ 500 cycles per extraction at C4
// (profiles/r05q_c4_stamps.txt).
#define SK_DPP_MIN(v, CTL) asm volatile("s_nop 1\n\tv_min_u32_dpp %0, %0, %0 " CTL : "+v"(v))
__device__ __forceinline__ uint32_t sk_wave_min32_all(uint32_t v) {
    SK_DPP_MIN(v, "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf");
    SK_DPP_MIN(v, "quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf");
    SK_DPP_MIN(v, "row_half_mirror row_mask:0xf bank_mask:0xf");
    SK_DPP_MIN(v, "row_mirror row_mask:0xf bank_mask:0xf");  // every lane: its row's minimum
    {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = min((uint32_t)p[0], (uint32_t)p[1]);
    }
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return min((uint32_t)p[0], (uint32_t)p[1]);
}
#undef SK_DPP_MIN
template <int EPL>
__device__ __forceinline__ int select_k(int K, const uint64_t (&kr)[EPL], const bool (&cl)[EPL],
                                        const uint64_t (&dk)[UPL], uint64_t (&sel)[FIT_KMAX],
                                        bool (&seld)[FIT_KMAX], uint64_t& kth,
                                        int32_t (&drank)[UPL]) {
    constexpr int NE = EPL + UPL;
    uint64_t q[NE];
#pragma unroll
    for (int k = 0; k < EPL; ++k) q[k] = cl[k] ? kr[k] : KEY_INF;
#pragma unroll
    for (int i = 0; i < UPL; ++i) q[EPL + i] = dk[i];
#pragma unroll
    for (int r = 0; r < NE; ++r)  // odd-even transposition sort, ascending (NE <= 6)
#pragma unroll
        for (int i = r & 1; i + 1 < NE; i += 2) {
            const uint64_t lo = umin64(q[i], q[i + 1]), hi = umax64(q[i], q[i + 1]);
            q[i] = lo;
            q[i + 1] = hi;
        }
    int got = 0;
    kth = KEY_INF;
#pragma unroll
    for (int s = 0; s < FIT_KMAX; ++s) {
        sel[s] = KEY_INF;
        seld[s] = false;
    }
#pragma unroll
    for (int i = 0; i < UPL; ++i) drank[i] = -1;
#pragma unroll
    for (int s = 0; s < FIT_KMAX; ++s) {
        if (s >= K) break;  // uniform
        const uint32_t hh = (uint32_t)(q[0] >> 32), ll = (uint32_t)q[0];
        const uint32_t mh = sk_wave_min32_all(hh);
        const uint32_t ml = sk_wave_min32_all(hh == mh ? ll : 0xffffffffu);
        const uint64_t b = ((uint64_t)mh << 32) | ml;
        if (b == KEY_INF) break;  // uniform: fewer than K keys
        bool d = false;
#pragma unroll
        for (int i = 0; i < UPL; ++i) {
            const bool h = dk[i] == b;
            d = d || h;
            drank[i] = h ? s : drank[i];
        }
        sel[s] = b;
        seld[s] = __ballot(d) != 0ull;
        kth = b;
        ++got;
        const bool me = q[0] == b;  // keys are unique: one lane pops its head
#pragma unroll
        for (int e = 0; e + 1 < NE; ++e) q[e] = me ? q[e + 1] : q[e];
        q[NE - 1] = me ? KEY_INF : q[NE - 1];
    }
    if (got < K) kth = KEY_INF;
    return got;
}

struct CRow {  // node row of a candidate (prefetched)
    int32_t cpu, mem, gpu, avail;
    uint32_t mask;
    int32_t orig;
};

#ifdef FIT_STAMPS
// diagnostic: [8] jobs whose fitting dirty rows number <= 16 (and >= K), [9] those among them
// whose K smallest keys are all dirty rows (no clean key below the K-th dirty key)
#define STAMP_DIRTY_BELOW(A)                                                                    \
    {                                                                                           \
        int nd_ = 0;                                                                            \
        _Pragma("unroll") for (int i = 0; i < UPL; ++i) nd_ += __builtin_popcountll(__ballot(dk[i] != KEY_INF)); \
        unsigned long long a_ = 0, b_ = 0;                                                      \
        if (nd_ <= 16 && nd_ >= K_) {                                                           \
            a_ = 1;                                                                             \
            uint64_t q2_[UPL];                                                                  \
            _Pragma("unroll") for (int i = 0; i < UPL; ++i) q2_[i] = dk[i];                     \
            uint64_t td_ = KEY_INF;                                                             \
            for (int s2_ = 0; s2_ < K_; ++s2_) {                                                \
                uint64_t m_ = KEY_INF;                                                          \
                _Pragma("unroll") for (int i = 0; i < UPL; ++i) m_ = umin64(m_, q2_[i]);        \
                m_ = wave_min_key(m_);                                                          \
                _Pragma("unroll") for (int i = 0; i < UPL; ++i) q2_[i] = q2_[i] == m_ ? KEY_INF : q2_[i]; \
                td_ = m_;                                                                       \
            }                                                                                   \
            int cb_ = 0;                                                                        \
            _Pragma("unroll") for (int k = 0; k < EPL; ++k) cb_ += __builtin_popcountll(__ballot(cl[A][k] && kr[A][k] < td_)); \
            b_ = cb_ == 0 ? 1 : 0;                                                              \
        }                                                                                       \
        STAMP_CNT2(a_, b_);                                                                     \
    }
#else
#define STAMP_DIRTY_BELOW(A)
#endif

// Multi-node jobs whose fitting dirty rows number k..16 (46 % of C4's placed multi-node jobs): the
// k smallest dirty keys by compaction into lanes 0..15 (LDS scratch `scr`, 896 B) and rank by
// count (each of the ≤ 16 keys broadcast, every lane counts the smaller ones) — no sequential wave
// minima.  Exact when no clean candidate key is below the k-th dirty key (then the k smallest of
// all are these; 95 % of the cases): returns true and fills drank / kth, else false (the caller
// runs select_k).  nd = the number of fitting dirty rows, m0 / m1 their ballots.
__device__ __forceinline__ bool dirty_topk(int K, int nd, uint64_t m0, uint64_t m1, const uint64_t (&dk)[UPL],
                                           const uint64_t* kc, const bool* cc, int epl, uint32_t scr,
                                           int32_t (&drank)[UPL], uint64_t& kth) {
    static_assert(UPL == 2, "two dirty entries per lane");
    typedef __attribute__((address_space(3))) uint64_t* L64;
    typedef __attribute__((address_space(3))) int32_t* L32;
    const int lane = threadIdx.x & 63;
    const uint32_t lo0 = (uint32_t)m0, hi0 = (uint32_t)(m0 >> 32), lo1 = (uint32_t)m1, hi1 = (uint32_t)(m1 >> 32);
    const int p0 = (int)__builtin_amdgcn_mbcnt_hi(hi0, __builtin_amdgcn_mbcnt_lo(lo0, 0u));
    const int p1 = __builtin_popcountll(m0) + (int)__builtin_amdgcn_mbcnt_hi(hi1, __builtin_amdgcn_mbcnt_lo(lo1, 0u));
    const bool v0 = dk[0] != KEY_INF, v1 = dk[1] != KEY_INF;
    // branch-free: a lane without a fitting entry writes to its own trash slot (16 + lane)
    L64 keys = (L64)(uintptr_t)scr;
    L32 ranks = (L32)(uintptr_t)(scr + 8u * 80u);
    keys[v0 ? p0 : 16 + lane] = dk[0];
    keys[v1 ? p1 : 16 + lane] = dk[1];
    const uint64_t x = lane < nd ? keys[lane & 15] : KEY_INF;  // (one wave: LDS in order)
    int r = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {  // fully unrolled: faster than a loop over nd, or 32 keys
        const uint64_t y = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), j) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, j);
        r += y < x ? 1 : 0;
    }
    const uint64_t kb = __ballot(lane < nd && r == K - 1);
    const int kl = __builtin_ctzll(kb);
    const uint64_t t = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), kl) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, kl);
    bool below = false;
    for (int k = 0; k < epl; ++k) below = below || (cc[k] && kc[k] < t);
    if (__ballot(below) != 0ull) return false;  // a clean key among the k smallest
    ranks[lane] = r;  // (lanes 16..63: unused slots)
    const int32_t q0 = ranks[v0 ? p0 : 16 + lane], q1 = ranks[v1 ? p1 : 16 + lane];
    const int32_t r0 = v0 ? q0 : 64, r1 = v1 ? q1 : 64;
    drank[0] = r0 < K ? r0 : -1;
    drank[1] = r1 < K ? r1 : -1;
    kth = t;
    return true;
}

// Pipeline.  Iteration t: vector-load the keys of job t+2; derive the clean
// flags of job t+1 (bound + dirty bitmap, before job t's commit); resolve job t; clear the flag
// of any job-(t+1) candidate equal to the node job t dirtied; scalar-load job t+3's row and
// bound.  Every wait is then on data requested at least one iteration earlier.  The 4-slot
// job ring is indexed by literal constants only (4-way unrolled loop) so it stays in registers.
#define FIT_COMMIT_STEP(A, N1, N2, N3)                                                            \
    {                                                                                           \
        if (t >= P.w) goto done;                                                                \
        STAMP(0);                                                                               \
        {                                                                                       \
            const int tc_ = min(t + 2, wlast);                                                  \
            _Pragma("unroll") for (int k = 0; k < EPL; ++k) kr[N2][k] =                         \
                cand[off[k] + (int64_t)tc_ * per_rank];                                         \
        }                                                                                       \
        _Pragma("unroll") for (int k = 0; k < EPL; ++k) {                                       \
            const uint64_t kk_ = kr[N1][k];                                                     \
            const bool v_ = has[k] && kk_ <= jb[N1] && kk_ != KEY_INF;                          \
            const uint32_t rel_ = v_ ? (uint32_t)kk_ - nb : 0u;                                 \
            cl[N1][k] = v_ && !((bitmap[rel_ >> 5] >> (rel_ & 31)) & 1u);                       \
        }                                                                                       \
        STAMP(1);                                                                               \
        const int32_t jc = jcr[A], jm = jmr[A], jg = jgr[A], jw = jwr[A];                       \
        const uint32_t jp = jpr[A];                                                             \
        const uint64_t B = jb[A];                                                               \
        uint64_t cm = KEY_INF;                                                                  \
        _Pragma("unroll") for (int k = 0; k < EPL; ++k) cm =                                    \
            umin64(cm, cl[A][k] ? kr[A][k] : KEY_INF);                                          \
        STAMP(2);                                                                               \
        uint64_t dk[UPL];                                                                       \
        uint64_t dm = KEY_INF;                                                                  \
        _Pragma("unroll") for (int i = 0; i < UPL; ++i) {                                       \
            dk[i] = KEY_INF;                                                                    \
            if (i * 64 < nu) {                                                                  \
                const int32_t dc = ucpu[i] - jc, dmm = umem[i] - jm;                            \
                const int32_t dg = ugpu[i] - jg, da = uav[i] - jw;                              \
                const bool ok = (dc | dmm | dg | da) >= 0 && (umask[i] & jp) &&                 \
                                i * 64 + lane < nu;                                             \
                const uint32_t sc = (min((uint32_t)dg, 255u) << 24) |                           \
                                    (min((uint32_t)dc, 4095u) << 12) |                          \
                                    min((uint32_t)dmm >> 10, 4095u);                            \
                dk[i] = ok ? (((uint64_t)sc << 32) | upos[i]) : KEY_INF;                        \
                dm = umin64(dm, dk[i]);                                                         \
            }                                                                                   \
        }                                                                                       \
        STAMP(3);                                                                               \
        int32_t node = -1;                                                                      \
        uint32_t newpos = 0xffffffffu;                                                          \
        if (jkr[A] > 1) { /* multi-node job (uniform): the k smallest, all or nothing */        \
            const int K_ = jkr[A];                                                              \
            uint64_t sel_[FIT_KMAX];                                                            \
            bool seld_[FIT_KMAX];                                                               \
            uint64_t kth_ = KEY_INF;                                                            \
            int32_t drank_[UPL];                                                                \
            int got_;                                                                           \
            bool fast_ = false;                                                                 \
            if constexpr (FASTD) {                                                              \
                const uint64_t fm0_ = __ballot(dk[0] != KEY_INF), fm1_ = __ballot(dk[1] != KEY_INF); \
                const int fnd_ = __builtin_popcountll(fm0_) + __builtin_popcountll(fm1_);       \
                if (fnd_ >= K_ && fnd_ <= 16)                                                   \
                    fast_ = dirty_topk(K_, fnd_, fm0_, fm1_, dk, kr[A], cl[A], EPL, scr, drank_, kth_); \
            }                                                                                   \
            if (fast_) {                                                                        \
                got_ = K_;                                                                      \
                _Pragma("unroll") for (int s_ = 0; s_ < FIT_KMAX; ++s_) {                       \
                    sel_[s_] = KEY_INF;                                                         \
                    seld_[s_] = true;                                                           \
                }                                                                               \
            } else {                                                                            \
                got_ = select_k<EPL>(K_, kr[A], cl[A], dk, sel_, seld_, kth_, drank_);          \
            }                                                                                   \
            /* the picks' node rows, lane s holding pick s's: one memory round trip per job */  \
            uint32_t cpm_ = 0u; /* the clean picks (the only rows read from memory) */          \
            _Pragma("unroll") for (int s_ = 0; s_ < FIT_KMAX; ++s_) cpm_ |=                     \
                (s_ < got_ && !seld_[s_]) ? 1u << s_ : 0u;                                      \
            NodeRec mr_ = {0, 0, 0, 0, 0u, 0, 0, 0};                                            \
            if (cpm_ != 0u) { /* uniform: most jobs pick dirty rows only */                      \
                uint32_t myp_ = 0u;                                                             \
                _Pragma("unroll") for (int s_ = 0; s_ < FIT_KMAX; ++s_) myp_ =                  \
                    lane == s_ ? (uint32_t)sel_[s_] : myp_;                                     \
                if ((cpm_ >> lane) & 1u) mr_ = rec[myp_];                                       \
            }                                                                                   \
            STAMP(4);                                                                           \
            int nn_ = 0;                                                                        \
            _Pragma("unroll") for (int i = 0; i < FIT_KMAX; ++i) nn_ += i < K_ && !seld_[i];    \
            /* one uniform branch on the common path: a stop (a node outside the lists could  \
               win; the dirty set is full) or fewer than k nodes (unplaced) are the rare cases */ \
            const bool st1_ = B != KEY_INF && kth_ > B;                                         \
            const bool st2_ = got_ == K_ && nu + nn_ > UCAP;                                    \
            if (st1_ | st2_ | (got_ != K_)) {                                                   \
                if (st1_ | st2_) {                                                              \
                    stop = st1_ ? 1 : 2;                                                        \
                    goto done;                                                                  \
                }                                                                               \
            } else {                                                                            \
                int32_t pnd_ = -1;                                                              \
                STAMP_CNT((unsigned long long)(K_ - nn_));                                      \
                STAMP_DIRTY_BELOW(A);                                                           \
                /* the dirty-row picks (89 % at C4) all at once, branch-free: each lane updates \
                   its picked entries (an entry past nu is never picked: its key is INF) and    \
                   stores their node ids at their pick index; the other lanes store to the       \
                   job's pick-0 slot, which the parked placement overwrites later (in order) */  \
                {                                                                               \
                    int32_t o0_ = -1;                                                           \
                    bool h0_ = false;                                                           \
                    const int64_t ob_ = (int64_t)jqr[A] * kmax;                                 \
                    _Pragma("unroll") for (int i = 0; i < UPL; ++i) {                           \
                        const int32_t r_ = drank_[i];                                           \
                        const bool hit_ = r_ >= 0;                                              \
                        ucpu[i] -= hit_ ? jc : 0;                                               \
                        umem[i] -= hit_ ? jm : 0;                                               \
                        ugpu[i] -= hit_ ? jg : 0;                                               \
                        out[ob_ + (r_ > 0 ? r_ : 0)] = uorig[i];                                \
                        o0_ = r_ == 0 ? uorig[i] : o0_;                                         \
                        h0_ |= r_ == 0;                                                         \
                    }                                                                           \
                    const int32_t n0_ = __builtin_amdgcn_readlane(o0_, __builtin_ctzll(__ballot(h0_) | (1ull << 63))); \
                    node = seld_[0] ? n0_ : node;                                               \
                }                                                                               \
                if (nn_ > 0) { /* uniform: clean picks (none for most jobs) */                    \
                _Pragma("unroll") for (int s_ = 0; s_ < FIT_KMAX; ++s_) if (s_ < K_ && !seld_[s_]) { \
                    const uint64_t b_ = sel_[s_];                                               \
                    int32_t nd_;                                                                \
                    {                                                                           \
                        const uint32_t np_ = (uint32_t)b_;                                      \
                        NodeRec r;                                                              \
                        r.cpu = __builtin_amdgcn_readlane(mr_.cpu, s_);                         \
                        r.mem = __builtin_amdgcn_readlane(mr_.mem, s_);                         \
                        r.gpu = __builtin_amdgcn_readlane(mr_.gpu, s_);                         \
                        r.avail = __builtin_amdgcn_readlane(mr_.avail, s_);                     \
                        r.mask = (uint32_t)__builtin_amdgcn_readlane((int)mr_.mask, s_);        \
                        r.orig = __builtin_amdgcn_readlane(mr_.orig, s_);                       \
                        nd_ = r.orig;                                                           \
                        if (lane == (nu & 63)) {                                                \
                            _Pragma("unroll") for (int i = 0; i < UPL; ++i) if (i == (nu >> 6)) { \
                                ucpu[i] = r.cpu - jc;                                           \
                                umem[i] = r.mem - jm;                                           \
                                ugpu[i] = r.gpu - jg;                                           \
                                uav[i] = r.avail;                                               \
                                umask[i] = r.mask;                                              \
                                upos[i] = np_;                                                  \
                                uorig[i] = nd_;                                                 \
                            }                                                                   \
                            const uint32_t rel = np_ - nb;                                      \
                            bitmap[rel >> 5] |= 1u << (rel & 31);                               \
                        }                                                                       \
                        ++nu;                                                                   \
                        _Pragma("unroll") for (int k = 0; k < EPL; ++k) cl[N1][k] =             \
                            cl[N1][k] && (uint32_t)kr[N1][k] != np_;                            \
                    }                                                                           \
                    if (s_ == 0) node = nd_;                                                    \
                    else pnd_ = lane == s_ ? nd_ : pnd_;                                        \
                }                                                                               \
                /* picks 1..k-1 in one store after the loop: a store counts in vmcnt, so one    \
                   per pick would make the next pick's row wait for its acknowledgement */      \
                if (lane > 0 && lane < K_ && pnd_ >= 0) out[(int64_t)jqr[A] * kmax + lane] = pnd_; \
                }                                                                               \
                ++placed;                                                                       \
            }                                                                                   \
        } else {                                                                                \
        const uint64_t best = wave_min_key(umin64(cm, dm));                                     \
        STAMP(4);                                                                               \
        if (B != KEY_INF && best > B && __ballot(cm != KEY_INF) == 0ull) {                      \
            stop = 1; /* candidate list exhausted: rescan next round */                         \
            goto done;                                                                          \
        }                                                                                       \
        if (best != KEY_INF) {                                                                  \
            const uint64_t dmask = __ballot(dm == best);                                        \
            if (dmask) { /* a dirty row wins: update it in place */                             \
                int32_t o = 0;                                                                  \
                _Pragma("unroll") for (int i = 0; i < UPL; ++i) if (i * 64 < nu) {              \
                    const bool hit_ = dk[i] == best;                                            \
                    ucpu[i] -= hit_ ? jc : 0;                                                   \
                    umem[i] -= hit_ ? jm : 0;                                                   \
                    ugpu[i] -= hit_ ? jg : 0;                                                   \
                    o = hit_ ? uorig[i] : o;                                                    \
                }                                                                               \
                node = __builtin_amdgcn_readlane(o, __builtin_ctzll(dmask));                    \
            } else { /* a clean candidate wins: its row becomes dirty row nu */                 \
                if (nu == UCAP) {                                                               \
                    stop = 2;                                                                   \
                    goto done;                                                                  \
                }                                                                               \
                newpos = (uint32_t)best;                                                        \
                const NodeRec r = rec[newpos];                                                  \
                node = r.orig;                                                                  \
                if (lane == (nu & 63)) {                                                        \
                    _Pragma("unroll") for (int i = 0; i < UPL; ++i) if (i == (nu >> 6)) {       \
                        ucpu[i] = r.cpu - jc;                                                   \
                        umem[i] = r.mem - jm;                                                   \
                        ugpu[i] = r.gpu - jg;                                                   \
                        uav[i] = r.avail;                                                       \
                        umask[i] = r.mask;                                                      \
                        upos[i] = newpos;                                                       \
                        uorig[i] = node;                                                        \
                    }                                                                           \
                    const uint32_t rel = newpos - nb;                                           \
                    bitmap[rel >> 5] |= 1u << (rel & 31);                                       \
                }                                                                               \
                ++nu;                                                                           \
            }                                                                                   \
            ++placed;                                                                           \
        }                                                                                       \
        } /* k == 1 */                                                                          \
        STAMP(5);                                                                               \
        oq = lane == (t & 63) ? jqr[A] : oq; /* (selects: no exec branch) */                    \
        ov = lane == (t & 63) ? node : ov;                                                      \
        if ((t & 63) == 63) { /* uniform: flush 64 placements */                                \
            if (oq >= 0) out[(int64_t)oq * kmax] = ov;                                          \
            oq = -1;                                                                            \
        }                                                                                       \
        _Pragma("unroll") for (int k = 0; k < EPL; ++k) cl[N1][k] =                             \
            cl[N1][k] && (uint32_t)kr[N1][k] != newpos;                                         \
        {                                                                                       \
            const int tc_ = min(t + 3, wlast); /* slot N3 (job t-1's) receives job t+3 */       \
            const JobRec J_ = wjob[P.slot0 + tc_];                                              \
            jqr[N3] = J_.q;                                                                     \
            jcr[N3] = J_.cpu;                                                                   \
            jmr[N3] = J_.mem;                                                                   \
            jgr[N3] = J_.gpu;                                                                   \
            jwr[N3] = J_.wall;                                                                  \
            jpr[N3] = J_.pbit;                                                                  \
            jkr[N3] = J_.k;                                                                     \
            jb[N3] = bnd[P.slot0 + tc_];                                                        \
        }                                                                                       \
        ++t;                                                                                    \
    }

// BM: the bitmap's pointer type — an LDS (address space 3) pointer when the caller is a device
// function: through a generic pointer to dynamic LDS, a non-kernel function looks the LDS base up
// in a table per access (a scalar load and a full lgkmcnt wait, which also drains the job-row
// prefetch).
// The array pointers' types likewise: a device-function caller passes global (address space 1)
// pointers, since through generic ones every access is a flat one, which also counts in lgkmcnt —
// each LDS wait of a step would then wait for the key and job prefetches too.
template <int EPL, bool FASTD = false, typename BM, typename RecP, typename CandP, typename JobP,
          typename OutP>
__device__ __forceinline__ CommitResult commit_window(
    int c, const CompPlan& P, RecP __restrict__ rec, CandP __restrict__ cand,
    int64_t rank_stride, int nranks, CandP __restrict__ bnd,
    JobP __restrict__ wjob, OutP __restrict__ out, int kmax, BM bitmap, uint32_t scr = 0u) {
    const int lane = threadIdx.x & 63;
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = lane; i < nwords; i += 64) bitmap[i] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (single wave: LDS in order)

    const int per_rank = P.nslice * P.ks;
    const int E = nranks * per_rank;
    int64_t off[EPL];
    bool has[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + 64 * k;
        const int g = e / per_rank;
        has[k] = e < E;
        off[k] = has[k] ? g * rank_stride + P.cand_off + (e - g * per_rank) : P.cand_off;
    }
    const int wlast = P.w - 1;
    const uint32_t nb = (uint32_t)P.nb;

    int32_t ucpu[UPL], umem[UPL], ugpu[UPL], uav[UPL], uorig[UPL];
    uint32_t umask[UPL], upos[UPL];
#pragma unroll
    for (int i = 0; i < UPL; ++i) {
        ucpu[i] = umem[i] = ugpu[i] = uav[i] = uorig[i] = 0;
        umask[i] = upos[i] = 0u;
    }
    int nu = 0, placed = 0, stop = 0, t = 0;
    int32_t oq = -1, ov = -1;  // placement of job t parked in lane t & 63, stored 64 at a time

    uint64_t kr[4][EPL];
    bool cl[4][EPL];
    int32_t jqr[4], jcr[4], jmr[4], jgr[4], jwr[4], jkr[4];
    uint32_t jpr[4];
    uint64_t jb[4];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int tc = min(s, wlast);
        if (s < 2) {
#pragma unroll
            for (int k = 0; k < EPL; ++k) kr[s][k] = cand[off[k] + (int64_t)tc * per_rank];
        }
        const JobRec J = wjob[P.slot0 + tc];
        jqr[s] = J.q;
        jcr[s] = J.cpu;
        jmr[s] = J.mem;
        jgr[s] = J.gpu;
        jwr[s] = J.wall;
        jpr[s] = J.pbit;
        jkr[s] = J.k;
        jb[s] = bnd[P.slot0 + tc];
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const bool v = has[k] && kr[0][k] <= jb[0] && kr[0][k] != KEY_INF;
        const uint32_t rel = v ? (uint32_t)kr[0][k] - nb : 0u;
        cl[0][k] = v && !((bitmap[rel >> 5] >> (rel & 31)) & 1u);
    }
    STAMP_DECL
    for (;;) {
        FIT_COMMIT_STEP(0, 1, 2, 3)
        FIT_COMMIT_STEP(1, 2, 3, 0)
        FIT_COMMIT_STEP(2, 3, 0, 1)
        FIT_COMMIT_STEP(3, 0, 1, 2)
    }
done:
    STAMP_FLUSH(c, t)
    if (oq >= 0 && (lane < (t & 63))) out[(int64_t)oq * kmax] = ov;  // last partial group
    // write the dirty rows back for the next round's scan
#pragma unroll
    for (int i = 0; i < UPL; ++i)
        if (i * 64 + lane < nu) {
            const auto r = rec + upos[i];
            r->cpu = ucpu[i];
            r->mem = umem[i];
            r->gpu = ugpu[i];
        }
    return CommitResult{t, stop, nu, placed};
}
#undef FIT_COMMIT_STEP


}  // namespace fitgpu
