// fit_timeline.hip — SPEC §2b, time-windowed backfill over a slot horizon (BASELINE config C5):
// hand-written CDNA4 (gfx950) kernels.  DESIGN.md §3.8.
//
// Node state is each node's free-resource timeline, run-length encoded: a canonical list of runs
// (Seg: end slot, cpu, mem, gpu) in a fixed per-node slab of TL_MAX_SLOTS entries in HBM (only
// the used prefix is ever touched), plus a contiguous 96-B header per node (run count, column
// ceilings, partition mask, first TL_HEAD runs) that the scan streams.  The speculative rounds are
// the plain fit's (fit_common.h): k_scan_tl keeps the exact top-TL_KS keys per (job, block-slice)
// plus a bound against the round-start timelines; k_commit_tl walks the window in priority order
// with a dirty set of at most TL_UCAP nodes (two per lane) whose run lists (and prefix minima)
// live in LDS, re-evaluates them exactly per job and reserves each decision in place.
//   key = start << 54 | score << 22 | position   (earliest start, then best fit, then node)
// The sequential semantics reproduced bit-exactly is oracle/fitref_tl.c:ref_place_tl.
#include <algorithm>

#include "fit_common.h"
#include "fit_engine_ctl.h"

namespace fitgpu {

constexpr int TL_PM_STEPS = 32;     // LDS run lists hold <= 2 * TL_PM_STEPS = 64 runs
#ifndef TL_PAD
#define TL_PAD 1  // runs of padding between two lanes' LDS run-list regions (0: packed, bank-conflicted)
#endif
constexpr int TL_UPL = TL_UCAP / 64;  // dirty slots per lane
#ifndef TL_WAVE_WALKS
#define TL_WAVE_WALKS 12 // walking LDS lists up to which a job walks them one at a time wave-wide
#endif
constexpr int32_t TL_BIG = 0x7fffffff;

#ifdef FIT_STAMPS
// diagnostic build only.  scan: [0] node-loop cycles (sum over waves), [1] nodes, [2] long-walk
// batches, [3] nodes with > TL_HEAD runs, [4] waves.  commit: [comp][0..4] cycles in clean check /
// dirty eval / new dirty / reserve / tail, [5] jobs, [6] new dirty nodes, [7] round-end cycles
__device__ unsigned long long g_tlsc[8];
__device__ unsigned long long g_tlst[64][12];
#define TL_CLK(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define TL_ACC(i, a, b) tacc[i] += (b) - (a)
#else
#define TL_CLK(v)
#define TL_ACC(i, a, b)
#endif

// a VGPR zero the compiler cannot see through: keeps wave-uniform loads on the vector path
// (vmcnt, in order, so a load issued for the next item is not waited for with this one's)
__device__ __forceinline__ int tl_vzero() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

__device__ __forceinline__ uint64_t tl_key(int32_t s, int32_t mc, int32_t mm, int32_t mg,
                                           int32_t jc, int32_t jm, int32_t jg, uint32_t pos) {
    const uint32_t sc = (min((uint32_t)(mg - jg), 255u) << 24) |
                        (min((uint32_t)(mc - jc), 4095u) << 12) |
                        min((uint32_t)(mm - jm) >> 10, 4095u);
    return ((uint64_t)(uint32_t)s << 54) | ((uint64_t)sc << TL_POS_BITS) | pos;
}

// Per-lane state of the earliest-start walk over one node's runs.
struct TlWalk {
    int32_t ra, mc, mm, mg, a;  // start of the current feasible stretch (-1: none), its minima, run start
    bool live;
    // the first d-slot stretch's start and minima, frozen when it completes; the key is packed
    // once after the walk (tl_walk_key) instead of at every run (C5 129.4 -> 128.1 ms, round 3)
    int32_t kra, kmc, kmm, kmg;
    bool got;
};
__device__ __forceinline__ TlWalk tl_walk0(bool live) {
    return TlWalk{-1, 0, 0, 0, 0, live, 0, 0, 0, 0, false};
}

// One run: extend / break the feasible stretch; a stretch of d slots gives the key.  A lane
// stops once every start it could still find is later than `lim` (the start of its cut key).
// Straight-line: every lane computes the step, only a live lane's key / liveness change (a
// finished lane's stretch fields are never read again), so lanes that diverge on "fits" cost no
// exec-mask branches.  `vld` false: a lane's runs past its list's end (it stays false for the
// rest of the walk, so only the key and liveness need the gate).
__device__ __forceinline__ void tl_step_v(TlWalk& w, bool vld, int32_t end, int32_t c, int32_t m,
                                          int32_t g, int32_t jc, int32_t jm, int32_t jg, int32_t d,
                                          int32_t H, int32_t lim, uint32_t pos) {
    const bool f = (c >= jc) & (m >= jm) & (g >= jg);
    const bool nw = w.ra < 0;
    const int32_t ra = f ? (nw ? w.a : w.ra) : -1;
    const int32_t mc = nw ? c : min(w.mc, c), mm = nw ? m : min(w.mm, m), mg = nw ? g : min(w.mg, g);
    const bool done = f & (end - ra >= d);
    const bool kill = f ? (ra > lim) : ((end + d > H) | (end > lim));
    const bool fin = w.live & vld & done;
    w.kra = fin ? ra : w.kra;
    w.kmc = fin ? mc : w.kmc;
    w.kmm = fin ? mm : w.kmm;
    w.kmg = fin ? mg : w.kmg;
    w.got = w.got | fin;
    w.live = vld ? (w.live & !done & !kill) : w.live;
    w.ra = ra;
    w.mc = mc;
    w.mm = mm;
    w.mg = mg;
    w.a = end;
}

__device__ __forceinline__ void tl_step(TlWalk& w, int32_t end, int32_t c, int32_t m, int32_t g,
                                        int32_t jc, int32_t jm, int32_t jg, int32_t d, int32_t H,
                                        int32_t lim, uint32_t pos) {
    tl_step_v(w, true, end, c, m, g, jc, jm, jg, d, H, lim, pos);
}

// the walk's key (KEY_INF: no window found)
__device__ __forceinline__ uint64_t tl_walk_key(const TlWalk& w, int32_t jc, int32_t jm,
                                                int32_t jg, uint32_t pos) {
    return w.got ? tl_key(w.kra, w.kmc, w.kmm, w.kmg, jc, jm, jg, pos) : KEY_INF;
}

// Earliest start of a d-slot window whose every run holds (jc, jm, jg), and its key, for `live`
// lanes walking their node's runs [0, cnt) (any address space; the loop is wave-uniform).
__device__ __forceinline__ uint64_t tl_eval(const Seg* sg, int cnt, bool live, int32_t jc,
                                            int32_t jm, int32_t jg, int32_t d, int32_t H,
                                            uint32_t pos, uint64_t cut) {
    const int32_t lim = cut == KEY_INF ? H : (int32_t)(cut >> 54);
    TlWalk w = tl_walk0(live && d <= H);
    for (int i = 0;; ++i) {
        if (!__ballot(w.live && i < cnt)) break;
        if (w.live && i < cnt) {
            const Seg g = sg[i];
            tl_step(w, g.end, g.cpu, g.mem, g.gpu, jc, jm, jg, d, H, lim, pos);
        }
    }
    return tl_walk_key(w, jc, jm, jg, pos);
}

// Same walk, four runs per step (one round trip for four reads, one ballot per four runs).
// `cap`: readable entries behind sg (reads past the list are clamped into it and masked).
__device__ __forceinline__ uint64_t tl_eval4(const Seg* sg, int cnt, int cap, bool live, int32_t jc,
                                             int32_t jm, int32_t jg, int32_t d, int32_t H,
                                             uint32_t pos, uint64_t cut) {
    const int32_t lim = cut == KEY_INF ? H : (int32_t)(cut >> 54);
    TlWalk w = tl_walk0(live && d <= H);
    for (int i = 0;; i += 4) {
        if (!__ballot(w.live && i < cnt)) break;
        Seg g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = sg[min(i + u, cap - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            tl_step_v(w, i + u < cnt, g[u].end, g[u].cpu, g[u].mem, g[u].gpu, jc, jm, jg, d, H, lim, pos);
    }
    return tl_walk_key(w, jc, jm, jg, pos);
}

// ------------------------------------------------------------------------------ k_build_tl
// One thread per node position: base free columns + sorted release events → canonical runs and
// the node header.  Values are clamped to [-1, INT32_MAX]; slots >= min(H,
// avail / slot_min) hold -1.
__global__ void k_build_tl(const int32_t* __restrict__ cpu, const int32_t* __restrict__ mem,
                           const int32_t* __restrict__ gpu, const int32_t* __restrict__ av,
                           const uint32_t* __restrict__ mask, const int32_t* __restrict__ perm,
                           int32_t nn, int32_t H, int32_t slot_min, const int32_t* __restrict__ off,
                           const int32_t* __restrict__ rs, const int32_t* __restrict__ rc,
                           const int32_t* __restrict__ rm, const int32_t* __restrict__ rg,
                           Seg* __restrict__ slab, TlHdr* __restrict__ hdr,
                           uint32_t* __restrict__ err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    const int x = perm[i];
    Seg* sg = slab + (int64_t)i * TL_MAX_SLOTS;
    const int32_t u = av[x] < 0 ? 0 : min(av[x] / slot_min, H);
    int64_t ac = cpu[x], am = mem[x], ag = gpu[x];
    auto cl = [](int64_t v) { return (int32_t)max<int64_t>(-1, min<int64_t>(v, TL_BIG)); };
    int n = 0, a = 0;
    auto emit = [&](int32_t end, int32_t vc, int32_t vm, int32_t vg) {
        if (end <= a) return;
        if (n > 0 && sg[n - 1].cpu == vc && sg[n - 1].mem == vm && sg[n - 1].gpu == vg)
            sg[n - 1].end = end;
        else
            sg[n++] = Seg{end, vc, vm, vg};
        a = end;
    };
    bool bad = false;
    const int e0 = off ? off[x] : 0, e1 = off ? off[x + 1] : 0;
    if (e1 < e0) bad = true;
    for (int e = e0; e < e1 && !bad; ++e) {
        const int32_t r = rs[e];
        if ((e > e0 && r < rs[e - 1]) || rc[e] < 0 || rm[e] < 0 || rg[e] < 0) {
            bad = true;
            break;
        }
        if (r >= u) continue;  // after the usable horizon: validated only
        if (r > a) emit(r, cl(ac), cl(am), cl(ag));
        ac += rc[e];
        am += rm[e];
        ag += rg[e];
    }
    if (bad) {
        atomicOr(err, 1u);
        n = 0;
        a = 0;
    }
    emit(u, cl(ac), cl(am), cl(ag));
    emit(H, -1, -1, -1);
    TlHdr h;
    h.cnt = n;
    h.cpu = h.mem = h.gpu = -1;
    for (int k = 0; k < n; ++k) {
        h.cpu = max(h.cpu, sg[k].cpu);
        h.mem = max(h.mem, sg[k].mem);
        h.gpu = max(h.gpu, sg[k].gpu);
    }
    h.mask = mask[x];
    h.orig = x;
    h.pad[0] = h.pad[1] = 0;
    for (int k = 0; k < TL_HEAD; ++k) h.head[k] = k < n ? sg[k] : Seg{H, -1, -1, -1};
    hdr[i] = h;
}

// ----------------------------------------------------------------------------- k_scan_tl
// Block = SCAN_JOBS jobs (lanes) × one block-slice of SCAN_WAVES sub-slices; each wave walks its
// nodes in order.  Node headers (96 B, contiguous) stream in through two register sets with
// vector loads two nodes ahead (in-order vmcnt, so the wait for node x never waits for x+1);
// the rare walk past the header's runs reads the slab with scalar loads.  Top-TL_KS lists, bound
// and the LDS merge tree are k_scan's (fit_common.h).
// A round's first job tile (the commit waits for it; STAGE in scan_tile_tl) has every header of its
// block-slice and the runs TL_HEAD .. TL_HEAD + TL_STAGE_RUNS - 1 of every node in LDS: `r8` (that
// node's staged runs) replaces the slab for them.
constexpr int TL_STAGE_RUNS = 8;
template <bool STAGE = false, int K = TL_KS>
__device__ __forceinline__ void tl_scan_node(const TlHdr& h, int x, const JobRec& J, int32_t H,
                                             const Seg* __restrict__ slab, uint64_t (&key)[K],
                                             unsigned long long& batches,
                                             const Seg* __restrict__ r8 = nullptr) {
    const uint64_t cut = key[K - 1];
    const int32_t lim = cut == KEY_INF ? H : (int32_t)(cut >> 54);
    TlWalk w = tl_walk0((h.mask & J.pbit) != 0u && J.wall <= H && J.cpu <= h.cpu &&
                        J.mem <= h.mem && J.gpu <= h.gpu);
    const int cn = __builtin_amdgcn_readfirstlane(h.cnt);
#pragma unroll
    for (int i = 0; i < TL_HEAD; ++i)
        if (i < cn)
            tl_step(w, h.head[i].end, h.head[i].cpu, h.head[i].mem, h.head[i].gpu, J.cpu, J.mem,
                    J.gpu, J.wall, H, lim, (uint32_t)x);
    if (cn > TL_HEAD) {
        const Seg* sg = slab + (int64_t)x * TL_MAX_SLOTS;
        for (int b = TL_HEAD; b < cn; b += TL_HEAD) {
            if (!__ballot(w.live)) break;
            ++batches;
            Seg r4[TL_HEAD];
            if (STAGE && b < TL_HEAD + TL_STAGE_RUNS) {  // uniform
#pragma unroll
                for (int i = 0; i < TL_HEAD; ++i) r4[i] = r8[b - TL_HEAD + i];
            } else {
#pragma unroll
                for (int i = 0; i < TL_HEAD; ++i) r4[i] = sg[b + i];  // inside the slab (TL_HEAD | 1024)
            }
#pragma unroll
            for (int i = 0; i < TL_HEAD; ++i)
                if (b + i < cn)
                    tl_step(w, r4[i].end, r4[i].cpu, r4[i].mem, r4[i].gpu, J.cpu, J.mem, J.gpu,
                            J.wall, H, lim, (uint32_t)x);
        }
    }
    const uint64_t wk = tl_walk_key(w, J.cpu, J.mem, J.gpu, (uint32_t)x);
    if (wk < key[K - 1]) topk_insert(key, wk);
}

// One scan tile: SCAN_JOBS window jobs × block-slice s of the component (host-driven k_scan_tl
// and the persistent k_engine_tl workers).  xk: LDS merge buffer.
// PAIR (k_engine_tl's round-first tile, TL_T0PAIR; P here has half-size sub-slices over twice the
// block-slices): half-slices 2p and 2p+1 each keep their top TL_KS; the half that finishes first
// stores its list (the even half in the candidate slot of block-slice p, the odd half in the
// plan's pair scratch) and counts itself in `pairs[p]`, the second merges the other's list with
// its own into slot p and sets the bound — the same (list, bound) per block-slice as one
// full-size task, from two tasks on two CUs (the commit waits for this tile at every round
// start).  Returns whether the task completes its job tile's block-slice (wave 0).
// STAGE (k_engine_tl's first job tile of a round, which the commit waits for; needs
// SCAN_WAVES * P.sub <= TL_STAGE_NODES): the block first copies its block-slice's headers and every
// node's runs TL_HEAD .. TL_HEAD + TL_STAGE_RUNS - 1 into LDS with vector loads from all 512 lanes
// — one memory round trip — instead of streaming them per node two nodes ahead, each long walk
// another round trip (a lone first tile has nothing on its CU to hide them: ~40 us per task, C5).
constexpr int TL_STAGE_NODES = 256;
constexpr size_t TL_STAGE_BYTES = (sizeof(TlHdr) + sizeof(Seg) * TL_STAGE_RUNS) * TL_STAGE_NODES;
template <bool STAGE = false, int K = TL_KS, bool PAIR = false>
__device__ __forceinline__ bool scan_tile_tl(
    const CompPlan& P, int tile, int s, const Seg* __restrict__ slab,
    const TlHdr* __restrict__ hdr, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, uint64_t* __restrict__ cand, uint64_t* __restrict__ bnd,
    JobRec* __restrict__ wjob, int32_t H, int32_t slot_min, uint64_t (*xk)[K][64],
    unsigned char* __restrict__ stage = nullptr, unsigned* __restrict__ pairs = nullptr) {
    if (tile * SCAN_JOBS >= P.w) return true;  // block-uniform
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int t = tile * SCAN_JOBS + lane;
    const bool active = t < P.w;

    JobRec J;
    J.q = active ? jl[P.jbase + t] : 0;
    J.cpu = active ? jcpu[J.q] : 0;
    J.mem = active ? jmem[J.q] : 0;
    J.gpu = active ? jgpu[J.q] : 0;
    // wall → slots occupied: ceil(wall / slot_min), at least 1 (oracle ref_slots)
    const int64_t dw = active ? ((int64_t)jwall[J.q] + slot_min - 1) / slot_min : 1;
    J.wall = (int32_t)max<int64_t>(1, min<int64_t>(dw, TL_BIG));
    J.pbit = active ? (1u << jpart[J.q]) : 0u;
    J.k = 1;
    J.pad = 0;

    uint64_t key[K];
#pragma unroll
    for (int i = 0; i < K; ++i) key[i] = KEY_INF;
    const int n0 = P.sb + (s * SCAN_WAVES + wave) * P.sub;
    const int n1 = min(P.se, n0 + P.sub);
    unsigned long long batches = 0, longn = 0;
#if defined(FIT_STAMPS) && !defined(FIT_STAMPS_NOSCAN)
    const unsigned long long sc_t0 = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (STAGE) {
        typedef int32_t v4 __attribute__((ext_vector_type(4)));
        const int a = P.sb + s * SCAN_WAVES * P.sub, b = min(P.se, a + SCAN_WAVES * P.sub);
        const int nn = max(b - a, 0);
        TlHdr* const sh = reinterpret_cast<TlHdr*>(stage);
        Seg* const sr = reinterpret_cast<Seg*>(stage + sizeof(TlHdr) * TL_STAGE_NODES);
        {  // headers: 6 x 16 B per node; runs TL_HEAD.. of node i: slab row i, TL_STAGE_RUNS x 16 B
            constexpr int HV = sizeof(TlHdr) / 16;
            const v4* hs = reinterpret_cast<const v4*>(hdr + a);
            v4* hd = reinterpret_cast<v4*>(sh);
            for (int i = threadIdx.x; i < HV * nn; i += SCAN_WAVES * 64) hd[i] = hs[i];
            for (int i = threadIdx.x; i < TL_STAGE_RUNS * nn; i += SCAN_WAVES * 64) {
                const int k = i / TL_STAGE_RUNS, r = i - k * TL_STAGE_RUNS;  // inside the slab row
                const v4 v = *reinterpret_cast<const v4*>(slab + (int64_t)(a + k) * TL_MAX_SLOTS + TL_HEAD + r);
                *reinterpret_cast<v4*>(sr + i) = v;
            }
        }
        __syncthreads();
        for (int x = n0; x < n1; ++x) {
            const TlHdr h = sh[x - a];
            longn += h.cnt > TL_HEAD;
            tl_scan_node<true, K>(h, x, J, H, slab, key, batches, sr + (x - a) * TL_STAGE_RUNS);
        }
    } else if (n0 < n1) {
        const int z = tl_vzero();
        TlHdr h0 = hdr[n0 + z], h1 = hdr[min(n0 + 1, n1 - 1) + z];
        for (int x = n0; x < n1; x += 2) {
            longn += h0.cnt > TL_HEAD;
            tl_scan_node<false, K>(h0, x, J, H, slab, key, batches);
            h0 = hdr[min(x + 2, n1 - 1) + z];
            if (x + 1 < n1) {
                longn += h1.cnt > TL_HEAD;
                tl_scan_node<false, K>(h1, x + 1, J, H, slab, key, batches);
                h1 = hdr[min(x + 3, n1 - 1) + z];
            }
        }
    }
#if defined(FIT_STAMPS) && !defined(FIT_STAMPS_NOSCAN)  // NOSCAN: 5 same-address atomics per wave per task serialise in L2
    if (lane == 0) {
        atomicAdd(&g_tlsc[0], __builtin_amdgcn_s_memtime() - sc_t0);
        atomicAdd(&g_tlsc[1], (unsigned long long)max(n1 - n0, 0));
        atomicAdd(&g_tlsc[2], batches);
        atomicAdd(&g_tlsc[3], longn);
        atomicAdd(&g_tlsc[4], 1ull);
    }
#else
    (void)batches;
    (void)longn;
#endif
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
    if constexpr (!PAIR && FIT_COALESCED_LISTS) {
        // every thread: the lists out through LDS, coalesced (store_lists_through, fit_common.h)
        const int na = max(0, min(SCAN_JOBS, P.w - tile * SCAN_JOBS));
        store_lists_through<K>(reinterpret_cast<uint64_t*>(xk), wave == 0, lane, key, K,
                               cand + P.cand_off + ((int64_t)(tile * SCAN_JOBS) * P.nslice + s) * K,
                               (int64_t)P.nslice * K, na);
        if (wave != 0 || !active) return true;
        if (key[K - 1] != KEY_INF)
            atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                      (unsigned long long)key[K - 1]);
        if (s == 0) store_job<true>(wjob + P.slot0 + t, J);
        return true;
    }
    if (wave != 0) return true;
    if constexpr (PAIR) {
        const int ns = P.nslice >> 1, pr = s >> 1;
        uint64_t* const fin = cand + P.cand_off + ((int64_t)t * ns + pr) * K;
        uint64_t* const tmp = cand + P.pair_off + ((int64_t)lane * 32 + pr) * K;  // tile 0: t = lane
        uint64_t* const mine = (s & 1) ? tmp : fin;
        uint64_t* const other = (s & 1) ? fin : tmp;
        if (active) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                __hip_atomic_store(mine + i, key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (s == 0) store_job<true>(wjob + P.slot0 + t, J);
        }
        // R1: the list stored through and drained before the count the partner reads
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned prev = 0u;
        if (lane == 0) prev = __hip_atomic_fetch_add(pairs + pr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_readfirstlane((int)prev) == 0) return false;  // the partner merges
        if (active) {
            uint64_t o[K];
#pragma unroll
            for (int i = 0; i < K; ++i)
                o[i] = __hip_atomic_load(other + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    uint64_t* dst = cand + P.cand_off + ((int64_t)t * P.nslice + s) * K;
    // written through (sc1): k_engine_tl's commit reads them in the same launch and the worker
    // counts the tile done with no release fence (scan_tile, fit_common.h)
#pragma unroll
    for (int i = 0; i < K; ++i)
        __hip_atomic_store(dst + i, key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (key[K - 1] != KEY_INF)
        atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                  (unsigned long long)key[K - 1]);
    if (s == 0) store_job<true>(wjob + P.slot0 + t, J);
    return true;
}

__global__ __launch_bounds__(SCAN_WAVES * 64) void k_scan_tl(
    const Seg* __restrict__ slab, const TlHdr* __restrict__ hdr,
    const int32_t* __restrict__ jl, const int32_t* __restrict__ jcpu,
    const int32_t* __restrict__ jmem, const int32_t* __restrict__ jgpu,
    const int32_t* __restrict__ jwall, const uint16_t* __restrict__ jpart,
    const CompPlan* __restrict__ plan, int ncomp, uint64_t* __restrict__ cand,
    uint64_t* __restrict__ bnd, JobRec* __restrict__ wjob, int32_t H, int32_t slot_min) {
    __shared__ uint64_t xk[SCAN_WAVES / 2][TL_KS][64];
    const int c = find_comp(plan, ncomp, blockIdx.x);
    const CompPlan P = plan[c];
    const int local = blockIdx.x - P.blk0;
    const int tile = __builtin_amdgcn_readfirstlane(local / P.nslice);
    const int s = __builtin_amdgcn_readfirstlane(local - tile * P.nslice);
    scan_tile_tl(P, tile, s, slab, hdr, jl, jcpu, jmem, jgpu, jwall, jpart, cand, bnd, wjob, H,
                 slot_min, xk);
}

// --------------------------------------------------------------------------- k_commit_tl
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Three independent inclusive min-scans (a run list's cpu / mem / gpu columns), interleaved so
// that each fused v_min_i32_dpp reads a VGPR written two instructions earlier (the DPP hazard's
// two wait states, cdna_hip_programming.md) — 18 VALU and one s_nop.  A lane whose DPP source does
// not exist (row_shr at a row's start) or whose row the row_mask leaves out keeps its value
// (bound_ctrl not set), i.e. min(v, TL_BIG) = v.
__device__ __forceinline__ void wave_scan_min3(int32_t& a, int32_t& b, int32_t& c) {
#define TL_L3(CTL) "v_min_i32_dpp %0, %0, %0 " CTL "\n\tv_min_i32_dpp %1, %1, %1 " CTL \
                   "\n\tv_min_i32_dpp %2, %2, %2 " CTL "\n\t"
    asm volatile("s_nop 1\n\t"
                 TL_L3("row_shr:1 row_mask:0xf bank_mask:0xf")
                 TL_L3("row_shr:2 row_mask:0xf bank_mask:0xf")
                 TL_L3("row_shr:4 row_mask:0xf bank_mask:0xf")
                 TL_L3("row_shr:8 row_mask:0xf bank_mask:0xf")
                 TL_L3("row_bcast:15 row_mask:0xa bank_mask:0xf")
                 TL_L3("row_bcast:31 row_mask:0xc bank_mask:0xf")
                 : "+v"(a), "+v"(b), "+v"(c));
#undef TL_L3
}

// Prefix minima of an LDS run list (<= 64 runs): PM[i] = min over runs [0, i] per column.
// With them, "fits from slot 0 for d slots" and that window's minimum are one search over the
// run ends — the dirty-node fast path.
__device__ __forceinline__ void tl_pm_build(const Seg* L, int4* PM, int n) {
    const int lane = threadIdx.x & 63;
    const Seg g = lane < n ? L[lane] : Seg{0, TL_BIG, TL_BIG, TL_BIG};
    int32_t vc = g.cpu, vm = g.mem, vg = g.gpu;
    wave_scan_min3(vc, vm, vg);
    if (lane < n) PM[lane] = make_int4(vc, vm, vg, 0);
}

// The walk of tl_eval4 over an LDS run list of n <= 64 runs, by the whole wave (one run per
// lane) instead of one lane: a window can only start where a maximal stretch of fitting runs
// starts (slot 0 or the end of a run that does not fit), so the earliest window is the first run
// w that fits and ends >= d slots after its stretch's start ra; its minima are those of the runs
// from the stretch's first to w.  Same key as the serial walk (tl_step), including the `lim` cut.
__device__ __forceinline__ uint64_t tl_walk_wave(const Seg* L, int n, int32_t jc, int32_t jm,
                                                 int32_t jg, int32_t d, int32_t lim, uint32_t pos) {
    const int lane = threadIdx.x & 63;
    const bool v = lane < n;
    const Seg g = v ? L[lane] : Seg{TL_BIG, 0, 0, 0};
    const bool f = v && g.cpu >= jc && g.mem >= jm && g.gpu >= jg;
    const uint64_t below = __ballot(!f) & ((1ull << lane) - 1ull);
    const int sidx = below ? 64 - __builtin_clzll(below) : 0;  // first run of this lane's stretch
    const int32_t pe = __shfl(g.end, max(sidx - 1, 0));
    const int32_t ra = sidx ? pe : 0;
    const uint64_t mw = __ballot(f && g.end - ra >= d);
    if (!mw) return KEY_INF;
    const int w = __builtin_ctzll(mw);
    const int32_t st = __builtin_amdgcn_readlane(ra, w);
    if (st > lim) return KEY_INF;
    const int s0 = __builtin_amdgcn_readlane(sidx, w);
    const bool in = lane >= s0 && lane <= w;
    int32_t sc = in ? g.cpu : TL_BIG, sm = in ? g.mem : TL_BIG, sg = in ? g.gpu : TL_BIG;
    wave_scan_min3(sc, sm, sg);
    const int32_t mc = __builtin_amdgcn_readlane(sc, 63);
    const int32_t mm = __builtin_amdgcn_readlane(sm, 63);
    const int32_t mg = __builtin_amdgcn_readlane(sg, 63);
    return tl_key(st, mc, mm, mg, jc, jm, jg, pos);
}

// Reserve (jc, jm, jg) on slots [s, e) of a run list, general form (any length, any address
// space), by the whole wave: the runs from the one before the window to the end are split at s
// and e into LDS scratch (prefix sums over piece counts), equal neighbours merge, and the result
// is written back.  Returns the new run count.
__device__ __forceinline__ int tl_reserve_any(Seg* sg, int n, int32_t s, int32_t e, int32_t jc,
                                              int32_t jm, int32_t jg, Seg* scr) {
    const int lane = threadIdx.x & 63;
    int i0 = n;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        const uint64_t m = __ballot(i < n && sg[i].end > s);
        if (m) {
            i0 = b + __builtin_ctzll(m);
            break;
        }
    }
    const int r0 = max(i0 - 1, 0);
    int np = 0;
    for (int b = r0; b < n; b += 64) {
        const int i = b + lane;
        const bool v = i < n;
        const Seg g = v ? sg[i] : Seg{0, 0, 0, 0};
        const int32_t a = (v && i > 0) ? sg[i - 1].end : 0;
        const bool ov = v && a < e && g.end > s;
        const bool hd = ov && a < s;
        const bool tl = ov && g.end > e;
        const int pc = v ? (ov ? 1 + (int)hd + (int)tl : 1) : 0;
        const uint64_t m0 = __ballot(pc & 1), m1 = __ballot(pc >> 1);
        int o = np + lanes_below(m0) + 2 * lanes_below(m1);
        if (v) {
            if (!ov) {
                scr[o] = g;
            } else {
                if (hd) scr[o++] = Seg{s, g.cpu, g.mem, g.gpu};
                scr[o++] = Seg{min(g.end, e), g.cpu - jc, g.mem - jm, g.gpu - jg};
                if (tl) scr[o] = g;
            }
        }
        np += __popcll(m0) + 2 * __popcll(m1);
    }
    int no = 0;
    for (int b = 0; b < np; b += 64) {
        const int k = b + lane;
        const Seg p = k < np ? scr[k] : Seg{0, 0, 0, 0};
        const Seg q = k + 1 < np ? scr[k + 1] : Seg{0, -2, -2, -2};
        const bool keep = k < np && (k + 1 >= np || p.cpu != q.cpu || p.mem != q.mem || p.gpu != q.gpu);
        const uint64_t mk = __ballot(keep);
        if (keep) sg[r0 + no + lanes_below(mk)] = p;
        no += __popcll(mk);
    }
    return r0 + no;
}

// Reserve on an LDS list of n <= 64 runs held in registers: one read, the edges resolved with
// readlanes, one write of the shifted runs.  Runs overlapping [s, e) lose the demand; the run
// holding s (e) splits when s (e) falls inside it; the first (last) reduced run merges into its
// left (right) neighbour when their values become equal — the only places the list can change
// shape, so it stays canonical.  Returns the new count, or -1 (list untouched) if it would
// exceed `cap` runs.
__device__ __forceinline__ int tl_reserve_lds(Seg* L, int n, int cap, int32_t s, int32_t e,
                                              int32_t jc, int32_t jm, int32_t jg) {
    const int lane = threadIdx.x & 63;
    const bool v = lane < n;
    const Seg g = v ? L[lane] : Seg{TL_BIG, 0, 0, 0};
    const int32_t a = (v && lane > 0) ? L[lane - 1].end : 0;
    const uint64_t mov = __ballot(v && a < e && g.end > s);
    const int i0 = __builtin_ctzll(mov), i1 = 63 - __builtin_clzll(mov);
    const int32_t a0 = __builtin_amdgcn_readlane(a, i0), e1 = __builtin_amdgcn_readlane(g.end, i1);
    const int head = a0 < s, tail = e1 > e;
    const int32_t c0 = __builtin_amdgcn_readlane(g.cpu, i0) - jc;
    const int32_t m0 = __builtin_amdgcn_readlane(g.mem, i0) - jm;
    const int32_t g0 = __builtin_amdgcn_readlane(g.gpu, i0) - jg;
    const int32_t c1 = __builtin_amdgcn_readlane(g.cpu, i1) - jc;
    const int32_t m1 = __builtin_amdgcn_readlane(g.mem, i1) - jm;
    const int32_t g1 = __builtin_amdgcn_readlane(g.gpu, i1) - jg;
    const int il = max(i0 - 1, 0), ir = min(i1 + 1, 63);
    const int mergeL = !head && i0 > 0 && __builtin_amdgcn_readlane(g.cpu, il) == c0 &&
                       __builtin_amdgcn_readlane(g.mem, il) == m0 &&
                       __builtin_amdgcn_readlane(g.gpu, il) == g0;
    const int mergeR = !tail && i1 < n - 1 && __builtin_amdgcn_readlane(g.cpu, ir) == c1 &&
                       __builtin_amdgcn_readlane(g.mem, ir) == m1 &&
                       __builtin_amdgcn_readlane(g.gpu, ir) == g1;
    const int nn = n + head + tail - mergeL - mergeR;
    if (nn > cap) return -1;
    const int sh = head - mergeL;                       // index shift of the reduced runs
    const int st = head + tail - mergeL - mergeR;       // index shift of the runs after them
    if (v && lane >= i0 && lane <= i1) {
        if (lane == i0 && head) L[i0] = Seg{s, g.cpu, g.mem, g.gpu};
        if (!(lane == i1 && mergeR))
            L[lane + sh] = Seg{min(g.end, e), g.cpu - jc, g.mem - jm, g.gpu - jg};
        if (lane == i1 && tail) L[i1 + sh + 1] = g;
    } else if (v && lane > i1 && st != 0) {
        L[lane + st] = g;
    }
    return nn;
}

// One wave per component: the speculative-prefix commit (fit_common.h) over timelines.  A node
// that becomes dirty has its run list copied into an LDS region of R (<= 64) runs with prefix
// minima (lists that are or grow longer move to the global slab and take the general paths).
// Per job, on the fast path, every wait is on LDS or on loads issued one job earlier: the job
// stream (row, bound, candidate keys) is prefetched with vector loads (in-order vmcnt), and the
// dirty evaluation, reservation and prefix-minimum update are LDS-only.
// One component's window, by one wave (the host-driven k_commit_tl: its window's scan is complete
// before the launch, so nothing here waits; k_engine_tl commits on the decider / helper split).  smem: commit_tl_lds_bytes() of LDS.
template <int EPL>
__device__ __forceinline__ CommitResult commit_tl_window(
    const CompPlan& P, int c, unsigned char* smem, Seg* __restrict__ slab,
    TlHdr* __restrict__ hdr, const uint64_t* __restrict__ cand, int64_t rank_stride, int nranks,
    const uint64_t* __restrict__ bnd, const JobRec* __restrict__ wjob,
    const int32_t* __restrict__ perm, int32_t* __restrict__ out, int32_t* __restrict__ outs,
    int32_t H, int32_t R) {
    Seg* scr = reinterpret_cast<Seg*>(smem);                // general-path scratch
    // TL_UCAP regions of R runs, TL_PAD runs apart beyond R: a lane's region starts 16 B further
    // along the banks than its neighbour's, so the lanes' reads of their own lists (the 4-ary
    // search, the prefix-minimum read) spread over the banks instead of all hitting one (a
    // 1,024-B stride maps every lane of a ds_read_b32 group to the same bank: 32-way)
    const int32_t RS = R > 0 ? R + TL_PAD : 0;  // no regions when R = 0 (every list global)
    Seg* lr = scr + TL_MAX_SLOTS;
    int4* pmr = reinterpret_cast<int4*>(lr + TL_UCAP * RS);  // their prefix minima
    uint32_t* bitmap = reinterpret_cast<uint32_t*>(pmr + TL_UCAP * RS);
    const int lane = threadIdx.x & 63;
    if (P.w == 0) return CommitResult{0, 0, 0, 0};
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = lane; i < nwords; i += 64) bitmap[i] = 0u;

    const int per_rank = P.nslice * TL_KS;
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
    const uint32_t nb = (uint32_t)P.nb;
    const int z = tl_vzero();
    int nu = 0, placed = 0, stop = 0, t = 0;
    // this lane's dirty node (lane < nu): position, mask, id, run count, column ceilings, and
    // whether its list lives in the global slab instead of LDS
    // dirty slot u = i * 64 + lane, i < TL_UPL (register arrays indexed by literals / unrolled loops)
    uint32_t upos[TL_UPL], umask[TL_UPL];
    int32_t uorig[TL_UPL], ucnt[TL_UPL], ucc[TL_UPL], ucm[TL_UPL], ucg[TL_UPL];
    bool uglob[TL_UPL];
#pragma unroll
    for (int i = 0; i < TL_UPL; ++i) {
        upos[i] = umask[i] = 0u;
        uorig[i] = -1;
        ucnt[i] = 0;
        ucc[i] = ucm[i] = ucg[i] = -1;
        uglob[i] = false;
    }
    // the placement of job t is parked in lane t & 63 and stored 64 at a time (no store per job:
    // on gfx9 stores count in vmcnt, and the next prefetch wait would wait for them)
    int32_t oq = -1, on = -1, os = -1;

#ifdef FIT_STAMPS
    unsigned long long tacc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    auto ld64 = [&](const uint64_t* p) { return *p; };
    auto ldjob = [&](const JobRec* p) { return *p; };
    JobRec J = ldjob(wjob + P.slot0 + z);
    uint64_t B = ld64(bnd + P.slot0 + z);
    uint64_t kr[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) kr[k] = ld64(cand + off[k]);
    for (; t < P.w; ++t) {
        TL_CLK(c0);
        uint64_t cm = KEY_INF;
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            const uint64_t kk = kr[k];
            const bool v = has[k] && kk <= B && kk != KEY_INF;
            const uint32_t rel = v ? ((uint32_t)kk & TL_POS_MASK) - nb : 0u;
            const bool clean = v && !((bitmap[rel >> 5] >> (rel & 31)) & 1u);
            cm = umin64(cm, clean ? kk : KEY_INF);
        }
        const int32_t jq = __builtin_amdgcn_readfirstlane(J.q);
        const int32_t jc = __builtin_amdgcn_readfirstlane(J.cpu);
        const int32_t jm = __builtin_amdgcn_readfirstlane(J.mem);
        const int32_t jg = __builtin_amdgcn_readfirstlane(J.gpu);
        const int32_t jd = __builtin_amdgcn_readfirstlane(J.wall);
        const uint32_t jp = (uint32_t)__builtin_amdgcn_readfirstlane((int)J.pbit);
        const uint64_t Bc =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(B >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)B);
        {  // the next job's stream, in flight during this one
            const int tn = min(t + 1, P.w - 1);
            J = ldjob(wjob + P.slot0 + tn + z);
            B = ld64(bnd + P.slot0 + tn + z);
#pragma unroll
            for (int k = 0; k < EPL; ++k) kr[k] = ld64(cand + off[k] + (int64_t)tn * per_rank);
        }
        const uint64_t cw = wave_min_key(cm);
        // a clean node can only win as cw: fetch its header, first 64 runs and id now, so a new
        // dirty node costs no memory round trip when the decision comes
        const uint32_t cpos = cw != KEY_INF ? ((uint32_t)cw & TL_POS_MASK) : (uint32_t)P.nb;
        const TlHdr ch = hdr[cpos + z];
        const Seg crun = slab[(int64_t)cpos * TL_MAX_SLOTS + lane];
        const int32_t corig = ch.orig;
        TL_CLK(c1);
        TL_ACC(0, c0, c1);
        // LDS lists: a start at slot 0 through the prefix minima — k = the first run ending at or
        // after d, by a 4-ary search (three rounds of three independent reads); a later start
        // (only when it can still win) or a global list walks the runs
        uint64_t dk[TL_UPL], dkm = KEY_INF;
        bool walk[TL_UPL], anyw = false, fit0 = false;
#pragma unroll
        for (int i = 0; i < TL_UPL; ++i) {
            const bool dl = i * 64 + lane < nu && (umask[i] & jp) != 0u && jc <= ucc[i] &&
                            jm <= ucm[i] && jg <= ucg[i] && jd <= H;
            dk[i] = KEY_INF;
            walk[i] = dl && uglob[i];
            if (dl && !uglob[i]) {
                const Seg* const mine = lr + (i * 64 + lane) * RS;
                int k = 0;
#pragma unroll
                for (int q = 16; q >= 1; q >>= 2) {
                    // k + 3q - 1 <= 63: clamp into the region, read unconditionally (the three
                    // reads issue together), mask past the list
                    const int i1 = k + q - 1, i2 = k + 2 * q - 1, i3 = k + 3 * q - 1;
                    const int32_t y1 = mine[min(i1, R - 1)].end, y2 = mine[min(i2, R - 1)].end,
                                  y3 = mine[min(i3, R - 1)].end;
                    const int32_t x1 = i1 < ucnt[i] ? y1 : TL_BIG;
                    const int32_t x2 = i2 < ucnt[i] ? y2 : TL_BIG;
                    const int32_t x3 = i3 < ucnt[i] ? y3 : TL_BIG;
                    k += q * ((x1 < jd) + (x2 < jd) + (x3 < jd));
                }
                const int4 pk = pmr[(i * 64 + lane) * RS + k];
                if (pk.x >= jc && pk.y >= jm && pk.z >= jg) {
                    dk[i] = tl_key(0, pk.x, pk.y, pk.z, jc, jm, jg, upos[i]);
                    fit0 = true;
                } else {
                    walk[i] = cw == KEY_INF || (cw >> 54) > 0;
                }
            }
        }
        // a walk of an LDS list only runs after its start-0 window failed, so it can only find a
        // later start: once any dirty list fits from slot 0, those walks cannot win (global lists
        // still walk, cut at start 0, as they may hold a better-scored start-0 window)
        const bool any0 = __ballot(fit0) != 0;
        uint64_t cutw = any0 ? 0ull : cw;
#pragma unroll
        for (int i = 0; i < TL_UPL; ++i) {
            walk[i] = walk[i] && (uglob[i] || !any0);
            anyw = anyw || walk[i];
        }
        TL_CLK(c1b);
        TL_ACC(8, c1, c1b);
        if (__ballot(anyw)) {
#ifdef FIT_STAMPS
            tacc[10] += 1;
#endif
            const int32_t wlim = cutw == KEY_INF ? H : (int32_t)(cutw >> 54);
#pragma unroll
            for (int i = 0; i < TL_UPL; ++i) {
                if (!__ballot(walk[i])) continue;
                // LDS lists: one wave-wide walk per walking list when few lists walk, else one
                // lane per list (the serial walks run side by side)
                uint64_t wl = KEY_INF;
                const uint64_t mlds = __ballot(walk[i] && !uglob[i]);
                if (__popcll(mlds) > TL_WAVE_WALKS) {
                    wl = tl_eval4(lr + (i * 64 + lane) * RS, ucnt[i], R, walk[i] && !uglob[i], jc,
                                  jm, jg, jd, H, upos[i], cutw);
                } else for (uint64_t mwl = mlds; mwl; mwl &= mwl - 1) {
                    const int ll = __builtin_ctzll(mwl);
                    const int n = __builtin_amdgcn_readlane(ucnt[i], ll);
                    const uint32_t p = (uint32_t)__builtin_amdgcn_readlane((int)upos[i], ll);
                    const uint64_t k = tl_walk_wave(lr + (i * 64 + ll) * RS, n, jc, jm, jg, jd, wlim, p);
                    if (lane == ll) wl = k;
                }
                uint64_t wg = KEY_INF;
                if (__ballot(walk[i] && uglob[i]))
                    wg = tl_eval4(slab + (int64_t)upos[i] * TL_MAX_SLOTS, ucnt[i], TL_MAX_SLOTS,
                                  walk[i] && uglob[i], jc, jm, jg, jd, H, upos[i], cutw);
                dk[i] = walk[i] ? (uglob[i] ? wg : wl) : dk[i];
            }
        }
#pragma unroll
        for (int i = 0; i < TL_UPL; ++i) dkm = umin64(dkm, dk[i]);
        TL_CLK(c1c);
        TL_ACC(9, c1b, c1c);
        const uint64_t best = umin64(cw, wave_min_key(dkm));
        TL_CLK(c2);
        TL_ACC(1, c1, c2);
        if (Bc != KEY_INF && best > Bc) {
            stop = 1;  // a node outside the candidate lists could win: rescan next round
            break;
        }
        int32_t node = -1, start = -1;
        if (best != KEY_INF) {
            const uint32_t pos = (uint32_t)best & TL_POS_MASK;
            int l = -1;  // winning dirty slot
#pragma unroll
            for (int i = TL_UPL - 1; i >= 0; --i) {
                const uint64_t dm = __ballot(dk[i] == best);
                if (dm) l = i * 64 + __builtin_ctzll(dm);
            }
            TL_CLK(c3);
            if (l < 0) {  // a clean candidate wins: it becomes dirty slot nu
                if (nu == TL_UCAP) {
                    stop = 2;
                    break;
                }
                l = nu++;
                // pos == cpos: the winner is the clean best (prefetched above)
                const TlHdr& h0 = ch;
                const int n0 = __builtin_amdgcn_readfirstlane(h0.cnt);
                const bool g = n0 > R;
                if (!g) {
                    Seg* dst = lr + l * RS;
                    if (lane < n0) dst[lane] = crun;  // n0 <= R <= 64
                    tl_pm_build(dst, pmr + l * RS, n0);
                }
                {
                    TL_CLK(c3h);
                    TL_ACC(11, c3, c3h);  // header + runs wait, LDS copy, prefix minima
                }
                const int32_t o0 = corig;
#pragma unroll
                for (int i = 0; i < TL_UPL; ++i)
                    if (i * 64 + lane == l) {
                        upos[i] = pos;
                        umask[i] = h0.mask;
                        uorig[i] = o0;
                        ucnt[i] = n0;
                        ucc[i] = h0.cpu;
                        ucm[i] = h0.mem;
                        ucg[i] = h0.gpu;
                        uglob[i] = g;
                    }
                if (lane == 0) {
                    const uint32_t rel = pos - nb;
                    bitmap[rel >> 5] |= 1u << (rel & 31);
                }
#ifdef FIT_STAMPS
                tacc[6] += 1;
#endif
            }
            TL_CLK(c4);
            TL_ACC(2, c3, c4);
            const int li = l >> 6, ll = l & 63;
            bool g = false;
            int n = 0, orig = -1;
#pragma unroll
            for (int i = 0; i < TL_UPL; ++i)
                if (i == li) {
                    g = __builtin_amdgcn_readlane((int)uglob[i], ll) != 0;
                    n = __builtin_amdgcn_readlane(ucnt[i], ll);
                    orig = __builtin_amdgcn_readlane(uorig[i], ll);
                }
            start = (int32_t)(best >> 54);
            int nn;
            if (!g) {
                Seg* L = lr + l * RS;
                nn = tl_reserve_lds(L, n, R, start, start + jd, jc, jm, jg);
                if (nn >= 0) {
                    tl_pm_build(L, pmr + l * RS, nn);
                } else {  // outgrows its LDS region: move the list to the global slab
                    Seg* gl = slab + (int64_t)pos * TL_MAX_SLOTS;
                    if (lane < n) gl[lane] = L[lane];
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    nn = tl_reserve_any(gl, n, start, start + jd, jc, jm, jg, scr);
#pragma unroll
                    for (int i = 0; i < TL_UPL; ++i)
                        if (i * 64 + lane == l) uglob[i] = true;
                }
            } else {
                nn = tl_reserve_any(slab + (int64_t)pos * TL_MAX_SLOTS, n, start, start + jd, jc,
                                    jm, jg, scr);
            }
#pragma unroll
            for (int i = 0; i < TL_UPL; ++i)
                if (i * 64 + lane == l) ucnt[i] = nn;
            node = orig;
            ++placed;
            TL_CLK(c5);
            TL_ACC(3, c4, c5);
        }
        TL_CLK(c6);
        if (lane == (t & 63)) {
            oq = jq;
            on = node;
            os = start;
        }
        if ((t & 63) == 63) {  // uniform
            if (oq >= 0) {
                out[oq] = on;
                outs[oq] = os;
            }
            oq = -1;
        }
        TL_CLK(c7);
        TL_ACC(4, c6, c7);
    }
    if (oq >= 0 && lane < (t & 63)) {  // the last partial group
        out[oq] = on;
        outs[oq] = os;
    }
    TL_CLK(e0);
    // round end: LDS lists back to their slabs (the next scan reads them), headers for all
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // global-list writes before re-reads
    for (int l = 0; l < nu; ++l) {
        const int li = l >> 6, ll = l & 63;
        uint32_t p = 0;
        int n = 0;
        bool gl = false;
#pragma unroll
        for (int i = 0; i < TL_UPL; ++i)
            if (i == li) {
                p = (uint32_t)__builtin_amdgcn_readlane((int)upos[i], ll);
                n = __builtin_amdgcn_readlane(ucnt[i], ll);
                gl = __builtin_amdgcn_readlane((int)uglob[i], ll) != 0;
            }
        Seg* dst = slab + (int64_t)p * TL_MAX_SLOTS;
        Seg hd = Seg{H, -1, -1, -1};
        if (!gl) {
            const Seg* src = lr + l * RS;
            if (lane < n) {
                hd = src[lane];
                dst[lane] = hd;
            }
        } else if (lane < TL_HEAD && lane < n) {
            hd = dst[lane];
        }
        if (lane < TL_HEAD) hdr[p].head[lane] = hd;
    }
#pragma unroll
    for (int i = 0; i < TL_UPL; ++i)
        if (i * 64 + lane < nu) hdr[upos[i]].cnt = ucnt[i];
#ifdef FIT_STAMPS
    TL_CLK(e1);
    tacc[7] += e1 - e0;
    tacc[5] += t;
    if (lane == 0)
        for (int i = 0; i < 12; ++i) atomicAdd(&g_tlst[c & 63][i], tacc[i]);
#endif
    return CommitResult{t, stop, nu, placed};
}

template <int EPL>
__global__ __launch_bounds__(64) void k_commit_tl(
    Seg* __restrict__ slab, TlHdr* __restrict__ hdr, const CompPlan* __restrict__ plan,
    const uint64_t* __restrict__ cand, int64_t rank_stride, int nranks,
    const uint64_t* __restrict__ bnd, const JobRec* __restrict__ wjob,
    const int32_t* __restrict__ perm, int32_t* __restrict__ out, int32_t* __restrict__ outs,
    CommitResult* __restrict__ res, int32_t H, int32_t R) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int c = blockIdx.x;
    const CompPlan P = plan[c];
    const CommitResult r = commit_tl_window<EPL>(P, c, smem, slab, hdr, cand, rank_stride, nranks,
                                                 bnd, wjob, perm, out, outs, H, R);
    if (threadIdx.x == 0) res[c] = r;
}

}  // namespace fitgpu
#include "fit_commit_tl_mw.h"
namespace fitgpu {

// ------------------------------------------------------------------------------ k_engine_tl
// The whole backfill placement in ONE launch, on k_engine's protocol
// (fit_persistent.hip, fit_engine_ctl.h): blocks [0, C) are committers — one wave each runs the
// component's rounds (publish its scan tiles to the device task ring, wait for them, commit the
// window with commit_tl_window); blocks [C, C+W) are scan workers running scan_tile_tl.
// Components advance at their own pace and their scans share the chip; no host round trips.
// MODE 0: one launch holds both (blocks [0, C) commit, the rest scan); MODE 1 / 2: the committers
// and the scan workers as two concurrent launches (FIT_TL_SPLIT, engine.cpp): the workers' launch
// then carries only the scan's registers and LDS, so several worker blocks share a CU (one block
// per CU when the committer's 160 KB of LDS and its helpers' VGPRs size every block of the launch).
// A MODE 1 block counts itself into `resident` (host-mapped) so that the host launches the
// workers only once every committer holds its CU.
#ifndef TL_T0PAIR
#define TL_T0PAIR 1  // k_engine_tl: a round's first job tile as 2 x nslice half-size block-slices, paired
#endif
// the worker's LDS: merge buffer, task slot, then the first tile's stage (scan_tile_tl STAGE)
constexpr size_t TL_STAGE_OFF = (sizeof(uint64_t) * (SCAN_WAVES / 2) * TL_KS * 64 + 16 + 63) & ~(size_t)63;

template <int MODE>
__global__ __launch_bounds__(SCAN_WAVES * 64) void k_engine_tl(
    EngineCtl* __restrict__ ctl, unsigned long long* __restrict__ ring,
    const CompState* __restrict__ cs, CompOut* __restrict__ co, CompPlan* __restrict__ plans,
    int ncomp, Seg* __restrict__ slab, TlHdr* __restrict__ hdr, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, uint64_t* __restrict__ cand, uint64_t* __restrict__ bnd,
    JobRec* __restrict__ wjob, const int32_t* __restrict__ perm, int32_t* __restrict__ out,
    int32_t* __restrict__ outs, int32_t H, int32_t slot_min, int32_t R,
    int64_t* __restrict__ wbusy, unsigned* __restrict__ resident, unsigned wd) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) stamp_start(ctl);

    if (MODE == 1 || (MODE == 0 && (int)blockIdx.x < ncomp)) {
        if (MODE == 1 && threadIdx.x == 0)
            __hip_atomic_fetch_add(resident, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // ================================================================ committer
        // wave 0 runs the round protocol (publish the window's tiles), then all 8 waves commit
        // it (fit_commit_tl_mw.h: wave 0 decides, waves 1..7 pre-resolve)
        __shared__ int s_fail;
        const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const int c = blockIdx.x;
        const CompState S = cs[c];
        if (threadIdx.x == 0) reinterpret_cast<TmShared*>(smem)->wd = wd;  // commit waits' deadline
        int32_t cursor = S.jstart, win = S.wmin;
        unsigned target[2] = {0u, 0u};  // tiles published by the rounds of each parity (fit_engine_ctl.h)
        unsigned used[2] = {0u, 0u};    // job tiles whose bounds the last round of each parity reset
                                        // and its scans lowered (k_engine's, fit_persistent.hip)
        int64_t evals = 0, placed = 0, rounds = 0, sr = 0, sd = 0, tc = 0, tw = 0;
        bool fail = false;
        bool glob = false;  // the last window wrote a global-slab list (plain stores)
        while (cursor < S.jend) {
            const int w = min(win, S.jend - cursor);
            const unsigned rnd = (unsigned)rounds + 1u;  // task round tag
            const int par = (int)(rnd & 1u);              // buffer set of this round
            CompPlan P;
            P.nb = S.nb;
            P.ne = S.ne;
            P.sb = S.sb;
            P.se = S.se;
            P.nslice = S.nslice;
            P.sub = S.sub;
            P.ks = S.ks;
            P.jbase = cursor;
            P.w = w;
            P.blk0 = 0;
            P.cand_off = par ? S.cand_alt : S.cand_off;
            P.slot0 = par ? S.slot_alt : S.slot0;
            // the round's first job tile as pairs of half-slices (scan_tile_tl PAIR): the commit
            // waits for it at every round start
            P.k0 = (TL_T0PAIR && 2 * S.nslice <= 64) ? 2 : 0;
            P.pair_off = S.pair_off + (par ? PAIR_AREA : 0);
            const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
            if (wave == 0) {
                // the tiles of the window before last (this round's buffer set; also those past
                // its stop) must all be complete before their buffers and counters are reused
                bool f = !wait_tiles(ctl, c, par, target[par], wd, rnd);
                const unsigned ntj = (unsigned)((w + SCAN_JOBS - 1) / SCAN_JOBS);
                store_through(&plans[2 * c + par], P);  // as k_engine's (fit_persistent.hip)
                const int nres = min((int)used[par] * SCAN_JOBS, S.wmax);  // within the slot region
                for (int i = lane; i < nres; i += 64) store_through64(&bnd[P.slot0 + i], KEY_INF);
                for (unsigned i = lane; i < ntj; i += 64)
                    __hip_atomic_store(&ctl->tdone[par][c][i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane < 32) __hip_atomic_store(&ctl->tpair[par][c][lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // plan, bound / counter reset and the last window's run lists and headers were
                // stored through (sc1; R1: drained before the publish); a global-slab list was
                // not: release it (≈1.7-6.5 us on the round-start path otherwise)
                if (glob) release_agent();
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // the first TL_AHEAD job tiles now, the rest by the helpers just in time
                // (tm_tile_ready)
                const unsigned npub = TL_AHEAD > 0 ? min(ntj, (unsigned)TL_AHEAD) : ntj;
#ifdef FIT_STAMPS
                if (lane == 0) {  // before the tasks turn visible: a worker may pick tile 0 at once
                    __hip_atomic_store(&ctl->pub[c], __builtin_amdgcn_s_memrealtime(),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                }
#endif
                if (P.k0 & 2) {
                    engine_publish(ctl, comp_ring(ring, c, ncomp), 0u, 1u, 2u * (unsigned)S.nslice, rnd, (unsigned)c);
                    if (npub > 1u) engine_publish(ctl, comp_ring(ring, c, ncomp), 1u, npub, (unsigned)S.nslice, rnd, (unsigned)c);
                } else {
                    engine_publish(ctl, comp_ring(ring, c, ncomp), 0u, npub, (unsigned)S.nslice, rnd, (unsigned)c);
                }
                if (lane == 0) reinterpret_cast<TmShared*>(smem)->pubt = npub;
                acquire_agent();  // run lists written back by this block: CU-wide fresh view
                if (lane == 0) s_fail = f;
                fail = f;
            }
            __syncthreads();
            if (s_fail) break;  // block-uniform
            const int64_t t1 = (int64_t)__builtin_amdgcn_s_memrealtime();
            // committed while its tiles are scanned: per-tile readiness inside
            const unsigned ntj = (unsigned)((w + SCAN_JOBS - 1) / SCAN_JOBS);
            const CommitResult r =
                commit_tl_window_mw(P, smem, slab, hdr, cand, bnd, wjob, out, outs, H, R,
                                    MwTiles{&ctl->tdone[par][c][0], (unsigned)S.nslice,
                                            TL_AHEAD > 0 ? comp_ring(ring, c, ncomp) : nullptr, ctl, rnd, (unsigned)c, ntj,
                                            nullptr},
                                    glob);
            // every tile published this round (the committer's and the helpers') must be complete
            // before the next round reuses the buffers: count them (pubt is stable after the
            // commit's closing barrier)
            if (wave == 0) {
                target[par] += (reinterpret_cast<TmShared*>(smem)->pubt + ((P.k0 & 2) ? 1u : 0u)) * (unsigned)S.nslice;
                used[par] = reinterpret_cast<TmShared*>(smem)->pubt;
            }
            if (threadIdx.x == 0) engine_round_finished(ctl, c, rnd);
            if (r.stop == 3) {  // a commit wait gave up: TmShared::fail names it (TRIP_PEER: drained)
                if (threadIdx.x == 0) {
                    const TmShared* M = reinterpret_cast<const TmShared*>(smem);
                    const unsigned site = M->fail ? M->fail : (unsigned)TRIP_HELPER_TILE;
                    const unsigned tl = site == TRIP_HELPER_TILE ? M->trip_arg : 0u;
                    trip_record(ctl, site == TRIP_PEER ? 0u : 2u, site, (unsigned)c, rnd, M->trip_arg,
                                M->pubt, ld_agent(&ctl->tdone[par][c][tl & (ENGINE_TILES - 1)]),
                                (unsigned)S.nslice, (unsigned long long)t1);
                }
                break;
            }
            if (r.done == 0) {  // the next round would rescan the same state: never progresses
                if (threadIdx.x == 0)
                    trip_record(ctl, 4u, TRIP_NO_PROGRESS, (unsigned)c, rnd, (unsigned)cursor,
                                reinterpret_cast<const TmShared*>(smem)->pubt, 0u, 0u,
                                (unsigned long long)t1);
                break;
            }
            const int64_t t2 = (int64_t)__builtin_amdgcn_s_memrealtime();
            tw += t1 - t0;
            tc += t2 - t1;
            evals += (int64_t)w * (S.se - S.sb);
            placed += r.placed;
            ++rounds;
            sr += r.stop == 1;
            sd += r.stop == 2;
            cursor += r.done;
            const int nw = r.stop ? 2 * r.done : 2 * w;
            win = max(S.wmin, min(S.wmax, nw));
        }
        if (wave != 0) return;
        (void)fail;  // every failure above recorded its own trip (or drained after another's)
        release_agent();  // last window's run lists / placements (kernel end also flushes)
        if (lane == 0) {
            co[c] = CompOut{evals, placed, cursor - S.jstart, rounds, sr, sd, tc, tw};
            __hip_atomic_fetch_add(&ctl->finished, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }

    // ======================================================================== scan worker
    const unsigned wgrp = worker_group(ncomp);  // this XCD's ring group (fit_engine_ctl.h)
    TaskClaim claim;
    uint64_t(*xk)[TL_KS][64] = reinterpret_cast<uint64_t(*)[TL_KS][64]>(smem);
    unsigned long long* task_slot =
        reinterpret_cast<unsigned long long*>(smem + sizeof(uint64_t) * (SCAN_WAVES / 2) * TL_KS * 64);
    int64_t busy = 0;     // realtime ticks (100 MHz) spent scanning
    int64_t scanned = 0;  // (job, node) evaluations of the tiles scanned (dropped ones excluded)
    for (;;) {
        if (threadIdx.x == 0) {
            unsigned long long task = next_task(ctl, ring, ncomp, wgrp, claim, wd);
            if (task != TASK_EXIT && task_dropped(ctl, task)) task |= TASK_SKIP;
            *task_slot = task;
        }
        __syncthreads();
        const unsigned long long task = *task_slot;
        if (task == TASK_EXIT) {  // block-uniform
            if (threadIdx.x == 0) {
                const int wi = MODE == 2 ? (int)blockIdx.x : (int)blockIdx.x - ncomp;
                wbusy[2 * wi] = busy;
                wbusy[2 * wi + 1] = scanned;
            }
            return;
        }
        const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
        const bool skip = (task & TASK_SKIP) != 0ull;  // block-uniform
        const int c = (int)(task & 63u);
        const int s = (int)task_slice(task);
        const int tile = (int)task_tile(task);
        const int par = (int)(task_round(task) & 1u);  // the round's buffer set
        bool counts = true;  // (thread 0) the task completes its tile's block-slice (TL_T0PAIR)
        if (!skip) {
            if (threadIdx.x == 0) acquire_agent();
            else __builtin_amdgcn_s_dcache_inv();
            __syncthreads();
            CompPlan P = plans[2 * c + par];
            if (tile == 0 && (P.k0 & 2)) {  // the paired first tile: half-size block-slices (TL_T0PAIR)
                P.sub = (P.sub + 1) / 2;
                P.nslice *= 2;
                unsigned* const pr = &ctl->tpair[par][c][0];
                if (SCAN_WAVES * P.sub <= TL_STAGE_NODES)  // block-uniform
                    counts = scan_tile_tl<true, TL_KS, true>(P, tile, s, slab, hdr, jl, jcpu, jmem, jgpu,
                                                             jwall, jpart, cand, bnd, wjob, H, slot_min,
                                                             xk, smem + TL_STAGE_OFF, pr);
                else
                    counts = scan_tile_tl<false, TL_KS, true>(P, tile, s, slab, hdr, jl, jcpu, jmem, jgpu,
                                                              jwall, jpart, cand, bnd, wjob, H, slot_min,
                                                              xk, nullptr, pr);
            } else if (tile == 0 && SCAN_WAVES * P.sub <= TL_STAGE_NODES)  // block-uniform
                scan_tile_tl<true>(P, tile, s, slab, hdr, jl, jcpu, jmem, jgpu, jwall, jpart, cand, bnd,
                                   wjob, H, slot_min, xk, smem + TL_STAGE_OFF);
            else
                scan_tile_tl(P, tile, s, slab, hdr, jl, jcpu, jmem, jgpu, jwall, jpart, cand, bnd, wjob,
                             H, slot_min, xk);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
#ifdef FIT_STAMPS
            if (threadIdx.x == 0 && tile == 0) {  // a round's first tile: pickup delay, scan time
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                atomicAdd(&g_tlsc[5], (unsigned long long)t0 - ctl->pub[c]);
                atomicAdd(&g_tlsc[6], now - (unsigned long long)t0);
                atomicAdd(&g_tlsc[7], 1ull);
            }
#endif
            const int a = P.sb + s * SCAN_WAVES * P.sub, b = min(P.se, a + SCAN_WAVES * P.sub);
            scanned += (int64_t)max(min(SCAN_JOBS, P.w - tile * SCAN_JOBS), 0) * max(b - a, 0);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            // the tile's outputs were written through and every storing wave waited for them
            // (vmcnt(0) above, then the barrier): the counts need no release fence (R1)
            if (counts)
                __hip_atomic_fetch_add(&ctl->tdone[par][c][tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the tile count must land before the done count: once a committer sees `done` reach
            // its target it resets the tile counters for the next round, and a late increment
            // would then mark a tile of that round complete before it was scanned
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&ctl->done[c][2 + par], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            busy += (int64_t)__builtin_amdgcn_s_memrealtime() - t0;
        }
        __syncthreads();  // task_slot is rewritten by thread 0 next iteration
    }
}

// Dense read-back (tests, fit_read_timeline): one block per node position, threads over slots.
__global__ void k_expand_tl(const int32_t* __restrict__ perm, const Seg* __restrict__ slab,
                            const TlHdr* __restrict__ hdr, int32_t H, int32_t* __restrict__ oc,
                            int32_t* __restrict__ om, int32_t* __restrict__ og) {
    const int i = blockIdx.x;
    const Seg* sg = slab + (int64_t)i * TL_MAX_SLOTS;
    const int n = hdr[i].cnt;
    const int64_t base = (int64_t)perm[i] * H;
    for (int t = threadIdx.x; t < H; t += blockDim.x) {
        int lo = 0, hi = n - 1;  // first run with end > t
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sg[mid].end > t) hi = mid;
            else lo = mid + 1;
        }
        const Seg g = sg[lo];
        oc[base + t] = g.cpu;
        om[base + t] = g.mem;
        og[base + t] = g.gpu;
    }
}

#ifdef FIT_STAMPS
extern "C" int fit_debug_tl_stamps(unsigned long long* out /* 64 x 12 + 8 */, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tlst), sizeof(g_tlst)) != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out + 64 * 12, HIP_SYMBOL(g_tlsc), sizeof(g_tlsc)) != hipSuccess) return -2;
    if (reset) {
        static unsigned long long zero[64][12];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tlst), zero, sizeof(zero)) != hipSuccess) return -2;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tlsc), zero, sizeof(g_tlsc)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

// ------------------------------------------------------------------ host launch wrappers
hipError_t launch_build_tl(hipStream_t st, const int32_t* cpu, const int32_t* mem,
                           const int32_t* gpu, const int32_t* av, const uint32_t* mask,
                           const int32_t* perm, int32_t nn, int32_t H, int32_t slot_min,
                           const int32_t* off, const int32_t* rs, const int32_t* rc,
                           const int32_t* rm, const int32_t* rg, Seg* slab, TlHdr* hdr,
                           uint32_t* err) {
    if (nn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_build_tl, dim3((nn + 255) / 256), dim3(256), 0, st, cpu, mem, gpu, av,
                       mask, perm, nn, H, slot_min, off, rs, rc, rm, rg, slab, hdr, err);
    return hipGetLastError();
}

hipError_t launch_scan_tl(int blocks, hipStream_t st, const Seg* slab, const TlHdr* hdr,
                          const int32_t* jl, const int32_t* jcpu, const int32_t* jmem,
                          const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart,
                          const CompPlan* plan, int ncomp, uint64_t* cand, uint64_t* bnd,
                          JobRec* wjob, int32_t H, int32_t slot_min) {
    hipLaunchKernelGGL(k_scan_tl, dim3(blocks), dim3(SCAN_WAVES * 64), 0, st, slab, hdr, jl, jcpu,
                       jmem, jgpu, jwall, jpart, plan, ncomp, cand, bnd, wjob, H, slot_min);
    return hipGetLastError();
}

// LDS of k_commit_tl: general-path scratch + TL_UCAP dirty-list regions of R runs with their
// prefix minima + the dirty bitmap.  R is as large as 160 KiB allows, at most 64 runs.
constexpr size_t TL_LDS_LIMIT = 160 * 1024;
int commit_tl_runs(int32_t max_component_nodes) {
    const size_t fixed = sizeof(Seg) * TL_MAX_SLOTS + (size_t)((max_component_nodes + 31) / 32) * 4;
    if (fixed >= TL_LDS_LIMIT) return 0;
    const size_t fit = (TL_LDS_LIMIT - fixed) / ((sizeof(Seg) + sizeof(int4)) * TL_UCAP);
    if (fit <= (size_t)TL_PAD) return 0;
    return (int)std::min<size_t>(2 * TL_PM_STEPS, fit - TL_PAD);
}

size_t commit_tl_lds_bytes(int32_t max_component_nodes) {
    const int runs = commit_tl_runs(max_component_nodes);
    return sizeof(Seg) * TL_MAX_SLOTS +
           (sizeof(Seg) + sizeof(int4)) * (size_t)TL_UCAP * (runs > 0 ? runs + TL_PAD : 0) +
           (size_t)((max_component_nodes + 31) / 32) * 4;
}

hipError_t launch_commit_tl(int ncomp, int epl, size_t lds, hipStream_t st, Seg* slab,
                            TlHdr* hdr, const CompPlan* plan, const uint64_t* cand,
                            int64_t rank_stride, int nranks, const uint64_t* bnd,
                            const JobRec* wjob, const int32_t* perm, int32_t* out, int32_t* outs,
                            CommitResult* res, int32_t H, int32_t R) {
#define FIT_COMMIT_TL(EPL)                                                                    \
    hipLaunchKernelGGL(k_commit_tl<EPL>, dim3(ncomp), dim3(64), lds, st, slab, hdr, plan,     \
                       cand, rank_stride, nranks, bnd, wjob, perm, out, outs, res, H, R)
    if (epl <= 1) FIT_COMMIT_TL(1);
    else if (epl <= 2) FIT_COMMIT_TL(2);
    else if (epl <= 4) FIT_COMMIT_TL(4);
    else if (epl <= 8) FIT_COMMIT_TL(8);
    else return hipErrorInvalidValue;
#undef FIT_COMMIT_TL
    return hipGetLastError();
}

// k_engine_tl: the committer takes a whole CU's LDS (run lists of up to 64 runs stay in LDS; the
// scan workers are mostly idle at one block per CU: DESIGN.md §3.8).  Regions are R + TL_PAD runs
// apart with R + TL_PAD odd (an even multiple of 16 B puts the lanes' own-list reads on one bank).
constexpr size_t TL_ENGINE_LDS = 160 * 1024;
static size_t engine_tl_fixed(int32_t max_component_nodes) {
    const size_t head = tm_fixed_bytes();
    return head + (size_t)((max_component_nodes + 31) / 32) * 4;
}
int engine_tl_runs(int32_t max_component_nodes) {
    const size_t fixed = engine_tl_fixed(max_component_nodes);
    if (fixed >= TL_ENGINE_LDS) return 0;
    const size_t fit = (TL_ENGINE_LDS - fixed) / ((sizeof(Seg) + sizeof(int4)) * TL_UCAP);
    if (fit <= (size_t)TL_PAD) return 0;
    int r = (int)std::min<size_t>(2 * TL_PM_STEPS, fit - TL_PAD);
    if (((r + TL_PAD) & 1) == 0) --r;
    return r;
}

size_t engine_tl_scan_lds_bytes() { return TL_STAGE_OFF + TL_STAGE_BYTES; }

size_t engine_tl_lds_bytes(int32_t max_component_nodes) {
    const int runs = engine_tl_runs(max_component_nodes);
    const size_t commit = engine_tl_fixed(max_component_nodes) +
                          (sizeof(Seg) + sizeof(int4)) * (size_t)TL_UCAP * (runs > 0 ? runs + TL_PAD : 0);
    return std::max(commit, engine_tl_scan_lds_bytes());
}

int engine_tl_blocks_per_cu(size_t lds, int mode) {
    int n = 0;
    const hipError_t e =
        mode == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_engine_tl<2>, SCAN_WAVES * 64, lds)
        : mode == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_engine_tl<1>, SCAN_WAVES * 64, lds)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_engine_tl<0>, SCAN_WAVES * 64, lds);
    return e == hipSuccess ? n : 0;
}

hipError_t launch_engine_tl(int blocks, size_t lds, hipStream_t st, void* ctl, void* ring,
                            const void* cs, void* co, CompPlan* plans, int ncomp, Seg* slab,
                            TlHdr* hdr, const int32_t* jl, const int32_t* jcpu,
                            const int32_t* jmem, const int32_t* jgpu, const int32_t* jwall,
                            const uint16_t* jpart, uint64_t* cand, uint64_t* bnd, JobRec* wjob,
                            const int32_t* perm, int32_t* out, int32_t* outs, int32_t H,
                            int32_t slot_min, int32_t R, int64_t* wbusy, int mode,
                            unsigned* resident, unsigned wd) {
#define FIT_ENGINE_TL(M_)                                                                         \
    hipLaunchKernelGGL(k_engine_tl<M_>, dim3(blocks), dim3(SCAN_WAVES * 64), lds, st,          \
                       static_cast<EngineCtl*>(ctl), static_cast<unsigned long long*>(ring),     \
                       static_cast<const CompState*>(cs), static_cast<CompOut*>(co), plans, ncomp,\
                       slab, hdr, jl, jcpu, jmem, jgpu, jwall, jpart, cand, bnd, wjob, perm, out,  \
                       outs, H, slot_min, R, wbusy, resident, wd)
    if (mode == 1) FIT_ENGINE_TL(1);
    else if (mode == 2) FIT_ENGINE_TL(2);
    else FIT_ENGINE_TL(0);
#undef FIT_ENGINE_TL
    return hipGetLastError();
}

hipError_t launch_expand_tl(hipStream_t st, const int32_t* perm, const Seg* slab,
                            const TlHdr* hdr, int32_t nn, int32_t H, int32_t* oc, int32_t* om,
                            int32_t* og) {
    if (nn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_expand_tl, dim3(nn), dim3(256), 0, st, perm, slab, hdr, H, oc, om, og);
    return hipGetLastError();
}

}  // namespace fitgpu
