// fit_commit_tl_mw.h — the backfill commit (SPEC §2b, config C5) of one component's window by a
// whole 8-wave workgroup, on the decider / helper split of fit_commit_mw.h.
// Included by fit_timeline.hip after the run-list primitives it uses (tl_key, tl_eval4,
// tl_walk_wave, tl_reserve_lds, tl_reserve_any, wave_scan_min).
//
// Wave 0 is the DECIDER, waves 1..7 are HELPERS.  Helper h pre-resolves jobs t = h-1 (mod 7)
// against a snapshot of the dirty state taken once the decider has resolved v >= t - 7 jobs: it
// writes into record t & 7 the t - v + 1 (<= 8) smallest keys <= B among
//   (clean candidates of t)  ∪  (t's earliest-start keys on the dirty run lists held in LDS),
// each tagged with its dirty slot or as clean (with the node's header fields), and stages the run
// list of its first clean item in LDS.  The decider, at job t, drops every item whose node was
// written by one of its last <= 7 decisions (the "written ring", lanes 0..7: slot, position, run
// count, job), evaluates those ring nodes on their CURRENT LDS lists (prefix-minimum search for a
// start at slot 0, wave-wide walks only when a later start could still win), and takes
//     best = min(surviving items, live ring keys, keys of the global-slab dirty lists).
// Exact for the reason given in fit_commit_mw.h: if the record held t - v + 1 items at least one
// survives and bounds every unlisted node; if fewer, it held every candidate <= B.  Dirty lists
// that outgrew their LDS region (global slab, `gm` bit per slot) are never read by helpers (the
// decider writes them through memory the helpers would need an acquire to see); the decider
// evaluates them itself, every job — they are rare (C5: at most 57 runs per node, R = 63).
//
// The decider's job is then: ring search + item merge, one reservation on an LDS run list with its
// prefix-minimum rebuild, and for a clean winner one LDS copy of its staged runs — where the
// single-wave commit (commit_tl_window) also evaluated every dirty list (64 lanes of 4-ary
// searches and walks), the clean candidates and the winner's header / run loads per job.
//
// LDS protocol: fit_commit_mw.h's (workgroup release / acquire on LDS).
#pragma once
#include "fit_commit_mw.h"

namespace fitgpu {

constexpr int TM_M = 8;   // items per record (> snapshot lag)
constexpr int TM_R = 8;   // record ring
constexpr int TM_H = SCAN_WAVES - 1;  // helpers: waves 1..7
static_assert(TM_H >= 1 && TM_H <= SCAN_WAVES - 1, "helpers are waves 1..7");
static_assert(TL_UCAP == 64, "one dirty slot per lane: ring / slot bit masks are 64 wide");
constexpr int TM_CPL = TL_KS * TL_SLICES / 64;  // clean candidates per helper lane
static_assert(TM_CPL * 64 == TL_KS * TL_SLICES && TM_CPL >= 1 && TM_CPL <= 2,
              "64 or 128 candidates per job (one or two per helper lane)");

struct alignas(16) TmItem {  // 48 B
    uint32_t klo, khi;       // key = start << 54 | score << 22 | position
    int32_t tag, orig;       // dirty slot (>= 0) or -1 (clean); node id
    uint32_t mask;
    int32_t cnt, cc, cm;     // run count, column ceilings (clean items: from the node header)
    int32_t cg, pad0, pad1, pad2;
};

struct alignas(16) TmHdr {  // 64 B
    uint32_t ready;          // t + 1 once record t is complete (release store, last)
    int32_t v, n, q;         // snapshot, items, job index in the caller's order
    int32_t jc, jm, jg, jd;  // demand, slots occupied
    uint32_t pbit, spos;     // partition bit; position of the staged run list (~0: none)
    int32_t scnt, pad;       // its run count
    uint32_t blo, bhi, pad2, pad3;  // bound B
};

struct alignas(16) TmRec {
    TmHdr h;
    TmItem it[TM_M];
};

struct alignas(16) TmSlot {  // one dirty slot, current (written by the decider)
    uint32_t pos, mask;
    int32_t orig, cnt;
    int32_t cc, cm, cg, glob;
};

struct alignas(16) TmShared {
    uint64_t dn;       // {decided (low 32), nu (high 32)}: the helpers' snapshot, release-stored
    uint32_t halt;     // decider stopped
    uint32_t fail;     // helper / decider watchdog: the TripSite of the first wait that gave up
    int32_t res[4];    // CommitResult of the window
    uint32_t pubt;     // job tiles of the window published to the task ring (just in time)
    uint32_t wd;       // watchdog: realtime ticks a wait may last (set by the committer)
    uint32_t trip_arg; // the failed wait's tile / record
    uint32_t pad[1];
    uint32_t wclk[8];  // per wave: its long wait's start (wait_clock_over)
    TmRec rec[TM_R];
    Seg stage[TM_R][64];     // the run list of each record's first clean item
    TmSlot slot[TL_UCAP];
    Seg scr[TL_MAX_SLOTS];   // general-path scratch (tl_reserve_any)
    // followed by: run-list regions (TL_UCAP x RS Seg), their prefix minima (TL_UCAP x RS int4),
    // the dirty bitmap ((ne - nb + 31) / 32 words)
};

__host__ __device__ constexpr size_t tm_fixed_bytes() { return sizeof(TmShared); }

// The clock of a wave's long wait (the TL helpers' tile waits), kept in LDS so that the spin loop
// holds no register for it: the loop calls this every 1024 spins (an SMEM round trip for the
// realtime counter); the first call starts the clock.  Low 32 bits of the 100 MHz counter: waits up
// to 42.9 s (the deadline's range).  The loop clears its slot when it ends after a check.  (k_engine's
// helpers keep a spin bound instead: fit_commit_mw.h MW_SPIN_LIMIT; here the check measured no cost,
// C5 117.5 vs 117.3 ms.)
__device__ __forceinline__ bool wait_clock_over(uint32_t* wclk, const uint32_t* wd) {
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) & 7;
    const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime() | 1u;
    const uint32_t t0 = __hip_atomic_load(&wclk[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (t0 == 0u) {
        __hip_atomic_store(&wclk[w], now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return false;
    }
    return now - t0 > __hip_atomic_load(wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wait_clock_end(uint32_t* wclk, unsigned spins) {
    if (spins >= 1023u)
        __hip_atomic_store(&wclk[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) & 7], 0u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// lds_opaque for an LDS address that depends on runtime values (region / prefix-minimum bases
// follow R): made uniform first, so it can live in an SGPR
template <class T>
__device__ __forceinline__ T* tm_lds(T* p) {
    uint32_t a = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p);
    asm volatile("" : "+s"(a));
    return (T*)(__attribute__((address_space(3))) T*)(uintptr_t)a;
}

#ifndef TL_AHEAD
#define TL_AHEAD 2  // job tiles published ahead of the helper that needs them (0: all up front).
                    // C5 k_engine_tl: 1 / 2 / 4 / 8 -> 174.7 / 129.9 / 133.8 / 140.5 ms (r03d/e):
                    // tiles past a round's stop are scanned for nothing, too few starve the helpers
#endif

// Publish the window's job tiles [pubt, upto) (uniform; lane 0 claims the range by an LDS CAS) —
// fit_commit_mw.h mw_publish for this layout.
__device__ __noinline__ void tm_publish(const MwTiles& T, TmShared* S, unsigned upto) {
    const int lane = threadIdx.x & 63;
    unsigned from = upto;
    if (lane == 0) {
        unsigned cur = lds_ld(&S->pubt);
        while (cur < upto) {
            if (__hip_atomic_compare_exchange_strong(&S->pubt, &cur, upto, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                from = cur;
                break;
            }
        }
    }
    from = (unsigned)__builtin_amdgcn_readlane((int)from, 0);
    if (from >= upto) return;
    // what the tasks' scans read was stored through or released by the committer wave before the
    // block barrier this wave has passed: no fence here (fit_commit_mw.h mw_publish)
    engine_publish(T.ctl, T.ring, from, upto, T.need, T.round, T.comp);
}

// The tile-readiness wait of fit_commit_mw.h for this shared layout: tiles are published just in
// time (a helper that moves on to tile k publishes up to k + TL_AHEAD - 1 first), so a round that
// stops early leaves at most TL_AHEAD tiles scanned for nothing, and the next round's first tile
// is not queued behind a whole window.
__device__ __forceinline__ bool tm_tile_ready(const MwTiles& T, int tt, int& ready, TmShared* S) {
    if (!T.tdone) return true;
    const int tile = __builtin_amdgcn_readfirstlane(tt) / SCAN_JOBS;
    if (tile < ready) return true;
    if (T.ring && (unsigned)tile + TL_AHEAD > lds_ld(&S->pubt))
        tm_publish(T, S, min((unsigned)tile + TL_AHEAD, T.ntj));
    const unsigned* tdone = T.tdone;
    const unsigned need = T.need;
    for (unsigned sp = 0;; ++sp) {
        if (__hip_atomic_load(gview(tdone) + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) {
            wait_clock_end(S->wclk, sp);
            break;
        }
        if (lds_ld(&S->halt) | lds_ld(&S->fail)) return false;
        if ((sp & 1023u) == 1023u) {
            // (no check of other blocks' trips here: the load of ctl->error made the helper spill,
            // C3 +2 ms; after a trip elsewhere this wait ends at its own deadline)
            if (wait_clock_over(S->wclk, &S->wd)) {
                commit_fail(&S->fail, &S->trip_arg, TRIP_HELPER_TILE, (uint32_t)tile);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
    // sc1 loads of the tile's outputs, no acquire fence (fit_commit_mw.h ld_through)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ready = tile + 1;
    return true;
}

// Prefix-minimum search for a start at slot 0 on an LDS run list (per lane; a lane's own list):
// the first run ending at or after d (4-ary search, three rounds of three independent reads),
// then that window's minima.  Key or KEY_INF.
__device__ __forceinline__ uint64_t tm_fit0(const Seg* L, const int4* PM, int cnt, int R, bool ok,
                                            int32_t jc, int32_t jm, int32_t jg, int32_t jd,
                                            uint32_t pos, bool& fit0) {
    int k = 0;
#pragma unroll
    for (int q = 16; q >= 1; q >>= 2) {
        const int i1 = k + q - 1, i2 = k + 2 * q - 1, i3 = k + 3 * q - 1;
        const int32_t y1 = L[min(i1, R - 1)].end, y2 = L[min(i2, R - 1)].end, y3 = L[min(i3, R - 1)].end;
        const int32_t x1 = i1 < cnt ? y1 : TL_BIG;
        const int32_t x2 = i2 < cnt ? y2 : TL_BIG;
        const int32_t x3 = i3 < cnt ? y3 : TL_BIG;
        k += q * ((x1 < jd) + (x2 < jd) + (x3 < jd));
    }
    const int4 pk = PM[min(k, R - 1)];
    fit0 = ok && pk.x >= jc && pk.y >= jm && pk.z >= jg;
    return fit0 ? tl_key(0, pk.x, pk.y, pk.z, jc, jm, jg, pos) : KEY_INF;
}


typedef __attribute__((address_space(3))) v4i32 lds_v4i32;
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ void lds_st4(uint32_t a, v4i32 v) { *(lds_v4i32*)(uintptr_t)a = v; }
__device__ __forceinline__ int32_t lds_ld1(uint32_t a) {
    return *(const __attribute__((address_space(3))) int32_t*)(uintptr_t)a;
}
// the previous lane's value (lane 0: `first`) / the next lane's (lane 63: `last`): DPP wave shifts
__device__ __forceinline__ int32_t wave_shr1(int32_t v, int32_t first) {
    return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int32_t wave_shl1(int32_t v, int32_t last) {
    return __builtin_amdgcn_update_dpp(last, v, 0x130, 0xf, 0xf, false);
}

// Reserve (jc, jm, jg) on slots [s, e) of a run list of n <= 64 runs held in registers (run
// `lane` in g) and write the new list and its prefix minima to the LDS region L / PM — every run
// at its new index, so a list entering the region (a new dirty node) needs no copy first, and the
// prefix minima come from the registers (no read-back).  Same edge rules as tl_reserve_lds: the
// runs overlapping [s, e) lose the demand, the run holding s (e) splits, the first (last) reduced
// run merges into an equal left (right) neighbour.  The prefix minimum of a run at its new index
// is the inclusive scan over the reduced values (a split-off piece keeps the unreduced values,
// never below the reduced ones, so it changes no prefix after it; the head piece's own is the
// scan before it with its values).  Lanes without a write store to `trash` (no exec branches).
// Returns the new count, or -1 (nothing written) if it would exceed `cap`.
__device__ __forceinline__ int tm_reserve(uint32_t L, uint32_t PM, uint32_t trash, const Seg& g, int n,
                                          int cap, int32_t s, int32_t e, int32_t jc, int32_t jm,
                                          int32_t jg) {
    const int lane = threadIdx.x & 63;
    // every cross-lane value first (DPP reads with the full wave active), then only selects
    const int32_t a = wave_shr1(g.end, 0);  // the run's start
    const int32_t lc = wave_shr1(g.cpu, 0), lm = wave_shr1(g.mem, 0), lg = wave_shr1(g.gpu, 0);
    const int32_t nc = wave_shl1(g.cpu, 0), nm = wave_shl1(g.mem, 0), ng = wave_shl1(g.gpu, 0);
    const bool v = lane < n;
    const int32_t rc = g.cpu - jc, rm = g.mem - jm, rg = g.gpu - jg;
    const uint64_t mov = __ballot(v & (a < e) & (g.end > s));
    const uint64_t mh = __ballot(v & (a < s)), mt = __ballot(v & (g.end > e));
    const uint64_t meqL = __ballot((lc == rc) & (lm == rm) & (lg == rg));
    const uint64_t meqR = __ballot((nc == rc) & (nm == rm) & (ng == rg));
    const int i0 = __builtin_ctzll(mov), i1 = 63 - __builtin_clzll(mov);
    const int head = (int)((mh >> i0) & 1ull), tail = (int)((mt >> i1) & 1ull);
    const int mergeL = (int)((meqL >> i0) & 1ull) & (head ^ 1) & (int)(i0 > 0);
    const int mergeR = (int)((meqR >> i1) & 1ull) & (tail ^ 1) & (int)(i1 < n - 1);
    const int nn = n + head + tail - mergeL - mergeR;
    if (nn > cap) return -1;
    const int sh = head - mergeL;                  // index shift of the reduced runs
    const int st = head + tail - mergeL - mergeR;  // index shift of the runs after them
    const bool inr = (lane >= i0) & (lane <= i1);
    const Seg u{inr ? min(g.end, e) : g.end, inr ? rc : g.cpu, inr ? rm : g.mem, inr ? rg : g.gpu};
    int32_t pc = v ? u.cpu : TL_BIG, pm = v ? u.mem : TL_BIG, pg = v ? u.gpu : TL_BIG;
    wave_scan_min3(pc, pm, pg);
    const int32_t xc = wave_shr1(pc, TL_BIG), xm = wave_shr1(pm, TL_BIG), xg = wave_shr1(pg, TL_BIG);
    // every run at its new index (the two a merge drops excluded)
    const int dest = lane + (lane < i0 ? 0 : (lane > i1 ? st : sh));
    const bool wp = v & !((mergeL != 0) & (lane == i0 - 1)) & !((mergeR != 0) & (lane == i1));
    const uint32_t od = 16u * (uint32_t)dest;
    lds_st4(wp ? L + od : trash, v4i32{u.end, u.cpu, u.mem, u.gpu});
    lds_st4(wp ? PM + od : trash, v4i32{pc, pm, pg, 0});
    // the head piece (lane i0): [a, s) unreduced at i0, its prefix minima the scan before it
    const bool wh = (head != 0) & (lane == i0);
    const uint32_t oh = 16u * (uint32_t)i0;
    lds_st4(wh ? L + oh : trash, v4i32{s, g.cpu, g.mem, g.gpu});
    lds_st4(wh ? PM + oh : trash, v4i32{min(xc, g.cpu), min(xm, g.mem), min(xg, g.gpu), 0});
    // the tail piece (lane i1): [e, end) unreduced after the reduced runs
    const bool wt = (tail != 0) & (lane == i1);
    const uint32_t ot = 16u * (uint32_t)(i1 + sh + 1);
    lds_st4(wt ? L + ot : trash, v4i32{g.end, g.cpu, g.mem, g.gpu});
    lds_st4(wt ? PM + ot : trash, v4i32{pc, pm, pg, 0});
    return nn;
}

#ifdef FIT_STAMPS
// diagnostic build: g_tlst[comp][i] (fit_timeline.hip).  Coarse (FIT_STAMPS): [0] decider waits
// for each round's first record, [1] decider loop cycles, [5] jobs, [6] new dirty nodes, [7]
// round-end write-back, [8] rounds, [9] jobs that walked, [10] helper snapshot -> record cycles,
// [11] helper records.  Fine (FIT_STAMPS_FINE, every s_memtime drains the LDS queue, so the
// phases are inflated): [0] record waits, [1] decision (ring search + item merge), [2] exception
// path (walks, global lists), [3] new dirty copy, [4] reservation + prefix minima, [8] whole
// apply phase.
#define TM_CNT(i, x) D.acc[i] += (x)
#ifdef FIT_STAMPS_FINE
#define TM_CLK(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define TM_ADD(i, x) D.acc[i] += (x)
#else
#define TM_CLK(v)
#define TM_ADD(i, x)
#endif
#else
#define TM_CNT(i, x)
#define TM_CLK(v)
#define TM_ADD(i, x)
#endif

// ------------------------------------------------------------------------------- helper
struct TmJob {
    uint64_t kk[TM_CPL], B;
    JobRec J;
};

__device__ __noinline__ void tm_helper(const CompPlan& Pref, TmShared* Sin, Seg* lr_, int4* pmr_,
                                       uint32_t* bitmap_, int32_t RS, int32_t R,
                                       const Seg* __restrict__ slab_, const TlHdr* __restrict__ hdr_,
                                       const uint64_t* __restrict__ cand_,
                                       const uint64_t* __restrict__ bnd_,
                                       const JobRec* __restrict__ wjob_, int h, int32_t H,
                                       MwTiles Tin) {
    const MwTiles T = tiles_sgpr(Tin);  // no scratch loads in the loop (fit_commit_mw.h)
    const GAS Seg* const slab = gview(slab_);
    const GAS TlHdr* const hdr = gview(hdr_);
    const GAS uint64_t* const cand = gview(cand_);
    const GAS uint64_t* const bnd = gview(bnd_);
    const GAS JobRec* const wjob = gview(wjob_);
    const CompPlan P = plan_sgpr(Pref);
    TmShared* const S = tm_lds(Sin);
    Seg* const lr = tm_lds(lr_);
    int4* const pmr = tm_lds(pmr_);
    uint32_t* const bitmap = tm_lds(bitmap_);
    const int lane = threadIdx.x & 63;
    const int E = P.nslice * TL_KS;  // candidates per job (lane + 64 c, c < TM_CPL)
    const int wlast = P.w - 1;
    const int z = opaque_zero();
    const uint32_t nb = (uint32_t)P.nb;
    int t = rfl(h - 1);
    int ready = 0;
    auto load = [&](int tt, TmJob& o) -> bool {
        tt = min(tt, wlast) + z;
        if (!tm_tile_ready(T, tt, ready, S)) return false;
#pragma unroll
        for (int c = 0; c < TM_CPL; ++c)
            o.kk[c] = lane + 64 * c < E ? ld_through(cand + P.cand_off + (int64_t)tt * E + lane + 64 * c) : KEY_INF;
        o.J = ld_job_through(wjob + P.slot0 + tt);
        o.B = ld_through(bnd + P.slot0 + tt);
        return true;
    };
    TmJob cur, nxt;
#ifdef FIT_STAMPS
    unsigned long long hs_acc = 0, hs_n = 0;
    struct Flush {
        unsigned long long &a, &n;
        __device__ ~Flush() {
            if ((threadIdx.x & 63) == 0) {
                atomicAdd(&g_tlst[blockIdx.x & 63][10], a);
                atomicAdd(&g_tlst[blockIdx.x & 63][11], n);
            }
        }
    } flush{hs_acc, hs_n};
#endif
    if (!load(t, cur)) return;
    for (;;) {
        if (t >= P.w) break;
        if (!load(t + TM_H, nxt)) break;  // the next job's stream, in flight during this one
        // snapshot: the decider has resolved at least t - (TM_M - 1) jobs (so it has read record
        // slot t & 7's previous job)
        uint64_t dn;
        for (unsigned sp = 0;; ++sp) {
            dn = __hip_atomic_load(&S->dn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int lag = t - (TM_M - 1) - rfl((int32_t)(uint32_t)dn);
            if (lag <= 0) break;
            if ((sp & 7u) == 7u && (lds_ld(&S->halt) | lds_ld(&S->fail))) return;
            if (sp > MW_SPIN_LIMIT) {  // within the block: a spin bound only (fit_commit_mw.h)
                commit_fail(&S->fail, &S->trip_arg, TRIP_HELPER_SNAP, (uint32_t)t);
                return;
            }
            for (int s = min(lag, 8); s > 0; --s) __builtin_amdgcn_s_sleep(2);
        }
        lds_acquire();
#ifdef FIT_STAMPS
        const unsigned long long hs0 = __builtin_amdgcn_s_memtime();
#endif
        const int v = rfl((int32_t)(uint32_t)dn);
        const int nu = rfl((int32_t)(uint32_t)(dn >> 32));
        const JobRec& J = cur.J;
        const uint64_t B = cur.B;
        const int32_t jc = rfl(J.cpu), jm = rfl(J.mem), jg = rfl(J.gpu), jd = rfl(J.wall);
        const uint32_t jp = (uint32_t)rfl((int)J.pbit);
        // clean candidates of this lane
        uint64_t xc[TM_CPL];
#pragma unroll
        for (int c = 0; c < TM_CPL; ++c) {
            const uint64_t k = cur.kk[c];
            const bool ok = k <= B && k != KEY_INF;
            const uint32_t rel = ok ? ((uint32_t)k & TL_POS_MASK) - nb : 0u;
            const bool dirty = (bitmap[rel >> 5] >> (rel & 31)) & 1u;
            xc[c] = ok && !dirty ? k : KEY_INF;
        }
        // dirty slot of this lane (slot = lane < nu), LDS lists only
        const TmSlot si = S->slot[lane < nu ? lane : 0];
        const bool dl = lane < nu && !si.glob && (si.mask & jp) != 0u && jd <= H && jc <= si.cc &&
                        jm <= si.cm && jg <= si.cg;
        bool fit0 = false;
        const Seg* const mine = lr + lane * RS;
        uint64_t xd = tm_fit0(mine, pmr + lane * RS, si.cnt, R, dl, jc, jm, jg, jd, si.pos, fit0);
        // a later start on a list that cannot start at 0: only keys <= B count, so only when B's
        // start is later than 0 (lane-parallel walks over the lists, cut at B)
        const bool walk = dl && !fit0;
        const int32_t limB = B == KEY_INF ? H : (int32_t)(B >> 54);
        if (__ballot(walk) && limB > 0) {
            const uint64_t wk = tl_eval4(mine, si.cnt, R, walk, jc, jm, jg, jd, H, si.pos, B);
            xd = walk ? wk : xd;
        }
        xd = xd <= B ? xd : KEY_INF;
        // extraction: the nmax smallest entries, one wave minimum (two 32-bit passes) each; every
        // entry remembers which item it became (sel: 4 bits per entry; entries 0..TM_CPL-1 clean,
        // TM_CPL dirty), the lane's entries sorted once so each lane offers its smallest
        const int nmax = min(TM_M, t - v + 1);
        constexpr int NE = TM_CPL + 1;
        uint64_t q[NE];
        int o[NE];
#pragma unroll
        for (int c = 0; c < TM_CPL; ++c) {
            q[c] = xc[c];
            o[c] = c;
        }
        q[TM_CPL] = xd;
        o[TM_CPL] = TM_CPL;
        auto cswap = [&](int i, int j) {
            const bool sw = q[j] < q[i];
            const uint64_t qi = q[i], qj = q[j];
            const int oi = o[i], oj = o[j];
            q[i] = sw ? qj : qi;
            q[j] = sw ? qi : qj;
            o[i] = sw ? oj : oi;
            o[j] = sw ? oi : oj;
        };
        if constexpr (NE == 2) {
            cswap(0, 1);
        } else {
            cswap(0, 1);
            cswap(1, 2);
            cswap(0, 1);
        }
        uint32_t sel = 0u;
        int n = 0;
#pragma unroll
        for (int i = 0; i < TM_M; ++i) {
            if (i >= nmax) break;  // uniform: a record needs nmax items at most
            const uint32_t hh = (uint32_t)(q[0] >> 32), ll = (uint32_t)q[0];
            const uint32_t mh = wave_min32_all(hh);
            const uint32_t ml = wave_min32_all(hh == mh ? ll : 0xffffffffu);
            const bool take = i < nmax && (mh & ml) != 0xffffffffu;
            const bool me = take && hh == mh && ll == ml;  // keys of distinct nodes are unique
            n += take ? 1 : 0;
            sel = me ? sel | ((uint32_t)(i + 1) << (4 * o[0])) : sel;
#pragma unroll
            for (int e = 0; e + 1 < NE; ++e) {
                q[e] = me ? q[e + 1] : q[e];
                o[e] = me ? o[e + 1] : o[e];
            }
            q[NE - 1] = me ? KEY_INF : q[NE - 1];
        }
        n = rfl(n);
        // clean items need their node's header fields; the first clean item's run list is staged
        uint32_t ixc[TM_CPL], cpos[TM_CPL];
        uint32_t fmin = 15u;
#pragma unroll
        for (int c = 0; c < TM_CPL; ++c) {
            ixc[c] = (sel >> (4 * c)) & 15u;
            cpos[c] = ixc[c] ? ((uint32_t)xc[c] & TL_POS_MASK) : nb;
            fmin = min(fmin, ixc[c] ? ixc[c] : 15u);
        }
        const uint32_t ix1 = (sel >> (4 * TM_CPL)) & 15u;
        const uint32_t first = wave_min32_all(fmin);
        uint32_t spos = 0xffffffffu;
        int fl = 0, fc = 0;
#pragma unroll
        for (int c = TM_CPL - 1; c >= 0; --c) {
            const uint64_t fm = __ballot(ixc[c] != 0u && ixc[c] == first);
            if (fm) {
                fl = __builtin_ctzll(fm);
                fc = c;
                spos = (uint32_t)readlane((int32_t)cpos[c], fl);
            }
        }
        TlHdr ch[TM_CPL];
#pragma unroll
        for (int c = 0; c < TM_CPL; ++c) {
            const GAS v4i32* hp = (const GAS v4i32*)(hdr + cpos[c]);
            const v4i32 a = hp[0], b = hp[1];
            ch[c].cnt = a.x;
            ch[c].cpu = a.y;
            ch[c].mem = a.z;
            ch[c].gpu = a.w;
            ch[c].mask = (uint32_t)b.x;
            ch[c].orig = b.y;
        }
        const v4i32 sv = *(const GAS v4i32*)(slab + (int64_t)(spos != 0xffffffffu ? spos : nb) * TL_MAX_SLOTS + lane);
        const Seg srun{sv.x, sv.y, sv.z, sv.w};
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next job's prefetch too (older)
        TmRec* const Rr = &S->rec[t & (TM_R - 1)];
#pragma unroll
        for (int c = 0; c < TM_CPL; ++c)
            if (ixc[c])
                Rr->it[ixc[c] - 1u] = TmItem{(uint32_t)xc[c], (uint32_t)(xc[c] >> 32), -1, ch[c].orig,
                                             ch[c].mask, ch[c].cnt, ch[c].cpu, ch[c].mem, ch[c].gpu, 0, 0, 0};
        if (ix1)
            Rr->it[ix1 - 1u] = TmItem{(uint32_t)xd, (uint32_t)(xd >> 32), lane, si.orig, si.mask, si.cnt,
                                      si.cc, si.cm, si.cg, 0, 0, 0};
        int32_t scnt = 0;
        if (spos != 0xffffffffu) {
            scnt = readlane(fc == 0 ? ch[0].cnt : ch[TM_CPL - 1].cnt, fl);
            if (scnt <= R && lane < scnt) S->stage[t & (TM_R - 1)][lane] = srun;
        }
        const uint32_t spos2w = 0xffffffffu;  // header words of a second staged list (none)
        const int32_t scnt2 = 0;
        if (lane == 0) {
            *reinterpret_cast<v4i32*>(&Rr->h.jc) = v4i32{jc, jm, jg, jd};
            *reinterpret_cast<v4u32*>(&Rr->h.pbit) = v4u32{jp, spos, (uint32_t)scnt, spos2w};
            *reinterpret_cast<v4u32*>(&Rr->h.blo) = v4u32{(uint32_t)B, (uint32_t)(B >> 32), (uint32_t)scnt2, 0xffffffffu};
            Rr->h.v = v;
            Rr->h.n = n;
            Rr->h.q = J.q;
            lds_release();  // items, stage and header before the ready word
            lds_st(&Rr->h.ready, (uint32_t)t + 1u);
        }
#ifdef FIT_STAMPS
        hs_acc += __builtin_amdgcn_s_memtime() - hs0;
        ++hs_n;
#endif
        cur = nxt;
        t += TM_H;
    }
}

// ------------------------------------------------------------------------------ decider
struct TmRing {  // lanes 0..7: job t's decision in lane t & 7
    int32_t slot;   // dirty slot
    int32_t ro;     // its LDS region's first run (slot * RS)
    uint32_t pos;   // node position
    uint32_t mask;
    int32_t cnt;    // its list's run count after that decision
    int32_t orig;
    int32_t job;    // window job that wrote it (-1: dead)
};

struct TmRecRegs {  // one record as this lane sees it: header (every lane) and item lane & 7
    v4u32 h0, h1, h2, h3;  // {ready, v, n, q}, {jc, jm, jg, jd}, {pbit, spos, scnt, -}, {B lo, B hi}
    v4u32 i0, i1, i2;      // {klo, khi, tag, orig}, {mask, cnt, cc, cm}, {cg, ...}
};

__device__ __forceinline__ void tm_read_rec(const TmRec* R, int i8, TmRecRegs& x) {
    const __attribute__((address_space(3))) v4u32* hp = lds4(&R->h);
    const __attribute__((address_space(3))) v4u32* ip = lds4(&R->it[i8]);
    x.h0 = hp[0];
    x.h1 = hp[1];
    x.h2 = hp[2];
    x.h3 = hp[3];
    x.i0 = ip[0];
    x.i1 = ip[1];
    x.i2 = ip[2];
}

struct TmCtx {  // the decider's window constants (SGPRs)
    TmShared* S;
    Seg* lr;
    int4* pmr;
    uint32_t* bitmap;
    Seg* slab;
    int32_t* out;
    int32_t* outs;
    int32_t RS, R, H, w;
    uint32_t nb;
};

struct TmDec {
    int t, nu, placed, stop;
    uint64_t gm;  // dirty slots whose list lives in the global slab
    uint32_t rb[TM_R];  // LDS byte address of ring entry i's run-list region (uniform)
    uint32_t rbv;       // the same per lane: lane l holds rb[l >> 3]
    bool exit;
#ifdef FIT_STAMPS
    unsigned long long acc[10];
#endif
};

// Current key of job (jc..jd, jp) on a global-slab dirty list (lane 0 walks it; uniform result).
__device__ __forceinline__ uint64_t tm_glob_key(const TmCtx& X, int slot, int32_t jc, int32_t jm,
                                                int32_t jg, int32_t jd, uint32_t jp, uint64_t cut) {
    const TmSlot s = X.S->slot[slot];
    const int lane = threadIdx.x & 63;
    const uint32_t pos = (uint32_t)rfl((int32_t)s.pos);
    const bool ok = (s.mask & jp) != 0u && jd <= X.H;
    const uint64_t k = tl_eval4(X.slab + (int64_t)pos * TL_MAX_SLOTS, min(rfl(s.cnt), TL_MAX_SLOTS),
                                TL_MAX_SLOTS, ok && lane == 0, jc, jm, jg, jd, X.H, pos, cut);
    return ((uint64_t)(uint32_t)readlane((int32_t)(k >> 32), 0) << 32) | (uint32_t)readlane((int32_t)k, 0);
}

template <int E>
__device__ __forceinline__ void tm_decide(const TmCtx& X, TmDec& D, TmRing& R, TmRecRegs& cur,
                                          TmRecRegs& nxt, uint32_t& flag, int32_t& oq, int32_t& on,
                                          int32_t& os) {
    TmShared* const S = X.S;
    const int lane = threadIdx.x & 63;
    const int t = D.t;
    if (t >= X.w) D.exit = true;
    const TmRec* Rn = &S->rec[(E + 1) & (TM_R - 1)];  // t == E (mod 8) while the window runs
    const uint32_t flag_n = lds_ld(&Rn->h.ready);

    struct Dec {
        uint64_t bs, cand;
        int w;
        bool tr;          // this lane's ring key beat its item
        bool anywalk;     // a live ring list fails at slot 0 (a walk may find a later start)
    };
    auto decide = [&](const TmRecRegs& x) {
        Dec d;
        const int32_t v = (int32_t)x.h0.y, n = (int32_t)x.h0.z;
        const int32_t jc = (int32_t)x.h1.x, jm = (int32_t)x.h1.y, jg = (int32_t)x.h1.z, jd = (int32_t)x.h1.w;
        const uint32_t jp = x.h2.x;
        const bool live = R.job >= v;
        const bool isg = live && ((D.gm >> (R.slot & 63)) & 1ull);
        const bool ok = live && (R.mask & jp) != 0u && jd <= X.H;
        bool fit0 = false;
        // ring list i's first run ending at or after jd: run `lane` of all 8 lists (one round
        // trip), a ballot each (a list ends at H >= jd, so the first set bit is a real run), then
        // lane i reads list i's prefix minima there
        uint64_t rk;
        {
            int32_t kk = 0;
            // lane l: run l & 7 of ring list l >> 3; lane i < 8 takes the first set bit of byte i
            // (a list shorter than eight runs ends at H >= d, so its byte has a real run set);
            // a live list whose first eight runs all end before d takes the general search below
            const int32_t e8 = lds_ld1(D.rbv + 16u * (uint32_t)min(lane & 7, X.R - 1));
            const uint64_t m8 = __ballot(e8 >= jd);
            const uint32_t byte = (uint32_t)(m8 >> (8 * (lane & 7))) & 0xffu;
            kk = (int32_t)__builtin_ctz(byte | 0x100u);
            if (__builtin_expect(__ballot(lane < 8 && ok && !isg && byte == 0u) != 0ull, 0)) {
                const uint32_t lo = 16u * (uint32_t)min(lane, X.R - 1);
                int32_t ev[TM_R];
#pragma unroll
                for (int i = 0; i < TM_R; ++i) ev[i] = lds_ld1(D.rb[i] + lo);
#pragma unroll
                for (int i = 0; i < TM_R; ++i) {
                    const uint64_t m = __ballot(ev[i] >= jd);
                    kk = writelane(m ? (int)__builtin_ctzll(m) : 0, i, kk);
                }
            }
            const int4 pk = X.pmr[R.ro + min(kk, X.R - 1)];
            fit0 = ok && !isg && pk.x >= jc && pk.y >= jm && pk.z >= jg;
            rk = fit0 ? tl_key(0, pk.x, pk.y, pk.z, jc, jm, jg, R.pos) : KEY_INF;
        }
        d.anywalk = __ballot(ok && !fit0) != 0ull;
        // item staleness: its node is in the live ring (lanes 8..15 hold a copy of the ring, so
        // row_ror:k, k = 0..7, shows lane i < 8 every ring entry once)
        const uint32_t ip = x.i0.x & TL_POS_MASK;
        const uint32_t P0 = live ? R.pos : 0xffffffffu;  // positions are < 2^22
        const uint32_t P8 = dpp32<0x128>(P0);
        const uint32_t P2 = (lane & 8) ? P8 : P0;
        const uint32_t d0 = ip ^ P2, d1 = dpp_ror_xor<1, true>(P2, ip),
                       d2 = dpp_ror_xor<2, false>(P2, ip), d3 = dpp_ror_xor<3, false>(P2, ip),
                       d4 = dpp_ror_xor<4, false>(P2, ip), d5 = dpp_ror_xor<5, false>(P2, ip),
                       d6 = dpp_ror_xor<6, false>(P2, ip), d7 = dpp_ror_xor<7, false>(P2, ip);
        const bool stale = min(min(min(d0, d1), min(d2, d3)), min(min(d4, d5), min(d6, d7))) == 0u;
        const uint64_t ik0 = ((uint64_t)x.i0.y << 32) | x.i0.x;
        const uint64_t ik = (lane < n && lane < 8 && !stale) ? ik0 : KEY_INF;
        d.tr = rk < ik;
        d.cand = d.tr ? rk : ik;
        const uint64_t best = min8_2pass(d.cand);
        d.bs = ((uint64_t)(uint32_t)readlane((int32_t)(best >> 32), 0) << 32) |
               (uint32_t)readlane((int32_t)(uint32_t)best, 0);
        d.w = __builtin_ctzll((__ballot(d.cand == d.bs) & 0xffull) | 0x100ull) & 7;
        return d;
    };
    TM_CLK(c0);
    Dec d = decide(cur);
    TM_CLK(c1);
    TM_ADD(1, c1 - c0);
    const uint64_t B = ((uint64_t)cur.h3.y << 32) | cur.h3.x;
    int gslot = -1;  // winner: a global-slab dirty list that is not in the ring
    {
        const uint64_t bm = d.bs < B ? d.bs : B;
        const bool need_walk = d.anywalk && (bm == KEY_INF || (bm >> 54) > 0);
        const bool rec_missing = flag != (uint32_t)t + 1u;
        if (__builtin_expect(!D.exit && (rec_missing || need_walk || D.gm != 0ull), 0)) {
            if (rec_missing) {  // record t not complete when read: wait for it, read it again
                TM_CLK(w0);
                for (unsigned sp = 0;; ++sp) {
                    flag = lds_ld(&S->rec[t & (TM_R - 1)].h.ready);
                    if (flag == (uint32_t)t + 1u) break;
                    if (sp > MW_SPIN_LIMIT || lds_ld(&S->fail)) {
                        commit_fail(&S->fail, &S->trip_arg, TRIP_DECIDER_REC, (uint32_t)t);
                        D.stop = 3;
                        D.exit = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(0);
                }
                lds_acquire();
                tm_read_rec(&S->rec[t & (TM_R - 1)], lane & 7, cur);
                TM_CLK(w1);
                TM_ADD(0, w1 - w0);
                d = decide(cur);
            }
            TM_CLK(x0);
            if (!D.exit) {
                const int32_t v = (int32_t)cur.h0.y;
                const int32_t jc = (int32_t)cur.h1.x, jm = (int32_t)cur.h1.y, jg = (int32_t)cur.h1.z,
                              jd = (int32_t)cur.h1.w;
                const uint32_t jp = cur.h2.x;
                const uint64_t Bc = ((uint64_t)cur.h3.y << 32) | cur.h3.x;
                uint64_t bm = d.bs < Bc ? d.bs : Bc;
                const bool live = R.job >= v;
                const bool isg = live && ((D.gm >> (R.slot & 63)) & 1ull);
                // ring lists on LDS that fail at slot 0: a later start can still win only if the
                // best so far starts later than 0 — walk them (wave-wide, one list at a time)
                if (d.anywalk && (bm == KEY_INF || (bm >> 54) > 0)) {
                    TM_CNT(9, 1);
                    const int32_t lim = bm == KEY_INF ? X.H : (int32_t)(bm >> 54);
                    const bool ok = live && !isg && (R.mask & jp) != 0u && jd <= X.H;
                    for (uint64_t m = __ballot(ok) & 0xffull; m; m &= m - 1) {
                        const int l = __builtin_ctzll(m);
                        const int sl = readlane(R.slot, l);
                        const uint32_t p = (uint32_t)readlane((int32_t)R.pos, l);
                        const uint64_t k = tl_walk_wave(X.lr + sl * X.RS, readlane(R.cnt, l), jc, jm, jg, jd,
                                                        lim, p);
                        if (lane == l && k < d.cand) {
                            d.cand = k;
                            d.tr = true;
                        }
                    }
                }
                uint64_t best = min8_2pass(d.cand);
                best = ((uint64_t)(uint32_t)readlane((int32_t)(best >> 32), 0) << 32) |
                       (uint32_t)readlane((int32_t)(uint32_t)best, 0);
                // global-slab lists: the decider evaluates them all, every job
                uint64_t gb = KEY_INF;
                for (uint64_t m = D.gm; m; m &= m - 1) {
                    const int s = __builtin_ctzll(m);
                    const uint64_t cut = umin64(umin64(best, gb), Bc);
                    const uint64_t k = tm_glob_key(X, s, jc, jm, jg, jd, jp, cut);
                    if (k < gb) {
                        gb = k;
                        gslot = s;
                    }
                }
                if (gb < best) {
                    best = gb;
                } else {
                    gslot = -1;
                }
                bm = best;
                d.bs = best;
                d.w = __builtin_ctzll((__ballot(d.cand == d.bs) & 0xffull) | 0x100ull) & 7;
            }
            TM_CLK(x1);
            TM_ADD(2, x1 - x0);
        }
    }
    // stops: a node outside the candidate lists could win (rescan), or the dirty set is full
    const uint64_t Bn = ((uint64_t)cur.h3.y << 32) | cur.h3.x;
    const bool placed0 = d.bs != KEY_INF;
    const int w = d.w;
    const bool wtr = gslot < 0 && readlane(d.tr ? 1 : 0, w) != 0;
    const int32_t itag = readlane((int32_t)cur.i0.z, w);
    const bool fresh0 = placed0 && gslot < 0 && !wtr && itag < 0;
    if (!D.exit && ((Bn != KEY_INF && d.bs > Bn) || (fresh0 && D.nu >= TL_UCAP))) {
        D.stop = (Bn != KEY_INF && d.bs > Bn) ? 1 : 2;
        D.exit = true;
    }
    const bool go = !D.exit;
    const bool placed = placed0 && go;
    const bool fresh = fresh0 && go;
    const uint32_t pos = (uint32_t)d.bs & TL_POS_MASK;
    const int32_t start = placed ? (int32_t)(d.bs >> 54) : -1;
    const int32_t jc = (int32_t)cur.h1.x, jm = (int32_t)cur.h1.y, jg = (int32_t)cur.h1.z, jd = (int32_t)cur.h1.w;
    int32_t slot, cnt, orig;
    uint32_t mask;
    if (gslot >= 0) {
        const TmSlot s = S->slot[gslot];
        slot = gslot;
        cnt = rfl(s.cnt);
        orig = rfl(s.orig);
        mask = (uint32_t)rfl((int32_t)s.mask);
    } else if (wtr) {
        slot = readlane(R.slot, w);
        cnt = readlane(R.cnt, w);
        orig = readlane(R.orig, w);
        mask = (uint32_t)readlane((int32_t)R.mask, w);
    } else {
        slot = fresh ? D.nu : itag;
        cnt = readlane((int32_t)cur.i1.y, w);
        orig = readlane((int32_t)cur.i0.w, w);
        mask = (uint32_t)readlane((int32_t)cur.i1.x, w);
    }
    TM_CLK(a0);
#ifdef FIT_STAMPS_FINE
    unsigned long long a1 = a0;
#endif
    if (placed) {
        Seg* const L = X.lr + slot * X.RS;
        int4* const PM = X.pmr + slot * X.RS;
        bool glob = (D.gm >> slot) & 1ull;
        // the list in registers (run `lane`): a new dirty node's from the helper's stage (or the
        // slab), an LDS list's from its region; tm_reserve writes the whole new list
        Seg g{0, 0, 0, 0};
        int nn = -1;
        if (fresh) {  // a clean winner becomes dirty slot nu
            glob = cnt > X.R;
            if (!glob) {
                // typed loads on both sides: a plain select of the two pointers becomes one flat
                // load, which waits on the vector-memory path even for the LDS stage
                if (cur.h2.y == pos && (int32_t)cur.h2.z == cnt) {  // staged by the helper
                    const v4u32 x = lds4(&S->stage[t & (TM_R - 1)][lane])[0];
                    g = Seg{(int32_t)x.x, (int32_t)x.y, (int32_t)x.z, (int32_t)x.w};
                } else {  // not the staged item (written meanwhile)
                    const v4i32 x = *(const GAS v4i32*)(X.slab + (int64_t)pos * TL_MAX_SLOTS + lane);
                    g = Seg{x.x, x.y, x.z, x.w};
                }
            }
            if (lane == 0) {
                const uint32_t rel = pos - X.nb;
                X.bitmap[rel >> 5] |= 1u << (rel & 31);
                S->slot[slot] = TmSlot{pos, mask, orig, cnt, readlane((int32_t)cur.i1.z, w),
                                       readlane((int32_t)cur.i1.w, w), readlane((int32_t)cur.i2.x, w),
                                       glob ? 1 : 0};
            }
            if (glob) D.gm |= 1ull << slot;
            D.nu += 1;
            TM_CNT(6, 1);
        } else if (!glob) {
            const v4u32 x = lds4(L + min(lane, X.R - 1))[0];
            g = Seg{(int32_t)x.x, (int32_t)x.y, (int32_t)x.z, (int32_t)x.w};
        }
#ifdef FIT_STAMPS_FINE
        a1 = __builtin_amdgcn_s_memtime();
        TM_ADD(3, a1 - a0);
#endif
        if (!glob) {
            nn = tm_reserve(lds_addr(L), lds_addr(PM), lds_addr(&S->scr[lane]), g, cnt, X.R, start,
                            start + jd, jc, jm, jg);
            if (nn < 0) {  // outgrows its LDS region: the list moves to the global slab
                Seg* gl = X.slab + (int64_t)pos * TL_MAX_SLOTS;
                if (!fresh && lane < cnt) gl[lane] = g;  // a new dirty node's list is there already
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                nn = tl_reserve_any(gl, cnt, start, start + jd, jc, jm, jg, S->scr);
                D.gm |= 1ull << slot;
                glob = true;
            }
        } else {
            nn = tl_reserve_any(X.slab + (int64_t)pos * TL_MAX_SLOTS, cnt, start, start + jd, jc, jm, jg,
                                S->scr);
        }
        if (lane == 0) {  // the helpers' view of the slot
            S->slot[slot].cnt = nn;
            S->slot[slot].glob = glob ? 1 : 0;
        }
        cnt = nn;
        {
            TM_CLK(a2);
            TM_ADD(4, a2 - a1);
        }
        // ring: an older entry of the same slot dies; lane E takes job t
        R.job = (R.slot == slot) ? -1 : R.job;
        R.slot = writelane_c<E>(slot, R.slot);
        D.rb[E] = (uint32_t)rfl((int32_t)lds_addr(L));
        D.rbv = ((lane >> 3) == E) ? D.rb[E] : D.rbv;
        R.ro = writelane_c<E>(slot * X.RS, R.ro);
        R.pos = (uint32_t)writelane_c<E>((int32_t)pos, (int32_t)R.pos);
        R.mask = (uint32_t)writelane_c<E>((int32_t)mask, (int32_t)R.mask);
        R.cnt = writelane_c<E>(cnt, R.cnt);
        R.orig = writelane_c<E>(orig, R.orig);
        R.job = writelane_c<E>(t, R.job);
        D.placed += 1;
    } else if (go) {
        R.job = writelane_c<E>(-1, R.job);  // nothing written by job t
    }
    // publish the decisions so far (release store of {decided, nu}: the reservation's list and
    // prefix-minimum writes before it), then read record t+1's data after acquiring its ready
    // word (the load above is long done) — at the end of the step, so the next step starts
    // without draining the LDS queue and the record reads overlap the parking below
    lds_release();
    __hip_atomic_store(&S->dn, ((uint64_t)(uint32_t)D.nu << 32) | (uint32_t)(t + (go ? 1 : 0)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    flag = flag_n;
    lds_acquire();
    tm_read_rec(Rn, lane & 7, nxt);
    // placement of job t parked in lane t & 63, stored 64 at a time
    oq = writelane(rfl((int32_t)cur.h0.w), t & 63, oq);
    on = writelane(placed ? orig : -1, t & 63, on);
    os = writelane(start, t & 63, os);
    if (E == 7 && go && (t & 63) == 63) {  // uniform, once per 64 jobs
        if (oq >= 0) {
            ((GAS int32_t*)X.out)[oq] = on;
            ((GAS int32_t*)X.outs)[oq] = os;
        }
        oq = -1;
    }
    D.t = t + (go ? 1 : 0);
#ifdef FIT_STAMPS
    {
        TM_CLK(a3);
        TM_ADD(8, a3 - a0);
        TM_CNT(5, go ? 1 : 0);
    }
#endif
}

__device__ __noinline__ CommitResult tm_decider(const CompPlan& Pref, TmShared* Sin, Seg* lr_,
                                                int4* pmr_, uint32_t* bitmap_, int32_t RS, int32_t R_,
                                                Seg* slab, int32_t* out, int32_t* outs, int32_t H) {
    const CompPlan P = plan_sgpr(Pref);
    TmCtx X;
    X.S = tm_lds(Sin);
    X.lr = tm_lds(lr_);
    X.pmr = tm_lds(pmr_);
    X.bitmap = tm_lds(bitmap_);
    X.slab = slab;
    X.out = out;
    X.outs = outs;
    X.RS = rfl(RS);
    X.R = rfl(R_);
    X.H = rfl(H);
    X.w = P.w;
    X.nb = (uint32_t)P.nb;
    TmShared* const S = X.S;
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_s_setprio(3);  // shares its SIMD with a helper wave
    TmDec D{};
    D.exit = false;
    for (int i = 0; i < TM_R; ++i) D.rb[i] = lds_addr(X.lr);
    D.rbv = lds_addr(X.lr);
    TmRing R{-1, 0, 0xffffffffu, 0u, 0, -1, -1};
    int32_t oq = -1, on = -1, os = -1;
    TmRecRegs ra, rb;
    uint32_t flag = 0;
#if defined(FIT_STAMPS) && !defined(FIT_STAMPS_FINE)
    const unsigned long long k0 = __builtin_amdgcn_s_memtime();
#endif
    if (P.w > 0) {
        for (unsigned sp = 0;; ++sp) {
            flag = lds_ld(&S->rec[0].h.ready);
            if (flag == 1u) break;
            if (sp > MW_SPIN_LIMIT || lds_ld(&S->fail)) {
                commit_fail(&S->fail, &S->trip_arg, TRIP_DECIDER_REC, 0u);
                D.stop = 3;
                D.exit = true;
                break;
            }
            __builtin_amdgcn_s_sleep(0);
        }
        lds_acquire();
        tm_read_rec(&S->rec[0], lane & 7, ra);
    } else {
        D.exit = true;
    }
#if defined(FIT_STAMPS) && !defined(FIT_STAMPS_FINE)
    const unsigned long long k1 = __builtin_amdgcn_s_memtime();
    D.acc[0] += k1 - k0;
    D.acc[8] += 1;
#endif
    while (!D.exit) {
        tm_decide<0>(X, D, R, ra, rb, flag, oq, on, os);
        tm_decide<1>(X, D, R, rb, ra, flag, oq, on, os);
        tm_decide<2>(X, D, R, ra, rb, flag, oq, on, os);
        tm_decide<3>(X, D, R, rb, ra, flag, oq, on, os);
        tm_decide<4>(X, D, R, ra, rb, flag, oq, on, os);
        tm_decide<5>(X, D, R, rb, ra, flag, oq, on, os);
        tm_decide<6>(X, D, R, ra, rb, flag, oq, on, os);
        tm_decide<7>(X, D, R, rb, ra, flag, oq, on, os);
    }
    const int t = D.t;
#if defined(FIT_STAMPS) && !defined(FIT_STAMPS_FINE)
    D.acc[1] += __builtin_amdgcn_s_memtime() - k1;
#endif
    if (oq >= 0 && lane < (t & 63)) {  // the last partial group
        ((GAS int32_t*)out)[oq] = on;
        ((GAS int32_t*)outs)[oq] = os;
    }
    lds_release();
    __hip_atomic_store(&S->dn, ((uint64_t)(uint32_t)D.nu << 32) | (uint32_t)t, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    lds_st(&S->halt, 1u);
#ifdef FIT_STAMPS
    if (lane == 0)
        for (int i = 0; i < 10; ++i) atomicAdd(&g_tlst[blockIdx.x & 63][i], D.acc[i]);
#endif
    return CommitResult{t, D.stop, D.nu, D.placed};
}

// All 8 waves of the committer block call this; returns the same result in every wave.  smem:
// engine_tl_lds_bytes(); R: LDS run-list capacity per dirty slot (engine_tl_runs).  glob: set when
// a dirty list of the window lives in the global slab — written with plain stores, which the next
// round must release before its scan reads them; every other write-back is stored through.
__device__ __forceinline__ CommitResult commit_tl_window_mw(
    const CompPlan& P, unsigned char* smem, Seg* __restrict__ slab, TlHdr* __restrict__ hdr,
    const uint64_t* __restrict__ cand, const uint64_t* __restrict__ bnd,
    const JobRec* __restrict__ wjob, int32_t* __restrict__ out, int32_t* __restrict__ outs,
    int32_t H, int32_t R, MwTiles T, bool& glob) {
    TmShared* S = reinterpret_cast<TmShared*>(smem);
    const int32_t RS = R + TL_PAD;
    Seg* lr = reinterpret_cast<Seg*>(smem + sizeof(TmShared));
    int4* pmr = reinterpret_cast<int4*>(lr + TL_UCAP * RS);
    uint32_t* bitmap = reinterpret_cast<uint32_t*>(pmr + TL_UCAP * RS);
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = threadIdx.x; i < nwords; i += SCAN_WAVES * 64) bitmap[i] = 0u;
    if (threadIdx.x < TM_R) S->rec[threadIdx.x].h.ready = 0u;
    if (threadIdx.x < 8) S->wclk[threadIdx.x] = 0u;
    if (threadIdx.x == 0) {
        S->dn = 0ull;
        S->halt = 0u;
        S->fail = 0u;
    }
    __syncthreads();
    if (P.w > 0) {
        if (wave == 0) {
            const CommitResult r = tm_decider(P, S, lr, pmr, bitmap, RS, R, slab, out, outs, H);
            if (threadIdx.x == 0) {
                S->res[0] = r.done;
                S->res[1] = r.stop;
                S->res[2] = r.dirty;
                S->res[3] = r.placed;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // placements, global-slab lists
        } else {
            tm_helper(P, S, lr, pmr, bitmap, RS, R, slab, hdr, cand, bnd, wjob, wave, H, T);
        }
    } else if (threadIdx.x == 0) {
        S->res[0] = S->res[1] = S->res[2] = S->res[3] = 0;
    }
    __syncthreads();
    const CommitResult r{S->res[0], S->res[1], S->res[2], S->res[3]};
    // round end: LDS lists back to their slabs (the next scan reads them), headers for all
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int lane = threadIdx.x & 63;
    // (slot l by wave l & 7; a global-slab list only by wave 0, which wrote it: its own stores are
    // ordered before its loads, another wave's L1 could hold the lines stale)
#ifdef FIT_STAMPS
    const unsigned long long e0 = __builtin_amdgcn_s_memtime();
#endif
    glob = false;
    for (int l = 0; l < r.dirty; ++l) {
        const TmSlot s = S->slot[l];
        const bool gl = rfl(s.glob) != 0;
        glob |= gl;
        if (gl ? wave != 0 : (l & (SCAN_WAVES - 1)) != wave) continue;
        const uint32_t p = (uint32_t)rfl((int32_t)s.pos);
        const int n = rfl(s.cnt);
        Seg* dst = slab + (int64_t)p * TL_MAX_SLOTS;
        Seg hd = Seg{H, -1, -1, -1};
        // written through (two 8-B sc1 stores per run): the release at the next round's start then
        // finds few dirty L2 lines to write back (fit_engine_ctl.h store_through)
        auto put = [](Seg* d, const Seg& v) {
            uint64_t* w = reinterpret_cast<uint64_t*>(d);
            store_through64(w, (uint64_t)(uint32_t)v.end | ((uint64_t)(uint32_t)v.cpu << 32));
            store_through64(w + 1, (uint64_t)(uint32_t)v.mem | ((uint64_t)(uint32_t)v.gpu << 32));
        };
        if (!gl) {
            const Seg* src = lr + l * RS;
            if (lane < n) {
                hd = src[lane];
                put(dst + lane, hd);
            }
        } else if (lane < TL_HEAD && lane < n) {
            hd = dst[lane];
        }
        if (lane < TL_HEAD) put(&hdr[p].head[lane], hd);
        if (lane == 0) __hip_atomic_store(&hdr[p].cnt, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
#ifdef FIT_STAMPS
    if (threadIdx.x == 0) atomicAdd(&g_tlst[blockIdx.x & 63][7], __builtin_amdgcn_s_memtime() - e0);
#endif
    __syncthreads();
    if (S->fail) return CommitResult{r.done, 3, r.dirty, r.placed};
    return r;
}

}  // namespace fitgpu
