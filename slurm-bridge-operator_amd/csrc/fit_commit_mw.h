// fit_commit_mw.h — the commit of one component's window by a whole 8-wave workgroup
// (DESIGN.md §3.7): one DECIDER wave walks the jobs in priority order; seven HELPER waves
// pre-resolve the jobs ahead of it against a slightly stale snapshot of the dirty state.
//
// Why it is exact.  Let the decider have resolved jobs [0, v) when a helper snapshots the
// state for job t (v >= t - (MW_M - 1), enforced by the helper).  The helper records the MW_M
// smallest keys <= B among (clean candidates of t) ∪ (dirty rows), each item tagged clean (with
// its node row) or dirty (its slot).  When the decider reaches t, only the nodes written by jobs
// [v, t) — at most MW_M - 1 of them, the decider's own last decisions, kept in its "written
// ring" — can differ from the snapshot.  It drops every item whose node is in the live part of
// the ring and evaluates the live ring rows at their current state.  If the list held MW_M items,
// at least one survives and every unlisted node has a key above it; if it held fewer, it held
// every candidate <= B.  Either way
//     best = min(surviving items, live ring rows)
// is the sequential answer restricted to keys <= B, and the SPEC stop rule reduces to
// "best > B with B finite" (a clean candidate is always <= B).  The argument needs nothing of a
// row or bitmap word the helper read after the snapshot: any node changed after v is in the live
// ring, so a torn or newer read of it only produces an item the decider drops.
//
// "Jobs" above are the window's LIVE jobs (round 3): a job that no node fits at the round's start
// is unplaced whatever the decisions before it, so the helpers skip it (per-tile feasibility
// masks from the scan, mw_skip_live) and record i, ring lane i & 7 and the snapshot counts all
// index the i-th live job; the record header carries its window index, and a record whose index
// is the window size ends the window.
//
// Cost model (measured on gfx950, tools/ubench: one wave alone) — what shapes the code below:
// a dependent VALU op ≈ 4.7 cycles, any scalar branch ≈ 25-30, a VALU → SGPR → SALU hand-off
// ≈ 20-36, v_readlane → v_writelane ≈ 8.6, one LDS round trip ≈ 50-64.  So the decider's job
// step is straight-line VALU with ONE exception branch per job (record not ready, B exceeded,
// dirty set full, end of window), the written ring lives in lanes 0..7 (slot = job & 7, a
// compile-time lane in the 8-way unrolled loop), item staleness is a lane-parallel XOR against
// the ring rotated with DPP row_ror, the minimum over ring rows and items is three 64-bit DPP
// steps over 8 lanes, and the next job's record is read while this one is decided.  The
// decision's bookkeeping (dirty row, bitmap bit, placement) is issued by the decider itself as
// fire-and-forget LDS writes.
//
// LDS protocol (one workgroup), C++ memory model at workgroup scope on LDS ("local"):
//   decider → helpers: dirty rows, bitmap, then {decided, nu} by a release store;
//   helpers: relaxed poll of {decided, nu}, then an acquire fence, then rows / bitmap.
//   helper → decider: record items and header, then the record's ready word by a release store;
//   decider: relaxed load of the ready word, an acquire fence, then the record's data.
// On gfx950 (no threadgroup split) a workgroup-scope release / acquire on LDS is an
// `s_waitcnt lgkmcnt(0)` before the store / after the load (checked in the ISA); both sit where
// the counter is already drained, so the protocol costs no cycles on the decider's chain.
#pragma once
#include "fit_common.h"
#include "fit_engine_ctl.h"

namespace fitgpu {

#ifndef MW_ITEMS
#define MW_ITEMS 8
#endif
constexpr int MW_M = MW_ITEMS;          // items per pre-resolved record (> snapshot lag)
constexpr int MW_R = 8;                 // record ring; slot t & 7 frees once job t-8 is decided
#ifndef MW_SNAP
#define MW_SNAP MW_ITEMS  // a helper snapshots job t's state once the decider has resolved t - (MW_SNAP - 1)
#endif
static_assert(MW_SNAP >= 1 && MW_SNAP <= MW_ITEMS, "a later snapshot only shortens the ring span");
constexpr int MW_WAVES = SCAN_WAVES;    // 1 decider + MW_H helpers
constexpr int MW_H = MW_WAVES - 1;  // helpers: waves 1..7
static_assert(MW_M == 8, "the decider holds one item per lane of its 8-lane ring group");
static_assert(MW_R >= MW_M, "record slot reuse relies on the lag bound");

#ifndef MW_HSLEEP
#define MW_HSLEEP 1  // helper back-off per missing decided job, in units of 64 cycles (12 before the
                      // 4-entry helpers: C3 k_engine 32.2 -> 31.2 ms at 0-2)
#endif
constexpr int MW_EPL = (MAX_SLICES * KS + 63) / 64;  // candidate entries per helper lane
static_assert(MW_EPL <= 2, "at most two candidate entries per lane");

struct alignas(16) MwRow {  // dirty row, current state
    int32_t cpu, mem, gpu, avail;
    uint32_t mask, pos;
    int32_t orig, ver;  // ver: last job (window index) that created or changed it
};

struct alignas(16) MwItem {  // 48 B; the decider reads the first 36
    uint32_t pos, score;  // key = score << 32 | pos
    int32_t tag, orig;    // tag: dirty slot (>= 0) or -1 (a clean candidate; row below)
    int32_t cpu, mem, gpu, avail;
    uint32_t mask, pad0, pad1, pad2;
};

struct alignas(16) MwHdr {
    uint32_t ready;  // i + 1 once record i is complete (release store, last)
    int32_t v, n, q;
    int32_t cpu, mem, gpu, wall;
    uint32_t pbit;
    int32_t tj;      // the record's job (window index); P.w: the window has no live job left
    uint64_t B;
};

struct alignas(16) MwRec {
    MwHdr h;
    MwItem it[MW_M];
};

struct alignas(16) MwShared {
    uint64_t dn;       // {decided (low 32), nu (high 32)}: the helpers' snapshot, release-stored
    uint32_t halt;     // decider stopped
    uint32_t fail;     // helper / decider watchdog: the TripSite of the first wait that gave up
    int32_t res[4];    // CommitResult of the window
    uint32_t pubt;     // job tiles of the window published to the task ring (MwTiles::ring)
    uint32_t wd;       // watchdog: realtime ticks a wait may last (set by the committer; the
                       // commit's own waits use spin bounds, see MW_SPIN_LIMIT)
    uint32_t trip_arg; // the failed wait's tile / record
    uint32_t pad[5];
    MwRec rec[MW_R];
    MwRow rows[UCAP];
    uint32_t bitmap[1];  // (ne - nb + 31) / 32 words, dirty membership by position
};

__host__ __device__ constexpr size_t mw_lds_bytes(int32_t max_component_nodes) {
    return sizeof(MwShared) + (size_t)((max_component_nodes + 31) / 32) * 4;
}

#ifdef FIT_STAMPS
// [comp][0] decider cycles, [1] decider waiting for records (slow path), [2] decided jobs,
// [3] helper cycles (sum), [4] helper wait-for-snapshot, [5] helper jobs, [6] items written,
// [7] (unused), [8] (unused), [9] decider waits in each round's first 8 jobs,
// [10..12] first-tile scan (workers), [13] helper tile waits, [14] helper snapshot → record,
// [15] helper snapshot → extraction start, [16] committer: round end → tiles published (wait for
// the round before last, resets, release, publish), [17] decider: start → record 0 ready,
// [18] rounds
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

// ---- LDS hand-off primitives (workgroup scope, LDS only) ------------------------------------
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }

// The commit's waits — the helpers' waits for scan tiles, and the decider <-> helper waits inside
// the block — keep round 4's spin bound (MW_SPIN_LIMIT polls, ≈ 4-8 s).  Every other wait of the
// engine has a time deadline (fit_engine_ctl.h WaitClock), and those bound what the commit waits
// for: its tiles come from scan workers whose own waits trip on time and drain the launch.  A time
// check in the helper's tile-wait loop — any extra branch there, in fact — changes the code LLVM
// generates for the whole (VGPR-limited) helper (different unrolling and branch layout) and cost
// C3 +0.55 ms / C2 +0.3 ms in paired A/Bs (profiles/r05_watchdog_ab.txt); so the loop keeps its
// round-4 shape and only the failing branch records its site.
constexpr unsigned MW_SPIN_LIMIT = 1u << 24;

// A commit wait gave up (uniform call; helper or decider): the block's first failure names its
// TripSite and argument in `fail` / `trip_arg`; `fail` stops every wave of the block and the
// committer turns it into the launch's trip record (fit_engine_ctl.h trip_record).
// Every lane stores the same values (no lane test: a lane id kept live for it cost the decider a
// VGPR across its whole loop); two waves failing at once may leave the later one's site.
__device__ __forceinline__ void commit_fail(uint32_t* fail, uint32_t* trip_arg, uint32_t site,
                                            uint32_t arg) {
    if (lds_ld(fail) == 0u) {
        lds_st(trip_arg, arg);
        lds_st(fail, site);
    }
}

// Tile readiness: the window's scan tiles complete while the window is being
// committed; a helper waits for the (job tile)'s per-tile counter to reach nslice before reading
// that tile's candidates, bound and job row; an agent-scope acquire when a tile turns ready drops
// the CU's L1 (it may hold stale lines of these reused buffers), so the reads stay plain loads.
// tdone == nullptr: the whole window was acquired before the commit (no waits).
struct MwTiles {
    const unsigned* tdone;  // per-tile completed slice counts of this component's window
    unsigned need;          // nslice
    // just-in-time publishing (k_engine, ENGINE_AHEAD > 0): the committer publishes the window's
    // first ENGINE_AHEAD job tiles; a helper that moves on to tile k publishes the tiles up to
    // k + ENGINE_AHEAD - 1 first.  ring == nullptr: every tile was published up front.
    unsigned long long* ring;
    EngineCtl* ctl;
    unsigned round;  // task round tag
    unsigned comp;
    unsigned ntj;    // job tiles of the window
    // per job tile: jobs with a node that fits them at the round's start (k_engine's scan ORs
    // them in before it counts the tile done); nullptr: every job of the window is live
    const unsigned long long* feas;
};
#ifndef ENGINE_AHEAD
#define ENGINE_AHEAD 4  // 0: every tile of the window published up front
#endif

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

// Write-through reads of a scan tile's outputs (candidates, bound, job row), which the scan workers
// store through (sc1) and count with an agent-scope add: a helper that has seen the tile's count
// reach its target in a relaxed agent poll reads them with sc1 loads, which bypass this CU's L1,
// instead of an acquire fence (≈1.7 us, once per tile per helper, and on every round's start:
// cdna_hip_programming.md §6 Guideline 16; MI355X_MICROARCH.md hand-off table, row 1 — one block
// per CU, 8-B sc1 stores and loads, the polling wave loads after its poll matched).
__device__ __forceinline__ uint64_t ld_through(const GAS uint64_t* p) {
    return __hip_atomic_load(const_cast<GAS uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ JobRec ld_job_through(const GAS JobRec* p) {
    const GAS uint64_t* q = (const GAS uint64_t*)p;
    const uint64_t w0 = ld_through(q), w1 = ld_through(q + 1), w2 = ld_through(q + 2), w3 = ld_through(q + 3);
    JobRec r;
    r.q = (int32_t)(uint32_t)w0;
    r.cpu = (int32_t)(uint32_t)(w0 >> 32);
    r.mem = (int32_t)(uint32_t)w1;
    r.gpu = (int32_t)(uint32_t)(w1 >> 32);
    r.wall = (int32_t)(uint32_t)w2;
    r.pbit = (uint32_t)(w2 >> 32);
    r.k = (int32_t)(uint32_t)w3;
    r.pad = (int32_t)(uint32_t)(w3 >> 32);
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
    p.ks = rfl(q.ks);
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

// ---- DPP building blocks ---------------------------------------------------------------------
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    if constexpr (ROWMASK == 0xf)  // every lane has a source: a plain DPP move
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
    else  // lanes of rows outside the mask keep their value
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWMASK, 0xf, false);
}
// one 64-bit min step against the DPP-permuted value (2 moves, a 64-bit compare, 2 selects)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint64_t dpp_min64(uint64_t v) {
    const uint32_t lo = dpp32<CTRL, ROWMASK>((uint32_t)v), hi = dpp32<CTRL, ROWMASK>((uint32_t)(v >> 32));
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    return o < v ? o : v;
}
// minimum over each group of 8 lanes, in all 8 of them: quad swaps, then the half-row mirror
__device__ __forceinline__ uint64_t min8_64(uint64_t v) {
    v = dpp_min64<0xb1>(v);   // quad_perm [1,0,3,2]
    v = dpp_min64<0x4e>(v);   // quad_perm [2,3,0,1]
    return dpp_min64<0x141>(v);  // row_half_mirror
}
// Fused DPP ALU ops in inline asm (hipcc emits a DPP move plus the ALU op for the builtins).
// Each string opens with the two wait states a DPP read of a VGPR written by the previous VALU
// instruction needs (cdna_hip_programming.md: DPP hazard; `s_nop 1`).
#define MW_DPP_MIN(v, CTL) asm volatile("s_nop 1\n\tv_min_u32_dpp %0, %0, %0 " CTL : "+v"(v))
__device__ __forceinline__ uint32_t dppmin_qp1032(uint32_t v) { MW_DPP_MIN(v, "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"); return v; }
__device__ __forceinline__ uint32_t dppmin_qp2301(uint32_t v) { MW_DPP_MIN(v, "quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"); return v; }
__device__ __forceinline__ uint32_t dppmin_hmirror(uint32_t v) { MW_DPP_MIN(v, "row_half_mirror row_mask:0xf bank_mask:0xf"); return v; }
__device__ __forceinline__ uint32_t dppmin_mirror(uint32_t v) { MW_DPP_MIN(v, "row_mirror row_mask:0xf bank_mask:0xf"); return v; }
__device__ __forceinline__ uint32_t dppmin_bcast15(uint32_t v) { MW_DPP_MIN(v, "row_bcast:15 row_mask:0xa bank_mask:0xf"); return v; }
__device__ __forceinline__ uint32_t dppmin_bcast31(uint32_t v) { MW_DPP_MIN(v, "row_bcast:31 row_mask:0xc bank_mask:0xf"); return v; }
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp_min32(uint32_t v) {
    if constexpr (CTRL == 0xb1) return dppmin_qp1032(v);
    else if constexpr (CTRL == 0x4e) return dppmin_qp2301(v);
    else if constexpr (CTRL == 0x141) return dppmin_hmirror(v);
    else if constexpr (CTRL == 0x140) return dppmin_mirror(v);
    else if constexpr (CTRL == 0x142) return dppmin_bcast15(v);
    else return dppmin_bcast31(v);
}
// d = src ^ (x rotated by K within its row of 16 lanes); NOP: src of the DPP just written
template <int K, bool NOP>
__device__ __forceinline__ uint32_t dpp_ror_xor(uint32_t x, uint32_t y) {
    uint32_t d;
    if constexpr (NOP)
        asm volatile("s_nop 1\n\tv_xor_b32_dpp %0, %1, %2 row_ror:%3 row_mask:0xf bank_mask:0xf"
                     : "=v"(d) : "v"(x), "v"(y), "i"(K));
    else
        asm volatile("v_xor_b32_dpp %0, %1, %2 row_ror:%3 row_mask:0xf bank_mask:0xf"
                     : "=v"(d) : "v"(x), "v"(y), "i"(K));
    return d;
}
// 64-bit minimum over each group of 8 lanes, in all 8: the 32-bit minimum of the high words,
// then of the low words among the lanes holding it (fused DPP mins, no 64-bit compares)
__device__ __forceinline__ uint64_t min8_2pass(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    uint32_t mh = dpp_min32<0xb1>(hi);
    mh = dpp_min32<0x4e>(mh);
    mh = dpp_min32<0x141>(mh);
    uint32_t ml = hi == mh ? lo : 0xffffffffu;
    ml = dpp_min32<0xb1>(ml);
    ml = dpp_min32<0x4e>(ml);
    ml = dpp_min32<0x141>(ml);
    return ((uint64_t)mh << 32) | ml;
}
// 32-bit minimum over the wave, valid in lane 63
__device__ __forceinline__ uint32_t wave_min32_l63(uint32_t v) {
    v = dpp_min32<0xb1>(v);
    v = dpp_min32<0x4e>(v);
    v = dpp_min32<0x141>(v);
    v = dpp_min32<0x140>(v);
    v = dpp_min32<0x142, 0xa>(v);
    return dpp_min32<0x143, 0xc>(v);
}
// minimum over the wave, valid in lane 63
__device__ __forceinline__ uint64_t wave_min64_l63(uint64_t v) {
    v = dpp_min64<0xb1>(v);
    v = dpp_min64<0x4e>(v);
    v = dpp_min64<0x141>(v);       // row_half_mirror: 8-lane groups
    v = dpp_min64<0x140>(v);       // row_mirror: whole rows of 16
    v = dpp_min64<0x142, 0xa>(v);  // row_bcast:15 → rows 1 and 3
    return dpp_min64<0x143, 0xc>(v);  // row_bcast:31 → rows 2 and 3
}

// v_writelane_b32: lane `l` of `old` := SGPR `x` (no clang builtin on this toolchain)
__device__ __forceinline__ int32_t writelane(int32_t x, int l, int32_t old) {
    int32_t r;
    // the lane select goes through M0 (one SGPR operand per VALU instruction on gfx9)
    asm("v_writelane_b32 %0, %1, m0" : "=v"(r) : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(l), "0"(old));
    return r;
}
template <int L>
__device__ __forceinline__ int32_t writelane_c(int32_t x, int32_t old) {  // compile-time lane
    int32_t r;
    asm("v_writelane_b32 %0, %1, %2" : "=v"(r) : "s"(__builtin_amdgcn_readfirstlane(x)), "i"(L), "0"(old));
    return r;
}
__device__ __forceinline__ int32_t readlane(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Wait until job tt's scan tile is complete (uniform; `ready` = tiles known complete, they finish
// roughly in order).  false: the decider halted / a watchdog tripped.
// Publish the window's job tiles [pubt, upto) (uniform; lane 0 claims the range by an LDS CAS).
__device__ __noinline__ void mw_publish(const MwTiles& T, MwShared* S, unsigned upto) {
    const int lane = threadIdx.x & 63;
    unsigned from = upto;  // nothing claimed
    if (lane == 0) {
        unsigned cur = lds_ld(&S->pubt);
        while (cur < upto) {  // a failed exchange reloads cur
            if (__hip_atomic_compare_exchange_strong(&S->pubt, &cur, upto, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                from = cur;
                break;
            }
        }
    }
    from = (unsigned)__builtin_amdgcn_readlane((int)from, 0);
    if (from >= upto) return;
    // claimed [from, upto): what the tasks' scans read — the round's plan, bounds, tile counters
    // (written through) and node rows (written through, or released) — was stored and drained by
    // the committer wave before the block barrier this wave has passed: no fence here (R1)
    engine_publish(T.ctl, T.ring, from, upto, T.need, T.round, T.comp);
}

__device__ __forceinline__ bool mw_tile_ready(const MwTiles& T, int tt, int& ready, MwShared* S) {
    if (!T.tdone) return true;
    const int tile = __builtin_amdgcn_readfirstlane(tt) / SCAN_JOBS;
    if (tile < ready) return true;
    if (T.ring && (unsigned)tile + ENGINE_AHEAD > lds_ld(&S->pubt))
        mw_publish(T, S, min((unsigned)tile + ENGINE_AHEAD, T.ntj));
    for (unsigned sp = 0;; ++sp) {
        if (__hip_atomic_load(gview(T.tdone) + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
            T.need)
            break;
        if (lds_ld(&S->halt) | lds_ld(&S->fail)) return false;
        if (sp > MW_SPIN_LIMIT) {
            lds_st(&S->trip_arg, (uint32_t)tile);
            lds_st(&S->fail, TRIP_HELPER_TILE);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    // the tile's outputs are read with sc1 loads (ld_through): no acquire fence; this only keeps
    // the compiler from moving them above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ready = tile + 1;
    return true;
}

// ---------------------------------------------------------------------------- live jobs
// A job with no node that fits it at the round's start state is unplaced whatever the jobs
// before it take (node state only shrinks within a placement) and changes nothing: the commit
// skips it (its output is already FIT_UNPLACED from k_prefilter).  The decider then walks the
// LIVE jobs only: record i (ring lane i & 7, snapshot counts, ready word) belongs to the i-th
// live job of the window, whose window index the record's header carries; a record whose job
// index is the window size ends the window.  C3: ~14 % of a component's jobs (the ones nothing
// fits once the cluster has filled) no longer cost a decider step.
struct MwCursor {
    int ct;       // job tile of the cursor
    uint64_t cm;  // live jobs of tile ct not yet taken
};
// move the cursor to the next job tile (uniform): its live-job mask once the tile is complete;
// false: halted / watchdog.  Past the window's last tile the mask stays empty.
__device__ __forceinline__ bool mw_cursor_tile(const MwTiles& T, const CompPlan& P, MwCursor& C,
                                               int& ready, MwShared* S) {
    if ((C.ct + 1) * SCAN_JOBS >= P.w) {
        C.cm = 0ull;
        return true;
    }
    ++C.ct;
    const int n = min(SCAN_JOBS, P.w - C.ct * SCAN_JOBS);
    const uint64_t valid = n >= 64 ? ~0ull : (1ull << n) - 1ull;
    if (T.feas) {
        if (!mw_tile_ready(T, C.ct * SCAN_JOBS, ready, S)) return false;
        const uint64_t f = __hip_atomic_load(gview(T.feas) + C.ct, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)f);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(f >> 32));
        C.cm = (((uint64_t)hi << 32) | lo) & valid;
    } else {
        C.cm = valid;
    }
    return true;
}
// the k-th next live job (1 <= k <= 64, window index; P.w once the window has none left)
__device__ __forceinline__ bool mw_skip_live(const MwTiles& T, const CompPlan& P, MwCursor& C,
                                             int& ready, MwShared* S, int k, int& tj) {
    for (;;) {  // uniform; a tile holds ~7 records of each helper, so this rarely loops
        const int pc = __builtin_popcountll(C.cm);
        if (pc >= k) break;
        if ((C.ct + 1) * SCAN_JOBS >= P.w) {
            C.cm = 0ull;
            tj = P.w;
            return true;
        }
        k -= pc;
        if (!mw_cursor_tile(T, P, C, ready, S)) return false;
    }
    for (int j = 1; j < k; ++j) C.cm &= C.cm - 1ull;
    tj = C.ct * SCAN_JOBS + (int)__builtin_ctzll(C.cm);
    C.cm &= C.cm - 1ull;
    return true;
}

// The tile hand-off copied into SGPRs: mw_helper receives it in private memory (a by-value
// aggregate of an out-of-line callee), and every field read from there is a scratch load whose
// vmcnt wait would drain the helper's prefetched job stream.
template <class Q>
__device__ __forceinline__ Q* rfl_ptr(Q* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    return (Q*)(uintptr_t)(((uint64_t)(uint32_t)rfl((int32_t)(v >> 32)) << 32) |
                           (uint32_t)rfl((int32_t)(uint32_t)v));
}
__device__ __forceinline__ MwTiles tiles_sgpr(const MwTiles& T) {
    return MwTiles{rfl_ptr(T.tdone), (unsigned)rfl((int32_t)T.need), rfl_ptr(T.ring),
                   rfl_ptr(T.ctl), (unsigned)rfl((int32_t)T.round), (unsigned)rfl((int32_t)T.comp),
                   (unsigned)rfl((int32_t)T.ntj), rfl_ptr(T.feas)};
}

// ------------------------------------------------------------------------------- helper
// Helper entry lists: MW_EPL clean candidates + UPL dirty rows per lane, each key tagged with
// its entry index in the low bits (positions < 2^29, FIT_MAX_NODES), INF stays INF.
constexpr int UPL_MW = UCAP / 64;
constexpr int MW_NE = MW_EPL + UPL_MW;
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
// ascending sort of a lane's entries (static indices only): the optimal networks for 4 (5
// comparators) and 6 (12), odd-even transposition otherwise
template <int N>
__device__ __forceinline__ void mw_sort(uint64_t (&q)[N]) {
    if constexpr (N == 4) {
        mw_cas(q[0], q[1]); mw_cas(q[2], q[3]);
        mw_cas(q[0], q[2]); mw_cas(q[1], q[3]);
        mw_cas(q[1], q[2]);
    } else if constexpr (N == 6) {
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

// Extraction of the record's items: the nmax_ smallest tagged entries, one wave minimum each.
// straight-line: each minimum lands in every lane (DPP row minima, then the permlane16 / 32
// swaps of gfx950), so no VALU -> SGPR -> SALU hand-off sits on the helper's chain; the rounds
// stop at nmax_ (a uniform branch: round 4, C3 26.39 -> 26.02 ms, C2 14.95 -> 14.75 ms — a shorter
// helper record leaves the decider's SIMD and the LDS to the decider sooner); rounds past the last
// entry take nothing (stopping there too was slower)
__device__ __forceinline__ uint32_t wave_min32_all(uint32_t v) {
    v = dpp_min32<0xb1>(v);
    v = dpp_min32<0x4e>(v);
    v = dpp_min32<0x141>(v);
    v = dpp_min32<0x140>(v);  // every lane: its row's minimum
    {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = min((uint32_t)p[0], (uint32_t)p[1]);
    }
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return min((uint32_t)p[0], (uint32_t)p[1]);
}
#define MW_EXTRACT                                                                             \
        _Pragma("unroll") for (int i_ = 0; i_ < MW_M; ++i_) {                                  \
            if (i_ >= nmax_) break; /* uniform: a record needs nmax_ items at most */          \
            const uint32_t hh_ = (uint32_t)(q_[0] >> 32), ll_ = (uint32_t)q_[0];              \
            const uint32_t mh_ = wave_min32_all(hh_);                                          \
            const uint32_t ml_ = wave_min32_all(hh_ == mh_ ? ll_ : 0xffffffffu);               \
            const bool take_ = i_ < nmax_ && (mh_ & ml_) != 0xffffffffu;                       \
            const bool me_ = take_ && hh_ == mh_ && ll_ == ml_; /* tagged keys are unique */   \
            n_ += take_ ? 1 : 0;                                                               \
            sel_ = me_ ? sel_ | ((uint32_t)(i_ + 1) << (4u * (ml_ & 7u))) : sel_;              \
            _Pragma("unroll") for (int e = 0; e + 1 < MW_NE; ++e)                              \
                q_[e] = me_ ? q_[e + 1] : q_[e];                                               \
            q_[MW_NE - 1] = me_ ? KEY_INF : q_[MW_NE - 1];                                     \
        }                                                                                      \
        n_ = rfl(n_);

// Helper h (1..MW_H) pre-resolves records i = h-1, h-1+H, ... (record i: the i-th live job of the
// window, tj[] its window index).  Loads run two records ahead (keys, job row, bound) and one
// record ahead (the node rows of the candidates); the three register sets are indexed by literal
// constants only (3-way unrolled loop).
#define MW_HSTEP(A, B_, C)                                                                     \
    {                                                                                          \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) { /* record i+H's candidates' rows */\
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
            MW_CLK(tw0_);                                                                      \
            int tn_;                                                                           \
            if (!mw_skip_live(T, P, cur, ready, S, MW_H, tn_)) goto hdone;                     \
            tj[C] = tn_;                                                                       \
            const int tt_ = min(tn_, wlast) + z;                                               \
            if (!mw_tile_ready(T, tt_, ready, S)) goto hdone;                                  \
            {                                                                                  \
                MW_CLK(tw1_);                                                                  \
                MW_ACC(a_ht, tw1_ - tw0_);                                                     \
            }                                                                                  \
            _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e)                                  \
                kk[C][e] = has[e] ? ld_through(cand + eoff[e] + (int64_t)tt_ * E) : KEY_INF;   \
            jr[C] = ld_job_through(wjob + P.slot0 + tt_);                                      \
            jbd[C] = ld_through(bnd + P.slot0 + tt_);                                          \
        }                                                                                      \
        /* snapshot: the decider has resolved at least i - (MW_M - 1) records (and so has read  \
           record slot i & 7's previous one) */                                                \
        uint64_t dn_;                                                                          \
        MW_CLK(hw0_);                                                                          \
        for (unsigned sp_ = 0;; ++sp_) {                                                       \
            dn_ = __hip_atomic_load(&S->dn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   \
            const int lag_ = i - (MW_SNAP - 1) - rfl((int32_t)(uint32_t)dn_);                  \
            if (lag_ <= 0) break;                                                              \
            if ((sp_ & 7u) == 7u && (lds_ld(&S->halt) | lds_ld(&S->fail))) goto hdone;         \
            if (sp_ > MW_SPIN_LIMIT) {                                                         \
                lds_st(&S->fail, TRIP_HELPER_SNAP);                                            \
                goto hdone;                                                                    \
            }                                                                                  \
            /* the decider needs ~1k cycles a job: sleep about that long per missing job      \
               instead of polling (every poll is an LDS access the decider queues behind) */   \
            for (int s_ = min(lag_, 8); s_ > 0; --s_) __builtin_amdgcn_s_sleep(MW_HSLEEP);     \
        }                                                                                      \
        lds_acquire(); /* the rows / bitmap the decider released with dn_ */                   \
        const uint32_t v_ = (uint32_t)rfl((int32_t)(uint32_t)dn_);                             \
        const int nu_ = rfl((int32_t)(uint32_t)(dn_ >> 32));                                   \
        MwRec* R_ = &S->rec[i & (MW_R - 1)];                                                   \
        if (tj[A] >= P.w) { /* no live job left: the end record (B = 0, nothing fits) */       \
            if (lane == 0) {                                                                   \
                *reinterpret_cast<v4i32*>(&R_->h.cpu) = v4i32{0, 0, 0, 0};                     \
                *reinterpret_cast<uint4*>(&R_->h.pbit) = make_uint4(0u, (uint32_t)P.w, 0u, 0u);\
                R_->h.v = (int32_t)v_;                                                         \
                R_->h.n = 0;                                                                   \
                R_->h.q = -1;                                                                  \
                lds_release();                                                                 \
                lds_st(&R_->h.ready, (uint32_t)i + 1u);                                        \
            }                                                                                  \
            goto hdone;                                                                        \
        }                                                                                      \
        {                                                                                      \
            MW_CLK(hw1_);                                                                      \
            MW_ACC(a_hw, hw1_ - hw0_);                                                         \
            MW_ACC(a_hp, -(long long)hw1_);                                                    \
            MW_ACC(a_hx, -(long long)hw1_);                                                    \
        }                                                                                      \
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
        uint64_t xd[UPL_MW];                                                                   \
        MwRow wr_[UPL_MW];                                                                     \
        _Pragma("unroll") for (int u = 0; u < UPL_MW; ++u) {                                   \
            xd[u] = KEY_INF;                                                                   \
            wr_[u] = MwRow{0, 0, 0, 0, 0u, 0u, 0, 0};                                          \
            const int u_ = u * 64 + lane;                                                      \
            if (u * 64 < nu_) { /* uniform: rows [0, nu) exist */                              \
                wr_[u] = S->rows[u_ < nu_ ? u_ : 0];                                           \
                const uint64_t y_ = mw_key(wr_[u].cpu, wr_[u].mem, wr_[u].gpu, wr_[u].avail,   \
                                           wr_[u].mask, wr_[u].pos, J_.cpu, J_.mem, J_.gpu,    \
                                           J_.wall, J_.pbit);                                  \
                xd[u] = u_ < nu_ && y_ <= Bd_ ? y_ : KEY_INF;                                  \
            }                                                                                  \
        }                                                                                      \
        int n_ = 0;                                                                            \
        {                                                                                      \
            MW_CLK(hx_);                                                                       \
            MW_ACC(a_hx, hx_);                                                                 \
        }                                                                                      \
        /* every entry tagged with its index (pos << 3 | e keeps the order of distinct nodes) and\
           sorted per lane once; each extraction is then one wave minimum over the lane heads  \
           plus a predicated shift in the winning lane */                                      \
        uint64_t q_[MW_NE];                                                                    \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) q_[e] = mw_tag(x0[e], e);           \
        _Pragma("unroll") for (int u = 0; u < UPL_MW; ++u) q_[MW_EPL + u] = mw_tag(xd[u], MW_EPL + u);\
        mw_sort(q_);                                                                           \
        /* item index + 1 of each entry, 4 bits per entry (0: not taken) */                     \
        uint32_t sel_ = 0u;                                                                    \
        /* at most i - v nodes can change before record i is decided: i - v + 1 items suffice */\
        const int nmax_ = min(MW_M, i - (int)v_ + 1);                                          \
        MW_EXTRACT                                                                             \
        /* items: the lanes that gave an entry store it (exec-masked: only those lanes use   \
           the LDS, which the decider shares) */                                               \
        _Pragma("unroll") for (int e = 0; e < MW_EPL; ++e) {                                   \
            const uint32_t ix_ = (sel_ >> (4 * e)) & 15u;                                      \
            if (ix_)                                                                           \
                R_->it[ix_ - 1u] = MwItem{(uint32_t)x0[e], (uint32_t)(x0[e] >> 32), -1,        \
                                          ro[A][e], rc[A][e], rm[A][e], rg[A][e], ra[A][e],    \
                                          rk[A][e], 0u, 0u, 0u};                               \
        }                                                                                      \
        _Pragma("unroll") for (int u = 0; u < UPL_MW; ++u) {                                   \
            const uint32_t ix_ = (sel_ >> (4 * (MW_EPL + u))) & 15u;                           \
            if (ix_)                                                                           \
                R_->it[ix_ - 1u] = MwItem{(uint32_t)xd[u], (uint32_t)(xd[u] >> 32),            \
                                          u * 64 + lane, wr_[u].orig, wr_[u].cpu, wr_[u].mem,  \
                                          wr_[u].gpu, wr_[u].avail, wr_[u].mask, 0u, 0u, 0u};  \
        }                                                                                      \
        if (lane == 0) {                                                                       \
            *reinterpret_cast<v4i32*>(&R_->h.cpu) = v4i32{J_.cpu, J_.mem, J_.gpu, J_.wall};    \
            *reinterpret_cast<uint4*>(&R_->h.pbit) =                                           \
                make_uint4(J_.pbit, (uint32_t)tj[A], (uint32_t)Bd_, (uint32_t)(Bd_ >> 32));    \
            R_->h.v = (int32_t)v_;                                                             \
            R_->h.n = n_;                                                                      \
            R_->h.q = J_.q;                                                                    \
            lds_release(); /* items and header before the ready word */                        \
            lds_st(&R_->h.ready, (uint32_t)i + 1u);                                            \
        }                                                                                      \
        {                                                                                      \
            MW_CLK(hp1_);                                                                      \
            MW_ACC(a_hp, hp1_);                                                                \
        }                                                                                      \
        MW_ACC(a_hn, 1);                                                                       \
        MW_ACC(a_hi, n_);                                                                      \
        i += MW_H;                                                                             \
    }

__device__ __noinline__ void mw_helper(const CompPlan& Pref, MwShared* Sin,
                                       const NodeRec* __restrict__ rec_,
                                       const uint64_t* __restrict__ cand_,
                                       const uint64_t* __restrict__ bnd_,
                                       const JobRec* __restrict__ wjob_, int h, MwTiles Tin) {
    const MwTiles T = tiles_sgpr(Tin);
    const GAS NodeRec* const rec = gview(rec_);
    const GAS uint64_t* const cand = gview(cand_);
    const GAS uint64_t* const bnd = gview(bnd_);
    const GAS JobRec* const wjob = gview(wjob_);
    // by value: a reference into the caller's stack is re-read (flat load + full vmcnt wait) after
    // every LDS store, which would drain the job-stream prefetch each step
    const CompPlan P = plan_sgpr(Pref);
    MwShared* const S = lds_opaque(Sin);
    const int lane = threadIdx.x & 63;
    const int E = P.nslice * P.ks;
    bool has[MW_EPL];       // candidate entry lane + 64 e of the job's E entries
    int64_t eoff[MW_EPL];
#pragma unroll
    for (int e = 0; e < MW_EPL; ++e) {
        has[e] = lane + 64 * e < E;
        eoff[e] = P.cand_off + (has[e] ? lane + 64 * e : 0);
    }
    const int wlast = P.w - 1;
    const int z = opaque_zero();
    const int hh = rfl(h);  // uniform (h arrives in a VGPR: the callee is out of line)
    int i = hh - 1;         // record index

    uint64_t kk[3][MW_EPL], jbd[3];
    JobRec jr[3];
    int32_t rc[3][MW_EPL], rm[3][MW_EPL], rg[3][MW_EPL], ra[3][MW_EPL], ro[3][MW_EPL];
    uint32_t rk[3][MW_EPL];
    int tj[3];      // window index of the job of each register set (P.w: past the last live job)
    int ready = 0;  // scan tiles known complete
    MwCursor cur{-1, 0ull};
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // records i and i + H
        if (!mw_skip_live(T, P, cur, ready, S, s == 0 ? hh : MW_H, tj[s])) return;
        const int tt = min(tj[s], wlast) + z;
        if (!mw_tile_ready(T, tt, ready, S)) return;  // halted / watchdog
#pragma unroll
        for (int e = 0; e < MW_EPL; ++e)
            kk[s][e] = has[e] ? ld_through(cand + eoff[e] + (int64_t)tt * E) : KEY_INF;
        jr[s] = ld_job_through(wjob + P.slot0 + tt);
        jbd[s] = ld_through(bnd + P.slot0 + tt);
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
    MW_DECL(a_ht);  // waiting for scan tiles (prefetch of record i + 2H)
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
// One wave; lanes 0..7 carry the "written ring" (the decisions of the last 8 jobs: job t's entry
// in lane t & 7 — its node's position and row as that job left it, its dirty slot, the job) and
// record t's items (lane i: item i).  A ring entry is live for job t iff its job >= the record's
// snapshot v; when a node is written again its older entry dies, so a live entry always holds
// the node's current row.
struct MwRing {
    v4i32 a;       // cpu, mem, gpu, avail   (= MwRow's first 16 B)
    v4i32 b;       // mask, pos, orig, job   (= MwRow's last 16 B; job -1: dead)
    int32_t slot;  // dirty slot
};

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
struct MwRecRegs {  // one record as this lane sees it: header (every lane) and item lane & 7
    v4u32 h0, h1, h2;  // {ready, v, n, q}, {cpu, mem, gpu, wall}, {pbit, -, B lo, B hi}
    v4u32 i0, i1;      // {pos, score, tag, orig}, {cpu, mem, gpu, avail}
    uint32_t i2;       // mask
};

struct MwDec {
    int t, nu, placed, stop;  // t: records decided (live jobs)
    int done;                 // window jobs resolved when the walk ended (its stop / end record)
    bool exit;  // the window is finished (end, stop or watchdog): later steps change nothing
#ifdef MW_SEGSTAMP
    unsigned long long seg[8], prev;
#endif
};
// diagnostic (decbench only): cycles per segment of a decider step, s_memtime at each point
#ifdef MW_SEGSTAMP
__device__ unsigned long long g_seg[8];
#define MW_SEG(D_, i)                                                                           \
    do {                                                                                        \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        unsigned long long now_;                                                                \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now_)::"memory");            \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        if (i > 0) D_.seg[i] += now_ - D_.prev;                                                 \
        D_.prev = now_;                                                                         \
    } while (0)
#else
#define MW_SEG(D_, i)
#endif

__device__ __forceinline__ const __attribute__((address_space(3))) v4u32* lds4(const void* p) {
    return (const __attribute__((address_space(3))) v4u32*)(uintptr_t)p;
}
__device__ __forceinline__ void mw_read_rec(const MwRec* R, int i8, MwRecRegs& x) {
    const __attribute__((address_space(3))) v4u32* hp = lds4(&R->h);
    const __attribute__((address_space(3))) v4u32* ip = lds4(&R->it[i8]);
    x.h0 = hp[0];
    x.h1 = hp[1];
    x.h2 = hp[2];
    x.i0 = ip[0];
    x.i1 = ip[1];
    x.i2 = ((const __attribute__((address_space(3))) uint32_t*)ip)[8];
}

// One job of the decider: job D.t with record `cur` (its data read after an acquire of the ready
// word `flag`; refreshed in place on the slow path), `nxt` receives record t+1.  E = t & 7 is a
// compile-time constant.  Straight-line: the decision is computed unconditionally and selected (no
// exec-masked region), its bookkeeping is masked with `go` instead of branched around, and the
// only branch is the rare exception (record not ready, B exceeded, dirty set full).  Once D.exit
// is set the step has no effect: the caller tests it once per 8 jobs.
template <int E>
__device__ __forceinline__ void mw_decide(MwShared* S, const CompPlan& P, MwDec& D, MwRing& R,
                                          MwRecRegs& cur, MwRecRegs& nxt, uint32_t& flag,
                                          int32_t& oq, int32_t& ov, int32_t* out, int kmax,
                                          uint64_t& waitcyc) {
    const int lane = threadIdx.x & 63;
    const int t = D.t;
#ifdef MW_DECIDER_BENCH
    if (t >= P.w) D.exit = true;  // pre-filled records: no end record
#endif
    MW_SEG(D, 0);
    // publish the decisions so far (the previous job's row / bitmap writes were issued before
    // record t's reads, all of which are complete here): release store of {decided, nu}
    lds_release();
    __hip_atomic_store(&S->dn, ((uint64_t)(uint32_t)D.nu << 32) | (uint32_t)t, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    // ready word of record t+1 (relaxed; acquired below, before its data is read)
    // t == E (mod 8) while the window runs (each window starts at t = 0 and every step before an
    // exit advances t by one; after an exit the record read below is never used)
    const MwRec* Rn = &S->rec[(E + 1) & (MW_R - 1)];
    const uint32_t flag_n = lds_ld(&Rn->h.ready);
    MW_SEG(D, 1);

    // the decision of job t against record `x`
    struct Dec {
        uint64_t bs;  // best key (uniform)
        int32_t sc, sm, sg, sa, sk, so, ss;  // per lane: its candidate's row, demand subtracted
        int w, wslot;
        bool placed, fresh, stopB, full;
    };
    auto decide = [&](const MwRecRegs& x) {
        Dec d;
        const int32_t v = (int32_t)x.h0.y, n = (int32_t)x.h0.z;
        const int32_t jc = (int32_t)x.h1.x, jm = (int32_t)x.h1.y, jg = (int32_t)x.h1.z,
                      jw = (int32_t)x.h1.w;
        const uint32_t jp = x.h2.x;
        const uint64_t B = ((uint64_t)x.h2.w << 32) | x.h2.z;
        // live ring rows at their current state
        const bool live = R.b.w >= v;
        const uint64_t rk0 = mw_key(R.a.x, R.a.y, R.a.z, R.a.w, (uint32_t)R.b.x, (uint32_t)R.b.y,
                                    jc, jm, jg, jw, jp);
        const uint64_t rkey = live ? rk0 : KEY_INF;
        const uint32_t ip = x.i0.x;
        // item staleness: its node is in the live ring.  Lanes 8..15 take a copy of the ring
        // (row_ror:8), so row_ror:k, k = 0..7, shows lane i < 8 every ring entry once.
        const uint32_t P0 = live ? (uint32_t)R.b.y : 0xffffffffu;  // positions are < 2^29
        const uint32_t P8 = dpp32<0x128>(P0);
        const uint32_t P2 = (lane & 8) ? P8 : P0;
        const uint32_t d0 = ip ^ P2, d1 = dpp_ror_xor<1, true>(P2, ip),
                       d2 = dpp_ror_xor<2, false>(P2, ip), d3 = dpp_ror_xor<3, false>(P2, ip),
                       d4 = dpp_ror_xor<4, false>(P2, ip), d5 = dpp_ror_xor<5, false>(P2, ip),
                       d6 = dpp_ror_xor<6, false>(P2, ip), d7 = dpp_ror_xor<7, false>(P2, ip);
        const bool stale = min(min(min(d0, d1), min(d2, d3)), min(min(d4, d5), min(d6, d7))) == 0u;
        const uint64_t ik0 = ((uint64_t)x.i0.y << 32) | ip;
        const uint64_t ikey = (lane < n && !stale) ? ik0 : KEY_INF;
        const bool tr = rkey < ikey;  // this lane's ring row beats its item
        const uint64_t cand = tr ? rkey : ikey;
        // the winner's fields, demand already subtracted (selected per lane, read from one)
        d.sc = (tr ? R.a.x : (int32_t)x.i1.x) - jc;
        d.sm = (tr ? R.a.y : (int32_t)x.i1.y) - jm;
        d.sg = (tr ? R.a.z : (int32_t)x.i1.z) - jg;
        d.sa = tr ? R.a.w : (int32_t)x.i1.w;
        d.sk = tr ? R.b.x : (int32_t)x.i2;
        d.so = tr ? R.b.z : (int32_t)x.i0.w;
        d.ss = tr ? R.slot : (int32_t)x.i0.z;
        const uint64_t best = min8_2pass(cand);
        // lanes 0..7 all hold `best`; the winner is the lane whose candidate equals it
        const uint64_t mine = __ballot(cand == best) & 0xffull;
        d.w = __builtin_ctzll(mine | 0x100ull) & 7;
        const uint32_t bhi = (uint32_t)readlane((int32_t)(best >> 32), 0);
        const uint32_t blo = (uint32_t)readlane((int32_t)(uint32_t)best, 0);
        d.bs = ((uint64_t)bhi << 32) | blo;
        d.placed = d.bs != KEY_INF;
        d.wslot = readlane(d.ss, d.w);
        d.fresh = d.placed && d.wslot < 0;
        d.full = d.fresh && D.nu >= UCAP;
        d.stopB = B != KEY_INF && d.bs > B;
        return d;
    };
    Dec d = decide(cur);
    MW_SEG(D, 2);
#ifdef MW_DECIDER_BENCH
    const bool rec_missing = false;  // diagnostic: records pre-filled, never "not ready"
#else
    const bool rec_missing = flag != (uint32_t)t + 1u;
#endif
    if (__builtin_expect(!D.exit && (rec_missing || d.stopB || d.full), 0)) {  // the one branch
        if (rec_missing) {  // record t not complete when read: wait for it, read it again
            MW_CLK(c0);
            for (unsigned sp = 0;; ++sp) {
                flag = lds_ld(&S->rec[t & (MW_R - 1)].h.ready);
                if (flag == (uint32_t)t + 1u) break;
                if (sp > MW_SPIN_LIMIT || lds_ld(&S->fail)) {
                    lds_st(&S->fail, TRIP_DECIDER_REC);
                    D.stop = 3;
                    D.exit = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(0);
            }
            lds_acquire();
            mw_read_rec(&S->rec[t & (MW_R - 1)], lane & 7, cur);
            {
                MW_CLK(c1);
                MW_ACC(waitcyc, c1 - c0);
            }
            d = decide(cur);
        }
        if (!D.exit && (d.stopB || d.full)) {
            // the end record (no live job left: B = 0, nothing fits) or a stop at the record's
            // job: candidate list exhausted (rescan) / dirty set full
            D.done = (int32_t)cur.h2.y;
            if (D.done < P.w) D.stop = d.stopB ? 1 : 2;
            D.exit = true;
        }
    }
    // ---- apply job t (masked by `go`; the ring is not read again once D.exit is set) ----------
    MW_SEG(D, 3);
    const bool go = !D.exit;
    const bool placed = d.placed && go, fresh = d.fresh && go;
    const int w = d.w;
    const int32_t pos = (int32_t)(uint32_t)d.bs;
    const int32_t nc = readlane(d.sc, w), nm = readlane(d.sm, w), ng = readlane(d.sg, w);
    const int32_t na = readlane(d.sa, w), nk = readlane(d.sk, w), no = readlane(d.so, w);
    const int32_t slot = fresh ? D.nu : d.wslot;
    // an older ring entry of the same node dies (lane E is rewritten below)
    R.b.w = (placed && R.b.y == pos) ? -1 : R.b.w;
    R.a.x = writelane_c<E>(nc, R.a.x);
    R.a.y = writelane_c<E>(nm, R.a.y);
    R.a.z = writelane_c<E>(ng, R.a.z);
    R.a.w = writelane_c<E>(na, R.a.w);
    R.b.x = writelane_c<E>(nk, R.b.x);
    R.b.y = writelane_c<E>(pos, R.b.y);
    R.b.z = writelane_c<E>(no, R.b.z);
    R.b.w = writelane_c<E>(placed ? t : -1, R.b.w);
    R.slot = writelane_c<E>(slot, R.slot);
    MW_SEG(D, 4);
    // read record t+1's data after acquiring its ready word (the load above is long done)
    flag = flag_n;
    lds_acquire();
    mw_read_rec(Rn, lane & 7, nxt);
    MW_SEG(D, 5);
    // bookkeeping: dirty row, bitmap bit — fire-and-forget LDS writes, no branch: lane E alone
    // (exec = its bit, or none when the job is not placed) stores the new row and ORs the bitmap
    // bit (0 when the node was already dirty): 3 LDS ops of one lane instead of 64 lanes' worth of
    // traffic in the LDS pipe the helpers share
    {
        typedef __attribute__((address_space(3))) MwRow* LRow;
        const uint32_t ra = (uint32_t)(uintptr_t)(LRow)&S->rows[slot];
        const uint32_t rel = (uint32_t)pos - (uint32_t)P.nb;
        const uint32_t ba = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)&S->bitmap[rel >> 5];
        const uint32_t bv = fresh ? 1u << (rel & 31) : 0u;
        const uint32_t pl = (uint32_t)rfl(placed ? 1 : 0);
        const uint64_t m = ((uint64_t)(uint32_t)rfl((int32_t)(pl << E)) |
                            ((uint64_t)(uint32_t)rfl(0) << 32));  // exec mask: SGPR pair
        uint64_t sv;
        asm volatile(
            "s_mov_b64 %[sv], exec\n\t"
            "s_mov_b64 exec, %[m]\n\t"
            "ds_write_b128 %[ra], %[a]\n\t"
            "ds_write_b128 %[ra], %[b] offset:16\n\t"
            "ds_or_b32 %[ba], %[bv]\n\t"
            "s_mov_b64 exec, %[sv]"
            : [sv] "=&s"(sv)
            : [m] "s"(m), [ra] "v"(ra), [a] "v"(R.a), [b] "v"(R.b), [ba] "v"(ba), [bv] "v"(bv)
            : "memory");
    }
    D.nu += fresh;
    D.placed += placed;
    MW_SEG(D, 6);
    // placement of job t parked in lane t & 63 (after an exit that lane is past the last store)
    oq = writelane(rfl((int32_t)cur.h0.w), t & 63, oq);
    ov = writelane(placed ? no : -1, t & 63, ov);
    if (E == 7 && go && (t & 63) == 63) {  // uniform, once per 64 jobs: store 64 placements
        if (oq >= 0) ((GAS int32_t*)out)[(int64_t)oq * kmax] = ov;
        oq = -1;
    }
    D.t = t + (go ? 1 : 0);
    MW_SEG(D, 7);
}

// Out of line (as is mw_helper): called once per round, each gets its own register allocation
// instead of sharing the persistent kernel's (which otherwise spills SGPRs in this loop).
__device__ __noinline__ CommitResult mw_decider(const CompPlan& Pref, MwShared* Sin,
                                                int32_t* __restrict__ out, int kmax) {
    const CompPlan P = plan_sgpr(Pref);  // by value (see mw_helper)
    MwShared* const S = lds_opaque(Sin);
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_s_setprio(3);  // shares its SIMD with a helper wave
    MwDec D{0, 0, 0, 0, 0, false};
#ifdef MW_SEGSTAMP
    for (int i = 0; i < 8; ++i) D.seg[i] = 0;
    D.prev = 0;
#endif
    MwRing R;
    R.a = v4i32{0, 0, 0, 0};
    R.b = v4i32{0, -1, -1, -1};  // dead, position matching no item
    R.slot = -1;
    int32_t oq = -1, ov = -1;  // placement of job t parked in lane t & 63, stored 64 at a time
    uint64_t waitcyc = 0;
    MW_CLK(d0);
    // record 0: wait for its ready word, acquire, read
    MwRecRegs ra, rb;
    uint32_t flag = 0;
    if (P.w > 0) {
        for (unsigned sp = 0;; ++sp) {
            flag = lds_ld(&S->rec[0].h.ready);
#ifdef MW_DECIDER_BENCH
            break;
#endif
            if (flag == 1u) break;
            if (sp > MW_SPIN_LIMIT || lds_ld(&S->fail)) {
                lds_st(&S->fail, TRIP_DECIDER_REC);
                D.stop = 3;
                D.exit = true;
                break;
            }
            __builtin_amdgcn_s_sleep(0);
        }
        lds_acquire();
        mw_read_rec(&S->rec[0], lane & 7, ra);
    } else {
        D.exit = true;
    }
    {
        MW_CLK(r0c);
        MW_ADD(17, r0c - d0);
        MW_ADD(18, 1);
    }
    // 8-way unrolled: the ring lane (t & 7) is a constant in every step; the two record register
    // sets alternate with the step's parity; the exit is tested once per 8 steps
    while (!D.exit) {
        mw_decide<0>(S, P, D, R, ra, rb, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<1>(S, P, D, R, rb, ra, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<2>(S, P, D, R, ra, rb, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<3>(S, P, D, R, rb, ra, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<4>(S, P, D, R, ra, rb, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<5>(S, P, D, R, rb, ra, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<6>(S, P, D, R, ra, rb, flag, oq, ov, out, kmax, waitcyc);
        mw_decide<7>(S, P, D, R, rb, ra, flag, oq, ov, out, kmax, waitcyc);
    }
    const int t = D.t;
    if (oq >= 0 && lane < (t & 63)) ((GAS int32_t*)out)[(int64_t)oq * kmax] = ov;  // last group
    // final {decided, nu}, then halt (the helpers' exit)
    lds_release();
    __hip_atomic_store(&S->dn, ((uint64_t)(uint32_t)D.nu << 32) | (uint32_t)t, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    lds_st(&S->halt, 1u);
    MW_CLK(d1);
    MW_ADD(0, d1 - d0);
#ifdef MW_SEGSTAMP
    if (lane == 0)
        for (int i = 0; i < 8; ++i) g_seg[i] = D.seg[i];
#endif
    MW_ADD(1, waitcyc);
    MW_ADD(2, t);
#ifdef MW_DECIDER_BENCH
    D.done = t;
#endif
    return CommitResult{D.done, D.stop, D.nu, D.placed};
}

// All MW_WAVES waves of the block call this; returns the same result in every wave.
__device__ __forceinline__ CommitResult commit_window_mw(const CompPlan& P, MwShared* S,
                                                         NodeRec* __restrict__ rec,
                                                         const uint64_t* __restrict__ cand,
                                                         const uint64_t* __restrict__ bnd,
                                                         const JobRec* __restrict__ wjob,
                                                         int32_t* __restrict__ out, int kmax,
                                                         MwTiles T = MwTiles{nullptr, 0u, nullptr, nullptr, 0u, 0u, 0u, nullptr}) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = threadIdx.x; i < nwords; i += MW_WAVES * 64) S->bitmap[i] = 0u;
    if (threadIdx.x < MW_R) S->rec[threadIdx.x].h.ready = 0u;
    if (threadIdx.x == 0) {
        S->dn = 0ull;
        S->halt = 0u;
        S->fail = 0u;
    }
    __syncthreads();
    if (wave == 0) {
        const CommitResult r = mw_decider(P, S, out, kmax);
        if (threadIdx.x == 0) {
            S->res[0] = r.done;
            S->res[1] = r.stop;
            S->res[2] = r.dirty;
            S->res[3] = r.placed;
        }
    } else {
        mw_helper(P, S, rec, cand, bnd, wjob, wave, T);  // waves 1.. : helpers 1..MW_H
    }
    __syncthreads();
    const CommitResult r{S->res[0], S->res[1], S->res[2], S->res[3]};
    // write the dirty rows back for the next round's scan, through (sc1: the next round's
    // publish needs no release fence for them; {cpu, mem} as one 8-B word, then gpu)
    for (int u = threadIdx.x; u < r.dirty; u += MW_WAVES * 64) {
        const MwRow w = S->rows[u];
        NodeRec* d = rec + w.pos;
        __hip_atomic_store(reinterpret_cast<uint64_t*>(&d->cpu),
                           (uint64_t)(uint32_t)w.cpu | ((uint64_t)(uint32_t)w.mem << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&d->gpu, w.gpu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
    __syncthreads();
    return r;
}

}  // namespace fitgpu
