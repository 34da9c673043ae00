// fit_persistent.hip — the whole placement in ONE launch.
//
// Blocks [0, C) are committers: wave 0 of block c owns partition component c; it publishes each
// round's scan tiles into a device task ring, waits for its per-component done counter, then
// runs commit_window (fit_common.h) on the results.  Blocks [C, C+W) are scan workers: they
// claim tiles from the ring in order and run scan_tile.  Components therefore advance at their
// own pace — no host round trip and no global round barrier — while the scan work of all of
// them shares the whole chip.
//
// Cross-workgroup hand-offs follow cdna_hip_programming.md §6 Guideline 16 (placement-
// independent, agent scope):
//   producer: plain stores → every storing wave `s_waitcnt vmcnt(0)` → barrier → one lane
//             release fence → `s_waitcnt vmcnt(0)` → relaxed agent atomic (counter / granule)
//   consumer: relaxed agent poll → ONE acquire fence → `s_waitcnt vmcnt(0)` (→ barrier) → plain
//             loads; plus `s_dcache_inv` because node rows, plans and job rows are read through
//             the scalar cache, which an acquire fence does not invalidate.
// Every spin is bounded; a watchdog trip sets ctl->error and drains every block.
#include <algorithm>

#include "fit_commit_mw.h"
#include "fit_engine_ctl.h"

namespace fitgpu {

// Windows holding a multi-node job: the single-wave commit (fit_common.h), kept out of line so
// its registers are allocated apart from the decider / helper / worker loops.
__device__ __noinline__ CommitResult engine_commit_single(int c, const CompPlan P, NodeRec* rec,
                                                          const uint64_t* cand,
                                                          const uint64_t* bnd, const JobRec* wjob,
                                                          int32_t* out, int kmax,
                                                          uint32_t* bitmap, uint32_t* scratch) {
    // the bitmap's LDS address as an opaque SGPR value: seen through, the compiler re-derives it
    // from the dynamic-LDS offset table at every access (a scalar load + lgkmcnt(0) wait each);
    // the arrays as global pointers (commit_window: no flat accesses)
    typedef __attribute__((address_space(3))) uint32_t* LdsWords;
    uint32_t a = (uint32_t)(uintptr_t)(LdsWords)bitmap;
    asm volatile("" : "+s"(a));
#ifdef __HIP_DEVICE_COMPILE__
#define FIT_GLOBAL(T, p) ((__attribute__((address_space(1))) T*)(p))
#else  // (the host pass only parses device code)
#define FIT_GLOBAL(T, p) ((T*)(p))
#endif
    uint32_t sa = (uint32_t)(uintptr_t)(LdsWords)scratch;  // 256 B of LDS the helpers do not use here
    asm volatile("" : "+s"(sa));
    return commit_window<MW_EPL, true>(c, P, FIT_GLOBAL(NodeRec, rec), FIT_GLOBAL(const uint64_t, cand), 0,
                                       1, FIT_GLOBAL(const uint64_t, bnd), FIT_GLOBAL(const JobRec, wjob),
                                       FIT_GLOBAL(int32_t, out), kmax, (LdsWords)(uintptr_t)a, sa);
#undef FIT_GLOBAL
}

#ifndef FIT_K0
#define FIT_K0 4  // > 0: a round's first job tile keeps FIT_K0 keys per block-slice (scan_tile KW)
#endif
#ifndef FIT_K0W
#define FIT_K0W 8  // > 0: the first job tile after a rescan inside the previous round's first tile keeps
                   // FIT_K0W keys per block-slice, unpaired, for K0W_ROUNDS rounds ("wide"): runs of
                   // identical jobs (array tasks) drain the FIT_K0 lists' bound within a few jobs
#endif
#ifndef K0W_ROUNDS
#define K0W_ROUNDS 8
#endif
#ifndef K_T0PAIR4
#define K_T0PAIR4 1  // ... also a 4-key component's (C3o: one 100k-node component, 32 slices x 4 keys)
#endif
#ifndef K_T0PAIR
#define K_T0PAIR 1  // k_engine: a k = 1 window's first job tile as 2 x nslice half-size block-slices, paired
#endif
// A round's first job tile stages its block-slice's node rows in LDS behind the merge buffer and
// the task slot (scan_tile STAGE) when they fit: SCAN_WAVES * P.sub <= STAGE_ROWS (C3: 8 x 98).
constexpr size_t STAGE_OFF = (sizeof(uint64_t) * (SCAN_WAVES / 2) * KS * 64 + 16 + 63) & ~(size_t)63;
constexpr int STAGE_ROWS = 1024;

__global__ __launch_bounds__(SCAN_WAVES * 64) void k_engine(
    EngineCtl* __restrict__ ctl, unsigned long long* __restrict__ ring,
    const CompState* __restrict__ cs, CompOut* __restrict__ co, CompPlan* __restrict__ plans,
    int ncomp, NodeRec* __restrict__ rec, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, const uint16_t* __restrict__ jk,
    uint64_t* __restrict__ cand, uint64_t* __restrict__ bnd, JobRec* __restrict__ wjob,
    int32_t* __restrict__ out, int kmax, int64_t* __restrict__ wbusy,
    const int32_t* __restrict__ jpk, unsigned wd) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) stamp_start(ctl);

    if ((int)blockIdx.x < ncomp) {
        // ================================================================== committer
        // Wave 0 runs the round protocol (publish tiles, wait, acquire); then all 8 waves commit
        // the window together: wave 0 decides, waves 1..7 pre-resolve (fit_commit_mw.h).
        __shared__ int s_fail;
        const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const int c = blockIdx.x;
        const CompState S = cs[c];
        MwShared* M = reinterpret_cast<MwShared*>(smem);
        if (threadIdx.x == 0) M->wd = wd;  // the commit waits' deadline (fit_commit_mw.h)
        int32_t cursor = S.jstart, win = S.wmin;
        unsigned target[2] = {0u, 0u};  // tiles published by the rounds of each parity
        // job tiles published by the last round of each parity: only their bounds can differ from
        // KEY_INF (the host sets them all before the launch), so only those are reset
        unsigned used[2] = {0u, 0u};
        int64_t evals = 0, placed = 0, rounds = 0, sr = 0, sd = 0, tc = 0, tw = 0;
        bool prev_multi = false;  // the previous round ran the single-wave commit (plain row stores)
        int wide_left = 0;        // rounds left whose first tile is wide (FIT_K0W)
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
            int64_t t0 = 0;
            // a window holding a multi-node job is committed by wave 0 alone (commit_window
            // handles k > 1) after its whole scan; the decider/helper pipeline covers k = 1
            // windows and starts at once: helpers wait per job tile (MwTiles)
            const bool multi = jpk[cursor + w] != jpk[cursor];
            // a multi-node job needs k <= KS keys in its first tile; a k = 1 window's first tile
            // keeps FIT_K0 keys per block-slice and is scanned as paired half-slices (K_T0PAIR)
            // (the pair scratch holds 4 keys: the FIT_K0 list, or a 4-key component's own, C3o)
            // — unless a recent round stopped for a rescan inside its first tile: then FIT_K0W keys
            // per block-slice, unpaired (bit 2; components with ks <= FIT_K0W keep their first tile)
            const bool wide = !multi && FIT_K0W > 0 && FIT_K0W < S.ks && wide_left > 0;
            const bool pair = !multi && !wide && K_T0PAIR && 2 * S.nslice <= 64 &&
                              ((FIT_K0 > 0 && FIT_K0 <= 4 && FIT_K0 < S.ks) || (K_T0PAIR4 && S.ks <= 4));
            P.k0 = multi ? 0 : wide ? 4 : (1 | (pair ? 2 : 0));
            P.pair_off = S.pair_off + (par ? PAIR_AREA : 0);
            MW_CLK(rs0);
            if (wave == 0) {
                t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
                // the tiles of the round before last (this round's buffer set; also those past its
                // stop) must all be complete before their buffers and counters are reused; the
                // previous round's may still be in flight, in the other set
                bool fail = !wait_tiles(ctl, c, par, target[par], wd, rnd);
                const unsigned ntj = (unsigned)((w + SCAN_JOBS - 1) / SCAN_JOBS);
                // written through (sc1), like the tile counters: the helpers that publish tiles
                // just in time need no release of their own (R1: stored, drained, then the
                // block barrier, then their task stores)
                store_through(&plans[2 * c + par], P);
                const int nres = min((int)used[par] * SCAN_JOBS, S.wmax);  // within the slot region
                for (int i = lane; i < nres; i += 64) store_through64(&bnd[P.slot0 + i], KEY_INF);
                for (unsigned i = lane; i < ntj; i += 64) {
                    __hip_atomic_store(&ctl->tdone[par][c][i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&ctl->tfeas[par][c][i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (pair && lane < 32)
                    __hip_atomic_store(&ctl->tpair[par][c][lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // node rows: the multi-wave commit writes them back through (commit_window_mw);
                // the single-wave commit of a multi-node window writes them plainly: release those
                if (prev_multi) release_agent();
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // just-in-time publishing (ENGINE_AHEAD > 0, k = 1 windows): the first
                // ENGINE_AHEAD job tiles now, the rest by the helpers as they reach them
                // (fit_commit_mw.h mw_publish), so the ring never holds a whole window of tiles
                // that a new round's first tile would queue behind — and the tiles past a stop
                // are never scanned
                const unsigned npub = (ENGINE_AHEAD > 0 && !multi) ? min(ntj, (unsigned)ENGINE_AHEAD) : ntj;
                if (lane == 0) M->pubt = npub;
                const unsigned ntiles = npub * (unsigned)S.nslice;
#ifdef FIT_STAMPS
                // before the tasks turn visible: a worker may pick tile 0 at once
                if (lane == 0) {
                    __hip_atomic_store(&ctl->pub[c], __builtin_amdgcn_s_memrealtime(),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                }
#endif
                if (pair) {  // tile 0 as 2 x nslice half-slices, then the rest
                    engine_publish(ctl, comp_ring(ring, c, ncomp), 0u, 1u, 2u * (unsigned)S.nslice, rnd, (unsigned)c);
                    if (npub > 1u) engine_publish(ctl, comp_ring(ring, c, ncomp), 1u, npub, (unsigned)S.nslice, rnd, (unsigned)c);
                    target[par] += (unsigned)S.nslice;  // tile 0's extra tasks
                } else {
                    engine_publish(ctl, comp_ring(ring, c, ncomp), 0u, npub, (unsigned)S.nslice, rnd, (unsigned)c);
                }
                if (npub == ntj) target[par] += ntiles;  // else: after the commit (M->pubt)
                if (multi && !fail) fail = !wait_tiles(ctl, c, par, target[par], wd, rnd);
                acquire_agent();  // node rows written by this block: CU-wide view for all waves
                if (lane == 0) s_fail = fail;
                {
                    MW_CLK(rs1);
                    MW_ADD(16, rs1 - rs0);
                }
            }
            __syncthreads();
            if (s_fail) break;  // block-uniform
            const int64_t t1 = (int64_t)__builtin_amdgcn_s_memrealtime();
            // a window holding a multi-node job is committed by wave 0 alone (commit_window
            // handles k > 1); the decider/helper pipeline covers k = 1 windows
            CommitResult R;
            if (!multi) {
                const unsigned ntj = (unsigned)((w + SCAN_JOBS - 1) / SCAN_JOBS);
                const bool jit = ENGINE_AHEAD > 0 && M->pubt < ntj;  // block-uniform (before the barrier)
                R = commit_window_mw(P, M, rec, cand, bnd, wjob, out, kmax,
                                     MwTiles{&ctl->tdone[par][c][0], (unsigned)S.nslice,
                                             jit ? comp_ring(ring, c, ncomp) : nullptr, ctl, rnd, (unsigned)c, ntj,
                                             &ctl->tfeas[par][c][0]});
                // every tile published this round (the committer's and the helpers') must be
                // complete before a later round reuses its buffer set: count them
                if (jit && wave == 0) target[par] += M->pubt * (unsigned)S.nslice;
            } else {
                if (wave == 0) {
                    const CommitResult r0 =
                        engine_commit_single(c, P, rec, cand, bnd, wjob, out, kmax, M->bitmap,
                                             reinterpret_cast<uint32_t*>(&M->rows[0]));
                    if (lane == 0) {
                        M->res[0] = r0.done;
                        M->res[1] = r0.stop;
                        M->res[2] = r0.dirty;
                        M->res[3] = r0.placed;
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // row write-back stores
                }
                __syncthreads();
                R = CommitResult{M->res[0], M->res[1], M->res[2], M->res[3]};
                __syncthreads();
            }
            if (wave == 0) used[par] = M->pubt;  // stable after the commit's closing barrier
            if (threadIdx.x == 0) engine_round_finished(ctl, c, rnd);
            if (R.stop == 3) {  // a commit wait gave up: M->fail names it (TRIP_PEER: drained)
                if (threadIdx.x == 0) {
                    const unsigned site = M->fail ? M->fail : (unsigned)TRIP_SINGLE_TILE;
                    const unsigned tl = site == TRIP_HELPER_TILE ? M->trip_arg : 0u;
                    trip_record(ctl, site == TRIP_PEER ? 0u : 2u, site, (unsigned)c, rnd, M->trip_arg,
                                M->pubt, ld_agent(&ctl->tdone[par][c][tl & (ENGINE_TILES - 1)]),
                                (unsigned)S.nslice, (unsigned long long)t1);
                }
                break;
            }
            if (R.done == 0) {  // the next round would rescan the same state: never progresses
                if (threadIdx.x == 0)
                    trip_record(ctl, 4u, TRIP_NO_PROGRESS, (unsigned)c, rnd, (unsigned)cursor, M->pubt,
                                0u, 0u, (unsigned long long)t1);
                break;
            }
            prev_multi = multi;
            const int64_t t2 = (int64_t)__builtin_amdgcn_s_memrealtime();
            tw += t1 - t0;
            tc += t2 - t1;
            evals += (int64_t)w * (S.se - S.sb);
            placed += R.placed;
            ++rounds;
            sr += R.stop == 1;
            sd += R.stop == 2;
            if (R.stop == 1 && R.done < SCAN_JOBS) wide_left = K0W_ROUNDS;
            else if (wide_left > 0) --wide_left;
            cursor += R.done;
#ifndef ENGINE_WGROW
#define ENGINE_WGROW 10  // next window after a stop, in eighths of the jobs the round resolved
#endif
            const int nw = R.stop ? (ENGINE_WGROW * R.done) / 8 : 2 * w;
            win = max(S.wmin, min(S.wmax, nw));
        }
        if (wave != 0) return;
        release_agent();  // last round's node rows / placements (kernel end also flushes)
        if (lane == 0) {
            co[c] = CompOut{evals, placed, cursor - S.jstart, rounds, sr, sd, tc, tw};
            __hip_atomic_fetch_add(&ctl->finished, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }

    // ====================================================================== scan worker
    const unsigned wgrp = worker_group(ncomp);  // this XCD's ring group (fit_engine_ctl.h)
    TaskClaim claim;
    unsigned long long* task_slot =
        reinterpret_cast<unsigned long long*>(smem + sizeof(uint64_t) * (SCAN_WAVES / 2) * KS * 64);
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
                wbusy[2 * (blockIdx.x - ncomp)] = busy;
                wbusy[2 * (blockIdx.x - ncomp) + 1] = scanned;
            }
            return;
        }
        const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
        const bool skip = (task & TASK_SKIP) != 0ull;  // block-uniform
        const int c = (int)(task & 63u);
        const int s = (int)task_slice(task);
        const int tile = (int)task_tile(task);
        const int par = (int)(task_round(task) & 1u);  // the round's buffer set
        bool counts = true;  // (thread 0) the task completes its tile's block-slice (K_T0PAIR)
        if (!skip) {
            if (threadIdx.x == 0) acquire_agent();
            else __builtin_amdgcn_s_dcache_inv();
            __syncthreads();
            CompPlan P = plans[2 * c + par];
            const bool pair = tile == 0 && (P.k0 & 2);  // half-size block-slices, paired
            if (pair) {
                P.sub = (P.sub + 1) / 2;
                P.nslice *= 2;
            }
            switch (P.ks) {  // block-uniform; the host picks one of these (engine.cpp)
#define SCAN_K(K_)                                                                               \
    case K_:                                                                                      \
        if (FIT_K0W > 0 && FIT_K0W < K_ && tile == 0 && (P.k0 & 4)) { /* wide, unpaired */          \
            constexpr int KW_ = (FIT_K0W > 0 && FIT_K0W < K_ ? FIT_K0W : K_);                        \
            uint64_t(*xkw)[KW_][64] = reinterpret_cast<uint64_t(*)[KW_][64]>(smem);                 \
            if (SCAN_WAVES * P.sub <= STAGE_ROWS) /* block-uniform */                               \
                scan_tile<true, KW_, K_, true>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart,   \
                                               jk, cand, bnd, wjob, xkw, &ctl->tfeas[par][c][tile],    \
                                               reinterpret_cast<NodeRec*>(smem + STAGE_OFF));     \
            else                                                                                  \
                scan_tile<true, KW_, K_>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, \
                                         cand, bnd, wjob, xkw, &ctl->tfeas[par][c][tile]);             \
        } else if (FIT_K0 > 0 && FIT_K0 < K_ && tile == 0 && (P.k0 & 1)) {                        \
            constexpr int K0_ = (FIT_K0 > 0 && FIT_K0 < K_ ? FIT_K0 : K_);                        \
            uint64_t(*xk0)[K0_][64] = reinterpret_cast<uint64_t(*)[K0_][64]>(smem);               \
            bool done_ = false;                                                                   \
            if constexpr (K0_ <= 4) { /* the pair scratch holds 4 keys */                          \
                done_ = pair;                                                                     \
                if (pair && SCAN_WAVES * P.sub <= STAGE_ROWS) /* block-uniform */                  \
                    counts = scan_tile<true, K0_, K_, true, true>(                                \
                        P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, xk0, \
                        &ctl->tfeas[par][c][tile], reinterpret_cast<NodeRec*>(smem + STAGE_OFF),     \
                        &ctl->tpair[par][c][0]);                                                  \
                else if (pair)                                                                    \
                    counts = scan_tile<true, K0_, K_, false, true>(                               \
                        P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, xk0, \
                        &ctl->tfeas[par][c][tile], nullptr, &ctl->tpair[par][c][0]);              \
            }                                                                                     \
            if (done_) {                                                                          \
            } else if (SCAN_WAVES * P.sub <= STAGE_ROWS) /* block-uniform */                       \
                scan_tile<true, K0_, K_, true>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, \
                                               jk, cand, bnd, wjob, xk0, &ctl->tfeas[par][c][tile],    \
                                               reinterpret_cast<NodeRec*>(smem + STAGE_OFF));     \
            else                                                                                  \
                scan_tile<true, K0_, K_>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, \
                                         cand, bnd, wjob, xk0, &ctl->tfeas[par][c][tile]);             \
        } else if (K_ <= 4 && pair) { /* a 4-key component's first tile, paired */               \
            if constexpr (K_ <= 4) {                                                              \
                uint64_t(*xk4)[K_][64] = reinterpret_cast<uint64_t(*)[K_][64]>(smem);             \
                if (SCAN_WAVES * P.sub <= STAGE_ROWS) /* block-uniform */                         \
                    counts = scan_tile<true, K_, K_, true, true>(                                 \
                        P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, xk4, \
                        &ctl->tfeas[par][c][tile], reinterpret_cast<NodeRec*>(smem + STAGE_OFF),     \
                        &ctl->tpair[par][c][0]);                                                  \
                else                                                                              \
                    counts = scan_tile<true, K_, K_, false, true>(                                \
                        P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, xk4, \
                        &ctl->tfeas[par][c][tile], nullptr, &ctl->tpair[par][c][0]);              \
            }                                                                                     \
        } else {                                                                                  \
            scan_tile<true, K_>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand,    \
                                bnd, wjob, reinterpret_cast<uint64_t(*)[K_][64]>(smem),           \
                                &ctl->tfeas[par][c][tile]);                                            \
        }                                                                                         \
        break;
                SCAN_K(16)
                SCAN_K(8)
                SCAN_K(4)
                SCAN_K(2)
#undef SCAN_K
                default:  // no scan kernel for this key count: trip the watchdog, never guess
                    if (threadIdx.x == 0)
                        trip_record(ctl, 8u, TRIP_NO_KERNEL, (unsigned)c, task_round(task), (unsigned)P.ks,
                                    0u, 0u, 0u, realtime());
                    break;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
#ifdef FIT_STAMPS
            if (threadIdx.x == 0 && tile == 0) {  // the round's first tile: pickup delay, scan time
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                atomicAdd(&g_mw[c][10], (unsigned long long)t0 - ctl->pub[c]);
                atomicAdd(&g_mw[c][11], 1ull);
                atomicAdd(&g_mw[c][12], now - (unsigned long long)t0);
            }
#endif
            const int a = P.sb + s * SCAN_WAVES * P.sub, b = min(P.se, a + SCAN_WAVES * P.sub);
            scanned += (int64_t)max(min(SCAN_JOBS, P.w - tile * SCAN_JOBS), 0) * max(b - a, 0);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            // the tile's outputs were written through (scan_tile: sc1 stores, agent atomics) and
            // every storing wave waited for them (vmcnt(0) above, then the barrier): the counts
            // need no release fence (cdna_hip_programming.md §6 Guideline 16 R1)
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

size_t engine_lds_bytes(int32_t max_component_nodes) {
    const size_t scan = STAGE_OFF + sizeof(NodeRec) * STAGE_ROWS;
    return std::max(scan, mw_lds_bytes(max_component_nodes));
}

size_t engine_ctl_bytes() { return sizeof(EngineCtl); }
size_t engine_ctl_error_offset() { return offsetof(EngineCtl, error); }
size_t engine_ctl_trip_offset() { return offsetof(EngineCtl, trip); }
size_t engine_ring_bytes() { return sizeof(unsigned long long) * QRING * QGROUPS; }
size_t engine_ring_tasks() { return QCAP; }  // task slots per ring
int engine_ring_groups() { return (int)QGROUPS; }  // rings (components c % groups share one)

int engine_blocks_per_cu(size_t lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_engine, SCAN_WAVES * 64, lds) !=
        hipSuccess)
        return 0;
    return n;
}

hipError_t launch_engine(int blocks, size_t lds, hipStream_t st, void* ctl, void* ring,
                         const void* cs, void* co, CompPlan* plans, int ncomp, NodeRec* rec,
                         const int32_t* jl, const int32_t* jcpu, const int32_t* jmem,
                         const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart,
                         const uint16_t* jk, uint64_t* cand, uint64_t* bnd, JobRec* wjob,
                         int32_t* out, int kmax, int64_t* wbusy, const int32_t* jpk, unsigned wd) {
    hipLaunchKernelGGL(k_engine, dim3(blocks), dim3(SCAN_WAVES * 64), lds, st,
                       static_cast<EngineCtl*>(ctl), static_cast<unsigned long long*>(ring),
                       static_cast<const CompState*>(cs), static_cast<CompOut*>(co), plans, ncomp,
                       rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, out, kmax,
                       wbusy, jpk, wd);
    return hipGetLastError();
}

}  // namespace fitgpu

#ifdef FIT_TILE0_STAMPS
extern "C" int fit_debug_tile0(unsigned long long* out /* 8 */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(fitgpu::g_tile0), sizeof(fitgpu::g_tile0)) == hipSuccess ? 0 : -2;
}
#endif
#ifdef FIT_STAMPS
// the single-wave commit's segment stamps of this TU (multi-node windows; fit_common.h STAMP)
extern "C" int fit_debug_commit_stamps_pe(unsigned long long* out /* 64 x 8 */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(fitgpu::g_stamps), sizeof(fitgpu::g_stamps)) ==
                   hipSuccess ? 0 : -2;
}
extern "C" int fit_debug_mw_stamps(unsigned long long* out /* 64 x 16 */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(fitgpu::g_mw), sizeof(fitgpu::g_mw)) == hipSuccess
               ? 0 : -2;
}
#endif
