// fit_engine_ctl.h — control block and agent-scope hand-off primitives of the persistent
// single-launch engines (k_engine: fit_persistent.hip; k_engine_tl: fit_timeline.hip).
// DESIGN.md §3.6.  Cross-workgroup hand-offs follow cdna_hip_programming.md §6 Guideline 16.
#pragma once
#include <hip/hip_runtime.h>

#include "fit_device.h"

namespace fitgpu {

#ifndef FIT_QCAP_LOG2
#define FIT_QCAP_LOG2 18
#endif
constexpr unsigned QCAP = 1u << FIT_QCAP_LOG2;  // task ring entries (8-byte {epoch, tile} granules)
// XCD-aware task rings (round 6; A/B switch, off): FIT_XCD_RINGS 1 gives one
// ring per group of components, group g = c % G with G = min(8, ncomp), and a scan worker serves
// only its own XCD's group (HW_REG_XCC_ID % G), so a component's node data is read by the CUs of
// one XCD and stays in that XCD's L2.  Measured (profiles/r06_xcd_rings_ab.txt): live traffic
// C5 22.5 -> 12.9 GB and C3 3.6 -> 2.3 GB per launch — the node headers every XCD re-fetched
// are the re-read — but k_engine_tl +11 % and k_engine +2 %: a round start's burst of tiles gets
// an eighth of the workers.  Letting idle workers take other groups' published tasks (claim by
// add: +2 % / +0.4 %, 20.0 GB; by compare-and-swap below the tail, with a shared ring for the
// round-first tiles: 2.3x slower) gave the traffic back or worse.  0: one ring, a worker claims
// the next index at once and waits for its slot.  A ring is QRING entries: a 256-B header (tail
// counter at entry 0, head counter at entry 16, own lines) and QCAP task slots.
#ifndef FIT_XCD_RINGS
#define FIT_XCD_RINGS 0
#endif
constexpr unsigned QGROUPS = FIT_XCD_RINGS ? 8u : 1u;
constexpr unsigned QHDR = 32u;              // header entries of a ring
constexpr unsigned QRING = QHDR + QCAP;     // entries per ring
__device__ __forceinline__ unsigned ring_groups(int ncomp) {
    return ncomp < (int)QGROUPS ? (unsigned)max(ncomp, 1) : QGROUPS;
}
// the ring of component c's group
__device__ __forceinline__ unsigned long long* comp_ring(unsigned long long* rings, int c, int ncomp) {
    return rings + (size_t)((unsigned)c % ring_groups(ncomp)) * QRING;
}
// the group of this CU's XCD
__device__ __forceinline__ unsigned worker_group(int ncomp) {
#if FIT_XCD_RINGS
    const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;  // HW_REG_XCC_ID
    return xcc % ring_groups(ncomp);
#else
    (void)ncomp;
    return 0u;
#endif
}
__device__ __forceinline__ unsigned* ring_tail(unsigned long long* ring) { return reinterpret_cast<unsigned*>(ring); }
__device__ __forceinline__ unsigned* ring_head(unsigned long long* ring) { return reinterpret_cast<unsigned*>(ring + 16); }
constexpr int ENGINE_TILES = 128;    // job tiles per window (window <= 8192 jobs)
constexpr unsigned long long TASK_EXIT = ~0ull;

// ---- watchdog (round 5) ----------------------------------------------------------------------
// The cross-block waits of the persistent engines are bounded in TIME: `wd` ticks of the 100 MHz
// realtime counter since the wait began (a kernel argument; fit_set_watchdog_us, default 10 s) —
// the scan workers' ring waits, the committers' round-start waits and k_engine_tl's helpers' tile
// waits.  A spin count cannot tell a long legitimate wait (another tenant's kernel holding the CUs)
// from a hang.  k_engine's in-block commit waits (helpers' tile waits, decider <-> helper
// hand-offs, fit_commit_mw.h) keep a spin bound (MW_SPIN_LIMIT, a few seconds): a clock there
// costs the VGPR-limited helper +0.55 ms at C3, and what they wait for comes
// from blocks whose own waits are timed.
// The first trip of a launch records where it happened (TripRec); fit_last_error reports it.
__device__ __forceinline__ unsigned long long realtime() { return __builtin_amdgcn_s_memrealtime(); }
// The clock of one wait, free while the wait is short: it is read every 64 spins only (an SMEM
// round trip), and its first read starts it — a spin costs one scalar compare, so the decider's
// and the helpers' hot waits keep their round-4 shape.  `wd` (or the LDS word holding it) is read
// only at a check.
#ifndef FIT_WD_ROUND
#define FIT_WD_ROUND 1   // committer round-start wait: time deadline (0: spin bound; A/B switch)
#endif
#ifndef FIT_WD_WORKER
#define FIT_WD_WORKER 1  // scan worker task wait: time deadline (0: spin bound; A/B switch)
#endif
constexpr unsigned WD_SPINS = 1u << 25;  // the spin bound of a switched-off deadline
struct WaitClock {
    unsigned long long t0 = 0ull;
    __device__ __forceinline__ bool over(unsigned spins, unsigned wd) {
        if ((spins & 63u) != 63u) return false;
        const unsigned long long now = realtime();
        if (t0 == 0ull) {
            t0 = now;
            return false;
        }
        return now - t0 > (unsigned long long)wd;
    }
    __device__ __forceinline__ bool over_lds(unsigned spins, const uint32_t* wd_lds) {
        if ((spins & 63u) != 63u) return false;
        const unsigned long long now = realtime();
        if (t0 == 0ull) {
            t0 = now;
            return false;
        }
        return now - t0 > (unsigned long long)__hip_atomic_load(wd_lds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

struct alignas(128) EngineCtl {  // zeroed by a memset before every launch
    unsigned pad0[64];  // (round 5's global ring counters: now in each ring's header)
    unsigned finished;  // components done
    unsigned error;     // 1 = watchdog
    unsigned pad2[30];
    // per component (own 128-B line each): [1] the last finished round's tag, [2 + p] scan tiles
    // completed of the rounds with parity p
    unsigned done[32][32];
    // Per-round buffers come in two sets, by round parity p = round & 1 (plans, candidates, bounds,
    // window job rows, these counters and masks): a new round needs only the tiles of the round
    // before last (same set) to be complete — long done — instead of waiting for the previous
    // round's tiles still being scanned after its commit stopped.
    unsigned tdone[2][32][ENGINE_TILES];  // per parity, component, window job tile: slices completed
    // per component, per window job tile: bit j = job j of the tile has a node that fits it at
    // the round's start state (OR over the block-slices; k_engine).  A job without one is
    // unplaced whatever the round decides before it (node state only shrinks within a
    // placement): the commit skips it (fit_commit_mw.h, "live jobs")
    unsigned long long tfeas[2][32][ENGINE_TILES];
    // k_engine_tl's round-first tile scanned as pairs of half-slices (TL_T0PAIR): per parity,
    // component and pair, the halves finished (the second merges both lists)
    unsigned tpair[2][32][32];
    unsigned long long pub[32];        // FIT_STAMPS: realtime of each component's last publish
    unsigned long long t_start;        // realtime when the first block started (min, TripRec::when)
    TripRec trip;
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Record a trip (one lane): the first trip of the launch claims ctl->trip and describes itself;
// every trip ORs its error bit, which drains all blocks.  Inlined: as a call it made k_engine's
// worker loop keep more registers (154 -> 159 VGPRs, six more call sites).
static __device__ __forceinline__ void trip_record(EngineCtl* ctl, unsigned bit, unsigned site, unsigned comp,
                                               unsigned round, unsigned arg, unsigned pubt, unsigned tdone,
                                               unsigned need, unsigned long long t0) {
    if (site != TRIP_PEER &&
        __hip_atomic_fetch_or(&ctl->trip.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        const unsigned long long now = realtime();
        TripRec& r = ctl->trip;
        r.site = site;
        r.comp = comp;
        r.round = round;
        r.arg = arg;
        r.q_head = 0u;  // per-group rings: the waiting worker's claimed index is in `arg`
        r.q_tail = 0u;
        r.pubt = pubt;
        r.tdone = tdone;
        r.need = need;
        r.block = blockIdx.x;
        r.waited = now - t0;
        const unsigned long long ts = __hip_atomic_load(&ctl->t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.when = ts && now > ts ? now - ts : 0ull;
    }
    __hip_atomic_fetch_or(&ctl->error, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the launch's start stamp (the first block to arrive; one lane per block)
__device__ __forceinline__ void stamp_start(EngineCtl* ctl) {
#ifdef FIT_WD_NO_STAMP
    return;
#endif
    const unsigned long long now = realtime();
    unsigned long long none = 0ull;
    if (__hip_atomic_load(&ctl->t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull)
        __hip_atomic_compare_exchange_strong(&ctl->t_start, &none, now, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Task word: {epoch:32 | skip:1 | round:12 | tile:7 | slice:6 | component:6}.  done[c][1] holds
// the round tag of component c's last finished commit: a task of that round or an earlier one is
// dropped unscanned (it only counts as done) — a round that stops early leaves its later tiles
// unneeded, and scanning them would delay both the next round's start and other components'
// tiles.  Rounds finish in order, so "earlier" is a 12-bit modular comparison.
static_assert(ENGINE_TILES <= 128, "7 tile bits");
__device__ __forceinline__ unsigned task_slice(unsigned long long task) {
    return (unsigned)(task >> 6) & 0x3fu;  // up to 64 block-slices per job
}
constexpr unsigned long long TASK_SKIP = 1ull << 31;
__device__ __forceinline__ unsigned long long engine_task(unsigned long long epoch, unsigned round,
                                                          unsigned tile, unsigned sl, unsigned c) {
    return (epoch << 32) | ((unsigned long long)(round & 0xfffu) << 19) | (tile << 12) |
           (sl << 6) | c;
}
__device__ __forceinline__ unsigned task_tile(unsigned long long task) {
    return (unsigned)(task >> 12) & 0x7fu;
}
__device__ __forceinline__ unsigned task_round(unsigned long long task) {
    return (unsigned)(task >> 19) & 0xfffu;
}
__device__ __forceinline__ bool task_dropped(EngineCtl* ctl, unsigned long long task) {
    const unsigned c = (unsigned)task & 63u;
    return ((ld_agent(&ctl->done[c][1]) - task_round(task)) & 0xfffu) < 0x800u;
}
// the committer of component c has finished round `round`: drop what is left of its tiles
__device__ __forceinline__ void engine_round_finished(EngineCtl* ctl, int c, unsigned round) {
    __hip_atomic_store(&ctl->done[c][1], round & 0xfffu, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Publish job tiles [from, upto) of component c's window (every block-slice of each) to the task
// ring of c's group (`ring`: comp_ring): one wave, uniform arguments.  The caller has released
// (agent scope) what the tasks' scans read — the round's plan, bound / tile-counter resets and
// node state.
__device__ __forceinline__ void engine_publish(EngineCtl* ctl, unsigned long long* ring,
                                               unsigned from, unsigned upto, unsigned nslice,
                                               unsigned round, unsigned c) {
    (void)ctl;
    const unsigned lane = threadIdx.x & 63u;
    const unsigned n = (upto - from) * nslice;
    unsigned base = 0;
    if (lane == 0)
        base = __hip_atomic_fetch_add(ring_tail(ring), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = (unsigned)__builtin_amdgcn_readlane((int)base, 0);
    for (unsigned i = lane; i < n; i += 64) {
        const unsigned idx = base + i;
        const unsigned tile = from + i / nslice, sl = i % nslice;
        __hip_atomic_store(ring + QHDR + (idx & (QCAP - 1)), engine_task(idx / QCAP + 1, round, tile, sl, c),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Write-through (sc1) copy of a small record by the lanes of one wave: 8-B relaxed agent-scope
// stores (cdna_hip_programming.md §6 Guideline 16 R1), so it needs no release fence of its own.
template <class T>
__device__ __forceinline__ void store_through(T* dst, const T& v) {
    static_assert(sizeof(T) % 8 == 0, "8-byte words");
    const unsigned lane = threadIdx.x & 63u;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(&v);
    uint64_t* d = reinterpret_cast<uint64_t*>(dst);
    for (unsigned i = lane; i < sizeof(T) / 8; i += 64)
        __hip_atomic_store(d + i, s[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_through64(uint64_t* dst, uint64_t v) {
    __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void acquire_agent() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_dcache_inv();  // scalar cache: node rows, plans, job rows are s_loaded
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void release_agent() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ROCm 7.2 can drop the fence's own wait
}

// The next task of a scan worker (thread 0): claim the next index of its ring (FIT_XCD_RINGS
// above) and wait for the slot; TASK_EXIT once every component has finished or a block tripped.
struct TaskClaim {
    unsigned long long* ring = nullptr;
    unsigned idx = 0;
    bool held = false;
};
__device__ __forceinline__ unsigned long long next_task(EngineCtl* ctl, unsigned long long* rings, int ncomp,
                                                        unsigned own, TaskClaim& cl, unsigned wd) {
    WaitClock clk;
    for (unsigned spins = 0;; ++spins) {
        if (!cl.held) {
            cl.ring = rings + (size_t)own * QRING;
            cl.idx = __hip_atomic_fetch_add(ring_head(cl.ring), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cl.held = true;
        }
        if (cl.held) {
            const unsigned long long g = __hip_atomic_load(cl.ring + QHDR + (cl.idx & (QCAP - 1)), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            if ((g >> 32) == (unsigned long long)(cl.idx / QCAP + 1)) {
                cl.held = false;
                return g;
            }
        }
        if (ld_agent(&ctl->finished) == (unsigned)ncomp || ld_agent(&ctl->error)) return TASK_EXIT;
        if (FIT_WD_WORKER ? clk.over(spins, wd) : spins > WD_SPINS) {
            trip_record(ctl, 1u, TRIP_WORKER_RING, 0u, 0u, cl.idx, 0u, ld_agent(&ctl->finished),
                        (unsigned)ncomp, clk.t0);
            return TASK_EXIT;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Spin (wave 0 of a committer) until component c has completed `target` scan tiles of the
// rounds with parity p.  false: another block tripped, or this wait outlasted `wd` (recorded).
__device__ __forceinline__ bool wait_tiles(EngineCtl* ctl, int c, int p, unsigned target,
                                           unsigned wd, unsigned round) {
    WaitClock clk;
    for (unsigned spins = 0;; ++spins) {
        const unsigned d = ld_agent(&ctl->done[c][2 + p]);
        if (d >= target) return true;
        if (ld_agent(&ctl->error)) return false;
        if (FIT_WD_ROUND ? clk.over(spins, wd) : spins > WD_SPINS) {
            if ((threadIdx.x & 63u) == 0u)
                trip_record(ctl, 1u, TRIP_ROUND_START, (unsigned)c, round, target, 0u, d, target, clk.t0);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

}  // namespace fitgpu
