// fit_engine_ctl.h — control block and agent-scope hand-off primitives of the persistent
// single-launch engines (k_engine: fit_persistent.hip; k_engine_tl: fit_timeline.hip).
// DESIGN.md §3.6.  Cross-workgroup hand-offs follow cdna_hip_programming.md §6 Guideline 16.
#pragma once
#include <hip/hip_runtime.h>

namespace fitgpu {

#ifndef FIT_QCAP_LOG2
#define FIT_QCAP_LOG2 18
#endif
constexpr unsigned QCAP = 1u << FIT_QCAP_LOG2;  // task ring entries (8-byte {epoch, tile} granules)
constexpr int ENGINE_TILES = 128;    // job tiles per window (window <= 8192 jobs)
constexpr unsigned SPIN_LIMIT = 1u << 25;
constexpr unsigned long long TASK_EXIT = ~0ull;

struct alignas(128) EngineCtl {  // zeroed by a memset before every launch
    unsigned q_tail;   // tiles reserved by committers
    unsigned pad0[31];
    unsigned q_head;   // tiles claimed by workers
    unsigned pad1[31];
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
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// ring: one wave, uniform arguments.  The caller has released (agent scope) what the tasks'
// scans read — the round's plan, bound / tile-counter resets and node state.
__device__ __forceinline__ void engine_publish(EngineCtl* ctl, unsigned long long* ring,
                                               unsigned from, unsigned upto, unsigned nslice,
                                               unsigned round, unsigned c) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned n = (upto - from) * nslice;
    unsigned base = 0;
    if (lane == 0)
        base = __hip_atomic_fetch_add(&ctl->q_tail, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = (unsigned)__builtin_amdgcn_readlane((int)base, 0);
    for (unsigned i = lane; i < n; i += 64) {
        const unsigned idx = base + i;
        const unsigned tile = from + i / nslice, sl = i % nslice;
        __hip_atomic_store(ring + (idx & (QCAP - 1)), engine_task(idx / QCAP + 1, round, tile, sl, c),
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

// Spin (wave 0 of a committer) until component c has completed `target` scan tiles of the
// rounds with parity p.
__device__ __forceinline__ bool wait_tiles(EngineCtl* ctl, int c, int p, unsigned target) {
    for (unsigned spins = 0; ld_agent(&ctl->done[c][2 + p]) < target;) {
        if (++spins > SPIN_LIMIT || ld_agent(&ctl->error)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

}  // namespace fitgpu
