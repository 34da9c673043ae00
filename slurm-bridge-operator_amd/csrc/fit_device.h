// fit_device.h — data layouts shared by the HIP kernels and the host engine.
#pragma once
#include <stdint.h>

namespace fitgpu {

#ifndef FIT_KS
#define FIT_KS 16
#endif
constexpr int KS = FIT_KS;      // candidates kept per (job, block-slice) by fit_scan
// the per-wave insertion network and the LDS bitonic merge tree of k_scan need a power of two
// (a FIT_KS=12 build placed jobs wrongly before this check)
// k_engine's workers dispatch on the per-component key count with cases 16, 8, 4 and 2 only
// (fit_persistent.hip): a larger FIT_KS would have no case
static_assert(KS >= 2 && KS <= 16 && (KS & (KS - 1)) == 0, "FIT_KS must be a power of two in [2, 16]");
constexpr int SCAN_WAVES = 8;   // waves per scan block; each walks one sub-slice of nodes
constexpr int SCAN_JOBS = 64;   // jobs per scan block (lanes = jobs, shared by the 8 waves)
#ifndef FIT_MIN_SUB
#define FIT_MIN_SUB 64
#endif
constexpr int MIN_SUB = FIT_MIN_SUB;  // minimum nodes per wave sub-slice
#ifndef FIT_MAX_SLICES
#define FIT_MAX_SLICES (128 / FIT_KS)
#endif
constexpr int MAX_SLICES = FIT_MAX_SLICES;  // block-slices per job per rank (sub-slice grows past this)
#ifndef FIT_TL_KS
#define FIT_TL_KS 4
#endif
constexpr int TL_KS = FIT_TL_KS;  // candidates per (job, block-slice) of the backfill scan
static_assert(TL_KS >= 1 && TL_KS <= 64 && (TL_KS & (TL_KS - 1)) == 0, "FIT_TL_KS must be a power of two");
#ifndef FIT_UCAP
#define FIT_UCAP 128  // 256: fewer dirty-full stops, but 6 helper entries per lane instead of 4
#endif                 // (C3 k_engine 33.6 -> 32.3 ms at 128, C2 -4 %, C3o +2 %)
constexpr int UCAP = FIT_UCAP;       // dirty-node capacity per component per round (UCAP / 64 per lane)
constexpr int MAX_COMPONENT_NODES = 1 << 20;  // LDS dirty bitmap limit (128 KiB)
constexpr uint64_t KEY_INF = ~0ull;
constexpr int FIT_KMAX = 8;     // nodes per multi-node job (include/fitgpu.h FIT_MAX_K)

// One Slurm node row in HBM, 32 B: read by fit_scan with one scalar s_load_dwordx8.
struct alignas(32) NodeRec {
    int32_t cpu, mem, gpu, avail;  // free cpus, free MiB, free GPUs, availability horizon (min)
    uint32_t mask;                 // partition membership bits
    int32_t orig;                  // node id in the caller's order (Client.Nodes order)
    int32_t pad0, pad1;
};

// Job row of the current window, written by fit_scan (slice 0), read by fit_commit.
struct alignas(32) JobRec {
    int32_t q;        // job index in the caller's priority order
    int32_t cpu, mem, gpu, wall;
    uint32_t pbit;    // 1u << partition
    int32_t k;        // nodes per job
    int32_t pad;
};

// Per-component plan for one round (host-built, uploaded each round).
struct alignas(16) CompPlan {
    int32_t nb, ne;      // component's node positions [nb, ne)
    int32_t sb, se;      // this rank's scan range inside it
    int32_t nslice;      // block-slices per job on every rank (<= MAX_SLICES)
    int32_t sub;         // nodes per wave sub-slice (block-slice = SCAN_WAVES * sub)
    int32_t jbase;       // first window job's index into the component job list
    int32_t w;           // window size (jobs)
    int32_t blk0;        // first fit_scan block of this component
    int32_t ks;          // keys kept per (job, block-slice): KS, or fewer for a large component
    int64_t cand_off;    // u64 offset of the component's candidates inside one rank section
    int32_t slot0;       // first window slot (global over components)
    int32_t k0;          // persistent engines, the round's first job tile: bit 0 keeps FIT_K0 keys
                         // (k_engine, k = 1 window); bit 1 scans it as paired half-slices (*_T0PAIR);
                         // bit 2 keeps FIT_K0W keys, unpaired (k_engine, after a first-tile rescan)
    int32_t pair_off;    // u64 offset of the round's half-slice list scratch (bit 1 of k0)
};

// Persistent engine (fit_persistent.hip): per-component state written by the host, results
// written by the component's committer wave.
struct CompState {
    int32_t nb, ne, sb, se, nslice, sub;
    int32_t jstart, jend;  // component job list range
    int64_t cand_off;      // fixed candidate region of this component (even rounds)
    int32_t slot0;         // fixed window slot region (even rounds)
    int32_t wmin, wmax;
    int32_t ks;            // keys per (job, block-slice) (CompPlan::ks)
    int64_t cand_alt;      // the same for odd rounds (fit_engine_ctl.h: two buffer sets by parity)
    int32_t slot_alt;
    int32_t pair_off;      // half-slice list scratch (even rounds; odd: + PAIR_AREA)
};

struct CompOut {
    int64_t evals, placed, done_jobs, rounds, stops_rescan, stops_dirty;
    int64_t t_commit, t_wait;  // 100 MHz realtime ticks spent committing / waiting for scans
};

// ---- SPEC §2b time-windowed backfill (fit_timeline.hip) --------------------
#ifndef FIT_TL_SPLIT_DEF
#define FIT_TL_SPLIT_DEF 0  // k_engine_tl as two concurrent launches (committers / scan workers); env FIT_TL_SPLIT
#endif
constexpr int TL_MAX_SLOTS = 1024;  // horizon limit (slots); the C5 horizon
#ifndef TL_UCAP_DEF
#define TL_UCAP_DEF 64
#endif
constexpr int TL_UCAP = TL_UCAP_DEF;  // dirty nodes per component per round (TL_UCAP / 64 per lane)
#ifndef FIT_TL_CAND
#define FIT_TL_CAND 128
#endif
constexpr int TL_CAND = FIT_TL_CAND;  // candidates per job of the timeline scan (64 or 128)
static_assert((TL_CAND == 64 || TL_CAND == 128) && TL_CAND % TL_KS == 0, "FIT_TL_CAND: 64 or 128");
constexpr int TL_SLICES = TL_CAND / TL_KS;  // block-slices per job (over all ranks) in the timeline scan
// The persistent engines' paired first tile (K_T0PAIR, TL_T0PAIR): one half-slice list of up to 4
// keys per (job, pair) held until its partner half merges it, per component and round parity
constexpr int PAIR_AREA = SCAN_JOBS * 32 * 4;
static_assert(TL_KS <= 4, "pair scratch holds 4 keys per (job, pair)");
constexpr int TL_MIN_SUB = 16;      // minimum nodes per wave sub-slice in the timeline scan (C5: 32 block-slices;
                                    // 32 gave 25 slices, 100 candidates: 129.8 vs 127.1 ms, r03j)
constexpr int TL_POS_BITS = 22;     // key = start << 54 | score << 22 | position
constexpr uint32_t TL_POS_MASK = (1u << TL_POS_BITS) - 1u;

// One run of equal free resources on a node's timeline: slots [previous end, end).  A node's
// list is canonical (adjacent runs differ) and ends at the horizon; at most TL_MAX_SLOTS runs.
struct alignas(16) Seg {
    int32_t end, cpu, mem, gpu;
};

constexpr int TL_HEAD = 4;  // runs of each node copied into its header (the scan's common case)

// Per-node header of a run list, 96 B, contiguous over nodes (the scan streams it): run count,
// the largest free value of each column over the timeline as built (reservations only lower
// values, so it stays an upper bound: a job whose demand exceeds it can never fit the node),
// partition mask, node id, and a copy of the first TL_HEAD runs.
struct alignas(32) TlHdr {
    int32_t cnt, cpu, mem, gpu;
    uint32_t mask;
    int32_t orig;  // node id in the caller's order (so a new dirty node needs no perm[] load)
    int32_t pad[2];
    Seg head[TL_HEAD];
};

struct CommitResult {
    int32_t done;   // jobs resolved this round (prefix of the window)
    int32_t stop;   // 0 window exhausted, 1 candidate list ran out, 2 dirty set full
    int32_t dirty;  // distinct nodes touched
    int32_t placed;
};

// Component node offsets for the direct small placement (k_small): nb[c] .. nb[c + 1].
struct SmallComps {
    int32_t nb[33];
};

// A small batch carried in k_small's kernel arguments (fit_place: no copy to the device; the
// kernarg segment holds up to 4 KB, this is 2,560 B).
constexpr int SMALL_ARGJ = 128;
struct SmallBatch {
    int32_t cpu[SMALL_ARGJ], mem[SMALL_ARGJ], gpu[SMALL_ARGJ], wall[SMALL_ARGJ];
    uint16_t part[SMALL_ARGJ], nk[SMALL_ARGJ];
};

// Persistent engines' watchdog trip record (fit_engine_ctl.h; read back by engine.cpp).
enum TripSite : unsigned {
    TRIP_NONE = 0,
    TRIP_WORKER_RING = 1,   // scan worker: its claimed ring slot got no task (arg = ring index)
    TRIP_ROUND_START = 2,   // committer: tiles of the round before last not done (arg = target)
    TRIP_HELPER_TILE = 3,   // commit helper: a job tile's scan not done (arg = tile)
    TRIP_HELPER_SNAP = 4,   // commit helper: the decider did not advance (arg = record)
    TRIP_DECIDER_REC = 5,   // decider: a helper record not ready (arg = record)
    TRIP_SINGLE_TILE = 6,   // single-wave commit: a job tile's scan not done (arg = tile)
    TRIP_NO_PROGRESS = 7,   // a round resolved no job
    TRIP_NO_KERNEL = 8,     // no scan kernel for the plan's key count
    TRIP_PEER = 9,          // drained after another block's trip
};
struct TripRec {  // the launch's first trip (claim 0 -> 1); plain stores, read after the kernel
    unsigned claim, site, comp, round;
    unsigned arg, q_head, q_tail, pubt;
    unsigned tdone, need, block, pad;
    unsigned long long waited;  // realtime ticks (10 ns) the wait lasted
    unsigned long long when;    // realtime at the trip, minus the launch's start stamp
};

}  // namespace fitgpu
