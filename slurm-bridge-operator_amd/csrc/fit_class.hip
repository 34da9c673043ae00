// fit_class.hip — the demand-class engine: the default for
// placements whose live jobs are mostly multi-node (engine.cpp cls_mode 3), opt-in otherwise.
//
// A component's pending queue has few distinct per-node demands: a job's CLASS is its (cpu, mem,
// gpu) of one partition (the reference derives them from a handful of labels,
// pkg/slurm-bridge-operator/pod.go:97-107,143-162).  Instead of a candidate list per JOB (the
// persistent engine's scan, §3.2), this engine keeps a candidate SET per CLASS that lives for the
// whole placement and is updated at every commit — one 512-thread workgroup per partition
// component, its node rows in LDS, no scan workers and no rounds.
//
// Per class c: a set S_c of at most CLS_SET node positions and a bound L_c with the invariant
//     every node NOT in S_c has key_c >= L_c          (key_c: SPEC §2's key without the walltime
//                                                      term; the walltime is a per-job filter)
// Listed keys are evaluated at query time from the current rows, so a commit touches a class only
// when the committed node x is unlisted and its new key falls below L_c: x joins S_c (room left),
// takes the slot of a dead entry (a listed node the class no longer fits: rows only shrink, so it
// never will again), or L_c drops to x's key (x stays out, >= the new bound).  Keys only fall
// within a placement, so an unlisted node whose row did not change stays >= L_c.
//
// Query of job t (class c, walltime w, k nodes): the candidates are S_c's entries plus the nodes of
// the last CLS_RING commits (the "ring": commits the class's bookkeeper may not have processed yet),
// all evaluated with w at the current rows.  The k smallest distinct candidate keys are the
// sequential answer when the k-th is < L_c (every other node is >= L_c), or when L_c is infinite
// (every feasible node is listed).  Otherwise the set is EXHAUSTED: the whole workgroup refills it
// from a scan of the component (the per-thread minimum of its nodes below the smallest per-thread
// second key, so again every unlisted node is >= the new L_c) and the job is queried again; if the
// walltime or k still defeats the set, the workgroup resolves the job by an exact scan.
//
// Waves: 0 = DECIDER (the chain: query, commit — all k picks of a job at once, one lane each —
// record); 1..3 = BOOKKEEPERS (wave 1+b owns classes
// [64b, 64b+64), one per lane: for each commit record (x, old row, new row) it decides membership
// by the old key against its own register copy of L, and appends x or lowers L — the only writer
// of its classes' sets and bounds); 4 = JOB STAGER (the component's job fields into an LDS ring
// ahead of the decider); 5..7 join the block operations only (refill, exact pick).
//
// LDS protocol (workgroup scope, as fit_commit_mw.h): decider → bookkeepers: record, release,
// ncommit, then the row; bookkeepers: relaxed poll of ncommit, acquire, record.  Bookkeeper →
// decider: set entry then count (append), bound (lowering), release, prog[b].  The decider waits for
// prog[b] >= ncommit - CLS_RING before reading a class's count, entries and bound (in that order):
// any commit the bookkeeper has not processed is in the ring, and an append or lowering the read
// tears only concerns the node of such a commit.  Block operations run between __syncthreads()
// with every bookkeeper drained (prog == ncommit).
#include "fit_common.h"

namespace fitgpu {

constexpr int CLS_MAX = 192;                 // classes per component: 3 bookkeeper waves × 64
constexpr int CLS_RING = 8;                  // the decider's last commits (lanes 56..63)
constexpr int CLS_SET = 64 - CLS_RING;       // set capacity (lanes 0..55)
constexpr int CLS_REC = 32;                  // commit-record ring
constexpr int CLS_THREADS = 512;
constexpr int CLS_NPT = 16;                  // nodes per thread in the block operations
constexpr int CLS_TS = 512;                  // classify hash slots per component
constexpr int CLS_POOL = CLS_THREADS;        // refill pool (one key per thread at most)
constexpr int CLS_BK = 3;                    // bookkeeper waves
constexpr int CLS_JR = 256;                  // staged job ring (wave 4 → the decider)
#ifndef CLS_PROBES
#define CLS_PROBES 16
#endif
constexpr int CLS_PROBE = CLS_PROBES;        // a full set's insert: slots probed for a dead entry
constexpr unsigned CLS_SPIN = 1u << 26;      // spin bound of an in-block wait (a bug, not a load)

enum : unsigned { CLS_OP_EXIT = 1, CLS_OP_REFILL = 2, CLS_OP_PICK = 3 };

// compiler barrier: keeps one wave's LDS operations in program order (the LDS executes a wave's
// DS instructions in issue order, so a store published by a later store is visible to any wave
// that observes the later one)
#define CLS_CBAR() asm volatile("" ::: "memory")

#ifdef FIT_STAMPS
// diagnostic build: the decider's cycles by segment per component (s_memtime), read by
// fit_debug_class_stamps: [0] bookkeeper wait, [1] query, [2] refill (drain + op), [3] exact pick,
// [4] commit, [5] job-chunk loads, [6] jobs, [7] commits
__device__ unsigned long long g_cls_st[32][8];
// refill phases seen by the decider wave: [0] until barrier A, [1] scan + B1, [2] pool + B2,
// [3] set build (wave 0), [4] barrier C, [5] refills
__device__ unsigned long long g_cls_op[32][8];
#define CLS_OPT(v) const unsigned long long v = (wave == 0) ? __builtin_amdgcn_s_memtime() : 0ull
#define CLS_OPADD(i, a, b) do { if (tid == 0) atomicAdd(&g_cls_op[blockIdx.x & 31][i], (b) - (a)); } while (0)
#define CLS_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define CLS_ACC(i, a, b) (st_acc[i] += (b) - (a))
#else
#define CLS_T(v)
#define CLS_ACC(i, a, b)
#define CLS_OPT(v)
#define CLS_OPADD(i, a, b)
#endif

struct ClsSlot {  // classify hash slot (global, 32 B)
    unsigned long long tag;
    int32_t cpu, mem, gpu, part;
    int32_t idp;  // id + 1, 0 = not yet published
    int32_t pad;
};

struct alignas(16) ClsRec {  // one commit: node x (component position), its row before and after,
    int32_t x, oc, om, og;      // and the out[] entry it fills (bookkeeper 0 stores it)
    int32_t nc, nm, ng, oi;
};

struct alignas(16) ClsHdr {  // a class's set count and bound, read together (one ds_read_b128)
    uint32_t cnt, pad;
    unsigned long long L;
};

struct ClsCtl {
    alignas(16) unsigned prog[4];    // commits processed per bookkeeper (read together)
    unsigned ncommit;                // commits published by the decider
    int32_t staged;                  // jobs [t0, staged) of the list are in the job ring
    int32_t jdone;                   // the decider's position in the list (ring flow control)
    unsigned op_epoch, op, op_cls, op_k;
    int32_t op_wall;
    unsigned pool_n, npick, ncls;
    unsigned long long red[2][8];    // cross-wave minima
    unsigned long long pick[FIT_KMAX];
};

// LDS layout after the rows: everything but the rows is fixed-size
struct ClsLds {
    ClsCtl ctl;
    int4 dem[CLS_MAX];               // class demand (cpu, mem, gpu, part)
    ClsHdr hdr[CLS_MAX];
    ClsRec rec[CLS_REC];
    int4 jring[CLS_JR];              // (q, class, wall, k) of the staged jobs
    unsigned long long pool[CLS_POOL];
    uint16_t set[CLS_MAX][CLS_SET];
    ClsRec sink[64];                 // the decider's lanes 1..63 store here instead of branching
};

__device__ __forceinline__ unsigned lds_ld(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// v_writelane_b32: lane `l` of `old` := uniform x (no clang builtin on this toolchain)
__device__ __forceinline__ int32_t cls_writelane(int32_t x, int l, int32_t old) {
    int32_t r;
    asm("v_writelane_b32 %0, %1, m0" : "=v"(r) : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(l), "0"(old));
    return r;
}
__device__ __forceinline__ uint4 ld_prog(const unsigned* p) {  // the bookkeepers' progress words
    uint4 v;
    v.x = lds_ld(p);
    v.y = lds_ld(p + 1);
    v.z = lds_ld(p + 2);
    v.w = 0u;
    return v;
}
__device__ __forceinline__ void cls_acq() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void cls_rel() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }

// SPEC §2 key of a row for a demand; the walltime test only when WALL (sets are walltime-free)
template <bool WALL>
__device__ __forceinline__ uint64_t cls_key(const int4 r, int32_t dc, int32_t dm, int32_t dg, int32_t w,
                                            uint32_t pos) {
    const int32_t a = r.x - dc, b = r.y - dm, g = r.z - dg;
    const bool ok = WALL ? ((a | b | g | (r.w - w)) >= 0) : ((a | b | g) >= 0);
    const uint32_t sc = (min((uint32_t)g, 255u) << 24) | (min((uint32_t)a, 4095u) << 12) |
                        min((uint32_t)b >> 10, 4095u);
    return ok ? (((uint64_t)sc << 32) | pos) : KEY_INF;
}

__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// ---- classify: a dense class id per job and component (two launches over all jobs) -----------
__device__ __forceinline__ uint64_t cls_hash(int32_t a, int32_t b, int32_t c, int32_t d) {
    uint64_t z = ((uint64_t)(uint32_t)a << 32 | (uint32_t)b) * 0x9E3779B97F4A7C15ull;
    z ^= ((uint64_t)(uint32_t)c << 32 | (uint32_t)d) + 0xBF58476D1CE4E5B9ull + (z << 6) + (z >> 2);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Two launches, so that the lookups need no acquire: INSERT puts every distinct (partition, cpu,
// mem, gpu) of a component into its hash table (the first inserter of a tuple also numbers it and
// stores its demand); LOOKUP, after the kernel boundary has made the table visible, finds each
// job's tuple with plain loads and checks it field by field.  Two tuples with one 64-bit tag (the
// second one's insert stops at the first one's slot) end in a failed lookup, which makes the
// component ineligible — the placement then runs the persistent engine.
__device__ __forceinline__ bool cls_job_tuple(int q, const int8_t* __restrict__ jcomp, const int32_t* __restrict__ jcpu,
                                              const int32_t* __restrict__ jmem, const int32_t* __restrict__ jgpu,
                                              const uint16_t* __restrict__ jpart, int* c, int4* t) {
    const int jc = jcomp[q];
    if (jc < 0) return false;  // rejected or invalid: never placed by the engine
    *c = jc & 0x3f;            // k_prefilter tags a multi-node job's component with 0x40
    *t = make_int4(jcpu[q], jmem[q], jgpu[q], jpart[q]);
    return true;
}

__global__ __launch_bounds__(256) void k_classify(const int8_t* __restrict__ jcomp,
                                                  const int32_t* __restrict__ jcpu,
                                                  const int32_t* __restrict__ jmem,
                                                  const int32_t* __restrict__ jgpu,
                                                  const uint16_t* __restrict__ jpart, int32_t nj,
                                                  ClsSlot* __restrict__ tab, int4* __restrict__ dem,
                                                  int32_t* __restrict__ ncls) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nj) return;
    int c;
    int4 t;
    if (!cls_job_tuple(q, jcomp, jcpu, jmem, jgpu, jpart, &c, &t)) return;
    const uint64_t h = cls_hash(t.x, t.y, t.z, t.w);
    const unsigned long long tag = h | 1ull;
    ClsSlot* T = tab + (size_t)c * CLS_TS;
    unsigned s = (unsigned)h & (CLS_TS - 1);
    for (int probe = 0; probe < CLS_TS; ++probe) {
        unsigned long long cur = __hip_atomic_load(&T[s].tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == 0ull) {
            unsigned long long exp = 0ull;
            if (__hip_atomic_compare_exchange_strong(&T[s].tag, &exp, tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                T[s].cpu = t.x;
                T[s].mem = t.y;
                T[s].gpu = t.z;
                T[s].part = t.w;
                const int nid = atomicAdd(&ncls[c], 1);
                if (nid < CLS_MAX) dem[(size_t)c * CLS_MAX + nid] = t;
                T[s].idp = nid + 1;  // read by the lookup launch
                return;
            }
            cur = exp;
        }
        if (cur == tag) return;  // this tuple (or a tag twin, caught by the lookup) is in
        s = (s + 1) & (CLS_TS - 1);
    }
    atomicMax(&ncls[c], CLS_TS);  // table full: the component is not eligible
}

__global__ __launch_bounds__(256) void k_classify_lookup(const int8_t* __restrict__ jcomp,
                                                         const int32_t* __restrict__ jcpu,
                                                         const int32_t* __restrict__ jmem,
                                                         const int32_t* __restrict__ jgpu,
                                                         const uint16_t* __restrict__ jpart, int32_t nj,
                                                         const ClsSlot* __restrict__ tab,
                                                         int32_t* __restrict__ ncls, int16_t* __restrict__ jcls) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nj) return;
    int c;
    int4 t;
    if (!cls_job_tuple(q, jcomp, jcpu, jmem, jgpu, jpart, &c, &t)) return;
    const uint64_t h = cls_hash(t.x, t.y, t.z, t.w);
    const unsigned long long tag = h | 1ull;
    const ClsSlot* T = tab + (size_t)c * CLS_TS;
    unsigned s = (unsigned)h & (CLS_TS - 1);
    int id = -1;
    for (int probe = 0; probe < CLS_TS; ++probe) {
        const ClsSlot& e = T[s];
        if (e.tag == 0ull) break;
        if (e.tag == tag) {
            if (e.cpu == t.x && e.mem == t.y && e.gpu == t.z && e.part == t.w) id = e.idp - 1;
            break;
        }
        s = (s + 1) & (CLS_TS - 1);
    }
    jcls[q] = (int16_t)(id >= 0 && id < CLS_MAX ? id : -1);
    if (id < 0) atomicMax(&ncls[c], CLS_TS);  // not found (a tag twin): the component is not eligible
}

// ---- block operations (every wave, between barriers) ------------------------------------------
// Returns the op.  REFILL: S_c, cnt_c, L_c from the current rows (written by wave 0 after the pool
// is built).  PICK: the k smallest keys with the walltime, in ctl.pick[0..npick).
__device__ __forceinline__ unsigned cls_block_op(ClsLds* S, const int4* rows, int32_t n, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    CLS_OPT(o0);
    __syncthreads();  // A: the op's parameters
    CLS_OPT(o1);
    const unsigned op = S->ctl.op;
    if (op == CLS_OP_EXIT) return op;
    const unsigned cl = S->ctl.op_cls;
    const int4 d = S->dem[cl];
    if (op == CLS_OP_REFILL) {
        uint64_t k1 = KEY_INF, k2 = KEY_INF;  // this thread's two smallest keys
#pragma unroll
        for (int i = 0; i < CLS_NPT; ++i) {
            if (i * CLS_THREADS >= n) break;  // uniform: the rows end
            const int p = tid + CLS_THREADS * i;
            if (p < n) {
                const uint64_t k = cls_key<false>(rows[p], d.x, d.y, d.z, 0, (uint32_t)p);
                const bool lt1 = k < k1;
                k2 = lt1 ? k1 : umin64(k2, k);
                k1 = lt1 ? k : k1;
            }
        }
        const uint64_t m = wave_min_key(k2);
        if (lane == 0) S->ctl.red[0][wave] = m;
        __syncthreads();  // B1
        CLS_OPT(o2);
        uint64_t B = S->ctl.red[0][0];
#pragma unroll
        for (int i = 1; i < 8; ++i) B = umin64(B, S->ctl.red[0][i]);
        // every node of this thread other than k1 is >= its k2 >= B: the threads' k1 below B are
        // every node below B (≈ 32 of them: a set with room, so the bookkeepers' inserts do not
        // lower the bound at once — three keys per thread filled the set and doubled the refills)
        if (k1 < B) {
            const unsigned idx = atomicAdd(&S->ctl.pool_n, 1u);
            S->pool[idx] = k1;
        }
        __syncthreads();  // B2
        CLS_OPT(o3);
        if (wave == 0) {
            const unsigned P = (unsigned)__builtin_amdgcn_readfirstlane((int)S->ctl.pool_n);
            uint64_t e[CLS_POOL / 64];
#pragma unroll
            for (int j = 0; j < CLS_POOL / 64; ++j) {  // only the chunks the pool reaches (≈ 32 keys)
                e[j] = KEY_INF;
                if ((unsigned)(64 * j) < P) {
                    const unsigned i = lane + 64 * j;
                    e[j] = i < P ? S->pool[i] : KEY_INF;
                }
            }
            uint64_t T = B;  // the new bound
            if (P > (unsigned)CLS_SET) {
                // T = the (CLS_SET + 1)-th smallest pool key: quickselect on (lo, hi) with the
                // first in-range key as the pivot (the pool is in arrival order).  Should it not
                // converge, T = the smallest key: an empty set and a valid bound (the job then
                // takes the exact path)
                uint64_t lo = 0ull, hi = KEY_INF, tmin = KEY_INF;
#pragma unroll
                for (int j = 0; j < CLS_POOL / 64; ++j) tmin = umin64(tmin, e[j]);
                tmin = wave_min_key(tmin);
                T = tmin;
                for (int it = 0; it < 4 * CLS_POOL; ++it) {
                    uint64_t piv = KEY_INF;
#pragma unroll
                    for (int j = 0; j < CLS_POOL / 64; ++j) {
                        const uint64_t bal = __ballot(e[j] >= lo && e[j] < hi);
                        if (piv == KEY_INF && bal) piv = rdlane64(e[j], __builtin_ctzll(bal));
                    }
                    unsigned cntl = 0;
#pragma unroll
                    for (int j = 0; j < CLS_POOL / 64; ++j) cntl += (unsigned)__popcll(__ballot(e[j] < piv));
                    if (cntl == (unsigned)CLS_SET) {
                        T = piv;
                        break;
                    }
                    if (cntl < (unsigned)CLS_SET) lo = piv + 1;
                    else hi = piv;
                }
            }
            unsigned base = 0;
#pragma unroll
            for (int j = 0; j < CLS_POOL / 64; ++j) {
                if ((unsigned)(64 * j) >= P) break;  // uniform
                const bool in = e[j] < T;
                const uint64_t bal = __ballot(in);
                if (in) S->set[cl][base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
                    (uint16_t)(uint32_t)e[j];
                base += (unsigned)__popcll(bal);
            }
            if (lane == 0) {
                S->hdr[cl].cnt = base;
                S->hdr[cl].L = T;
            }
        }
        CLS_OPT(o4);
        __syncthreads();  // C: the new set and bound
        CLS_OPT(o5);
        CLS_OPADD(0, o0, o1);
        CLS_OPADD(1, o1, o2);
        CLS_OPADD(2, o2, o3);
        CLS_OPADD(3, o3, o4);
        CLS_OPADD(4, o4, o5);
        CLS_OPADD(5, 0ull, 1ull);
        return op;
    }
    // CLS_OP_PICK: exact k smallest with the walltime (extraction r excludes keys <= prev)
    const int32_t w = S->ctl.op_wall;
    const unsigned k = S->ctl.op_k;
    uint64_t prev = 0ull;
    unsigned got = 0;
    for (unsigned r = 0; r < k; ++r) {
        uint64_t m = KEY_INF;
#pragma unroll
        for (int i = 0; i < CLS_NPT; ++i) {
            if (i * CLS_THREADS >= n) break;  // uniform: the rows end
            const int p = tid + CLS_THREADS * i;
            if (p < n) {
                const uint64_t key = cls_key<true>(rows[p], d.x, d.y, d.z, w, (uint32_t)p);
                if ((r == 0 || key > prev) && key < m) m = key;
            }
        }
        const uint64_t wm = wave_min_key(m);
        if (lane == 0) S->ctl.red[r & 1][wave] = wm;
        __syncthreads();
        uint64_t g = S->ctl.red[r & 1][0];
#pragma unroll
        for (int i = 1; i < 8; ++i) g = umin64(g, S->ctl.red[r & 1][i]);
        if (g == KEY_INF) break;  // block-uniform
        prev = g;
        if (tid == 0) S->ctl.pick[r] = g;
        got = r + 1;
    }
    if (tid == 0) S->ctl.npick = got;
    __syncthreads();  // C
    return op;
}

// ---- the decider's block-operation call ---------------------------------------------------------
struct ClsDec {
    unsigned ncommit;
    unsigned epoch;
    bool fail;
};

__device__ __forceinline__ bool cls_drain(ClsLds* S, unsigned ncommit) {
    for (int b = 0; b < CLS_BK; ++b) {
        unsigned sp = 0;
        while (lds_ld(&S->ctl.prog[b]) != ncommit)
            if (++sp > CLS_SPIN) return false;
    }
    cls_acq();
    return true;
}

__device__ __forceinline__ void cls_request(ClsLds* S, ClsDec& D, unsigned op, unsigned cl, int32_t w, unsigned k) {
    if ((threadIdx.x & 63) == 0) {
        S->ctl.op = op;
        S->ctl.op_cls = cl;
        S->ctl.op_wall = w;
        S->ctl.op_k = k;
        S->ctl.pool_n = 0;
    }
    cls_rel();
    if ((threadIdx.x & 63) == 0) lds_st(&S->ctl.op_epoch, ++D.epoch);
    else ++D.epoch;
}

// ---- the engine -----------------------------------------------------------------------------
struct ClsComps {
    int32_t nb[33];
    uint32_t owned;  // bit c: this rank places component c (component sharding; all at world 1)
};

__global__ __launch_bounds__(CLS_THREADS) void k_class(
    NodeRec* __restrict__ rec, ClsComps C, const int32_t* __restrict__ jb, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jwall, const uint16_t* __restrict__ jk, const int16_t* __restrict__ jcls,
    const int4* __restrict__ gdem, const int32_t* __restrict__ gncls, int32_t kmax, int32_t* __restrict__ out,
    CompOut* __restrict__ co, unsigned* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (!((C.owned >> c) & 1u)) return;  // another rank's component (merged after the launch)
    const int32_t nb = C.nb[c], n = C.nb[c + 1] - nb;
    int4* rows = reinterpret_cast<int4*>(smem);
    ClsLds* S = reinterpret_cast<ClsLds*>(smem + sizeof(int4) * (size_t)((n + 7) & ~7));
    const unsigned ncls = (unsigned)gncls[c];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // ---- load: rows, class demands, empty sets with L = 0 (nothing certified: a class's first
    // query refills its set)
    for (int p = tid; p < n; p += CLS_THREADS) {
        const NodeRec r = rec[nb + p];
        rows[p] = make_int4(r.cpu, r.mem, r.gpu, r.avail);
    }
    for (int i = tid; i < CLS_MAX * CLS_SET / 2; i += CLS_THREADS)
        reinterpret_cast<uint32_t*>(&S->set[0][0])[i] = 0u;  // entries past a count: position 0
    for (int i = tid; i < CLS_MAX; i += CLS_THREADS) {
        S->dem[i] = i < (int)ncls ? gdem[(size_t)c * CLS_MAX + i] : make_int4(0, 0, 0, 0);
        S->hdr[i].cnt = 0u;
        S->hdr[i].pad = 0u;
        S->hdr[i].L = 0ull;
    }
    if (tid == 0) {
        S->ctl.ncommit = 0;
        S->ctl.staged = jb[c];
        S->ctl.jdone = jb[c];
        for (int b = 0; b < 4; ++b) S->ctl.prog[b] = 0;
        S->ctl.op_epoch = 0;
        S->ctl.op = 0;
        S->ctl.ncls = ncls;
    }
    __syncthreads();

    if (wave == 0) {
        // ================= DECIDER =================
        // While job t is decided, the next job's class header, demand, set entries and bookkeeper
        // progress (A) are already in flight; its candidates' rows (B) are read after job t's
        // commits, so they are current.  A k-node job commits all its picks at once, one lane
        // each (its row from LDS, its record, its new row) with one count store.
        ClsDec D{0u, 0u, false};
        int64_t placed = 0, refills = 0, picks = 0, lowers = 0, evals = 0;
#ifdef FIT_STAMPS
        unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
        const int32_t t0j = jb[c], t1j = jb[c + 1];
        // job fields from the staged ring (wave 4 copies them from HBM ahead of the decider, so the
        // decider's loop issues no vector-memory instruction: a vmcnt wait there would also wait for
        // stores)
        struct JobF {
            int32_t q, cl, w, k;
        };
        int32_t staged_seen = t0j;
        auto ring_at = [&](int32_t t) {  // raw (per-lane copies), consumed a step later
            unsigned sp = 0;
            while (staged_seen <= t && ++sp <= CLS_SPIN)
                staged_seen = __builtin_amdgcn_readfirstlane((int)lds_ld(reinterpret_cast<unsigned*>(&S->ctl.staged)));
            CLS_CBAR();
            return S->jring[t & (CLS_JR - 1)];
        };
        auto conv = [&](const int4 v) {
            JobF f;
            f.q = __builtin_amdgcn_readfirstlane(v.x);
            f.cl = __builtin_amdgcn_readfirstlane(v.y);
            f.w = __builtin_amdgcn_readfirstlane(v.z);
            f.k = __builtin_amdgcn_readfirstlane(v.w);
            return f;
        };
        int32_t rpos = -1;  // lanes CLS_SET..63: the last CLS_RING committed positions
        // A (issued one job ahead, consumed a job later): class header (cnt, L) and demand, the
        // set entry of this lane, the bookkeepers' progress — progress first: the set read must not
        // be older than the progress it is checked against
        struct QA {
            uint32_t cnt;        // raw (per-lane copies of one value)
            uint64_t L;
            int4 d;
            int32_t sp;
            uint4 pg;
        };
        auto load_a = [&](int32_t cl) {
            QA a;
            a.pg = ld_prog(S->ctl.prog);
            CLS_CBAR();
            const ClsHdr h = S->hdr[cl];
            a.cnt = h.cnt;
            a.L = h.L;
            a.d = S->dem[cl];
            a.sp = lane < CLS_SET ? (int32_t)S->set[cl][lane] : -1;
            return a;
        };
        // the candidates' positions: set entries below the count, then the ring
        auto cand_pos = [&](const QA& a) {
            const int cnt = min((int)__builtin_amdgcn_readfirstlane((int)a.cnt), CLS_SET);
            const int32_t p = lane < CLS_SET ? (lane < cnt ? a.sp : -1) : rpos;
            return p < n ? p : -1;
        };
        // the job's picks, parked one per lane (lane j = pick j's position; pick 0 in x0)
        uint32_t pkl = 0;
        // query: the k smallest distinct candidate keys; returns how many were found and the k-th
        int32_t x0 = 0;  // the first pick (SGPR): a k = 1 job parks nothing
        auto extract = [&](uint64_t key, int k, uint64_t& kth) {
            int ln = 0;
            uint64_t m = wave_min_key_lane(key, ln);
            kth = m;
            x0 = (int32_t)(uint32_t)m;
            if (m == KEY_INF) return 0;
            int np = 1;
            for (int j = 1; j < k; ++j) {  // uniform; multi-node jobs only
                key = key == m ? KEY_INF : key;
                m = wave_min_key_lane(key, ln);
                if (m == KEY_INF) break;
                pkl = (uint32_t)cls_writelane((int)(uint32_t)m, j, (int)pkl);
                kth = m;
                np = j + 1;
            }
            return np;
        };
        JobF F{0, 0, 0, 1}, F1{0, 0, 0, 1};
        int4 rj2 = make_int4(0, 0, 0, 1);
        QA A{0u, 0ull, make_int4(0, 0, 0, 0), -1, make_uint4(0, 0, 0, 0)};
        int32_t pos = -1;
        int4 row = make_int4(0, 0, 0, 0);
        if (t0j < t1j) {
            F = conv(ring_at(t0j));
            if (t0j + 1 < t1j) F1 = conv(ring_at(t0j + 1));
            if (t0j + 2 < t1j) rj2 = ring_at(t0j + 2);
            A = load_a(F.cl);
            pos = cand_pos(A);
            row = rows[pos >= 0 ? pos : 0];
        }
        for (int32_t t = t0j; t < t1j; ++t) {
            CLS_T(tj0);
            if (F.cl < 0 || F.cl >= (int)ncls) {
                D.fail = true;
                break;
            }
            const bool has_next = t + 1 < t1j;
            // ---- query job t: its candidates' keys first (the rows were read at the end of the
            // previous step, after its commits: current, nothing to patch)
            const int4 d = make_int4(__builtin_amdgcn_readfirstlane(A.d.x), __builtin_amdgcn_readfirstlane(A.d.y),
                                     __builtin_amdgcn_readfirstlane(A.d.z), 0);
            uint64_t Lc = rdlane64(A.L, 0);
            const uint64_t key0 = pos >= 0 ? cls_key<true>(row, d.x, d.y, d.z, F.w, (uint32_t)pos) : KEY_INF;
            asm volatile("" ::"v"((uint32_t)key0), "v"((uint32_t)(key0 >> 32)) : "memory");
            CLS_T(tq1);
            // then A(t+1) and job t+3's fields, in flight during the extraction
            QA A1 = load_a(has_next ? F1.cl : 0);
            const int4 rj3 = t + 3 < t1j ? ring_at(t + 3) : make_int4(0, 0, 0, 1);
            *(lane == 0 ? &S->ctl.jdone : &S->sink[lane].x) = t;  // ring entries below t are free
            CLS_T(tq2);
            int np;
            uint64_t kth;
            bool reload_next = false;
            np = extract(key0, F.k, kth);
            evals += 64;
            // the k-th pick below the bound, or the bound infinite: exact (np < k: unplaced)
            bool certified = Lc == KEY_INF || (np == F.k && kth < Lc);
            CLS_T(tj1);
            if (!certified) {
                // ---- exhausted: the workgroup refills the class's set and the job is queried
                // again; if the walltime or k still defeats the fresh set it is resolved exactly
                if (!cls_drain(S, D.ncommit)) {
                    D.fail = true;
                    break;
                }
                CLS_T(tdr);
                CLS_ACC(5, tj1, tdr);  // stamps: the drain's share of a refill
                cls_request(S, D, CLS_OP_REFILL, (unsigned)F.cl, 0, 0);
                cls_block_op(S, rows, n, tid);
                ++refills;
                evals += n;
                A = load_a(F.cl);
                pos = cand_pos(A);
                const int4 rq = rows[pos >= 0 ? pos : 0];
                Lc = rdlane64(A.L, 0);
                np = extract(pos >= 0 ? cls_key<true>(rq, d.x, d.y, d.z, F.w, (uint32_t)pos) : KEY_INF, F.k, kth);
                evals += 64;
                certified = Lc == KEY_INF || (np == F.k && kth < Lc);
                if (!certified) {
                    cls_request(S, D, CLS_OP_PICK, (unsigned)F.cl, F.w, (unsigned)F.k);
                    cls_block_op(S, rows, n, tid);
                    np = (int)S->ctl.npick;
                    // lane j < np: pick j
                    const uint64_t m = lane < np ? S->ctl.pick[lane < FIT_KMAX ? lane : 0] : 0ull;
                    pkl = (uint32_t)m;
                    x0 = (int32_t)(uint32_t)S->ctl.pick[0];
                    ++picks;
                    evals += (int64_t)F.k * n;
                }
                reload_next = true;  // a refill may have replaced the next job's set
            }
            CLS_T(tj2);
            CLS_T(tb1);
            // ---- commit job t (all or nothing: np == k), every pick at once: lane j < k takes
            // pick j — its current row from LDS (each pick is a distinct node), its record in
            // ring slot ncommit + j, its new row; then one count store for all of them
            if (np == F.k) {
                ++placed;
                {  // every record slot this job writes must be free (all bookkeepers past it)
                    unsigned pmin = min(min((unsigned)__builtin_amdgcn_readfirstlane((int)A.pg.x),
                                            (unsigned)__builtin_amdgcn_readfirstlane((int)A.pg.y)),
                                        (unsigned)__builtin_amdgcn_readfirstlane((int)A.pg.z));
                    unsigned sp = 0;
                    while (pmin + (unsigned)CLS_REC < D.ncommit + (unsigned)F.k && ++sp <= CLS_SPIN) {
                        const uint4 g = ld_prog(S->ctl.prog);
                        pmin = min(min((unsigned)__builtin_amdgcn_readfirstlane((int)g.x),
                                       (unsigned)__builtin_amdgcn_readfirstlane((int)g.y)),
                                   (unsigned)__builtin_amdgcn_readfirstlane((int)g.z));
                    }
                    if (sp > CLS_SPIN) {
                        D.fail = true;
                        break;
                    }
                }
                const bool pk = lane < F.k;
                const int32_t xl = lane == 0 ? x0 : (int32_t)pkl;  // lane j < k: pick j's position
                const int4 o = rows[pk ? xl : 0];
                const int4 nw = make_int4(o.x - d.x, o.y - d.y, o.z - d.z, o.w);
                // lanes past k store into their own sink slots (no branch on the chain)
                ClsRec* rp = pk ? &S->rec[(D.ncommit + (unsigned)lane) & (CLS_REC - 1)] : &S->sink[lane];
                *reinterpret_cast<int4*>(&rp->x) = make_int4(xl, o.x, o.y, o.z);
                *reinterpret_cast<int4*>(&rp->nc) = make_int4(nw.x, nw.y, nw.z, F.q * kmax + lane);
                CLS_CBAR();  // records, then the count (one wave's LDS operations run in order)
                const unsigned n0 = D.ncommit;
                D.ncommit += (unsigned)F.k;
                *(lane == 0 ? &S->ctl.ncommit : reinterpret_cast<unsigned*>(&S->sink[lane].oc)) = D.ncommit;
                *(pk ? &rows[xl] : reinterpret_cast<int4*>(&S->sink[lane].nc)) = nw;
                // ring lanes CLS_SET..63: commit n0 + j lands in lane CLS_SET + ((n0 + j) & 7)
                const int jr = (int)(((unsigned)(lane - CLS_SET) - n0) & (unsigned)(CLS_RING - 1));
                const int32_t xr = __builtin_amdgcn_ds_bpermute(jr << 2, xl);
                if (lane >= CLS_SET && jr < F.k) rpos = xr;
                evals += 2 * (int64_t)ncls * F.k;  // the bookkeepers' old / new key of every class
#ifdef FIT_STAMPS
                st_acc[7] += (unsigned long long)F.k;
#endif
            }
            CLS_T(tj3);
#ifdef FIT_STAMPS
            st_acc[1] += tq1 - tj0;   // head: key
            st_acc[3] += tq2 - tq1;   // A(t+1) issue, ring
            st_acc[0] += tj1 - tq2;   // extraction, certification
            st_acc[2] += tj2 - tj1;
            st_acc[4] += tj3 - tb1;   // commit
            st_acc[6] += 1;
#endif
            if (!has_next) break;
            // ---- the next job's bookkeeper must be within the ring of this moment
            {
                const int b1 = F1.cl >> 6;
                const unsigned need = D.ncommit > (unsigned)CLS_RING ? D.ncommit - (unsigned)CLS_RING : 0u;
                const unsigned pb = (unsigned)__builtin_amdgcn_readfirstlane(
                    (int)(b1 == 0 ? A1.pg.x : (b1 == 1 ? A1.pg.y : A1.pg.z)));
                if (pb < need) {
                    CLS_T(tw0);
                    unsigned sp = 0;
                    while (lds_ld(&S->ctl.prog[b1]) < need && ++sp <= CLS_SPIN) {
                    }
                    if (sp > CLS_SPIN) {
                        D.fail = true;
                        break;
                    }
                    reload_next = true;
                    CLS_T(tw1);
                }
            }
            if (reload_next) A1 = load_a(F1.cl);  // re-read A for the next job now
            // B(t+1): the next job's candidate rows, after this job's commits (current rows)
            pos = cand_pos(A1);
            row = rows[pos >= 0 ? pos : 0];
            F = F1;
            F1 = conv(rj2);
            rj2 = rj3;
            A = A1;
        }
        // drain, then the exit op (a failed drain still exits: the error word says why)
        const bool drained = cls_drain(S, D.ncommit);
        if (!drained || D.fail) {
            if (lane == 0) atomicOr(err, 1u);
        }
        cls_request(S, D, CLS_OP_EXIT, 0, 0, 0);
        cls_block_op(S, rows, n, tid);
#ifdef FIT_STAMPS
        if (lane == 0)
            for (int i = 0; i < 8; ++i) g_cls_st[c & 31][i] = st_acc[i];
#endif
        if (lane == 0) {
            CompOut o;
            o.evals = evals;
            o.placed = placed;
            o.done_jobs = t1j - t0j;
            o.rounds = refills;
            o.stops_rescan = picks;
            o.stops_dirty = lowers;
            o.t_commit = (int64_t)(__builtin_amdgcn_s_memrealtime() - t0);
            o.t_wait = 0;
            co[c] = o;
        }
    } else if (wave <= CLS_BK) {
        // ================= BOOKKEEPER =================
        const int b = wave - 1;
        const unsigned cls = (unsigned)(b * 64 + lane);
        const bool valid = cls < ncls;
        const int4 d = valid ? S->dem[cls] : make_int4(0, 0, 0, 0);
        uint64_t myL = valid ? S->hdr[cls].L : 0ull;
        unsigned mycnt = valid ? S->hdr[cls].cnt : 0u;
        unsigned probe_at = 0;  // the next set slot a full set's insert probes for a dead entry
        unsigned p = 0, ep = 0;
        for (;;) {
            const unsigned nc = lds_ld(&S->ctl.ncommit);
            CLS_CBAR();  // the record is read after the count that published it
            if (p < nc) {
                const ClsRec R = S->rec[p & (CLS_REC - 1)];
                if (b == 0 && lane == 0) out[R.oi] = nb + R.x;  // position; k_class_out maps it to the id
                const uint64_t kn = cls_key<false>(make_int4(R.nc, R.nm, R.ng, 0), d.x, d.y, d.z, 0, (uint32_t)R.x);
                const bool cand = valid && kn < myL;
                if (__ballot(cand)) {
                    // membership by the old key: listed nodes are below the bound (or were, before a
                    // lowering: then x is re-offered and only lowers the bound again — no duplicate,
                    // a full set takes no entry)
                    const uint64_t ko = cls_key<false>(make_int4(R.oc, R.om, R.og, 0), d.x, d.y, d.z, 0, (uint32_t)R.x);
                    const bool ins = cand && !(ko < myL);
                    if (ins) {
                        if (mycnt < (unsigned)CLS_SET) {
                            S->set[cls][mycnt] = (uint16_t)R.x;
                            ++mycnt;
                            CLS_CBAR();  // entry, then count
                            lds_st(&S->hdr[cls].cnt, mycnt);
                        } else {
                            // full: x takes the slot of a dead entry — a node the class no longer
                            // fits at the current rows, which only shrink (a torn row read mixes
                            // old and new values, so "does not fit" is never wrong) — found among
                            // a few probes from a rotating cursor; else the bound falls to x's key
                            // and x stays out.  A concurrent query sees the dead node or x (x is in
                            // the decider's ring): either is harmless.
                            bool took = false;
                            for (int pr = 0; pr < CLS_PROBE && !took; ++pr) {
                                const unsigned i = probe_at;
                                probe_at = probe_at + 1u < (unsigned)CLS_SET ? probe_at + 1u : 0u;
                                const int y = S->set[cls][i];
                                if (cls_key<false>(rows[y], d.x, d.y, d.z, 0, (uint32_t)y) == KEY_INF) {
                                    S->set[cls][i] = (uint16_t)R.x;
                                    took = true;
                                }
                            }
                            if (!took) {
                                myL = kn;
                                S->hdr[cls].L = kn;
                            }
                        }
                    }
                }
                CLS_CBAR();
                ++p;
                lds_st(&S->ctl.prog[b], p);
                continue;
            }
            const unsigned e = lds_ld(&S->ctl.op_epoch);
            if (e != ep) {
                ep = e;
                const unsigned op = cls_block_op(S, rows, n, tid);
                if (op == CLS_OP_EXIT) break;
                if (valid) {
                    myL = S->hdr[cls].L;
                    mycnt = S->hdr[cls].cnt;
                }
                continue;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    } else if (wave == CLS_BK + 1) {
        // ================= JOB STAGER (and block operations) =================
        // The component's job list → (q, class, wall, k) in the LDS ring, a chunk of 64 jobs per
        // step in a three-stage pipeline (list entries; then the job columns they index; then the
        // ring), so every wait here is for loads issued a step earlier; between steps the wave
        // polls for block operations like the bookkeepers.
        const int32_t t0j = jb[c], t1j = jb[c + 1];
        unsigned ep = 0;
        int32_t a_base = -1, a_q = 0, a_c = 0, a_w = 0, a_k = 1;  // chunk whose columns are loaded
        int32_t b_base = -1, b_q = 0;                            // chunk whose list entries are loaded
        if (t0j < t1j) {
            b_base = t0j;
            if (t0j + lane < t1j) b_q = jl[t0j + lane];
        }
        for (;;) {
            const unsigned e = lds_ld(&S->ctl.op_epoch);
            if (e != ep) {
                ep = e;
                if (cls_block_op(S, rows, n, tid) == CLS_OP_EXIT) break;
                continue;
            }
            bool work = false;
            if (a_base >= 0) {
                const int32_t jd = __builtin_amdgcn_readfirstlane(lds_ld(reinterpret_cast<unsigned*>(&S->ctl.jdone)));
                if (a_base + 64 <= jd + CLS_JR) {
                    if (a_base + lane < t1j) S->jring[(a_base + lane) & (CLS_JR - 1)] = make_int4(a_q, a_c, a_w, a_k);
                    CLS_CBAR();  // entries, then the count
                    lds_st(reinterpret_cast<unsigned*>(&S->ctl.staged), (unsigned)min(a_base + 64, t1j));
                    a_base = -1;
                    work = true;
                }
            }
            if (a_base < 0 && b_base >= 0) {
                a_base = b_base;
                a_q = b_q;
                if (a_base + lane < t1j) {
                    a_c = jcls[a_q];
                    a_w = jwall[a_q];
                    a_k = jk ? max((int)jk[a_q], 1) : 1;
                }
                b_base = b_base + 64 < t1j ? b_base + 64 : -1;
                if (b_base >= 0 && b_base + lane < t1j) b_q = jl[b_base + lane];
                work = true;
            }
            if (!work) __builtin_amdgcn_s_sleep(2);
        }
    } else {
        // ================= block-operation waves =================
        for (;;)
            if (cls_block_op(S, rows, n, tid) == CLS_OP_EXIT) break;
    }
    __syncthreads();
    for (int p = tid; p < n; p += CLS_THREADS) {
        const int4 r = rows[p];
        rec[nb + p].cpu = r.x;
        rec[nb + p].mem = r.y;
        rec[nb + p].gpu = r.z;
    }
}

// positions written by k_class → node ids (rec[pos].orig); FIT_UNPLACED / FIT_REJECTED stay
__global__ __launch_bounds__(256) void k_class_out(int32_t* __restrict__ out, int64_t n,
                                                   const NodeRec* __restrict__ rec) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t v = out[i];
    if (v >= 0) out[i] = rec[v].orig;
}

// ---- host-side entry points ---------------------------------------------------------------------
#ifdef FIT_STAMPS
extern "C" int fit_debug_class_stamps(unsigned long long* out /* 2 x 32 x 8: decider, refill phases */) {
    if (hipMemcpyFromSymbol(out + 32 * 8, HIP_SYMBOL(g_cls_op), sizeof(g_cls_op)) != hipSuccess) return -2;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cls_st), sizeof(g_cls_st)) == hipSuccess ? 0 : -2;
}
#endif
size_t class_lds_bytes(int32_t max_component_nodes) {
    return sizeof(int4) * (size_t)((max_component_nodes + 7) & ~7) + sizeof(ClsLds);
}
int class_max() { return CLS_MAX; }
int class_table_slots() { return CLS_TS; }
size_t class_slot_bytes() { return sizeof(ClsSlot); }
int class_max_nodes() { return CLS_THREADS * CLS_NPT; }

hipError_t launch_classify(hipStream_t st, const int8_t* jcomp, const int32_t* jcpu, const int32_t* jmem,
                           const int32_t* jgpu, const uint16_t* jpart, int32_t nj, void* tab, int4* dem,
                           int32_t* ncls, int16_t* jcls) {
    if (nj <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_classify, dim3((nj + 255) / 256), dim3(256), 0, st, jcomp, jcpu, jmem, jgpu, jpart, nj,
                       static_cast<ClsSlot*>(tab), dem, ncls);
    hipLaunchKernelGGL(k_classify_lookup, dim3((nj + 255) / 256), dim3(256), 0, st, jcomp, jcpu, jmem, jgpu, jpart,
                       nj, static_cast<const ClsSlot*>(tab), ncls, jcls);
    return hipGetLastError();
}

hipError_t launch_class(hipStream_t st, int ncomp, size_t lds, NodeRec* rec, const int32_t* nbv, uint32_t owned,
                        const int32_t* jb, const int32_t* jl, const int32_t* jwall, const uint16_t* jk,
                        const int16_t* jcls, const int4* dem, const int32_t* ncls, int32_t kmax, int32_t* out,
                        CompOut* co, unsigned* err) {
    if (ncomp <= 0 || ncomp > 32) return hipErrorInvalidValue;
    ClsComps C;
    for (int k = 0; k <= 32; ++k) C.nb[k] = nbv[k < ncomp ? k : ncomp];
    C.owned = owned;
    hipLaunchKernelGGL(k_class, dim3(ncomp), dim3(CLS_THREADS), lds, st, rec, C, jb, jl, jwall, jk, jcls, dem, ncls,
                       kmax, out, co, err);
    return hipGetLastError();
}

hipError_t launch_class_out(hipStream_t st, int32_t* out, int64_t n, const NodeRec* rec) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_class_out, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n, rec);
    return hipGetLastError();
}

}  // namespace fitgpu
