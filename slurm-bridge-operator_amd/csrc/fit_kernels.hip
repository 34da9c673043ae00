// fit_kernels.hip — hand-written CDNA4 (gfx950) kernels of the batched best-fit engine.
//
// DESIGN.md §3.  Two kernels per speculative round:
//   k_scan   : every window job × every node of its partition component (this rank's shard),
//              lanes = jobs, node rows wave-uniform (scalar loads → SGPRs), per-lane sorted
//              top-KS of the packed key (score << 32 | position) in VGPRs.  No MFMA: integer
//              compares / subtracts / mins only (VALU-bound).
//   k_commit : one wave per component walks its window in priority order and resolves each
//              job exactly against (clean candidates ∪ dirty nodes): the speculative-prefix
//              commit.  Dirty rows live in VGPRs (≤ 4 per lane), membership in an LDS bitmap.
// The sequential semantics they reproduce bit-exactly is oracle/fitref.c:ref_place.
#include "fit_common.h"

namespace fitgpu {

__global__ __launch_bounds__(SCAN_WAVES * 64) void k_scan(
    const NodeRec* __restrict__ rec, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, const uint16_t* __restrict__ jk,
    const CompPlan* __restrict__ plan, int ncomp, uint64_t* __restrict__ cand,
    uint64_t* __restrict__ bnd, JobRec* __restrict__ wjob) {
    __shared__ uint64_t xk[SCAN_WAVES / 2][KS][64];  // lane-contiguous: conflict-free b64 access
    const int c = find_comp(plan, ncomp, blockIdx.x);
    const CompPlan P = plan[c];
    const int local = blockIdx.x - P.blk0;
    // integer division expands to VALU code: pin the (uniform) results to SGPRs
    const int tile = __builtin_amdgcn_readfirstlane(local / P.nslice);
    const int s = __builtin_amdgcn_readfirstlane(local - tile * P.nslice);
    scan_tile<false, KS>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, xk);
}

template <int EPL>
__global__ __launch_bounds__(64) void k_commit(
    NodeRec* __restrict__ rec, const CompPlan* __restrict__ plan,
    const uint64_t* __restrict__ cand, int64_t rank_stride, int nranks,
    const uint64_t* __restrict__ bnd, const JobRec* __restrict__ wjob,
    int32_t* __restrict__ out, int kmax, CommitResult* __restrict__ res) {
    extern __shared__ uint32_t bitmap[];
    const int c = blockIdx.x;
    const CompPlan P = plan[c];
    if (P.w == 0) {
        if (threadIdx.x == 0) res[c] = CommitResult{0, 0, 0, 0};
        return;
    }
    const CommitResult R =
        commit_window<EPL>(c, P, rec, cand, rank_stride, nranks, bnd, wjob, out, kmax, bitmap);
    if (threadIdx.x == 0) res[c] = R;
}

// ------------------------------------------------------------------- prefilter / setup
// out[] init, component id per job, rejected marks (FIT_REJECTED) — DESIGN.md §3.1.
// The verdict on job q: -3 invalid job (negative demand or nodes_k > kmax), -2 rejected by its
// partition's limits, -1 partition without nodes, else its component | 0x40 for a multi-node
// job.  *rej (the FIT_REJECTED rows) and *k (rows of the job) for the out[] init.
__device__ __forceinline__ int job_code(int q, const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
                                        const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
                                        const uint16_t* __restrict__ jpart, const uint16_t* __restrict__ jk,
                                        int32_t kmax, const int32_t* __restrict__ ptab, int32_t np,
                                        bool* rej, int* k) {
    const int p = jpart[q];
    *k = jk ? max((int)jk[q], 1) : 1;
    bool r = p >= np;
    if (!r) {
        const int mt = ptab[p], mc = ptab[32 + p], mm = ptab[64 + p];
        r = (mt >= 0 && jwall[q] > mt) || (mc >= 0 && jcpu[q] > mc) || (mm >= 0 && jmem[q] > mm);
    }
    *rej = r;
    int comp = r ? -2 : ptab[96 + p];
    if (comp >= 0 && *k > 1) comp |= 0x40;
    if (*k > kmax || jcpu[q] < 0 || jmem[q] < 0 || jwall[q] < 0 || (jgpu && jgpu[q] < 0)) comp = -3;
    return comp;
}

__global__ void k_prefilter(const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
                            const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall, const uint16_t* __restrict__ jpart,
                            const uint16_t* __restrict__ jk, int32_t nj, int32_t kmax,
                            const int32_t* __restrict__ ptab /* [4][32]: time,cpus,mem,comp */,
                            int32_t np, int32_t* __restrict__ out, int8_t* __restrict__ jcomp) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nj) return;
    bool rej;
    int k;
    jcomp[q] = (int8_t)job_code(q, jcpu, jmem, jgpu, jwall, jpart, jk, kmax, ptab, np, &rej, &k);
    for (int i = 0; i < kmax; ++i) out[(int64_t)q * kmax + i] = (rej && i < k) ? -2 : -1;
}

__global__ void k_gather_nodes(const int32_t* __restrict__ cpu, const int32_t* __restrict__ mem,
                               const int32_t* __restrict__ gpu, const int32_t* __restrict__ av,
                               const uint32_t* __restrict__ mask, const int32_t* __restrict__ perm,
                               int32_t nn, NodeRec* __restrict__ rec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    const int x = perm[i];
    NodeRec r;
    // clamp to >= -1: same feasibility for demands >= 0, no int32 overflow in free - demand
    r.cpu = max(cpu[x], -1);
    r.mem = max(mem[x], -1);
    r.gpu = max(gpu[x], -1);
    r.avail = max(av[x], -1);
    r.mask = mask[x];
    r.orig = x;
    r.pad0 = r.pad1 = 0;
    rec[i] = r;
}

__global__ void k_scatter_nodes(const NodeRec* __restrict__ rec, int32_t nn,
                                int32_t* __restrict__ cpu, int32_t* __restrict__ mem,
                                int32_t* __restrict__ gpu) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    const NodeRec r = rec[i];
    // a clamped (negative) field is never chosen, hence never changed: keep the caller's value
    if (r.cpu >= 0) cpu[r.orig] = r.cpu;
    if (r.mem >= 0) mem[r.orig] = r.mem;
    if (r.gpu >= 0) gpu[r.orig] = r.gpu;
}


// ------------------------------------------------------------------- device job lists
// Per-component job lists in priority order (stable counting sort by component over the
// prefilter's ids), plus jpk (multi-node jobs before each list position) — DESIGN.md §3.1.
// Three passes over blocks of JL_BLOCK jobs: per-(block, component) counts by wave ballots, an
// exclusive scan over blocks per component, and the scatter (block offset + wave offset + lane
// rank), so the order inside each component is the caller's.
constexpr int JL_BLOCK = 1024;
constexpr int JL_MAXC = 32;

__global__ __launch_bounds__(JL_BLOCK) void k_jl_count(const int8_t* __restrict__ jcomp, int32_t nj,
                                                       int ncomp, int32_t* __restrict__ bc,
                                                       int32_t* __restrict__ bm,
                                                       int32_t* __restrict__ g) {
    __shared__ int32_t wc[JL_BLOCK / 64][JL_MAXC], wm[JL_BLOCK / 64][JL_MAXC];
    const int q = blockIdx.x * JL_BLOCK + threadIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k = q < nj ? jcomp[q] : -1;
    const int comp = k >= 0 ? (k & 0x3f) : -1;
    const bool multi = k >= 0 && (k & 0x40);
    for (int cc = 0; cc < ncomp; ++cc) {
        const uint64_t m = __ballot(comp == cc), mm = __ballot(comp == cc && multi);
        if (lane == 0) {
            wc[wave][cc] = __popcll(m);
            wm[wave][cc] = __popcll(mm);
        }
    }
    __shared__ int32_t brj, bbad;
    if (threadIdx.x == 0) brj = bbad = 0;
    __syncthreads();
    const uint64_t rj = __ballot(k == -2), bad = __ballot(k == -3);
    if (lane == 0 && rj) atomicAdd(&brj, (int)__popcll(rj));  // LDS; one global atomic per block
    if (lane == 0 && bad) bbad = 1;
    __syncthreads();
    if (threadIdx.x == 0 && brj) atomicAdd(&g[0], brj);
    if (threadIdx.x == 0 && bbad) atomicOr(&g[1], 1);
    if ((int)threadIdx.x < ncomp) {
        int a = 0, b = 0;
        for (int w = 0; w < JL_BLOCK / 64; ++w) {
            a += wc[w][threadIdx.x];
            b += wm[w][threadIdx.x];
        }
        bc[blockIdx.x * JL_MAXC + threadIdx.x] = a;
        bm[blockIdx.x * JL_MAXC + threadIdx.x] = b;
    }
}

// exclusive scan over blocks per component (32 row-chunks × 32 components on 1024 threads), then
// the component offsets jb / mb (C + 1 each)
__global__ __launch_bounds__(1024) void k_jl_scan(int nblocks, int ncomp, int32_t* __restrict__ bc,
                                                  int32_t* __restrict__ bm, int32_t* __restrict__ jb,
                                                  int32_t* __restrict__ mb) {
    __shared__ int32_t pa[32][JL_MAXC + 1], pb[32][JL_MAXC + 1];
    const int cc = threadIdx.x & 31, r = threadIdx.x >> 5;
    const int chunk = (nblocks + 31) / 32, i0 = r * chunk, i1 = min(nblocks, i0 + chunk);
    int a = 0, b = 0;
    if (cc < ncomp)
        for (int i = i0; i < i1; ++i) {
            a += bc[i * JL_MAXC + cc];
            b += bm[i * JL_MAXC + cc];
        }
    pa[r][cc] = a;
    pb[r][cc] = b;
    __syncthreads();
    if (threadIdx.x < 32) {  // per component: exclusive over the 32 chunks; totals in row 32
        int x = 0, y = 0;
        for (int k = 0; k < 32; ++k) {
            const int u = pa[k][cc], v = pb[k][cc];
            pa[k][cc] = x;
            pb[k][cc] = y;
            x += u;
            y += v;
        }
        pa[0][JL_MAXC] = 0;  // unused
        if (cc < ncomp) {
            jb[cc] = x;  // component total for now
            mb[cc] = y;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // component offsets from totals
        int x = 0, y = 0;
        for (int k = 0; k < ncomp; ++k) {
            const int u = jb[k], v = mb[k];
            jb[k] = x;
            mb[k] = y;
            x += u;
            y += v;
        }
        jb[ncomp] = x;
        mb[ncomp] = y;
    }
    if (cc < ncomp) {
        a = pa[r][cc];
        b = pb[r][cc];
        for (int i = i0; i < i1; ++i) {
            const int u = bc[i * JL_MAXC + cc], v = bm[i * JL_MAXC + cc];
            bc[i * JL_MAXC + cc] = a;
            bm[i * JL_MAXC + cc] = b;
            a += u;
            b += v;
        }
    }
}

__global__ __launch_bounds__(JL_BLOCK) void k_jl_scatter(
    const int8_t* __restrict__ jcomp, int32_t nj, int ncomp, const int32_t* __restrict__ bc,
    const int32_t* __restrict__ bm, const int32_t* __restrict__ jb, const int32_t* __restrict__ mb,
    int32_t* __restrict__ jl, int32_t* __restrict__ jpk) {
    __shared__ int32_t wc[JL_BLOCK / 64][JL_MAXC], wm[JL_BLOCK / 64][JL_MAXC];
    const int q = blockIdx.x * JL_BLOCK + threadIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k = q < nj ? jcomp[q] : -1;
    const int comp = k >= 0 ? (k & 0x3f) : -1;
    const bool multi = k >= 0 && (k & 0x40);
    int rank = 0, mrank = 0;
    for (int cc = 0; cc < ncomp; ++cc) {
        const uint64_t m = __ballot(comp == cc), mm = __ballot(comp == cc && multi);
        if (lane == 0) {
            wc[wave][cc] = __popcll(m);
            wm[wave][cc] = __popcll(mm);
        }
        if (comp == cc) {
            rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            mrank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0));
        }
    }
    __syncthreads();
    if (comp >= 0) {
        int wo = 0, wmo = 0;
        for (int w = 0; w < wave; ++w) {
            wo += wc[w][comp];
            wmo += wm[w][comp];
        }
        const int pos = jb[comp] + bc[blockIdx.x * JL_MAXC + comp] + wo + rank;
        const int before = mb[comp] + bm[blockIdx.x * JL_MAXC + comp] + wmo + mrank;
        jl[pos] = q;
        jpk[pos + 1] = before + (multi ? 1 : 0);
    }
    if (q == 0) jpk[0] = 0;
}
}  // namespace fitgpu

// ---------------------------------------------------------------- host launch wrappers
namespace fitgpu {

hipError_t launch_scan(int blocks, hipStream_t st, const NodeRec* rec, const int32_t* jl,
                       const int32_t* jcpu, const int32_t* jmem, const int32_t* jgpu,
                       const int32_t* jwall, const uint16_t* jpart, const uint16_t* jk,
                       const CompPlan* plan, int ncomp, uint64_t* cand, uint64_t* bnd,
                       JobRec* wjob) {
    hipLaunchKernelGGL(k_scan, dim3(blocks), dim3(SCAN_WAVES * 64), 0, st, rec, jl, jcpu, jmem, jgpu,
                       jwall, jpart, jk, plan, ncomp, cand, bnd, wjob);
    return hipGetLastError();
}

hipError_t launch_commit(int ncomp, int epl, size_t lds_bytes, hipStream_t st, NodeRec* rec,
                         const CompPlan* plan, const uint64_t* cand, int64_t rank_stride,
                         int nranks, const uint64_t* bnd, const JobRec* wjob, int32_t* out,
                         int kmax, CommitResult* res) {
#define FIT_COMMIT(EPL)                                                                      \
    hipLaunchKernelGGL(k_commit<EPL>, dim3(ncomp), dim3(64), lds_bytes, st, rec, plan, cand, \
                       rank_stride, nranks, bnd, wjob, out, kmax, res)
    if (epl <= 1) FIT_COMMIT(1);
    else if (epl <= 2) FIT_COMMIT(2);
    else if (epl <= 4) FIT_COMMIT(4);
    else if (epl <= 8) FIT_COMMIT(8);
    else if (epl <= 16) FIT_COMMIT(16);
    else return hipErrorInvalidValue;
#undef FIT_COMMIT
    return hipGetLastError();
}

// ------------------------------------------------------------- direct small placement
// A placement of a few jobs (an admission batch: fit_admitter coalesces the PodSyncWorkers'
// CreatePod calls, a handful of pods at a time) in ONE launch and nothing else — no prefilter,
// no job-list kernels, no memset.  Every block first runs the prefilter over
// all jobs (job_code; a few dozen jobs): it initialises the out[] rows of its own jobs (block 0
// also those of rejected, invalid and nodeless ones) and learns whether any job is invalid, in
// which case no block touches the node table (the call fails with FIT_E_INVAL).  Then block c
// walks component c's jobs in priority order (index order, compacted 512 at a time into LDS)
// one at a time, each against every node of the component — SPEC §2 directly, no candidate
// lists, no rounds.  Per job: every thread keeps the minimum key of its strided nodes, a wave
// DPP minimum then an LDS minimum over the 8 waves gives the block's; a multi-node job takes its
// k smallest distinct keys by k such extractions (each excludes the keys already taken: keys are
// unique), all or nothing.  The chosen rows are updated in place in `rec` by the threads that
// hold the choice; the block barrier makes them visible to the next job's scan (same
// workgroup).  Cost per job ≈ one pass over the component's rows (L2-resident) and 2 barriers
// per extraction: a few microseconds, so it is used only for small placements (engine.cpp
// small_direct) — a large one goes through the rounds.
// stat[0] = rejected jobs, stat[1] = 1 if a job is invalid, stat[2 + c] = jobs placed in c.
constexpr int SMALL_THREADS = 512;

__device__ __forceinline__ int small_place_job(NodeRec* rec, int nb, int ne, const JobRec& J, int k,
                                               int32_t kmax, int32_t* __restrict__ out, uint64_t* wmin,
                                               int32_t* sel) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = J.q;
    uint64_t prev = 0ull;  // keys <= prev are taken (extraction r excludes them)
    uint64_t kth = KEY_INF;
    for (int r = 0; r < k; ++r) {
        uint64_t m = KEY_INF;
        for (int p = nb + (int)threadIdx.x; p < ne; p += SMALL_THREADS) {
            const NodeRec x = rec[p];
            const uint64_t key = fit_key(x.cpu, x.mem, x.gpu, x.avail, x.mask, (uint32_t)p, J);
            m = (key < m && (r == 0 || key > prev)) ? key : m;
        }
        const uint64_t w = wave_min_key(m);
        if (lane == 0) wmin[wave] = w;
        __syncthreads();
        uint64_t b = wmin[0];
#pragma unroll
        for (int i = 1; i < SMALL_THREADS / 64; ++i) b = umin64(b, wmin[i]);
        __syncthreads();  // wmin is rewritten by the next extraction
        if (b == KEY_INF) {  // fewer than k nodes fit: nothing is taken
            kth = KEY_INF;
            break;
        }
        if (m == b) sel[r] = (int32_t)(uint32_t)b;  // the one thread holding it (keys are unique)
        prev = b;
        kth = b;
    }
    __syncthreads();  // sel[]
    if (kth == KEY_INF) return 0;
    if ((int)threadIdx.x < k) {
        const int p = sel[threadIdx.x];
        const NodeRec x = rec[p];
        rec[p].cpu = x.cpu - J.cpu;
        rec[p].mem = x.mem - J.mem;
        rec[p].gpu = x.gpu - J.gpu;
        out[(int64_t)q * kmax + threadIdx.x] = x.orig;
    }
    __syncthreads();  // the updated rows, before the next job's scan
    return 1;
}

// The same for a component of at most SMALL_THREADS × SMALL_RPT rows, held in VGPRs: thread t
// owns rows nb + t + 512 i (i < rpt), loaded once per launch with every load in flight, so a job
// costs ALU and two barriers per extraction instead of a pass over L2 (a pass of dependent loads
// is ~1 µs of latency per row a thread holds).  The winner of extraction r updates its own
// registers, writes the row back to `rec` (the table the next call and fit_read_nodes see) and
// the placement; the next job reads only its own registers, so no trailing barrier is needed.
constexpr int SMALL_RPT = 16;

__device__ __forceinline__ int small_place_job_regs(NodeRec* rec, int nb, int rpt, const JobRec& J, int k,
                                                    int32_t kmax, int32_t* __restrict__ out, uint64_t* wmin,
                                                    int32_t* sel,
                                                    int32_t (&rc)[SMALL_RPT], int32_t (&rm)[SMALL_RPT],
                                                    int32_t (&rg)[SMALL_RPT], const int32_t (&ra)[SMALL_RPT],
                                                    const uint32_t (&rk)[SMALL_RPT], const int32_t (&ro)[SMALL_RPT]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = J.q;
    uint64_t prev = 0ull;
    uint64_t kth = KEY_INF;
    uint32_t won = 0;  // extractions this thread won
    for (int r = 0; r < k; ++r) {
        uint64_t m = KEY_INF;
#pragma unroll
        for (int i = 0; i < SMALL_RPT; ++i) {
            if (i < rpt) {
                const uint64_t key = fit_key(rc[i], rm[i], rg[i], ra[i], rk[i],
                                             (uint32_t)(nb + (int)threadIdx.x + i * SMALL_THREADS), J);
                m = (key < m && (r == 0 || key > prev)) ? key : m;
            }
        }
        const uint64_t w = wave_min_key(m);
        if (lane == 0) wmin[wave] = w;
        __syncthreads();
        uint64_t b = wmin[0];
#pragma unroll
        for (int i = 1; i < SMALL_THREADS / 64; ++i) b = umin64(b, wmin[i]);
        __syncthreads();  // wmin is rewritten by the next extraction
        if (b == KEY_INF) {
            kth = KEY_INF;
            break;
        }
        if (m == b) {
            sel[r] = (int32_t)(uint32_t)b;
            won |= 1u << r;
        }
        prev = b;
        kth = b;
    }
    if (kth == KEY_INF) return 0;
    for (int r = 0; won; ++r, won >>= 1) {
        if (!(won & 1u)) continue;
        const int p = sel[r];
        const int ii = (p - nb) / SMALL_THREADS;
#pragma unroll
        for (int i = 0; i < SMALL_RPT; ++i) {
            if (i == ii) {
                rc[i] -= J.cpu;
                rm[i] -= J.mem;
                rg[i] -= J.gpu;
                rec[p].cpu = rc[i];
                rec[p].mem = rm[i];
                rec[p].gpu = rg[i];
                out[(int64_t)q * kmax + r] = ro[i];
            }
        }
    }
    return 1;
}

__device__ __forceinline__ void small_body(
    NodeRec* rec, const SmallComps& C, int32_t ncomp, const int32_t* __restrict__ ptab, int32_t np,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, const uint16_t* __restrict__ jk, int32_t nj, int32_t kmax,
    int32_t* __restrict__ out, int32_t* __restrict__ stat) {
    __shared__ uint64_t wmin[SMALL_THREADS / 64];
    __shared__ int32_t sel[FIT_KMAX];
    __shared__ int32_t list[SMALL_THREADS];   // (job, k) of the chunk's own jobs in priority order
    __shared__ int4 ljob[SMALL_THREADS];      // their (cpu, mem, gpu, wall): read from LDS per job
    __shared__ int32_t lpart[SMALL_THREADS];
    __shared__ int32_t wcnt[SMALL_THREADS / 64];
    __shared__ int32_t s_bad, s_rej;
    const int c = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_bad = s_rej = 0;
    __syncthreads();
    // 1. the prefilter, over every job in every block (each needs the invalid-job verdict)
    int bad = 0, rj = 0;
    for (int q = threadIdx.x; q < nj; q += SMALL_THREADS) {
        bool rej;
        int k;
        const int code = job_code(q, jcpu, jmem, jgpu, jwall, jpart, jk, kmax, ptab, np, &rej, &k);
        bad |= code == -3;
        rj += code == -2;
        if ((code >= 0 ? (code & 0x3f) : 0) == c)
            for (int i = 0; i < kmax; ++i) out[(int64_t)q * kmax + i] = (rej && i < k) ? -2 : -1;
    }
    if (bad) s_bad = 1;
    if (rj) atomicAdd(&s_rej, rj);
    __syncthreads();
    if (s_bad) {  // the call fails and must leave the node table as it was
        if (threadIdx.x == 0) {
            stat[2 + c] = 0;
            if (c == 0) {
                stat[0] = s_rej;
                stat[1] = 1;
            }
        }
        return;
    }
    // 2. component c's jobs in priority order
    int32_t placed = 0;
    if (c < ncomp) {
        const int nb = C.nb[c], ne = C.nb[c + 1];
        // rows in VGPRs when the component fits (SMALL_RPT per thread), else a pass per extraction
        const int rpt = (ne - nb + SMALL_THREADS - 1) / SMALL_THREADS;
        const bool regs = rpt <= SMALL_RPT;
        int32_t rc[SMALL_RPT], rm[SMALL_RPT], rg[SMALL_RPT], ra[SMALL_RPT], ro[SMALL_RPT];
        uint32_t rk[SMALL_RPT];
#pragma unroll
        for (int i = 0; i < SMALL_RPT; ++i) {
            const int p = nb + (int)threadIdx.x + i * SMALL_THREADS;
            NodeRec x;
            x.cpu = x.mem = x.gpu = x.avail = -1;
            x.mask = 0u;
            x.orig = -1;
            if (regs && p < ne) x = rec[p];
            rc[i] = x.cpu;
            rm[i] = x.mem;
            rg[i] = x.gpu;
            ra[i] = x.avail;
            rk[i] = x.mask;  // 0: a padding row fits no job
            ro[i] = x.orig;
        }
        for (int base = 0; base < nj; base += SMALL_THREADS) {
            const int q = base + (int)threadIdx.x;
            bool mine = false;
            int k = 1;
            if (q < nj) {
                bool rej;
                const int code = job_code(q, jcpu, jmem, jgpu, jwall, jpart, jk, kmax, ptab, np, &rej, &k);
                mine = code >= 0 && (code & 0x3f) == c;
            }
            const uint64_t m = __ballot(mine);
            if (lane == 0) wcnt[wave] = __popcll(m);
            __syncthreads();
            int off = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < SMALL_THREADS / 64; ++w) {
                const int n = wcnt[w];
                off += w < wave ? n : 0;
                tot += n;
            }
            // (q, k) packed: k <= FIT_KMAX; the job's columns beside it (this thread loaded them
            // for job_code: no global read per job in the walk)
            if (mine) {
                const int at = off + __popcll(m & ((1ull << lane) - 1ull));
                list[at] = q * 32 + k;
                ljob[at] = make_int4(jcpu[q], jmem[q], jgpu[q], jwall[q]);
                lpart[at] = jpart[q];
            }
            __syncthreads();
            for (int t = 0; t < tot; ++t) {
                const int e = list[t];
                const int4 f = ljob[t];
                JobRec J;
                J.q = e >> 5;
                J.cpu = f.x;
                J.mem = f.y;
                J.gpu = f.z;
                J.wall = f.w;
                J.pbit = 1u << lpart[t];
                placed += regs ? small_place_job_regs(rec, nb, rpt, J, e & 31, kmax, out, wmin, sel, rc, rm, rg, ra,
                                                      rk, ro)
                               : small_place_job(rec, nb, ne, J, e & 31, kmax, out, wmin, sel);
            }
            __syncthreads();  // list[] and wcnt[] are rewritten by the next chunk
        }
    }
    if (threadIdx.x == 0) {
        stat[2 + c] = placed;
        if (c == 0) {
            stat[0] = s_rej;
            stat[1] = 0;
        }
    }
}

__global__ __launch_bounds__(SMALL_THREADS) void k_small(
    NodeRec* rec, SmallComps C, int32_t ncomp, const int32_t* __restrict__ ptab, int32_t np,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, const uint16_t* __restrict__ jk, int32_t nj, int32_t kmax,
    int32_t* __restrict__ out, int32_t* __restrict__ stat) {
    small_body(rec, C, ncomp, ptab, np, jcpu, jmem, jgpu, jwall, jpart, jk, nj, kmax, out, stat);
}

// The batch in the kernel arguments (nj <= SMALL_ARGJ): copied into LDS first, then as k_small.
__global__ __launch_bounds__(SMALL_THREADS) void k_small_args(
    NodeRec* rec, SmallComps C, int32_t ncomp, const int32_t* __restrict__ ptab, int32_t np, SmallBatch B,
    int32_t has_nk, int32_t nj, int32_t kmax, int32_t* __restrict__ out, int32_t* __restrict__ stat) {
    __shared__ SmallBatch sb;
    for (int i = threadIdx.x; i < nj; i += SMALL_THREADS) {
        sb.cpu[i] = B.cpu[i];
        sb.mem[i] = B.mem[i];
        sb.gpu[i] = B.gpu[i];
        sb.wall[i] = B.wall[i];
        sb.part[i] = B.part[i];
        sb.nk[i] = B.nk[i];
    }
    __syncthreads();
    small_body(rec, C, ncomp, ptab, np, sb.cpu, sb.mem, sb.gpu, sb.wall, sb.part, has_nk ? sb.nk : nullptr, nj, kmax,
               out, stat);
}

hipError_t launch_small_args(hipStream_t st, int ncomp, NodeRec* rec, const SmallComps& C, const int32_t* ptab,
                             int32_t np, const SmallBatch& B, bool has_nk, int32_t nj, int32_t kmax, int32_t* out,
                             int32_t* stat) {
    if (nj > SMALL_ARGJ) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_small_args, dim3(ncomp > 0 ? ncomp : 1), dim3(SMALL_THREADS), 0, st, rec, C, ncomp, ptab,
                       np, B, has_nk ? 1 : 0, nj, kmax, out, stat);
    return hipGetLastError();
}

// grid: max(ncomp, 1) blocks (block 0 initialises the rows of jobs that no component owns)
hipError_t launch_small(hipStream_t st, int ncomp, NodeRec* rec, const SmallComps& C,
                        const int32_t* ptab, int32_t np, const int32_t* jcpu, const int32_t* jmem,
                        const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart,
                        const uint16_t* jk, int32_t nj, int32_t kmax, int32_t* out, int32_t* stat) {
    hipLaunchKernelGGL(k_small, dim3(ncomp > 0 ? ncomp : 1), dim3(SMALL_THREADS), 0, st, rec, C, ncomp, ptab,
                       np, jcpu, jmem, jgpu, jwall, jpart, jk, nj, kmax, out, stat);
    return hipGetLastError();
}

#ifdef FIT_STAMPS
extern "C" int fit_debug_commit_stamps(unsigned long long* out /* 64 x 8 */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) == hipSuccess ? 0 : -2;
}
#endif

hipError_t launch_prefilter(hipStream_t st, const int32_t* jcpu, const int32_t* jmem,
                            const int32_t* jgpu, const int32_t* jwall, const uint16_t* jpart, const uint16_t* jk,
                            int32_t nj, int32_t kmax, const int32_t* ptab, int32_t np,
                            int32_t* out, int8_t* jcomp) {
    if (nj == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prefilter, dim3((nj + 255) / 256), dim3(256), 0, st, jcpu, jmem, jgpu, jwall,
                       jpart, jk, nj, kmax, ptab, np, out, jcomp);
    return hipGetLastError();
}

// scratch: bc, bm = nblocks * JL_MAXC ints each; g = 2 ints (zeroed here); jb, mb = ncomp + 1
size_t joblists_scratch_ints(int32_t nj) { return (size_t)2 * ((nj + JL_BLOCK - 1) / JL_BLOCK) * JL_MAXC; }

hipError_t launch_joblists(hipStream_t st, const int8_t* jcomp, int32_t nj, int ncomp,
                           int32_t* scratch, int32_t* g, int32_t* jb, int32_t* mb, int32_t* jl,
                           int32_t* jpk) {
    if (ncomp > JL_MAXC) return hipErrorInvalidValue;
    const int nblocks = (nj + JL_BLOCK - 1) / JL_BLOCK;
    int32_t* bc = scratch;
    int32_t* bm = scratch + (size_t)nblocks * JL_MAXC;
    hipError_t e = hipMemsetAsync(g, 0, 2 * sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    if (nj > 0) {
        hipLaunchKernelGGL(k_jl_count, dim3(nblocks), dim3(JL_BLOCK), 0, st, jcomp, nj, ncomp, bc, bm, g);
    }
    hipLaunchKernelGGL(k_jl_scan, dim3(1), dim3(1024), 0, st, nblocks, ncomp, bc, bm, jb, mb);
    if (nj > 0) {
        hipLaunchKernelGGL(k_jl_scatter, dim3(nblocks), dim3(JL_BLOCK), 0, st, jcomp, nj, ncomp, bc,
                           bm, jb, mb, jl, jpk);
    } else {
        e = hipMemsetAsync(jpk, 0, sizeof(int32_t), st);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_gather_nodes(hipStream_t st, const int32_t* cpu, const int32_t* mem,
                               const int32_t* gpu, const int32_t* av, const uint32_t* mask,
                               const int32_t* perm, int32_t nn, NodeRec* rec) {
    if (nn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_nodes, dim3((nn + 255) / 256), dim3(256), 0, st, cpu, mem, gpu,
                       av, mask, perm, nn, rec);
    return hipGetLastError();
}

hipError_t launch_scatter_nodes(hipStream_t st, const NodeRec* rec, int32_t nn, int32_t* cpu,
                                int32_t* mem, int32_t* gpu) {
    if (nn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_nodes, dim3((nn + 255) / 256), dim3(256), 0, st, rec, nn, cpu,
                       mem, gpu);
    return hipGetLastError();
}

}  // namespace fitgpu
