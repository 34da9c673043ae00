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
#include <hip/hip_runtime.h>

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

// ---- wave-wide 64-bit min over all 64 lanes (DPP; call with a full EXEC mask) ----------
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)(uint32_t)v, CTRL,
                                                        ROWMASK, 0xf, false);
    uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)(uint32_t)(v >> 32),
                                                        CTRL, ROWMASK, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    v = umin64(v, dpp64<0xb1, 0xf>(v));   // quad_perm [1,0,3,2]
    v = umin64(v, dpp64<0x4e, 0xf>(v));   // quad_perm [2,3,0,1]
    v = umin64(v, dpp64<0x124, 0xf>(v));  // row_ror:4
    v = umin64(v, dpp64<0x128, 0xf>(v));  // row_ror:8
    v = umin64(v, dpp64<0x142, 0xa>(v));  // row_bcast:15
    v = umin64(v, dpp64<0x143, 0xc>(v));  // row_bcast:31
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

// sorted ascending insert of x into key[0..KS) dropping the largest (static indices only)
__device__ __forceinline__ void topk_insert(uint64_t (&key)[KS], uint64_t x) {
#pragma unroll
    for (int i = KS - 1; i > 0; --i) {
        uint64_t a = key[i - 1], b = key[i];
        key[i] = a > x ? a : (b > x ? x : b);
    }
    key[0] = key[0] > x ? x : key[0];
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
__device__ __forceinline__ void scan_row(const NodeRec& r, int x, const JobRec& J,
                                         uint64_t (&key)[KS], uint32_t& lim) {
    const int32_t dc = r.cpu - J.cpu, dm = r.mem - J.mem, dg = r.gpu - J.gpu;
    const int32_t da = r.avail - J.wall;
    const int32_t dp = (int32_t)((r.mask & J.pbit) - 1u);  // -1: not a member (or idle lane)
    const int32_t bad = dc | dm | dg | da | dp;
    const uint32_t sc = (min((uint32_t)dg, 255u) << 24) | (min((uint32_t)dc, 4095u) << 12) |
                        min((uint32_t)dm >> 10, 4095u);
    if (bad >= 0 && sc <= lim) {
        topk_insert(key, ((uint64_t)sc << 32) | (uint32_t)x);
        const uint64_t last = key[KS - 1];
        lim = last == KEY_INF ? 0xffffffffu : (uint32_t)(last >> 32) - 1u;
    }
}

// -------------------------------------------------------------------------------- k_scan
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan(
    const NodeRec* __restrict__ rec, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, const uint16_t* __restrict__ jk,
    const CompPlan* __restrict__ plan, int ncomp, uint64_t* __restrict__ cand,
    uint64_t* __restrict__ bnd, JobRec* __restrict__ wjob) {
    const int c = find_comp(plan, ncomp, blockIdx.x);
    const CompPlan P = plan[c];
    const int local = blockIdx.x - P.blk0;
    // integer division expands to VALU code: pin the (uniform) results to SGPRs
    const int tile = __builtin_amdgcn_readfirstlane(local / P.nslice);
    const int s = __builtin_amdgcn_readfirstlane(local - tile * P.nslice);
    const int t = tile * SCAN_BLOCK + threadIdx.x;
    // wave-uniform by construction; readfirstlane tells the compiler so (keeps the node loop
    // counter and row addresses in SGPRs)
    const int wave_first =
        __builtin_amdgcn_readfirstlane(tile * SCAN_BLOCK + (int)(threadIdx.x & ~63u));
    if (wave_first >= P.w) return;  // whole wave outside the window
    const bool active = t < P.w;

    JobRec J;
    J.q = active ? jl[P.jbase + t] : 0;
    J.cpu = active ? jcpu[J.q] : 0;
    J.mem = active ? jmem[J.q] : 0;
    J.gpu = active ? jgpu[J.q] : 0;
    J.wall = active ? jwall[J.q] : 0;
    J.pbit = active ? (1u << jpart[J.q]) : 0u;  // 0 → nothing feasible
    J.k = active ? (jk ? max((int)jk[J.q], 1) : 1) : 1;
    J.pad = 0;

    uint64_t key[KS];
#pragma unroll
    for (int i = 0; i < KS; ++i) key[i] = KEY_INF;
    // candidate test: score <= lim, lim = (K-th score - 1) once the list is full.  An equal
    // score never beats the K-th entry (positions only grow); a spurious insert when the K-th
    // score is 0 is dropped by the 64-bit insertion network, so the list stays exact.
    uint32_t lim = 0xffffffffu;

    const int n0 = P.sb + s * SLICE;
    const int n1 = min(P.se, n0 + SLICE);
    int x = n0;
    // 4 rows per batch: four s_load_dwordx8 in flight per wait
    for (; x + 4 <= n1; x += 4) {
        NodeRec r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = rec[x + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) scan_row(r[u], x + u, J, key, lim);
    }
    for (; x < n1; ++x) scan_row(rec[x], x, J, key, lim);
    const bool full = key[KS - 1] != KEY_INF;
    if (!active) return;
    uint64_t* dst = cand + P.cand_off + ((int64_t)t * P.nslice + s) * KS;
#pragma unroll
    for (int i = 0; i < KS; i += 2) {
        ulonglong2 v;
        v.x = key[i];
        v.y = key[i + 1];
        *reinterpret_cast<ulonglong2*>(dst + i) = v;
    }
    // every node outside this slice's list has a key > key[KS-1] (list full) — bound B
    if (full) atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                        (unsigned long long)key[KS - 1]);
    if (s == 0) wjob[P.slot0 + t] = J;
}

// ------------------------------------------------------------------------------ k_commit
constexpr int UPL = UCAP / 64;  // dirty slots per lane

__global__ __launch_bounds__(64) void k_commit(
    NodeRec* __restrict__ rec, const CompPlan* __restrict__ plan,
    const uint64_t* __restrict__ cand, int64_t rank_stride, int nranks,
    const uint64_t* __restrict__ bnd, const JobRec* __restrict__ wjob,
    int32_t* __restrict__ out, int kmax, CommitResult* __restrict__ res) {
    extern __shared__ uint32_t bitmap[];
    const int c = blockIdx.x;
    const CompPlan P = plan[c];
    const int lane = threadIdx.x;
    if (P.w == 0) {
        if (lane == 0) res[c] = CommitResult{0, 0, 0, 0};
        return;
    }
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = lane; i < nwords; i += 64) bitmap[i] = 0u;
    __syncthreads();

    int32_t ucpu[UPL], umem[UPL], ugpu[UPL], uav[UPL], uorig[UPL];
    uint32_t umask[UPL], upos[UPL];
#pragma unroll
    for (int i = 0; i < UPL; ++i) {
        ucpu[i] = umem[i] = ugpu[i] = uav[i] = uorig[i] = 0;
        umask[i] = 0u;
        upos[i] = 0u;
    }
    int nu = 0, placed = 0, stop = 0, t = 0;
    const int per_rank = P.nslice * KS;
    const int E = nranks * per_rank;

    for (; t < P.w; ++t) {
        const JobRec J = wjob[P.slot0 + t];
        const uint64_t B = bnd[P.slot0 + t];
        // best clean candidate held by this lane
        uint64_t cm = KEY_INF;
        for (int e = lane; e < E; e += 64) {
            const int g = e / per_rank;
            const int r = e - g * per_rank;
            const uint64_t k = cand[g * rank_stride + P.cand_off + (int64_t)t * per_rank + r];
            if (k != KEY_INF && k <= B) {
                const uint32_t rel = (uint32_t)k - (uint32_t)P.nb;
                const bool dirty = (bitmap[rel >> 5] >> (rel & 31)) & 1u;
                if (!dirty) cm = umin64(cm, k);
            }
        }
        // current keys of the dirty rows held by this lane
        uint64_t dk[UPL];
        uint64_t dm = KEY_INF;
#pragma unroll
        for (int i = 0; i < UPL; ++i) {
            dk[i] = (i * 64 + lane < nu)
                        ? fit_key(ucpu[i], umem[i], ugpu[i], uav[i], umask[i], upos[i], J)
                        : KEY_INF;
            dm = umin64(dm, dk[i]);
        }
        const uint64_t best = wave_min_u64(umin64(cm, dm));
        const bool any_clean = __ballot(cm != KEY_INF) != 0ull;
        if (!any_clean && B != KEY_INF && best > B) {  // list exhausted: rescan next round
            stop = 1;
            break;
        }
        if (best == KEY_INF) continue;  // FIT_UNPLACED (out pre-set to -1)
        const uint64_t from_dirty = __ballot(dm == best);
        if (from_dirty) {
#pragma unroll
            for (int i = 0; i < UPL; ++i)
                if (dk[i] == best) {
                    ucpu[i] -= J.cpu;
                    umem[i] -= J.mem;
                    ugpu[i] -= J.gpu;
                    out[(int64_t)J.q * kmax] = uorig[i];
                }
        } else {
            if (nu == UCAP) {
                stop = 2;
                break;
            }
            const uint32_t pos = (uint32_t)best;
            const int owner = nu & 63, slot = nu >> 6;
            if (lane == owner) {
                const NodeRec r = rec[pos];
#pragma unroll
                for (int i = 0; i < UPL; ++i)
                    if (i == slot) {
                        ucpu[i] = r.cpu - J.cpu;
                        umem[i] = r.mem - J.mem;
                        ugpu[i] = r.gpu - J.gpu;
                        uav[i] = r.avail;
                        umask[i] = r.mask;
                        upos[i] = pos;
                        uorig[i] = r.orig;
                    }
                out[(int64_t)J.q * kmax] = r.orig;
                const uint32_t rel = pos - (uint32_t)P.nb;
                bitmap[rel >> 5] |= 1u << (rel & 31);
            }
            ++nu;
            __syncthreads();  // bitmap write visible to the next job's lookups
        }
        ++placed;
    }
    // write the dirty rows back for the next round's scan
#pragma unroll
    for (int i = 0; i < UPL; ++i)
        if (i * 64 + lane < nu) {
            NodeRec* r = rec + upos[i];
            r->cpu = ucpu[i];
            r->mem = umem[i];
            r->gpu = ugpu[i];
        }
    if (lane == 0) res[c] = CommitResult{t, stop, nu, placed};
}

// ------------------------------------------------------------------- prefilter / setup
// out[] init, component id per job, rejected marks (FIT_REJECTED) — DESIGN.md §3.1.
__global__ void k_prefilter(const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
                            const int32_t* __restrict__ jwall, const uint16_t* __restrict__ jpart,
                            const uint16_t* __restrict__ jk, int32_t nj, int32_t kmax,
                            const int32_t* __restrict__ ptab /* [4][32]: time,cpus,mem,comp */,
                            int32_t np, int32_t* __restrict__ out, int8_t* __restrict__ jcomp) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nj) return;
    const int p = jpart[q];
    const int k = jk ? max((int)jk[q], 1) : 1;
    bool rej = p >= np;
    if (!rej) {
        const int mt = ptab[p], mc = ptab[32 + p], mm = ptab[64 + p];
        rej = (mt >= 0 && jwall[q] > mt) || (mc >= 0 && jcpu[q] > mc) || (mm >= 0 && jmem[q] > mm);
    }
    int8_t comp = rej ? (int8_t)-2 : (int8_t)ptab[96 + p];  // -1: partition has no nodes
    jcomp[q] = comp;
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

}  // namespace fitgpu

// ---------------------------------------------------------------- host launch wrappers
namespace fitgpu {

hipError_t launch_scan(int blocks, hipStream_t st, const NodeRec* rec, const int32_t* jl,
                       const int32_t* jcpu, const int32_t* jmem, const int32_t* jgpu,
                       const int32_t* jwall, const uint16_t* jpart, const uint16_t* jk,
                       const CompPlan* plan, int ncomp, uint64_t* cand, uint64_t* bnd,
                       JobRec* wjob) {
    hipLaunchKernelGGL(k_scan, dim3(blocks), dim3(SCAN_BLOCK), 0, st, rec, jl, jcpu, jmem, jgpu,
                       jwall, jpart, jk, plan, ncomp, cand, bnd, wjob);
    return hipGetLastError();
}

hipError_t launch_commit(int ncomp, size_t lds_bytes, hipStream_t st, NodeRec* rec,
                         const CompPlan* plan, const uint64_t* cand, int64_t rank_stride,
                         int nranks, const uint64_t* bnd, const JobRec* wjob, int32_t* out,
                         int kmax, CommitResult* res) {
    hipLaunchKernelGGL(k_commit, dim3(ncomp), dim3(64), lds_bytes, st, rec, plan, cand,
                       rank_stride, nranks, bnd, wjob, out, kmax, res);
    return hipGetLastError();
}

hipError_t launch_prefilter(hipStream_t st, const int32_t* jcpu, const int32_t* jmem,
                            const int32_t* jwall, const uint16_t* jpart, const uint16_t* jk,
                            int32_t nj, int32_t kmax, const int32_t* ptab, int32_t np,
                            int32_t* out, int8_t* jcomp) {
    if (nj == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prefilter, dim3((nj + 255) / 256), dim3(256), 0, st, jcpu, jmem, jwall,
                       jpart, jk, nj, kmax, ptab, np, out, jcomp);
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
