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
    scan_tile<false>(P, tile, s, rec, jl, jcpu, jmem, jgpu, jwall, jpart, jk, cand, bnd, wjob, xk);
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
__global__ void k_prefilter(const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
                            const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall, const uint16_t* __restrict__ jpart,
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
    // -3: invalid job (negative demand or nodes_k > kmax), -2: rejected by partition limits,
    // -1: partition has no nodes, else component | 0x40 for a multi-node job
    int8_t comp = rej ? (int8_t)-2 : (int8_t)ptab[96 + p];
    if (comp >= 0 && k > 1) comp = (int8_t)(comp | 0x40);
    if (k > kmax || jcpu[q] < 0 || jmem[q] < 0 || jwall[q] < 0 || (jgpu && jgpu[q] < 0))
        comp = (int8_t)-3;
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
    else return hipErrorInvalidValue;
#undef FIT_COMMIT
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
