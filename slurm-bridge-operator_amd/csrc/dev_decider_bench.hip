// dev_decider_bench.hip — diagnostic only (never linked into the product): the decider loop of
// fit_commit_mw.h alone on one wave, records pre-filled in LDS and no helper waves, to measure
// its intrinsic cycles per job.  Built into fitgpu/libdecbench.so by `make decbench`.
#define MW_DECIDER_BENCH 1
#include "fit_commit_mw.h"

namespace fitgpu {
__global__ __launch_bounds__(64) void k_dec_bench(int w, int32_t* out, unsigned long long* cyc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    MwShared* S = reinterpret_cast<MwShared*>(smem);
    const int lane = threadIdx.x;
    // eight records: 8 clean items each with distinct positions, demand 1 cpu
    for (int r = 0; r < MW_R; ++r) {
        if (lane == 0) {
            S->rec[r].h = MwHdr{0u, 0, MW_M, r, 1, 1, 0, 0, 1u, 0u, KEY_INF};
        }
        if (lane < MW_M) {
            S->rec[r].it[lane] = MwItem{(uint32_t)(r * MW_M + lane), (uint32_t)(lane + 1), r * MW_M + lane,
                                        r * MW_M + lane, 1000000, 1000000, 0, 0, 1u, 0u, 0u, 0u};
        }
    }
    for (int i = lane; i < 64; i += 64) S->bitmap[i] = 0u;
    if (lane == 0) S->dn = 0ull;
    __syncthreads();
    CompPlan P{};
    P.nb = 0;
    P.ne = 2048;
    P.w = w;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const CommitResult r = mw_decider(P, S, out, 1);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = r.done;
        cyc[2] = r.placed;
        cyc[3] = r.dirty;
    }
}
}  // namespace fitgpu

extern "C" int dec_bench(int w, unsigned long long* host_out) {
    int32_t* out;
    unsigned long long* cyc;
    if (hipMalloc(&out, sizeof(int32_t) * (w + 64)) != hipSuccess) return -1;
    if (hipMalloc(&cyc, 64) != hipSuccess) return -1;
    const size_t lds = fitgpu::mw_lds_bytes(2048);
    hipLaunchKernelGGL(fitgpu::k_dec_bench, dim3(1), dim3(64), lds, 0, w, out, cyc);
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    hipMemcpy(host_out, cyc, 32, hipMemcpyDeviceToHost);
#ifdef MW_SEGSTAMP
    hipMemcpyFromSymbol(host_out + 4, HIP_SYMBOL(fitgpu::g_seg), 64);
#endif
    hipFree(out);
    hipFree(cyc);
    return 0;
}
