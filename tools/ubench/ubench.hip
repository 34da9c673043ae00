// Instruction-latency micro-benchmarks for one wave on gfx950 (dev tool; not part of the product).
// Each test runs a 64-long dependent chain 16 times between s_memtime stamps; prints cycles/op.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void k_ubench(unsigned long long* out, int* sink) {
    __shared__ int lds[256];
    const int lane = threadIdx.x;
    lds[lane] = lane;
    __syncthreads();
    int v = lane, r = 0;
    unsigned long long t0, t1;
    int s = 1;
#define TIME(idx, body)                                                          \
    t0 = __builtin_amdgcn_s_memtime();                                           \
    for (int it = 0; it < 16; ++it) { body }                                     \
    t1 = __builtin_amdgcn_s_memtime();                                           \
    if (lane == 0) out[idx] = t1 - t0;
    // 0: dependent v_add
    TIME(0, asm volatile(REP64("v_add_u32 %0, %0, 1\n") : "+v"(v));)
    // 1: dependent s_add
    TIME(1, asm volatile(REP64("s_add_u32 %0, %0, 1\n") : "+s"(s) :: "scc");)
    // 2: independent v_add (4 chains)
    {
        int a = v, b = v, c = v, d = v;
        TIME(2, asm volatile(REP8(REP8("v_add_u32 %0, %0, 1\nv_add_u32 %1, %1, 1\nv_add_u32 %2, %2, 1\nv_add_u32 %3, %3, 1\n")) : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
        v = a + b + c + d;
    }
    // 3: v_readlane → s_add → v_add (VALU→SGPR→VALU round trip)
    TIME(3, asm volatile(REP64("v_readlane_b32 %1, %0, 0\ns_nop 4\ns_add_u32 %1, %1, 1\nv_add_u32 %0, %1, %0\n") : "+v"(v), "+s"(s) :: "scc");)
    // 4: ds_read dependent chain (address = value read)
    {
        int addr = 0;
        TIME(4, asm volatile(REP64("ds_read_b32 %0, %0\ns_waitcnt lgkmcnt(0)\n") : "+v"(addr));)
        r += addr;
    }
    // 5: dpp min chain
    TIME(5, asm volatile(REP64("s_nop 1\nv_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n") : "+v"(v));)
    // 6: v_cmp → s_cbranch (not taken) chain
    TIME(6, asm volatile(REP64("v_cmp_eq_u32 vcc, -1, %0\ns_cbranch_vccnz 1f\n1:\n") : "+v"(v) :: "vcc");)
    // 7: s_cmp → s_cbranch taken to next instruction
    TIME(7, asm volatile(REP64("s_cmp_eq_u32 %0, %0\ns_cbranch_scc1 1f\n1:\n") : "+s"(s) :: "scc");)
    // 8: s_waitcnt lgkmcnt(0) alone (nothing outstanding)
    TIME(8, asm volatile(REP64("s_waitcnt lgkmcnt(0)\n"));)
    // 9: v_writelane chain via m0
    TIME(9, asm volatile("s_mov_b32 m0, 3\n" REP64("v_writelane_b32 %0, %1, m0\n") : "+v"(v) : "s"(s) : "m0");)
    // 10: ds_write then ds_read same address, wait (LDS store→load)
    {
        int addr = 0, x = lane;
        TIME(10, asm volatile(REP64("ds_write_b32 %1, %0\nds_read_b32 %0, %1\ns_waitcnt lgkmcnt(0)\n") : "+v"(x) : "v"(addr));)
        r += x;
    }
    // 11: v_cmp_lt_u64 + 2 cndmask (64-bit select) chain
    {
        unsigned long long a = lane, b = 5;
        int x = lane, y = 3;
        TIME(11, asm volatile(REP64("v_cmp_lt_u64 vcc, %1, %2\nv_cndmask_b32 %0, %3, %0, vcc\n") : "+v"(x) : "v"(a), "v"(b), "v"(y) : "vcc");)
        r += x;
    }
    // 12: s_and_saveexec + restore (exec toggling)
    TIME(12, asm volatile(REP64("s_and_saveexec_b64 s[20:21], -1\ns_or_b64 exec, exec, s[20:21]\n") ::: "s20", "s21");)
    // 13: v_readfirstlane chain into s_cmp
    TIME(13, asm volatile(REP64("v_readfirstlane_b32 %1, %0\ns_cmp_eq_u32 %1, 0\n") : "+v"(v), "+s"(s) :: "scc");)
    // 14: ballot → s_ff1 → v_readlane by that lane → v_add (select-a-lane round trip)
    {
        int x = lane;
        TIME(14, asm volatile(REP64("v_cmp_eq_u32 vcc, 5, %0\ns_ff1_i32_b64 %1, vcc\nv_readlane_b32 %1, %0, %1\nv_add_u32 %0, %1, %0\n") : "+v"(x), "+s"(s) :: "vcc");)
        r += x;
    }
    // 15: DPP row_ror:1 mov chain (2 wait states each)
    TIME(15, asm volatile(REP64("s_nop 1\nv_mov_b32_dpp %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf\n") : "+v"(v));)
    // 16: ds_bpermute dependent chain
    {
        int x = lane * 4;
        TIME(16, asm volatile(REP64("ds_bpermute_b32 %0, %0, %0\ns_waitcnt lgkmcnt(0)\n") : "+v"(x));)
        r += x;
    }
    // 17: ds_read_b128 dependent chain (address from the first dword)
    {
        int x = 0;
        TIME(17, asm volatile(REP64("ds_read_b128 v[40:43], %0\ns_waitcnt lgkmcnt(0)\nv_and_b32 %0, 0, v40\n") : "+v"(x) :: "v40", "v41", "v42", "v43");)
        r += x;
    }
    // 18: v_readlane (lane 0) → v_writelane m0 → (chain through the VGPR)
    TIME(18, asm volatile("s_mov_b32 m0, 3\n" REP64("v_readlane_b32 %1, %0, 0\nv_writelane_b32 %0, %1, m0\n") : "+v"(v), "+s"(s) :: "m0");)
    // 19: 8-lane 64-bit min step via DPP (2 movs + cmp + 2 cndmask) dependent chain
    TIME(19, asm volatile("v_mov_b32 v40, %0\nv_mov_b32 v41, 0\n" REP64("s_nop 1\nv_mov_b32_dpp v42, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp v43, v41 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_cmp_lt_u64 vcc, v[42:43], v[40:41]\nv_cndmask_b32 v40, v40, v42, vcc\nv_cndmask_b32 v41, v41, v43, vcc\n") "v_add_u32 %0, %0, v40\n" : "+v"(v) :: "vcc", "v40", "v41", "v42", "v43");)
    // 20: readfirstlane → s_cmp → s_cbranch_scc taken (loop control from a VGPR)
    TIME(20, asm volatile(REP64("v_readfirstlane_b32 %1, %0\ns_cmp_eq_u32 %1, %1\ns_cbranch_scc1 1f\n1:\n") : "+v"(v), "+s"(s) :: "scc");)
    // 21: v_cmp → s_and_b64 vcc, exec → s_cbranch_vccz (taken)
    TIME(21, asm volatile(REP64("v_cmp_eq_u32 vcc, %0, %0\ns_and_b64 vcc, exec, vcc\ns_cbranch_vccz 1f\n1:\n") : "+v"(v) :: "vcc");)
    // 22: v_add_u32 + v_cndmask dependent (VALU-only select chain)
    TIME(22, asm volatile(REP64("v_cmp_gt_u32 vcc, %0, 7\nv_cndmask_b32 %0, 3, %0, vcc\n") : "+v"(v) :: "vcc");)
    // 23: v_min3_u32 dep chain
    TIME(23, asm volatile(REP64("v_min3_u32 %0, %0, %0, 60\n") : "+v"(v));)
    sink[lane] = v + r + s;
}

int main() {
    unsigned long long* d;
    int* sk;
    hipMalloc(&d, 64 * 8);
    hipMalloc(&sk, 256 * 4);
    hipMemset(d, 0, 64 * 8);
    unsigned long long h[64];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_ubench, dim3(1), dim3(64), 0, 0, d, sk);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
    const char* names[] = {"v_add dep", "s_add dep", "v_add 4 indep chains (per instr)", "readlane+s_add+v_add (per triple, +s_nop4)",
                           "ds_read dep+wait", "s_nop1+v_min_dpp", "v_cmp+cbranch(not taken) pair", "s_cmp+cbranch(taken) pair",
                           "s_waitcnt alone", "v_writelane m0", "ds_write+ds_read+wait", "v_cmp_u64+cndmask pair",
                           "saveexec+restore pair", "readfirstlane+s_cmp pair",
                           "ballot+s_ff1+readlane(sel)+v_add", "s_nop1+dpp row_ror mov", "ds_bpermute dep+wait",
                           "ds_read_b128 dep+wait+v_and", "readlane+writelane(m0) pair", "8-lane u64 min step (5 VALU)",
                           "readfirstlane+s_cmp+cbranch taken", "v_cmp+s_and vcc+cbranch_vccz", "v_cmp+cndmask pair",
                           "v_min3 dep"};
    for (int i = 0; i < 24; ++i) printf("%-44s %6.2f cyc\n", names[i], h[i] / (64.0 * 16));
    return 0;
}
