// fit_timeline.hip — SPEC §2b, time-windowed backfill over a slot horizon (BASELINE config C5):
// hand-written CDNA4 (gfx950) kernels.  DESIGN.md §3.8.
//
// Node state is each node's free-resource timeline, run-length encoded: a canonical list of runs
// (Seg: end slot, cpu, mem, gpu) in a fixed per-node slab of TL_MAX_SLOTS entries in HBM (only
// the used prefix is ever touched, so the working set is the live runs, L2/MALL resident).  The
// speculative rounds are the same as the plain fit (fit_common.h): k_scan_tl keeps the exact
// top-KS keys per (job, block-slice) plus a bound against the round-start timelines; k_commit_tl
// walks the window in priority order with a dirty set of at most TL_UCAP nodes (one per lane),
// re-evaluating dirty nodes exactly on their current runs, and reserves each decision in place.
//   key = start << 54 | score << 22 | position   (earliest start, then best fit, then node)
// The sequential semantics reproduced bit-exactly is oracle/fitref_tl.c:ref_place_tl.
#include "fit_common.h"

namespace fitgpu {

__device__ __forceinline__ uint64_t tl_key(int32_t s, int32_t mc, int32_t mm, int32_t mg,
                                           int32_t jc, int32_t jm, int32_t jg, uint32_t pos) {
    const uint32_t sc = (min((uint32_t)(mg - jg), 255u) << 24) |
                        (min((uint32_t)(mc - jc), 4095u) << 12) |
                        min((uint32_t)(mm - jm) >> 10, 4095u);
    return ((uint64_t)(uint32_t)s << 54) | ((uint64_t)sc << TL_POS_BITS) | pos;
}

// Earliest start of a d-slot window whose every run holds (jc, jm, jg), and its key.  One lane
// per (job, node); `live` lanes walk the node's runs [0, cnt).  A lane stops early once every
// start it could still find is later than `cut`'s start (its key would lose to `cut`).  The loop
// is wave-uniform (ballot exit), so with a uniform `sg` the run loads are scalar.
__device__ __forceinline__ uint64_t tl_eval(const Seg* sg, int cnt, bool live, int32_t jc,
                                            int32_t jm, int32_t jg, int32_t d, int32_t H,
                                            uint32_t pos, uint64_t cut) {
    const int32_t lim = cut == KEY_INF ? H : (int32_t)(cut >> 54);
    uint64_t key = KEY_INF;
    int32_t ra = -1, mc = 0, mm = 0, mg = 0, a = 0;
    live = live && d <= H;
    for (int i = 0;; ++i) {
        const bool l = live && i < cnt;
        if (!__ballot(l)) break;
        if (l) {
            const Seg g = sg[i];
            if (g.cpu >= jc && g.mem >= jm && g.gpu >= jg) {
                if (ra < 0) {
                    ra = a;
                    mc = g.cpu;
                    mm = g.mem;
                    mg = g.gpu;
                } else {
                    mc = min(mc, g.cpu);
                    mm = min(mm, g.mem);
                    mg = min(mg, g.gpu);
                }
                if (g.end - ra >= d) {
                    key = tl_key(ra, mc, mm, mg, jc, jm, jg, pos);
                    live = false;
                } else if (ra > lim) {
                    live = false;
                }
            } else {
                ra = -1;
                if (g.end + d > H || g.end > lim) live = false;  // no (competitive) start left
            }
            a = g.end;
        }
    }
    return key;
}

// ------------------------------------------------------------------------------ k_build_tl
// One thread per node position: base free columns + sorted release events → canonical runs.
// Values are clamped to [-1, INT32_MAX]; slots >= min(H, avail / slot_min) hold -1.
__global__ void k_build_tl(const int32_t* __restrict__ cpu, const int32_t* __restrict__ mem,
                           const int32_t* __restrict__ gpu, const int32_t* __restrict__ av,
                           const int32_t* __restrict__ perm, int32_t nn, int32_t H,
                           int32_t slot_min, const int32_t* __restrict__ off,
                           const int32_t* __restrict__ rs, const int32_t* __restrict__ rc,
                           const int32_t* __restrict__ rm, const int32_t* __restrict__ rg,
                           Seg* __restrict__ slab, int32_t* __restrict__ segcnt,
                           uint32_t* __restrict__ err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    const int x = perm[i];
    Seg* sg = slab + (int64_t)i * TL_MAX_SLOTS;
    const int32_t u = av[x] < 0 ? 0 : min(av[x] / slot_min, H);
    int64_t ac = cpu[x], am = mem[x], ag = gpu[x];
    auto cl = [](int64_t v) { return (int32_t)max<int64_t>(-1, min<int64_t>(v, 0x7fffffff)); };
    int n = 0, a = 0;
    auto emit = [&](int32_t end, int32_t vc, int32_t vm, int32_t vg) {
        if (end <= a) return;
        if (n > 0 && sg[n - 1].cpu == vc && sg[n - 1].mem == vm && sg[n - 1].gpu == vg)
            sg[n - 1].end = end;
        else
            sg[n++] = Seg{end, vc, vm, vg};
        a = end;
    };
    bool bad = false;
    const int e0 = off ? off[x] : 0, e1 = off ? off[x + 1] : 0;
    if (e1 < e0) bad = true;
    for (int e = e0; e < e1 && !bad; ++e) {
        const int32_t r = rs[e];
        if ((e > e0 && r < rs[e - 1]) || rc[e] < 0 || rm[e] < 0 || rg[e] < 0) {
            bad = true;
            break;
        }
        if (r >= u) continue;  // after the usable horizon: validated only
        if (r > a) emit(r, cl(ac), cl(am), cl(ag));
        ac += rc[e];
        am += rm[e];
        ag += rg[e];
    }
    if (bad) {
        atomicOr(err, 1u);
        n = 0;
        a = 0;
    }
    emit(u, cl(ac), cl(am), cl(ag));
    emit(H, -1, -1, -1);
    segcnt[i] = n;
}

// ----------------------------------------------------------------------------- k_scan_tl
// Block = SCAN_JOBS jobs (lanes) × one block-slice of SCAN_WAVES sub-slices; each wave walks
// its nodes' runs with wave-uniform (scalar) loads and keeps the exact top-KS keys per lane;
// the 8 lists merge through LDS exactly as in k_scan (fit_common.h).
__global__ __launch_bounds__(SCAN_WAVES * 64) void k_scan_tl(
    const NodeRec* __restrict__ rec, const Seg* __restrict__ slab,
    const int32_t* __restrict__ segcnt, const int32_t* __restrict__ jl,
    const int32_t* __restrict__ jcpu, const int32_t* __restrict__ jmem,
    const int32_t* __restrict__ jgpu, const int32_t* __restrict__ jwall,
    const uint16_t* __restrict__ jpart, const CompPlan* __restrict__ plan, int ncomp,
    uint64_t* __restrict__ cand, uint64_t* __restrict__ bnd, JobRec* __restrict__ wjob,
    int32_t H, int32_t slot_min) {
    __shared__ uint64_t xk[SCAN_WAVES / 2][KS][64];
    const int c = find_comp(plan, ncomp, blockIdx.x);
    const CompPlan P = plan[c];
    const int local = blockIdx.x - P.blk0;
    const int tile = __builtin_amdgcn_readfirstlane(local / P.nslice);
    const int s = __builtin_amdgcn_readfirstlane(local - tile * P.nslice);
    if (tile * SCAN_JOBS >= P.w) return;  // block-uniform
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int t = tile * SCAN_JOBS + lane;
    const bool active = t < P.w;

    JobRec J;
    J.q = active ? jl[P.jbase + t] : 0;
    J.cpu = active ? jcpu[J.q] : 0;
    J.mem = active ? jmem[J.q] : 0;
    J.gpu = active ? jgpu[J.q] : 0;
    // wall → slots occupied: ceil(wall / slot_min), at least 1 (oracle ref_slots)
    const int64_t dw = active ? ((int64_t)jwall[J.q] + slot_min - 1) / slot_min : 1;
    J.wall = (int32_t)max<int64_t>(1, min<int64_t>(dw, 0x7fffffff));
    J.pbit = active ? (1u << jpart[J.q]) : 0u;
    J.k = 1;
    J.pad = 0;

    uint64_t key[KS];
#pragma unroll
    for (int i = 0; i < KS; ++i) key[i] = KEY_INF;
    const int n0 = P.sb + (s * SCAN_WAVES + wave) * P.sub;
    const int n1 = min(P.se, n0 + P.sub);
    for (int x = n0; x < n1; ++x) {
        const NodeRec r = rec[x];
        const bool live = (r.mask & J.pbit) != 0u;
        const uint64_t k = tl_eval(slab + (int64_t)x * TL_MAX_SLOTS, segcnt[x], live, J.cpu,
                                   J.mem, J.gpu, J.wall, H, (uint32_t)x, key[KS - 1]);
        if (k < key[KS - 1]) topk_insert(key, k);
    }
#pragma unroll
    for (int h = SCAN_WAVES / 2; h >= 1; h >>= 1) {
        if (wave >= h && wave < 2 * h) {
#pragma unroll
            for (int i = 0; i < KS; ++i) xk[wave - h][i][lane] = key[i];
        }
        __syncthreads();
        if (wave < h) {
            uint64_t o[KS];
#pragma unroll
            for (int i = 0; i < KS; ++i) o[i] = xk[wave][i][lane];
            merge_lists(key, o);
        }
        __syncthreads();
    }
    if (wave != 0 || !active) return;
    uint64_t* dst = cand + P.cand_off + ((int64_t)t * P.nslice + s) * KS;
#pragma unroll
    for (int i = 0; i < KS; i += 2) {
        ulonglong2 v;
        v.x = key[i];
        v.y = key[i + 1];
        *reinterpret_cast<ulonglong2*>(dst + i) = v;
    }
    if (key[KS - 1] != KEY_INF)
        atomicMin(reinterpret_cast<unsigned long long*>(bnd + P.slot0 + t),
                  (unsigned long long)key[KS - 1]);
    if (s == 0) wjob[P.slot0 + t] = J;
}

// --------------------------------------------------------------------------- k_commit_tl
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Reserve (jc, jm, jg) on slots [s, e) of one node's run list, by the whole wave: the runs from
// the one before the window to the end are split at s and e into LDS scratch (pass 1, prefix
// sums over piece counts), then equal neighbours merge and the list is written back (pass 2).
// Only the two window edges can create runs or merge, so the list stays canonical.
__device__ void tl_reserve(Seg* sg, int32_t* cntp, int32_t s, int32_t e, int32_t jc, int32_t jm,
                           int32_t jg, Seg* scr) {
    const int lane = threadIdx.x & 63;
    const int n = __builtin_amdgcn_readfirstlane(*cntp);
    int i0 = n;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        const uint64_t m = __ballot(i < n && sg[i].end > s);
        if (m) {
            i0 = b + __builtin_ctzll(m);
            break;
        }
    }
    const int r0 = max(i0 - 1, 0);
    int np = 0;
    for (int b = r0; b < n; b += 64) {
        const int i = b + lane;
        const bool v = i < n;
        const Seg g = v ? sg[i] : Seg{0, 0, 0, 0};
        const int32_t a = (v && i > 0) ? sg[i - 1].end : 0;
        const bool ov = v && a < e && g.end > s;
        const bool hd = ov && a < s;
        const bool tl = ov && g.end > e;
        const int pc = v ? (ov ? 1 + (int)hd + (int)tl : 1) : 0;
        const uint64_t m0 = __ballot(pc & 1), m1 = __ballot(pc >> 1);
        int o = np + lanes_below(m0) + 2 * lanes_below(m1);
        if (v) {
            if (!ov) {
                scr[o] = g;
            } else {
                if (hd) scr[o++] = Seg{s, g.cpu, g.mem, g.gpu};
                scr[o++] = Seg{min(g.end, e), g.cpu - jc, g.mem - jm, g.gpu - jg};
                if (tl) scr[o] = g;
            }
        }
        np += __popcll(m0) + 2 * __popcll(m1);
    }
    int no = 0;
    for (int b = 0; b < np; b += 64) {
        const int k = b + lane;
        const bool v = k < np;
        const Seg p = v ? scr[k] : Seg{0, 0, 0, 0};
        const Seg q = k + 1 < np ? scr[k + 1] : Seg{0, -2, -2, -2};
        const bool keep = v && (k + 1 >= np || p.cpu != q.cpu || p.mem != q.mem || p.gpu != q.gpu);
        const uint64_t mk = __ballot(keep);
        if (keep) sg[r0 + no + lanes_below(mk)] = p;
        no += __popcll(mk);
    }
    if (lane == 0) *cntp = r0 + no;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // later reads of this list see the writes
}

// One wave per component: the speculative-prefix commit of the plain fit (fit_common.h) with
// run-list evaluation of the dirty nodes (one per lane) and in-place reservation.
template <int EPL>
__global__ __launch_bounds__(64) void k_commit_tl(
    const NodeRec* __restrict__ rec, Seg* __restrict__ slab, int32_t* __restrict__ segcnt,
    const CompPlan* __restrict__ plan, const uint64_t* __restrict__ cand, int64_t rank_stride,
    int nranks, const uint64_t* __restrict__ bnd, const JobRec* __restrict__ wjob,
    int32_t* __restrict__ out, int32_t* __restrict__ outs, CommitResult* __restrict__ res,
    int32_t H) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Seg* scr = reinterpret_cast<Seg*>(smem);
    uint32_t* bitmap = reinterpret_cast<uint32_t*>(smem + sizeof(Seg) * TL_MAX_SLOTS);
    const int c = blockIdx.x;
    const CompPlan P = plan[c];
    const int lane = threadIdx.x & 63;
    if (P.w == 0) {
        if (lane == 0) res[c] = CommitResult{0, 0, 0, 0};
        return;
    }
    const int nwords = (P.ne - P.nb + 31) >> 5;
    for (int i = lane; i < nwords; i += 64) bitmap[i] = 0u;

    const int per_rank = P.nslice * KS;
    const int E = nranks * per_rank;
    int64_t off[EPL];
    bool has[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + 64 * k;
        const int g = e / per_rank;
        has[k] = e < E;
        off[k] = has[k] ? g * rank_stride + P.cand_off + (e - g * per_rank) : P.cand_off;
    }
    const uint32_t nb = (uint32_t)P.nb;
    int nu = 0, placed = 0, stop = 0, t = 0;
    uint32_t upos = 0u, umask = 0u;  // dirty node of this lane (lane < nu)
    for (; t < P.w; ++t) {
        const JobRec J = wjob[P.slot0 + t];
        const uint64_t B = bnd[P.slot0 + t];
        uint64_t cm = KEY_INF;
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
            const uint64_t kk = cand[off[k] + (int64_t)t * per_rank];
            const bool v = has[k] && kk <= B && kk != KEY_INF;
            const uint32_t rel = v ? ((uint32_t)kk & TL_POS_MASK) - nb : 0u;
            const bool clean = v && !((bitmap[rel >> 5] >> (rel & 31)) & 1u);
            cm = umin64(cm, clean ? kk : KEY_INF);
        }
        const uint64_t cw = wave_min_key(cm);
        const bool dl = lane < nu && (umask & J.pbit) != 0u;
        const uint64_t dk = tl_eval(slab + (int64_t)upos * TL_MAX_SLOTS, dl ? segcnt[upos] : 0, dl,
                                    J.cpu, J.mem, J.gpu, J.wall, H, upos, cw);
        const uint64_t best = umin64(cw, wave_min_key(dk));
        if (B != KEY_INF && best > B) {
            stop = 1;  // a node outside the candidate lists could win: rescan next round
            break;
        }
        int32_t node = -1, start = -1;
        if (best != KEY_INF) {
            const uint32_t pos = (uint32_t)best & TL_POS_MASK;
            if (__ballot(dk == best) == 0ull) {  // a clean candidate wins: it becomes dirty
                if (nu == TL_UCAP) {
                    stop = 2;
                    break;
                }
                if (lane == nu) {
                    upos = pos;
                    umask = rec[pos].mask;
                }
                if (lane == 0) {
                    const uint32_t rel = pos - nb;
                    bitmap[rel >> 5] |= 1u << (rel & 31);
                }
                ++nu;
            }
            start = (int32_t)(best >> 54);
            tl_reserve(slab + (int64_t)pos * TL_MAX_SLOTS, segcnt + pos, start, start + J.wall,
                       J.cpu, J.mem, J.gpu, scr);
            node = rec[pos].orig;
            ++placed;
        }
        if (lane == 0) {
            out[J.q] = node;
            outs[J.q] = start;
        }
    }
    if (lane == 0) res[c] = CommitResult{t, stop, nu, placed};
}

// Dense read-back (tests, fit_read_timeline): one block per node position, threads over slots.
__global__ void k_expand_tl(const NodeRec* __restrict__ rec, const Seg* __restrict__ slab,
                            const int32_t* __restrict__ segcnt, int32_t H,
                            int32_t* __restrict__ oc, int32_t* __restrict__ om,
                            int32_t* __restrict__ og) {
    const int i = blockIdx.x;
    const Seg* sg = slab + (int64_t)i * TL_MAX_SLOTS;
    const int n = segcnt[i];
    const int64_t base = (int64_t)rec[i].orig * H;
    for (int t = threadIdx.x; t < H; t += blockDim.x) {
        int lo = 0, hi = n - 1;  // first run with end > t
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sg[mid].end > t) hi = mid;
            else lo = mid + 1;
        }
        const Seg g = sg[lo];
        oc[base + t] = g.cpu;
        om[base + t] = g.mem;
        og[base + t] = g.gpu;
    }
}

// ------------------------------------------------------------------ host launch wrappers
hipError_t launch_build_tl(hipStream_t st, const int32_t* cpu, const int32_t* mem,
                           const int32_t* gpu, const int32_t* av, const int32_t* perm,
                           int32_t nn, int32_t H, int32_t slot_min, const int32_t* off,
                           const int32_t* rs, const int32_t* rc, const int32_t* rm,
                           const int32_t* rg, Seg* slab, int32_t* segcnt, uint32_t* err) {
    if (nn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_build_tl, dim3((nn + 255) / 256), dim3(256), 0, st, cpu, mem, gpu, av,
                       perm, nn, H, slot_min, off, rs, rc, rm, rg, slab, segcnt, err);
    return hipGetLastError();
}

hipError_t launch_scan_tl(int blocks, hipStream_t st, const NodeRec* rec, const Seg* slab,
                          const int32_t* segcnt, const int32_t* jl, const int32_t* jcpu,
                          const int32_t* jmem, const int32_t* jgpu, const int32_t* jwall,
                          const uint16_t* jpart, const CompPlan* plan, int ncomp, uint64_t* cand,
                          uint64_t* bnd, JobRec* wjob, int32_t H, int32_t slot_min) {
    hipLaunchKernelGGL(k_scan_tl, dim3(blocks), dim3(SCAN_WAVES * 64), 0, st, rec, slab, segcnt,
                       jl, jcpu, jmem, jgpu, jwall, jpart, plan, ncomp, cand, bnd, wjob, H,
                       slot_min);
    return hipGetLastError();
}

size_t commit_tl_lds_bytes(int32_t max_component_nodes) {
    return sizeof(Seg) * TL_MAX_SLOTS + (size_t)((max_component_nodes + 31) / 32) * 4;
}

hipError_t launch_commit_tl(int ncomp, int epl, size_t lds, hipStream_t st, const NodeRec* rec,
                            Seg* slab, int32_t* segcnt, const CompPlan* plan,
                            const uint64_t* cand, int64_t rank_stride, int nranks,
                            const uint64_t* bnd, const JobRec* wjob, int32_t* out, int32_t* outs,
                            CommitResult* res, int32_t H) {
#define FIT_COMMIT_TL(EPL)                                                                    \
    hipLaunchKernelGGL(k_commit_tl<EPL>, dim3(ncomp), dim3(64), lds, st, rec, slab, segcnt,   \
                       plan, cand, rank_stride, nranks, bnd, wjob, out, outs, res, H)
    if (epl <= 1) FIT_COMMIT_TL(1);
    else if (epl <= 2) FIT_COMMIT_TL(2);
    else if (epl <= 4) FIT_COMMIT_TL(4);
    else if (epl <= 8) FIT_COMMIT_TL(8);
    else return hipErrorInvalidValue;
#undef FIT_COMMIT_TL
    return hipGetLastError();
}

hipError_t launch_expand_tl(hipStream_t st, const NodeRec* rec, const Seg* slab,
                            const int32_t* segcnt, int32_t nn, int32_t H, int32_t* oc,
                            int32_t* om, int32_t* og) {
    if (nn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_expand_tl, dim3(nn), dim3(256), 0, st, rec, slab, segcnt, H, oc, om, og);
    return hipGetLastError();
}

}  // namespace fitgpu
