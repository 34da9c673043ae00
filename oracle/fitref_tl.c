/* oracle/fitref_tl.c — CPU restatement of SPEC §2b, time-windowed backfill (TEST INFRASTRUCTURE
 * ONLY: the checker, never the product; see fitref.h for who may load it).
 *
 * The reference has walltime only as a partition limit (pkg/slurm-agent/parse.go:128-138, MaxTime)
 * and as the job's `--time` (pkg/slurm-bridge-operator/parse.go:84-91); it has no reservation
 * timeline and no backfill — slurmctld's backfill is external C.  So, like
 * ref_place, this is "parity unpinned" vs the reference: it restates DESIGN.md §2b, which reuses
 * the reference's walltime units (ParseDuration → minutes) and the partition MaxTime rejection.
 *
 * Deliberately naive: a dense [node][slot][dim] int32 timeline, an O(H) slot walk per (job, node),
 * no segments, no candidate lists — nothing shared with the GPU algorithm.
 */
#include <stdint.h>
#include <string.h>

#include "fitref.h"

static int32_t clamp_i64(int64_t v) {
    if (v < -1) return -1;
    if (v > INT32_MAX) return INT32_MAX;
    return (int32_t)v;
}

/* DESIGN.md §2b "timeline": slot t < U holds base + Σ releases with slot <= t (slots <= 0 count
 * from the start), clamped to [-1, INT32_MAX]; U = min(H, avail_min / slot_min); t >= U holds -1
 * (the node is not available there, nothing fits). */
int ref_build_timeline(int32_t n, int32_t H, int32_t slot_min, const int32_t* cpu_free,
                       const int32_t* mem_free, const int32_t* gpu_free, const int32_t* avail_min,
                       const int32_t* rel_off, const int32_t* rel_slot, const int32_t* rel_cpu,
                       const int32_t* rel_mem, const int32_t* rel_gpu, int32_t* tl) {
    if (n < 0 || H < 1 || H > 1024 || slot_min < 1) return -1;
    for (int32_t x = 0; x < n; x++) {
        int64_t u = avail_min[x] < 0 ? 0 : avail_min[x] / slot_min;
        if (u > H) u = H;
        int64_t acc[3] = {cpu_free[x], mem_free[x], gpu_free[x]};
        int32_t e = rel_off ? rel_off[x] : 0, e1 = rel_off ? rel_off[x + 1] : 0;
        for (int32_t t = 0; t < H; t++) {
            for (; e < e1 && rel_slot[e] <= t; e++) {
                if (e > rel_off[x] && rel_slot[e] < rel_slot[e - 1]) return -1; /* not sorted */
                if (rel_cpu[e] < 0 || rel_mem[e] < 0 || rel_gpu[e] < 0) return -1;
                acc[0] += rel_cpu[e];
                acc[1] += rel_mem[e];
                acc[2] += rel_gpu[e];
            }
            int32_t* v = tl + ((int64_t)x * H + t) * 3;
            for (int k = 0; k < 3; k++) v[k] = t < u ? clamp_i64(acc[k]) : -1;
        }
        for (; e < e1; e++) /* releases past the horizon: validated, otherwise ignored */
            if ((e > rel_off[x] && rel_slot[e] < rel_slot[e - 1]) || rel_cpu[e] < 0 ||
                rel_mem[e] < 0 || rel_gpu[e] < 0)
                return -1;
    }
    return 0;
}

/* slots a job of `wall` minutes occupies: ceil(wall / slot_min), at least 1 */
int32_t ref_slots(int32_t wall, int32_t slot_min) {
    int64_t d = ((int64_t)wall + slot_min - 1) / slot_min;
    return d < 1 ? 1 : (d > INT32_MAX ? INT32_MAX : (int32_t)d);
}

/* Key of (job, node) on the current timeline: earliest feasible start s, then the
 * best-fit score of the window minimum, then the node id.  UINT64_MAX: no start fits. */
uint64_t ref_key_tl(int32_t x, int32_t H, const int32_t* row /* [H][3] */, uint32_t mask,
                    int32_t cpu, int32_t mem, int32_t gpu, int32_t d, int32_t part,
                    int32_t* out_start) {
    *out_start = -1;
    if (!((mask >> part) & 1u) || d > H) return UINT64_MAX;
    int32_t run = 0, s = -1;
    for (int32_t t = 0; t < H; t++) {
        const int32_t* v = row + (int64_t)t * 3;
        if (v[0] >= cpu && v[1] >= mem && v[2] >= gpu) {
            if (++run == d) {
                s = t - d + 1;
                break;
            }
        } else {
            run = 0;
            if (t + 1 + d > H) break; /* no window fits after t */
        }
    }
    if (s < 0) return UINT64_MAX;
    int32_t mc = INT32_MAX, mm = INT32_MAX, mg = INT32_MAX;
    for (int32_t t = s; t < s + d; t++) {
        const int32_t* v = row + (int64_t)t * 3;
        if (v[0] < mc) mc = v[0];
        if (v[1] < mm) mm = v[1];
        if (v[2] < mg) mg = v[2];
    }
    uint32_t gr = (uint32_t)(mg - gpu), cr = (uint32_t)(mc - cpu), mr = (uint32_t)(mm - mem) >> 10;
    if (gr > 255u) gr = 255u;
    if (cr > 4095u) cr = 4095u;
    if (mr > 4095u) mr = 4095u;
    const uint64_t score = ((uint64_t)gr << 24) | ((uint64_t)cr << 12) | mr;
    *out_start = s;
    return ((uint64_t)s << 54) | (score << 22) | (uint32_t)x;
}

/* SPEC §2b sequential priority-order backfill.  out_node[j]: node id, -1 unplaced, -2 rejected;
 * out_start[j]: start slot (or -1).  tl is updated in place.  stats: placed, unplaced, rejected,
 * evals. */
int ref_place_tl(int32_t n, int32_t H, int32_t slot_min, int32_t* tl, const uint32_t* part_mask,
                 int32_t p, const int32_t* max_time, const int32_t* max_cpus,
                 const int32_t* max_mem, int32_t j, const int32_t* cpu, const int32_t* mem,
                 const int32_t* gpu, const int32_t* wall, const uint16_t* part, int32_t* out_node,
                 int32_t* out_start, int64_t* stats) {
    if (n < 0 || n > (1 << 22) || j < 0 || p < 0 || p > 32 || H < 1 || H > 1024 || slot_min < 1)
        return -1;
    for (int32_t q = 0; q < j; q++)
        if (cpu[q] < 0 || mem[q] < 0 || gpu[q] < 0 || wall[q] < 0) return -1;
    int64_t placed = 0, unplaced = 0, rejected = 0, evals = 0;
    for (int32_t q = 0; q < j; q++) {
        const int pq = part[q];
        out_node[q] = -1;
        out_start[q] = -1;
        if (pq >= p || (max_time[pq] >= 0 && wall[q] > max_time[pq]) ||
            (max_cpus[pq] >= 0 && cpu[q] > max_cpus[pq]) ||
            (max_mem[pq] >= 0 && mem[q] > max_mem[pq])) {
            out_node[q] = -2;
            rejected++;
            continue;
        }
        const int32_t d = ref_slots(wall[q], slot_min);
        uint64_t best = UINT64_MAX;
        for (int32_t x = 0; x < n; x++) {
            int32_t s;
            const uint64_t k = ref_key_tl(x, H, tl + (int64_t)x * H * 3, part_mask[x], cpu[q],
                                          mem[q], gpu[q], d, pq, &s);
            if (k < best) best = k;
        }
        evals += n;
        if (best == UINT64_MAX) {
            unplaced++;
            continue;
        }
        const int32_t x = (int32_t)(best & 0x3fffffu), s = (int32_t)(best >> 54);
        for (int32_t t = s; t < s + d; t++) {
            int32_t* v = tl + ((int64_t)x * H + t) * 3;
            v[0] -= cpu[q];
            v[1] -= mem[q];
            v[2] -= gpu[q];
        }
        out_node[q] = x;
        out_start[q] = s;
        placed++;
    }
    if (stats) {
        stats[0] = placed;
        stats[1] = unplaced;
        stats[2] = rejected;
        stats[3] = evals;
    }
    return 0;
}
