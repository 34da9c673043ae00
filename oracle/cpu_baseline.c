/* oracle/cpu_baseline.c — fair CPU baselines of the placement path (TEST / BENCH INFRASTRUCTURE:
 * bench.py's cpu_baseline leg and tests/ only; never linked into or called by the product).
 *
 * Same SPEC semantics as ref_place / ref_place_tl (fitref.c:498-560, fitref_tl.c:102-154) —
 * the results are identical (tests/test_cpu_baseline.py) — but organised the way a competent CPU
 * implementation would be, so the GPU is compared against more than the naive port:
 *
 *   component-aware  Partitions that share no node are independent.  Each job is
 *                    evaluated only against the nodes of its partition component, held as a
 *                    contiguous SoA copy (cache-resident), with a branch-free key loop the
 *                    compiler vectorises (target_clones: AVX-512 / AVX2 / baseline x86-64).
 *   multicore        The components are independent sequences, so they run on separate threads
 *                    (largest first, claimed from a shared counter); within a component the
 *                    sequential priority order is kept.  BASELINE.md's "parallel per-job argmin,
 *                    serial commit" variant needs a barrier per job (~1 µs at 16 threads) on a
 *                    ~6k-node scan of ~10 µs, so this decomposition dominates it at C3; at one
 *                    component (c3o) both degenerate to the single-thread scan.
 *
 * cpu_place: k = 1 jobs (C2/C3/c3o).  cpu_place_k: multi-node jobs (config C4, --nodes=k, the
 * k smallest distinct keys, all or nothing: fitref.c ref_place's rule), components on threads.
 * The backfill variant is §2b's one-node search.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fitref.h"

typedef struct {
    int32_t nc;            /* components */
    int32_t comp_of_part[32];
    int32_t* nodes;        /* node ids grouped by component, ascending inside each */
    int32_t* nb;           /* nc + 1 offsets into nodes */
    int32_t* jobs;         /* job ids grouped by component, priority order inside each */
    int32_t* jb;           /* nc + 1 offsets into jobs */
} comps_t;

static int find(int* par, int x) {
    while (par[x] != x) x = par[x] = par[par[x]];
    return x;
}

static int rejected_job(int32_t q, int32_t p, const int32_t* mt, const int32_t* mc, const int32_t* mm,
                        const int32_t* cpu, const int32_t* mem, const int32_t* wall, const uint16_t* part) {
    const int pq = part[q];
    return pq >= p || (mt[pq] >= 0 && wall[q] > mt[pq]) || (mc[pq] >= 0 && cpu[q] > mc[pq]) ||
           (mm[pq] >= 0 && mem[q] > mm[pq]);
}

/* union-find over the partitions the nodes join (like engine.cpp load_nodes_common) */
static int build_comps(comps_t* C, int32_t n, const uint32_t* mask, int32_t p, const int32_t* mt,
                       const int32_t* mc, const int32_t* mm, int32_t j, const int32_t* cpu,
                       const int32_t* mem, const int32_t* wall, const uint16_t* part, int32_t* out) {
    int par[32], used[32] = {0}, root[32];
    for (int i = 0; i < 32; i++) par[i] = i, root[i] = -1;
    for (int32_t x = 0; x < n; x++) {
        uint32_t m = mask[x];
        if (!m) continue;
        int lo = __builtin_ctz(m);
        for (; m; m &= m - 1) {
            int b = __builtin_ctz(m), ra = find(par, lo), rb = find(par, b);
            used[b] = 1;
            if (ra != rb) par[ra > rb ? ra : rb] = ra < rb ? ra : rb;
        }
    }
    C->nc = 0;
    for (int q = 0; q < 32; q++) {
        C->comp_of_part[q] = -1;
        if (!used[q]) continue;
        int r = find(par, q);
        if (root[r] < 0) root[r] = C->nc++;
        C->comp_of_part[q] = root[r];
    }
    C->nb = calloc(C->nc + 1, sizeof(int32_t));
    C->jb = calloc(C->nc + 1, sizeof(int32_t));
    C->nodes = malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    C->jobs = malloc(sizeof(int32_t) * (j > 0 ? j : 1));
    if (!C->nb || !C->jb || !C->nodes || !C->jobs) return -1;
    for (int32_t x = 0; x < n; x++)
        if (mask[x]) C->nb[C->comp_of_part[__builtin_ctz(mask[x])] + 1]++;
    for (int k = 0; k < C->nc; k++) C->nb[k + 1] += C->nb[k];
    int32_t* fill = malloc(sizeof(int32_t) * (C->nc + 1));
    memcpy(fill, C->nb, sizeof(int32_t) * (C->nc + 1));
    for (int32_t x = 0; x < n; x++)
        if (mask[x]) C->nodes[fill[C->comp_of_part[__builtin_ctz(mask[x])]]++] = x;
    /* jobs: rejected → -2 now; jobs of partitions without nodes stay -1 (unplaced) */
    for (int32_t q = 0; q < j; q++) {
        out[q] = -1;
        if (rejected_job(q, p, mt, mc, mm, cpu, mem, wall, part)) {
            out[q] = -2;
            continue;
        }
        int k = C->comp_of_part[part[q]];
        if (k >= 0) C->jb[k + 1]++;
    }
    for (int k = 0; k < C->nc; k++) C->jb[k + 1] += C->jb[k];
    memcpy(fill, C->jb, sizeof(int32_t) * (C->nc + 1));
    for (int32_t q = 0; q < j; q++) {
        if (out[q] == -2) continue;
        int k = C->comp_of_part[part[q]];
        if (k >= 0) C->jobs[fill[k]++] = q;
    }
    free(fill);
    return 0;
}

static void free_comps(comps_t* C) {
    free(C->nb);
    free(C->jb);
    free(C->nodes);
    free(C->jobs);
}

/* ---------------------------------------------------------------- plain fit, one component */
typedef struct {
    int32_t *cf, *mf, *gf;  /* per-position free columns */
    const int32_t* av;
    const uint32_t* mk;
    const int32_t* id;
} soa_t;

/* min key over positions [0, len) — branch-free so the loop vectorises */
__attribute__((target_clones("avx512f", "avx2", "default")))
static uint64_t scan_min(int32_t len, const int32_t* cf, const int32_t* mf, const int32_t* gf,
                         const int32_t* av, const uint32_t* mk, const int32_t* id, int32_t c,
                         int32_t m, int32_t g, int32_t w, uint32_t pbit) {
    uint64_t best = UINT64_MAX;
    for (int32_t i = 0; i < len; i++) {
        const int32_t dc = cf[i] - c, dm = mf[i] - m, dg = gf[i] - g, da = av[i] - w;
        const int ok = ((dc | dm | dg | da) >= 0) & ((mk[i] & pbit) != 0);
        uint32_t gr = (uint32_t)dg, cr = (uint32_t)dc, mr = (uint32_t)dm >> 10;
        gr = gr > 255u ? 255u : gr;
        cr = cr > 4095u ? 4095u : cr;
        mr = mr > 4095u ? 4095u : mr;
        const uint64_t key = ((uint64_t)((gr << 24) | (cr << 12) | mr) << 32) | (uint32_t)id[i];
        const uint64_t k2 = ok ? key : UINT64_MAX;
        best = k2 < best ? k2 : best;
    }
    return best;
}

typedef struct {
    const comps_t* C;
    int32_t *cpu_free, *mem_free, *gpu_free;
    const int32_t* avail;
    const uint32_t* mask;
    const int32_t *cpu, *mem, *gpu, *wall;
    const uint16_t* part;
    int32_t* out;
    const int32_t* order; /* components, largest first */
    volatile int32_t next;
    int64_t placed, evals;
    pthread_mutex_t mu;
} plain_job_t;

static void place_component(plain_job_t* T, int k, int64_t* placed, int64_t* evals) {
    const comps_t* C = T->C;
    const int32_t nb = C->nb[k], len = C->nb[k + 1] - nb;
    int32_t* cf = malloc(sizeof(int32_t) * (len > 0 ? len : 1) * 4);
    uint32_t* mk = malloc(sizeof(uint32_t) * (len > 0 ? len : 1));
    int32_t *mf = cf + len, *gf = mf + len, *av = gf + len;
    const int32_t* id = C->nodes + nb;
    for (int32_t i = 0; i < len; i++) {
        const int32_t x = id[i];
        cf[i] = T->cpu_free[x];
        mf[i] = T->mem_free[x];
        gf[i] = T->gpu_free[x];
        av[i] = T->avail[x];
        mk[i] = T->mask[x];
    }
    /* position of a node id inside the component (ids ascend) */
    for (int32_t t = C->jb[k]; t < C->jb[k + 1]; t++) {
        const int32_t q = C->jobs[t];
        const uint64_t best = scan_min(len, cf, mf, gf, av, mk, id, T->cpu[q], T->mem[q],
                                       T->gpu[q], T->wall[q], 1u << T->part[q]);
        *evals += len;
        if (best == UINT64_MAX) continue;
        const int32_t x = (int32_t)(uint32_t)best;
        int32_t lo = 0, hi = len - 1;
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (id[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        cf[lo] -= T->cpu[q];
        mf[lo] -= T->mem[q];
        gf[lo] -= T->gpu[q];
        T->out[q] = x;
        ++*placed;
    }
    for (int32_t i = 0; i < len; i++) {
        const int32_t x = id[i];
        T->cpu_free[x] = cf[i];
        T->mem_free[x] = mf[i];
        T->gpu_free[x] = gf[i];
    }
    free(cf);
    free(mk);
}

static void* plain_worker(void* arg) {
    plain_job_t* T = arg;
    int64_t placed = 0, evals = 0;
    for (;;) {
        const int32_t i = __atomic_fetch_add(&T->next, 1, __ATOMIC_RELAXED);
        if (i >= T->C->nc) break;
        place_component(T, T->order[i], &placed, &evals);
    }
    pthread_mutex_lock(&T->mu);
    T->placed += placed;
    T->evals += evals;
    pthread_mutex_unlock(&T->mu);
    return NULL;
}

static int32_t* lpt_order(const comps_t* C, int64_t (*work)(const comps_t*, int)) {
    int32_t* o = malloc(sizeof(int32_t) * (C->nc > 0 ? C->nc : 1));
    for (int i = 0; i < C->nc; i++) o[i] = i;
    for (int i = 1; i < C->nc; i++) /* insertion sort, descending work (nc <= 32) */
        for (int k = i; k > 0 && work(C, o[k]) > work(C, o[k - 1]); k--) {
            int32_t t = o[k];
            o[k] = o[k - 1];
            o[k - 1] = t;
        }
    return o;
}

static int64_t comp_work(const comps_t* C, int k) {
    return (int64_t)(C->jb[k + 1] - C->jb[k]) * (C->nb[k + 1] - C->nb[k]);
}

/* Plain fit (k = 1).  stats: placed, unplaced, rejected, evals.  threads <= 1: one thread. */
int cpu_place(int32_t n, int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free,
              const int32_t* avail_min, const uint32_t* part_mask, int32_t p,
              const int32_t* max_time, const int32_t* max_cpus, const int32_t* max_mem, int32_t j,
              const int32_t* cpu, const int32_t* mem, const int32_t* gpu, const int32_t* wall,
              const uint16_t* part, int32_t* out, int64_t* stats, int32_t threads) {
    if (n < 0 || j < 0 || p < 0 || p > 32) return -1;
    for (int32_t q = 0; q < j; q++)
        if (cpu[q] < 0 || mem[q] < 0 || gpu[q] < 0 || wall[q] < 0) return -1;
    comps_t C;
    memset(&C, 0, sizeof C);
    if (build_comps(&C, n, part_mask, p, max_time, max_cpus, max_mem, j, cpu, mem, wall, part, out)) {
        free_comps(&C);
        return -1;
    }
    plain_job_t T;
    memset(&T, 0, sizeof T);
    T.C = &C;
    T.cpu_free = cpu_free;
    T.mem_free = mem_free;
    T.gpu_free = gpu_free;
    T.avail = avail_min;
    T.mask = part_mask;
    T.cpu = cpu;
    T.mem = mem;
    T.gpu = gpu;
    T.wall = wall;
    T.part = part;
    T.out = out;
    T.order = lpt_order(&C, comp_work);
    pthread_mutex_init(&T.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    int started = 0;
    for (int i = 1; i < threads; i++)
        if (pthread_create(&th[started], NULL, plain_worker, &T) == 0) started++;
    plain_worker(&T);
    for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
    int64_t rejected = 0;
    for (int32_t q = 0; q < j; q++) rejected += out[q] == -2;
    if (stats) {
        stats[0] = T.placed;
        stats[1] = j - T.placed - rejected;
        stats[2] = rejected;
        stats[3] = T.evals;
    }
    pthread_mutex_destroy(&T.mu);
    free((void*)T.order);
    free_comps(&C);
    return 0;
}

/* ------------------------------------------------ plain fit with multi-node jobs (config C4) */
/* every position's key (UINT64_MAX = infeasible) — branch-free so the loop vectorises */
__attribute__((target_clones("avx512f", "avx2", "default")))
static void scan_keys(int32_t len, const int32_t* cf, const int32_t* mf, const int32_t* gf,
                      const int32_t* av, const uint32_t* mk, const int32_t* id, int32_t c, int32_t m,
                      int32_t g, int32_t w, uint32_t pbit, uint64_t* keys) {
    for (int32_t i = 0; i < len; i++) {
        const int32_t dc = cf[i] - c, dm = mf[i] - m, dg = gf[i] - g, da = av[i] - w;
        const int ok = ((dc | dm | dg | da) >= 0) & ((mk[i] & pbit) != 0);
        uint32_t gr = (uint32_t)dg, cr = (uint32_t)dc, mr = (uint32_t)dm >> 10;
        gr = gr > 255u ? 255u : gr;
        cr = cr > 4095u ? 4095u : cr;
        mr = mr > 4095u ? 4095u : mr;
        const uint64_t key = ((uint64_t)((gr << 24) | (cr << 12) | mr) << 32) | (uint32_t)id[i];
        keys[i] = ok ? key : UINT64_MAX;
    }
}

typedef struct {
    plain_job_t base;
    const uint16_t* nodes_k;
    int32_t kmax;
} k_job_t;

static int32_t pos_of(const int32_t* id, int32_t len, int32_t x) {
    int32_t lo = 0, hi = len - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (id[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

static void place_component_k(k_job_t* K, int k, int64_t* placed, int64_t* evals) {
    plain_job_t* T = &K->base;
    const comps_t* C = T->C;
    const int32_t nb = C->nb[k], len = C->nb[k + 1] - nb, kmax = K->kmax;
    int32_t* cf = malloc(sizeof(int32_t) * (len > 0 ? len : 1) * 4);
    uint32_t* mk = malloc(sizeof(uint32_t) * (len > 0 ? len : 1));
    uint64_t* keys = malloc(sizeof(uint64_t) * (len > 0 ? len : 1));
    int32_t *mf = cf + len, *gf = mf + len, *av = gf + len;
    const int32_t* id = C->nodes + nb;
    for (int32_t i = 0; i < len; i++) {
        const int32_t x = id[i];
        cf[i] = T->cpu_free[x];
        mf[i] = T->mem_free[x];
        gf[i] = T->gpu_free[x];
        av[i] = T->avail[x];
        mk[i] = T->mask[x];
    }
    for (int32_t t = C->jb[k]; t < C->jb[k + 1]; t++) {
        const int32_t q = C->jobs[t];
        int kq = K->nodes_k ? K->nodes_k[q] : 1;
        if (kq == 0) kq = 1;
        const int32_t c = T->cpu[q], m = T->mem[q], g = T->gpu[q];
        uint64_t best[64];
        if (kq == 1) {
            best[0] = scan_min(len, cf, mf, gf, av, mk, id, c, m, g, T->wall[q], 1u << T->part[q]);
        } else {  /* the kq smallest keys: one vectorised key pass, then a sorted insertion */
            scan_keys(len, cf, mf, gf, av, mk, id, c, m, g, T->wall[q], 1u << T->part[q], keys);
            for (int i = 0; i < kq; i++) best[i] = UINT64_MAX;
            for (int32_t i = 0; i < len; i++) {
                const uint64_t key = keys[i];
                if (key >= best[kq - 1]) continue;
                int u = kq - 1;
                while (u > 0 && best[u - 1] > key) {
                    best[u] = best[u - 1];
                    u--;
                }
                best[u] = key;
            }
        }
        *evals += len;
        if (best[kq - 1] == UINT64_MAX) continue; /* fewer than kq nodes fit: nothing taken */
        int32_t* o = T->out + (int64_t)q * kmax;
        for (int i = 0; i < kq; i++) {
            const int32_t x = (int32_t)(uint32_t)best[i], a = pos_of(id, len, x);
            cf[a] -= c;
            mf[a] -= m;
            gf[a] -= g;
            o[i] = x;
        }
        ++*placed;
    }
    for (int32_t i = 0; i < len; i++) {
        const int32_t x = id[i];
        T->cpu_free[x] = cf[i];
        T->mem_free[x] = mf[i];
        T->gpu_free[x] = gf[i];
    }
    free(cf);
    free(mk);
    free(keys);
}

static void* k_worker(void* arg) {
    k_job_t* K = arg;
    plain_job_t* T = &K->base;
    int64_t placed = 0, evals = 0;
    for (;;) {
        const int32_t i = __atomic_fetch_add(&T->next, 1, __ATOMIC_RELAXED);
        if (i >= T->C->nc) break;
        place_component_k(K, T->order[i], &placed, &evals);
    }
    pthread_mutex_lock(&T->mu);
    T->placed += placed;
    T->evals += evals;
    pthread_mutex_unlock(&T->mu);
    return NULL;
}

/* Plain fit with multi-node jobs: out[q * kmax + i] as ref_place writes it (fitref.c:650-712).
 * stats: placed, unplaced, rejected, evals.  threads <= 1: one thread. */
int cpu_place_k(int32_t n, int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free,
                const int32_t* avail_min, const uint32_t* part_mask, int32_t p,
                const int32_t* max_time, const int32_t* max_cpus, const int32_t* max_mem, int32_t j,
                const int32_t* cpu, const int32_t* mem, const int32_t* gpu, const int32_t* wall,
                const uint16_t* part, const uint16_t* nodes_k, int32_t kmax, int32_t* out,
                int64_t* stats, int32_t threads) {
    if (n < 0 || j < 0 || p < 0 || p > 32 || kmax < 1 || kmax > 64) return -1;
    for (int32_t q = 0; q < j; q++) {
        const int kq = nodes_k ? (nodes_k[q] ? nodes_k[q] : 1) : 1;
        if (kq > kmax || cpu[q] < 0 || mem[q] < 0 || gpu[q] < 0 || wall[q] < 0) return -1;
    }
    int32_t* code = malloc(sizeof(int32_t) * (j > 0 ? j : 1)); /* per job: -1 or -2 */
    comps_t C;
    memset(&C, 0, sizeof C);
    if (!code || build_comps(&C, n, part_mask, p, max_time, max_cpus, max_mem, j, cpu, mem, wall, part, code)) {
        free(code);
        free_comps(&C);
        return -1;
    }
    int64_t rejected = 0;
    for (int32_t q = 0; q < j; q++) {
        const int kq = nodes_k ? (nodes_k[q] ? nodes_k[q] : 1) : 1;
        int32_t* o = out + (int64_t)q * kmax;
        for (int i = 0; i < kmax; i++) o[i] = -1;
        if (code[q] == -2) {
            for (int i = 0; i < kq; i++) o[i] = -2;
            rejected++;
        }
    }
    free(code);
    k_job_t K;
    memset(&K, 0, sizeof K);
    plain_job_t* T = &K.base;
    T->C = &C;
    T->cpu_free = cpu_free;
    T->mem_free = mem_free;
    T->gpu_free = gpu_free;
    T->avail = avail_min;
    T->mask = part_mask;
    T->cpu = cpu;
    T->mem = mem;
    T->gpu = gpu;
    T->wall = wall;
    T->part = part;
    T->out = out;
    T->order = lpt_order(&C, comp_work);
    K.nodes_k = nodes_k;
    K.kmax = kmax;
    pthread_mutex_init(&T->mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    int started = 0;
    for (int i = 1; i < threads; i++)
        if (pthread_create(&th[started], NULL, k_worker, &K) == 0) started++;
    k_worker(&K);
    for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
    if (stats) {
        stats[0] = T->placed;
        stats[1] = j - T->placed - rejected;
        stats[2] = rejected;
        stats[3] = T->evals;
    }
    pthread_mutex_destroy(&T->mu);
    free((void*)T->order);
    free_comps(&C);
    return 0;
}

/* ------------------------------------------------------------------ backfill (SPEC §2b) */
typedef struct {
    const comps_t* C;
    int32_t H, slot_min;
    int32_t* tl; /* dense [n][H][3] */
    const uint32_t* mask;
    const int32_t *cpu, *mem, *gpu, *wall;
    const uint16_t* part;
    int32_t *out, *outs;
    const int32_t* order;
    volatile int32_t next;
    int64_t placed, evals;
    pthread_mutex_t mu;
} tl_job_t;

static void* tl_worker(void* arg) {
    tl_job_t* T = arg;
    const comps_t* C = T->C;
    const int32_t H = T->H;
    int64_t placed = 0, evals = 0;
    for (;;) {
        const int32_t i = __atomic_fetch_add(&T->next, 1, __ATOMIC_RELAXED);
        if (i >= C->nc) break;
        const int k = T->order[i];
        const int32_t* id = C->nodes + C->nb[k];
        const int32_t len = C->nb[k + 1] - C->nb[k];
        for (int32_t t = C->jb[k]; t < C->jb[k + 1]; t++) {
            const int32_t q = C->jobs[t];
            const int32_t d = ref_slots(T->wall[q], T->slot_min);
            uint64_t best = UINT64_MAX;
            for (int32_t a = 0; a < len; a++) {
                const int32_t x = id[a];
                int32_t s;
                const uint64_t key = ref_key_tl(x, H, T->tl + (int64_t)x * H * 3, T->mask[x], T->cpu[q],
                                                T->mem[q], T->gpu[q], d, T->part[q], &s);
                if (key < best) best = key;
            }
            evals += len;
            if (best == UINT64_MAX) continue;
            const int32_t x = (int32_t)(best & 0x3fffffu), s = (int32_t)(best >> 54);
            for (int32_t u = s; u < s + d; u++) {
                int32_t* v = T->tl + ((int64_t)x * H + u) * 3;
                v[0] -= T->cpu[q];
                v[1] -= T->mem[q];
                v[2] -= T->gpu[q];
            }
            T->out[q] = x;
            T->outs[q] = s;
            placed++;
        }
    }
    pthread_mutex_lock(&T->mu);
    T->placed += placed;
    T->evals += evals;
    pthread_mutex_unlock(&T->mu);
    return NULL;
}

int cpu_place_tl(int32_t n, int32_t H, int32_t slot_min, int32_t* tl, const uint32_t* part_mask,
                 int32_t p, const int32_t* max_time, const int32_t* max_cpus, const int32_t* max_mem,
                 int32_t j, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
                 const int32_t* wall, const uint16_t* part, int32_t* out_node, int32_t* out_start,
                 int64_t* stats, int32_t threads) {
    if (n < 0 || n > (1 << 22) || j < 0 || p < 0 || p > 32 || H < 1 || H > 1024 || slot_min < 1)
        return -1;
    for (int32_t q = 0; q < j; q++)
        if (cpu[q] < 0 || mem[q] < 0 || gpu[q] < 0 || wall[q] < 0) return -1;
    comps_t C;
    memset(&C, 0, sizeof C);
    if (build_comps(&C, n, part_mask, p, max_time, max_cpus, max_mem, j, cpu, mem, wall, part,
                    out_node)) {
        free_comps(&C);
        return -1;
    }
    for (int32_t q = 0; q < j; q++) out_start[q] = -1;
    tl_job_t T;
    memset(&T, 0, sizeof T);
    T.C = &C;
    T.H = H;
    T.slot_min = slot_min;
    T.tl = tl;
    T.mask = part_mask;
    T.cpu = cpu;
    T.mem = mem;
    T.gpu = gpu;
    T.wall = wall;
    T.part = part;
    T.out = out_node;
    T.outs = out_start;
    T.order = lpt_order(&C, comp_work);
    pthread_mutex_init(&T.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    int started = 0;
    for (int i = 1; i < threads; i++)
        if (pthread_create(&th[started], NULL, tl_worker, &T) == 0) started++;
    tl_worker(&T);
    for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
    int64_t rejected = 0;
    for (int32_t q = 0; q < j; q++) rejected += out_node[q] == -2;
    if (stats) {
        stats[0] = T.placed;
        stats[1] = j - T.placed - rejected;
        stats[2] = rejected;
        stats[3] = T.evals;
    }
    pthread_mutex_destroy(&T.mu);
    free((void*)T.order);
    free_comps(&C);
    return 0;
}
