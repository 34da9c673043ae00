/* oracle/round_model.c — CPU model of the GPU round algorithm (TEST INFRASTRUCTURE ONLY).
 *
 * Makes exactly the decisions the HIP kernels make (component split, per-slice top-K scan,
 * candidate merge with bound B, dirty-set commit with stop rules) so that
 *  (1) tests can show on CPU that the speculative-prefix algorithm reproduces ref_place()
 *      bit-exactly for any parameters, and
 *  (2) the GPU's round / commit / stop counters can be checked against this model.
 * It is not a product path and is never linked into libfitgpu.so.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KEY_INF UINT64_MAX

typedef struct {
    int32_t slice;     /* nodes per scan slice */
    int32_t ks;        /* candidates kept per (job, slice) */
    int32_t km;        /* candidates kept per job after merge (<= 64) */
    int32_t ucap;      /* dirty-set capacity per component per round */
    int32_t wmin, wmax;/* window bounds (jobs per component per round) */
    int32_t shards;    /* node shards per component (multi-GPU node sharding), >= 1 */
} model_params;

/* stats: [0] rounds [1] scan evals [2] dirty evals [3] stops_rescan [4] stops_ucap
 *        [5] commits [6] max window used [7] placed */
static uint64_t node_key(int32_t pos, int32_t cf, int32_t mf, int32_t gf, int32_t av, uint32_t mask,
                         int32_t c, int32_t m, int32_t g, int32_t w, int32_t p) {
    if (!((mask >> p) & 1u)) return KEY_INF;
    if (cf < c || mf < m || gf < g || av < w) return KEY_INF;
    uint32_t gr = (uint32_t)(gf - g), cr = (uint32_t)(cf - c), mr = (uint32_t)(mf - m) >> 10;
    if (gr > 255u) gr = 255u;
    if (cr > 4095u) cr = 4095u;
    if (mr > 4095u) mr = 4095u;
    return ((uint64_t)((gr << 24) | (cr << 12) | mr) << 32) | (uint32_t)pos;
}

static void insert_sorted(uint64_t* a, int k, uint64_t key) {
    if (key >= a[k - 1]) return;
    int i = k - 1;
    while (i > 0 && a[i - 1] > key) {
        a[i] = a[i - 1];
        i--;
    }
    a[i] = key;
}

static int find_root(int* par, int x) {
    while (par[x] != x) x = par[x] = par[par[x]];
    return x;
}

int model_place(int32_t n, int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free,
                const int32_t* avail_min, const uint32_t* part_mask, int32_t p,
                const int32_t* max_time, const int32_t* max_cpus, const int32_t* max_mem,
                int32_t j, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
                const int32_t* wall, const uint16_t* part, const model_params* prm,
                int32_t* out, int64_t* stats) {
    memset(stats, 0, 8 * sizeof(int64_t));
    if (prm->km > 64 || prm->ks < 1 || prm->km < 1 || prm->ucap < 1) return -1;
    /* components: union partitions that share a node */
    int par[33];
    for (int i = 0; i < 33; i++) par[i] = i;
    for (int32_t x = 0; x < n; x++) {
        uint32_t m = part_mask[x];
        if (!m) continue;
        int lo = __builtin_ctz(m);
        for (uint32_t r = m & (m - 1); r; r &= r - 1) {
            int a = find_root(par, lo), b = find_root(par, __builtin_ctz(r));
            if (a != b) par[a < b ? b : a] = a < b ? a : b;
        }
    }
    int comp_of_part[32], ncomp = 0, root_comp[33];
    for (int i = 0; i < 33; i++) root_comp[i] = -1;
    int used[32] = {0};
    for (int32_t x = 0; x < n; x++)
        for (uint32_t r = part_mask[x]; r; r &= r - 1) used[__builtin_ctz(r)] = 1;
    for (int q = 0; q < 32; q++) {
        comp_of_part[q] = -1;
        if (!used[q]) continue;
        int rt = find_root(par, q);
        if (root_comp[rt] < 0) root_comp[rt] = ncomp++;
        comp_of_part[q] = root_comp[rt];
    }
    /* stable node order by component; pos -> orig */
    int32_t* nb = calloc((size_t)ncomp + 1, sizeof(int32_t));
    for (int32_t x = 0; x < n; x++)
        if (part_mask[x]) nb[comp_of_part[__builtin_ctz(part_mask[x])] + 1]++;
    for (int c = 0; c < ncomp; c++) nb[c + 1] += nb[c];
    int32_t nn = nb[ncomp];
    int32_t *orig = malloc(sizeof(int32_t) * (nn + 1)), *fill = malloc(sizeof(int32_t) * (ncomp + 1));
    int32_t *cf = malloc(sizeof(int32_t) * (nn + 1)), *mf = malloc(sizeof(int32_t) * (nn + 1));
    int32_t *gf = malloc(sizeof(int32_t) * (nn + 1)), *av = malloc(sizeof(int32_t) * (nn + 1));
    uint32_t* mk = malloc(sizeof(uint32_t) * (nn + 1));
    memcpy(fill, nb, sizeof(int32_t) * (ncomp + 1));
    for (int32_t x = 0; x < n; x++) {
        if (!part_mask[x]) continue;
        int32_t q = fill[comp_of_part[__builtin_ctz(part_mask[x])]]++;
        orig[q] = x;
        cf[q] = cpu_free[x];
        mf[q] = mem_free[x];
        gf[q] = gpu_free[x];
        av[q] = avail_min[x];
        mk[q] = part_mask[x];
    }
    /* per-component job lists in priority order; prefilter */
    int32_t* jb = calloc((size_t)ncomp + 1, sizeof(int32_t));
    int32_t* jc = malloc(sizeof(int32_t) * (j + 1));
    for (int32_t q = 0; q < j; q++) {
        int pq = part[q];
        out[q] = -1;
        jc[q] = -1;
        if (pq >= p || (max_time[pq] >= 0 && wall[q] > max_time[pq]) ||
            (max_cpus[pq] >= 0 && cpu[q] > max_cpus[pq]) || (max_mem[pq] >= 0 && mem[q] > max_mem[pq])) {
            out[q] = -2;
            continue;
        }
        if (pq >= 32 || comp_of_part[pq] < 0) continue; /* partition without nodes: unplaced */
        jc[q] = comp_of_part[pq];
        jb[jc[q] + 1]++;
    }
    for (int c = 0; c < ncomp; c++) jb[c + 1] += jb[c];
    int32_t* jl = malloc(sizeof(int32_t) * (jb[ncomp] + 1));
    int32_t* jf = malloc(sizeof(int32_t) * (ncomp + 1));
    memcpy(jf, jb, sizeof(int32_t) * (ncomp + 1));
    for (int32_t q = 0; q < j; q++)
        if (jc[q] >= 0) jl[jf[jc[q]]++] = q;

    int32_t* cursor = malloc(sizeof(int32_t) * (ncomp + 1));
    int32_t* win = malloc(sizeof(int32_t) * (ncomp + 1));
    for (int c = 0; c < ncomp; c++) {
        cursor[c] = jb[c];
        win[c] = prm->wmin;
    }
    int32_t wcap = prm->wmax;
    uint64_t* cand = malloc(sizeof(uint64_t) * (size_t)wcap * prm->km);
    uint64_t* bound = malloc(sizeof(uint64_t) * (size_t)wcap);
    int32_t smax = 1;
    for (int c = 0; c < ncomp; c++) {
        const int32_t nsh = prm->shards > 1 ? prm->shards : 1;
        const int32_t per = (nb[c + 1] - nb[c] + nsh - 1) / nsh;
        int32_t s = nsh * ((per + prm->slice - 1) / prm->slice);
        if (s > smax) smax = s;
    }
    uint64_t* sl = malloc(sizeof(uint64_t) * (size_t)prm->ks);
    uint64_t* mg = malloc(sizeof(uint64_t) * ((size_t)prm->ks * smax + prm->km));
    int32_t* upos = malloc(sizeof(int32_t) * prm->ucap);
    int32_t *ucf = malloc(sizeof(int32_t) * prm->ucap), *umf = malloc(sizeof(int32_t) * prm->ucap);
    int32_t* ugf = malloc(sizeof(int32_t) * prm->ucap);
    int32_t* slot_of = malloc(sizeof(int32_t) * (nn + 1));
    for (int32_t x = 0; x < nn; x++) slot_of[x] = -1;

    for (;;) {
        int any = 0;
        for (int c = 0; c < ncomp; c++) any |= cursor[c] < jb[c + 1];
        if (!any) break;
        stats[0]++;
        for (int c = 0; c < ncomp; c++) {
            if (cursor[c] >= jb[c + 1]) continue;
            int32_t w = win[c];
            if (w > jb[c + 1] - cursor[c]) w = jb[c + 1] - cursor[c];
            if (w > stats[6]) stats[6] = w;
            int32_t n0 = nb[c], n1 = nb[c + 1];
            /* scan + merge */
            for (int32_t t = 0; t < w; t++) {
                int32_t q = jl[cursor[c] + t];
                uint64_t B = KEY_INF;
                int nm = 0;
                const int32_t nsh = prm->shards > 1 ? prm->shards : 1;
                const int32_t per = (n1 - n0 + nsh - 1) / nsh;
                for (int32_t sh = 0; sh < nsh; ++sh)
                for (int32_t s0 = n0 + sh * per; s0 < n0 + (sh + 1) * per && s0 < n1; s0 += prm->slice) {
                    int32_t se = n0 + (sh + 1) * per < n1 ? n0 + (sh + 1) * per : n1;
                    int32_t s1 = s0 + prm->slice < se ? s0 + prm->slice : se;
                    for (int i = 0; i < prm->ks; i++) sl[i] = KEY_INF;
                    int64_t feas = 0;
                    for (int32_t x = s0; x < s1; x++) {
                        uint64_t key = node_key(x, cf[x], mf[x], gf[x], av[x], mk[x], cpu[q], mem[q],
                                                gpu[q], wall[q], part[q]);
                        if (key != KEY_INF) {
                            feas++;
                            insert_sorted(sl, prm->ks, key);
                        }
                    }
                    stats[1] += s1 - s0;
                    if (feas > prm->ks && sl[prm->ks - 1] < B) B = sl[prm->ks - 1];
                    for (int i = 0; i < prm->ks; i++)
                        if (sl[i] != KEY_INF) mg[nm++] = sl[i];
                }
                /* keep entries <= B, sorted, at most km */
                uint64_t* cl = cand + (size_t)t * prm->km;
                for (int i = 0; i < prm->km; i++) cl[i] = KEY_INF;
                for (int i = 0; i < nm; i++)
                    if (mg[i] <= B) insert_sorted(cl, prm->km, mg[i]);
                int cnt = 0;
                for (int i = 0; i < prm->km; i++) cnt += cl[i] != KEY_INF;
                if (cnt == prm->km) {
                    int over = 0;
                    for (int i = 0; i < nm; i++) over += mg[i] <= B;
                    if (over > prm->km) B = cl[prm->km - 1];
                }
                bound[t] = B;
            }
            /* commit */
            int32_t nu = 0, done = 0;
            int stop = 0;
            for (int32_t t = 0; t < w; t++) {
                int32_t q = jl[cursor[c] + t];
                uint64_t* cl = cand + (size_t)t * prm->km;
                uint64_t e = KEY_INF;
                for (int i = 0; i < prm->km && cl[i] != KEY_INF; i++)
                    if (slot_of[(uint32_t)cl[i]] < 0) {
                        e = cl[i];
                        break;
                    }
                uint64_t d = KEY_INF;
                for (int32_t u = 0; u < nu; u++) {
                    int32_t x = upos[u];
                    uint64_t key = node_key(x, ucf[u], umf[u], ugf[u], av[x], mk[x], cpu[q], mem[q],
                                            gpu[q], wall[q], part[q]);
                    if (key < d) d = key;
                }
                stats[2] += nu;
                uint64_t best;
                if (e != KEY_INF) best = e < d ? e : d;
                else if (bound[t] == KEY_INF) best = d;
                else if (d <= bound[t]) best = d;
                else {
                    stop = 1;
                    break;
                }
                if (best == KEY_INF) {
                    out[q] = -1;
                    done++;
                    continue;
                }
                int32_t x = (int32_t)(uint32_t)best;
                int32_t s = slot_of[x];
                if (s < 0) {
                    if (nu == prm->ucap) {
                        stop = 2;
                        break;
                    }
                    s = nu++;
                    slot_of[x] = s;
                    upos[s] = x;
                    ucf[s] = cf[x];
                    umf[s] = mf[x];
                    ugf[s] = gf[x];
                }
                ucf[s] -= cpu[q];
                umf[s] -= mem[q];
                ugf[s] -= gpu[q];
                out[q] = orig[x];
                stats[7]++;
                done++;
            }
            if (stop == 1) stats[3]++;
            if (stop == 2) stats[4]++;
            for (int32_t u = 0; u < nu; u++) { /* write back dirty rows */
                int32_t x = upos[u];
                cf[x] = ucf[u];
                mf[x] = umf[u];
                gf[x] = ugf[u];
                slot_of[x] = -1;
            }
            stats[5] += done;
            cursor[c] += done;
            /* window policy: double when the whole window committed, else 2x what committed */
            int32_t nw = stop ? 2 * done : 2 * w;
            if (nw < prm->wmin) nw = prm->wmin;
            if (nw > prm->wmax) nw = prm->wmax;
            win[c] = nw;
        }
    }
    for (int32_t x = 0; x < nn; x++) {
        cpu_free[orig[x]] = cf[x];
        mem_free[orig[x]] = mf[x];
        gpu_free[orig[x]] = gf[x];
    }
    free(nb); free(orig); free(fill); free(cf); free(mf); free(gf); free(av); free(mk);
    free(jb); free(jc); free(jl); free(jf); free(cursor); free(win); free(cand); free(bound);
    free(sl); free(mg); free(upos); free(ucf); free(umf); free(ugf); free(slot_of);
    return 0;
}
