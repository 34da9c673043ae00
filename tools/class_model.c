/* tools/class_model.c — CPU model of a commit chain on persistent demand-class candidate lists
 * (diagnostic only, never linked into the product).
 *
 * One component, SPEC §2 keys (oracle/fitref.c ref_key restated, as tools/spec_model.c).  A job's
 * CLASS is its (partition, cpu, mem, gpu) — what decides its key on every node except the walltime
 * test.  Per class c the chain keeps a list of the K smallest keys over the nodes its shape fits
 * (walltime ignored) and a bound L_c, with the invariant
 *
 *     list_c = { nodes n : key_c(n) < L_c }   (sorted, |list_c| <= K)
 *
 * A commit changes ONE node row; every key of that node can only fall (or turn infeasible), so per
 * class: a listed node is moved up or dropped, an unlisted node whose new key is < L_c is inserted
 * (evicting the last entry and lowering L_c to its key when the list is full).  A job of class c
 * with walltime w takes the first k listed entries with avail >= w — exact while they exist, since
 * every unlisted node's key is >= L_c.  When fewer than k qualify and L_c is finite, the list is
 * EXHAUSTED: the job is resolved by a scan of the component and the list refilled by another.
 *
 * The model places the whole queue that way, checks every placement against a plain sequential
 * best fit (the oracle's rule) when `check` is set, and counts what a one-wave chain would execute:
 * node-vs-class evaluations per commit, classes whose list changed, entries inspected by queries,
 * exhaustions and refill scans.
 *
 *   gcc -O2 -shared -fPIC -o tools/libclass_model.so tools/class_model.c */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t key_of(int32_t cf, int32_t mf, int32_t gf, uint32_t mk, int32_t pos, int32_t c,
                              int32_t m, int32_t g, uint32_t pbit) {
    const int32_t dc = cf - c, dm = mf - m, dg = gf - g;
    if ((dc | dm | dg) < 0 || !(mk & pbit)) return UINT64_MAX;
    uint32_t gr = (uint32_t)dg, cr = (uint32_t)dc, mr = (uint32_t)dm >> 10;
    gr = gr > 255u ? 255u : gr;
    cr = cr > 4095u ? 4095u : cr;
    mr = mr > 4095u ? 4095u : mr;
    return ((uint64_t)((gr << 24) | (cr << 12) | mr) << 32) | (uint32_t)pos;
}

typedef struct {
    int64_t jobs, placed, unplaced, dead_fast;  /* dead_fast: unplaced with an empty list, L = inf */
    int64_t commits;                            /* node-row updates (sum of k over placed jobs) */
    int64_t evals_commit;                       /* node-vs-class evaluations at commits */
    int64_t affected;                           /* class lists changed by commits */
    int64_t affected_max;                       /* most lists changed by one commit */
    int64_t inserts, moves, drops, evicts;
    int64_t query_entries;                      /* list entries inspected by queries */
    int64_t exhaust;                            /* queries the list could not answer */
    int64_t refills;                            /* class-list rebuilds (initial builds excluded) */
    int64_t mismatches;                         /* placements that differ from plain best fit */
    int64_t first_mismatch;
    int64_t lim_pick;                           /* picks on a node with a finite avail */
    int64_t skipped_wall;                       /* listed entries skipped by the walltime test */
} cm_stats;

/* rebuild class c's list: the K smallest keys (and L = the (K+1)-th, or inf) */
static void build_list(int32_t n, const int32_t* cf, const int32_t* mf, const int32_t* gf,
                       const uint32_t* mk, int32_t c, int32_t m, int32_t g, uint32_t pbit, int32_t K,
                       uint64_t* lst, int32_t* len, uint64_t* L) {
    int32_t cnt = 0;
    uint64_t tmp[65];
    for (int32_t x = 0; x < n; ++x) {
        const uint64_t k = key_of(cf[x], mf[x], gf[x], mk[x], x, c, m, g, pbit);
        if (k == UINT64_MAX) continue;
        if (cnt == K + 1 && k >= tmp[K]) continue;
        int32_t i = cnt < K + 1 ? cnt++ : K;
        while (i > 0 && tmp[i - 1] > k) {
            tmp[i] = tmp[i - 1];
            --i;
        }
        tmp[i] = k;
    }
    *len = cnt < K ? cnt : K;
    memcpy(lst, tmp, sizeof(uint64_t) * (size_t)*len);
    *L = cnt > K ? tmp[K] : UINT64_MAX;
}

/* nodes: n rows of one component (positions 0..n-1, modified in place); jobs in priority order with
 * their class id cls[] (0..C-1) and class demands ccpu/cmem/cgpu/cpart; kk = nodes per job.
 * out[j*8+i]: chosen positions (-1).  K <= 64.  Returns 0. */
int class_chain(int32_t n, int32_t* cf, int32_t* mf, int32_t* gf, const int32_t* av, const uint32_t* mk,
                int32_t j, const int32_t* cls, const int32_t* wall, const uint16_t* kk, int32_t C,
                const int32_t* ccpu, const int32_t* cmem, const int32_t* cgpu, const uint16_t* cpart,
                int32_t K, int32_t check, int32_t* out, cm_stats* S) {
    memset(S, 0, sizeof *S);
    S->first_mismatch = -1;
    uint64_t* lst = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)C * (size_t)K);
    int32_t* len = (int32_t*)calloc((size_t)C, sizeof(int32_t));
    uint64_t* L = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)C);
    for (int32_t c = 0; c < C; ++c)
        build_list(n, cf, mf, gf, mk, ccpu[c], cmem[c], cgpu[c], 1u << cpart[c], K, lst + (size_t)c * K,
                   len + c, L + c);
    for (int32_t t = 0; t < j; ++t) {
        const int32_t c = cls[t];
        const int32_t k = kk ? (kk[t] > 0 ? kk[t] : 1) : 1;
        const int32_t dc = ccpu[c], dm = cmem[c], dg = cgpu[c];
        const uint32_t pb = 1u << cpart[c];
        int32_t pick[8], np = 0;
        uint64_t* lc = lst + (size_t)c * K;
        for (int32_t i = 0; i < len[c] && np < k; ++i) {
            ++S->query_entries;
            const int32_t x = (int32_t)(uint32_t)lc[i];
            if (av[x] >= wall[t]) pick[np++] = x;
            else ++S->skipped_wall;
        }
        if (np < k && L[c] != UINT64_MAX) {
            /* exhausted: the list cannot prove the answer; resolve by a scan, refill the list */
            ++S->exhaust;
            np = 0;
            uint64_t best[8];
            for (int32_t x = 0; x < n; ++x) {
                if (av[x] < wall[t]) continue;
                const uint64_t key = key_of(cf[x], mf[x], gf[x], mk[x], x, dc, dm, dg, pb);
                if (key == UINT64_MAX) continue;
                if (np == k && key >= best[k - 1]) continue;
                int32_t i = np < k ? np++ : k - 1;
                while (i > 0 && best[i - 1] > key) {
                    best[i] = best[i - 1];
                    --i;
                }
                best[i] = key;
            }
            for (int32_t i = 0; i < np; ++i) pick[i] = (int32_t)(uint32_t)best[i];
            ++S->refills;
            build_list(n, cf, mf, gf, mk, dc, dm, dg, pb, K, lc, len + c, L + c);
        }
        ++S->jobs;
        if (np < k) {
            if (len[c] == 0 && L[c] == UINT64_MAX) ++S->dead_fast;
            ++S->unplaced;
            np = 0;
        } else {
            ++S->placed;
        }
        if (check) {
            /* the plain sequential answer: the k smallest feasible keys now */
            uint64_t best[8];
            int32_t nb = 0;
            for (int32_t x = 0; x < n; ++x) {
                if (av[x] < wall[t]) continue;
                const uint64_t key = key_of(cf[x], mf[x], gf[x], mk[x], x, dc, dm, dg, pb);
                if (key == UINT64_MAX) continue;
                if (nb == k && key >= best[k - 1]) continue;
                int32_t i = nb < k ? nb++ : k - 1;
                while (i > 0 && best[i - 1] > key) {
                    best[i] = best[i - 1];
                    --i;
                }
                best[i] = key;
            }
            int ok = (nb < k) ? (np == 0) : (np == k);
            for (int32_t i = 0; ok && i < np; ++i) ok = (int32_t)(uint32_t)best[i] == pick[i];
            if (!ok) {
                if (S->first_mismatch < 0) S->first_mismatch = t;
                ++S->mismatches;
            }
        }
        for (int32_t i = 0; i < 8; ++i) out[(int64_t)t * 8 + i] = i < np ? pick[i] : -1;
        /* commit: every picked node loses the demand; every class list re-evaluates it */
        for (int32_t i = 0; i < np; ++i) {
            const int32_t x = pick[i];
            if (av[x] != INT32_MAX) ++S->lim_pick;
            const int32_t ocf = cf[x], omf = mf[x], ogf = gf[x];
            cf[x] -= dc;
            mf[x] -= dm;
            gf[x] -= dg;
            ++S->commits;
            int64_t aff = 0;
            for (int32_t q = 0; q < C; ++q) {
                ++S->evals_commit;
                const uint32_t qb = 1u << cpart[q];
                const uint64_t ko = key_of(ocf, omf, ogf, mk[x], x, ccpu[q], cmem[q], cgpu[q], qb);
                const uint64_t kn = key_of(cf[x], mf[x], gf[x], mk[x], x, ccpu[q], cmem[q], cgpu[q], qb);
                uint64_t* lq = lst + (size_t)q * K;
                if (ko < L[q]) {  /* listed: remove ko, re-insert kn if feasible (kn < ko < L) */
                    int32_t p = 0;
                    while (p < len[q] && lq[p] != ko) ++p;
                    if (p == len[q]) abort(); /* invariant broken */
                    memmove(lq + p, lq + p + 1, sizeof(uint64_t) * (size_t)(len[q] - p - 1));
                    --len[q];
                    if (kn == UINT64_MAX) {
                        ++S->drops;
                    } else {
                        int32_t i2 = len[q]++;
                        while (i2 > 0 && lq[i2 - 1] > kn) {
                            lq[i2] = lq[i2 - 1];
                            --i2;
                        }
                        lq[i2] = kn;
                        ++S->moves;
                    }
                    ++aff;
                } else if (kn < L[q]) {  /* newly below the bound: insert, evict past K */
                    int32_t i2 = len[q];
                    if (len[q] == K && kn > lq[K - 1]) {  /* full and last: the bound drops to it */
                        L[q] = kn;
                        ++S->evicts;
                        ++aff;
                        continue;
                    }
                    if (len[q] == K) {
                        L[q] = lq[K - 1];
                        i2 = K - 1;
                        ++S->evicts;
                    } else {
                        ++len[q];
                    }
                    while (i2 > 0 && lq[i2 - 1] > kn) {
                        lq[i2] = lq[i2 - 1];
                        --i2;
                    }
                    lq[i2] = kn;
                    ++S->inserts;
                    ++aff;
                }
            }
            S->affected += aff;
            if (aff > S->affected_max) S->affected_max = aff;
        }
    }
    free(lst);
    free(len);
    free(L);
    return 0;
}

/* The LAZY variant: per class an unsorted SET of up to K node positions and a bound L_c with the
 * weaker invariant  "every node NOT in set_c has key_c >= L_c".  Listed keys are evaluated at query
 * time from the current rows, so a commit touches a class only when the committed node x is
 * unlisted and its new key is below L_c: x is added (room left) or L_c drops to x's key (set full —
 * x stays out, still >= the new bound).  A query takes the k smallest current keys of the set among
 * the nodes with avail >= wall; they are the answer when the k-th is < L_c (every unlisted node is
 * >= L_c) or L_c is infinite; otherwise the set is EXHAUSTED and refilled by a scan (the K smallest
 * keys now, L_c = the (K+1)-th).  Infeasible entries are dropped at queries (keys never recover).
 * evict_max: a full set evicts its largest current key when x's is smaller (counts evals). */
int class_chain_lazy(int32_t n, int32_t* cf, int32_t* mf, int32_t* gf, const int32_t* av, const uint32_t* mk,
                     int32_t j, const int32_t* cls, const int32_t* wall, const uint16_t* kk, int32_t C,
                     const int32_t* ccpu, const int32_t* cmem, const int32_t* cgpu, const uint16_t* cpart,
                     int32_t K, int32_t check, int32_t evict_max, int32_t* out, cm_stats* S) {
    memset(S, 0, sizeof *S);
    S->first_mismatch = -1;
    uint64_t* lst = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)C * (size_t)K);
    int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * (size_t)C * (size_t)K);
    int32_t* len = (int32_t*)calloc((size_t)C, sizeof(int32_t));
    uint64_t* L = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)C);
    uint8_t* mem = (uint8_t*)calloc((size_t)C * (size_t)n, 1);  /* membership */
    for (int32_t c = 0; c < C; ++c) {
        build_list(n, cf, mf, gf, mk, ccpu[c], cmem[c], cgpu[c], 1u << cpart[c], K, lst + (size_t)c * K,
                   len + c, L + c);
        for (int32_t i = 0; i < len[c]; ++i) {
            pos[(size_t)c * K + i] = (int32_t)(uint32_t)lst[(size_t)c * K + i];
            mem[(size_t)c * n + pos[(size_t)c * K + i]] = 1;
        }
    }
    for (int32_t t = 0; t < j; ++t) {
        const int32_t c = cls[t];
        const int32_t k = kk ? (kk[t] > 0 ? kk[t] : 1) : 1;
        const int32_t dc = ccpu[c], dm = cmem[c], dg = cgpu[c];
        const uint32_t pb = 1u << cpart[c];
        int32_t* pc = pos + (size_t)c * K;
        uint64_t best[8];
        int32_t nb = 0;
        for (int32_t i = 0; i < len[c];) {
            ++S->query_entries;
            const int32_t x = pc[i];
            const uint64_t key = key_of(cf[x], mf[x], gf[x], mk[x], x, dc, dm, dg, pb);
            if (key == UINT64_MAX) {  /* infeasible for good: drop */
                mem[(size_t)c * n + x] = 0;
                pc[i] = pc[--len[c]];
                ++S->drops;
                continue;
            }
            ++i;
            if (av[x] < wall[t]) {
                ++S->skipped_wall;
                continue;
            }
            if (nb == k && key >= best[k - 1]) continue;
            int32_t q = nb < k ? nb++ : k - 1;
            while (q > 0 && best[q - 1] > key) {
                best[q] = best[q - 1];
                --q;
            }
            best[q] = key;
        }
        int32_t np = 0, pick[8];
        const int exact = L[c] == UINT64_MAX || (nb == k && best[k - 1] < L[c]);
        if (!exact) {
            ++S->exhaust;
            nb = 0;
            for (int32_t x = 0; x < n; ++x) {
                if (av[x] < wall[t]) continue;
                const uint64_t key = key_of(cf[x], mf[x], gf[x], mk[x], x, dc, dm, dg, pb);
                if (key == UINT64_MAX) continue;
                if (nb == k && key >= best[k - 1]) continue;
                int32_t q = nb < k ? nb++ : k - 1;
                while (q > 0 && best[q - 1] > key) {
                    best[q] = best[q - 1];
                    --q;
                }
                best[q] = key;
            }
            ++S->refills;
            for (int32_t i = 0; i < len[c]; ++i) mem[(size_t)c * n + pc[i]] = 0;
            uint64_t* lc = lst + (size_t)c * K;
            build_list(n, cf, mf, gf, mk, dc, dm, dg, pb, K, lc, len + c, L + c);
            for (int32_t i = 0; i < len[c]; ++i) {
                pc[i] = (int32_t)(uint32_t)lc[i];
                mem[(size_t)c * n + pc[i]] = 1;
            }
        }
        ++S->jobs;
        if (nb == k) {
            ++S->placed;
            np = k;
            for (int32_t i = 0; i < k; ++i) pick[i] = (int32_t)(uint32_t)best[i];
        } else {
            ++S->unplaced;
            if (len[c] == 0 && L[c] == UINT64_MAX) ++S->dead_fast;
        }
        if (check) {
            uint64_t b2[8];
            int32_t n2 = 0;
            for (int32_t x = 0; x < n; ++x) {
                if (av[x] < wall[t]) continue;
                const uint64_t key = key_of(cf[x], mf[x], gf[x], mk[x], x, dc, dm, dg, pb);
                if (key == UINT64_MAX) continue;
                if (n2 == k && key >= b2[k - 1]) continue;
                int32_t q = n2 < k ? n2++ : k - 1;
                while (q > 0 && b2[q - 1] > key) {
                    b2[q] = b2[q - 1];
                    --q;
                }
                b2[q] = key;
            }
            int ok = (n2 < k) ? (np == 0) : (np == k);
            for (int32_t i = 0; ok && i < np; ++i) ok = (int32_t)(uint32_t)b2[i] == pick[i];
            if (!ok) {
                if (S->first_mismatch < 0) S->first_mismatch = t;
                ++S->mismatches;
            }
        }
        for (int32_t i = 0; i < 8; ++i) out[(int64_t)t * 8 + i] = i < np ? pick[i] : -1;
        for (int32_t i = 0; i < np; ++i) {
            const int32_t x = pick[i];
            if (av[x] != INT32_MAX) ++S->lim_pick;
            cf[x] -= dc;
            mf[x] -= dm;
            gf[x] -= dg;
            ++S->commits;
            int64_t aff = 0;
            for (int32_t q = 0; q < C; ++q) {
                ++S->evals_commit;
                if (mem[(size_t)q * n + x]) continue;
                const uint64_t kn = key_of(cf[x], mf[x], gf[x], mk[x], x, ccpu[q], cmem[q], cgpu[q], 1u << cpart[q]);
                if (kn >= L[q]) continue;
                int32_t* pq = pos + (size_t)q * K;
                ++aff;
                if (len[q] < K) {
                    pq[len[q]++] = x;
                    mem[(size_t)q * n + x] = 1;
                    ++S->inserts;
                } else if (evict_max) {
                    /* evict the largest current key of the set if it is above kn */
                    int32_t wi = -1;
                    uint64_t wk = 0;
                    for (int32_t i = 0; i < K; ++i) {
                        const int32_t y = pq[i];
                        const uint64_t ky = key_of(cf[y], mf[y], gf[y], mk[y], y, ccpu[q], cmem[q], cgpu[q], 1u << cpart[q]);
                        if (wi < 0 || ky > wk) wi = i, wk = ky;
                    }
                    ++S->moves;  /* counts full-set evaluations */
                    if (wk > kn) {
                        mem[(size_t)q * n + pq[wi]] = 0;
                        pq[wi] = x;
                        mem[(size_t)q * n + x] = 1;
                        if (wk < L[q]) L[q] = wk;
                        ++S->evicts;
                    } else {
                        L[q] = kn;
                    }
                } else {
                    L[q] = kn;
                    ++S->evicts;
                }
            }
            S->affected += aff;
            if (aff > S->affected_max) S->affected_max = aff;
        }
    }
    free(lst);
    free(pos);
    free(len);
    free(L);
    free(mem);
    return 0;
}
