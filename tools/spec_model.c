/* tools/spec_model.c — CPU model of a multi-job decider step (diagnostic only,
 * never linked into the product).
 *
 * One component, SPEC §2 keys (fitref.c ref_key restated), k = 1 jobs.  A step starts at job t with
 * the state S_t every earlier decision left; jobs t, t+1, ..., t+m-1 each take their best key
 * against S_t (in parallel, as 8-lane groups of one wave would).  Job t+i's speculative choice is
 * VALID when no earlier job of the step wrote its chosen node and every node an earlier job of the
 * step wrote keys above it once updated (the rule that makes it the sequential answer); the step
 * commits the valid prefix.  Output: the histogram of committed jobs per step, and why a step
 * ended early (cause[0]: the job's best node is one an earlier job of the step took — best fit
 * keeps packing the same node; cause[1]: a node an earlier job took now fits it tighter).
 *
 *   gcc -O2 -shared -fPIC -o tools/libspec_model.so tools/spec_model.c */
#include <stdint.h>
#include <string.h>

static uint64_t key_of(int32_t cf, int32_t mf, int32_t gf, int32_t av, uint32_t mk, int32_t id,
                       int32_t c, int32_t m, int32_t g, int32_t w, uint32_t pbit) {
    const int32_t dc = cf - c, dm = mf - m, dg = gf - g, da = av - w;
    if ((dc | dm | dg | da) < 0 || !(mk & pbit)) return UINT64_MAX;
    uint32_t gr = (uint32_t)dg, cr = (uint32_t)dc, mr = (uint32_t)dm >> 10;
    gr = gr > 255u ? 255u : gr;
    cr = cr > 4095u ? 4095u : cr;
    mr = mr > 4095u ? 4095u : mr;
    return ((uint64_t)((gr << 24) | (cr << 12) | mr) << 32) | (uint32_t)id;
}

/* nodes: n rows (cf, mf, gf, av, mk, id) of one component (modified in place); jobs in priority
 * order.  hist[s] += 1 for every step that committed s jobs (s <= m <= 64).  Returns the steps. */
int64_t spec_steps(int32_t n, int32_t* cf, int32_t* mf, int32_t* gf, const int32_t* av,
                   const uint32_t* mk, const int32_t* id, int32_t j, const int32_t* c,
                   const int32_t* m, const int32_t* g, const int32_t* w, const uint16_t* part,
                   int32_t mstep, int64_t* hist, int32_t live_only, int64_t* cause) {
    int64_t steps = 0;
    int32_t t = 0;
    int32_t pos[64];
    uint64_t best[64];
    while (t < j) {
        int32_t cnt = 0, q = t;
        /* the step's jobs: the next mstep (live ones only when live_only: a job nothing fits at
         * the step's start is unplaced whatever happens and costs no decider step) */
        int32_t js[64];
        while (cnt < mstep && q < j) {
            const uint32_t pb = 1u << part[q];
            uint64_t b = UINT64_MAX;
            int32_t bp = -1;
            for (int32_t x = 0; x < n; ++x) {
                const uint64_t k = key_of(cf[x], mf[x], gf[x], av[x], mk[x], id[x], c[q], m[q], g[q], w[q], pb);
                if (k < b) b = k, bp = x;
            }
            if (live_only && b == UINT64_MAX) {
                ++q;
                continue;
            }
            js[cnt] = q;
            best[cnt] = b;
            pos[cnt] = bp;
            ++cnt;
            ++q;
        }
        if (cnt == 0) break;
        /* validate in order, applying the valid prefix */
        int32_t ok = 0;
        for (int32_t i = 0; i < cnt; ++i) {
            const int32_t qq = js[i];
            const uint32_t pb = 1u << part[qq];
            int valid = 1;
            for (int32_t e = 0; e < i && valid; ++e) {
                const int32_t x = pos[e];
                if (x < 0) continue;
                if (x == pos[i]) {
                    valid = 0;
                    if (cause) cause[0]++; /* the node an earlier job of the step took */
                } else if (key_of(cf[x], mf[x], gf[x], av[x], mk[x], id[x], c[qq], m[qq], g[qq], w[qq], pb) < best[i]) {
                    valid = 0;
                    if (cause) cause[1]++; /* a node an earlier job took now fits tighter */
                }
            }
            if (!valid) break;
            if (pos[i] >= 0) {
                cf[pos[i]] -= c[qq];
                mf[pos[i]] -= m[qq];
                gf[pos[i]] -= g[qq];
            }
            ++ok;
        }
        hist[ok]++;
        ++steps;
        t = js[ok - 1] + 1;
    }
    return steps;
}
