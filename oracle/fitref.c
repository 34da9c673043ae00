/* oracle/fitref.c — plain-C restatement of the reference's resource-fit path.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  Never linked into or called by the product library (libfitgpu.so).
 *
 * Go semantics restated here (ASCII inputs; scontrol output is ASCII):
 *   strings.Fields   -> split on runs of ' ', '\t', '\n', '\v', '\f', '\r'
 *   strings.Split    -> exact separator split (n+1 pieces for n separators)
 *   strconv.ParseInt(s, 10, 0/64) -> optional sign, decimal digits only, range error clamps
 * Every function cites the reference file:line it follows.  See fitref.h for parity status.
 */
#include "fitref.h"

#include <stdlib.h>
#include <string.h>

#define NS_PER_SEC 1000000000LL
#define NS_PER_MIN (60LL * NS_PER_SEC)
#define NS_PER_HOUR (60LL * NS_PER_MIN)

/* ---------------------------------------------------------------- Go helpers */
static int go_space(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

/* strconv.ParseInt(s[:n], 10, 64): 0 ok, -1 syntax error (value 0), -2 range error (clamped). */
static int go_parse_int(const char* s, size_t n, int64_t* out) {
    *out = 0;
    if (n == 0) return -1;
    int neg = 0;
    size_t i = 0;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
        if (n == 1) return -1;
    }
    uint64_t cutoff = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
    uint64_t v = 0;
    int range = 0;
    for (; i < n; i++) {
        char c = s[i];
        if (c < '0' || c > '9') {
            *out = 0;
            return -1;
        }
        if (!range) {
            uint64_t d = (uint64_t)(c - '0');
            if (v > (cutoff - d) / 10) {
                range = 1;
            } else {
                v = v * 10 + d;
            }
        }
    }
    if (range) {
        *out = neg ? INT64_MIN : INT64_MAX;
        return -2;
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 0;
}

/* strconv.Atoi: syntax error -> 0, range error -> clamped value (Go returns it with err). */
static int64_t go_atoi(const char* s, size_t n) {
    int64_t v;
    int rc = go_parse_int(s, n, &v);
    if (rc == -1) return 0;
    return v;
}

typedef struct {
    const char* p;
    size_t n;
} span;

/* next token of strings.Fields over [*cur, end) */
static int next_field(const char** cur, const char* end, span* tok) {
    const char* c = *cur;
    while (c < end && go_space(*c)) c++;
    if (c >= end) {
        *cur = c;
        return 0;
    }
    const char* b = c;
    while (c < end && !go_space(*c)) c++;
    tok->p = b;
    tok->n = (size_t)(c - b);
    *cur = c;
    return 1;
}

/* strings.Split(field, "=") has exactly 2 pieces <=> exactly one '=' in the field. */
static int split_kv(span f, span* k, span* v) {
    const char* eq = NULL;
    for (size_t i = 0; i < f.n; i++) {
        if (f.p[i] == '=') {
            if (eq) return 0;
            eq = f.p + i;
        }
    }
    if (!eq) return 0;
    k->p = f.p;
    k->n = (size_t)(eq - f.p);
    v->p = eq + 1;
    v->n = f.n - k->n - 1;
    return 1;
}

static int span_eq(span s, const char* lit) {
    size_t n = strlen(lit);
    return s.n == n && memcmp(s.p, lit, n) == 0;
}

/* strings.TrimSpace (ASCII) */
static span trim_space(const char* s, size_t n) {
    size_t b = 0, e = n;
    while (b < e && go_space(s[b])) b++;
    while (e > b && go_space(s[e - 1])) e--;
    span r = {s + b, e - b};
    return r;
}

/* first piece of strings.Split(v, ",") */
static span first_comma_piece(span v) {
    for (size_t i = 0; i < v.n; i++)
        if (v.p[i] == ',') {
            span r = {v.p, i};
            return r;
        }
    return v;
}

/* --------------------------------------------------- ParseDuration parse.go:36-109 */
static int parse_duration_span(const char* s, size_t n, int64_t* out_ns) {
    if (n == 0 || (n == 9 && memcmp(s, "UNLIMITED", 9) == 0)) return 1; /* :39-41 */
    span parts[4];
    int np = 0;
    size_t b = 0;
    for (size_t i = 0; i <= n; i++) { /* strings.Split(duration, ":") :46 */
        if (i == n || s[i] == ':') {
            if (np == 3) return -1; /* > 3 parts :47-49 */
            parts[np].p = s + b;
            parts[np].n = i - b;
            np++;
            b = i + 1;
        }
    }
    int64_t days = 0, hours = 0, minutes = 0, seconds = 0;
    const char* dash = memchr(parts[0].p, '-', parts[0].n); /* :50 */
    if (dash) {
        size_t di = (size_t)(dash - parts[0].p);
        if (go_parse_int(parts[0].p, di, &days)) return -1;                       /* :52 */
        if (go_parse_int(dash + 1, parts[0].n - di - 1, &hours)) return -1;       /* :56 */
        if (np > 1 && go_parse_int(parts[1].p, parts[1].n, &minutes)) return -1;  /* :60-65 */
        if (np > 2 && go_parse_int(parts[2].p, parts[2].n, &seconds)) return -1;  /* :66-71 */
    } else {
        switch (np) { /* :73-101 */
            case 1:
                if (go_parse_int(parts[0].p, parts[0].n, &minutes)) return -1;
                break;
            case 2:
                if (go_parse_int(parts[0].p, parts[0].n, &minutes)) return -1;
                if (go_parse_int(parts[1].p, parts[1].n, &seconds)) return -1;
                break;
            case 3:
                if (go_parse_int(parts[0].p, parts[0].n, &hours)) return -1;
                if (go_parse_int(parts[1].p, parts[1].n, &minutes)) return -1;
                if (go_parse_int(parts[2].p, parts[2].n, &seconds)) return -1;
                break;
        }
    }
    /* :104-107, time.Duration arithmetic wraps on overflow */
    uint64_t d = 0;
    d += (uint64_t)(24 * NS_PER_HOUR) * (uint64_t)days;
    d += (uint64_t)NS_PER_HOUR * (uint64_t)hours;
    d += (uint64_t)NS_PER_MIN * (uint64_t)minutes;
    d += (uint64_t)NS_PER_SEC * (uint64_t)seconds;
    *out_ns = (int64_t)d;
    return 0;
}

int ref_parse_duration(const char* s, int64_t* out_ns) {
    *out_ns = 0;
    return parse_duration_span(s, strlen(s), out_ns);
}

/* -------------------------------------------------- parseResources parse.go:111-190 */
int ref_parse_resources(const char* text, ref_resources* out) {
    memset(out, 0, sizeof(*out));
    span t = trim_space(text, strlen(text)); /* :114 */
    enum { K_MAXTIME, K_MAXCPU, K_TOTCPU, K_MAXMEM, K_MAXNODES, K_TOTNODES, K_N };
    static const char* keys[K_N] = {"MaxTime", "MaxCPUsPerNode", "TotalCPUs",
                                    "MaxMemPerNode", "MaxNodes", "TotalNodes"};
    int have[K_N] = {0};
    span val[K_N];
    const char* cur = t.p;
    const char* end = t.p + t.n;
    span f, k, v;
    while (next_field(&cur, end, &f)) { /* :118-124: fMap[k] = append(..., Split(v, ",")...) */
        if (!split_kv(f, &k, &v)) continue;
        for (int i = 0; i < K_N; i++)
            if (!have[i] && span_eq(k, keys[i])) {
                have[i] = 1;
                val[i] = first_comma_piece(v); /* fMap[k][0] */
            }
    }
    if (have[K_MAXTIME]) { /* :128-138 */
        int64_t d;
        int rc = parse_duration_span(val[K_MAXTIME].p, val[K_MAXTIME].n, &d);
        if (rc < 0) return -1;
        out->wall_ns = rc == 1 ? -1 : d;
    }
    if (have[K_MAXCPU]) { /* :139-157 */
        if (span_eq(val[K_MAXCPU], "UNLIMITED")) {
            out->cpu_per_node = -1;
            if (have[K_TOTCPU]) {
                int64_t c;
                if (go_parse_int(val[K_TOTCPU].p, val[K_TOTCPU].n, &c)) return -1;
                out->cpu_per_node = c;
            }
        } else {
            int64_t c;
            if (go_parse_int(val[K_MAXCPU].p, val[K_MAXCPU].n, &c)) return -1;
            out->cpu_per_node = c;
        }
    }
    if (have[K_MAXMEM]) { /* :158-168 */
        if (span_eq(val[K_MAXMEM], "UNLIMITED")) {
            out->mem_per_node = -1;
        } else {
            int64_t m;
            if (go_parse_int(val[K_MAXMEM].p, val[K_MAXMEM].n, &m)) return -1;
            out->mem_per_node = m;
        }
    }
    if (have[K_MAXNODES]) { /* :169-187 */
        if (span_eq(val[K_MAXNODES], "UNLIMITED")) {
            out->nodes = -1;
            if (have[K_TOTNODES]) {
                int64_t c;
                if (go_parse_int(val[K_TOTNODES].p, val[K_TOTNODES].n, &c)) return -1;
                out->nodes = c;
            }
        } else {
            int64_t c;
            if (go_parse_int(val[K_MAXNODES].p, val[K_MAXNODES].n, &c)) return -1;
            out->nodes = c;
        }
    }
    return 0;
}

/* helper: iterate strings.Split(s, "\n\n") pieces */
static const char* next_record(const char* cur, const char* end, span* rec, int* done) {
    const char* b = cur;
    for (const char* c = cur; c + 1 < end; c++) {
        if (c[0] == '\n' && c[1] == '\n') {
            rec->p = b;
            rec->n = (size_t)(c - b);
            return c + 2;
        }
    }
    rec->p = b;
    rec->n = (size_t)(end - b);
    *done = 1;
    return end;
}

static int put_name(char* buf, int buflen, int* used, const char* p, size_t n) {
    if (*used + (int)n + 1 > buflen) return -1;
    memcpy(buf + *used, p, n);
    buf[*used + n] = 0;
    *used += (int)n + 1;
    return 0;
}

/* ------------------------------------------- parsePartitionsNames parse.go:192-210 */
int ref_parse_partitions_names(const char* raw, char* buf, int buflen) {
    span t = trim_space(raw, strlen(raw));
    const char* cur = t.p;
    const char* end = t.p + t.n;
    int count = 0, used = 0, done = 0;
    while (!done) {
        span rec, f, k, v, name = {"", 0};
        cur = next_record(cur, end, &rec, &done);
        const char* c = rec.p;
        while (next_field(&c, rec.p + rec.n, &f))
            if (split_kv(f, &k, &v) && span_eq(k, "PartitionName")) name = v; /* last wins */
        if (put_name(buf, buflen, &used, name.p, name.n)) return -1;
        count++;
    }
    return count;
}

/* ------------------------------------------------- parsePartition parse.go:278-289 */
int ref_parse_partition(const char* raw, char* buf, int buflen) {
    const char* cur = raw;
    const char* end = raw + strlen(raw);
    int count = 0, used = 0;
    span f, k, v;
    while (next_field(&cur, end, &f)) {
        if (!split_kv(f, &k, &v) || !span_eq(k, "Nodes")) continue;
        size_t b = 0;
        for (size_t i = 0; i <= v.n; i++) { /* strings.Split(s[1], ",") */
            if (i == v.n || v.p[i] == ',') {
                if (put_name(buf, buflen, &used, v.p + b, i - b)) return -1;
                count++;
                b = i + 1;
            }
        }
    }
    return count;
}

/* ------------------------------------------------------ parseNode parse.go:291-308 */
static void parse_node_span(const char* p, size_t n, ref_node* out) {
    memset(out, 0, sizeof(*out));
    const char* cur = p;
    span f, k, v;
    while (next_field(&cur, p + n, &f)) {
        if (!split_kv(f, &k, &v)) continue;
        int64_t x;
        if (span_eq(k, "CPUTot")) {
            go_parse_int(v.p, v.n, &x); /* error ignored: `_ =` at :297 */
            out->cpus = x;
        } else if (span_eq(k, "CPUAlloc")) {
            go_parse_int(v.p, v.n, &x);
            out->allo_cpus = x;
        } else if (span_eq(k, "RealMemory")) {
            go_parse_int(v.p, v.n, &x);
            out->memory = x;
        } else if (span_eq(k, "AllocMem")) {
            go_parse_int(v.p, v.n, &x);
            out->allo_memory = x;
        }
    }
}

void ref_parse_node(const char* raw, ref_node* out) { parse_node_span(raw, strlen(raw), out); }

/* Client.Nodes record loop, pkg/slurm-agent/slurm.go:354-363 */
int ref_parse_nodes(const char* scontrol_out, ref_node* out, int cap) {
    span t = trim_space(scontrol_out, strlen(scontrol_out));
    const char* cur = t.p;
    const char* end = t.p + t.n;
    int count = 0, done = 0;
    while (!done && count < cap) {
        span rec;
        cur = next_record(cur, end, &rec, &done);
        if (rec.n == 0) continue; /* :357-359 */
        parse_node_span(rec.p, rec.n, &out[count++]);
    }
    return count;
}

/* ------------------ extractBatchResourcesFromScript pkg/slurm-bridge-operator/parse.go:30-124 */
static int apply_sbatch_param(ref_job_resources* r, span param, span value) {
    int64_t x;
    if (span_eq(param, "--time") || span_eq(param, "-t")) { /* :84-91 */
        int64_t d;
        int rc = parse_duration_span(value.p, value.n, &d);
        if (rc < 0) return -1;
        if (rc == 0) r->wall_ns = d;
    } else if (span_eq(param, "--nodes") || span_eq(param, "-N")) { /* :92-102 */
        const char* dash = memchr(value.p, '-', value.n);
        if (dash) value.n = (size_t)(dash - value.p);
        if (go_parse_int(value.p, value.n, &x)) return -1;
        r->nodes = x;
    } else if (span_eq(param, "--mem-per-cpu")) { /* :103-109 */
        if (go_parse_int(value.p, value.n, &x)) return -1;
        r->mem_per_cpu = x;
    } else if (span_eq(param, "--cpus-per-task") || span_eq(param, "-c")) { /* :110-115 */
        if (go_parse_int(value.p, value.n, &x)) return -1;
        r->cpus_per_task = x;
    } else if (span_eq(param, "--ntasks-per-node")) { /* :116-121 */
        if (go_parse_int(value.p, value.n, &x)) return -1;
        r->ntasks_per_node = x;
    }
    return 0;
}

int ref_extract_batch_resources(const char* script, ref_job_resources* out) {
    memset(out, 0, sizeof(*out));
    const char* cur = script;
    const char* end = script + strlen(script);
    while (cur < end) { /* bufio.Scanner(ScanLines) :36-38 */
        const char* nl = memchr(cur, '\n', (size_t)(end - cur));
        const char* le = nl ? nl : end;
        span line = {cur, (size_t)(le - cur)};
        cur = nl ? nl + 1 : end;
        if (line.n > 0 && line.p[line.n - 1] == '\r') line.n--;
        if (line.n > 64 * 1024) break; /* bufio.ErrTooLong ends the scan */
        if (line.n == 0 || (line.n >= 2 && line.p[0] == '#' && line.p[1] == '!')) continue; /* :40 */
        if (line.n < 7 || memcmp(line.p, "#SBATCH", 7) != 0) break;                       /* :44 */
        span params[256];
        int np = 0;
        const char* c = line.p + 7;
        span f;
        while (np < 256 && next_field(&c, line.p + line.n, &f)) params[np++] = f; /* :48 */
        for (int j = 0; j < np; j++) {
            span param = params[j], value = {"", 0};
            const char* eq = memchr(param.p, '=', param.n);
            if (eq) { /* :54-57 */
                value.p = eq + 1;
                value.n = param.n - (size_t)(eq - param.p) - 1;
                param.n = (size_t)(eq - param.p);
            } else { /* :58-61: `i < len(params)-1` with i == -1 is always true */
                if (j + 1 >= np) return -3; /* params[j+1] out of range: the reference panics */
                value = params[j + 1];
                j++;
            }
            if (apply_sbatch_param(out, param, value)) return -1;
        }
    }
    return 0;
}

/* setRequireResourceBySpec pod.go:70-89 + setDefaultRequireResource pod.go:97-107 */
void ref_apply_spec_and_defaults(ref_job_resources* r, int64_t nodes, int64_t cpus_per_task,
                                 int64_t mem_per_cpu, int64_t ntasks_per_node, const char* array,
                                 int64_t ntasks) {
    if (nodes > 0) r->nodes = nodes;
    if (cpus_per_task > 0) r->cpus_per_task = cpus_per_task;
    if (mem_per_cpu > 0) r->mem_per_cpu = mem_per_cpu;
    if (ntasks_per_node > 0) r->ntasks_per_node = ntasks_per_node;
    if (array && array[0]) {
        strncpy(r->array, array, sizeof(r->array) - 1);
        r->array[sizeof(r->array) - 1] = 0;
    }
    if (ntasks > 0) r->ntasks = ntasks;
    if (r->nodes == 0) r->nodes = 1;
    if (r->cpus_per_task == 0) r->cpus_per_task = 1;
    if (r->mem_per_cpu == 0) r->mem_per_cpu = 1024;
}

/* parseArrayLen parse.go:126-135 */
int64_t ref_parse_array_len(const char* array) {
    size_t n = strlen(array);
    const char* dash = memchr(array, '-', n);
    if (dash) {
        size_t a = (size_t)(dash - array);
        const char* s1 = dash + 1;
        const char* dash2 = memchr(s1, '-', n - a - 1);
        size_t b = dash2 ? (size_t)(dash2 - s1) : n - a - 1;
        int64_t start = go_atoi(array, a), endi = go_atoi(s1, b);
        return (int64_t)((uint64_t)endi - (uint64_t)start + 1);
    }
    int64_t pieces = 1;
    for (size_t i = 0; i < n; i++) pieces += array[i] == ',';
    return pieces;
}

/* genResourceListForPod pod.go:143-162 */
void ref_pod_request(const ref_job_resources* r, int64_t* cpu, int64_t* memory) {
    uint64_t c;
    if (r->ntasks > 0)
        c = (uint64_t)r->cpus_per_task * (uint64_t)r->ntasks;
    else if (r->ntasks_per_node > 0 && r->nodes > 0)
        c = (uint64_t)r->cpus_per_task * (uint64_t)r->ntasks_per_node * (uint64_t)r->nodes;
    else
        c = (uint64_t)r->cpus_per_task;
    if (r->array[0]) c *= (uint64_t)ref_parse_array_len(r->array);
    *cpu = (int64_t)c;
    *memory = (int64_t)(c * (uint64_t)r->mem_per_cpu * 1024u);
}

/* DESIGN.md §2 "demand": the engine's per-node request of one (task of a) job.  Restated from the
 * SPEC text, not from the product: k = nodes (>= 1); tasks per node = ntasksPerNode, else
 * ceil(ntasks / k), else 1; cpu = cpusPerTask x tasks per node; mem = cpu x memPerCpu (MiB);
 * wall = walltime rounded up to whole minutes.  -1: a value outside the engine's int32 / k range. */
int ref_job_demand(const ref_job_resources* r, int32_t* cpu, int32_t* mem, int32_t* wall,
                   uint16_t* k) {
    int64_t nodes = r->nodes >= 1 ? r->nodes : 1;
    int64_t per_node_tasks = 1;
    if (r->ntasks_per_node >= 1)
        per_node_tasks = r->ntasks_per_node;
    else if (r->ntasks >= 1)
        per_node_tasks = r->ntasks / nodes + (r->ntasks % nodes != 0);
    int64_t cpt = r->cpus_per_task >= 1 ? r->cpus_per_task : 1;
    int64_t mpc = r->mem_per_cpu >= 1 ? r->mem_per_cpu : 1024;
    if (nodes > 65535 || r->wall_ns < 0) return -1;
    /* overflow-safe products against INT32_MAX */
    if (per_node_tasks > INT32_MAX / cpt) return -1;
    int64_t c = per_node_tasks * cpt;
    if (mpc > INT32_MAX / c + 1 || c * mpc > INT32_MAX) return -1;
    int64_t minutes = r->wall_ns / NS_PER_MIN + (r->wall_ns % NS_PER_MIN != 0);
    if (minutes > INT32_MAX) return -1;
    *cpu = (int32_t)c;
    *mem = (int32_t)(c * mpc);
    *wall = (int32_t)minutes;
    *k = (uint16_t)nodes;
    return 0;
}

static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

static int all_digits(const char* s, size_t n) {
    if (n == 0) return 0;
    for (size_t i = 0; i < n; i++)
        if (s[i] < '0' || s[i] > '9') return 0;
    return 1;
}

/* Slurm's --array syntax (sbatch(1) "--array=<indexes>": comma-separated ids and ranges "a-b",
 * ranges with a step "a-b:s", an optional "%N" limit on simultaneously running tasks).  The
 * ids are listed explicitly, sorted and de-duplicated here.  -1: malformed / id > 4194303. */
static int array_ids(const char* array, int64_t* tasks, int64_t* running, int64_t* max_id) {
    span a = trim_space(array, strlen(array));
    int64_t limit = -1;
    const char* pct = memchr(a.p, '%', a.n);
    size_t body = a.n;
    if (pct) {
        size_t off = (size_t)(pct - a.p) + 1;
        if (!all_digits(a.p + off, a.n - off) || go_parse_int(a.p + off, a.n - off, &limit) || limit < 1)
            return -1;
        body = (size_t)(pct - a.p);
    }
    if (body == 0) return -1;
    size_t cap = 1024, cnt = 0;
    int64_t* ids = malloc(cap * sizeof *ids);
    if (!ids) return -1;
    size_t i = 0;
    int bad = 0;
    while (i <= body && !bad) {
        size_t j = i;
        while (j < body && a.p[j] != ',') j++;
        /* item [i, j): lo[-hi[:step]] */
        const char* it = a.p + i;
        size_t n = j - i;
        const char* d = memchr(it, '-', n);
        const char* c = memchr(it, ':', n);
        int64_t lo, hi, st = 1;
        size_t nlo = d ? (size_t)(d - it) : (c ? (size_t)(c - it) : n);
        if (c && !d) bad = 1;
        if (!bad && (!all_digits(it, nlo) || go_parse_int(it, nlo, &lo))) bad = 1;
        hi = lo;
        if (!bad && d) {
            size_t off = nlo + 1, nhi = (c ? (size_t)(c - it) : n) - off;
            if (!all_digits(it + off, nhi) || go_parse_int(it + off, nhi, &hi)) bad = 1;
        }
        if (!bad && c) {
            size_t off = (size_t)(c - it) + 1;
            if (!all_digits(it + off, n - off) || go_parse_int(it + off, n - off, &st) || st < 1) bad = 1;
        }
        if (!bad && (hi < lo || hi > 4194303)) bad = 1;
        for (int64_t x = lo; !bad && x <= hi; x += st) {
            if (cnt == cap) {
                cap *= 2;
                int64_t* g = realloc(ids, cap * sizeof *ids);
                if (!g) {
                    bad = 1;
                    break;
                }
                ids = g;
            }
            ids[cnt++] = x;
        }
        i = j + 1;
    }
    if (bad) {
        free(ids);
        return -1;
    }
    qsort(ids, cnt, sizeof *ids, cmp_i64);
    const int64_t ids_max = cnt ? ids[cnt - 1] : -1;
    int64_t distinct = 0;
    for (size_t q = 0; q < cnt; q++) distinct += q == 0 || ids[q] != ids[q - 1];
    free(ids);
    *tasks = distinct;
    *running = (limit > 0 && limit < distinct) ? limit : distinct;
    *max_id = cnt ? ids_max : -1;
    return 0;
}

int ref_array_tasks(const char* array, int64_t* tasks, int64_t* running) {
    int64_t max_id;
    return array_ids(array, tasks, running, &max_id);
}

/* One sizecar pod's admission requests: the script's #SBATCH header
 * (extractBatchResourcesFromScript, parse.go:30-69) under the labels newSubmitRequestForPod
 * reads (provider.go:74-123: strconv.ParseInt, skipped on error), which getSbatchOpts passes as
 * command-line flags that win over #SBATCH lines (pkg/slurm-agent/slurm.go:189-229); defaults
 * pod.go:97-107; ref_job_demand; one request per simultaneously running array task.
 * labels[6] = nodes, cpus-per-task, mem-per-cpu, ntasks-per-node, array, ntask (NULL = absent).
 * out[i*4 + 0..3] = cpu, mem, wall, k for min(n, cap) tasks.  Returns n, or -1 (malformed header
 * or array, the reference's error / panic cases included) / -2 (demand out of range, or an array
 * task id >= max_array_size: Slurm's MaxArraySize, which sbatch enforces). */
int ref_pod_demand(const char* const* labels, const char* script, int64_t max_array_size,
                   int32_t* out, int cap) {
    ref_job_resources r;
    memset(&r, 0, sizeof r);
    if (script && ref_extract_batch_resources(script, &r) != 0) return -1;
    int64_t v[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 6; i++) {
        if (i == 4 || !labels[i]) continue;
        int64_t x;
        if (go_parse_int(labels[i], strlen(labels[i]), &x) == 0) v[i] = x;
    }
    ref_apply_spec_and_defaults(&r, v[0], v[1], v[2], v[3], NULL, v[5]);
    int32_t c, m, w;
    uint16_t k;
    if (ref_job_demand(&r, &c, &m, &w, &k) != 0 || k > 8) return -2;
    int64_t tasks = 1, running = 1, max_id = 0;
    if (labels[4] && labels[4][0] && array_ids(labels[4], &tasks, &running, &max_id) != 0) return -1;
    if (max_id >= max_array_size) return -2;
    for (int64_t i = 0; i < running && i < cap; i++) {
        out[i * 4 + 0] = c;
        out[i * 4 + 1] = m;
        out[i * 4 + 2] = w;
        out[i * 4 + 3] = k;
    }
    return (int)running;
}

/* GetPartitionCapacity pkg/slurm-virtual-kubelet/node.go:169-199 */
void ref_partition_capacity(const ref_node* nodes, int n, int64_t* cpu, int64_t* memory,
                            int64_t* gpu, int64_t* pods) {
    uint64_t c = 0, m = 0, g = 0;
    for (int i = 0; i < n; i++) {
        c += (uint64_t)nodes[i].cpus;
        m += (uint64_t)nodes[i].memory;
        g += (uint64_t)nodes[i].gpus;
    }
    *cpu = (int64_t)c;
    *memory = (int64_t)(m * (2u << 10)); /* :193 — MiB × 2048 (sic) */
    *gpu = (int64_t)g;
    *pods = (int64_t)c; /* :197 */
}

/* ----------------------------------------------------------- SPEC best fit */
uint64_t ref_key(int32_t node_id, int32_t cpu_free, int32_t mem_free, int32_t gpu_free,
                 int32_t avail, uint32_t mask, int32_t cpu, int32_t mem, int32_t gpu, int32_t wall,
                 int32_t part) {
    if (!((mask >> part) & 1u)) return UINT64_MAX;
    if (cpu_free < cpu || mem_free < mem || gpu_free < gpu || avail < wall) return UINT64_MAX;
    uint32_t gr = (uint32_t)(gpu_free - gpu);
    uint32_t cr = (uint32_t)(cpu_free - cpu);
    uint32_t mr = (uint32_t)(mem_free - mem) >> 10;
    if (gr > 255u) gr = 255u;
    if (cr > 4095u) cr = 4095u;
    if (mr > 4095u) mr = 4095u;
    uint32_t score = (gr << 24) | (cr << 12) | mr;
    return ((uint64_t)score << 32) | (uint32_t)node_id;
}

int ref_place(int32_t n, int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free,
              const int32_t* avail_min, const uint32_t* part_mask,
              int32_t p, const int32_t* max_time, const int32_t* max_cpus, const int32_t* max_mem,
              int32_t j, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
              const int32_t* wall, const uint16_t* part, const uint16_t* nodes_k, int32_t kmax,
              int32_t* out, int64_t* stats) {
    if (n < 0 || j < 0 || kmax < 1 || p < 0 || p > 32) return -1;
    for (int32_t q = 0; q < j; q++) {
        int k = nodes_k ? nodes_k[q] : 1;
        if (k == 0) k = 1;
        if (k > kmax || cpu[q] < 0 || mem[q] < 0 || gpu[q] < 0 || wall[q] < 0) return -1;
    }
    int64_t placed = 0, unplaced = 0, rejected = 0, evals = 0;
    uint64_t best[64];
    if (kmax > 64) return -1;
    for (int32_t q = 0; q < j; q++) {
        int k = nodes_k ? nodes_k[q] : 1;
        if (k == 0) k = 1;
        int32_t* o = out + (int64_t)q * kmax;
        for (int i = 0; i < kmax; i++) o[i] = -1;
        int pq = part[q];
        if (pq >= p || (max_time[pq] >= 0 && wall[q] > max_time[pq]) ||
            (max_cpus[pq] >= 0 && cpu[q] > max_cpus[pq]) ||
            (max_mem[pq] >= 0 && mem[q] > max_mem[pq])) {
            for (int i = 0; i < k; i++) o[i] = -2;
            rejected++;
            continue;
        }
        for (int i = 0; i < k; i++) best[i] = UINT64_MAX;
        for (int32_t x = 0; x < n; x++) {
            uint64_t key = ref_key(x, cpu_free[x], mem_free[x], gpu_free[x], avail_min[x],
                                   part_mask[x], cpu[q], mem[q], gpu[q], wall[q], pq);
            if (key < best[k - 1]) { /* insertion into the sorted k-best */
                int i = k - 1;
                while (i > 0 && best[i - 1] > key) {
                    best[i] = best[i - 1];
                    i--;
                }
                best[i] = key;
            }
        }
        evals += n;
        if (best[k - 1] == UINT64_MAX) {
            unplaced++;
            continue;
        }
        for (int i = 0; i < k; i++) {
            int32_t x = (int32_t)(uint32_t)best[i];
            o[i] = x;
            cpu_free[x] -= cpu[q];
            mem_free[x] -= mem[q];
            gpu_free[x] -= gpu[q];
        }
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

/* ------------------------------------------------------------ generator twin */
uint64_t ref_rnd(uint64_t seed, uint32_t stream, uint64_t idx) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx * 64u + stream + 1u);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
