// ingest.cpp — host-side mirrors of the reference's text ingest and demand arithmetic that feed
// the placement engine.  Same names, argument meaning and error
// behaviour as the Go functions cited on each; one deliberate difference: where the reference
// panics (a bare flag as the last #SBATCH token, pkg/slurm-bridge-operator/parse.go:58-60) this
// returns FIT_E_PARSE.  Text is handled as ASCII (scontrol output is ASCII).
#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/fitgpu.h"

namespace {

using sv = std::string_view;

bool is_space(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

sv trim_space(sv s) {  // strings.TrimSpace
    while (!s.empty() && is_space(s.front())) s.remove_prefix(1);
    while (!s.empty() && is_space(s.back())) s.remove_suffix(1);
    return s;
}

std::vector<sv> fields(sv s) {  // strings.Fields
    std::vector<sv> out;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && is_space(s[i])) ++i;
        size_t b = i;
        while (i < s.size() && !is_space(s[i])) ++i;
        if (i > b) out.push_back(s.substr(b, i - b));
    }
    return out;
}

std::vector<sv> split(sv s, sv sep) {  // strings.Split (sep non-empty)
    std::vector<sv> out;
    size_t b = 0;
    for (;;) {
        size_t p = s.find(sep, b);
        if (p == sv::npos) {
            out.push_back(s.substr(b));
            return out;
        }
        out.push_back(s.substr(b, p - b));
        b = p + sep.size();
    }
}

// strconv.ParseInt(s, 10, 64): 0 ok, 1 syntax error (v = 0), 2 range error (v clamped)
int parse_int(sv s, int64_t& v) {
    v = 0;
    if (s.empty()) return 1;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        s.remove_prefix(1);
        if (s.empty()) return 1;
    }
    const uint64_t lim = neg ? (1ull << 63) : (1ull << 63) - 1;
    uint64_t acc = 0;
    bool over = false;
    for (char ch : s) {
        if (ch < '0' || ch > '9') {
            v = 0;
            return 1;
        }
        const uint64_t d = (uint64_t)(ch - '0');
        if (!over && acc > (lim - d) / 10) over = true;
        if (!over) acc = acc * 10 + d;
    }
    if (over) {
        v = neg ? INT64_MIN : INT64_MAX;
        return 2;
    }
    v = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return 0;
}

// ParseDuration, pkg/slurm-agent/parse.go:36-109
int parse_duration(sv d, int64_t& ns) {
    ns = 0;
    if (d == "UNLIMITED" || d.empty()) return FIT_E_UNLIMITED;
    const std::vector<sv> parts = split(d, ":");
    if (parts.size() > 3) return FIT_E_PARSE;
    int64_t days = 0, hours = 0, minutes = 0, seconds = 0;
    const size_t i = parts[0].find('-');
    if (i != sv::npos) {
        if (parse_int(parts[0].substr(0, i), days)) return FIT_E_PARSE;
        if (parse_int(parts[0].substr(i + 1), hours)) return FIT_E_PARSE;
        if (parts.size() > 1 && parse_int(parts[1], minutes)) return FIT_E_PARSE;
        if (parts.size() > 2 && parse_int(parts[2], seconds)) return FIT_E_PARSE;
    } else if (parts.size() == 1) {
        if (parse_int(parts[0], minutes)) return FIT_E_PARSE;
    } else if (parts.size() == 2) {
        if (parse_int(parts[0], minutes) || parse_int(parts[1], seconds)) return FIT_E_PARSE;
    } else {
        if (parse_int(parts[0], hours) || parse_int(parts[1], minutes) ||
            parse_int(parts[2], seconds))
            return FIT_E_PARSE;
    }
    constexpr uint64_t S = 1000000000ull, M = 60 * S, H = 60 * M;
    uint64_t acc = 24 * H * (uint64_t)days;  // time.Duration arithmetic wraps
    acc += H * (uint64_t)hours;
    acc += M * (uint64_t)minutes;
    acc += S * (uint64_t)seconds;
    ns = (int64_t)acc;
    return FIT_OK;
}

// value of the first "key=v1,v2,..." field (fMap[key][0] in parseResources), if present
bool first_value(const std::vector<sv>& fs, sv key, sv& out) {
    for (sv f : fs) {
        const std::vector<sv> kv = split(f, "=");
        if (kv.size() != 2 || kv[0] != key) continue;
        out = split(kv[1], ",")[0];
        return true;
    }
    return false;
}

int put_names(const std::vector<sv>& names, char* buf, int32_t buflen) {
    int32_t used = 0;
    for (sv s : names) {
        if (used + (int32_t)s.size() + 1 > buflen) return FIT_E_INVAL;
        if (!s.empty()) memcpy(buf + used, s.data(), s.size());
        buf[used + s.size()] = 0;
        used += (int32_t)s.size() + 1;
    }
    return (int)names.size();
}

void parse_node(sv raw, fit_node& n) {  // parseNode, parse.go:291-308
    n = fit_node{};
    for (sv f : fields(raw)) {
        const std::vector<sv> kv = split(f, "=");
        if (kv.size() != 2) continue;
        int64_t v;
        if (kv[0] == "CPUTot") {
            parse_int(kv[1], v);  // errors ignored (`_ =`), value as ParseInt returns it
            n.cpus = v;
        } else if (kv[0] == "CPUAlloc") {
            parse_int(kv[1], v);
            n.allo_cpus = v;
        } else if (kv[0] == "RealMemory") {
            parse_int(kv[1], v);
            n.memory = v;
        } else if (kv[0] == "AllocMem") {
            parse_int(kv[1], v);
            n.allo_memory = v;
        }
    }
}

// applySbatchParam, pkg/slurm-bridge-operator/parse.go:82-124
int apply_sbatch_param(fit_job_resources& r, sv param, sv value) {
    int64_t v;
    if (param == "--time" || param == "-t") {
        int64_t ns;
        const int rc = parse_duration(value, ns);
        if (rc == FIT_E_PARSE) return FIT_E_PARSE;
        if (rc == FIT_OK) r.wall_ns = ns;
    } else if (param == "--nodes" || param == "-N") {
        const size_t i = value.find('-');  // min nodes only
        if (i != sv::npos) value = value.substr(0, i);
        if (parse_int(value, v)) return FIT_E_PARSE;
        r.nodes = v;
    } else if (param == "--mem-per-cpu") {
        if (parse_int(value, v)) return FIT_E_PARSE;
        r.mem_per_cpu = v;
    } else if (param == "--cpus-per-task" || param == "-c") {
        if (parse_int(value, v)) return FIT_E_PARSE;
        r.cpus_per_task = v;
    } else if (param == "--ntasks-per-node") {
        if (parse_int(value, v)) return FIT_E_PARSE;
        r.ntasks_per_node = v;
    }
    return FIT_OK;
}

int64_t atoi_go(sv s) {  // strconv.Atoi value as returned alongside an error
    int64_t v;
    return parse_int(s, v) == 1 ? 0 : v;
}

}  // namespace

extern "C" {

int fit_parse_duration(const char* s, int64_t* out_ns) {
    if (!s || !out_ns) return FIT_E_INVAL;
    return parse_duration(sv(s), *out_ns);
}

int fit_parse_resources(const char* text, fit_resources* out) {  // parse.go:111-190
    if (!text || !out) return FIT_E_INVAL;
    *out = fit_resources{};
    const std::vector<sv> fs = fields(trim_space(sv(text)));
    sv v, tot;
    if (first_value(fs, "MaxTime", v)) {
        int64_t ns;
        const int rc = parse_duration(v, ns);
        if (rc == FIT_E_PARSE) return FIT_E_PARSE;
        out->wall_ns = rc == FIT_E_UNLIMITED ? -1 : ns;
    }
    int64_t x;
    if (first_value(fs, "MaxCPUsPerNode", v)) {
        if (v == "UNLIMITED") {
            out->cpu_per_node = -1;
            if (first_value(fs, "TotalCPUs", tot)) {
                if (parse_int(tot, x)) return FIT_E_PARSE;
                out->cpu_per_node = x;
            }
        } else {
            if (parse_int(v, x)) return FIT_E_PARSE;
            out->cpu_per_node = x;
        }
    }
    if (first_value(fs, "MaxMemPerNode", v)) {
        if (v == "UNLIMITED") {
            out->mem_per_node = -1;
        } else {
            if (parse_int(v, x)) return FIT_E_PARSE;
            out->mem_per_node = x;
        }
    }
    if (first_value(fs, "MaxNodes", v)) {
        if (v == "UNLIMITED") {
            out->nodes = -1;
            if (first_value(fs, "TotalNodes", tot)) {
                if (parse_int(tot, x)) return FIT_E_PARSE;
                out->nodes = x;
            }
        } else {
            if (parse_int(v, x)) return FIT_E_PARSE;
            out->nodes = x;
        }
    }
    return FIT_OK;
}

int fit_parse_nodes(const char* text, fit_node* out, int32_t cap) {  // slurm.go:354-363
    if (!text || (cap > 0 && !out) || cap < 0) return FIT_E_INVAL;
    int32_t n = 0;
    for (sv rec : split(trim_space(sv(text)), "\n\n")) {
        if (rec.empty()) continue;
        if (n == cap) return FIT_E_INVAL;
        parse_node(rec, out[n++]);
    }
    return n;
}

int fit_parse_partition(const char* text, char* buf, int32_t buflen) {  // parse.go:278-289
    if (!text || !buf) return FIT_E_INVAL;
    std::vector<sv> nodes;
    for (sv f : fields(sv(text))) {
        const std::vector<sv> kv = split(f, "=");
        if (kv.size() == 2 && kv[0] == "Nodes")
            for (sv n : split(kv[1], ",")) nodes.push_back(n);
    }
    return put_names(nodes, buf, buflen);
}

int fit_parse_partitions_names(const char* text, char* buf, int32_t buflen) {  // :192-210
    if (!text || !buf) return FIT_E_INVAL;
    std::vector<sv> names;
    for (sv p : split(trim_space(sv(text)), "\n\n")) {
        sv name;
        for (sv f : fields(p)) {
            const std::vector<sv> kv = split(f, "=");
            if (kv.size() == 2 && kv[0] == "PartitionName") name = kv[1];
        }
        names.push_back(name);
    }
    return put_names(names, buf, buflen);
}

int fit_extract_batch_resources(const char* script, fit_job_resources* out) {  // parse.go:30-69
    if (!script || !out) return FIT_E_INVAL;
    *out = fit_job_resources{};
    sv rest(script);
    while (!rest.empty()) {  // bufio.Scanner / ScanLines
        const size_t nl = rest.find('\n');
        sv line = rest.substr(0, nl);
        rest = nl == sv::npos ? sv() : rest.substr(nl + 1);
        if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
        if (line.size() > 64 * 1024) break;  // bufio.ErrTooLong stops the scan
        if (line.empty() || line.substr(0, 2) == "#!") continue;
        if (line.substr(0, 7) != "#SBATCH") break;
        const std::vector<sv> params = fields(line.substr(7));
        for (size_t j = 0; j < params.size(); ++j) {
            sv param = params[j], value;
            const size_t i = param.find('=');
            if (i != sv::npos) {
                value = param.substr(i + 1);
                param = param.substr(0, i);
            } else {
                // the reference always takes params[j+1] here (`i < len(params)-1`, i == -1)
                if (j + 1 >= params.size()) return FIT_E_PARSE;  // reference: index panic
                value = params[++j];
            }
            const int rc = apply_sbatch_param(*out, param, value);
            if (rc) return rc;
        }
    }
    return FIT_OK;
}

void fit_apply_spec(fit_job_resources* r, int64_t nodes, int64_t cpus_per_task,
                    int64_t mem_per_cpu, int64_t ntasks_per_node, const char* array,
                    int64_t ntasks) {  // pod.go:70-107
    if (!r) return;
    if (nodes > 0) r->nodes = nodes;
    if (cpus_per_task > 0) r->cpus_per_task = cpus_per_task;
    if (mem_per_cpu > 0) r->mem_per_cpu = mem_per_cpu;
    if (ntasks_per_node > 0) r->ntasks_per_node = ntasks_per_node;
    if (array && array[0]) {
        const size_t n = std::min(strlen(array), sizeof(r->array) - 1);
        memcpy(r->array, array, n);
        r->array[n] = 0;
    }
    if (ntasks > 0) r->ntasks = ntasks;
    if (r->nodes == 0) r->nodes = 1;
    if (r->cpus_per_task == 0) r->cpus_per_task = 1;
    if (r->mem_per_cpu == 0) r->mem_per_cpu = 1024;
}

int64_t fit_array_len(const char* array) {  // parse.go:126-135
    if (!array) return 0;
    const sv a(array);
    if (a.find('-') != sv::npos) {
        const std::vector<sv> s = split(a, "-");
        return (int64_t)((uint64_t)atoi_go(s[1]) - (uint64_t)atoi_go(s[0]) + 1);
    }
    return (int64_t)split(a, ",").size();
}

void fit_pod_request(const fit_job_resources* r, int64_t* cpu, int64_t* memory) {  // :143-162
    if (!r || !cpu || !memory) return;
    uint64_t n;
    if (r->ntasks > 0)
        n = (uint64_t)r->cpus_per_task * (uint64_t)r->ntasks;
    else if (r->ntasks_per_node > 0 && r->nodes > 0)
        n = (uint64_t)r->cpus_per_task * (uint64_t)r->ntasks_per_node * (uint64_t)r->nodes;
    else
        n = (uint64_t)r->cpus_per_task;
    if (r->array[0]) n *= (uint64_t)fit_array_len(r->array);
    *cpu = (int64_t)n;
    *memory = (int64_t)(n * (uint64_t)r->mem_per_cpu * 1024u);
}

int fit_job_demand(const fit_job_resources* r, int32_t* cpu, int32_t* mem_mib, int32_t* wall_min,
                   uint16_t* nodes_k) {
    // DESIGN.md §2 "demand": per-node cpus = cpusPerTask × tasks per node, where tasks per node =
    // ntasksPerNode, else ceil(ntasks / nodes), else 1; mem = cpus × memPerCpu (MiB, Slurm's
    // --mem-per-cpu unit); walltime rounded up to whole minutes; nodes = --nodes (min).
    if (!r || !cpu || !mem_mib || !wall_min || !nodes_k) return FIT_E_INVAL;
    const int64_t k = r->nodes > 0 ? r->nodes : 1;
    int64_t tpn = 1;
    if (r->ntasks_per_node > 0) tpn = r->ntasks_per_node;
    else if (r->ntasks > 0) tpn = r->ntasks / k + (r->ntasks % k != 0);  // no overflow at INT64_MAX
    const int64_t cpt = r->cpus_per_task > 0 ? r->cpus_per_task : 1;
    const int64_t mpc = r->mem_per_cpu > 0 ? r->mem_per_cpu : 1024;
    if (k > 65535 || tpn > INT32_MAX || cpt > INT32_MAX || tpn * cpt > INT32_MAX ||
        mpc > INT32_MAX || tpn * cpt * mpc > INT32_MAX || r->wall_ns < 0)
        return FIT_E_INVAL;
    const int64_t w = (r->wall_ns + 59999999999ll) / 60000000000ll;
    if (w > INT32_MAX) return FIT_E_INVAL;
    *cpu = (int32_t)(tpn * cpt);
    *mem_mib = (int32_t)(tpn * cpt * mpc);
    *wall_min = (int32_t)w;
    *nodes_k = (uint16_t)k;
    return FIT_OK;
}

void fit_partition_capacity(const fit_node* nodes, int32_t n, int64_t* cpu, int64_t* memory,
                            int64_t* gpu, int64_t* pods) {  // node.go:169-199
    uint64_t c = 0, m = 0, g = 0;
    for (int32_t i = 0; nodes && i < n; ++i) {
        c += (uint64_t)nodes[i].cpus;
        m += (uint64_t)nodes[i].memory;
        g += (uint64_t)nodes[i].gpus;
    }
    if (cpu) *cpu = (int64_t)c;
    if (memory) *memory = (int64_t)(m * (2u << 10));  // node.go:193 — MiB × 2048, as the ref
    if (gpu) *gpu = (int64_t)g;
    if (pods) *pods = (int64_t)c;  // node.go:197
}

// ---------------------------------------------------------------- node-table ingest (f3)
// the Client.Nodes record loop + parseNode (slurm.go:354-363, parse.go:291-308)
// extended with the fields the reference drops — NodeName, Gres / GresUsed (a1: Gpus and AlloGpus
// are never set there), State and Partitions — straight into the engine's SoA columns, and Slurm
// hostlist expansion (a3: parsePartition splits "node[1-3,5]" into "node[1-3" and "5]").

}  // extern "C"

namespace {

// Split on `sep` outside parentheses / brackets ("gpu:4(S:0,1),mps:100" → 2 items).
std::vector<sv> split_top(sv s, char sep) {
    std::vector<sv> out;
    int depth = 0;
    size_t b = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        const char ch = s[i];
        if (ch == '(' || ch == '[') ++depth;
        else if ((ch == ')' || ch == ']') && depth > 0) --depth;
        else if (ch == sep && depth == 0) {
            out.push_back(s.substr(b, i - b));
            b = i + 1;
        }
    }
    out.push_back(s.substr(b));
    return out;
}

// Σ of the counts of "gpu" entries of a Gres / GresUsed value: name[:type]:count[(...)], count
// with an optional K/M/G multiplier (Slurm's suffixes), "(null)" = none.  -1: malformed count.
int64_t gres_gpus(sv v) {
    int64_t total = 0;
    for (sv item : split_top(v, ',')) {
        const size_t paren = item.find('(');
        if (paren != sv::npos) item = item.substr(0, paren);
        if (item.substr(0, 3) != "gpu" || (item.size() > 3 && item[3] != ':')) continue;
        const std::vector<sv> parts = split(item, ":");
        if (parts.size() < 2) {  // bare "gpu": one
            total += 1;
            continue;
        }
        sv cnt = parts.back();
        int64_t mul = 1;
        if (!cnt.empty() && (cnt.back() == 'K' || cnt.back() == 'M' || cnt.back() == 'G')) {
            mul = cnt.back() == 'K' ? 1024 : cnt.back() == 'M' ? 1024 * 1024 : 1024 * 1024 * 1024;
            cnt.remove_suffix(1);
        }
        int64_t c;
        if (parse_int(cnt, c) != 0) {
            if (parts.size() == 2) {  // "gpu:a100" (type, no count): one
                total += 1;
                continue;
            }
            return -1;
        }
        total += c * mul;
    }
    return total;
}

// A node takes new work unless a State token says otherwise (DOWN*, IDLE+DRAIN, ...); the flags
// follow `scontrol show node` (base state + '+'-joined flags, '*' = not responding).  The short
// suffixes of sinfo-style states stand for the same flags as their long '+' forms, so IDLE~ and
// IDLE+POWERED_DOWN decide alike: ~ POWERED_DOWN, % POWERING_DOWN, ! POWER_DOWN (pending),
// $ MAINT, @ REBOOT_REQUESTED, ^ REBOOT_ISSUED refuse new work; # POWERING_UP and - PLANNED
// do not.
bool state_schedulable(sv v) {
    if (v.empty()) return true;
    if (v.find('*') != sv::npos) return false;  // not responding
    for (sv tok : split(v, "+")) {
        while (!tok.empty() && strchr("~#!%$@^-", tok.back())) {
            if (strchr("~!%$@^", tok.back())) return false;
            tok.remove_suffix(1);
        }
        static const char* const bad[] = {"DOWN",     "DRAIN",         "DRAINED",      "DRAINING",
                                          "FAIL",     "FAILING",       "FUTURE",       "MAINT",
                                          "POWERED_DOWN", "POWER_DOWN", "POWERING_DOWN",
                                          "REBOOT_ISSUED", "REBOOT_REQUESTED", "INVAL", "UNKNOWN",
                                          "NOT_RESPONDING"};
        for (const char* b : bad)
            if (tok == b) return false;
    }
    return true;
}

int32_t to_i32(int64_t v) {
    return v > INT32_MAX ? INT32_MAX : v < INT32_MIN ? INT32_MIN : (int32_t)v;
}

// One bracket group "01-03,7" → the numbers as strings, zero padded to the width of the lower
// bound when it has a leading zero (Slurm hostlist).  false: malformed.
bool expand_ranges(sv body, std::vector<std::string>& out) {
    for (sv r : split(body, ",")) {
        const size_t dash = r.find('-');
        sv lo = dash == sv::npos ? r : r.substr(0, dash), hi = dash == sv::npos ? r : r.substr(dash + 1);
        int64_t a, b;
        if (lo.empty() || hi.empty() || lo[0] == '-' || lo[0] == '+' || hi[0] == '-' || hi[0] == '+' ||
            parse_int(lo, a) || parse_int(hi, b) || b < a || b - a > 1000000)
            return false;
        const size_t width = (lo.size() > 1 && lo[0] == '0') ? lo.size() : 0;
        for (int64_t x = a; x <= b; ++x) {
            std::string d = std::to_string(x);
            if (d.size() < width) d.insert(0, width - d.size(), '0');
            out.push_back(std::move(d));
        }
    }
    return true;
}

// One hostlist item (no top-level comma): prefix[r]mid[r]...suffix → cartesian expansion.
bool expand_item(sv item, std::vector<std::string>& out) {
    std::vector<std::string> acc{std::string()};
    size_t i = 0;
    while (i < item.size()) {
        const size_t lb = item.find('[', i);
        if (lb == sv::npos) {
            for (auto& a : acc) a.append(item.substr(i));
            break;
        }
        const size_t rb = item.find(']', lb);
        if (rb == sv::npos) return false;
        for (auto& a : acc) a.append(item.substr(i, lb - i));
        std::vector<std::string> nums;
        if (!expand_ranges(item.substr(lb + 1, rb - lb - 1), nums)) return false;
        std::vector<std::string> next;
        next.reserve(acc.size() * nums.size());
        for (auto& a : acc)
            for (auto& n : nums) next.push_back(a + n);
        acc.swap(next);
        i = rb + 1;
    }
    for (auto& a : acc)
        if (!a.empty()) out.push_back(std::move(a));
    return true;
}

}  // namespace

extern "C" {

int fit_expand_hostlist(const char* expr, char* buf, int32_t buflen) {
    if (!expr || !buf || buflen < 0) return FIT_E_INVAL;
    std::vector<std::string> names;
    for (sv item : split_top(trim_space(sv(expr)), ','))
        if (!item.empty() && !expand_item(item, names)) return FIT_E_PARSE;
    std::vector<sv> views(names.begin(), names.end());
    return put_names(views, buf, buflen);
}

int fit_node_names(const char* entries, int32_t n, char* buf, int32_t buflen) {
    if (n < 0 || (n > 0 && !entries) || !buf || buflen < 0) return FIT_E_INVAL;
    // parsePartition split the Nodes= value on every comma (parse.go:278-289): joining the pieces
    // with commas gives the value back, and the hostlist parser splits it at top-level commas only
    std::string joined;
    const char* p = entries;
    for (int32_t i = 0; i < n; ++i, p += strlen(p) + 1) {
        if (i) joined += ',';
        joined += p;
    }
    std::vector<std::string> names;
    for (sv item : split_top(trim_space(sv(joined)), ','))
        if (!item.empty() && !expand_item(item, names)) return FIT_E_PARSE;
    // one engine row per name: a name listed twice would give `scontrol show nodes` a record count
    // the table cannot be matched against
    std::vector<sv> views(names.begin(), names.end());
    std::vector<sv> sorted(views);
    std::sort(sorted.begin(), sorted.end());
    // (FIT_E_PARSE, not FIT_E_INVAL: callers grow the buffer on FIT_E_INVAL and must not retry this)
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) return FIT_E_PARSE;
    return put_names(views, buf, buflen);
}

int fit_ingest_nodes(const char* text, const char* partitions, int32_t np, int32_t cap,
                     int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free, int32_t* avail_min,
                     uint32_t* part_mask, char* names, int32_t names_len) {
    if (!text || cap < 0 || np < 0 || np > FIT_MAX_PARTITIONS || (np > 0 && !partitions) ||
        (cap > 0 && (!cpu_free || !mem_free || !gpu_free || !avail_min || !part_mask)))
        return FIT_E_INVAL;
    std::vector<sv> pnames;
    for (const char* p = partitions; (int32_t)pnames.size() < np; p += strlen(p) + 1) pnames.push_back(p);
    std::vector<sv> node_names;
    int32_t n = 0;
    for (sv rec : split(trim_space(sv(text)), "\n\n")) {  // Client.Nodes, slurm.go:354-363
        if (rec.empty()) continue;
        if (n == cap) return FIT_E_INVAL;
        fit_node base;
        parse_node(rec, base);  // CPUTot / CPUAlloc / RealMemory / AllocMem exactly as parseNode
        sv name, state;
        int64_t gpus = 0, used = 0;
        uint32_t mask = 0;
        for (sv f : fields(rec)) {
            const std::vector<sv> kv = split(f, "=");
            if (kv.size() != 2) continue;  // same key rule as parseNode (parse.go:294)
            if (kv[0] == "NodeName") name = kv[1];
            else if (kv[0] == "State") state = kv[1];
            else if (kv[0] == "Gres" || kv[0] == "GresUsed") {
                const int64_t g = gres_gpus(kv[1]);
                if (g < 0) return FIT_E_PARSE;
                (kv[0] == "Gres" ? gpus : used) = g;
            } else if (kv[0] == "Partitions") {
                for (sv pn : split(kv[1], ","))
                    for (int32_t p = 0; p < np; ++p)
                        if (pnames[p] == pn) mask |= 1u << p;
            }
        }
        cpu_free[n] = to_i32(base.cpus - base.allo_cpus);
        mem_free[n] = to_i32(base.memory - base.allo_memory);
        gpu_free[n] = to_i32(gpus - used);
        avail_min[n] = INT32_MAX;  // no horizon in `scontrol show nodes`; reservations set it
        part_mask[n] = state_schedulable(state) ? mask : 0u;
        node_names.push_back(name);
        ++n;
    }
    if (names) {
        const int rc = put_names(node_names, names, names_len);
        if (rc < 0) return rc;
    }
    return n;
}

}  // extern "C"

// ------------------------------------------------------------- CreatePod call site (a10)
// What CreatePod (pkg/slurm-virtual-kubelet/provider.go:35-60) holds — the pod's labels and its
// script — turned into engine requests, and the engine's decision written back into the script
// (include/fitgpu.h "CreatePod call site").  The Go side passes strings through; every rule
// lives here, where the tests reach it.

namespace {

// Slurm --array item "a", "a-b" or "a-b:s" → its ids into `ids` (a bitmap over task ids)
bool array_item(sv it, std::vector<bool>& ids) {
    constexpr int64_t MAX_ID = (1 << 22) - 1;
    sv range = it, step;
    const size_t colon = it.find(':');
    if (colon != sv::npos) {
        range = it.substr(0, colon);
        step = it.substr(colon + 1);
    }
    const size_t dash = range.find('-');
    sv lo = dash == sv::npos ? range : range.substr(0, dash);
    sv hi = dash == sv::npos ? range : range.substr(dash + 1);
    int64_t a, b, s = 1;
    auto digits = [](sv x) { return !x.empty() && x.find_first_not_of("0123456789") == sv::npos; };
    if (!digits(lo) || !digits(hi) || parse_int(lo, a) || parse_int(hi, b) || b < a || b > MAX_ID)
        return false;
    if (colon != sv::npos && (dash == sv::npos || !digits(step) || parse_int(step, s) || s < 1))
        return false;
    if ((int64_t)ids.size() <= b) ids.resize((size_t)b + 1, false);
    for (int64_t x = a; x <= b; x += s) ids[(size_t)x] = true;
    return true;
}

}  // namespace

namespace fitgpu {

// The script with `#SBATCH --nodelist=<names>` as the last line of its #SBATCH header
// (fit_script_with_nodelist, fit_admitter_script).  Length written, or FIT_E_INVAL (out too small).
int script_with_names(const char* script, const std::vector<std::string_view>& names, char* out,
                      int32_t outlen) {
    std::string dir = "#SBATCH --nodelist=";
    for (size_t i = 0; i < names.size(); ++i) {
        if (i) dir += ',';
        dir.append(names[i]);
    }
    dir += '\n';
    // the header: the leading lines extractBatchResourcesFromScript walks (parse.go:36-52) —
    // empty lines, "#!" lines and "#SBATCH" lines; the directive goes after its last #SBATCH
    // line (or the shebang / nothing when there is none)
    const sv s(script);
    size_t pos = 0, ins = 0;
    bool seen_sbatch = false;
    while (pos < s.size()) {
        const size_t nl = s.find('\n', pos);
        const size_t end = nl == sv::npos ? s.size() : nl + 1;
        sv line = s.substr(pos, (nl == sv::npos ? s.size() : nl) - pos);
        if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
        if (line.substr(0, 7) == "#SBATCH") {
            seen_sbatch = true;
            ins = end;
        } else if (line.empty() || line.substr(0, 2) == "#!") {
            if (!seen_sbatch && line.substr(0, 2) == "#!") ins = end;
        } else {
            break;
        }
        pos = end;
    }
    std::string res;
    res.reserve(s.size() + dir.size() + 1);
    res.append(s.substr(0, ins));
    if (ins > 0 && s[ins - 1] != '\n') res += '\n';  // a header that ends without a newline
    res += dir;
    res.append(s.substr(ins));
    if (!out || (int64_t)res.size() + 1 > outlen) return FIT_E_INVAL;
    memcpy(out, res.data(), res.size());
    out[res.size()] = 0;
    return (int)res.size();
}

}  // namespace fitgpu

namespace {

// a label value as newSubmitRequestForPod reads it: strconv.ParseInt(v, 10, 64), skipped on error
int64_t label_int(const char* v) {
    if (!v) return 0;
    int64_t x;
    return parse_int(sv(v), x) == 0 ? x : 0;
}

// Slurm's MaxArraySize (slurm.conf; default 1001): task ids run 0 .. MaxArraySize - 1, and sbatch
// refuses an --array with a larger id before the job exists
std::atomic<int32_t> g_max_array_size{1001};

// fit_array_tasks plus the largest task id
int array_parse(const char* array, int64_t* tasks, int64_t* max_running, int64_t* max_id) {
    sv a = trim_space(sv(array));
    int64_t limit = INT64_MAX;
    const size_t pct = a.find('%');
    if (pct != sv::npos) {
        const sv l = a.substr(pct + 1);
        if (l.empty() || l.find_first_not_of("0123456789") != sv::npos || parse_int(l, limit) ||
            limit < 1)
            return FIT_E_PARSE;
        a = a.substr(0, pct);
    }
    if (a.empty()) return FIT_E_PARSE;
    std::vector<bool> ids;
    for (sv it : split(a, ","))
        if (!array_item(it, ids)) return FIT_E_PARSE;
    int64_t n = 0, last = -1;
    for (size_t x = 0; x < ids.size(); ++x)
        if (ids[x]) ++n, last = (int64_t)x;
    *tasks = n;
    *max_running = n < limit ? n : limit;
    // the largest id a step actually reaches (`0-1001:3` ends at 999), not the range's bound
    *max_id = last;
    return FIT_OK;
}

}  // namespace

extern "C" {

int fit_array_tasks(const char* array, int64_t* tasks, int64_t* max_running) {
    if (!array || !tasks || !max_running) return FIT_E_INVAL;
    int64_t max_id;
    return array_parse(array, tasks, max_running, &max_id);
}

int32_t fit_set_max_array_size(int32_t n) {
    if (n < 1 || n > (1 << 22)) return FIT_E_INVAL;
    return g_max_array_size.exchange(n);
}

// Does the script ask sbatch for an array (--array[=v] / -a v / -av)?  extractBatchResourcesFromScript
// ignores it, but sbatch honours it: the pod is then an array job and is never pinned.  sbatch reads
// #SBATCH directives up to the first line that is neither blank nor a comment, so a plain '#'
// comment does not end them here (extractBatchResourcesFromScript, pkg/slurm-bridge-operator/
// parse.go:36-46, stops at the first non-#SBATCH line; for the demand the engine follows it, for
// this flag it follows sbatch — a missed array would be pinned with --nodelist).
static bool script_has_array(const char* script) {
    for (const char* p = script; p && *p;) {
        const char* e = strchr(p, '\n');
        const sv line(p, e ? (size_t)(e - p) : strlen(p));
        p = e ? e + 1 : nullptr;
        size_t b = 0;
        while (b < line.size() && isspace((unsigned char)line[b])) ++b;
        if (b == line.size()) continue;  // blank
        if (line[b] != '#') break;       // the first command: sbatch reads no further directive
        if (line.substr(0, 7) != "#SBATCH") continue;  // the shebang, a plain comment
        size_t i = 7;
        while (i < line.size()) {
            while (i < line.size() && isspace((unsigned char)line[i])) ++i;
            size_t j = i;
            while (j < line.size() && !isspace((unsigned char)line[j])) ++j;
            const sv tok = line.substr(i, j - i);
            if (tok == "--array" || tok.substr(0, 8) == "--array=" || tok.substr(0, 2) == "-a") return true;
            i = j;
        }
    }
    return false;
}

int fit_pod_demand(const fit_pod_labels* labels, const char* script, uint16_t part,
                   int64_t priority, fit_admit_req* out, int32_t cap) {
    if (cap < 0 || (cap > 0 && !out)) return FIT_E_INVAL;
    fit_pod_labels none{};
    const fit_pod_labels& L = labels ? *labels : none;
    fit_job_resources r{};
    if (script) {
        const int rc = fit_extract_batch_resources(script, &r);  // parse.go:30-69
        if (rc) return rc;
    }
    // the labels reach sbatch as command-line flags, which override the #SBATCH lines; the array
    // is counted from the full label (fit_apply_spec keeps 63 characters of it)
    fit_apply_spec(&r, label_int(L.nodes), label_int(L.cpus_per_task), label_int(L.mem_per_cpu),
                   label_int(L.ntasks_per_node), nullptr, label_int(L.ntasks));
    int32_t cpu, mem, wall;
    uint16_t k;
    const int rc = fit_job_demand(&r, &cpu, &mem, &wall, &k);
    if (rc) return rc;
    if (k > FIT_MAX_K) return FIT_E_INVAL;
    int64_t tasks = 1, running = 1, max_id = 0;
    if (L.array && L.array[0]) {
        const int ra = array_parse(L.array, &tasks, &running, &max_id);
        if (ra) return ra;
    }
    // sbatch would refuse the array (ids >= MaxArraySize): no request, so one pod's label can
    // never turn into a batch of millions of tasks
    if (max_id >= g_max_array_size.load()) return FIT_E_INVAL;
    // an array job (label or #SBATCH --array): its tasks share one sbatch, never pinned
    const uint16_t fl = ((L.array && L.array[0]) || script_has_array(script)) ? FIT_REQ_ARRAY : 0;
    for (int64_t i = 0; i < running && i < cap; ++i)
        out[i] = fit_admit_req{priority, cpu, mem, 0, wall, part, k, fl, 0};
    return (int)running;
}

int fit_script_with_nodelist(const char* script, const char* names, int32_t n_names,
                             const int32_t* node, int32_t k, char* out, int32_t outlen) {
    if (!script || (n_names > 0 && !names) || n_names < 0 || k < 1 || k > FIT_MAX_K || !node ||
        !out || outlen < 1)
        return FIT_E_INVAL;
    std::vector<sv> nm;
    nm.reserve((size_t)n_names);
    for (const char* p = names; (int32_t)nm.size() < n_names; p += strlen(p) + 1) nm.push_back(p);
    std::vector<sv> picked;
    for (int32_t i = 0; i < k; ++i) {
        if (node[i] < 0 || node[i] >= n_names || nm[(size_t)node[i]].empty()) return FIT_E_INVAL;
        picked.push_back(nm[(size_t)node[i]]);
    }
    return fitgpu::script_with_names(script, picked, out, outlen);
}

int fit_partition_limits(int64_t wall_time_s, int64_t cpu_per_node, int64_t mem_per_node,
                         int32_t* max_time_min, int32_t* max_cpus_per_node,
                         int32_t* max_mem_per_node) {
    if (!max_time_min || !max_cpus_per_node || !max_mem_per_node) return FIT_E_INVAL;
    // ≤ 0: UNLIMITED (parseResources' -1, parse.go:128-187; a -1 ns walltime is 0 s after
    // api/slurm.go:309) or unset (0)
    auto lim = [](int64_t v) { return v <= 0 ? -1 : v > INT32_MAX ? INT32_MAX : (int32_t)v; };
    *max_time_min = wall_time_s <= 0 ? -1 : lim((wall_time_s + 59) / 60);
    *max_cpus_per_node = lim(cpu_per_node);
    *max_mem_per_node = lim(mem_per_node);
    return FIT_OK;
}

int fit_node_columns(const fit_node* nodes, int32_t n, uint32_t part_mask, int32_t* cpu_free,
                     int32_t* mem_free, int32_t* gpu_free, int32_t* avail_min, uint32_t* mask) {
    if (n < 0 || (n > 0 && (!nodes || !cpu_free || !mem_free || !gpu_free || !avail_min || !mask)))
        return FIT_E_INVAL;
    for (int32_t i = 0; i < n; ++i) {  // free = total − alloc (workload.proto:165-174)
        cpu_free[i] = to_i32(nodes[i].cpus - nodes[i].allo_cpus);
        mem_free[i] = to_i32(nodes[i].memory - nodes[i].allo_memory);
        gpu_free[i] = to_i32(nodes[i].gpus - nodes[i].allo_gpus);
        avail_min[i] = INT32_MAX;
        mask[i] = part_mask;
    }
    return n;
}

int fit_release_events(int32_t n, int32_t m, const int32_t* job_off, const int32_t* job_nodes,
                       const int64_t* rem_min, const int32_t* cpu, const int32_t* mem,
                       const int32_t* gpu, int32_t slots, int32_t slot_min, int32_t* rel_off,
                       int32_t* rel_slot, int32_t* rel_cpu, int32_t* rel_mem, int32_t* rel_gpu,
                       int32_t cap) {
    if (n < 0 || m < 0 || slots < 1 || slot_min < 1 || cap < 0 || !rel_off ||
        (m > 0 && (!job_off || !rem_min || !cpu || !mem || !gpu)))
        return FIT_E_INVAL;
    if (m > 0 && job_off[0] != 0) return FIT_E_INVAL;
    for (int32_t i = 0; i < m; ++i)
        if (job_off[i + 1] < job_off[i] || cpu[i] < 0 || mem[i] < 0 || gpu[i] < 0) return FIT_E_INVAL;
    const int32_t e = m > 0 ? job_off[m] : 0;
    if (e > 0 && !job_nodes) return FIT_E_INVAL;
    if (e > cap || (e > 0 && (!rel_slot || !rel_cpu || !rel_mem || !rel_gpu))) return FIT_E_INVAL;
    // one event per (job, node): node, slot, job — ordered by node, then slot, then job order
    struct Ev {
        int32_t node, slot, job;
    };
    std::vector<Ev> ev;
    ev.reserve((size_t)e);
    for (int32_t i = 0; i < m; ++i) {
        // minutes left → the slot whose start the release reaches: ceil(rem / slot_min), at least
        // 1 (a job past its end time holds its nodes until Slurm ends it), capped at the horizon
        const int64_t r = rem_min[i] <= 0 ? 1 : (rem_min[i] + slot_min - 1) / slot_min;
        const int32_t sl = (int32_t)std::min<int64_t>(std::max<int64_t>(r, 1), slots);
        for (int32_t k = job_off[i]; k < job_off[i + 1]; ++k) {
            const int32_t x = job_nodes[k];
            if (x < 0 || x >= n) return FIT_E_INVAL;
            ev.push_back(Ev{x, sl, i});
        }
    }
    std::stable_sort(ev.begin(), ev.end(), [](const Ev& a, const Ev& b) {
        return a.node != b.node ? a.node < b.node : a.slot < b.slot;
    });
    std::fill(rel_off, rel_off + n + 1, 0);
    for (const Ev& v : ev) ++rel_off[v.node + 1];
    for (int32_t x = 0; x < n; ++x) rel_off[x + 1] += rel_off[x];
    for (int32_t k = 0; k < e; ++k) {
        const Ev& v = ev[(size_t)k];
        rel_slot[k] = v.slot;
        rel_cpu[k] = cpu[v.job];
        rel_mem[k] = mem[v.job];
        rel_gpu[k] = gpu[v.job];
    }
    return e;
}

}  // extern "C"
