// admit_load — CreatePod admission load from native threads (bench.py --workload admit).
//
// The Go call site admits from 10 PodSyncWorker goroutines on OS threads
// (pkg/slurm-virtual-kubelet/options/options.go:107, provider.go:35-60); bench.py's Python callers
// share one interpreter lock, so their arrival pattern is the interpreter's, not the library's.
// This driver calls the C-ABI from C++ threads instead: C callers, each admitting `per` pods one
// after the other (the next as soon as the last returns), all through one fit_admitter.
//
//   admit_load <dir> <callers> <per> <max_batch> <max_wait_us>
//
// <dir> holds raw little-endian arrays written by bench.py: nodes.i32 (n × {cpu, mem, gpu,
// avail, mask}), parts.i32 (p × {max_time, max_cpus, max_mem}), jobs.i32 (j × {cpu, mem, gpu,
// wall, part, nodes_k}).  Prints one JSON object: per-pod latency p50 / p99 / max (µs), pods/s,
// batches.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "fitgpu.h"

namespace {

std::vector<int32_t> read_i32(const std::string& path) {
    std::vector<int32_t> v;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return v;
    int32_t x;
    while (fread(&x, sizeof x, 1, f) == 1) v.push_back(x);
    fclose(f);
    return v;
}

int die(const char* what, int rc) {
    fprintf(stderr, "admit_load: %s failed: %d %s\n", what, rc, fit_last_error());
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: admit_load <dir> <callers> <per> <max_batch> <max_wait_us>\n");
        return 2;
    }
    const std::string dir = argv[1];
    const int callers = atoi(argv[2]), per = atoi(argv[3]), max_batch = atoi(argv[4]), max_wait = atoi(argv[5]);
    const std::vector<int32_t> nd = read_i32(dir + "/nodes.i32"), pt = read_i32(dir + "/parts.i32"),
                               jb = read_i32(dir + "/jobs.i32");
    if (nd.empty() || nd.size() % 5 || pt.empty() || pt.size() % 3 || jb.size() % 6 ||
        jb.size() / 6 < (size_t)callers * per + 20) {
        fprintf(stderr, "admit_load: bad input files in %s\n", dir.c_str());
        return 2;
    }
    const int32_t n = (int32_t)(nd.size() / 5), p = (int32_t)(pt.size() / 3);
    std::vector<int32_t> cpu(n), mem(n), gpu(n), av(n), mt(p), mc(p), mm(p);
    std::vector<uint32_t> mask(n);
    for (int32_t i = 0; i < n; ++i) {
        cpu[i] = nd[5 * i], mem[i] = nd[5 * i + 1], gpu[i] = nd[5 * i + 2], av[i] = nd[5 * i + 3];
        mask[i] = (uint32_t)nd[5 * i + 4];
    }
    for (int32_t i = 0; i < p; ++i) mt[i] = pt[3 * i], mc[i] = pt[3 * i + 1], mm[i] = pt[3 * i + 2];
    auto req = [&](int64_t q) {
        fit_admit_req r{};
        r.priority = q;
        r.cpu = jb[6 * q], r.mem_mib = jb[6 * q + 1], r.gpu = jb[6 * q + 2], r.wall_min = jb[6 * q + 3];
        r.part = (uint16_t)jb[6 * q + 4], r.nodes_k = (uint16_t)jb[6 * q + 5];
        return r;
    };

    fit_opts o{};
    o.device = 0;
    o.world = 1;
    fit_ctx* ctx = nullptr;
    int rc = fit_create(&o, &ctx);
    if (rc) return die("fit_create", rc);
    if ((rc = fit_load_partitions(ctx, p, mt.data(), mc.data(), mm.data()))) return die("fit_load_partitions", rc);
    fit_admitter* a = nullptr;
    if ((rc = fit_admitter_create(ctx, max_batch, max_wait, &a))) return die("fit_admitter_create", rc);
    auto load = [&] {
        return fit_admitter_load_nodes(a, n, cpu.data(), mem.data(), gpu.data(), av.data(), mask.data());
    };
    if ((rc = load())) return die("fit_admitter_load_nodes", rc);
    const int64_t base = 20;  // warmup: the first launches, then the table again
    for (int64_t q = 0; q < base; ++q) {
        fit_admit_req r = req(q);
        fit_admit_res s;
        if ((rc = fit_admit(a, &r, &s))) return die("fit_admit (warmup)", rc);
    }
    if ((rc = load())) return die("fit_admitter_load_nodes", rc);

    std::vector<std::vector<double>> lat(callers);
    std::vector<std::vector<int64_t>> bat(callers);
    std::atomic<int> ready{0}, err{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int w = 0; w < callers; ++w) {
        th.emplace_back([&, w] {
            lat[w].reserve(per);
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (int i = 0; i < per; ++i) {
                const int64_t q = base + (int64_t)w * per + i;
                fit_admit_req r = req(q);
                fit_admit_res s;
                const auto t0 = std::chrono::steady_clock::now();
                if (fit_admit(a, &r, &s)) {
                    err.fetch_add(1);
                    return;
                }
                lat[w].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
                bat[w].push_back(s.batch);
            }
        });
    }
    while (ready.load() < callers) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    for (auto& t : th) t.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fit_admitter_destroy(a);
    fit_destroy(ctx);
    if (err.load()) {
        fprintf(stderr, "admit_load: %d callers failed: %s\n", err.load(), fit_last_error());
        return 1;
    }
    std::vector<double> all;
    std::set<int64_t> batches;
    for (int w = 0; w < callers; ++w) {
        all.insert(all.end(), lat[w].begin(), lat[w].end());
        batches.insert(bat[w].begin(), bat[w].end());
    }
    std::sort(all.begin(), all.end());
    auto pct = [&](double f) { return all[std::min(all.size() - 1, (size_t)(f * (all.size() - 1) + 0.5))]; };
    printf("{\"pods_per_s\": %.1f, \"p50_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f, \"batches\": %zu, "
           "\"pods_per_batch\": %.2f, \"nodes\": %d, \"partitions\": %d, \"callers\": %d}\n",
           all.size() / el, pct(0.50), pct(0.99), all.back(), batches.size(),
           (double)all.size() / std::max<size_t>(batches.size(), 1), n, p, callers);
    return 0;
}
