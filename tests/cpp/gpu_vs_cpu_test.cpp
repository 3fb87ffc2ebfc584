// gpu_vs_cpu_test.cpp — the reference's test/gpu_vs_cpu_test.cpp:22-339 on MI355X.
// Same data (mt19937(12345) normal: database then queries, ids 0..N-1), same index
// protocol (train on min(N, 10000), add all, warm-up search of 10, timed search of
// Q; qps = Q*1000/ms). The "CPU" run is the oracle (the reference CPU path
// restatement, single-threaded); the "GPU" run is vdb::IVFFlatIndex. Unlike the
// reference (which only range-checks, gpu_vs_cpu_test.cpp:200-226) the two result
// sets must be bit-identical; exit status 1 otherwise.
// Usage: gpu_vs_cpu_test [N Q D nlist] (ctest: 10000 100 64 32).
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <random>
#include <string>
#include <vector>

#include "../../oracle/cpu_ref.h"
#include "vdb/ivf_flat_index.h"

using namespace vdb;
using clk = std::chrono::high_resolution_clock;

struct Result {
    double train_ms = 0, add_ms = 0, search_ms = 0, qps = 0;
    std::vector<float> D;
    std::vector<uint64_t> I;
};

static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

int main(int argc, char** argv) {
    size_t N = 50000, Q = 1000;
    uint32_t D = 128, nlist = 128, nprobe = 8, k = 10;
    if (argc > 1) N = std::stoul(argv[1]);
    if (argc > 2) Q = std::stoul(argv[2]);
    if (argc > 3) D = std::stoul(argv[3]);
    if (argc > 4) nlist = std::stoul(argv[4]);

    std::vector<float> v(N * D), q(Q * D);
    std::vector<uint64_t> ids(N);
    std::mt19937 gen(12345);
    std::normal_distribution<float> dist(0.0f, 1.0f);
    for (auto& x : v) x = dist(gen);
    for (auto& x : q) x = dist(gen);
    for (size_t i = 0; i < N; ++i) ids[i] = i;
    const size_t train = std::min<size_t>(N, 10000);
    std::cout << "Dataset: " << N << " x " << D << "D, queries " << Q << ", nlist " << nlist << ", nprobe " << nprobe
              << ", k " << k << std::endl;

    Result cpu, gpu;
    {  // CPU path (oracle)
        oracle_ivf* o = oracle_create(D, nlist, 0);
        auto t0 = clk::now();
        oracle_train(o, v.data(), train);
        auto t1 = clk::now();
        oracle_add(o, v.data(), ids.data(), N);
        auto t2 = clk::now();
        cpu.D.resize(Q * k);
        cpu.I.resize(Q * k);
        oracle_search(o, q.data(), std::min<size_t>(Q, 10), nprobe, k, cpu.D.data(), cpu.I.data());
        auto t3 = clk::now();
        oracle_search(o, q.data(), Q, nprobe, k, cpu.D.data(), cpu.I.data());
        auto t4 = clk::now();
        cpu.train_ms = ms(t0, t1);
        cpu.add_ms = ms(t1, t2);
        cpu.search_ms = ms(t3, t4);
        cpu.qps = Q * 1000.0 / cpu.search_ms;
        oracle_destroy(o);
    }
    {  // GPU path
        TransferManager::Config tcfg;
        tcfg.pinned_pool_size = 256 << 20;
        tcfg.device_pool_size = 512 << 20;
        TransferManager tm(tcfg);
        IVFFlatIndex::Config cfg;
        cfg.dimension = D;
        cfg.nlist = nlist;
        cfg.metric = kernels::Metric::L2;
        cfg.max_gpu_memory = 256 << 20;
        if (const char* d = std::getenv("VDB_TEST_DEVICES")) {  // e.g. "0,1": the index sharded over GPUs
            for (const char* p = d; *p;) {
                cfg.devices.push_back(std::atoi(p));
                while (*p && *p != ',') ++p;
                if (*p == ',') ++p;
            }
            std::cout << "GPU index sharded over " << cfg.devices.size() << " device(s): " << d << std::endl;
        }
        IVFFlatIndex index(cfg, &tm);
        auto t0 = clk::now();
        index.train(v.data(), train);
        auto t1 = clk::now();
        index.add(v.data(), ids.data(), N);
        auto t2 = clk::now();
        IVFFlatIndex::SearchParams p;
        p.nprobe = nprobe;
        p.k = k;
        gpu.D.resize(Q * k);
        gpu.I.resize(Q * k);
        index.search(q.data(), std::min<size_t>(Q, 10), p, gpu.D.data(), gpu.I.data());
        auto t3 = clk::now();
        index.search(q.data(), Q, p, gpu.D.data(), gpu.I.data());
        auto t4 = clk::now();
        gpu.train_ms = ms(t0, t1);
        gpu.add_ms = ms(t1, t2);
        gpu.search_ms = ms(t3, t4);
        gpu.qps = Q * 1000.0 / gpu.search_ms;
        std::cout << "GPU memory: " << index.get_gpu_memory_usage() / (1024 * 1024) << " MB" << std::endl;
    }
    size_t invalid = 0, diff = 0;
    for (size_t i = 0; i < Q * k; ++i) {
        if ((gpu.I[i] >= N && gpu.I[i] != UINT64_MAX) || !std::isfinite(gpu.D[i]) || gpu.D[i] < 0) ++invalid;
        if (gpu.I[i] != cpu.I[i] || std::memcmp(&gpu.D[i], &cpu.D[i], 4) != 0) ++diff;
    }
    std::cout << std::fixed << std::setprecision(2);
    std::cout << std::left << std::setw(14) << "Metric" << std::setw(14) << "CPU" << std::setw(14) << "GPU" << std::endl;
    std::cout << std::setw(14) << "Train (ms)" << std::setw(14) << cpu.train_ms << std::setw(14) << gpu.train_ms << std::endl;
    std::cout << std::setw(14) << "Add (ms)" << std::setw(14) << cpu.add_ms << std::setw(14) << gpu.add_ms << std::endl;
    std::cout << std::setw(14) << "Search (ms)" << std::setw(14) << cpu.search_ms << std::setw(14) << gpu.search_ms << std::endl;
    std::cout << std::setw(14) << "QPS" << std::setw(14) << cpu.qps << std::setw(14) << gpu.qps << std::endl;
    std::cout << "invalid results: " << invalid << ", results differing from the CPU path: " << diff << std::endl;
    return (invalid == 0 && diff == 0) ? 0 : 1;
}
