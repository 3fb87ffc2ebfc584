// simple_test.cpp — the reference's test/simple_test.cpp:13-229 against the MI355X
// engine: device present, raw device allocation, TransferManager pinned/device
// pools, and an IVF-Flat index (D=64, nlist=16, N=1000, Q=10, train on 100,
// nprobe=4, k=5, mt19937(42) data). Beyond the reference's range checks
// (simple_test.cpp:177-196) the results are compared bit for bit with the CPU
// oracle (oracle/cpu_ref.cpp, the reference CPU path restatement).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <iostream>
#include <random>
#include <vector>

#include "../../oracle/cpu_ref.h"
#include "vdb/ivf_flat_index.h"
#include "vdb/transfer_manager.h"

using namespace vdb;

static bool test_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        std::cerr << "no HIP device" << std::endl;
        return false;
    }
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    std::cout << "Device 0: " << p.name << " (" << p.gcnArchName << ") " << (p.totalGlobalMem >> 30) << " GB"
              << std::endl;
    return true;
}

static bool test_memory_allocation() {
    float* d = nullptr;
    if (hipMalloc(&d, 1024 * sizeof(float)) != hipSuccess) return false;
    (void)hipFree(d);
    std::cout << "device allocation: OK" << std::endl;
    return true;
}

static bool test_transfer_manager() {
    TransferManager::Config cfg;
    cfg.pinned_pool_size = 64 << 20;
    cfg.device_pool_size = 128 << 20;
    TransferManager tm(cfg);
    void* pin = tm.allocate_pinned(1024);
    void* dev = tm.allocate_device(1024);
    if (!pin || !dev) return false;
    std::memset(pin, 0x5A, 1024);
    void* back = tm.allocate_pinned(1024);
    tm.enqueue_transfer({pin, dev, 1024, TransferManager::CopyKind::HostToDevice, nullptr, nullptr});
    tm.synchronize();
    bool called = false;
    tm.enqueue_transfer({dev, back, 1024, TransferManager::CopyKind::DeviceToHost, nullptr, [&] { called = true; }});
    tm.synchronize();
    const bool same = std::memcmp(pin, back, 1024) == 0;
    const bool valid = TransferManager::validate_device_pointer(dev) && !TransferManager::validate_device_pointer(pin);
    tm.free_pinned(pin);
    tm.free_pinned(back);
    tm.free_device(dev);
    std::cout << "TransferManager: " << (same && called && valid ? "OK" : "FAILED") << std::endl;
    return same && called && valid;
}

static bool test_ivf_flat_index() {
    TransferManager::Config tcfg;
    tcfg.pinned_pool_size = 64 << 20;
    tcfg.device_pool_size = 128 << 20;
    TransferManager tm(tcfg);
    IVFFlatIndex::Config cfg;
    cfg.dimension = 64;
    cfg.nlist = 16;
    cfg.metric = kernels::Metric::L2;
    cfg.use_gpu = true;
    IVFFlatIndex index(cfg, &tm);

    const size_t n = 1000, nq = 10;
    std::vector<float> v(n * 64), q(nq * 64);
    std::vector<uint64_t> ids(n);
    std::mt19937 gen(42);
    std::normal_distribution<float> dist(0.0f, 1.0f);
    for (auto& x : v) x = dist(gen);
    for (auto& x : q) x = dist(gen);
    for (size_t i = 0; i < n; ++i) ids[i] = i;

    index.train(v.data(), 100);
    index.add(v.data(), ids.data(), n);
    const uint32_t k = 5;
    IVFFlatIndex::SearchParams params;
    params.nprobe = 4;
    params.k = k;
    std::vector<float> D(nq * k);
    std::vector<uint64_t> I(nq * k);
    index.search(q.data(), nq, params, D.data(), I.data());

    oracle_ivf* o = oracle_create(64, 16, 0);
    oracle_train(o, v.data(), 100);
    oracle_add(o, v.data(), ids.data(), n);
    std::vector<float> Dr(nq * k);
    std::vector<uint64_t> Ir(nq * k);
    oracle_search(o, q.data(), nq, 4, k, Dr.data(), Ir.data());
    oracle_destroy(o);

    bool valid = true, same = true;
    for (size_t i = 0; i < nq * k; ++i) {
        if (I[i] >= n && I[i] != UINT64_MAX) valid = false;
        if (I[i] != Ir[i] || std::memcmp(&D[i], &Dr[i], 4) != 0) same = false;
    }
    for (size_t qi = 0; qi < nq; ++qi) {
        std::cout << "Query " << qi << " results: ";
        for (uint32_t j = 0; j < k; ++j) std::cout << "(" << I[qi * k + j] << ", " << D[qi * k + j] << ") ";
        std::cout << std::endl;
    }
    std::cout << "IVF-Flat index: " << (valid && same ? "OK" : "FAILED") << " (bit-identical to CPU path: "
              << (same ? "yes" : "no") << "), total " << index.get_total_vectors() << ", GPU memory "
              << index.get_gpu_memory_usage() << " bytes" << std::endl;

    // save / load round trip
    const std::string path = "/tmp/vdb_simple_test.ivf";
    index.save(path);
    IVFFlatIndex again(cfg, &tm);
    again.load(path);
    std::vector<float> D2(nq * k);
    std::vector<uint64_t> I2(nq * k);
    again.search(q.data(), nq, params, D2.data(), I2.data());
    const bool rt = std::memcmp(D2.data(), D.data(), D.size() * 4) == 0 && I2 == I;
    std::cout << "save/load round trip: " << (rt ? "OK" : "FAILED") << std::endl;
    return valid && same && rt && index.get_total_vectors() == n;
}

int main() {
    bool ok = true;
    ok &= test_device();
    ok &= test_memory_allocation();
    ok &= test_transfer_manager();
    ok &= test_ivf_flat_index();
    std::cout << (ok ? "All tests PASSED" : "Some tests FAILED") << std::endl;
    return ok ? 0 : 1;
}
