// vdb/transfer_manager.h — drop-in for the reference's engine/transfer_manager.h:21-164.
//
// Same public surface (Config, Transfer, allocate_/free_ pinned and device memory,
// a stream pool, enqueue_transfer / enqueue_batch, synchronize, memory stats), rebuilt
// for MI355X: device memory comes from a HIP stream-ordered memory pool
// (hipMallocAsync) whose release threshold is the configured device pool size, pinned
// memory from a size-class free list over hipHostMalloc, and streams are non-blocking
// HIP streams. Streams and copy kinds are opaque here (void*, CopyKind), so including
// this header needs no device headers; the reference's cudaStream_t / cudaMemcpyKind
// map onto them one-to-one.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

namespace vdb {

class TransferManager {
public:
    struct Config {
        size_t pinned_pool_size = 1ULL << 30;  // transfer_manager.h:25
        size_t device_pool_size = 4ULL << 30;  // transfer_manager.h:26
        int num_streams = 4;                   // transfer_manager.h:27
        bool use_async = true;                 // transfer_manager.h:28
        int device = 0;
    };

    enum class CopyKind { HostToHost = 0, HostToDevice = 1, DeviceToHost = 2, DeviceToDevice = 3, Default = 4 };

    struct Transfer {
        void* src;
        void* dst;
        size_t size;
        CopyKind kind;
        void* stream;                    // hipStream_t; nullptr = a pool stream
        std::function<void()> callback;  // runs on a runtime thread when the copy is done
    };

    struct MemoryStats {
        size_t total_device_allocated = 0;
        size_t total_pinned_allocated = 0;
        size_t active_allocations = 0;
        size_t peak_device_usage = 0;
        size_t peak_pinned_usage = 0;
    };

    explicit TransferManager(const Config& config);
    ~TransferManager();
    TransferManager(const TransferManager&) = delete;
    TransferManager& operator=(const TransferManager&) = delete;

    void* allocate_pinned(size_t size);
    void free_pinned(void* ptr);
    void* allocate_device(size_t size);
    void free_device(void* ptr);

    void* get_stream();
    void return_stream(void* stream);

    void enqueue_transfer(const Transfer& transfer);
    void enqueue_batch(const std::vector<Transfer>& transfers);
    void synchronize();
    void synchronize_stream(void* stream);
    size_t get_pending_transfers() const { return pending_.load(); }

    MemoryStats get_memory_stats() const;
    static bool validate_device_pointer(void* ptr);
    const Config& config() const { return config_; }

private:
    struct Impl;
    Config config_;
    std::unique_ptr<Impl> impl_;
    std::atomic<size_t> pending_{0};
};

}  // namespace vdb
