// transfer_manager.cpp — MI355X TransferManager (include/vdb/transfer_manager.h).
//
// Replaces the reference's first-fit block pools (engine/transfer_manager.cpp:12-162)
// with HIP's stream-ordered allocator: one hipMemPool per manager whose release
// threshold is Config::device_pool_size, so freed blocks stay cached on the device
// up to that size and are reused without a driver round trip. Pinned host memory
// is kept in power-of-two size classes (cached up to Config::pinned_pool_size).
// Copies are hipMemcpyAsync on a pool stream or the caller's; completion callbacks
// and the pending counter ride on hipLaunchHostFunc (transfer_manager.cpp:231-261).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "vdb/transfer_manager.h"

namespace vdb {

namespace {
void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
size_t size_class(size_t n) {
    size_t c = 4096;
    while (c < n) c <<= 1;
    return c;
}
hipMemcpyKind to_hip(TransferManager::CopyKind k) {
    switch (k) {
        case TransferManager::CopyKind::HostToHost: return hipMemcpyHostToHost;
        case TransferManager::CopyKind::HostToDevice: return hipMemcpyHostToDevice;
        case TransferManager::CopyKind::DeviceToHost: return hipMemcpyDeviceToHost;
        case TransferManager::CopyKind::DeviceToDevice: return hipMemcpyDeviceToDevice;
        default: return hipMemcpyDefault;
    }
}
}  // namespace

struct TransferManager::Impl {
    int device = 0;
    hipMemPool_t pool = nullptr;
    hipStream_t alloc_stream = nullptr;
    mutable std::mutex mu;
    std::unordered_map<void*, size_t> device_allocs, pinned_allocs;
    std::unordered_map<size_t, std::vector<void*>> pinned_free;
    size_t pinned_cached = 0;
    size_t dev_used = 0, pin_used = 0, dev_peak = 0, pin_peak = 0;
    std::vector<hipStream_t> streams;
    std::queue<hipStream_t> avail;
    std::mutex smu;
    std::condition_variable scv;
    size_t rr = 0;
};

struct HostCallback {
    std::function<void()> fn;
    std::atomic<size_t>* pending;
};

static void run_callback(void* p) {
    auto* cb = static_cast<HostCallback*>(p);
    if (cb->fn) cb->fn();
    cb->pending->fetch_sub(1);
    delete cb;
}

TransferManager::TransferManager(const Config& config) : config_(config), impl_(new Impl()) {
    impl_->device = config.device;
    hip_ok(hipSetDevice(config.device), "hipSetDevice");
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = config.device;
    hip_ok(hipMemPoolCreate(&impl_->pool, &props), "hipMemPoolCreate");
    uint64_t threshold = config.device_pool_size;
    hip_ok(hipMemPoolSetAttribute(impl_->pool, hipMemPoolAttrReleaseThreshold, &threshold), "pool threshold");
    hip_ok(hipStreamCreateWithFlags(&impl_->alloc_stream, hipStreamNonBlocking), "hipStreamCreate");
    for (int i = 0; i < std::max(1, config.num_streams); ++i) {
        hipStream_t s;
        hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
        impl_->streams.push_back(s);
        impl_->avail.push(s);
    }
}

TransferManager::~TransferManager() {
    (void)hipSetDevice(impl_->device);
    (void)hipDeviceSynchronize();
    for (auto& kv : impl_->device_allocs) (void)hipFreeAsync(kv.first, impl_->alloc_stream);
    (void)hipStreamSynchronize(impl_->alloc_stream);
    for (auto& kv : impl_->pinned_allocs) (void)hipHostFree(kv.first);
    for (auto& kv : impl_->pinned_free)
        for (void* p : kv.second) (void)hipHostFree(p);
    for (hipStream_t s : impl_->streams) (void)hipStreamDestroy(s);
    (void)hipStreamDestroy(impl_->alloc_stream);
    (void)hipMemPoolDestroy(impl_->pool);
}

void* TransferManager::allocate_pinned(size_t size) {
    const size_t c = size_class(std::max<size_t>(size, 1));
    std::lock_guard<std::mutex> g(impl_->mu);
    void* p = nullptr;
    auto& fl = impl_->pinned_free[c];
    if (!fl.empty()) {
        p = fl.back();
        fl.pop_back();
        impl_->pinned_cached -= c;
    } else if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
        return nullptr;
    }
    impl_->pinned_allocs[p] = c;
    impl_->pin_used += c;
    impl_->pin_peak = std::max(impl_->pin_peak, impl_->pin_used);
    return p;
}

void TransferManager::free_pinned(void* ptr) {
    if (!ptr) return;
    std::lock_guard<std::mutex> g(impl_->mu);
    auto it = impl_->pinned_allocs.find(ptr);
    if (it == impl_->pinned_allocs.end()) return;
    const size_t c = it->second;
    impl_->pinned_allocs.erase(it);
    impl_->pin_used -= c;
    if (impl_->pinned_cached + c <= config_.pinned_pool_size) {
        impl_->pinned_free[c].push_back(ptr);
        impl_->pinned_cached += c;
    } else {
        (void)hipHostFree(ptr);
    }
}

void* TransferManager::allocate_device(size_t size) {
    std::lock_guard<std::mutex> g(impl_->mu);
    void* p = nullptr;
    if (hipSetDevice(impl_->device) != hipSuccess) return nullptr;
    if (hipMallocFromPoolAsync(&p, std::max<size_t>(size, 1), impl_->pool, impl_->alloc_stream) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    // Make the block usable from any stream right away (the reference's pool hands
    // out memory synchronously).
    if (hipStreamSynchronize(impl_->alloc_stream) != hipSuccess) return nullptr;
    impl_->device_allocs[p] = size;
    impl_->dev_used += size;
    impl_->dev_peak = std::max(impl_->dev_peak, impl_->dev_used);
    return p;
}

void TransferManager::free_device(void* ptr) {
    if (!ptr) return;
    std::lock_guard<std::mutex> g(impl_->mu);
    auto it = impl_->device_allocs.find(ptr);
    if (it == impl_->device_allocs.end()) return;
    impl_->dev_used -= it->second;
    impl_->device_allocs.erase(it);
    (void)hipSetDevice(impl_->device);
    // Work already queued on other streams may still read the block.
    (void)hipDeviceSynchronize();
    (void)hipFreeAsync(ptr, impl_->alloc_stream);
}

void* TransferManager::get_stream() {
    std::unique_lock<std::mutex> lk(impl_->smu);
    impl_->scv.wait(lk, [&] { return !impl_->avail.empty(); });
    hipStream_t s = impl_->avail.front();
    impl_->avail.pop();
    return s;
}

void TransferManager::return_stream(void* stream) {
    {
        std::lock_guard<std::mutex> lk(impl_->smu);
        impl_->avail.push(static_cast<hipStream_t>(stream));
    }
    impl_->scv.notify_one();
}

void TransferManager::enqueue_transfer(const Transfer& t) {
    hip_ok(hipSetDevice(impl_->device), "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(t.stream);
    if (!s) {
        std::lock_guard<std::mutex> lk(impl_->smu);
        s = impl_->streams[impl_->rr++ % impl_->streams.size()];
    }
    if (!config_.use_async) {
        hip_ok(hipMemcpy(t.dst, t.src, t.size, to_hip(t.kind)), "hipMemcpy");
        if (t.callback) t.callback();
        return;
    }
    hip_ok(hipMemcpyAsync(t.dst, t.src, t.size, to_hip(t.kind), s), "hipMemcpyAsync");
    pending_.fetch_add(1);
    auto* cb = new HostCallback{t.callback, &pending_};
    hipError_t e = hipLaunchHostFunc(s, run_callback, cb);
    if (e != hipSuccess) {
        delete cb;
        pending_.fetch_sub(1);
        hip_ok(e, "hipLaunchHostFunc");
    }
}

void TransferManager::enqueue_batch(const std::vector<Transfer>& transfers) {
    for (const Transfer& t : transfers) enqueue_transfer(t);
}

void TransferManager::synchronize() {
    hip_ok(hipSetDevice(impl_->device), "hipSetDevice");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    while (pending_.load() != 0) {
    }  // host callbacks finish right after the device work they follow
}

void TransferManager::synchronize_stream(void* stream) {
    hip_ok(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
}

TransferManager::MemoryStats TransferManager::get_memory_stats() const {
    std::lock_guard<std::mutex> g(impl_->mu);
    MemoryStats m;
    m.total_device_allocated = impl_->dev_used;
    m.total_pinned_allocated = impl_->pin_used;
    m.active_allocations = impl_->device_allocs.size() + impl_->pinned_allocs.size();
    m.peak_device_usage = impl_->dev_peak;
    m.peak_pinned_usage = impl_->pin_peak;
    return m;
}

bool TransferManager::validate_device_pointer(void* ptr) {
    if (!ptr) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

}  // namespace vdb
