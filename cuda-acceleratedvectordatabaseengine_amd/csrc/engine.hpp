// engine.hpp — the index handle of the MI355X IVF-Flat engine (host side): one handle =
// one index on one device; engine.cpp binds it to the C ABI of include/vdb_ivf.h and
// group.cpp adds the multi-GPU forms (RCCL exchange, one handle per device).
//
// One handle = one index on one device. The whole index is HBM-resident in an
// interleaved list arena (kernels.hpp); a search is a short sequence of kernels
// per batch of queries, all enqueued on one stream with no host synchronisation:
//   pad queries -> coarse distances -> probe selection -> probe inversion (plan)
//   -> ivf_scan -> per-(query, probe) top-k -> per-query merge -> slot carry.
// Build-side calls (train/add/set_shard) synchronise where the reference
// algorithm needs a host decision (k-means++ draws from std::mt19937 on the host,
// exactly as ivf_flat_index.cpp:53-92 does).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <map>
#include <memory>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <queue>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/vdb_ivf.h"
#include "kernels.hpp"
#include "floor.hpp"
#include "uring.hpp"

namespace vdbe {

extern thread_local std::string g_last_error;

struct VdbError : std::runtime_error {
    int code;
    VdbError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        int code = (e == hipErrorOutOfMemory) ? VDB_ERR_OUT_OF_MEMORY : VDB_ERR_DEVICE;
        (void)hipGetLastError();
        throw VdbError(code, std::string(what) + ": " + hipGetErrorString(e));
    }
}
#define HIPCHECK(x) check((x), #x)

inline void check_nccl(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw VdbError(VDB_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}
#define NCCLCHECK(x) check_nccl((x), #x)

inline void require(bool ok, const std::string& msg, int code = VDB_ERR_INVALID_ARGUMENT) {
    if (!ok) throw VdbError(code, msg);
}

template <class F>
int guarded(F&& f) {
    try {
        f();
        return VDB_OK;
    } catch (const VdbError& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_last_error = "host allocation failed";
        return VDB_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return VDB_ERR_DEVICE;
    }
}

// Stream-ordered device memory for the engine's long-lived buffers (list arena, HBM list
// cache, search workspaces): one hipMemPool per device whose release threshold keeps freed
// memory reserved for the process (288 GB of HBM3E: an add's relayout and a workspace's
// growth reuse it without driver calls), allocated and freed on a per-device allocation
// stream. hipFreeAsync never synchronises the device the way hipFree does; the engine only
// releases a pooled buffer once no queued work can read it (stream synchronised, searches
// quiesced, or the workspace slot's previous call done).
// Off by default: on ROCm 7 buffers from the pool serialised the three batches a device
// runs in flight (1/8-shard rehearsal, 3 in flight: 93.7K QPS before the pool, 81.3K with
// it, 0.68 -> 0.79 ms per batch at an unchanged scan time); plain hipMalloc buffers overlap.
#ifndef VDB_DEVICE_POOL
#define VDB_DEVICE_POOL 0
#endif
struct DevicePool {
    hipMemPool_t pool = nullptr;
    hipStream_t stream = nullptr;
};
inline DevicePool& device_pool(int dev) {
    static std::mutex mu;
    static DevicePool pools[64];
    std::lock_guard<std::mutex> g(mu);
    require(dev >= 0 && dev < 64, "device ordinal out of range", VDB_ERR_INVALID_ARGUMENT);
    DevicePool& dp = pools[dev];
    if (!dp.pool) {
        hipMemPoolProps props = {};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        HIPCHECK(hipMemPoolCreate(&dp.pool, &props));
        uint64_t keep = ~0ull;
        HIPCHECK(hipMemPoolSetAttribute(dp.pool, hipMemPoolAttrReleaseThreshold, &keep));
        HIPCHECK(hipStreamCreateWithFlags(&dp.stream, hipStreamNonBlocking));
    }
    return dp;
}

// Growable device buffer (capacity in elements).
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    bool host = false;  // page-locked host memory the device reads and writes directly
    bool pooled = false;  // device memory from the device's stream-ordered pool
    int dev = 0;          // (pooled) the device the memory belongs to
    DevBuf() = default;
    explicit DevBuf(bool pool) : pooled(pool && VDB_DEVICE_POOL) {}
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) {
            if (host) (void)hipHostFree(p);
            else if (pooled) (void)hipFreeAsync(p, device_pool(dev).stream);
            else (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    T* ensure(size_t n) {
        if (n <= cap && p) return p;
        release();
        size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        if (host) {
            HIPCHECK(hipHostMalloc((void**)&p, bytes, hipHostMallocMapped | hipHostMallocPortable));
        } else if (pooled) {
            HIPCHECK(hipGetDevice(&dev));
            DevicePool& dp = device_pool(dev);
            HIPCHECK(hipMallocFromPoolAsync((void**)&p, bytes, dp.pool, dp.stream));
            HIPCHECK(hipStreamSynchronize(dp.stream));  // usable from any stream right away
        } else {
            HIPCHECK(hipMalloc(&p, bytes));
        }
        cap = std::max<size_t>(n, 1);
        return p;
    }
    size_t device_bytes() const { return (p && !host) ? cap * sizeof(T) : 0; }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
        std::swap(host, o.host);
        std::swap(pooled, o.pooled);
        std::swap(dev, o.dev);
    }
};

// Page-locked host buffer (fast device-to-host copies of build-time scratch).
template <class T>
struct PinnedBuf {
    T* p = nullptr;
    explicit PinnedBuf(size_t n) { HIPCHECK(hipHostMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T))); }
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
};

inline uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

struct EventSet {
    hipEvent_t begin, coarse_end, scan_begin, scan_end, end;
    hipEvent_t collect_begin, collect_end;  // deferred screened scan: around its collect kernel
    bool collected = false;
    hipEvent_t x_end, m_end;  // multi-GPU: the all-gather done (comm stream), the rank merge done
    bool xchg = false;        // this batch (or call) ended in an exchange
};

// One host-API search() call waiting in the coalescing queue.
struct PendingSearch {
    const float* q;
    uint32_t n, nprobe, k;
    float* dist;
    uint64_t* ids;
    int rc = 1;  // 1 = pending, then a VDB_* code
    std::string err;
};

// Request coalescing (the reference's intent: QueryServiceImpl::Config max_batch_size /
// coalesce_window_ms, query_service.h:25-31, never implemented there): concurrent
// vdb_ivf_search callers enqueue; a dispatcher thread takes every compatible waiting call
// (same nprobe and k), up to max_queries, stages the queries in page-locked memory and
// enqueues ONE device search on a staging slot's own stream (H2D, search, D2H), then
// goes straight on to the next batch: up to kHostSlots batches are in flight, so one
// batch's copies and coarse step overlap the previous batch's scan (the pipelining the
// reference's DoubleBuffer / StreamScheduler intended, transfer_manager.h:168-239). A
// completion thread waits for each batch in issue order and hands the results back.
// Per-call slot semantics stay exact (request boundaries, kernels' req_start).
struct HostBatch {
    std::vector<PendingSearch*> reqs;
    uint32_t nq = 0, P = 0, K = 0;
    DevBuf<float> hq, hd;     // page-locked staging
    DevBuf<uint64_t> hi;
    DevBuf<uint32_t> hreq;
    DevBuf<float> dq, dd;     // device
    DevBuf<uint64_t> di;
    DevBuf<uint32_t> dreq;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    int rc = VDB_OK;
    std::string err;
    HostBatch() { hq.host = hd.host = hi.host = hreq.host = true; }
};

struct Coalescer {
    static constexpr int kHostSlots = 3;
    std::mutex m;
    std::condition_variable wake, done, slot_free, issued;
    std::deque<PendingSearch*> queue;
    std::deque<HostBatch*> inflight;  // issue order
    std::vector<HostBatch*> free_slots;
    HostBatch slots[kHostSlots];
    std::thread dispatcher, completer;
    bool stop = false, dispatch_done = false;
    uint64_t batches = 0, requests = 0;
};

}  // namespace vdbe

using namespace vdbe;

#ifndef VDB_SLOTS
#define VDB_SLOTS 3  // 4 measured slower at the 1/8 shard: 108K QPS at 4 in flight, 90K at 3, vs 128K (3 slots, 3 in flight)
#endif

struct vdb_ivf {
    uint32_t dim = 0, nlist = 0, dp = 0, d4 = 0;
    int metric = 0;
    int device = 0;
    uint64_t max_gpu_memory = 0;
    hipStream_t stream = nullptr;
    mutable std::mutex mu;

    DevBuf<float> cent_rm;   // [nlist][dp], zero pads
    DevBuf<float4> cent_il;  // [ceil(nlist/64)][d4][64]

    std::vector<uint64_t> count;      // per list, global (emptiness semantics)
    std::vector<uint8_t> owned;       // lists this handle scans
    std::vector<uint64_t> block_off;  // arena block offset per owned list
    uint64_t arena_blocks = 0;
    DevBuf<float4> arena{true};
    DevBuf<uint64_t> arena_ids{true};
    DevBuf<uint64_t> d_block_off;
    DevBuf<uint32_t> d_count_local, d_count_global, d_nseg;
    std::vector<uint64_t> nseg_prefix;  // sum of the j largest local segment counts
    uint64_t total = 0;
    uint32_t rank = 0, world = 1;
    uint32_t batch = 256;
    int stale = 1;
    bool wide_scan = true;
    int coarse_mode = 1;  // 1: MFMA bounds + exact re-rank (L2/IP); 0: exact VALU distances
    uint32_t wide_stride = 1;  // wide-item dispatch permutation (1 = plan order; measured best)
    uint32_t seg_blocks = 8;  // current segment size (blocks of 64 vectors; upload_directory sets it)
    uint32_t seg_blocks_opt = 0;                // 0 = automatic (upload_directory)
    bool bounded_stats = false;                 // count the bounded scan's re-ranks and blocks (profile_read)
    // wide items of at least this many queries are bounded on the matrix cores and
    // re-ranked exactly (ivf_scan_bounded); 0 = never. Off by default: on the bench
    // workloads the exact re-ranks (per-list top-k insertions, ~5% of pairs, each a
    // gathered re-read of an evicted vector) cost more than the VALU it saves
    // (DESIGN.md "Bounded scan: measured and rejected as default").
    uint32_t scan_mfma_min = 0;
    // persistent scan grid in workgroups (0: 2 per CU on the whole chip)
    uint32_t scan_blocks = 0;
    uint32_t segs_item_opt = 0;   // segments per wide item (0: one per wave, taken dynamically)
    uint32_t wide_group = 16;     // queries per wide item at most: 16 (4-wave workgroups) or 32 (8-wave)
    bool fused_scan = true;       // narrow items inside the wide scan's grid (option fused_scan; +2-3 %)
    bool fused_merge = true;      // the four per-batch merges as one launch (option fused_merge)
    // At most this many scans of batches in flight overlap (0: no limit): a batch's scan
    // waits for the scan issued `scan_window` batches earlier to finish, so the GPU serves
    // batches closer to issue order (latency spread at several batches in flight).
    uint32_t scan_window = 0;
    uint64_t scan_seq = 0;
    int scan_hist[8] = {};  // slot index of the scans issued, by sequence number
    uint32_t narrow_blocks = 64;  // persistent narrow-scan workgroups beside the wide scan (1/8 shard: +1.5 % vs 512)

    // Screened scan (screen.hip, option "screen", on by default): every (query, vector)
    // distance is bounded on the matrix cores from a bf16 shadow of the lists and computed
    // exactly (the reference's sequential fp32 sum) only where it can reach the list's
    // top-k; results are bit-identical to the exact scan. Built from the arena by the first
    // search after the lists change: the shadow in MFMA operand order (half the arena's
    // bytes), the fp32 rows in slot order (then the lists' only fp32 copy: the arena is
    // released and rebuilt from them on demand), per-slot norms. The tier keeps the shadow,
    // norms and ids of every stored list resident (screen_update_tier). Not built for
    // Cosine, or when an allocation fails (the exact scan serves); max_gpu_memory caps list
    // bytes only.
    bool screen_opt = true;
    bool screen_ready = false;
    bool screen_stale = false;  // lists or centroids changed since the last build
    uint32_t screen_segs_auto = 4;  // segments per screened wide item (upload_directory; option segs_per_item)
    uint32_t screen_group = 0;      // queries per screened wide item at most: 16 or 32, 0 = automatic (option screen_group)
    // Shadow format of the deferred screen (option screen_i8): 1 = int8 with a per-vector scale
    // (half the bf16 shadow's bytes, a ~4.6x wider bound); 0 = bf16. The inline kernel
    // (screen_defer 0) always uses bf16.
    // 2 (default) = automatic (want_i8): int8 for lists in HBM, at both item widths (16- and
    // 32-query items), kept unless the calibration batch at the build vetoes it
    // (screen_calibrate: survivors beyond k per pair above 1.5 % of the pairs, or an overflow:
    // a regime where its wider bound re-checks more than its smaller stream saves); bf16 in the
    // tier (each survivor is a row read from the home). Round 5, same box: cfg3 collect 1.40
    // vs 2.43 ms (bf16), cfg4 shard 2.15 vs 3.38 ms; the mixture is vetoed (6.2 % excess).
    int screen_i8 = 2;
    bool i8_vetoed = false;  // (automatic: the calibration vetoed int8 for this handle)
    uint32_t last_P = 0;     // the nprobe of the search that triggers a screen build
    bool want_i8() const {
        if (!screen_defer) return false;
        if (screen_i8 != 2) return screen_i8 == 1;
        return !tiered() && !i8_vetoed;
    }
    uint32_t screen_thr_every = 0;  // deferred collect: blocks between re-reads of the shared thresholds, 0 = automatic (option screen_thr_every)
    // Deferred re-checks (option screen_defer, default 1): the scan only collects candidates
    // against upper-bound thresholds; survivors of each pair's final threshold are re-checked
    // exactly afterwards from the arena (screen.hip ivf_screen_collect). 0: the inline kernel
    // (re-checks as candidates appear, from a row-major fp32 copy of the lists).
    bool screen_defer = true;
    uint32_t screen_cand_cap = 4u << 20;  // collected candidates per batch (an overflowing pair is recomputed whole)
    // Two-pass exact re-check (option screen_recheck2, default on; rows in HBM): per pair first the k
    // survivors of smallest lower bound, then only the others whose lower bound is not above
    // the k-th exact distance so far (screen.hip ivf_screen_recheck2); 0: every survivor of the
    // final threshold (ivf_screen_exact_lane + ivf_screen_pair_topk). Results are identical.
    bool screen_recheck2 = true;
    // One fp32 copy of the lists in HBM: while the screen is built, the row-major copy
    // (screen_rows, slot order: what the exact re-checks read) is the only one and the
    // interleaved arena is released (arena_dropped). Exact-path searches (k > 64, the
    // run-time floor's batches) scan the row-major copy itself (ScanArgs::rows_layout: no
    // rebuild, no quiesce, no second copy); what needs the interleaved layout (an add /
    // relayout, the screen off, the opt-in bounded scan, Cosine) rebuilds it from the rows
    // first (ensure_arena: one interleave pass). Footprint while screening: rows + shadow +
    // norms + ids ~ 1.5x the lists, whatever k the searches ask for.
    bool arena_dropped = false;
    // The screen in the list-cache tier (an index larger than HBM, configs[4]): the shadow,
    // norms and ids of EVERY stored list stay HBM-resident (half the fp32 list bytes), packed
    // by sblock_off; the fp32 rows stay at the home and only the survivors' rows are read per
    // batch: straight from the page-locked host arena over PCIe, or, from a file home, by
    // io_uring into page-locked staging and one copy to HBM (fetch_survivor_rows). No list is
    // loaded into the cache for such a batch (the cache serves the exact-path searches).
    std::vector<uint64_t> sblock_off;  // tier: per stored list its first shadow block
    std::vector<uint32_t> sblist_host; // tier, file home: per shadow block its list
    uint64_t sblocks = 0;
    DevBuf<uint64_t> d_sblock_off;
    DevBuf<uint64_t> screen_ids;       // tier: the ids in shadow slot order
    DevBuf<float> fetch_stage;         // tier, file home: page-locked staging of the survivors' rows
    DevBuf<char> fetch_bounce;         // ... O_DIRECT reads: 4 KiB-aligned supersets, one slot per read in flight
    bool tier_row_direct = true;       // option tier_row_direct: survivor rows with O_DIRECT (no page cache)
    uint32_t tier_row_qd = 256;        // option tier_row_qd: survivor-row reads in flight (their own ring)
    std::unique_ptr<UringReader> row_uring;
    DevBuf<float> fetch_dev;           // ... on the device ([n][dim], padded into the slot's srows)
    std::vector<uint2> fetch_surv;     // ... their (slot, pair)
    uint64_t screen_rows_fetched = 0, screen_row_bytes = 0, screen_tier_batches = 0, screen_reruns = 0;
    uint64_t screen_rows_cached = 0;   // ... survivor rows copied from the HBM cache instead
    bool tier_row_cache = true;        // option tier_row_cache: the idle cache holds the largest lists' rows
    DevBuf<ulonglong2> cache_src;      // ... per batch {row index, cache slot} of those survivors
    std::vector<ulonglong2> cache_src_host;
    uint32_t tier_cand_cap = 0;        // ... a candidate capacity grown by an overflow
    // ... at most this many candidates per batch (option tier_cand_max; never below
    // screen_cand_cap): a batch that needs more is served by the exact list-cache path
    uint32_t tier_cand_max = 32u << 20;
    // (option collect_stamps, diagnostics) timeline records of the collect kernel's items
    DevBuf<unsigned long long> stamps_buf;
    uint32_t stamps_cap = 0, stamp_batch = 0;
    uint64_t screen_tier_fallbacks = 0;
    bool force_exact = false;          // (that path's batches: never screened)
    // Run-time floor under the screen (lists in HBM; floor.hpp): every deferred batch reports
    // its survivors (or an overflow of its candidate buffer), its (query, vector) pairs and k x
    // its valid (query, list) pairs into a ring of page-locked host memory, read without
    // synchronisation when a later batch is planned. A batch whose survivors beyond those
    // exceed screen_floor_ppm of its pairs (a regime where the bound is wider than the
    // distance spread) sends the next batches to the exact scan, with backoff, then one
    // probe batch retries the screen. (Break-even at cfg3: the exact scan 4.9 ms against the
    // screen's 2.7 ms plus ~4.6 ns per survivor, ~9 % of the batch's 5.0M pairs; 5 % leaves
    // room for the retries.) Results are the same either way; only speed changes.
    ScreenFloor floor;
    DevBuf<uint4> floor_host;  // page-locked: ScreenFloor::kRing report entries
    const volatile uint32_t* floor_entry(uint32_t i) const { return (const volatile uint32_t*)(floor_host.p + i); }
    DevBuf<uint4> screen_sh;
    DevBuf<float> screen_rows;
    DevBuf<float4> screen_meta;
    DevBuf<float> screen_scale;  // int8 shadow: per slot s_b
    bool screen_fmt_i8 = false;  // the shadow built is int8 (else bf16)
    DevBuf<uint32_t> screen_blist;  // the list of every arena block (residuals against its centroid)

    // List-cache tier (option list_cache_bytes > 0), the reference's residency model
    // (load_list_to_gpu on first touch under a byte cap, evict_list_from_gpu,
    // ivf_flat_index.cpp:387-471) for indexes larger than HBM: the arena then lives in
    // page-locked host memory and HBM holds a cache of whole lists. Before a batch is
    // planned, every list it probes is made resident (DMA of its blocks), evicting the
    // least recently used lists the batch does not probe; the scan reads the cache
    // through the same directory (d_block_off), so the kernels are unchanged.
    static constexpr uint64_t kAbsent = ~0ull;
    uint64_t cache_blocks = 0;  // capacity in 64-vector blocks (0: tier off, the arena is in HBM)
    DevBuf<float4> cache{true};
    DevBuf<uint64_t> cache_ids{true};
    std::vector<uint64_t> cache_off;        // per list: cache block offset or kAbsent
    std::vector<uint64_t> last_use;         // per list: batch tick of the last probe
    std::map<uint64_t, uint64_t> free_ext;  // free cache extents: block offset -> blocks
    uint64_t use_tick = 0, cache_used = 0;
    uint64_t resident_n = 0, storable_n = 0;  // cached lists / non-empty lists stored here
    uint64_t cache_loads = 0, cache_evictions = 0, cache_bytes_in = 0;
    DevBuf<uint32_t> probe_stage;  // pinned: the batch's probes, read by the host
    DevBuf<uint64_t> dir_stage;    // pinned: directory upload source
    // Recorded after every cache load and directory upload, on the stream that made
    // them. Every tier-mode batch waits for it before it plans and scans, so a search
    // on another stream whose lists are all cached never reads blocks or directory
    // entries still in flight (a miss quiesces the other streams first, so the latest
    // recording covers every earlier load).
    hipEvent_t tier_ev = nullptr;
    bool tier_ev_used = false;

    // File home for the tier (vdb_ivf_open_lists): the lists stay in an index file written
    // by vdb_ivf_save and are read into the cache on demand: io_uring reads (O_DIRECT when
    // the file system allows it) into a ring of page-locked staging buffers, H2D copies,
    // then pad + interleave kernels into the cache's block layout.
    int home_fd = -1;
    int home_fd_direct = -1;         // O_DIRECT descriptor of the same file (or -1: buffered)
    // O_DIRECT granule the file system accepts for offsets and sizes, probed at open: 512 on
    // most (a 3,072-B survivor row then reads 3,072 or 3,584 B), else 4096 (4 KiB-aligned
    // supersets, 1.5-2 pages per row)
    uint32_t dio_align = 4096;
    std::vector<uint64_t> file_off;  // per list: file offset of its ids (vectors follow)
    struct Stage {                   // one page-locked staging buffer of the read ring
        DevBuf<char> buf;
        hipEvent_t copied = nullptr;  // its H2D copies are done: the buffer may be refilled
        bool copying = false;
        int reads = 0;                // reads in flight
        uint64_t m = 0, dst_block = 0;
        size_t ids_delta = 0, vec_delta = 0;
    };
    static constexpr int kStages = 8;
    Stage stages[kStages];
    std::unique_ptr<UringReader> uring;
    DevBuf<float> drows, dpad;       // device: a chunk's rows, then zero-padded to dp (search stream)
    DevBuf<float> drows_cs, dpad_cs; // the same for loads on copy_stream (they may run concurrently)
    uint64_t file_bytes_read = 0;
    // tier pipeline: loads for the next sub-batch run on copy_stream beside the scan
    hipStream_t copy_stream = nullptr;
    hipEvent_t sb_done[2] = {nullptr, nullptr}, load_ev = nullptr, tier_call_ev = nullptr;
    bool tier_call_used = false;
    uint64_t tier_prefetches = 0, tier_sync_loads = 0, tier_subbatches = 0;

    // Search workspaces: a ring of slots so that searches issued on different streams
    // run concurrently (one batch's small kernels and scan tail overlap the next
    // batch's scan). A call takes the next slot; its stream first waits for the
    // slot's previous batch (slot.done), wherever that ran.
    struct SearchSlot {
        DevBuf<float> qpad{true}, cd{true}, cdelta{true}, part_d{true}, slot_d{true}, carry_d{true}, carry2_d{true};
        DevBuf<uint64_t> part_i{true}, slot_i{true}, carry_i{true}, carry2_i{true};
        uint32_t carry_sel = 0;  // fused merge: the carry buffer the call's next batch reads (ping-pong)
        uint64_t xfill = 0;      // (exchange_emulate_world) the record size the other ranks' empty records were filled for
        const float* q = nullptr;  // the batch's zero-padded queries: qpad, or the caller's rows when dim == dp
        DevBuf<uint32_t> probes{true}, nseg_qp{true}, pbqp{true}, sorted_pair{true}, pbs{true}, counters{true},
            l1base{true}, cand{true}, thr{true};
        DevBuf<uint2> l1_items{true};
        DevBuf<float> l1_d{true};
        DevBuf<uint64_t> l1_i{true};
        DevBuf<vdbk::ScanItem> items{true}, items_w{true};
        DevBuf<uint16_t> qres{true};  // screened scan: per (query, probe) bf16 A rows [B * P][dp]
        DevBuf<float4> pst{true};     // ... and their norms
        DevBuf<float> qscale{true};   // ... and (int8 shadow) their scales
        DevBuf<uint32_t> thr4{true};  // ... and, per sorted pair, 4 quarter-list thresholds
        // deferred screened scan: collected candidates, per sorted pair survivor counts, offsets and
        // overflow marks, the survivors' slots grouped per pair, and (tier) their fetched rows
        DevBuf<uint4> scand{true};
        DevBuf<uint32_t> scnt{true}, soff{true}, ovf{true}, ubcnt{true};
        DevBuf<uint2> surv{true};
        DevBuf<float> ublist{true}, sdist{true};
        DevBuf<float> srows{true};
        DevBuf<float> slb{true};         // screened tier, two-pass: the survivors' lower bounds
        DevBuf<uint8_t> smark{true};     // ... their pass marks (1 A, 2 B)
        DevBuf<uint32_t> rowmap{true};   // ... survivor -> compact fetched row
        DevBuf<uint8_t> xrec{true}, xgat{true};  // multi-GPU: this rank's packed partials, the gathered records
        DevBuf<float> gq{true};            // group member: the call's queries on this device
        DevBuf<uint32_t> greq{true};       // group member: the call's request starts on this device
        hipStream_t side = nullptr;  // narrow-item scan, concurrent with the wide items
        hipStream_t gstream = nullptr;  // group member: the stream this slot's searches run on
        hipEvent_t x_ready = nullptr, x_done = nullptr;  // fences around this slot's collectives
        hipEvent_t fork = nullptr, join = nullptr, done = nullptr;
        hipEvent_t scan_done = nullptr;  // (scan_window) this slot's latest scan has finished
        bool used = false;
        uint64_t device_bytes() const {
            uint64_t b = 0;
            for (uint64_t x : {qpad.device_bytes(), cd.device_bytes(), cdelta.device_bytes(), part_d.device_bytes(),
                               slot_d.device_bytes(), carry_d.device_bytes(), carry2_d.device_bytes(),
                               part_i.device_bytes(), slot_i.device_bytes(), carry_i.device_bytes(),
                               carry2_i.device_bytes(), probes.device_bytes(), nseg_qp.device_bytes(), pbqp.device_bytes(),
                               sorted_pair.device_bytes(), pbs.device_bytes(), counters.device_bytes(),
                               l1base.device_bytes(), cand.device_bytes(), thr.device_bytes(), l1_items.device_bytes(),
                               l1_d.device_bytes(), l1_i.device_bytes(), items.device_bytes(), items_w.device_bytes(),
                               qres.device_bytes(), pst.device_bytes(), qscale.device_bytes(), thr4.device_bytes(), scand.device_bytes(),
                               scnt.device_bytes(), soff.device_bytes(), ovf.device_bytes(), ubcnt.device_bytes(),
                               surv.device_bytes(), ublist.device_bytes(), sdist.device_bytes(), srows.device_bytes(),
                               slb.device_bytes(), smark.device_bytes(), rowmap.device_bytes(),
                               xrec.device_bytes(), xgat.device_bytes(), gq.device_bytes(), greq.device_bytes()})
                b += x;
            return b;
        }
    };
    static constexpr int kSlots = VDB_SLOTS;  // workspace slots: batches one handle runs concurrently
    SearchSlot slots[kSlots];
    uint32_t next_slot = 0;

    // ---- multi-GPU: lists sharded over ranks (LPT), every rank runs the
    // coarse step for the whole batch, scans its own lists and merges its slots into ONE
    // packed record per batch (f32 dist[B][k] | pad | u64 ids[B][k]); one RCCL all-gather
    // of the records over xGMI, then the on-device unique-id merge. The communicator is
    // attached (one process per GPU, vdb_ivf_attach_comm) or owned by a group handle
    // (one process, one member handle per device, vdb_ivf_create_group).
    ncclComm_t comm = nullptr;
    bool comm_owned = false;
    uint32_t comm_rank = 0, comm_world = 1;
    // (option exchange_emulate_world, diagnostics) a communicator of world 1 exchanges records
    // the size of W ranks' (the batch's record plus W - 1 empty records of the same layout) and
    // merges W records: the per-batch cost of an 8-GPU node's exchange and rank merge on one
    // rank's timeline (one GPU cannot hold 8 ranks: RCCL refuses two ranks on one device); the
    // results stay this handle's own exact answer
    uint32_t xchg_emulate = 0;
    uint32_t xchg_records() const { return comm_world > 1 ? comm_world : std::max<uint32_t>(1, xchg_emulate); }
    // Every collective of the communicator runs on this one stream, fenced by events
    // against the search stream that produced / consumes its buffers: with several
    // batches in flight on several streams, every rank then executes its collectives in
    // the same (issue) order whatever the library does across streams.
    hipStream_t comm_stream = nullptr;

    // Order a collective on comm_stream after the work queued on s (returns comm_stream).
    void make_comm_stream() {  // with the communicator (the device must be current)
        // (high priority: a queue of its own, apart from the 4 the search streams share —
        // profiles/r05_hw_queue_probe.txt — and the exchange dispatched ahead of scan work)
        if (!comm_stream) {
            int lo = 0, hi = 0;
            HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHECK(hipStreamCreateWithPriority(&comm_stream, hipStreamNonBlocking, hi));
        }
    }
    hipStream_t comm_enter(SearchSlot& w, hipStream_t s) {
        if (!w.x_ready) {
            HIPCHECK(hipEventCreateWithFlags(&w.x_ready, hipEventDisableTiming));
            HIPCHECK(hipEventCreateWithFlags(&w.x_done, hipEventDisableTiming));
        }
        HIPCHECK(hipEventRecord(w.x_ready, s));
        HIPCHECK(hipStreamWaitEvent(comm_stream, w.x_ready, 0));
        return comm_stream;
    }
    // ... and the work queued on s next after it.
    void comm_leave(SearchSlot& w, hipStream_t s) {
        HIPCHECK(hipEventRecord(w.x_done, comm_stream));
        HIPCHECK(hipStreamWaitEvent(s, w.x_done, 0));
    }
    // Group handle: members[m] holds the lists owner[l] == m places on its device; the
    // group itself holds only the host-API staging on members[0]'s device.
    std::vector<std::unique_ptr<vdb_ivf>> members;
    std::vector<uint32_t> owner;  // per list: member storing it, or kUnplaced
    static constexpr uint32_t kUnplaced = 0xFFFFFFFFu;
    bool group_rccl = false;      // members on distinct devices: RCCL; else device copies (rehearsal)
    std::vector<hipEvent_t> gev;  // group call fences, 2 per member
    bool is_group() const { return !members.empty(); }
    vdb_ivf* head() { return is_group() ? members[0].get() : this; }
    // the handle storing list l (a group member, or this handle)
    vdb_ivf* store_of(uint32_t l) {
        if (!is_group()) return this;
        return owner[l] == kUnplaced ? members[0].get() : members[owner[l]].get();
    }
    DevBuf<float> out_d, qin;  // host-API staging (synchronous calls)
    DevBuf<uint64_t> out_i;
    DevBuf<uint32_t> d_req;    // coalesced calls: request start per query
    std::unique_ptr<Coalescer> co;
    std::mutex co_init_mu;
    bool coalesce = true;
    uint32_t coalesce_max_queries = 1024;
    uint32_t coalesce_window_us = 0;
    DevBuf<unsigned long long> stats, stats_scratch;

    bool prof = false;
    std::vector<EventSet> events;
    size_t events_used = 0;

    ~vdb_ivf() {
        stop_coalescer();
        // An exchange that missed its deadline never completes: nothing is waited for and
        // the communicator is left to the process's exit (destroying or aborting it could
        // hang, or free what a still-queued collective reads).
        const bool failed = comm_failed();
        stop_watch();
        members.clear();  // each member waits for and frees its own device work
        (void)hipSetDevice(device);
        if (!failed) {
            try {
                quiesce();  // pooled buffers are freed stream-ordered: no search may still read them
            } catch (...) {
            }
            if (stream) (void)hipStreamSynchronize(stream);
            for (auto& sl : slots)
                if (sl.gstream) (void)hipStreamSynchronize(sl.gstream);
        }
        if (comm) {
            if (comm_owned && !failed) (void)ncclCommDestroy(comm);
            comm = nullptr;
        }
        for (auto& e : gev) (void)hipEventDestroy(e);
        if (home_fd >= 0) ::close(home_fd);
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        for (auto& st : stages)
            if (st.copied) (void)hipEventDestroy(st.copied);
        for (hipEvent_t e : {sb_done[0], sb_done[1], load_ev, tier_call_ev, tier_ev})
            if (e) (void)hipEventDestroy(e);
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        if (home_fd_direct >= 0) ::close(home_fd_direct);
        for (auto& e : events)
            for (hipEvent_t x : {e.begin, e.coarse_end, e.scan_begin, e.scan_end, e.end, e.x_end, e.m_end, e.collect_begin, e.collect_end})
                (void)hipEventDestroy(x);
        for (auto& sl : slots) {
            if (sl.fork) (void)hipEventDestroy(sl.fork);
            if (sl.join) (void)hipEventDestroy(sl.join);
            if (sl.done) (void)hipEventDestroy(sl.done);
            if (sl.scan_done) (void)hipEventDestroy(sl.scan_done);
            if (sl.side) (void)hipStreamDestroy(sl.side);
            if (sl.gstream) (void)hipStreamDestroy(sl.gstream);
            if (sl.x_ready) (void)hipEventDestroy(sl.x_ready);
            if (sl.x_done) (void)hipEventDestroy(sl.x_done);
        }
        if (comm_stream) (void)hipStreamDestroy(comm_stream);
        if (stream) (void)hipStreamDestroy(stream);
    }

    void set_device() { HIPCHECK(hipSetDevice(device)); }

    // Every byte of device memory the handle holds (vdb_ivf_gpu_bytes_allocated): lists in
    // whatever layouts exist (arena, row-major copy, bf16 shadow, norms, ids, list cache),
    // centroids, directories, the search workspaces of every slot and the staging buffers.
    uint64_t device_footprint() const {
        uint64_t b = 0;
        for (uint64_t x : {cent_rm.device_bytes(), cent_il.device_bytes(), arena.device_bytes(), arena_ids.device_bytes(),
                           d_block_off.device_bytes(), d_count_local.device_bytes(), d_count_global.device_bytes(),
                           d_nseg.device_bytes(), screen_sh.device_bytes(), screen_rows.device_bytes(),
                           screen_meta.device_bytes(), screen_blist.device_bytes(), screen_scale.device_bytes(),
                           screen_ids.device_bytes(), d_sblock_off.device_bytes(), cache_src.device_bytes(),
                           cache.device_bytes(),
                           cache_ids.device_bytes(), drows.device_bytes(), dpad.device_bytes(), drows_cs.device_bytes(),
                           dpad_cs.device_bytes(), out_d.device_bytes(), qin.device_bytes(), out_i.device_bytes(),
                           d_req.device_bytes(), stats.device_bytes()})
            b += x;
        for (const auto& w : slots) b += w.device_bytes();
        if (co)
            for (const HostBatch& hb : co->slots)
                b += hb.dq.device_bytes() + hb.dd.device_bytes() + hb.di.device_bytes() + hb.dreq.device_bytes();
        return b;
    }

    // ---- host-API search: direct, or through the coalescing queue ----
    void search_host(const float* q, uint32_t n, uint32_t nprobe, uint32_t k, float* dist, uint64_t* ids,
                     const uint32_t* h_req_start) {
        set_device();
        HIPCHECK(hipMemcpyAsync(qin.ensure((size_t)n * dim), q, (size_t)n * dim * 4, hipMemcpyHostToDevice, stream));
        const uint32_t* dr = nullptr;
        if (h_req_start) {
            HIPCHECK(hipMemcpyAsync(d_req.ensure(n), h_req_start, (size_t)n * 4, hipMemcpyHostToDevice, stream));
            dr = d_req.p;
        }
        search_device(qin.p, n, nprobe, k, out_d.ensure((size_t)n * k), out_i.ensure((size_t)n * k), stream, dr);
        HIPCHECK(hipMemcpyAsync(dist, out_d.p, (size_t)n * k * 4, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipMemcpyAsync(ids, out_i.p, (size_t)n * k * 8, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
    }

    void start_coalescer() {
        if (co) return;
        co.reset(new Coalescer());
        set_device();
        for (HostBatch& hb : co->slots) {
            HIPCHECK(hipStreamCreateWithFlags(&hb.stream, hipStreamNonBlocking));
            HIPCHECK(hipEventCreateWithFlags(&hb.done, hipEventDisableTiming));
            co->free_slots.push_back(&hb);
        }
        co->dispatcher = std::thread([this] { dispatch_loop(); });
        co->completer = std::thread([this] { complete_loop(); });
    }

    void stop_coalescer() {
        if (!co) return;
        {
            std::lock_guard<std::mutex> g(co->m);
            co->stop = true;
        }
        co->wake.notify_all();
        co->slot_free.notify_all();
        if (co->dispatcher.joinable()) co->dispatcher.join();
        if (co->completer.joinable()) co->completer.join();
        (void)hipSetDevice(device);
        for (HostBatch& hb : co->slots) {
            if (hb.stream) (void)hipStreamDestroy(hb.stream);
            if (hb.done) (void)hipEventDestroy(hb.done);
        }
        co.reset();
    }

    void dispatch_loop() {
        Coalescer& c = *co;
        (void)hipSetDevice(device);
        for (;;) {
            HostBatch* hb = nullptr;
            {
                std::unique_lock<std::mutex> lk(c.m);
                c.wake.wait(lk, [&] { return c.stop || !c.queue.empty(); });
                if (c.queue.empty()) break;  // stop requested and nothing left
                // a free staging slot: at most kHostSlots batches in flight (calls keep
                // queueing meanwhile, so the next batch grows while the device is busy)
                c.slot_free.wait(lk, [&] { return !c.free_slots.empty(); });
                if (coalesce_window_us)
                    c.wake.wait_for(lk, std::chrono::microseconds(coalesce_window_us), [&] {
                        uint64_t t = 0;
                        for (auto* r : c.queue) t += r->n;
                        return c.stop || t >= coalesce_max_queries;
                    });
                hb = c.free_slots.back();
                c.free_slots.pop_back();
                hb->reqs.clear();
                hb->nq = 0;
                hb->P = c.queue.front()->nprobe;
                hb->K = c.queue.front()->k;
                for (auto it = c.queue.begin(); it != c.queue.end();) {
                    PendingSearch* r = *it;
                    if (r->nprobe == hb->P && r->k == hb->K && (hb->reqs.empty() || hb->nq + r->n <= coalesce_max_queries)) {
                        hb->reqs.push_back(r);
                        hb->nq += r->n;
                        it = c.queue.erase(it);
                    } else {
                        ++it;
                    }
                }
                c.batches++;
                c.requests += hb->reqs.size();
            }
            hb->rc = VDB_OK;
            hb->err.clear();
            try {
                const uint32_t nq = hb->nq, K = hb->K;
                float* hq = hb->hq.ensure((size_t)nq * dim);
                uint32_t* hr = hb->reqs.size() > 1 ? hb->hreq.ensure(nq) : nullptr;
                uint32_t o = 0;
                for (PendingSearch* r : hb->reqs) {
                    std::memcpy(hq + (size_t)o * dim, r->q, (size_t)r->n * dim * 4);
                    if (hr)
                        for (uint32_t i = 0; i < r->n; ++i) hr[o + i] = o;
                    o += r->n;
                }
                hb->hd.ensure((size_t)nq * K);
                hb->hi.ensure((size_t)nq * K);
                std::lock_guard<std::mutex> g(mu);  // held only while the batch is enqueued
                set_device();
                HIPCHECK(hipMemcpyAsync(hb->dq.ensure((size_t)nq * dim), hq, (size_t)nq * dim * 4, hipMemcpyHostToDevice,
                                        hb->stream));
                const uint32_t* dr = nullptr;
                if (hr) {
                    HIPCHECK(hipMemcpyAsync(hb->dreq.ensure(nq), hr, (size_t)nq * 4, hipMemcpyHostToDevice, hb->stream));
                    dr = hb->dreq.p;
                }
                search_device(hb->dq.p, nq, hb->P, K, hb->dd.ensure((size_t)nq * K), hb->di.ensure((size_t)nq * K),
                              hb->stream, dr);
                HIPCHECK(hipMemcpyAsync(hb->hd.p, hb->dd.p, (size_t)nq * K * 4, hipMemcpyDeviceToHost, hb->stream));
                HIPCHECK(hipMemcpyAsync(hb->hi.p, hb->di.p, (size_t)nq * K * 8, hipMemcpyDeviceToHost, hb->stream));
                HIPCHECK(hipEventRecord(hb->done, hb->stream));
            } catch (const VdbError& e) {
                hb->rc = e.code;
                hb->err = e.what();
            } catch (const std::exception& e) {
                hb->rc = VDB_ERR_DEVICE;
                hb->err = e.what();
            }
            {
                std::lock_guard<std::mutex> g(c.m);
                c.inflight.push_back(hb);
            }
            c.issued.notify_one();
        }
        {
            std::lock_guard<std::mutex> g(c.m);
            c.dispatch_done = true;
        }
        c.issued.notify_one();
    }

    void complete_loop() {
        Coalescer& c = *co;
        (void)hipSetDevice(device);
        for (;;) {
            HostBatch* hb = nullptr;
            {
                std::unique_lock<std::mutex> lk(c.m);
                c.issued.wait(lk, [&] { return !c.inflight.empty() || c.dispatch_done; });
                if (c.inflight.empty()) return;
                hb = c.inflight.front();
                c.inflight.pop_front();
            }
            if (hb->rc == VDB_OK) {
                const hipError_t e = hipEventSynchronize(hb->done);
                if (e != hipSuccess) {
                    hb->rc = VDB_ERR_DEVICE;
                    hb->err = std::string("search batch: ") + hipGetErrorString(e);
                }
            }
            if (hb->rc == VDB_OK) {
                uint32_t o = 0;
                for (PendingSearch* r : hb->reqs) {
                    std::memcpy(r->dist, hb->hd.p + (size_t)o * hb->K, (size_t)r->n * hb->K * 4);
                    std::memcpy(r->ids, hb->hi.p + (size_t)o * hb->K, (size_t)r->n * hb->K * 8);
                    o += r->n;
                }
            }
            {
                std::lock_guard<std::mutex> g(c.m);
                for (PendingSearch* r : hb->reqs) {
                    r->err = hb->err;
                    r->rc = hb->rc;
                }
                hb->reqs.clear();
                c.free_slots.push_back(hb);
            }
            c.done.notify_all();
            c.slot_free.notify_one();
        }
    }

    void search_coalesced(const float* q, uint32_t n, uint32_t nprobe, uint32_t k, float* dist, uint64_t* ids) {
        PendingSearch r{q, n, nprobe, k, dist, ids};
        {
            // not `mu`: the dispatcher takes that to enqueue a batch, and callers must be
            // able to queue meanwhile
            std::lock_guard<std::mutex> g(co_init_mu);
            start_coalescer();
        }
        std::unique_lock<std::mutex> lk(co->m);
        co->queue.push_back(&r);
        co->wake.notify_one();
        co->done.wait(lk, [&] { return r.rc != 1; });
        if (r.rc != VDB_OK) throw VdbError(r.rc, r.err);
    }

    // Wait for every search still in flight on any stream before the index changes
    // under it (buffers freed, lists moved, centroids rewritten).
    void quiesce() {
        for (auto& sl : slots)
            if (sl.used) HIPCHECK(hipEventSynchronize(sl.done));
    }

    // Upload the list directory and recompute the segment-count prefix.
    void upload_directory() {
        quiesce();
        // Segment size: the largest of 512/256/128/64 vectors that still cuts this
        // handle's lists into >= 4096 segments, so a shard of an 8-GPU node keeps
        // enough scan work items for load balance (measured on a 1/8 shard of the
        // 10M x 768 index: 256 beats 512 by 5 % and 64 by 9 %).
        uint64_t local = 0;
        for (uint32_t l = 0; l < nlist; ++l) local += owned[l] ? count[l] : 0;
        if (seg_blocks_opt) {
            seg_blocks = seg_blocks_opt;
        } else {
            seg_blocks = 8;  // 512 vectors at most by default (1024 is an explicit option)
            // (The screen keeps 512 at every shard size. 256-vector segments in items of 4 made
            // the 1/8 shard's one-in-flight scan faster (0.549 vs 0.575 ms) but its batches at
            // 3 in flight slower (0.47 vs 0.41 ms per step over the 8 emulated ranks: more
            // items, partials and merge work per batch), so throughput keeps 512.)
            const bool screen_may = screen_opt && metric != 2;
            while (!screen_may && seg_blocks > 1 && local / ((uint64_t)seg_blocks * 64) < 4096) seg_blocks >>= 1;
        }
        std::vector<uint32_t> cl(nlist), cg(nlist), ns(nlist);
        storable_n = 0;
        for (uint32_t l = 0; l < nlist; ++l) {
            require(count[l] < (1ull << 32), "list longer than 2^32 vectors", VDB_ERR_UNSUPPORTED);
            cg[l] = (uint32_t)count[l];
            cl[l] = owned[l] ? (uint32_t)count[l] : 0u;
            storable_n += cl[l] > 0;
            ns[l] = (uint32_t)cdiv(cl[l], (uint64_t)seg_blocks * 64);
        }
        upload_scan_directory(stream);
        HIPCHECK(hipMemcpyAsync(d_count_local.ensure(nlist), cl.data(), nlist * 4, hipMemcpyHostToDevice, stream));
        HIPCHECK(hipMemcpyAsync(d_count_global.ensure(nlist), cg.data(), nlist * 4, hipMemcpyHostToDevice, stream));
        HIPCHECK(hipMemcpyAsync(d_nseg.ensure(nlist), ns.data(), nlist * 4, hipMemcpyHostToDevice, stream));
        // Screened items: a wave carries its top-k across the segments it takes from one item,
        // so items of long lists take more segments (its thresholds tighten over more
        // vectors); short lists keep 4 for parallelism. By the size-weighted mean segment
        // count of the stored lists (measured: iid 10M x 768, 40 per list: 8; the 1/8 shard
        // of 100M x 768, ~200: 16; the mixture, 5: 4).
        {
            double wsum = 0.0, wseg = 0.0;
            for (uint32_t l = 0; l < nlist; ++l) {
                wsum += cl[l];
                wseg += (double)cl[l] * ns[l];
            }
            const double mean_seg = wsum > 0 ? wseg / wsum : 0.0;
            screen_segs_auto = mean_seg < 16.0 ? 4u : (mean_seg < 96.0 ? 8u : 16u);
        }
        std::vector<uint32_t> sorted(ns);
        std::sort(sorted.begin(), sorted.end(), std::greater<uint32_t>());
        nseg_prefix.assign(nlist + 1, 0);
        for (uint32_t j = 0; j < nlist; ++j) nseg_prefix[j + 1] = nseg_prefix[j] + sorted[j];
        HIPCHECK(hipStreamSynchronize(stream));  // host vectors above are stack-owned
        screen_stale = true;  // rebuilt by the next search (a bulk add appends in many calls)
    }

    // The interleaved arena back from the row-major copy (identical contents: the copy holds
    // every slot of every block, pads included) plus its zeroed slack block.
    void ensure_arena() {
        if (!arena_dropped) return;
        quiesce();
        const size_t vec4 = (size_t)(arena_blocks + 1) * d4 * 64;
        arena.ensure(vec4);
        HIPCHECK(hipMemsetAsync(arena.p + (size_t)arena_blocks * d4 * 64, 0, (size_t)d4 * 64 * sizeof(float4), stream));
        vdbk::launch_interleave(screen_rows.p, arena_blocks * 64, dp, arena.p, stream);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipStreamSynchronize(stream));
        arena_dropped = false;
    }
    // Drop the screen's data (the arena made whole first: the rows may be its only copy).
    void screen_release() {
        ensure_arena();
        screen_ready = false;
        screen_sh.release();
        screen_rows.release();
        screen_meta.release();
        screen_scale.release();
        screen_blist.release();
        screen_ids.release();
        d_sblock_off.release();
        sblocks = 0;
    }

    // (Re)build the screened scan's data from the arena, or drop it. Called by the first
    // search after the lists or centroids change (every search issued before the change
    // was quiesced by it, and none since has read the data) and by the options that
    // decide whether it exists.
    void screen_update() {
        screen_stale = false;
        ensure_arena();  // (the build reads the arena)
        screen_ready = false;
        // (Config::max_gpu_memory caps the resident list bytes, as the reference's
        // gpu_memory_used_ does; the screen's shadow is not list data and is not counted)
        if (tiered()) {
            screen_update_tier();
            return;
        }
        const bool want = screen_opt && metric != 2 && !arena.host && arena_blocks > 0;
        if (!want) {
            screen_release();
            return;
        }
        std::vector<uint32_t> blist(arena_blocks, 0);
        for (uint32_t l = 0; l < nlist; ++l)
            if (owned[l])
                for (uint64_t b = 0; b < list_blocks(l); ++b) blist[block_off[l] + b] = l;
        for (bool i8 = want_i8();; i8 = false) {
            if (i8 != screen_fmt_i8) {  // (a shadow of the other format: its buffers are sized for that)
                screen_sh.release();
                screen_scale.release();
            }
            screen_fmt_i8 = i8;
            try {
                screen_sh.ensure(vdbk::screen_shadow_u4(arena_blocks, d4, i8));
                // (+ one slack block: the exact scans' tile pipeline reads one block past a segment)
                screen_rows.ensure((size_t)(arena_blocks + 1) * 64 * dp);
                screen_meta.ensure((size_t)arena_blocks * 64);
                screen_blist.ensure(arena_blocks);
                if (i8) screen_scale.ensure((size_t)arena_blocks * 64);
            } catch (const VdbError&) {  // no room for it: the exact scan serves
                (void)hipGetLastError();
                screen_release();
                return;
            }
            HIPCHECK(hipMemcpyAsync(screen_blist.p, blist.data(), arena_blocks * 4, hipMemcpyHostToDevice, stream));
            HIPCHECK(hipMemsetAsync(screen_rows.p + (size_t)arena_blocks * 64 * dp, 0, (size_t)64 * dp * 4, stream));
            vdbk::launch_screen_build(arena.p, arena_blocks, d4, screen_blist.p, cent_rm.p, screen_sh.p, screen_rows.p,
                                      screen_meta.p, stream, i8 ? screen_scale.p : nullptr);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipStreamSynchronize(stream));
            screen_ready = true;
            floor.reset_state();  // (trips of a previous shadow say nothing about this one)
            if (!i8 || screen_i8 != 2 || screen_calibrate()) break;
            i8_vetoed = true;  // (the automatic format: int8 re-checks too much here, bf16 instead)
        }
        // the row-major copy is now the lists' fp32 copy: release the arena
        arena.release();
        arena_dropped = true;
    }

    // The automatic shadow format's calibration (option screen_i8 = 2), at the build: one
    // screened batch of (up to) 64 of the index's own vectors (one from each of 64 blocks spread
    // over the lists) as queries, at the nprobe of the search that triggered the build and k = 10.
    // int8 stays unless its survivors beyond k per valid (query, list) pair exceed
    // kCalibPpm of the (query, vector) pairs, or the candidates overflowed: a regime where
    // its ~5x wider bound re-checks more rows than its half-size stream saves (the two-level
    // mixture: 6.2 % and 44.4K vs 52.2K QPS; iid data: 0.3 %, 27.3K vs 25.3K).
    static constexpr uint64_t kCalibPpm = 15000;
    bool screen_calibrate() {
        const uint32_t P = std::min<uint32_t>(nlist, last_P ? last_P : 32), k = 10;
        // (at most one batch's queries at this nprobe: the plan kernel takes kPlanMaxPairs pairs)
        const uint32_t B = std::min<uint32_t>(64, batch_cap(P, k));
        if (!arena_blocks || vdbk::topk_regs(k) != 1) return true;
        DevBuf<float> q, od;
        DevBuf<uint64_t> oi;
        q.ensure((size_t)B * dim);
        od.ensure((size_t)B * k);
        oi.ensure((size_t)B * k);
        for (uint32_t j = 0; j < B; ++j) {  // (slot 0 of a block always holds a vector)
            const uint64_t slot = (uint64_t)(j * arena_blocks / B) * 64;
            HIPCHECK(hipMemcpyAsync(q.p + (size_t)j * dim, screen_rows.p + slot * dp, (size_t)dim * 4,
                                    hipMemcpyDeviceToDevice, stream));
        }
        SearchSlot w;
        ensure_workspace(w, B, P, k);
        if (!stats.p) {
            stats.ensure(16);
            HIPCHECK(hipMemsetAsync(stats.p, 0, 128, stream));
        }
        HIPCHECK(hipMemsetAsync(w.carry_i.p, 0xFF, (size_t)P * k * 8, stream));
        const bool prof0 = prof;
        prof = false;
        calibrating = true;  // (no floor report: the calibration batch never trips the floor)
        try {
            run_batch(w, q.p, B, P, k, od.p, oi.p, stream, nullptr, 0);
        } catch (...) {
            prof = prof0;
            calibrating = false;
            throw;
        }
        prof = prof0;
        calibrating = false;
        uint32_t hc[vdbk::kCounters];
        HIPCHECK(hipMemcpyAsync(hc, w.counters.p, sizeof(hc), hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        const uint64_t surv = hc[vdbk::kCtrSurv], pairs = hc[vdbk::kCtrPairs], kvalid = (uint64_t)k * hc[vdbk::kCtrValid];
        const bool overflow = hc[vdbk::kCtrOvf] != 0;
        calib_excess_ppm = pairs ? (surv > kvalid ? surv - kvalid : 0) * 1000000ull / pairs : 0;
        return !overflow && calib_excess_ppm <= kCalibPpm;
    }
    uint64_t calib_excess_ppm = 0;
    bool calibrating = false;

    // The tier's screen: shadow + norms + ids of every stored list in HBM (the deferred scan
    // only: its re-checks read the survivors' rows from the home). Host home: built from the
    // page-locked arena over PCIe. File home: the lists streamed through the io_uring read
    // pipeline once, a group of lists at a time, into a device block buffer, built from there.
    void screen_update_tier() {
        screen_release();
        if (!(screen_opt && screen_defer && metric != 2 && dp % 64 == 0)) return;
        sblock_off.assign(nlist, 0);
        uint64_t nb = 0;
        for (uint32_t l = 0; l < nlist; ++l) {
            if (!owned[l] || count[l] == 0) continue;
            sblock_off[l] = file_home() ? nb : block_off[l];
            nb = std::max<uint64_t>(nb, sblock_off[l] + list_blocks(l));
        }
        if (nb == 0) return;
        std::vector<uint32_t> blist(nb, 0);
        for (uint32_t l = 0; l < nlist; ++l)
            if (owned[l] && count[l])
                for (uint64_t b = 0; b < list_blocks(l); ++b) blist[sblock_off[l] + b] = l;
        const bool i8 = want_i8();
        screen_fmt_i8 = i8;
        try {
            screen_sh.ensure(vdbk::screen_shadow_u4(nb, d4, i8));
            if (i8) screen_scale.ensure((size_t)nb * 64);
            screen_meta.ensure((size_t)nb * 64);
            screen_blist.ensure(nb);
            screen_ids.ensure((size_t)(nb + 1) * 64);
            d_sblock_off.ensure(nlist);
        } catch (const VdbError&) {  // no room: the tier's exact path serves
            (void)hipGetLastError();
            screen_release();
            return;
        }
        HIPCHECK(hipMemcpyAsync(screen_blist.p, blist.data(), nb * 4, hipMemcpyHostToDevice, stream));
        HIPCHECK(hipMemcpyAsync(d_sblock_off.p, sblock_off.data(), nlist * 8, hipMemcpyHostToDevice, stream));
        if (!file_home()) {
            vdbk::launch_screen_build(arena.p, nb, d4, screen_blist.p, cent_rm.p, screen_sh.p, nullptr, screen_meta.p,
                                      stream, i8 ? screen_scale.p : nullptr);
            HIPCHECK(hipMemcpyAsync(screen_ids.p, arena_ids.p, nb * 64 * 8, hipMemcpyHostToDevice, stream));
        } else {
            // groups of consecutive stored lists through a device block buffer of <= 1 GiB
            const uint64_t gcap = std::max<uint64_t>(cdiv(*std::max_element(count.begin(), count.end()), 64),
                                                     (1ull << 30) / ((uint64_t)d4 * 64 * 16 + 512));
            DevBuf<float4> tv;
            DevBuf<uint64_t> ti;
            tv.ensure((gcap + 1) * d4 * 64);
            ti.ensure((gcap + 1) * 64);
            std::vector<std::pair<uint32_t, uint64_t>> loads;
            uint64_t g0 = 0, gend = 0;
            auto flush = [&]() {
                if (loads.empty()) return;
                HIPCHECK(hipMemsetAsync(tv.p, 0, (gend - g0) * d4 * 64 * sizeof(float4), stream));
                load_lists(loads, stream, tv.p, ti.p);
                vdbk::launch_screen_build(tv.p, gend - g0, d4, screen_blist.p + g0, cent_rm.p,
                                          screen_sh.p + g0 * (uint64_t)d4 * (i8 ? 16 : 32), nullptr, screen_meta.p + g0 * 64,
                                          stream, i8 ? screen_scale.p + g0 * 64 : nullptr);
                HIPCHECK(hipGetLastError());
                HIPCHECK(hipMemcpyAsync(screen_ids.p + g0 * 64, ti.p, (gend - g0) * 64 * 8, hipMemcpyDeviceToDevice,
                                        stream));
                HIPCHECK(hipStreamSynchronize(stream));  // (the buffers are refilled by the next group)
                loads.clear();
            };
            for (uint32_t l = 0; l < nlist; ++l) {
                if (!owned[l] || count[l] == 0) continue;
                if (!loads.empty() && sblock_off[l] + list_blocks(l) - g0 > gcap) flush();
                if (loads.empty()) g0 = sblock_off[l];
                loads.push_back({l, sblock_off[l] - g0});
                gend = sblock_off[l] + list_blocks(l);
            }
            flush();
            sblist_host = blist;
        }
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipStreamSynchronize(stream));
        sblocks = nb;
        screen_ready = true;
        if (file_home() && tier_row_cache) fill_row_cache();
    }

    // Screened tier, file home: the k <= 64 searches never use the list cache, so it is filled
    // with lists whose survivors' rows are then copied from HBM instead of read from the
    // file: by default the largest stored lists (on iid data also the most probed); with
    // weights (vdb_ivf_fill_row_cache: per list its expected survivor rows, e.g. the
    // histogram of the batches served so far, vdb_ivf_survivor_histogram) the lists that save
    // the most row reads per cached byte, by weight / length. The lists stay ordinary cached
    // lists: a k > 64 search may evict them.
    std::vector<double> row_cache_weight;  // (empty: by size)
    std::vector<uint64_t> surv_hist;       // per list: survivor rows of the tier's screened batches
    void fill_row_cache() {
        if (!cache_blocks) return;
        std::vector<uint32_t> order;
        for (uint32_t l = 0; l < nlist; ++l)
            if (owned[l] && count[l] && cache_off[l] == kAbsent) order.push_back(l);
        if (row_cache_weight.size() == nlist)
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
                const double wx = row_cache_weight[x] / (double)count[x], wy = row_cache_weight[y] / (double)count[y];
                return wx != wy ? wx > wy : count[x] > count[y];
            });
        else
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return count[x] > count[y]; });
        std::vector<std::pair<uint32_t, uint64_t>> loads;
        for (uint32_t l : order) {
            const uint64_t off = cache_alloc(list_blocks(l));
            if (off == kAbsent) continue;  // (a smaller list may still fit)
            cache_off[l] = off;
            ++resident_n;
            ++cache_loads;
            cache_bytes_in += list_blocks(l) * block_bytes(dp);
            loads.push_back({l, off});
        }
        if (loads.empty()) return;
        load_lists(loads, stream);
        upload_scan_directory(stream);
        HIPCHECK(hipStreamSynchronize(stream));
    }

    // Tier, file home: after the deferred scan's selection, read the survivors' rows of the
    // batch from the file (one read each, io_uring on the buffered descriptor: hot rows stay in
    // the page cache) into page-locked staging, copy them to the device and pad them to dp.
    // Returns the rows ([survivor][dp]) for the exact pass, or nullptr when the candidate
    // buffer overflowed (the caller re-runs the batch with a larger one).
    const float* fetch_survivor_rows(SearchSlot& w, uint32_t cap, uint32_t& need, hipStream_t s) {
        uint32_t hc[vdbk::kCounters];
        HIPCHECK(hipMemcpyAsync(hc, w.counters.p, sizeof(hc), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        if (hc[vdbk::kCtrOvf]) {  // (some candidate fell beyond the buffer; need: the slots reserved)
            need = hc[vdbk::kCtrCand];
            return nullptr;
        }
        const uint32_t n = hc[vdbk::kCtrSurv];
        fetch_surv.resize(n);
        if (n) HIPCHECK(hipMemcpyAsync(fetch_surv.data(), w.surv.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        fetch_stage.host = true;
        float* st = fetch_stage.ensure((size_t)std::max<uint32_t>(n, 1) * dim);
        if (row_uring && row_uring->capacity() < tier_row_qd) row_uring.reset();
        if (!row_uring) row_uring.reset(new UringReader(tier_row_qd));
        UringReader* const ur = row_uring.get();
        const uint64_t row_bytes = (uint64_t)dim * 4;
        // O_DIRECT (where the file system allows it): each read is the 4 KiB-aligned superset
        // of the row into a bounce slot, copied out on completion; else a buffered read
        // straight into the staging
        const bool direct = tier_row_direct && home_fd_direct >= 0;
        const uint32_t kQD = std::min(tier_row_qd, row_uring->capacity());
        const uint64_t span = ((row_bytes + 4095) / 4096 + 1) * 4096;
        char* bounce = nullptr;
        if (direct) {
            fetch_bounce.host = true;
            bounce = fetch_bounce.ensure(kQD * span + 4096);
            bounce = (char*)(((uintptr_t)bounce + 4095) & ~(uintptr_t)4095);
        }
        std::vector<uint32_t> slot_of(kQD), free_slots(kQD);
        for (uint32_t i = 0; i < kQD; ++i) free_slots[i] = kQD - 1 - i;
        std::vector<uint64_t> delta(kQD);
        uint64_t bytes_read = 0;
        // rows of lists in the HBM cache are copied from there (after the upload below); the
        // rest: one read per distinct row (a row surviving for several queries is read once),
        // issued in file order, the duplicates copied from the first reader's staging row
        cache_src_host.clear();
        std::vector<uint32_t> order;
        order.reserve(n);
        if (surv_hist.size() != nlist) surv_hist.assign(nlist, 0);
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t slot = fetch_surv[i].x;
            const uint32_t l = sblist_host[slot >> 6];
            ++surv_hist[l];
            if (tier_row_cache && !cache_off.empty() && cache_off[l] != kAbsent)
                cache_src_host.push_back({(unsigned long long)i,
                                          (unsigned long long)(cache_off[l] * 64 + (slot - sblock_off[l] * 64))});
            else
                order.push_back(i);
        }
        const uint32_t nf = (uint32_t)order.size();
        std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
            return fetch_surv[x].x != fetch_surv[y].x ? fetch_surv[x].x < fetch_surv[y].x : x < y;
        });
        std::vector<uint32_t> uniq;
        std::vector<std::pair<uint32_t, uint32_t>> dups;  // (survivor, survivor holding its row)
        uniq.reserve(nf);
        for (uint32_t t = 0; t < nf; ++t) {
            if (t && fetch_surv[order[t]].x == fetch_surv[order[t - 1]].x) dups.push_back({order[t], uniq.back()});
            else uniq.push_back(order[t]);
        }
        const uint32_t nu = (uint32_t)uniq.size();
        uint32_t next = 0, done = 0;
        try {
            while (done < nu) {
                while (next < nu && next - done < kQD) {  // (<= kQD queued or in flight)
                    const uint32_t si = uniq[next];
                    const uint64_t slot = fetch_surv[si].x;
                    const uint32_t l = sblist_host[slot >> 6];
                    const uint64_t r = slot - sblock_off[l] * 64;
                    const uint64_t off = file_off[l] + count[l] * 8 + r * row_bytes;
                    if (direct) {
                        const uint32_t b = free_slots.back();
                        free_slots.pop_back();
                        const uint64_t g = dio_align;  // (the file system's O_DIRECT granule)
                        const uint64_t a0 = off / g * g, a1 = (off + row_bytes + g - 1) / g * g;
                        delta[b] = off - a0;
                        slot_of[b] = si;
                        ur->read(home_fd_direct, bounce + (size_t)b * span, (uint32_t)(a1 - a0), a0,
                                 ((uint64_t)b << 32) | si);
                        bytes_read += a1 - a0;
                    } else {
                        ur->read(home_fd, st + (size_t)si * dim, (uint32_t)row_bytes, off, si);
                        bytes_read += row_bytes;
                    }
                    ++next;
                }
                for (const UringReader::Done& d : ur->wait(1)) {
                    const uint32_t b = (uint32_t)(d.tag >> 32), i = (uint32_t)d.tag;
                    const int64_t want = direct ? (int64_t)(delta[b] + row_bytes) : (int64_t)row_bytes;
                    require(d.result >= want,
                            "short read of a survivor row from the list file" +
                                (d.result < 0 ? std::string(": ") + std::strerror((int)-d.result) : ""),
                            VDB_ERR_STATE);
                    if (direct) {
                        std::memcpy(st + (size_t)i * dim, bounce + (size_t)b * span + delta[b], row_bytes);
                        free_slots.push_back(b);
                    }
                    ++done;
                }
            }
        } catch (...) {
            ur->drain();
            throw;
        }
        for (const auto& d : dups) std::memcpy(st + (size_t)d.first * dim, st + (size_t)d.second * dim, row_bytes);
        screen_rows_fetched += nu;
        screen_row_bytes += (uint64_t)nu * row_bytes;
        screen_rows_cached += cache_src_host.size();
        file_bytes_read += bytes_read;  // (with O_DIRECT: the aligned supersets the device delivered)
        float* rows = slot_buf(w, w.srows, (size_t)std::max<uint32_t>(n, 1) * dp);
        if (n) {
            if (dim == dp) {
                HIPCHECK(hipMemcpyAsync(rows, st, (size_t)n * row_bytes, hipMemcpyHostToDevice, s));
            } else {
                HIPCHECK(hipMemcpyAsync(fetch_dev.ensure((size_t)n * dim), st, (size_t)n * row_bytes,
                                        hipMemcpyHostToDevice, s));
                vdbk::launch_pad_rows(fetch_dev.p, n, dim, dp, rows, s);
                HIPCHECK(hipGetLastError());
            }
        }
        if (!cache_src_host.empty()) {  // (overwrites those rows' unused staging content)
            // (a k > 64 call may have loaded lists into the cache asynchronously: its loads end
            // before its last sub-batch, whose completion tier_call_ev marks)
            if (tier_call_used) HIPCHECK(hipEventSynchronize(tier_call_ev));
            const uint32_t nc = (uint32_t)cache_src_host.size();
            HIPCHECK(hipMemcpyAsync(cache_src.ensure(nc), cache_src_host.data(), (size_t)nc * sizeof(ulonglong2),
                                    hipMemcpyHostToDevice, s));
            vdbk::launch_gather_cache_rows(cache.p, d4, cache_src.p, nc, rows, s);
            HIPCHECK(hipGetLastError());
        }
        HIPCHECK(hipStreamSynchronize(s));  // (the staging and the cache's contents are reused later)
        return rows;
    }

    // Tier, file home, TWO-PASS re-check (option screen_recheck2): read the rows of the batch's
    // survivors marked `phase` (1: pass A, each pair's k smallest lower bounds; 2: pass B, the
    // others not above pass A's k-th exact distance; launch_tier_recheck) into the slot's
    // compact device rows, after those of the earlier phase; a row needed again (the same
    // vector surviving for another query, or in both phases) is read once. Rows of lists in the
    // HBM cache are copied from there. The survivor -> row map is uploaded. Phase 1 returns
    // false (need: the reserved candidate slots) when the candidate buffer overflowed: the
    // caller re-runs the batch with a larger one.
    std::vector<uint8_t> fetch_mark;
    std::vector<uint32_t> fetch_rowmap;
    std::unordered_map<uint64_t, uint32_t> fetch_slot_row;
    uint32_t fetch_n = 0, fetch_rows_n = 0;
    bool fetch_rows_phase(SearchSlot& w, int phase, uint32_t& need, hipStream_t s) {
        if (phase == 1) {
            uint32_t hc[vdbk::kCounters];
            HIPCHECK(hipMemcpyAsync(hc, w.counters.p, sizeof(hc), hipMemcpyDeviceToHost, s));
            HIPCHECK(hipStreamSynchronize(s));
            if (hc[vdbk::kCtrOvf]) {
                need = hc[vdbk::kCtrCand];
                return false;
            }
            fetch_n = hc[vdbk::kCtrSurv];
            fetch_surv.resize(fetch_n);
            if (fetch_n) HIPCHECK(hipMemcpyAsync(fetch_surv.data(), w.surv.p, (size_t)fetch_n * 8, hipMemcpyDeviceToHost, s));
            fetch_rows_n = 0;
            fetch_slot_row.clear();
            fetch_rowmap.assign(fetch_n, 0u);
        }
        const uint32_t n = fetch_n;
        fetch_mark.resize(n);
        if (n) HIPCHECK(hipMemcpyAsync(fetch_mark.data(), w.smark.p, n, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        if (surv_hist.size() != nlist) surv_hist.assign(nlist, 0);
        // this phase's survivors: a slot read before maps to its row; new slots get rows j0 ..
        const uint32_t j0 = fetch_rows_n;
        std::vector<uint32_t> todo;  // (a survivor per new slot)
        for (uint32_t i = 0; i < n; ++i) {
            if (fetch_mark[i] != (uint8_t)phase) continue;
            const uint64_t slot = fetch_surv[i].x;
            ++surv_hist[sblist_host[slot >> 6]];
            auto it = fetch_slot_row.find(slot);
            if (it != fetch_slot_row.end()) {
                fetch_rowmap[i] = it->second;
                continue;
            }
            const uint32_t j = fetch_rows_n++;
            fetch_slot_row.emplace(slot, j);
            fetch_rowmap[i] = j;
            todo.push_back(i);
        }
        const uint32_t nn = fetch_rows_n - j0;
        fetch_stage.host = true;
        float* st = fetch_stage.ensure((size_t)std::max<uint32_t>(nn, 1) * dim);
        if (row_uring && row_uring->capacity() < tier_row_qd) row_uring.reset();
        if (!row_uring) row_uring.reset(new UringReader(tier_row_qd));
        UringReader* const ur = row_uring.get();
        const uint64_t row_bytes = (uint64_t)dim * 4;
        const bool direct = tier_row_direct && home_fd_direct >= 0;
        const uint32_t kQD = std::min(tier_row_qd, row_uring->capacity());
        const uint64_t span = ((row_bytes + 4095) / 4096 + 1) * 4096;
        char* bounce = nullptr;
        if (direct) {
            fetch_bounce.host = true;
            bounce = fetch_bounce.ensure(kQD * span + 4096);
            bounce = (char*)(((uintptr_t)bounce + 4095) & ~(uintptr_t)4095);
        }
        // cached lists' rows from HBM; the rest read in file order
        cache_src_host.clear();
        std::vector<uint32_t> order;  // (positions in todo)
        order.reserve(todo.size());
        for (uint32_t t = 0; t < (uint32_t)todo.size(); ++t) {
            const uint64_t slot = fetch_surv[todo[t]].x;
            const uint32_t l = sblist_host[slot >> 6];
            if (tier_row_cache && !cache_off.empty() && cache_off[l] != kAbsent)
                cache_src_host.push_back({(unsigned long long)(j0 + t),
                                          (unsigned long long)(cache_off[l] * 64 + (slot - sblock_off[l] * 64))});
            else
                order.push_back(t);
        }
        std::sort(order.begin(), order.end(),
                  [&](uint32_t x, uint32_t y) { return fetch_surv[todo[x]].x < fetch_surv[todo[y]].x; });
        std::vector<uint32_t> slot_of(kQD), free_slots(kQD);
        for (uint32_t b = 0; b < kQD; ++b) free_slots[b] = kQD - 1 - b;
        std::vector<uint64_t> delta(kQD);
        uint64_t bytes_read = 0;
        const uint32_t nf = (uint32_t)order.size();
        uint32_t next = 0, done = 0;
        try {
            while (done < nf) {
                while (next < nf && next - done < kQD) {
                    const uint32_t t = order[next];
                    const uint64_t slot = fetch_surv[todo[t]].x;
                    const uint32_t l = sblist_host[slot >> 6];
                    const uint64_t off = file_off[l] + count[l] * 8 + (slot - sblock_off[l] * 64) * row_bytes;
                    if (direct) {
                        const uint32_t b = free_slots.back();
                        free_slots.pop_back();
                        const uint64_t g = dio_align;
                        const uint64_t a0 = off / g * g, a1 = (off + row_bytes + g - 1) / g * g;
                        delta[b] = off - a0;
                        slot_of[b] = t;
                        ur->read(home_fd_direct, bounce + (size_t)b * span, (uint32_t)(a1 - a0), a0, ((uint64_t)b << 32) | t);
                        bytes_read += a1 - a0;
                    } else {
                        ur->read(home_fd, st + (size_t)t * dim, (uint32_t)row_bytes, off, t);
                        bytes_read += row_bytes;
                    }
                    ++next;
                }
                for (const UringReader::Done& d : ur->wait(1)) {
                    const uint32_t b = (uint32_t)(d.tag >> 32), t = (uint32_t)d.tag;
                    const int64_t want = direct ? (int64_t)(delta[b] + row_bytes) : (int64_t)row_bytes;
                    require(d.result >= want,
                            "short read of a survivor row from the list file" +
                                (d.result < 0 ? std::string(": ") + std::strerror((int)-d.result) : ""),
                            VDB_ERR_STATE);
                    if (direct) {
                        std::memcpy(st + (size_t)t * dim, bounce + (size_t)b * span + delta[b], row_bytes);
                        free_slots.push_back(b);
                    }
                    ++done;
                }
            }
        } catch (...) {
            ur->drain();
            throw;
        }
        screen_rows_fetched += nf;
        screen_row_bytes += (uint64_t)nf * row_bytes;
        screen_rows_cached += cache_src_host.size();
        file_bytes_read += bytes_read;
        float* rows = slot_buf(w, w.srows, (size_t)std::max<uint32_t>(n, 1) * dp);
        if (nn) {
            if (dim == dp) {
                HIPCHECK(hipMemcpyAsync(rows + (size_t)j0 * dp, st, (size_t)nn * row_bytes, hipMemcpyHostToDevice, s));
            } else {
                HIPCHECK(hipMemcpyAsync(fetch_dev.ensure((size_t)std::max<uint32_t>(n, 1) * dim), st, (size_t)nn * row_bytes,
                                        hipMemcpyHostToDevice, s));
                vdbk::launch_pad_rows(fetch_dev.p, nn, dim, dp, rows + (size_t)j0 * dp, s);
                HIPCHECK(hipGetLastError());
            }
        }
        if (!cache_src_host.empty()) {  // (overwrites those rows' unused staging content)
            if (tier_call_used) HIPCHECK(hipEventSynchronize(tier_call_ev));
            const uint32_t nc = (uint32_t)cache_src_host.size();
            HIPCHECK(hipMemcpyAsync(cache_src.ensure(nc), cache_src_host.data(), (size_t)nc * sizeof(ulonglong2),
                                    hipMemcpyHostToDevice, s));
            vdbk::launch_gather_cache_rows(cache.p, d4, cache_src.p, nc, rows, s);
            HIPCHECK(hipGetLastError());
        }
        if (n) HIPCHECK(hipMemcpyAsync(w.rowmap.p, fetch_rowmap.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
        HIPCHECK(hipStreamSynchronize(s));  // (the staging, the map and the cache's contents are reused later)
        return true;
    }

    // Rebuild the arena so list l holds `keep[l]` of its current blocks at new
    // offsets sized for `new_count[l]` vectors (0 for lists this handle drops).
    void relayout(const std::vector<uint64_t>& new_count, const std::vector<uint8_t>& new_owned) {
        relayout(new_count, new_owned, arena.host);
    }
    void relayout(const std::vector<uint64_t>& new_count, const std::vector<uint8_t>& new_owned, bool host_arena) {
        quiesce();
        // the screen's data describes the old lists: drop it before the new arena is
        // allocated (peak HBM old + new arena, not that plus the shadow and rows); the next
        // search rebuilds it
        screen_release();
        screen_stale = true;
        std::vector<uint64_t> new_off(nlist, 0), old_off(nlist, 0);
        std::vector<uint32_t> nblocks(nlist, 0);
        uint64_t blocks = 0;
        for (uint32_t l = 0; l < nlist; ++l) {
            new_off[l] = blocks;
            if (new_owned[l]) blocks += cdiv(new_count[l], 64);
            if (owned[l] && new_owned[l] && count[l] > 0) {
                nblocks[l] = (uint32_t)cdiv(count[l], 64);
                old_off[l] = block_off[l];
            }
        }
        DevBuf<float4> na{!host_arena};
        DevBuf<uint64_t> ni{!host_arena};
        na.host = ni.host = host_arena;
        // one slack block past the last list: the scan prefetches one chunk and one
        // block of ids beyond the segment it streams
        const size_t vec4 = (size_t)(blocks + 1) * d4 * 64;
        na.ensure(vec4);
        ni.ensure((size_t)(blocks + 1) * 64);
        if (blocks) {
            HIPCHECK(hipMemsetAsync(na.p, 0, vec4 * sizeof(float4), stream));
            HIPCHECK(hipMemsetAsync(ni.p, 0xFF, (size_t)(blocks + 1) * 64 * 8, stream));
        }
        if (arena_blocks && blocks) {
            DevBuf<uint64_t> doo, dno;
            DevBuf<uint32_t> dnb;
            HIPCHECK(hipMemcpyAsync(doo.ensure(nlist), old_off.data(), nlist * 8, hipMemcpyHostToDevice, stream));
            HIPCHECK(hipMemcpyAsync(dno.ensure(nlist), new_off.data(), nlist * 8, hipMemcpyHostToDevice, stream));
            HIPCHECK(hipMemcpyAsync(dnb.ensure(nlist), nblocks.data(), nlist * 4, hipMemcpyHostToDevice, stream));
            vdbk::launch_copy_lists(arena.p, arena_ids.p, doo.p, dno.p, dnb.p, nlist, d4, na.p, ni.p, stream);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipStreamSynchronize(stream));
        }
        HIPCHECK(hipStreamSynchronize(stream));
        arena.swap(na);
        arena_ids.swap(ni);
        arena_blocks = blocks;
        block_off = new_off;
        owned = new_owned;
        cache_reset();  // list contents or offsets changed: nothing cached stays valid
    }

    // ---- list-cache tier ----
    bool tiered() const { return cache_blocks > 0; }
    uint64_t list_blocks(uint32_t l) const { return cdiv(count[l], 64); }
    static uint64_t block_bytes(uint32_t dp_) { return 64ull * ((uint64_t)dp_ * 4 + 8); }

    void cache_reset() {
        cache_off.assign(nlist, kAbsent);
        last_use.assign(nlist, 0);
        free_ext.clear();
        if (cache_blocks) free_ext[0] = cache_blocks;
        cache_used = 0;
        resident_n = 0;
    }

    uint64_t cache_alloc(uint64_t nb) {  // first fit
        for (auto it = free_ext.begin(); it != free_ext.end(); ++it) {
            if (it->second < nb) continue;
            const uint64_t off = it->first, len = it->second;
            free_ext.erase(it);
            if (len > nb) free_ext[off + nb] = len - nb;
            cache_used += nb;
            return off;
        }
        return kAbsent;
    }

    void cache_free(uint32_t l) {
        const uint64_t nb = list_blocks(l);
        auto it = free_ext.emplace(cache_off[l], nb).first;
        cache_off[l] = kAbsent;
        cache_used -= nb;
        --resident_n;
        auto nx = std::next(it);
        if (nx != free_ext.end() && it->first + it->second == nx->first) {
            it->second += nx->second;
            free_ext.erase(nx);
        }
        if (it != free_ext.begin()) {
            auto pv = std::prev(it);
            if (pv->first + pv->second == it->first) {
                pv->second += it->second;
                free_ext.erase(it);
            }
        }
    }

    // Scan directory: home offsets, or cache offsets in the tier (absent lists: 0,
    // never read: a list is made resident before any batch that probes it is planned).
    void upload_scan_directory(hipStream_t s) {
        const uint64_t* src = block_off.data();
        if (tiered()) {
            // the previous upload's source must have been read before it is rewritten
            if (tier_ev_used) HIPCHECK(hipEventSynchronize(tier_ev));
            dir_stage.host = true;
            uint64_t* st = dir_stage.ensure(nlist);
            for (uint32_t l = 0; l < nlist; ++l) st[l] = cache_off[l] == kAbsent ? 0 : cache_off[l];
            src = st;
        }
        HIPCHECK(hipMemcpyAsync(d_block_off.ensure(nlist), src, nlist * 8, hipMemcpyHostToDevice, s));
        if (!tiered()) {
            HIPCHECK(hipStreamSynchronize(s));  // src is the host vector
            return;
        }
        if (!tier_ev) HIPCHECK(hipEventCreateWithFlags(&tier_ev, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(tier_ev, s));  // covers the loads queued on s before it
        tier_ev_used = true;
    }

    // Cache residency planning. Lists that are empty or not stored here are never
    // cached. `want` (unique lists) must all be resident afterwards; lists marked in
    // `protect` are never evicted; a victim is the cached list whose next use (rank()
    // : larger = later, UINT64_MAX = never) is furthest away, then the least recently
    // used. Returns false, changing nothing, when `want` cannot be placed (over capacity,
    // or fragmentation with `repack` off); with `repack` every cached list outside `want`
    // is dropped and `want` is re-laid from offset 0 when fragmentation blocks a load.
    // The cache map changes at once; the data moves with load_lists, in stream order.
    template <class Rank>
    bool plan_loads(const std::vector<uint32_t>& want, const std::vector<uint8_t>& protect, Rank&& rank, bool repack,
                    std::vector<std::pair<uint32_t, uint64_t>>& loads) {
        loads.clear();
        uint64_t need = 0;
        std::vector<uint32_t> miss;
        for (uint32_t l : want) {
            need += list_blocks(l);
            if (cache_off[l] == kAbsent) miss.push_back(l);
        }
        if (need > cache_blocks) return false;
        if (miss.empty()) return true;
        auto by_size = [&](uint32_t a, uint32_t b) { return count[a] != count[b] ? count[a] > count[b] : a < b; };
        std::vector<uint32_t> victims;
        for (uint32_t l = 0; l < nlist; ++l)
            if (cache_off[l] != kAbsent && !protect[l]) victims.push_back(l);
        std::vector<uint64_t> rk(nlist, 0);
        for (uint32_t v : victims) rk[v] = rank(v);
        std::sort(victims.begin(), victims.end(), [&](uint32_t a, uint32_t b) {
            if (rk[a] != rk[b]) return rk[a] > rk[b];
            return last_use[a] != last_use[b] ? last_use[a] < last_use[b] : a < b;
        });
        // dry run on a copy of the extent map, so a failed plan changes nothing
        const std::map<uint64_t, uint64_t> free_save = free_ext;
        const std::vector<uint64_t> off_save = cache_off;
        const uint64_t used_save = cache_used, res_save = resident_n;
        std::sort(miss.begin(), miss.end(), by_size);
        size_t vi = 0;
        uint64_t evicted = 0;
        for (size_t m = 0; m < miss.size(); ++m) {
            const uint32_t l = miss[m];
            uint64_t off;
            while ((off = cache_alloc(list_blocks(l))) == kAbsent && vi < victims.size()) {
                cache_free(victims[vi++]);
                ++evicted;
            }
            if (off == kAbsent) {
                if (!repack) {  // undo: the caller falls back to a later, synchronous load
                    free_ext = free_save;
                    cache_off = off_save;
                    cache_used = used_save;
                    resident_n = res_save;
                    loads.clear();
                    return false;
                }
                // fragmented: keep only `want`, packed from offset 0 (they fit)
                for (uint32_t v = 0; v < nlist; ++v)
                    if (cache_off[v] != kAbsent) cache_free(v);
                miss = want;
                std::sort(miss.begin(), miss.end(), by_size);
                loads.clear();
                m = (size_t)-1;
                continue;
            }
            cache_off[l] = off;
            ++resident_n;
            loads.push_back({l, off});
        }
        cache_evictions += evicted;
        cache_loads += loads.size();
        for (auto& ld : loads) cache_bytes_in += list_blocks(ld.first) * block_bytes(dp);
        return true;
    }

    // Unique cacheable lists of a probe array.
    std::vector<uint32_t> cacheable(const uint32_t* lists, size_t n, std::vector<uint8_t>& mark) {
        std::vector<uint32_t> out;
        for (size_t i = 0; i < n; ++i) {
            const uint32_t l = lists[i];
            if (l >= nlist || mark[l] || !owned[l] || count[l] == 0) continue;
            mark[l] = 1;
            out.push_back(l);
        }
        for (uint32_t l : out) mark[l] = 0;
        return out;
    }

    // Make `lists` resident on stream s (warmup and single lists): LRU eviction.
    // False if together they exceed the cache.
    bool make_resident(const uint32_t* lists, size_t n, hipStream_t s) {
        ++use_tick;
        std::vector<uint8_t> mark(nlist, 0);
        const std::vector<uint32_t> want = cacheable(lists, n, mark);
        for (uint32_t l : want) last_use[l] = use_tick;
        std::vector<uint8_t> protect(nlist, 0);
        for (uint32_t l : want) protect[l] = 1;
        bool miss = false;
        for (uint32_t l : want) miss |= cache_off[l] == kAbsent;
        if (miss) quiesce();  // searches on other streams may still read the lists evicted below
        std::vector<std::pair<uint32_t, uint64_t>> loads;
        if (!plan_loads(want, protect, [](uint32_t) { return uint64_t(0); }, true, loads)) return false;
        if (loads.empty()) return true;
        load_lists(loads, s);
        upload_scan_directory(s);
        return true;
    }

    bool file_home() const { return home_fd >= 0; }

    void pread_all(void* dst, size_t bytes, uint64_t off) {
        char* p = (char*)dst;
        while (bytes) {
            const ssize_t r = ::pread(home_fd, p, bytes, (off_t)off);
            require(r > 0, "short read from the list file", VDB_ERR_STATE);
            p += r;
            bytes -= (size_t)r;
            off += (uint64_t)r;
            file_bytes_read += (uint64_t)r;
        }
    }

    // Copy planned lists into their cache blocks, ordered on stream s. Host-memory home:
    // one DMA per list. File home: every list is cut into chunks of whole 64-row blocks;
    // each chunk's ids and rows are read (io_uring, up to kStages chunks in flight) into
    // a page-locked staging buffer, copied to HBM, padded to dp and interleaved into the
    // cache's block layout; a buffer is refilled once its copies have landed.
    void load_lists(const std::vector<std::pair<uint32_t, uint64_t>>& loads, hipStream_t s,
                    float4* dst_v = nullptr, uint64_t* dst_i = nullptr) {
        float4* const tv = dst_v ? dst_v : cache.p;  // (the cache, or a caller's block buffer)
        uint64_t* const ti = dst_i ? dst_i : cache_ids.p;
        if (!file_home()) {
            for (auto& ld : loads) {
                const uint32_t l = ld.first;
                const uint64_t off = ld.second, nb = list_blocks(l);
                HIPCHECK(hipMemcpyAsync(tv + off * d4 * 64, arena.p + block_off[l] * d4 * 64,
                                        nb * d4 * 64 * sizeof(float4), hipMemcpyHostToDevice, s));
                HIPCHECK(hipMemcpyAsync(ti + off * 64, arena_ids.p + block_off[l] * 64, nb * 64 * 8,
                                        hipMemcpyHostToDevice, s));
            }
            return;
        }
        const uint64_t rows = std::max<uint64_t>(64, ((32ull << 20) / ((uint64_t)dim * 4)) / 64 * 64);
        const size_t ids_cap = (rows * 8 + 8192 + 4095) / 4096 * 4096;
        const size_t vec_cap = (rows * dim * 4 + 8192 + 4095) / 4096 * 4096;
        if (!uring) uring.reset(new UringReader(64));
        for (Stage& st : stages) {
            if (!st.copied) HIPCHECK(hipEventCreateWithFlags(&st.copied, hipEventDisableTiming));
            st.buf.host = true;
            st.buf.ensure(ids_cap + vec_cap);
        }
        // loads on the copy stream may overlap loads on a search stream: separate device staging
        DevBuf<float>& rows_d = s == copy_stream ? drows_cs : drows;
        DevBuf<float>& pad_d = s == copy_stream ? dpad_cs : dpad;
        rows_d.ensure(rows * dim);
        pad_d.ensure(rows * dp);
        struct Chunk {
            uint32_t l;
            uint64_t r0, m, dst_block;
        };
        std::vector<Chunk> chunks;
        for (auto& ld : loads)
            for (uint64_t r0 = 0; r0 < count[ld.first]; r0 += rows)
                chunks.push_back({ld.first, r0, std::min(rows, count[ld.first] - r0), ld.second + r0 / 64});
        const bool direct = home_fd_direct >= 0;
        // one read; with O_DIRECT the aligned superset of [off, off + len)
        auto read_into = [&](int si, char* dst, uint64_t off, uint64_t len, int part) -> size_t {
            const uint64_t tag = ((uint64_t)si << 1) | (uint64_t)part;
            if (!direct) {
                uring->read(home_fd, dst, (uint32_t)len, off, tag);
                return 0;
            }
            const uint64_t a0 = off & ~4095ull, a1 = (off + len + 4095) & ~4095ull;
            uring->read(home_fd_direct, dst, (uint32_t)(a1 - a0), a0, tag);
            return (size_t)(off - a0);
        };
        size_t next = 0;
        int reading = 0;
        try {
            while (next < chunks.size() || reading > 0) {
                for (int si = 0; si < kStages && next < chunks.size(); ++si) {
                    Stage& st = stages[si];
                    if (st.reads) continue;
                    if (st.copying) {
                        const hipError_t q = hipEventQuery(st.copied);
                        if (q == hipErrorNotReady) continue;
                        HIPCHECK(q);
                        st.copying = false;
                    }
                    const Chunk& c = chunks[next++];
                    const uint64_t base = file_off[c.l];
                    st.m = c.m;
                    st.dst_block = c.dst_block;
                    st.ids_delta = read_into(si, st.buf.p, base + c.r0 * 8, c.m * 8, 0);
                    st.vec_delta = read_into(si, st.buf.p + ids_cap, base + count[c.l] * 8 + c.r0 * dim * 4, c.m * dim * 4, 1);
                    st.reads = 2;
                    ++reading;
                    file_bytes_read += c.m * 8 + c.m * dim * 4;
                }
                if (reading == 0) {  // every buffer waits for its copies: wait for one
                    for (Stage& st : stages)
                        if (st.copying) {
                            HIPCHECK(hipEventSynchronize(st.copied));
                            st.copying = false;
                            break;
                        }
                    continue;
                }
                for (const UringReader::Done& d : uring->wait(1)) {
                    Stage& st = stages[d.tag >> 1];
                    const bool vec = d.tag & 1;
                    const int64_t want = (int64_t)((vec ? st.vec_delta : st.ids_delta) + st.m * (vec ? (uint64_t)dim * 4 : 8));
                    require(d.result >= want, "short read from the list file" +
                                                  (d.result < 0 ? std::string(": ") + std::strerror((int)-d.result) : ""),
                            VDB_ERR_STATE);
                    if (--st.reads) continue;
                    --reading;
                    HIPCHECK(hipMemcpyAsync(ti + st.dst_block * 64, st.buf.p + st.ids_delta, st.m * 8,
                                            hipMemcpyHostToDevice, s));
                    HIPCHECK(hipMemcpyAsync(rows_d.p, st.buf.p + ids_cap + st.vec_delta, st.m * dim * 4,
                                            hipMemcpyHostToDevice, s));
                    HIPCHECK(hipEventRecord(st.copied, s));
                    st.copying = true;
                    vdbk::launch_pad_rows(rows_d.p, st.m, dim, dp, pad_d.p, s);
                    vdbk::launch_interleave(pad_d.p, st.m, dp, tv + st.dst_block * d4 * 64, s);
                    HIPCHECK(hipGetLastError());
                }
            }
        } catch (...) {
            // A failed read (or submission) leaves other reads in flight: reap them and
            // reset the staging ring, and forget the cache map (the lists planned for this
            // load may be partly written), so the next load starts clean.
            uring->drain();
            for (Stage& st : stages) st.reads = 0;
            cache_reset();
            throw;
        }
    }

    // Serve the lists from an index file (vdb_ivf_save format) through the tier.
    void open_lists(const char* path) {
        require(tiered(), "open_lists needs the list-cache tier (set list_cache_bytes first)", VDB_ERR_STATE);
        quiesce();
        const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
        require(fd >= 0, std::string("cannot open ") + path, VDB_ERR_STATE);
        if (home_fd >= 0) ::close(home_fd);
        if (home_fd_direct >= 0) ::close(home_fd_direct);
        home_fd = fd;
        // lists are read with O_DIRECT where the file system allows it (no page-cache copy)
        home_fd_direct = ::open(path, O_RDONLY | O_CLOEXEC | O_DIRECT);
        dio_align = 4096;
        if (home_fd_direct >= 0) {  // (a 512-B read at a 512-B offset: accepted or EINVAL)
            void* pb = nullptr;
            if (posix_memalign(&pb, 4096, 4096) == 0) {
                if (::pread(home_fd_direct, pb, 512, 512) == 512) dio_align = 512;
                std::free(pb);
            }
        }
        char magic[8];
        uint32_t hdr[6] = {0, 0, 0, 0, 0, 0};
        pread_all(magic, 8, 0);
        const bool shard_file = std::memcmp(magic, "VDBIVS01", 8) == 0;  // (vdb_ivf_save of a sharded handle)
        pread_all(hdr, shard_file ? 24 : 16, 8);
        auto refuse = [&](const std::string& why) {
            ::close(home_fd);
            home_fd = -1;
            if (home_fd_direct >= 0) ::close(home_fd_direct);
            home_fd_direct = -1;
            throw VdbError(VDB_ERR_INVALID_ARGUMENT, why);
        };
        if ((!shard_file && std::memcmp(magic, "VDBIVF01", 8) != 0) || hdr[0] != dim || hdr[1] != nlist ||
            (int)hdr[2] != metric)
            refuse("index file does not match this index's configuration");
        if (shard_file && (hdr[4] == 0 || hdr[3] >= hdr[4])) refuse("shard file with an invalid (rank, world)");
        const uint64_t hdr_bytes = shard_file ? 32 : 24;
        std::vector<float> c((size_t)nlist * dim);
        pread_all(c.data(), c.size() * 4, hdr_bytes);
        uint64_t at = hdr_bytes + (uint64_t)c.size() * 4;
        std::vector<uint64_t> cnt(nlist, 0), stored(nlist, 0), off(nlist, 0);
        for (uint32_t l = 0; l < nlist; ++l) {
            uint64_t h2[2] = {0, 0};
            pread_all(h2, shard_file ? 16 : 8, at);
            cnt[l] = h2[0];
            stored[l] = shard_file ? h2[1] : h2[0];
            off[l] = at + (shard_file ? 16 : 8);
            at = off[l] + stored[l] * 8 + stored[l] * (uint64_t)dim * 4;
        }
        std::vector<uint8_t> own(nlist, 1);
        if (shard_file) {  // a list is this rank's when the file stores its rows (any plan)
            for (uint32_t l = 0; l < nlist; ++l) {
                if (stored[l] != 0 && stored[l] != cnt[l]) refuse("shard file stores part of a list");
                own[l] = cnt[l] != 0 && stored[l] == cnt[l];
            }
        }
        HIPCHECK(hipMemcpy2DAsync(cent_rm.p, dp * 4, c.data(), dim * 4, dim * 4, nlist, hipMemcpyHostToDevice, stream));
        refresh_centroid_layout();
        file_off = off;
        count = cnt;
        total = 0;
        for (uint32_t l = 0; l < nlist; ++l) total += cnt[l];
        screen_ready = false;  // (everything is replaced: no arena rebuild for the old lists)
        arena_dropped = false;
        screen_sh.release();
        screen_rows.release();
        screen_meta.release();
        screen_blist.release();
        arena.release();  // no home copy in memory: the file is the home
        arena_ids.release();
        arena_blocks = 0;
        block_off.assign(nlist, 0);
        owned = own;
        rank = shard_file ? hdr[3] : 0;
        world = shard_file ? hdr[4] : 1;
        cache_reset();
        upload_directory();
    }

    // Turn the tier on (bytes > 0: HBM cache of that many bytes, arena moved to host
    // memory) or off (arena back in HBM).
    void set_list_cache(uint64_t bytes) {
        quiesce();
        const uint64_t nb = bytes / block_bytes(dp);
        require(bytes == 0 || nb > 0, "list_cache_bytes is below one block of 64 vectors");
        require(nb > 0 || !file_home(), "lists served from a file need the list-cache tier", VDB_ERR_STATE);
        cache.release();
        cache_ids.release();
        cache_blocks = 0;
        if (!file_home() && (nb > 0) != arena.host) relayout(count, owned, nb > 0);  // moves the arena
        cache_blocks = nb;
        if (nb) {  // one slack block: the scan prefetches past a segment's end
            cache.ensure((nb + 1) * d4 * 64);
            cache_ids.ensure((nb + 1) * 64);
        }
        cache_reset();
        upload_directory();
    }

    // Config::max_gpu_memory: the reference caps the bytes of GPU-resident lists
    // (count * (dim * 4 + 8) each, gpu_memory_used_) and searches lists beyond the cap on
    // the CPU (ivf_flat_index.cpp:398-402, 526-530). Here, once the stored lists outgrow
    // the cap, the handle switches to the list-cache tier with an HBM cache of that many
    // bytes: lists home in page-locked host memory and the lists a batch probes are made
    // resident before it scans, so results are unchanged. 0 = no cap.
    uint64_t stored_list_bytes(const std::vector<uint64_t>& cnt) const {
        uint64_t b = 0;
        for (uint32_t l = 0; l < nlist; ++l)
            if (owned[l]) b += cnt[l] * ((uint64_t)dim * 4 + 8);
        return b;
    }
    bool tier_by_cap = false;  // the tier was entered because the lists outgrew max_gpu_memory
    void apply_memory_cap(const std::vector<uint64_t>& cnt) {
        if (file_home()) return;
        if (tier_by_cap && (max_gpu_memory == 0 || stored_list_bytes(cnt) <= max_gpu_memory)) {
            set_list_cache(0);  // the cap was lifted or raised above the lists: back to HBM
            tier_by_cap = false;
            return;
        }
        if (max_gpu_memory == 0 || max_gpu_memory == ~0ull || tiered()) return;
        if (stored_list_bytes(cnt) <= max_gpu_memory) return;
        require(max_gpu_memory >= block_bytes(dp),
                "max_gpu_memory is below one block of 64 vectors (set 0 for no cap)", VDB_ERR_OUT_OF_MEMORY);
        set_list_cache(max_gpu_memory);
        tier_by_cap = true;
    }

    // Row-major [n][dim] device input -> zero-padded [n][dp] (or the input itself).
    const float* padded_rows(const float* d_v, uint64_t n, DevBuf<float>& tmp) {
        if (dp == dim) return d_v;
        vdbk::launch_pad_rows(d_v, n, dim, dp, tmp.ensure(n * dp), stream);
        HIPCHECK(hipGetLastError());
        return tmp.p;
    }

    // Caller holds mu. Host centroids [nlist][dim] in (zero pads kept).
    void set_centroids_host(const float* c) {
        quiesce();
        HIPCHECK(hipMemcpy2DAsync(cent_rm.p, dp * 4, c, dim * 4, dim * 4, nlist, hipMemcpyHostToDevice, stream));
        refresh_centroid_layout();
        HIPCHECK(hipStreamSynchronize(stream));
    }

    // Caller holds mu. Append host rows to the given lists (input order per list).
    void add_to_lists_host(const float* v, const uint64_t* ids, const uint32_t* lists, uint64_t n) {
        if (n == 0) return;
        for (uint64_t i = 0; i < n; ++i) require(lists[i] < nlist, "list id out of range");
        DevBuf<float> dv, tmp;
        DevBuf<uint64_t> di;
        DevBuf<uint32_t> dl;
        HIPCHECK(hipMemcpyAsync(dv.ensure(n * dim), v, n * dim * 4, hipMemcpyHostToDevice, stream));
        HIPCHECK(hipMemcpyAsync(di.ensure(n), ids, n * 8, hipMemcpyHostToDevice, stream));
        HIPCHECK(hipMemcpyAsync(dl.ensure(n), lists, n * 4, hipMemcpyHostToDevice, stream));
        append(padded_rows(dv.p, n, tmp), di.p, dl.p, n);
        HIPCHECK(hipStreamSynchronize(stream));
    }

    // Caller holds mu. Centroids row-major [nlist][dim] into host memory.
    void export_centroids(float* c) {
        HIPCHECK(hipMemcpy2DAsync(c, dim * 4, cent_rm.p, dp * 4, dim * 4, nlist, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
    }

    // Caller holds mu. List l row-major (count x dim) with its ids, in add order.
    void export_list(uint32_t l, float* vectors, uint64_t* ids) {
        const uint64_t c = count[l];
        if (c == 0) return;
        require(owned[l], "list is not stored on this shard", VDB_ERR_STATE);
        if (file_home()) {  // the file holds the list row-major, as returned
            if (ids) pread_all(ids, c * 8, file_off[l]);
            if (vectors) pread_all(vectors, c * dim * 4, file_off[l] + c * 8);
            return;
        }
        if (arena_dropped) {  // the row-major copy holds the list in slot (= add) order
            if (vectors)
                HIPCHECK(hipMemcpy2DAsync(vectors, (size_t)dim * 4, screen_rows.p + block_off[l] * 64 * dp, (size_t)dp * 4,
                                          (size_t)dim * 4, c, hipMemcpyDeviceToHost, stream));
            if (ids) HIPCHECK(hipMemcpyAsync(ids, arena_ids.p + block_off[l] * 64, c * 8, hipMemcpyDeviceToHost, stream));
            HIPCHECK(hipStreamSynchronize(stream));
            return;
        }
        DevBuf<float> dv;
        DevBuf<uint64_t> di;
        vdbk::launch_export_list(arena.p, arena_ids.p, block_off[l], (uint32_t)c, dim, d4, dv.ensure(c * dim),
                                 di.ensure(c), stream);
        HIPCHECK(hipGetLastError());
        if (vectors) HIPCHECK(hipMemcpyAsync(vectors, dv.p, c * dim * 4, hipMemcpyDeviceToHost, stream));
        if (ids) HIPCHECK(hipMemcpyAsync(ids, di.p, c * 8, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
    }

    void refresh_centroid_layout() {
        quiesce();
        vdbk::launch_interleave(cent_rm.p, nlist, dp, cent_il.p, stream);
        HIPCHECK(hipGetLastError());
        screen_stale = true;  // the shadow holds residuals against the centroids
    }

    // assign_to_lists (cpp:259-295): exact argmin with ties to the lowest centroid. For
    // L2 / IP it is the coarse step's top-1: MFMA distance bounds, then the exact
    // sequential distances of every centroid that can still be the minimum
    // (ivf_assign_rerank: candidates whose lower bound <= the smallest upper bound; NaN
    // orders last, so an all-NaN row goes to list 0 as with the strict '<').
    // Rows are processed in chunks whose bound matrices fit a fixed workspace.
    void assign(const float* vpad, uint64_t n, uint32_t* out) {
        if (coarse_mode == 1 && metric != 2 && vdbk::rerank_rows(dp, 1) > 0) {
            const uint64_t budget = 1024ull << 20;  // bytes of the two bound matrices per chunk
            uint64_t chunk = std::max<uint64_t>(256, budget / ((uint64_t)nlist * 8) / 16 * 16);
            chunk = std::min<uint64_t>(chunk, n);
            DevBuf<float> ap, de;
            ap.ensure(chunk * nlist);
            de.ensure(chunk * nlist);
            for (uint64_t r0 = 0; r0 < n; r0 += chunk) {
                const uint32_t b = (uint32_t)std::min<uint64_t>(chunk, n - r0);
                vdbk::launch_coarse_mfma(metric, cent_rm.p, nlist, dp, vpad + r0 * dp, b, ap.p, de.p, stream);
                vdbk::launch_assign_rerank(metric, ap.p, de.p, cent_rm.p, nlist, dp, vpad + r0 * dp, b, out + r0, stream);
                HIPCHECK(hipGetLastError());
            }
            HIPCHECK(hipStreamSynchronize(stream));  // the chunk buffers are freed on return
            return;
        }
        vdbk::launch_assign(metric, vpad, n, dp, cent_il.p, nlist, out, stream);
        HIPCHECK(hipGetLastError());
    }

    // Stable grouping of row indices by key (input order kept within a key).
    void group_by_key(const uint32_t* keys, uint64_t n, DevBuf<uint32_t>& sorted_keys, DevBuf<uint32_t>& order) {
        require(n < (1ull << 31), "batch larger than 2^31 vectors", VDB_ERR_UNSUPPORTED);
        DevBuf<uint32_t> iota;
        vdbk::launch_iota(iota.ensure(n), n, stream);
        int bits = 1;
        while ((1ull << bits) < nlist) ++bits;
        size_t tb = 0;
        HIPCHECK(vdbk::radix_sort_pairs(nullptr, tb, keys, sorted_keys.ensure(n), iota.p, order.ensure(n), n, bits, stream));
        DevBuf<unsigned char> temp;
        temp.ensure(tb);
        HIPCHECK(vdbk::radix_sort_pairs(temp.p, tb, keys, sorted_keys.p, iota.p, order.p, n, bits, stream));
        HIPCHECK(hipStreamSynchronize(stream));
    }

    std::vector<uint32_t> key_counts(const uint32_t* keys, uint64_t n, DevBuf<uint32_t>& d_counts) {
        HIPCHECK(hipMemsetAsync(d_counts.ensure(nlist), 0, nlist * 4, stream));
        vdbk::launch_histogram(keys, n, d_counts.p, stream);
        HIPCHECK(hipGetLastError());
        std::vector<uint32_t> h(nlist);
        HIPCHECK(hipMemcpyAsync(h.data(), d_counts.p, nlist * 4, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        return h;
    }

    // ---- train: ivf_flat_index.cpp:49-145 ----
    void train(const float* d_v, uint64_t n) {
        require(n > 0, "train needs at least one vector");
        DevBuf<float> tmp, mind;
        const float* vpad = padded_rows(d_v, n, tmp);
        DevBuf<float4> v_il;
        vdbk::launch_interleave(vpad, n, dp, v_il.ensure(cdiv(n, 64) * d4 * 64), stream);
        HIPCHECK(hipGetLastError());

        std::mt19937 gen(42);
        std::uniform_int_distribution<uint64_t> pick(0, n - 1);
        const uint64_t first = pick(gen);
        HIPCHECK(hipMemcpyAsync(cent_rm.p, vpad + first * dp, dp * 4, hipMemcpyDeviceToDevice, stream));

        vdbk::launch_mindist_init(mind.ensure(n), n, stream);
        // The min-distance update (n x dim work) runs on the device; the two serial
        // float sums of cpp:87 and cpp:95-96 (n dependent adds each, inherently
        // sequential) run on the host over a pinned copy, in the reference's order.
        PinnedBuf<float> hmind(n);
        for (uint32_t c = 1; c < nlist; ++c) {
            vdbk::launch_mindist_update(v_il.p, n, d4, cent_rm.p + (size_t)(c - 1) * dp, mind.p, stream);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipMemcpyAsync(hmind.p, mind.p, n * sizeof(float), hipMemcpyDeviceToHost, stream));
            HIPCHECK(hipStreamSynchronize(stream));
            const float* md = hmind.p;
            float tot = 0.0f;
            for (uint64_t v = 0; v < n; ++v) tot += md[v];
            std::uniform_real_distribution<float> prob(0.0f, tot);
            const float target = prob(gen);
            float cumsum = 0.0f;
            for (uint64_t v = 0; v < n; ++v) {
                cumsum += md[v];
                if (cumsum >= target) {
                    HIPCHECK(hipMemcpyAsync(cent_rm.p + (size_t)c * dp, vpad + v * dp, dp * sizeof(float),
                                            hipMemcpyDeviceToDevice, stream));
                    break;
                }
            }
        }

        DevBuf<uint32_t> asg, skeys, order, counts, offsets;
        asg.ensure(n);
        for (int it = 0; it < 10; ++it) {
            refresh_centroid_layout();
            assign(vpad, n, asg.p);
            group_by_key(asg.p, n, skeys, order);
            std::vector<uint32_t> h = key_counts(asg.p, n, counts);
            std::vector<uint32_t> off(nlist, 0);
            for (uint32_t l = 1; l < nlist; ++l) off[l] = off[l - 1] + h[l - 1];
            HIPCHECK(hipMemcpyAsync(offsets.ensure(nlist), off.data(), nlist * 4, hipMemcpyHostToDevice, stream));
            vdbk::launch_centroid_update(vpad, dp, order.p, offsets.p, counts.p, nlist, dim, cent_rm.p, stream);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipStreamSynchronize(stream));
        }
        refresh_centroid_layout();
        HIPCHECK(hipStreamSynchronize(stream));
    }

    // ---- add: ivf_flat_index.cpp:148-202 ----
    void add(const float* d_v, const uint64_t* d_ids, uint64_t n) {
        if (n == 0) return;
        require(!file_home(), "lists are served from a file (vdb_ivf_open_lists): the index is read-only",
                VDB_ERR_STATE);
        DevBuf<float> tmp;
        const float* vpad = padded_rows(d_v, n, tmp);
        DevBuf<uint32_t> asg;
        assign(vpad, n, asg.ensure(n));
        append(vpad, d_ids, asg.p, n);
    }

    // Append rows to the given lists, keeping input order within each list
    // (cpp:160-192). `asg` holds one list id per row (device).
    void append(const float* vpad, const uint64_t* d_ids, const uint32_t* asg, uint64_t n) {
        require(!file_home(), "lists are served from a file (vdb_ivf_open_lists): the index is read-only",
                VDB_ERR_STATE);
        DevBuf<uint32_t> skeys, order, counts;
        group_by_key(asg, n, skeys, order);
        std::vector<uint32_t> added = key_counts(asg, n, counts);

        std::vector<uint64_t> new_count(count);
        for (uint32_t l = 0; l < nlist; ++l) new_count[l] += added[l];
        const std::vector<uint64_t> old_count = count;
        apply_memory_cap(new_count);  // (before the relayout: the arena moves home at most once)
        relayout(new_count, owned);

        std::vector<uint64_t> group_start(nlist, 0), base(nlist, ~0ull);
        for (uint32_t l = 1; l < nlist; ++l) group_start[l] = group_start[l - 1] + added[l - 1];
        for (uint32_t l = 0; l < nlist; ++l)
            if (owned[l]) base[l] = block_off[l] * 64 + old_count[l];
        DevBuf<uint64_t> d_gs, d_base, dest;
        HIPCHECK(hipMemcpyAsync(d_gs.ensure(nlist), group_start.data(), nlist * 8, hipMemcpyHostToDevice, stream));
        HIPCHECK(hipMemcpyAsync(d_base.ensure(nlist), base.data(), nlist * 8, hipMemcpyHostToDevice, stream));
        vdbk::launch_slots_from_order(skeys.p, n, d_gs.p, d_base.p, dest.ensure(n), stream);
        vdbk::launch_scatter_rows(vpad, d_ids, order.p, n, dp, dest.p, arena.p, arena_ids.p, stream);
        HIPCHECK(hipGetLastError());
        count = new_count;
        total += n;
        upload_directory();  // also waits for the stream before tmp buffers go
    }

    // owner: the plan (every list's rank), identical on every rank; null = the LPT plan
    // of vdb_shard_plan over the current list sizes.
    void set_shard(uint32_t r, uint32_t w, const uint32_t* owner_in = nullptr) {
        std::vector<uint32_t> owner(nlist);
        if (owner_in) std::copy(owner_in, owner_in + nlist, owner.begin());
        else vdb_shard_plan(count.data(), nlist, w, owner.data());
        std::vector<uint8_t> new_owned(nlist);
        for (uint32_t l = 0; l < nlist; ++l) {
            require(owner[l] < w, "shard plan names a rank outside the world");
            new_owned[l] = owner[l] == r;
        }
        // Lists this handle no longer scans must have been stored here before.
        for (uint32_t l = 0; l < nlist; ++l)
            require(!new_owned[l] || owned[l] || count[l] == 0, "shard needs a list this handle dropped", VDB_ERR_STATE);
        if (file_home()) {  // nothing in memory to move: the file holds every list
            quiesce();
            owned = new_owned;
            cache_reset();
        } else {
            relayout(count, new_owned);
        }
        rank = r;
        world = w;
        upload_directory();
    }

    // Group member: store exactly the lists `new_owned` marks (placement by the group).
    // A list may only move here while empty; lists leaving are dropped.
    void set_owned(const std::vector<uint8_t>& new_owned) {
        for (uint32_t l = 0; l < nlist; ++l)
            require(!new_owned[l] || owned[l] || count[l] == 0, "a placed list cannot move between members",
                    VDB_ERR_STATE);
        if (new_owned == owned) return;
        relayout(count, new_owned);
        upload_directory();
    }

    // Sharded build, for an index larger than one GPU (100M x 768 = 307 GB): the final
    // list sizes (from an assignment pass) fix this handle's lists before any add, so
    // appends store only the owned lists' rows and count the rest. The plan is the same
    // LPT as set_shard, so a later set_shard(r, w) keeps the same lists.
    void plan_shard(uint32_t r, uint32_t w, const uint64_t* final_sizes, const uint32_t* owner_in = nullptr) {
        require(total == 0, "plan_shard needs an empty index (call it between train and add)", VDB_ERR_STATE);
        require(!file_home(), "lists are served from a file (vdb_ivf_open_lists)", VDB_ERR_STATE);
        std::vector<uint32_t> owner(nlist);
        if (owner_in) std::copy(owner_in, owner_in + nlist, owner.begin());
        else vdb_shard_plan(final_sizes, nlist, w, owner.data());
        std::vector<uint8_t> new_owned(nlist);
        for (uint32_t l = 0; l < nlist; ++l) {
            require(owner[l] < w, "shard plan names a rank outside the world");
            new_owned[l] = owner[l] == r;
        }
        relayout(count, new_owned);
        rank = r;
        world = w;
        upload_directory();
    }

    // Probe census for a probe-weighted shard plan: counts[l] += how many of the n device
    // rows (a query-like sample) probe list l, by the exact probe selection of search.
    void probe_census(const float* d_rows, uint64_t n, uint32_t nprobe, uint64_t* counts) {
        const uint32_t P = std::min(nprobe, nlist);
        if (n == 0 || P == 0) return;
        quiesce();
        SearchSlot w;
        const uint32_t bmax = batch_cap(P, 1);
        ensure_workspace(w, (uint32_t)std::min<uint64_t>(bmax, n), P, 1);
        DevBuf<uint32_t> d_counts;
        HIPCHECK(hipMemsetAsync(d_counts.ensure(nlist), 0, nlist * 4, stream));
        for (uint64_t b0 = 0; b0 < n; b0 += bmax) {
            const uint32_t B = (uint32_t)std::min<uint64_t>(bmax, n - b0);
            coarse_batch(w, d_rows + b0 * dim, B, P, stream);
            vdbk::launch_histogram(w.probes.p, (uint64_t)B * P, d_counts.p, stream);
            HIPCHECK(hipGetLastError());
        }
        std::vector<uint32_t> h(nlist);
        HIPCHECK(hipMemcpyAsync(h.data(), d_counts.p, nlist * 4, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        for (uint32_t l = 0; l < nlist; ++l) counts[l] += h[l];
    }

    EventSet& next_events() {
        if (events_used == events.size()) {
            EventSet e;
            for (hipEvent_t* p : {&e.begin, &e.coarse_end, &e.scan_begin, &e.scan_end, &e.end, &e.x_end, &e.m_end,
                                  &e.collect_begin, &e.collect_end})
                HIPCHECK(hipEventCreate(p));
            events.push_back(e);
        }
        events[events_used].xchg = false;
        events[events_used].collected = false;
        return events[events_used++];
    }

    // Size every per-batch buffer of a slot for B queries up front; growing a buffer
    // frees the old one, so first wait for the slot's previous batch.
    void ensure_workspace(SearchSlot& w, uint32_t B, uint32_t P, uint32_t k) {
        const size_t BP = (size_t)B * P;
        const size_t max_items = (size_t)B * nseg_prefix[P];
        const size_t max_l1 = max_items / vdbk::kMergeFan + BP;
        const size_t max_wide = max_items / 4 + BP + 1;
        const bool grow = w.items_w.cap < max_wide || w.qpad.cap < (size_t)B * dp || w.cd.cap < (size_t)B * nlist ||
                          w.cdelta.cap < (size_t)B * nlist || w.cand.cap < (size_t)B * nlist ||
                          w.probes.cap < BP || w.thr.cap < BP || w.items.cap < max_items || w.part_d.cap < max_items * k ||
                          w.slot_d.cap < BP * k || w.carry_d.cap < (size_t)P * k || w.carry2_d.cap < (size_t)P * k ||
                          w.l1_items.cap < max_l1 ||
                          w.l1_d.cap < max_l1 * k;
        if (!grow) return;
        if (w.used) HIPCHECK(hipEventSynchronize(w.done));
        w.qpad.ensure((size_t)B * dp);
        w.cd.ensure((size_t)B * nlist);
        w.cdelta.ensure((size_t)B * nlist);
        w.cand.ensure((size_t)B * nlist);
        w.probes.ensure(BP);
        w.nseg_qp.ensure(BP);
        w.pbqp.ensure(BP);
        w.sorted_pair.ensure(BP);
        w.pbs.ensure(BP);
        w.counters.ensure(vdbk::kCounters);
        w.l1base.ensure(BP);
        w.thr.ensure(BP);
        w.l1_items.ensure(max_l1);
        w.l1_d.ensure(max_l1 * k);
        w.l1_i.ensure(max_l1 * k);
        w.items.ensure(max_items);
        w.items_w.ensure(max_wide);
        w.part_d.ensure(max_items * k);
        w.part_i.ensure(max_items * k);
        w.slot_d.ensure(BP * k);
        w.slot_i.ensure(BP * k);
        w.carry_d.ensure((size_t)P * k);
        w.carry_i.ensure((size_t)P * k);
        w.carry2_d.ensure((size_t)P * k);
        w.carry2_i.ensure((size_t)P * k);
    }

    // ---- search: ivf_flat_index.cpp:205-256, one batch of B queries ----
    // The batch's queries as the kernels read them, zero-padded rows [B][dp]: when dim is
    // already a multiple of the padding (768) the caller's rows are used in place (they
    // stay valid until the stream passes the search, as for any asynchronous call), else
    // a padded copy in w.qpad.
    void stage_queries(SearchSlot& w, const float* d_q, uint32_t B, hipStream_t s) {
        if (dim == dp && ((uintptr_t)d_q & 15) == 0) {  // (rows are read as float4)
            w.q = d_q;
            return;
        }
        vdbk::launch_pad_rows(d_q, B, dim, dp, w.qpad.p, s);
        w.q = w.qpad.p;
    }

    // Coarse step (select_nprobe_lists, cpp:298-336): padded queries into w.qpad, the
    // first min(nprobe, nlist) lists by (dist, list) into w.probes.
    void coarse_batch(SearchSlot& w, const float* d_q, uint32_t B, uint32_t P, hipStream_t s) {
        const int regs_p = vdbk::topk_regs(P);
        stage_queries(w, d_q, B, s);
        if (coarse_mode == 1 && metric != 2 && vdbk::rerank_rows(dp, regs_p) > 0) {
            vdbk::launch_coarse_mfma(metric, cent_rm.p, nlist, dp, w.q, B, w.cd.p, w.cdelta.p, s);
            vdbk::launch_select_rerank(metric, regs_p, w.cd.p, w.cdelta.p, cent_rm.p, nlist, dp, w.q, B, P,
                                       w.cand.p, w.probes.p, s);
        } else {
            vdbk::launch_coarse(metric, cent_il.p, nlist, d4, w.q, B, w.cd.p, s);
            vdbk::launch_select(regs_p, w.cd.p, nlist, B, P, w.probes.p, s);
        }
    }

    // Probe inversion, fine scan (search_list_cpu, cpp:339-384) and merges
    // (merge_results, cpp:474-518) of a batch whose padded queries are in w.qpad and
    // probes in w.probes.
    // Returns false (nothing merged) only for a screened batch of the tier's file home whose
    // candidates would need a buffer above tier_cand_max: the caller serves it through the
    // exact list-cache path instead (run_batch).
    bool scan_batch(SearchSlot& w, uint32_t B, uint32_t P, uint32_t k, float* out_d_, uint64_t* out_i_, hipStream_t s,
                    const uint32_t* req_start, uint32_t b0, EventSet* ev) {
        const int regs_k = vdbk::topk_regs(k);
        const uint32_t group = (uint32_t)vdbk::scan_group(regs_k);
        const uint32_t BP = B * P;
        const uint64_t max_items = (uint64_t)B * nseg_prefix[P];
        require(max_items < (1ull << 32), "batch too large", VDB_ERR_UNSUPPORTED);
        // (tier: lists and directory entries another stream loaded must have landed)
        if (tiered() && tier_ev_used) HIPCHECK(hipStreamWaitEvent(s, tier_ev, 0));
        const uint64_t max_l1 = max_items / vdbk::kMergeFan + BP;
        const uint64_t max_wide = max_items / 4 + BP + 1;
        last_P = P;
        if (screen_stale) screen_update();
        // the screened scan (default, L2 / IP, k <= 64): items of swq queries
        const uint32_t swq = screen_width(k, P);
        bool screened = swq != 0 && !force_exact;
        uint32_t floor_seq = 0;
        if (screened && !tiered() && screen_defer && !calibrating)  // the run-time floor (lists in HBM only)
            screened = floor.plan([this](uint32_t i) { return floor_entry(i); }, &floor_seq);
        // Exact scans on lists in HBM whose interleaved arena was released read the row-major
        // copy (4-wave items); the opt-in bounded scan needs the interleaved layout back.
        bool rows_l = !screened && arena_dropped && !tiered();
        if (rows_l && scan_mfma_min && regs_k == 1 && wide_scan && metric != 2) {
            ensure_arena();
            rows_l = false;
        }
        const int waves = wide_group == 32 && !rows_l ? 8 : 4;  // workgroup shape of the wide scan
        // (Cosine: every CPU-path distance is 0.0f, A5; its lists scan as narrow items only)
        const bool wide = regs_k == 1 && wide_scan && metric != 2 && vdbk::scan_wide_fits(d4, k, waves);
        // segments per item: one per wave (more adds tail latency, no throughput)
        const uint32_t segs_item = segs_item_opt ? segs_item_opt : (uint32_t)waves;
        // wide items of many queries: bounded on the matrix cores (L2 / IP, 16-query items)
        const uint32_t mfma_min = !screened && !rows_l && wide && waves == 4 && metric != 2 && !(VDB_SCAN_DIAG & 2) &&
                                          vdbk::scan_bounded_fits(d4, k)
                                      ? scan_mfma_min : 0u;
        const int plan_wide = screened ? (int)swq : (wide ? 4 * waves : 0);
        // (screened items: segs_per_item segments, default 4; a wave's top-k carries across
        // the segments it takes from one item)
        const uint32_t segs_screen = segs_item_opt ? segs_item_opt : screen_segs_auto;
        auto plan = [&](unsigned long long* st) {
            vdbk::launch_plan(w.probes.p, d_nseg.p, d_count_local.p, B, P, group, plan_wide, screened ? segs_screen : segs_item,
                              w.items.p, w.items_w.p, w.counters.p, w.sorted_pair.p, w.pbs.p, w.pbqp.p, w.nseg_qp.p,
                              w.l1base.p, w.l1_items.p, st, w.thr.p, mfma_min, s);
        };
        // (the automatic shadow's calibration batch counts into scratch: profile_read reports
        // the caller's batches only)
        plan(calibrating ? stats_scratch.ensure(16) : stats.p);
        const bool in_ring = &w >= slots && &w < slots + kSlots;
        if (scan_window && in_ring && scan_seq >= scan_window) {  // the scan issued scan_window batches ago
            const SearchSlot& prev = slots[scan_hist[(scan_seq - scan_window) % 8]];
            if (prev.scan_done) HIPCHECK(hipStreamWaitEvent(s, prev.scan_done, 0));
        }
        if (ev) HIPCHECK(hipEventRecord(ev->scan_begin, s));
        const float4* lists = tiered() ? cache.p : rows_l ? (const float4*)screen_rows.p : arena.p;
        vdbk::ScanArgs sa{lists, tiered() ? cache_ids.p : arena_ids.p, d_block_off.p, d_count_local.p, w.q, w.items.p, w.items_w.p,
                                w.counters.p, w.sorted_pair.p, w.pbs.p, w.part_d.p, w.part_i.p, d4, k,
                                wide_stride, w.counters.p + 4, seg_blocks, segs_item, 0, w.thr.p,
                                mfma_min, bounded_stats && !calibrating ? stats.p + 5 : nullptr};
        sa.rows_layout = rows_l ? 1u : 0u;
        // the bounded items first (the batch's most-probed lists), on the same stream
        if (mfma_min) vdbk::launch_scan_bounded(metric, (uint32_t)max_wide, sa, s);
        if (screened) {
            const bool defer = screen_defer;
            const bool i8s = defer && screen_fmt_i8;  // (int8 shadow: built only for the deferred scan)
            // (the tier's file home reads the survivors' rows on the host: the batch then
            // waits for its selection, and re-runs with a larger buffer if it overflowed)
            const bool tier_file = tiered() && file_home();
            // candidates at most: every (query, vector) pair the batch can have (B queries x the
            // P largest stored lists), capped by the option
            uint32_t ccap = (uint32_t)std::min<uint64_t>(
                screen_cand_cap, std::max<uint64_t>(1024, (uint64_t)B * nseg_prefix[P] * seg_blocks * 64));
            if (tier_file) ccap = std::max(ccap, tier_cand_cap);
            auto alloc_defer = [&]() {
                slot_buf(w, w.scnt, BP);
                slot_buf(w, w.ovf, BP);
                slot_buf(w, w.soff, (size_t)BP + 1);
                slot_buf(w, w.scand, ccap);
                slot_buf(w, w.surv, ccap);
                slot_buf(w, w.sdist, ccap);
                slot_buf(w, w.ubcnt, BP);
                slot_buf(w, w.ublist, (size_t)BP * vdbk::kUbLists * k);
                if (tier_file && screen_recheck2) {
                    slot_buf(w, w.slb, ccap);
                    slot_buf(w, w.smark, ccap);
                    slot_buf(w, w.rowmap, ccap);
                }
            };
            auto pairs = [&]() {
                vdbk::launch_screen_pairs(metric, w.q, B, P, w.probes.p, cent_rm.p, dp,
                                          slot_buf(w, w.qres, (size_t)BP * dp), slot_buf(w, w.pst, BP),
                                          slot_buf(w, w.thr4, (size_t)BP * 4), s, defer ? w.scnt.p : nullptr,
                                          defer ? w.ovf.p : nullptr, defer ? w.counters.p : nullptr,
                                          defer ? w.ubcnt.p : nullptr, i8s ? slot_buf(w, w.qscale, BP) : nullptr);
            };
            if (defer) alloc_defer();
            pairs();
            sa.thr4 = w.thr4.p;
            sa.shadow = screen_sh.p;
            sa.rows = screen_rows.p;
            sa.meta = screen_meta.p;
            sa.sscale = i8s ? screen_scale.p : nullptr;
            sa.qscale = i8s ? w.qscale.p : nullptr;
            sa.qres = w.qres.p;
            sa.pst = w.pst.p;
            sa.dp = dp;
            sa.P = P;
            sa.segs_item = segs_screen;
            sa.wide_q = swq;
            // (32-query items run one workgroup per CU, so a shared-threshold read's latency is
            // exposed: re-read every 4 blocks, cfg4 shard collect 4.14 -> 3.87 ms; 16-query
            // items hide it and keep the freshest value, 1/8 shard 0.543 vs 0.552 ms)
            sa.thr_every = screen_thr_every ? screen_thr_every : (swq == 32 ? 4u : 1u);
            if (tiered()) {  // the resident shadow's packing and ids; rows from the home
                sa.block_off = d_sblock_off.p;
                sa.ids = screen_ids.p;
                sa.rows = nullptr;
                sa.arena = file_home() ? nullptr : arena.p;  // (host home: page-locked, read over PCIe)
            }
            sa.fused = std::max<uint32_t>(1, std::min<uint32_t>(narrow_blocks, vdbk::kPersistentBlocks / 2));
            const uint64_t want = std::max<uint64_t>(max_wide, (max_items + 3) / 4);
            // (the persistent collect grid of 16-query items: 320 workgroups, 1.25 per CU, not 2:
            // the CU slots left over run the other batches in flight; measured on one box,
            // 320 / 352 / 384 / 512: headline 28.5K / 28.2K / 28.1K / 27.4K QPS, mixture 53.6K /
            // 53.9K / 54.0K / 52.0K, 1/8 shard at 3 in flight 184.5K / 182.7K / 181.8K / 174.4K)
            const uint64_t cap = scan_blocks ? scan_blocks : (swq == 32 ? vdbk::kPersistentBlocks / 2 : kCollectBlocks);
            const uint32_t grid = (uint32_t)std::min<uint64_t>(want, cap);
            if (defer) {
                const float* fetched = nullptr;
                const bool recheck2 = screen_recheck2 && !tiered();  // (rows in HBM, by slot)
                const bool tier2 = screen_recheck2 && tier_file;       // (rows from the file, two read phases)
                for (int pass = 0;; ++pass) {
                    if (pass) {  // a re-run after an overflow (tier, file home): plan and pairs reset the state
                        alloc_defer();
                        plan(stats_scratch.ensure(16));  // (statistics of the batch are counted once)
                        pairs();
                    }
                    sa.cand = w.scand.p;
                    sa.cand_cap = ccap;
                    sa.ccount = w.counters.p + vdbk::kCtrCand;
                    sa.ovf = w.ovf.p;
                    sa.ublist = w.ublist.p;
                    sa.ubcnt = w.ubcnt.p;
                    if (floor_seq) {  // (its own ring entry, whatever slot or stream runs it)
                        if (!floor_host.p) {
                            floor_host.host = true;
                            std::memset(floor_host.ensure(ScreenFloor::kRing), 0, ScreenFloor::kRing * sizeof(uint4));
                        }
                        sa.floor_out = floor_host.p + floor_seq % ScreenFloor::kRing;
                        sa.floor_seq = floor_seq;
                    }
                    sa.mstats = bounded_stats && !pass && !calibrating ? stats.p + 8 : nullptr;
                    if (stamps_cap) {
                        sa.stamps = stamps_buf.p;
                        sa.stamps_cap = stamps_cap;
                        sa.stamp_batch = stamp_batch++;
                    }
                    if (ev) HIPCHECK(hipEventRecord(ev->collect_begin, s));
                    vdbk::launch_screen_collect(metric, grid, sa, s);
                    if (ev) {
                        HIPCHECK(hipEventRecord(ev->collect_end, s));
                        ev->collected = true;
                    }
                    // (the two-pass re-check, rows in HBM: the survivors' lower bounds go where the
                    // one-pass path keeps their exact distances)
                    vdbk::launch_screen_select(sa, BP, w.scnt.p, w.soff.p, w.surv.p, w.ovf.p, s,
                                               recheck2 ? w.sdist.p : tier2 ? w.slb.p : nullptr);
                    if (!tier_file) break;
                    uint32_t need = 0;
                    if (tier2) {  // (pass A marked, its rows read; pass B after the loop)
                        vdbk::launch_tier_recheck(0, metric, sa, BP, w.nseg_qp.p, w.soff.p, w.scnt.p, w.surv.p, w.slb.p,
                                                  w.smark.p, nullptr, nullptr, nullptr, s);
                        if (fetch_rows_phase(w, 1, need, s)) {
                            fetched = w.srows.p;
                            break;
                        }
                    } else {
                        fetched = fetch_survivor_rows(w, ccap, need, s);
                        if (fetched) break;
                    }
                    const uint64_t grow = std::max<uint64_t>((uint64_t)need + need / 2, (uint64_t)ccap + 1024);
                    if (grow > std::max<uint64_t>(tier_cand_max, screen_cand_cap)) {
                        // (a regime where the bound is wider than the distance spread: the
                        // survivors' rows would cost more than the lists)
                        ++screen_tier_fallbacks;
                        return false;
                    }
                    ccap = (uint32_t)grow;
                    tier_cand_cap = ccap;  // (kept for the next batches)
                    ++screen_reruns;
                }
                if (tiered()) ++screen_tier_batches;
                if (tier2) {  // pass A's exact distances and pass B's marks; its rows; the pairs' top-k
                    vdbk::launch_tier_recheck(1, metric, sa, BP, w.nseg_qp.p, w.soff.p, w.scnt.p, w.surv.p, w.slb.p,
                                              w.smark.p, w.rowmap.p, w.srows.p, w.sdist.p, s);
                    uint32_t need = 0;
                    (void)fetch_rows_phase(w, 2, need, s);
                    vdbk::launch_tier_recheck(2, metric, sa, BP, w.nseg_qp.p, w.soff.p, w.scnt.p, w.surv.p, w.slb.p,
                                              w.smark.p, w.rowmap.p, w.srows.p, w.sdist.p, s);
                    HIPCHECK(hipGetLastError());
                } else {
                    vdbk::launch_screen_recheck(metric, sa, BP, w.probes.p, w.nseg_qp.p, w.soff.p, w.scnt.p, w.surv.p,
                                                w.ovf.p, fetched, w.sdist.p, ccap, (uint32_t)nseg_prefix[1], s,
                                                recheck2 ? w.sdist.p : nullptr);
                }
            } else {
                vdbk::launch_scan_screen(metric, grid, sa, s);
            }
        } else if (wide && fused_scan) {
            // one persistent grid takes both queues (no side stream, no fork/join)
            // (narrow_blocks counts 4-wave workgroups: as many waves start on the narrow queue)
            const uint32_t grid_cap = waves == 8 ? vdbk::kPersistentBlocks / 2 : vdbk::kPersistentBlocks;
            sa.fused = std::max<uint32_t>(1, std::min<uint32_t>(narrow_blocks * 4 / waves, grid_cap / 2));
            const uint64_t want = std::max<uint64_t>(max_wide, (max_items + 3) / 4);
            vdbk::launch_scan_wide(metric, (uint32_t)(scan_blocks ? std::min<uint64_t>(want, scan_blocks) : want), sa, s,
                                   waves);
        } else if (wide) {
            // narrow items on the side stream fill the CUs the wide items leave idle
            HIPCHECK(hipEventRecord(w.fork, s));
            HIPCHECK(hipStreamWaitEvent(w.side, w.fork, 0));
            vdbk::launch_scan_narrow(metric, regs_k, std::min<uint32_t>((uint32_t)((max_items + 3) / 4), narrow_blocks), sa,
                                     w.side);
            HIPCHECK(hipEventRecord(w.join, w.side));
            vdbk::launch_scan_wide(metric, (uint32_t)max_wide, sa, s, waves);
            HIPCHECK(hipStreamWaitEvent(s, w.join, 0));
        } else {
            vdbk::launch_scan_narrow(metric, regs_k, (uint32_t)((max_items + 3) / 4), sa, s);
        }
        if (ev) HIPCHECK(hipEventRecord(ev->scan_end, s));
        if (scan_window && in_ring) {
            if (!w.scan_done) HIPCHECK(hipEventCreateWithFlags(&w.scan_done, hipEventDisableTiming));
            HIPCHECK(hipEventRecord(w.scan_done, s));
            scan_hist[scan_seq % 8] = (int)(&w - slots);
            ++scan_seq;
        }
        if (fused_merge) {
            // one launch: slot folds, stale sources, unique top-k, the next batch's carry
            float* cd0 = w.carry_sel ? w.carry2_d.p : w.carry_d.p;
            uint64_t* ci0 = w.carry_sel ? w.carry2_i.p : w.carry_i.p;
            float* cd1 = w.carry_sel ? w.carry_d.p : w.carry2_d.p;
            uint64_t* ci1 = w.carry_sel ? w.carry_i.p : w.carry2_i.p;
            vdbk::launch_merge_fused(regs_k, w.probes.p, d_count_global.p, w.nseg_qp.p, w.pbqp.p, w.part_d.p, w.part_i.p, B,
                                     P, k, stale, req_start, b0, cd0, ci0, w.slot_d.p, w.slot_i.p, cd1, ci1, out_d_, out_i_,
                                     s);
            if (stale) w.carry_sel ^= 1u;
            if (ev) HIPCHECK(hipEventRecord(ev->end, s));
            HIPCHECK(hipGetLastError());
            return true;
        }
        vdbk::launch_merge_partials(regs_k, (uint32_t)max_l1, w.probes.p, d_count_global.p, w.nseg_qp.p, w.pbqp.p, w.l1base.p,
                                    w.l1_items.p, w.counters.p, w.part_d.p, w.part_i.p, k, w.l1_d.p, w.l1_i.p, s);
        vdbk::launch_slot_merge(regs_k, w.probes.p, d_count_global.p, w.nseg_qp.p, w.pbqp.p, w.l1base.p, w.part_d.p, w.part_i.p,
                                w.l1_d.p, w.l1_i.p, BP, k, w.slot_d.p, w.slot_i.p, s);
        vdbk::launch_query_merge(regs_k, w.probes.p, d_count_global.p, w.slot_d.p, w.slot_i.p, w.carry_d.p, w.carry_i.p, B, P, k,
                                 stale, req_start, b0, out_d_, out_i_, s);
        if (stale)
            vdbk::launch_carry(w.probes.p, d_count_global.p, B, P, k, w.slot_d.p, w.slot_i.p, req_start, b0, w.carry_d.p,
                               w.carry_i.p, s);
        if (ev) HIPCHECK(hipEventRecord(ev->end, s));
        HIPCHECK(hipGetLastError());
        return true;
    }

    // One batch, every list HBM-resident (or the tier with every stored list cached).
    bool run_batch(SearchSlot& w, const float* d_q, uint32_t B, uint32_t P, uint32_t k, float* out_d_,
                   uint64_t* out_i_, hipStream_t s, const uint32_t* req_start, uint32_t b0) {
        EventSet* ev = prof ? &next_events() : nullptr;
        if (ev) HIPCHECK(hipEventRecord(ev->begin, s));
        coarse_batch(w, d_q, B, P, s);
        if (ev) HIPCHECK(hipEventRecord(ev->coarse_end, s));
        if (!scan_batch(w, B, P, k, out_d_, out_i_, s, req_start, b0, ev)) {
            // the screened tier could not serve it (tier_cand_max): the exact list-cache path
            force_exact = true;
            try {
                search_tiered(w, d_q, B, P, k, out_d_, out_i_, s, req_start, b0);
            } catch (...) {
                force_exact = false;
                throw;
            }
            force_exact = false;
        }
        return true;
    }

    // ---- list-cache tier search (cache smaller than the index) ----
    // The probes of the whole call are computed first (coarse steps only), so loads and
    // evictions are planned against the call's known future:
    //  * the call is cut into sub-batches of at most `batch` queries whose probed lists
    //    fill at most half the cache (so the next sub-batch's lists load beside them; a
    //    query needing more gets a sub-batch of its own); results never depend on batch
    //    boundaries;
    //  * while sub-batch i scans, the lists of sub-batch i+1 are read from the home
    //    (file: io_uring into page-locked staging; host memory: DMA) and copied into free
    //    cache space on copy_stream; sub-batch i+1 waits for them by event;
    //  * a victim is the cached list whose next use in the call is furthest away (not
    //    used again: first), then the least recently used; sub-batch i's lists (and i+1's)
    //    are never evicted while i runs.
    // (qbase: the call-global index of d_q's first query, for the stale-slot semantics)
    void search_tiered(SearchSlot& w, const float* d_q, uint32_t n, uint32_t P, uint32_t k, float* d_dist,
                       uint64_t* d_ids, hipStream_t s, const uint32_t* req_start, uint32_t qbase = 0) {
        if (tier_call_used) HIPCHECK(hipEventSynchronize(tier_call_ev));  // probe_stage is reused
        const uint32_t bmax = batch_cap(P, k);
        // 1. probes of the whole call
        probe_stage.host = true;
        uint32_t* hp = probe_stage.ensure((size_t)n * P);
        for (uint32_t b0 = 0; b0 < n; b0 += bmax) {
            const uint32_t B = std::min(bmax, n - b0);
            coarse_batch(w, d_q + (size_t)b0 * dim, B, P, s);
            HIPCHECK(hipMemcpyAsync(hp + (size_t)b0 * P, w.probes.p, (size_t)B * P * 4, hipMemcpyDeviceToHost, s));
        }
        HIPCHECK(hipStreamSynchronize(s));
        // 2. sub-batches whose lists fit the cache
        std::vector<uint8_t> qmark(nlist, 0), umark(nlist, 0);  // (a query's lists, the sub-batch's lists)
        std::vector<uint32_t> sb_begin;
        std::vector<std::vector<uint32_t>> U;
        uint64_t blocks = 0;
        for (uint32_t q = 0; q < n; ++q) {
            const std::vector<uint32_t> ql = cacheable(hp + (size_t)q * P, P, qmark);
            uint64_t qb = 0, add = 0;
            for (uint32_t l : ql) {
                qb += list_blocks(l);
                if (!umark[l]) add += list_blocks(l);
            }
            require(qb <= cache_blocks, "list_cache_bytes cannot hold the lists one query probes", VDB_ERR_OUT_OF_MEMORY);
            // half the cache per sub-batch: the next one's lists can load beside it
            if (U.empty() || q - sb_begin.back() >= bmax || blocks + add > cache_blocks / 2) {
                if (!U.empty())
                    for (uint32_t l : U.back()) umark[l] = 0;
                sb_begin.push_back(q);
                U.emplace_back();
                blocks = 0;
            }
            for (uint32_t l : ql)
                if (!umark[l]) {
                    umark[l] = 1;
                    U.back().push_back(l);
                    blocks += list_blocks(l);
                }
        }
        const size_t nsb = U.size();
        sb_begin.push_back(n);
        // next-use ranks: for each list the sub-batches that use it, in order
        std::vector<std::vector<uint32_t>> uses(nlist);
        bool miss = false;
        for (size_t b = 0; b < nsb; ++b)
            for (uint32_t l : U[b]) {
                uses[l].push_back((uint32_t)b);
                miss |= cache_off[l] == kAbsent;
            }
        auto rank_after = [&](size_t cur) {
            return [&, cur](uint32_t l) -> uint64_t {
                const auto& u = uses[l];
                auto it = std::upper_bound(u.begin(), u.end(), (uint32_t)cur);
                return it == u.end() ? ~0ull : (uint64_t)*it;
            };
        };
        if (miss) quiesce();  // searches on other streams may still read lists evicted below
        if (!copy_stream) {
            HIPCHECK(hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking));
            for (auto& e : sb_done) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIPCHECK(hipEventCreateWithFlags(&load_ev, hipEventDisableTiming));
            HIPCHECK(hipEventCreateWithFlags(&tier_call_ev, hipEventDisableTiming));
        }
        // 3. sub-batches in order, each next one's lists loaded while the current one scans
        std::vector<uint8_t> protect(nlist, 0);
        std::vector<std::pair<uint32_t, uint64_t>> loads;
        bool prefetched = false;
        for (size_t b = 0; b < nsb; ++b) {
            const uint32_t b0 = sb_begin[b], B = sb_begin[b + 1] - b0;
            if (prefetched) {
                HIPCHECK(hipStreamWaitEvent(s, load_ev, 0));
            } else {  // load on s itself, after the previous sub-batch in stream order
                for (uint32_t l : U[b]) protect[l] = 1;
                const bool ok = plan_loads(U[b], protect, rank_after(b), true, loads);
                for (uint32_t l : U[b]) protect[l] = 0;
                require(ok, "list_cache_bytes cannot hold the lists one sub-batch probes", VDB_ERR_OUT_OF_MEMORY);
                if (!loads.empty()) {
                    load_lists(loads, s);
                    upload_scan_directory(s);
                    ++tier_sync_loads;
                }
            }
            ++use_tick;
            for (uint32_t l : U[b]) last_use[l] = use_tick;
            EventSet* ev = prof ? &next_events() : nullptr;
            if (ev) HIPCHECK(hipEventRecord(ev->begin, s));
            stage_queries(w, d_q + (size_t)b0 * dim, B, s);
            HIPCHECK(hipMemcpyAsync(w.probes.p, hp + (size_t)b0 * P, (size_t)B * P * 4, hipMemcpyHostToDevice, s));
            if (ev) HIPCHECK(hipEventRecord(ev->coarse_end, s));
            require(scan_batch(w, B, P, k, d_dist + (size_t)b0 * k, d_ids + (size_t)b0 * k, s, req_start, qbase + b0, ev),
                    "tier sub-batch not served", VDB_ERR_STATE);
            HIPCHECK(hipEventRecord(sb_done[b & 1], s));
            ++tier_subbatches;
            prefetched = false;
            if (b + 1 < nsb) {
                for (uint32_t l : U[b]) protect[l] = 1;
                for (uint32_t l : U[b + 1]) protect[l] = 1;
                const bool ok = plan_loads(U[b + 1], protect, rank_after(b + 1), false, loads);
                for (uint32_t l : U[b]) protect[l] = 0;
                for (uint32_t l : U[b + 1]) protect[l] = 0;
                if (ok) {
                    // victims may still be read by sub-batch b - 1 (not by b: protected)
                    if (b >= 1) HIPCHECK(hipStreamWaitEvent(copy_stream, sb_done[(b - 1) & 1], 0));
                    if (!loads.empty()) {
                        load_lists(loads, copy_stream);  // the host reads the file while b scans
                        upload_scan_directory(copy_stream);
                        ++tier_prefetches;
                    }
                    HIPCHECK(hipEventRecord(load_ev, copy_stream));
                    prefetched = true;
                }
            }
        }
        HIPCHECK(hipEventRecord(tier_call_ev, s));
        tier_call_used = true;
    }

    // The screened scan's item width for a search (16 or 32 queries), or 0 when the screen
    // does not serve it. ONE decision for scan_batch and for the tier's routing
    // (screen_serves): a search the tier sends past its list cache is always screened.
    // 32-query items (option screen_group; 0 = automatic: 32 from nprobe 64 up, where hub
    // lists are probed by many queries of a batch: cfg4 shard collect 4.45 vs 4.69 ms; 16
    // below: cfg3 2.54 vs 2.72 ms): the deferred kernel feeds each shadow tile to two A
    // operands (its LDS is static: any k <= 64); the inline kernel splits its waves in two
    // halves where the item's lists fit its LDS, else it runs 16-query items.
    uint32_t screen_width(uint32_t k, uint32_t P) const {
        if (!screen_ready || metric == 2 || vdbk::topk_regs(k) != 1) return 0;
        if (tiered() && !screen_defer) return 0;    // (the tier's screen is the deferred one)
        if (!screen_defer && screen_fmt_i8) return 0;  // (the inline kernel reads a bf16 shadow)
        const uint32_t want = screen_group ? screen_group : (screen_defer && P >= 64 ? 32u : 16u);
        if (want == 32 && vdbk::scan_screen_fits(k, dp, 32, screen_defer)) return 32;
        return vdbk::scan_screen_fits(k, dp, 16, screen_defer) ? 16 : 0;
    }
    // The screen serves a search with this k and nprobe (the tier: the deferred scan with its
    // shadow resident; built lazily, so a stale screen is rebuilt first).
    static constexpr uint32_t kCollectBlocks = 320;
    bool screen_serves(uint32_t k, uint32_t P) {
        last_P = P;
        if (screen_stale) screen_update();
        return screen_width(k, P) != 0;
    }

    // Queries per internal batch: the option `batch`, bounded so that batch x nprobe fits the
    // plan kernel (8192 pairs) and so that one slot's per-segment partials (B x the segments
    // of the P largest lists x k x 12 bytes) stay within kPartialBytes: the exact path at
    // k = 1000 on the 10M x 768 index would otherwise hold 1.5 GB of partials per slot.
    // Results never depend on batch boundaries.
    static constexpr uint64_t kPartialBytes = 384ull << 20;
    uint32_t batch_cap(uint32_t P, uint32_t k) const {
        uint32_t b = std::max<uint32_t>(1, std::min<uint32_t>(batch, vdbk::kPlanMaxPairs / P));
        const uint64_t per_query = (P < nseg_prefix.size() ? nseg_prefix[P] : 0) * (uint64_t)k * 12;
        if (per_query) b = std::max<uint32_t>(1, (uint32_t)std::min<uint64_t>(b, kPartialBytes / per_query));
        return b;
    }

    // Grow a slot-owned buffer; a buffer still read by the slot's previous call is
    // only freed once that call is done.
    template <class T>
    T* slot_buf(SearchSlot& w, DevBuf<T>& b, size_t n) {
        if (b.cap < n && b.p && w.used) HIPCHECK(hipEventSynchronize(w.done));
        return b.ensure(n);
    }

    // One reference search() call on this handle's device: take the next workspace slot,
    // order stream s after the slot's previous call, start the call's probe slots
    // (allocated once per call, cpp:210-211). `xworld` > 0 sizes the multi-GPU records.
    SearchSlot& begin_call(uint32_t n, uint32_t P, uint32_t k, hipStream_t s, uint32_t xworld) {
        if (!stats.p) {
            stats.ensure(16);
            HIPCHECK(hipMemsetAsync(stats.p, 0, 128, s));
        }
        SearchSlot& w = slots[next_slot];
        next_slot = (next_slot + 1) % kSlots;
        const uint32_t B = std::min(batch_cap(P, k), n);
        ensure_workspace(w, B, P, k);
        if (xworld) {
            const uint64_t rb = vdb_rank_record_bytes(B, k);
            // (emulated exchange: W records are sent; the other ranks' places hold empty records)
            if (comm_world == 1 && xchg_emulate > 1 && w.xrec.cap < rb * xworld) {
                slot_buf(w, w.xrec, rb * xworld);
                w.xfill = 0;
            }
            slot_buf(w, w.xrec, rb);
            slot_buf(w, w.xgat, rb * xworld);
        }
        if (w.used) HIPCHECK(hipStreamWaitEvent(s, w.done, 0));
        HIPCHECK(hipMemsetAsync(w.carry_i.p, 0xFF, (size_t)P * k * 8, s));
        w.carry_sel = 0;
        return w;
    }

    void end_call(SearchSlot& w, hipStream_t s) {
        HIPCHECK(hipEventRecord(w.done, s));
        w.used = true;
    }

    // The slot's packed record for a batch of B queries (vdb_rank_record_bytes layout).
    static float* rec_dist(SearchSlot& w) { return (float*)w.xrec.p; }
    static uint64_t* rec_ids(SearchSlot& w, uint32_t B, uint32_t k) {
        return (uint64_t*)(w.xrec.p + ((uint64_t)B * k * 4 + 7) / 8 * 8);
    }
    // Final results of a batch from `nranks` gathered records: unique-id top-k of the
    // union (= merge_results over every rank's lists, cpp:474-518).
    static void merge_gathered(SearchSlot& w, uint32_t nranks, uint32_t B, uint32_t k, float* od, uint64_t* oi,
                               hipStream_t s) {
        const uint64_t rec = vdb_rank_record_bytes(B, k);
        const float* d = (const float*)w.xgat.p;
        const uint64_t* ids = (const uint64_t*)(w.xgat.p + ((uint64_t)B * k * 4 + 7) / 8 * 8);
        vdbk::launch_rank_merge(vdbk::topk_regs(k), d, ids, rec / 4, rec / 8, nranks, B, k, od, oi, s);
        HIPCHECK(hipGetLastError());
    }

    // Group handle (group.cpp): the same call over every member's shard.
    void group_search_device(const float* d_q, uint32_t n, uint32_t P, uint32_t k, float* d_dist, uint64_t* d_ids,
                             hipStream_t s, const uint32_t* req_start);
    bool group_tiered() const {
        for (auto& mb : members)
            if (mb->tiered()) return true;
        return false;
    }

    // req_start: null (one reference search() call) or, for a coalesced batch of calls,
    // per query the call-global index of its request's first query (device memory).
    // With a communicator attached, every batch's partials are all-gathered over RCCL
    // and merged, so d_dist / d_ids receive the final results on every rank.
    void search_device(const float* d_q, uint32_t n, uint32_t nprobe, uint32_t k, float* d_dist, uint64_t* d_ids,
                       hipStream_t s, const uint32_t* req_start = nullptr) {
        if (n == 0 || k == 0) return;
        require(k <= (uint32_t)vdbk::kMaxK, "k above 1024 is not supported", VDB_ERR_UNSUPPORTED);
        const uint32_t P = std::min(nprobe, nlist);  // cpp:218-222 reads out of bounds beyond nlist
        if (P == 0) {
            vdbk::launch_fill_empty((uint64_t)n * k, d_dist, d_ids, s);
            HIPCHECK(hipGetLastError());
            return;
        }
        require(P <= (uint32_t)vdbk::kMaxK, "nprobe above 1024 is not supported", VDB_ERR_UNSUPPORTED);
        if (is_group()) {
            group_search_device(d_q, n, P, k, d_dist, d_ids, s, req_start);
            return;
        }
        const bool xchg = comm != nullptr;
        if (xchg)
            require((comm_world == world && comm_rank == rank) || (comm_world == 1 && xchg_emulate == world),
                    "the attached communicator's (rank, world) differs from the handle's shard", VDB_ERR_STATE);
        SearchSlot& w = begin_call(n, P, k, s, xchg ? xchg_records() : 0);
        if (xchg && (tiered() || comm_world > 1)) {
            // The exchange is per CALL at world > 1: the whole call's partials in one record,
            // ONE all-gather, one merge. A rank's own state (its tier, switched on by its own
            // shard's size against max_gpu_memory, and what its cache holds) decides how it
            // cuts a call into batches, so per-batch exchanges could differ in number and
            // size between ranks; per call, every rank issues the same collective whatever
            // its state. With 64-query calls (the bench) a call is one batch.
            slot_buf(w, w.xgat, vdb_rank_record_bytes(n, k) * comm_world);
            call_to_record(w, d_q, n, P, k, s, req_start);
            exchange(w, n, k, d_dist, d_ids, s);
            end_call(w, s);
            return;
        }
        if (tiered() && resident_n < storable_n && !screen_serves(k, P)) {  // (every stored list cached: the plain path)
            search_tiered(w, d_q, n, P, k, d_dist, d_ids, s, req_start);
            end_call(w, s);
            return;
        }
        const uint32_t bmax = batch_cap(P, k);
        for (uint32_t b0 = 0, B = std::min(bmax, n); b0 < n; b0 += B, B = std::min(B, n - b0)) {
            float* od = xchg ? rec_dist(w) : d_dist + (size_t)b0 * k;
            uint64_t* oi = xchg ? rec_ids(w, B, k) : d_ids + (size_t)b0 * k;
            run_batch(w, d_q + (size_t)b0 * dim, B, P, k, od, oi, s, req_start, b0);
            if (xchg) exchange(w, B, k, d_dist + (size_t)b0 * k, d_ids + (size_t)b0 * k, s);
        }
        end_call(w, s);
    }

    // This shard's partial results of a whole call (n queries) into the slot's packed
    // record: through the tier when some stored list is not cached, else the plain batches.
    void call_to_record(SearchSlot& w, const float* d_q, uint32_t n, uint32_t P, uint32_t k, hipStream_t s,
                        const uint32_t* req_start) {
        slot_buf(w, w.xrec, vdb_rank_record_bytes(n, k));
        float* rd = rec_dist(w);
        uint64_t* ri = rec_ids(w, n, k);
        if (tiered() && resident_n < storable_n && !screen_serves(k, P)) {
            search_tiered(w, d_q, n, P, k, rd, ri, s, req_start);
            return;
        }
        const uint32_t bmax = batch_cap(P, k);
        for (uint32_t b0 = 0, B = std::min(bmax, n); b0 < n; b0 += B, B = std::min(B, n - b0))
            run_batch(w, d_q + (size_t)b0 * dim, B, P, k, rd + (size_t)b0 * k, ri + (size_t)b0 * k, s, req_start,
                      b0);
    }

    // ONE all-gather of the slot's packed record (B queries) over the attached
    // communicator, on comm_stream fenced against s, then the on-device merge into the
    // final results. The enqueue is settled against the communicator's deadline and the
    // completion is handed to the watchdog (watch_exchange).
    void exchange(SearchSlot& w, uint32_t B, uint32_t k, float* od, uint64_t* oi, hipStream_t s) {
        if (comm_failed()) throw VdbError(VDB_ERR_DEVICE, comm_error_msg());
        EventSet* ev = prof && events_used ? &events[events_used - 1] : nullptr;  // (the call's last batch)
        const uint32_t nrec = xchg_records();
        if (comm_world == 1 && nrec > 1 && w.xfill != vdb_rank_record_bytes(B, k)) {
            // (emulation: the other ranks' places hold EMPTY records of this batch's layout —
            // (+inf or FLT_MAX, no id) entries the merge drops — so the emulated exchange moves
            // and merges W records and the results stay this rank's exact answer;
            // refilled whenever the record layout (B, k) changes)
            const uint64_t rb = vdb_rank_record_bytes(B, k);
            for (uint32_t r = 1; r < nrec; ++r)
                vdbk::launch_fill_empty((uint64_t)B * k, (float*)(w.xrec.p + rb * r),
                                        (uint64_t*)(w.xrec.p + rb * r + ((uint64_t)B * k * 4 + 7) / 8 * 8), s);
            HIPCHECK(hipGetLastError());
            w.xfill = rb;
        }
        const hipStream_t cs = comm_enter(w, s);
        nccl_settle(ncclAllGather(w.xrec.p, w.xgat.p, vdb_rank_record_bytes(B, k) * (comm_world == 1 ? nrec : 1), ncclUint8,
                                  comm, cs),
                    "ncclAllGather");
        if (ev) HIPCHECK(hipEventRecord(ev->x_end, cs));
        watch_exchange(cs);
        comm_leave(w, s);
        merge_gathered(w, nrec, B, k, od, oi, s);
        if (ev) {
            HIPCHECK(hipEventRecord(ev->m_end, s));
            ev->xchg = true;
        }
    }

    // ---- the communicator's deadline (option comm_timeout_ms) ----
    // Non-blocking RCCL (ncclCommInitRankConfig, blocking = 0): init and every collective
    // may return ncclInProgress and are polled to completion here, so a rank that never
    // joins or a connection that never forms ends in an error naming this rank instead of
    // a silent hang. Device-side completion of each exchange is watched by a host thread:
    // an all-gather still pending after the deadline (a peer stalled or died) marks the
    // communicator failed; later calls fail with that message, and vdb_ivf_comm_status
    // lets a caller that waits on its streams stop waiting. (The communicator is not
    // aborted from the watchdog: a collective still queued behind other work would then
    // run on released resources. The process is expected to exit.)
    uint32_t comm_timeout_ms = 120000;
    std::string rank_tag() const {
        return "rank " + std::to_string(comm_rank) + " of " + std::to_string(comm_world) + ": ";
    }
    void nccl_settle(ncclResult_t r, const char* what) {
        if (r == ncclSuccess) return;
        if (r != ncclInProgress) throw VdbError(VDB_ERR_DEVICE, rank_tag() + what + ": " + ncclGetErrorString(r));
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t spin = 0;; ++spin) {
            ncclResult_t st = ncclSuccess;
            const ncclResult_t q = ncclCommGetAsyncError(comm, &st);
            if (q != ncclSuccess) st = q;
            if (st == ncclSuccess) return;
            if (st != ncclInProgress)
                throw VdbError(VDB_ERR_DEVICE, rank_tag() + what + " failed: " + ncclGetErrorString(st));
            const double ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (ms > comm_timeout_ms) {
                set_comm_error(rank_tag() + what + " still in progress after " + std::to_string((int)ms) +
                               " ms (comm_timeout_ms): a peer rank is missing or stalled");
                throw VdbError(VDB_ERR_DEVICE, comm_error_msg());
            }
            if (spin > 1000) std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
    }
    struct Watch {
        std::mutex m;
        std::condition_variable cv;
        std::deque<std::pair<hipEvent_t, std::chrono::steady_clock::time_point>> pending;  // issue order
        std::vector<hipEvent_t> spare;
        std::thread th;
        bool stop = false;
        uint64_t issued = 0, completed = 0;
        std::string error;  // the first deadline miss (sticky until detach / a new attach)
    };
    std::unique_ptr<Watch> watch;
    bool comm_failed() {
        if (!watch) return false;
        std::lock_guard<std::mutex> g(watch->m);
        return !watch->error.empty();
    }
    std::string comm_error_msg() {
        if (!watch) return std::string();
        std::lock_guard<std::mutex> g(watch->m);
        return watch->error;
    }
    void set_comm_error(const std::string& e) {
        start_watch();
        std::lock_guard<std::mutex> g(watch->m);
        if (watch->error.empty()) {
            watch->error = e;
            std::fprintf(stderr, "[vdb_ivf] %s\n", e.c_str());
        }
    }
    void start_watch() {
        if (watch) return;
        watch.reset(new Watch());
        watch->th = std::thread([this] { watch_loop(); });
    }
    void stop_watch() {
        if (!watch) return;
        {
            std::lock_guard<std::mutex> g(watch->m);
            watch->stop = true;
        }
        watch->cv.notify_all();
        if (watch->th.joinable()) watch->th.join();
        for (auto& p : watch->pending) (void)hipEventDestroy(p.first);
        for (hipEvent_t e : watch->spare) (void)hipEventDestroy(e);
        watch.reset();
    }
    void watch_exchange(hipStream_t cs) {
        start_watch();
        hipEvent_t e = nullptr;
        {
            std::lock_guard<std::mutex> g(watch->m);
            if (!watch->spare.empty()) {
                e = watch->spare.back();
                watch->spare.pop_back();
            }
        }
        if (!e) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(e, cs));
        {
            std::lock_guard<std::mutex> g(watch->m);
            watch->pending.push_back({e, std::chrono::steady_clock::now()});
            ++watch->issued;
        }
        watch->cv.notify_one();
    }
    void watch_loop() {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(watch->m);
        while (!watch->stop) {
            if (watch->pending.empty()) {
                watch->cv.wait_for(lk, std::chrono::milliseconds(200));
                continue;
            }
            const hipEvent_t e = watch->pending.front().first;
            const auto t = watch->pending.front().second;
            lk.unlock();
            const hipError_t q = hipEventQuery(e);
            lk.lock();
            if (q == hipSuccess) {
                watch->pending.pop_front();
                watch->spare.push_back(e);
                ++watch->completed;
                continue;
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
            if (watch->error.empty() && (q != hipErrorNotReady || ms > comm_timeout_ms)) {
                watch->error = rank_tag() + "exchange " + std::to_string(watch->completed) + " (all-gather) " +
                               (q != hipErrorNotReady ? std::string("failed: ") + hipGetErrorString(q)
                                                      : "not complete after " + std::to_string((int)ms) +
                                                            " ms (comm_timeout_ms): a peer rank stalled or died");
                std::fprintf(stderr, "[vdb_ivf] %s\n", watch->error.c_str());
            }
            watch->cv.wait_for(lk, std::chrono::milliseconds(q == hipErrorNotReady ? 2 : 200));
        }
    }
};
