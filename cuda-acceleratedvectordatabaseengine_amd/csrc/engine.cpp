// engine.cpp — the C ABI of include/vdb_ivf.h over the index handle (engine.hpp) and the
// gfx950 kernels of kernels.hip.
#include "engine.hpp"

#include <cmath>

namespace vdbe {
thread_local std::string g_last_error;

namespace group {  // group.cpp: the same calls on a group handle (one member per device)
void train_device(vdb_ivf* g, const float* d_v, uint64_t n);
void set_centroids(vdb_ivf* g, const float* c);
void add_host(vdb_ivf* g, const float* v, const uint64_t* ids, const uint32_t* lists, uint64_t n);
void add_device(vdb_ivf* g, const float* d_v, const uint64_t* d_ids, const uint32_t* d_lists, uint64_t n);
uint64_t gpu_bytes(const vdb_ivf* g, bool allocated);
void set_option(vdb_ivf* g, const std::string& name, int64_t value);
void synchronize(vdb_ivf* g);
}  // namespace group

// Calls that act on one device's shard have no group meaning.
inline void no_group(const vdb_ivf* h, const char* what) {
    require(!h->is_group(), std::string(what) + " is not available on a group handle", VDB_ERR_UNSUPPORTED);
}
}  // namespace vdbe

extern "C" {

const char* vdb_last_error(void) { return g_last_error.c_str(); }
const char* vdb_version(void) { return "vdb_ivf 0.1.0 (gfx950)"; }
#ifndef VDB_BUILD_ID
#define VDB_BUILD_ID "unknown"
#endif
const char* vdb_build_id(void) { return VDB_BUILD_ID; }

int vdb_device_count(int* count) {
    return guarded([&] {
        require(count != nullptr, "null count");
        HIPCHECK(hipGetDeviceCount(count));
    });
}

int vdb_ivf_create(const vdb_ivf_config* cfg, vdb_ivf** out) {
    return guarded([&] {
        require(cfg && out, "null argument");
        // ivf_flat_index.cpp:17-19
        require(cfg->dimension > 0 && cfg->nlist > 0, "Invalid configuration: dimension and nlist must be > 0");
        require(cfg->metric >= 0 && cfg->metric <= 2, "unknown metric");
        require(cfg->nlist < (1u << 19) - 1, "nlist above 524286 is not supported", VDB_ERR_UNSUPPORTED);
        auto* h = new vdb_ivf();
        try {
            h->dim = cfg->dimension;
            h->nlist = cfg->nlist;
            // float4 tiles per vector, zero-padded to whole scan chunks so every chunk
            // load is unconditional (the +0.0f pad terms leave every sum's bits unchanged)
            h->d4 = (cfg->dimension + 4 * vdbk::kTileAlign - 1) / (4 * vdbk::kTileAlign) * vdbk::kTileAlign;
            h->dp = h->d4 * 4;
            h->metric = cfg->metric;
            h->device = cfg->device;
            h->max_gpu_memory = cfg->max_gpu_memory == ~0ull ? 0 : cfg->max_gpu_memory;  // 0: no cap
            h->set_device();
            HIPCHECK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
            for (auto& sl : h->slots) {
                HIPCHECK(hipStreamCreateWithFlags(&sl.side, hipStreamNonBlocking));
                HIPCHECK(hipEventCreateWithFlags(&sl.fork, hipEventDisableTiming));
                HIPCHECK(hipEventCreateWithFlags(&sl.join, hipEventDisableTiming));
                HIPCHECK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
            }
            h->cent_rm.ensure((size_t)h->nlist * h->dp);
            h->cent_il.ensure(cdiv(h->nlist, 64) * h->d4 * 64);
            HIPCHECK(hipMemsetAsync(h->cent_rm.p, 0, (size_t)h->nlist * h->dp * 4, h->stream));  // cpp:22
            h->refresh_centroid_layout();
            h->count.assign(h->nlist, 0);
            h->owned.assign(h->nlist, 1);
            h->block_off.assign(h->nlist, 0);
            h->upload_directory();
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int vdb_ivf_destroy(vdb_ivf* h) {
    return guarded([&] {
        if (!h) return;
        (void)hipSetDevice(h->device);
        (void)hipStreamSynchronize(h->stream);
        delete h;
    });
}

int vdb_ivf_train(vdb_ivf* h, const float* v, uint64_t n) {
    return guarded([&] {
        require(h && (v || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        require(n > 0, "train needs at least one vector");
        DevBuf<float> dv;
        HIPCHECK(hipMemcpyAsync(dv.ensure(n * h->dim), v, n * h->dim * 4, hipMemcpyHostToDevice, h->stream));
        if (h->is_group()) {
            HIPCHECK(hipStreamSynchronize(h->stream));
            group::train_device(h, dv.p, n);
            return;
        }
        h->train(dv.p, n);
    });
}

int vdb_ivf_train_device(vdb_ivf* h, const float* d_v, uint64_t n) {
    return guarded([&] {
        require(h && (d_v || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (h->is_group()) return group::train_device(h, d_v, n);
        h->train(d_v, n);
    });
}

int vdb_ivf_set_centroids(vdb_ivf* h, const float* c) {
    return guarded([&] {
        require(h && c, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (h->is_group()) return group::set_centroids(h, c);
        h->set_centroids_host(c);
    });
}

int vdb_ivf_get_centroids(vdb_ivf* h, float* c) {
    return guarded([&] {
        require(h && c, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        h->head()->set_device();
        h->head()->export_centroids(c);
        h->set_device();
    });
}

int vdb_ivf_add(vdb_ivf* h, const float* v, const uint64_t* ids, uint64_t n) {
    return guarded([&] {
        require(h && ((v && ids) || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (n == 0) return;
        if (h->is_group()) return group::add_host(h, v, ids, nullptr, n);
        DevBuf<float> dv;
        DevBuf<uint64_t> di;
        HIPCHECK(hipMemcpyAsync(dv.ensure(n * h->dim), v, n * h->dim * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHECK(hipMemcpyAsync(di.ensure(n), ids, n * 8, hipMemcpyHostToDevice, h->stream));
        h->add(dv.p, di.p, n);
        HIPCHECK(hipStreamSynchronize(h->stream));
    });
}

int vdb_ivf_add_device(vdb_ivf* h, const float* d_v, const uint64_t* d_ids, uint64_t n) {
    return guarded([&] {
        require(h && ((d_v && d_ids) || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (h->is_group()) return group::add_device(h, d_v, d_ids, nullptr, n);
        h->add(d_v, d_ids, n);
        HIPCHECK(hipStreamSynchronize(h->stream));
    });
}

int vdb_ivf_add_to_lists(vdb_ivf* h, const float* v, const uint64_t* ids, const uint32_t* lists, uint64_t n) {
    return guarded([&] {
        require(h && ((v && ids && lists) || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (h->is_group()) return group::add_host(h, v, ids, lists, n);
        h->add_to_lists_host(v, ids, lists, n);
    });
}

int vdb_ivf_assign_device(vdb_ivf* h, const float* d_v, uint64_t n, uint32_t* d_lists) {
    return guarded([&] {
        require(h && ((d_v && d_lists) || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (n == 0) return;
        vdb_ivf* a = h->head();  // a group assigns on its first member (device of d_v)
        a->set_device();
        DevBuf<float> tmp;
        a->assign(a->padded_rows(d_v, n, tmp), n, d_lists);
        HIPCHECK(hipStreamSynchronize(a->stream));
        h->set_device();
    });
}

int vdb_ivf_add_to_lists_device(vdb_ivf* h, const float* d_v, const uint64_t* d_ids, const uint32_t* d_lists,
                                uint64_t n) {
    return guarded([&] {
        require(h && ((d_v && d_ids && d_lists) || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        if (n == 0) return;
        if (h->is_group()) return group::add_device(h, d_v, d_ids, d_lists, n);
        // The grouping kernels index per-list arrays by these ids: check them first.
        std::vector<uint32_t> hl(n);
        HIPCHECK(hipMemcpyAsync(hl.data(), d_lists, n * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHECK(hipStreamSynchronize(h->stream));
        for (uint64_t i = 0; i < n; ++i) require(hl[i] < h->nlist, "list id out of range");
        DevBuf<float> tmp;
        h->append(h->padded_rows(d_v, n, tmp), d_ids, d_lists, n);
        HIPCHECK(hipStreamSynchronize(h->stream));
    });
}

int vdb_ivf_plan_shard(vdb_ivf* h, uint32_t rank, uint32_t world, const uint64_t* final_sizes) {
    return guarded([&] {
        require(h && final_sizes && world > 0 && rank < world, "invalid shard");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        no_group(h, "plan_shard");
        h->plan_shard(rank, world, final_sizes);
    });
}

// Index file: "VDBIVF01", u32 dim, u32 nlist, i32 metric, u32 reserved, centroids
// f32[nlist][dim], then per list: u64 count, u64 ids[count], f32 vectors[count][dim].
// Shard file: "VDBIVS01", u32 dim, u32 nlist, i32 metric, u32 rank, u32 world, u32 reserved,
// centroids, then per list: u64 count (global), u64 stored (count if the rank owns the
// list, else 0), u64 ids[stored], f32 vectors[stored][dim].
int vdb_ivf_save(vdb_ivf* h, const char* path) {
    return guarded([&] {
        require(h && path, "null argument");
        // One lock for the whole save: a concurrent add cannot make the per-list counts
        // disagree with the rows written.
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        // A sharded handle (set_shard / plan_shard, world > 1) writes a shard file: every
        // list's global count (emptiness semantics) but only its own lists' rows, served
        // later by vdb_ivf_open_lists on that rank (configs[4]: each rank's lists on its
        // own NVMe). A group or an unsharded handle writes the whole index.
        const bool shard_file = !h->is_group() && h->world > 1;
        if (h->file_home()) {  // fopen("wb") would truncate the file the lists are served from
            struct stat a, b;
            if (::stat(path, &a) == 0 && ::fstat(h->home_fd, &b) == 0)
                require(!(a.st_dev == b.st_dev && a.st_ino == b.st_ino),
                        "save() target is the index file this handle serves its lists from", VDB_ERR_STATE);
        }
        // Written to a temporary name and renamed, so a failed save never leaves a
        // truncated index under `path`.
        const std::string tmp = std::string(path) + ".tmp";
        FILE* f = std::fopen(tmp.c_str(), "wb");
        require(f != nullptr, std::string("cannot open ") + tmp, VDB_ERR_STATE);
        auto put = [&](const void* p, size_t b) {
            if (b && std::fwrite(p, 1, b, f) != b) throw VdbError(VDB_ERR_STATE, "short write");
        };
        try {
            if (shard_file) {
                const uint32_t hdr[6] = {h->dim, h->nlist, (uint32_t)h->metric, h->rank, h->world, 0};
                put("VDBIVS01", 8);
                put(hdr, sizeof(hdr));
            } else {
                const uint32_t hdr[4] = {h->dim, h->nlist, (uint32_t)h->metric, 0};
                put("VDBIVF01", 8);
                put(hdr, sizeof(hdr));
            }
            std::vector<float> c((size_t)h->nlist * h->dim);
            h->head()->set_device();
            h->head()->export_centroids(c.data());
            put(c.data(), c.size() * 4);
            std::vector<float> v;
            std::vector<uint64_t> ids;
            for (uint32_t l = 0; l < h->nlist; ++l) {
                const uint64_t cnt = h->count[l];
                const uint64_t stored = shard_file && !h->owned[l] ? 0 : cnt;
                v.resize(stored * h->dim);
                ids.resize(stored);
                vdb_ivf* st = h->store_of(l);  // (a group: the member storing the list)
                st->set_device();
                if (stored) st->export_list(l, v.data(), ids.data());
                put(&cnt, 8);
                if (shard_file) put(&stored, 8);
                put(ids.data(), stored * 8);
                put(v.data(), v.size() * 4);
            }
        } catch (...) {
            std::fclose(f);
            std::remove(tmp.c_str());
            throw;
        }
        if (std::fclose(f) != 0) {
            std::remove(tmp.c_str());
            throw VdbError(VDB_ERR_STATE, "close failed");
        }
        require(std::rename(tmp.c_str(), path) == 0, std::string("cannot rename to ") + path, VDB_ERR_STATE);
    });
}

int vdb_ivf_load(vdb_ivf* h, const char* path) {
    return guarded([&] {
        require(h && path, "null argument");
        // The reference declares load() without defining it (ivf_flat_index.h:67); here
        // it fills an empty handle. Appending a file's lists to rows assigned under other
        // centroids would mix two indexes, so a non-empty handle is refused.
        {
            std::lock_guard<std::mutex> g(h->mu);
            require(h->total == 0, "load() needs an empty index (this one holds vectors)", VDB_ERR_STATE);
        }
        FILE* f = std::fopen(path, "rb");
        require(f != nullptr, std::string("cannot open ") + path, VDB_ERR_STATE);
        auto get = [&](void* p, size_t b) {
            if (b && std::fread(p, 1, b, f) != b) {
                std::fclose(f);
                throw VdbError(VDB_ERR_STATE, "truncated index file");
            }
        };
        char magic[8];
        uint32_t hdr[4];
        get(magic, 8);
        get(hdr, sizeof(hdr));
        if (std::memcmp(magic, "VDBIVS01", 8) == 0) {
            std::fclose(f);
            throw VdbError(VDB_ERR_INVALID_ARGUMENT, "a shard file holds one rank's lists: serve it with open_lists");
        }
        if (std::memcmp(magic, "VDBIVF01", 8) != 0 || hdr[0] != h->dim || hdr[1] != h->nlist ||
            (int)hdr[2] != h->metric) {
            std::fclose(f);
            throw VdbError(VDB_ERR_INVALID_ARGUMENT, "index file does not match this index's configuration");
        }
        std::vector<float> c((size_t)h->nlist * h->dim);
        get(c.data(), c.size() * 4);
        std::vector<float> vs;
        std::vector<uint64_t> is;
        std::vector<uint32_t> ls;
        for (uint32_t l = 0; l < h->nlist; ++l) {
            uint64_t cnt = 0;
            get(&cnt, 8);
            const size_t o = is.size();
            is.resize(o + cnt);
            vs.resize((o + cnt) * h->dim);
            get(is.data() + o, cnt * 8);
            get(vs.data() + o * h->dim, cnt * h->dim * 4);
            ls.insert(ls.end(), cnt, l);
        }
        std::fclose(f);
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        require(h->total == 0, "load() needs an empty index (this one holds vectors)", VDB_ERR_STATE);
        std::vector<float> old((size_t)h->nlist * h->dim);
        h->head()->set_device();
        h->head()->export_centroids(old.data());
        h->set_device();
        auto set_c = [&](const float* cc) {
            if (h->is_group()) group::set_centroids(h, cc);
            else h->set_centroids_host(cc);
        };
        set_c(c.data());
        try {
            if (h->is_group()) group::add_host(h, vs.data(), is.data(), ls.data(), is.size());
            else h->add_to_lists_host(vs.data(), is.data(), ls.data(), is.size());
        } catch (...) {
            set_c(old.data());  // all or nothing: the empty handle keeps its centroids
            throw;
        }
    });
}

int vdb_ivf_search(vdb_ivf* h, const float* q, uint32_t n, uint32_t nprobe, uint32_t k, float* dist,
                   uint64_t* ids) {
    return guarded([&] {
        require(h && ((q && dist && ids) || n == 0 || k == 0), "null argument");
        if (n == 0 || k == 0) return;
        require(k <= (uint32_t)vdbk::kMaxK, "k above 1024 is not supported", VDB_ERR_UNSUPPORTED);
        // With a communicator of world > 1 every rank must issue the same collectives in the
        // same order; the coalescer's grouping of concurrent callers depends on timing, so
        // such a handle serves calls one at a time, in the order they take the lock.
        const bool ranked = h->comm && h->comm_world > 1;
        if (h->coalesce && !ranked) {
            h->search_coalesced(q, n, nprobe, k, dist, ids);  // concurrent callers share device batches
        } else {
            std::lock_guard<std::mutex> g(h->mu);
            h->search_host(q, n, nprobe, k, dist, ids, nullptr);
        }
    });
}

int vdb_ivf_search_device(vdb_ivf* h, const float* d_q, uint32_t n, uint32_t nprobe, uint32_t k, float* d_dist,
                          uint64_t* d_ids, void* stream) {
    return guarded([&] {
        require(h && ((d_q && d_dist && d_ids) || n == 0 || k == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        hipStream_t s = stream ? (hipStream_t)stream : h->stream;
        h->search_device(d_q, n, nprobe, k, d_dist, d_ids, s);
    });
}

int vdb_ivf_set_shard(vdb_ivf* h, uint32_t rank, uint32_t world) {
    return guarded([&] {
        require(h && world > 0 && rank < world, "invalid shard");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        no_group(h, "set_shard");
        h->set_shard(rank, world);
    });
}

int vdb_merge_ranks_device(const float* d_dist, const uint64_t* d_ids, uint32_t nranks, uint32_t n, uint32_t k,
                           float* d_out_dist, uint64_t* d_out_ids, void* stream) {
    return guarded([&] {
        if (n == 0 || k == 0) return;
        require(d_dist && d_ids && d_out_dist && d_out_ids && nranks > 0, "null argument");
        require(k <= (uint32_t)vdbk::kMaxK, "k above 1024 is not supported", VDB_ERR_UNSUPPORTED);
        vdbk::launch_rank_merge(vdbk::topk_regs(k), d_dist, d_ids, (uint64_t)n * k, (uint64_t)n * k, nranks, n, k,
                                d_out_dist, d_out_ids, (hipStream_t)stream);
        HIPCHECK(hipGetLastError());
    });
}

uint64_t vdb_rank_record_bytes(uint32_t n, uint32_t k) {
    return ((uint64_t)n * k * 4 + 7) / 8 * 8 + (uint64_t)n * k * 8;
}

int vdb_merge_ranks_packed_device(const void* d_records, uint32_t nranks, uint32_t n, uint32_t k, float* d_out_dist,
                                  uint64_t* d_out_ids, void* stream) {
    return guarded([&] {
        if (n == 0 || k == 0) return;
        require(d_records && d_out_dist && d_out_ids && nranks > 0, "null argument");
        require(k <= (uint32_t)vdbk::kMaxK, "k above 1024 is not supported", VDB_ERR_UNSUPPORTED);
        const uint64_t rec = vdb_rank_record_bytes(n, k);
        const float* d = (const float*)d_records;
        const uint64_t* ids = (const uint64_t*)((const char*)d_records + ((uint64_t)n * k * 4 + 7) / 8 * 8);
        vdbk::launch_rank_merge(vdbk::topk_regs(k), d, ids, rec / 4, rec / 8, nranks, n, k, d_out_dist, d_out_ids,
                                (hipStream_t)stream);
        HIPCHECK(hipGetLastError());
    });
}

// Longest-processing-time placement: lists by decreasing cost (ties: lower list id) each
// to the least-loaded rank (ties: lower rank). Integer costs: identical on every rank.
static void lpt_plan(const uint64_t* cost, uint32_t nlist, uint32_t world, uint32_t* owner) {
    std::vector<uint32_t> order(nlist);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
    using Load = std::pair<uint64_t, uint32_t>;  // (load, rank): least load, then lowest rank
    std::priority_queue<Load, std::vector<Load>, std::greater<Load>> pq;
    for (uint32_t r = 0; r < world; ++r) pq.push({0, r});
    for (uint32_t l : order) {
        Load top = pq.top();
        pq.pop();
        owner[l] = top.second;
        top.first += cost[l];
        pq.push(top);
    }
}

int vdb_shard_plan(const uint64_t* sizes, uint32_t nlist, uint32_t world, uint32_t* owner) {
    return guarded([&] {
        require(sizes && owner && world > 0, "invalid argument");
        lpt_plan(sizes, nlist, world, owner);
    });
}

int vdb_shard_plan_probe_weighted(const uint64_t* sizes, const uint64_t* probe_counts, uint64_t n_sample,
                                  uint32_t batch, uint32_t nlist, uint32_t world, uint32_t* owner) {
    return guarded([&] {
        require(sizes && probe_counts && owner && world > 0 && n_sample > 0 && batch > 0, "invalid argument");
        // Expected scan cost of list l per batch of `batch` queries, in units of one read
        // of one vector: M ~ Binomial(batch, p_l) queries probe it (p_l from the census);
        // the list is streamed once per group of kWideGroup queries (E[ceil(M / 16)]) and
        // every query adds its distance arithmetic (VALU ~ one read's time per 16 queries
        // at 768-D on MI355X, half-overlapped with the stream: 0.5 E[M] / 16).
        const uint32_t G = (uint32_t)vdbk::kWideGroup;
        std::vector<uint64_t> cost(nlist);
        std::vector<double> pm(batch + 1);
        for (uint32_t l = 0; l < nlist; ++l) {
            const double p = std::min(1.0, (double)probe_counts[l] / (double)n_sample);
            double reads = 0.0;
            if (p > 0.0) {  // E[ceil(M / G)] over the binomial pmf (log-space terms)
                const double lp = std::log(p), lq = p < 1.0 ? std::log1p(-p) : -INFINITY;
                double lc = 0.0;  // log C(batch, m)
                for (uint32_t m = 0; m <= batch; ++m) {
                    if (m) lc += std::log((double)(batch - m + 1)) - std::log((double)m);
                    const double lt = lc + (m ? m * lp : 0.0) + (batch - m ? (batch - m) * lq : 0.0);
                    reads += std::exp(lt) * (double)((m + G - 1) / G);
                }
            }
            const double c = (double)sizes[l] * (reads + 0.5 * (double)batch * p / (double)G);
            cost[l] = (uint64_t)std::llround(c * 1024.0) + (sizes[l] ? 1 : 0);  // (a stored list costs > 0)
        }
        lpt_plan(cost.data(), nlist, world, owner);
    });
}

int vdb_ivf_probe_census(vdb_ivf* h, const float* d_rows, uint64_t n, uint32_t nprobe, uint64_t* counts) {
    return guarded([&] {
        require(h && counts && (d_rows || n == 0), "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        std::fill(counts, counts + h->nlist, 0ull);
        vdb_ivf* a = h->head();  // (a group: its first member, the device of d_rows)
        a->set_device();
        a->probe_census(d_rows, n, nprobe, counts);
        h->set_device();
    });
}

int vdb_ivf_set_shard_owners(vdb_ivf* h, uint32_t rank, uint32_t world, const uint32_t* owner) {
    return guarded([&] {
        require(h && owner && world > 0 && rank < world, "invalid shard");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        no_group(h, "set_shard");
        h->set_shard(rank, world, owner);
    });
}

int vdb_ivf_plan_shard_owners(vdb_ivf* h, uint32_t rank, uint32_t world, const uint64_t* final_sizes,
                              const uint32_t* owner) {
    return guarded([&] {
        require(h && final_sizes && owner && world > 0 && rank < world, "invalid shard");
        std::lock_guard<std::mutex> g(h->mu);
        h->set_device();
        no_group(h, "plan_shard");
        h->plan_shard(rank, world, final_sizes, owner);
    });
}

int vdb_ivf_warmup(vdb_ivf* h, const uint32_t* lists, uint32_t n) {
    return guarded([&] {
        require(h && (lists || n == 0), "null argument");
        for (uint32_t i = 0; i < n; ++i) require(lists[i] < h->nlist, "list id out of range");
        // Without the list-cache tier every list is already HBM-resident. In the tier,
        // each list is loaded like load_list_to_gpu (ivf_flat_index.cpp:387-444): one
        // that cannot fit the cache is skipped (the reference returns false). A group
        // loads each list on the member storing it.
        std::lock_guard<std::mutex> g(h->mu);
        for (uint32_t i = 0; i < n; ++i) {
            vdb_ivf* st = h->store_of(lists[i]);
            if (!st->tiered()) continue;
            st->set_device();
            (void)st->make_resident(lists + i, 1, st->stream);
            HIPCHECK(hipStreamSynchronize(st->stream));
        }
        h->set_device();
    });
}

int vdb_ivf_evict(vdb_ivf* h, uint32_t list) {
    return guarded([&] {
        require(h && list < h->nlist, "list id out of range");
        // Without the tier residency is permanent and eviction is a no-op; in the tier
        // the list leaves the cache (evict_list_from_gpu, ivf_flat_index.cpp:447-471).
        std::lock_guard<std::mutex> g(h->mu);
        vdb_ivf* st = h->store_of(list);
        if (!st->tiered() || st->cache_off[list] == vdb_ivf::kAbsent) return;
        st->set_device();
        st->quiesce();
        st->cache_free(list);
        h->set_device();
    });
}

// IVFFlatIndex::get_gpu_memory_usage (ivf_flat_index.cpp:393-443, 707-709): the bytes of
// the GPU-resident lists, count * (dim * 4 + 8) each (every stored list, or the cached
// ones in the list-cache tier). vdb_ivf_gpu_bytes_allocated is the real footprint.
uint64_t vdb_ivf_gpu_bytes(const vdb_ivf* h) {
    if (!h) return 0;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->is_group()) return group::gpu_bytes(h, false);
    uint64_t b = 0;
    for (uint32_t l = 0; l < h->nlist; ++l) {
        const bool resident = h->tiered() ? h->cache_off[l] != vdb_ivf::kAbsent : (bool)h->owned[l];
        if (resident) b += h->count[l] * ((uint64_t)h->dim * 4 + 8);
    }
    return b;
}

uint64_t vdb_ivf_gpu_bytes_allocated(const vdb_ivf* h) {
    if (!h) return 0;
    std::lock_guard<std::mutex> g(h->mu);
    if (h->is_group()) return group::gpu_bytes(h, true);
    return h->device_footprint();
}

uint64_t vdb_ivf_ntotal(const vdb_ivf* h) { return h ? h->total : 0; }
uint32_t vdb_ivf_dimension(const vdb_ivf* h) { return h ? h->dim : 0; }
uint32_t vdb_ivf_nlist(const vdb_ivf* h) { return h ? h->nlist : 0; }

int vdb_ivf_list_sizes(const vdb_ivf* h, uint64_t* sizes) {
    return guarded([&] {
        require(h && sizes, "null argument");
        std::copy(h->count.begin(), h->count.end(), sizes);
    });
}

int vdb_ivf_get_list(vdb_ivf* h, uint32_t list, float* vectors, uint64_t* ids) {
    return guarded([&] {
        require(h && list < h->nlist, "list id out of range");
        std::lock_guard<std::mutex> g(h->mu);
        vdb_ivf* st = h->store_of(list);
        st->set_device();
        st->export_list(list, vectors, ids);
        h->set_device();
    });
}

int vdb_ivf_set_batch(vdb_ivf* h, uint32_t batch) {
    return guarded([&] {
        require(h && batch > 0, "invalid batch");
        std::lock_guard<std::mutex> g(h->mu);
        if (h->is_group()) return group::set_option(h, "batch", batch);
        h->batch = batch;
    });
}

int vdb_ivf_set_stale_slots(vdb_ivf* h, int enable) {
    return guarded([&] {
        require(h, "null handle");
        std::lock_guard<std::mutex> g(h->mu);
        if (h->is_group()) return group::set_option(h, "stale_slots", enable ? 1 : 0);
        h->stale = enable ? 1 : 0;
    });
}

int vdb_ivf_set_option(vdb_ivf* h, const char* name, int64_t value) {
    return guarded([&] {
        require(h && name, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        const std::string n(name);
        if (h->is_group()) return group::set_option(h, n, value);
        if (n == "coarse_mode") {
            require(value == 0 || value == 1, "coarse_mode is 0 or 1");
            h->coarse_mode = (int)value;
        } else if (n == "wide_scan") {
            h->wide_scan = value != 0;
        } else if (n == "wide_stride") {
            require(value >= 0 && value < (1ll << 31), "wide_stride out of range");
            h->wide_stride = (uint32_t)value;
        } else if (n == "seg_vectors") {
            require(value == 0 || value == 64 || value == 128 || value == 256 || value == 512 || value == 1024,
                    "seg_vectors is 0 (auto), 64, 128, 256, 512 or 1024");
            h->seg_blocks_opt = (uint32_t)(value / 64);
            h->set_device();
            h->upload_directory();
        } else if (n == "coalesce") {
            h->coalesce = value != 0;
        } else if (n == "coalesce_max_queries") {
            require(value > 0 && value < (1ll << 31), "coalesce_max_queries out of range");
            h->coalesce_max_queries = (uint32_t)value;
        } else if (n == "coalesce_window_us") {
            require(value >= 0 && value < 1000000, "coalesce_window_us out of range");
            h->coalesce_window_us = (uint32_t)value;
        } else if (n == "segs_per_item") {
            require(value == 0 || (value >= 4 && value <= 64), "segs_per_item is 0 (auto) or 4..64");
            h->segs_item_opt = (uint32_t)value;
        } else if (n == "wide_group") {
            require(value == 16 || value == 32, "wide_group is 16 or 32");
            h->wide_group = (uint32_t)value;
        } else if (n == "scan_blocks") {
            require(value >= 0 && value <= (int64_t)vdbk::kPersistentBlocks, "scan_blocks is 0 (auto) .. 512");
            h->scan_blocks = (uint32_t)value;
        } else if (n == "scan_mfma_min") {
            require(value >= 0 && value <= 16, "scan_mfma_min is 0 (never) .. 16");
            h->scan_mfma_min = (uint32_t)value;
        } else if (n == "screen") {
            h->set_device();
            h->quiesce();
            h->screen_opt = value != 0;
            h->screen_update();
        } else if (n == "screen_defer") {
            h->set_device();
            h->quiesce();
            h->screen_defer = value != 0;
            h->screen_update();
        } else if (n == "screen_recheck2") {
            h->set_device();
            h->quiesce();
            h->screen_recheck2 = value != 0;
        } else if (n == "screen_i8") {
            require(value >= 0 && value <= 2, "screen_i8 is 0 (bf16), 1 (int8) or 2 (automatic)");
            h->set_device();
            h->quiesce();
            h->screen_i8 = (int)value;
            h->i8_vetoed = false;
            h->screen_update();
        } else if (n == "screen_cand_cap") {
            require(value >= 1024 && value <= (1ll << 30), "screen_cand_cap is 1024 .. 2^30");
            h->set_device();
            h->quiesce();
            h->screen_cand_cap = (uint32_t)value;
        } else if (n == "exchange_emulate_world") {  // (diagnostics: see engine.hpp xchg_emulate)
            require(value >= 0 && value <= 64, "exchange_emulate_world is 0 .. 64");
            h->set_device();
            h->quiesce();
            h->xchg_emulate = (uint32_t)value;
        } else if (n == "collect_stamps") {  // (diagnostics: records of the collect kernel's items)
            require(value >= 0 && value <= (1ll << 24), "collect_stamps is 0 .. 2^24 records");
            h->set_device();
            h->quiesce();
            h->stamps_cap = (uint32_t)value;
            if (value) {
                h->stamps_buf.ensure((size_t)value * 4 + 2);
                HIPCHECK(hipMemset(h->stamps_buf.p, 0, 16));
            } else {
                h->stamps_buf.release();
            }
            h->stamp_batch = 0;
        } else if (n == "tier_cand_max") {
            require(value >= 1024 && value <= (1ll << 31), "tier_cand_max is 1024 .. 2^31");
            h->tier_cand_max = (uint32_t)value;
        } else if (n == "screen_floor_ppm") {
            require(value >= 0 && value <= 1000000, "screen_floor_ppm is 0 (never) .. 1000000");
            h->floor.ppm = (uint32_t)value;
            h->floor.reset_state();
        } else if (n == "screen_floor_min") {
            require(value >= 0, "screen_floor_min is >= 0");
            h->floor.min_pairs = (uint64_t)value;
        } else if (n == "screen_thr_every") {
            require(value >= 0 && value <= 1024, "screen_thr_every is 0 (automatic) .. 1024");
            h->screen_thr_every = (uint32_t)value;
        } else if (n == "screen_floor_skip") {
            require(value >= 1 && value < (1ll << 20), "screen_floor_skip is 1 .. 2^20");
            h->floor.skip = (uint32_t)value;
        } else if (n == "tier_row_cache") {
            h->set_device();
            h->quiesce();
            h->tier_row_cache = value != 0;
            if (h->tier_row_cache && h->tiered() && h->file_home() && h->screen_ready) h->fill_row_cache();
        } else if (n == "tier_row_qd") {
            require(value >= 1 && value <= 4096, "tier_row_qd is 1 .. 4096");
            h->tier_row_qd = (uint32_t)value;
        } else if (n == "tier_row_direct") {
            h->tier_row_direct = value != 0;
        } else if (n == "screen_group") {
            require(value == 0 || value == 16 || value == 32, "screen_group is 0 (auto), 16 or 32");
            h->screen_group = (uint32_t)value;
        } else if (n == "fused_scan") {
            h->fused_scan = value != 0;
        } else if (n == "fused_merge") {
            h->fused_merge = value != 0;
        } else if (n == "scan_window") {
            require(value >= 0 && value <= 7, "scan_window is 0 (no limit) .. 7");
            h->quiesce();
            h->scan_window = (uint32_t)value;
            h->scan_seq = 0;
        } else if (n == "narrow_blocks") {
            require(value > 0 && value <= 4096, "narrow_blocks out of range");
            h->narrow_blocks = (uint32_t)value;
        } else if (n == "list_cache_bytes") {
            require(value >= 0, "list_cache_bytes out of range");
            h->set_device();
            h->set_list_cache((uint64_t)value);
            h->max_gpu_memory = 0;  // explicit residency control replaces the Config cap
            h->tier_by_cap = false;
        } else if (n == "max_gpu_memory") {
            require(value >= 0, "max_gpu_memory out of range");
            h->set_device();
            h->max_gpu_memory = (uint64_t)value;
            h->apply_memory_cap(h->count);  // (on, or back off when the tier came from the cap)
        } else if (n == "bounded_stats") {
            h->bounded_stats = value != 0;  // statistics only: results never change
        } else if (n == "comm_timeout_ms") {
            require(value > 0 && value < (1ll << 31), "comm_timeout_ms out of range");
            h->comm_timeout_ms = (uint32_t)value;
        } else if (n == "batch") {
            require(value > 0 && value < (1ll << 31), "batch out of range");
            h->batch = (uint32_t)value;
        } else if (n == "stale_slots") {
            h->stale = value ? 1 : 0;
        } else {
            throw VdbError(VDB_ERR_INVALID_ARGUMENT, "unknown option " + n);
        }
    });
}

int vdb_ivf_cache_stats(vdb_ivf* h, vdb_ivf_cache_stats_t* out) {
    return guarded([&] {
        require(h && out, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        *out = vdb_ivf_cache_stats_t{};
        // (a group: the sums over its members' caches)
        std::vector<vdb_ivf*> hs;
        if (h->is_group())
            for (auto& mb : h->members) hs.push_back(mb.get());
        else
            hs.push_back(h);
        for (vdb_ivf* m : hs) {
            out->capacity_bytes += m->cache_blocks * vdb_ivf::block_bytes(m->dp);
            out->resident_bytes += m->cache_used * vdb_ivf::block_bytes(m->dp);
            out->loads += m->cache_loads;
            out->evictions += m->cache_evictions;
            out->bytes_loaded += m->cache_bytes_in;
            for (uint32_t l = 0; l < m->nlist && m->tiered(); ++l) out->resident_lists += m->cache_off[l] != vdb_ivf::kAbsent;
            out->file_bytes_read += m->file_bytes_read;
            out->subbatches += m->tier_subbatches;
            out->prefetches += m->tier_prefetches;
            out->sync_loads += m->tier_sync_loads;
            out->io_uring |= m->uring && m->uring->uring() ? 1 : 0;
            out->o_direct |= m->home_fd_direct >= 0 ? 1 : 0;
            if (m->tiered() && m->screen_ready) {
                out->screen_resident = 1;
                out->screen_bytes += m->screen_sh.device_bytes() + m->screen_meta.device_bytes() +
                                     m->screen_ids.device_bytes() + m->screen_blist.device_bytes();
            }
            out->screen_batches += m->screen_tier_batches;
            out->screen_rows_fetched += m->screen_rows_fetched;
            out->screen_row_bytes += m->screen_row_bytes;
            out->screen_reruns += m->screen_reruns;
            out->screen_rows_cached += m->screen_rows_cached;
            out->screen_fallbacks += m->screen_tier_fallbacks;
        }
    });
}

int vdb_ivf_collect_stamps(vdb_ivf* h, uint64_t* out, uint64_t cap, uint64_t* n, uint64_t* clock_hz) {
    return guarded([&] {
        require(h && n && clock_hz, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        no_group(h, "collect_stamps");
        h->set_device();
        *n = 0;
        int hz = 0;
        HIPCHECK(hipDeviceGetAttribute(&hz, hipDeviceAttributeWallClockRate, h->device));
        *clock_hz = (uint64_t)hz * 1000;  // (the attribute is in kHz)
        if (!h->stamps_cap) return;
        h->quiesce();
        HIPCHECK(hipStreamSynchronize(h->stream));
        uint32_t cnt = 0;
        HIPCHECK(hipMemcpy(&cnt, h->stamps_buf.p, 4, hipMemcpyDeviceToHost));
        *n = std::min<uint64_t>(cnt, h->stamps_cap);
        if (!out) return;  // (the count only)
        if (cap) HIPCHECK(hipMemcpy(out, h->stamps_buf.p + 2, std::min(cap, *n) * 32, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemset(h->stamps_buf.p, 0, 16));
        h->stamp_batch = 0;
    });
}

int vdb_ivf_survivor_histogram(vdb_ivf* h, uint64_t* out) {
    return guarded([&] {
        require(h && out, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        no_group(h, "survivor_histogram");
        for (uint32_t l = 0; l < h->nlist; ++l) out[l] = l < h->surv_hist.size() ? h->surv_hist[l] : 0;
    });
}

int vdb_ivf_fill_row_cache(vdb_ivf* h, const uint64_t* weights) {
    return guarded([&] {
        require(h, "null handle");
        std::lock_guard<std::mutex> g(h->mu);
        no_group(h, "fill_row_cache");
        h->set_device();
        h->quiesce();
        if (h->tier_call_used) HIPCHECK(hipEventSynchronize(h->tier_call_ev));
        if (weights) h->row_cache_weight.assign(weights, weights + h->nlist);
        else h->row_cache_weight.clear();
        if (!(h->tiered() && h->file_home() && h->tier_row_cache)) return;
        if (h->screen_stale) h->screen_update();  // (its build fills the cache itself)
        if (!h->screen_ready) return;
        h->cache_reset();  // (refilled in the new order)
        h->fill_row_cache();
    });
}

int vdb_ivf_open_lists(vdb_ivf* h, const char* path) {
    return guarded([&] {
        require(h && path, "null argument");
        std::lock_guard<std::mutex> g(h->mu);
        no_group(h, "open_lists");
        h->set_device();
        h->open_lists(path);
    });
}

int vdb_ivf_coalesce_stats(vdb_ivf* h, uint64_t* batches, uint64_t* requests) {
    return guarded([&] {
        require(h && batches && requests, "null argument");
        *batches = 0;
        *requests = 0;
        if (h->co) {
            std::lock_guard<std::mutex> g(h->co->m);
            *batches = h->co->batches;
            *requests = h->co->requests;
        }
    });
}

int vdb_ivf_set_coarse_mode(vdb_ivf* h, int mode) {
    return guarded([&] {
        require(h && (mode == 0 || mode == 1), "coarse mode is 0 (exact VALU) or 1 (MFMA + exact re-rank)");
        std::lock_guard<std::mutex> g(h->mu);
        if (h->is_group()) return group::set_option(h, "coarse_mode", mode);
        h->coarse_mode = mode;
    });
}

int vdb_ivf_profile_enable(vdb_ivf* h, int enable) {
    return guarded([&] {
        require(h, "null handle");
        std::lock_guard<std::mutex> g(h->mu);
        h->head()->prof = enable != 0;  // (a group: its first member, rank 0)
    });
}

int vdb_ivf_profile_reset(vdb_ivf* h) {
    return guarded([&] {
        require(h, "null handle");
        std::lock_guard<std::mutex> g(h->mu);
        if (h->is_group()) group::synchronize(h);
        vdb_ivf* p = h->head();
        p->set_device();
        HIPCHECK(hipDeviceSynchronize());
        p->events_used = 0;
        p->floor.batches = p->floor.trips = 0;
        HIPCHECK(hipMemsetAsync(p->stats.ensure(16), 0, 128, p->stream));
        HIPCHECK(hipStreamSynchronize(p->stream));
        h->set_device();
    });
}

int vdb_ivf_profile_read(vdb_ivf* h, vdb_ivf_profile* out) {
    return guarded([&] {
        require(h && out, "null argument");
        std::lock_guard<std::mutex> gl(h->mu);
        if (h->is_group()) group::synchronize(h);
        vdb_ivf* const hh = h;
        h = h->head();
        h->set_device();
        HIPCHECK(hipDeviceSynchronize());
        vdb_ivf_profile p{};
        for (size_t i = 0; i < h->events_used; ++i) {
            const EventSet& e = h->events[i];
            float a = 0, b = 0, c = 0, m = 0;
            HIPCHECK(hipEventElapsedTime(&a, e.scan_begin, e.scan_end));
            HIPCHECK(hipEventElapsedTime(&b, e.begin, e.coarse_end));
            HIPCHECK(hipEventElapsedTime(&c, e.begin, e.end));
            HIPCHECK(hipEventElapsedTime(&m, e.scan_end, e.end));
            p.scan_ms += a;
            p.coarse_ms += b;
            p.total_ms += c;
            p.local_merge_ms += m;
            p.scan_launches++;
            if (e.collected) {  // the deferred screen: the collect kernel, then its re-checks
                float cl = 0;
                float rc = 0;
                HIPCHECK(hipEventElapsedTime(&cl, e.collect_begin, e.collect_end));
                HIPCHECK(hipEventElapsedTime(&rc, e.collect_end, e.scan_end));
                p.collect_ms += cl;
                p.recheck_ms += rc;
            }
            if (e.xchg) {  // (the exchange of a batch, or of the whole call in the tier)
                float x = 0, r = 0;
                HIPCHECK(hipEventElapsedTime(&x, e.end, e.x_end));
                HIPCHECK(hipEventElapsedTime(&r, e.x_end, e.m_end));
                p.exchange_ms += x;
                p.rank_merge_ms += r;
                p.exchanges++;
            }
        }
        unsigned long long st[16] = {};
        if (h->stats.p) HIPCHECK(hipMemcpy(st, h->stats.p, 128, hipMemcpyDeviceToHost));
        p.distinct_lists = st[0];
        p.scan_vectors = st[1];
        p.work_items = st[2];
        p.batches = st[3];
        p.scan_bytes = st[1] * (uint64_t)h->dim * 4;
        p.pair_vectors = st[4];
        // (inline screen / bounded scan: st[5], st[6]; deferred screen: st[8] collected,
        // st[9] blocks, st[10] re-checked)
        p.exact_reranks = st[5] + st[10];
        p.bounded_blocks = st[6] + st[9];
        p.screen_collected = st[8];
        p.screen_floor_batches = h->floor.batches;
        p.screen_floor_trips = h->floor.trips;
        p.screen_shadow = h->screen_ready ? (h->screen_fmt_i8 ? 2u : 1u) : 0u;
        p.computed_vectors = st[7];
        *out = p;
        hh->set_device();
    });
}

int vdb_ivf_synchronize(vdb_ivf* h) {
    return guarded([&] {
        require(h, "null handle");
        if (h->is_group()) return group::synchronize(h);
        h->set_device();
        HIPCHECK(hipStreamSynchronize(h->stream));
    });
}

void* vdb_ivf_stream(vdb_ivf* h) { return h ? (void*)h->stream : nullptr; }

int vdb_gen_mixture_device(float* d_out, uint64_t rows, uint32_t dim, const float* d_centers, uint32_t ncomp,
                           float sigma, uint64_t seed, uint64_t row0, void* stream) {
    return guarded([&] {
        require((d_out && d_centers && ncomp > 0) || rows == 0, "invalid argument");
        vdbk::launch_gen_mixture(d_out, rows, dim, d_centers, ncomp, sigma, seed, row0, (hipStream_t)stream);
        HIPCHECK(hipGetLastError());
    });
}

int vdb_gen_normal_device(float* d_out, uint64_t n, uint64_t seed, uint64_t offset, void* stream) {
    return guarded([&] {
        require(d_out || n == 0, "null argument");
        vdbk::launch_gen_normal(d_out, n, seed, offset, (hipStream_t)stream);
        HIPCHECK(hipGetLastError());
    });
}

}  // extern "C"
