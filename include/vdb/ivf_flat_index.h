// vdb/ivf_flat_index.h — drop-in for the reference's engine/ivf_flat_index.h:14-105.
//
// Same public class surface: Config, SearchParams, train, add, search, search_batch,
// warmup_lists, evict_list, get_gpu_memory_usage, get_total_vectors, save, load,
// constructed with a borrowed TransferManager*. Every call goes through the C ABI of
// include/vdb_ivf.h to the MI355X engine; results are bit-identical to the reference's
// CPU path (use_gpu=false). Errors from the engine are rethrown as std::runtime_error;
// the constructor keeps std::invalid_argument for dimension == 0 || nlist == 0
// (ivf_flat_index.cpp:17-19).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "vdb/metric.h"
#include "vdb/transfer_manager.h"

struct vdb_ivf;

namespace vdb {

class IVFFlatIndex {
public:
    struct Config {
        uint32_t dimension;
        uint32_t nlist;
        kernels::Metric metric;
        bool use_gpu = true;
        size_t max_gpu_memory = 8ULL << 30;
        // Not in the reference (its index runs on device 0 only): more than one entry
        // shards the index by list over these GPUs (vdb_ivf_create_group); every call
        // below is unchanged and results are identical to one GPU.
        std::vector<int> devices = {};
    };

    struct SearchParams {
        uint32_t nprobe = 10;
        uint32_t k = 10;
        bool use_exact_rerank = false;  // accepted and unused, as in the reference
    };

    IVFFlatIndex(const Config& config, TransferManager* tm);
    ~IVFFlatIndex();
    IVFFlatIndex(const IVFFlatIndex&) = delete;
    IVFFlatIndex& operator=(const IVFFlatIndex&) = delete;

    void train(const float* vectors, uint64_t n_vectors);
    void add(const float* vectors, const uint64_t* ids, uint64_t n_vectors);
    void search(const float* queries, uint32_t n_queries, const SearchParams& params, float* distances,
                uint64_t* indices);
    // Declared but never defined in the reference: here request i searches the single
    // query queries[i] with params[i] into distances[i] / indices[i] (params[i].k slots).
    void search_batch(const std::vector<float*>& queries, const std::vector<SearchParams>& params,
                      std::vector<float*>& distances, std::vector<uint64_t*>& indices);

    void warmup_lists(const std::vector<uint32_t>& list_ids);
    void evict_list(uint32_t list_id);

    size_t get_gpu_memory_usage() const;
    size_t get_total_vectors() const;
    uint32_t get_dimension() const { return config_.dimension; }  // used by query_service.cpp:112

    void save(const std::string& path) const;
    void load(const std::string& path);

    vdb_ivf* handle() const { return h_; }

private:
    Config config_;
    TransferManager* tm_;
    vdb_ivf* h_ = nullptr;
};

}  // namespace vdb
