// ivf_flat_index.cpp — vdb::IVFFlatIndex (include/vdb/ivf_flat_index.h) over the C ABI.
//
// Mirrors the reference class surface (engine/ivf_flat_index.h:14-67); the work
// happens in libvdb_ivf.so on the GPU. Error mapping: the constructor throws
// std::invalid_argument like ivf_flat_index.cpp:17-19; engine failures become
// std::runtime_error (the server maps exceptions to INTERNAL, query_service.cpp:164).
#include "vdb/ivf_flat_index.h"

#include <stdexcept>
#include <string>

#include "vdb_ivf.h"

namespace vdb {

namespace {
void ok(int rc, const char* what) {
    if (rc != VDB_OK) throw std::runtime_error(std::string(what) + ": " + vdb_last_error());
}
}  // namespace

IVFFlatIndex::IVFFlatIndex(const Config& config, TransferManager* tm) : config_(config), tm_(tm) {
    if (config_.dimension == 0 || config_.nlist == 0)
        throw std::invalid_argument("Invalid configuration: dimension and nlist must be > 0");
    vdb_ivf_config c{};
    c.dimension = config_.dimension;
    c.nlist = config_.nlist;
    c.metric = static_cast<int32_t>(config_.metric);
    c.use_gpu = config_.use_gpu ? 1 : 0;
    c.max_gpu_memory = config_.max_gpu_memory;
    c.device = tm_ ? tm_->config().device : 0;
    if (config_.devices.size() > 1)
        ok(vdb_ivf_create_group(&c, config_.devices.data(), static_cast<uint32_t>(config_.devices.size()), &h_),
           "vdb_ivf_create_group");
    else
        ok(vdb_ivf_create(&c, &h_), "vdb_ivf_create");
}

IVFFlatIndex::~IVFFlatIndex() {
    if (h_) vdb_ivf_destroy(h_);
}

void IVFFlatIndex::train(const float* vectors, uint64_t n_vectors) {
    ok(vdb_ivf_train(h_, vectors, n_vectors), "train");
}

void IVFFlatIndex::add(const float* vectors, const uint64_t* ids, uint64_t n_vectors) {
    ok(vdb_ivf_add(h_, vectors, ids, n_vectors), "add");
}

void IVFFlatIndex::search(const float* queries, uint32_t n_queries, const SearchParams& params, float* distances,
                          uint64_t* indices) {
    ok(vdb_ivf_search(h_, queries, n_queries, params.nprobe, params.k, distances, indices), "search");
}

void IVFFlatIndex::search_batch(const std::vector<float*>& queries, const std::vector<SearchParams>& params,
                                std::vector<float*>& distances, std::vector<uint64_t*>& indices) {
    if (params.size() != queries.size() || distances.size() != queries.size() || indices.size() != queries.size())
        throw std::invalid_argument("search_batch: argument vectors differ in length");
    for (size_t i = 0; i < queries.size(); ++i) search(queries[i], 1, params[i], distances[i], indices[i]);
}

void IVFFlatIndex::warmup_lists(const std::vector<uint32_t>& list_ids) {
    ok(vdb_ivf_warmup(h_, list_ids.data(), static_cast<uint32_t>(list_ids.size())), "warmup_lists");
}

void IVFFlatIndex::evict_list(uint32_t list_id) { ok(vdb_ivf_evict(h_, list_id), "evict_list"); }

size_t IVFFlatIndex::get_gpu_memory_usage() const { return vdb_ivf_gpu_bytes(h_); }

size_t IVFFlatIndex::get_total_vectors() const { return vdb_ivf_ntotal(h_); }

void IVFFlatIndex::save(const std::string& path) const { ok(vdb_ivf_save(h_, path.c_str()), "save"); }

void IVFFlatIndex::load(const std::string& path) { ok(vdb_ivf_load(h_, path.c_str()), "load"); }

}  // namespace vdb
