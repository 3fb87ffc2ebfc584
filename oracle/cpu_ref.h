/*
 * oracle/cpu_ref.h — TEST INFRASTRUCTURE ONLY.
 *
 * C ABI of the CPU restatement of the reference's IVF-Flat CPU path
 * (`IVFFlatIndex` with `use_gpu=false`, /root/reference/engine/ivf_flat_index.cpp).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * the library built from this header; the product path never does.
 *
 * Parity status: the reference's own tests hold no golden values;
 * running the reference itself was denied in this environment, so
 * this restatement is pinned by the reference-derived known-answer test
 * (bench/benchmark.cpp:130-138 re-seeds the generator, so query i == vector i),
 * the reference's validity rules (test/gpu_vs_cpu_test.cpp:200-226), and an
 * independent numpy restatement (oracle/np_ref.py). See DESIGN.md "Oracle".
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_ivf oracle_ivf;

/* Metric ordinals follow kernels::Metric (kernels.cuh:24-28): L2=0, IP=1, Cosine=2. */
oracle_ivf* oracle_create(uint32_t dim, uint32_t nlist, int metric);
void oracle_destroy(oracle_ivf* h);

/* IVFFlatIndex::train (ivf_flat_index.cpp:49-145), CPU branch. */
void oracle_train(oracle_ivf* h, const float* vectors, uint64_t n);
/* Only the k-means++ seeding of train (ivf_flat_index.cpp:52-104). */
void oracle_train_seed_only(oracle_ivf* h, const float* vectors, uint64_t n);
/* IVFFlatIndex::add (ivf_flat_index.cpp:148-202), CPU branch. */
void oracle_add(oracle_ivf* h, const float* vectors, const uint64_t* ids, uint64_t n);
/* IVFFlatIndex::search (ivf_flat_index.cpp:205-256), CPU branch, single thread.
 * nprobe is clamped to nlist (the reference reads out of bounds there, UB). */
void oracle_search(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe,
                   uint32_t k, float* distances, uint64_t* indices);
/* Same results, queries spread over `threads` OpenMP threads (0 = all). */
void oracle_search_mt(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe,
                      uint32_t k, float* distances, uint64_t* indices, int threads);
/* Per-rank partial of a list-sharded search: the unique-id top-k over the probe
 * slots whose content comes from a list with owned[list] != 0 (stale slots
 * included, see ivf_flat_index.cpp:210-233). oracle_merge_ranks of all ranks'
 * partials equals oracle_search. */
void oracle_search_shard(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe,
                         uint32_t k, const uint8_t* owned, float* distances, uint64_t* indices);
void oracle_search_shard_mt(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k,
                            const uint8_t* owned, float* D, uint64_t* I, int threads);
/* oracle_search_shard over a shard streamed in one list at a time: begin records the call's
 * probes (the centroids and every list's count must be set), then for each owned probed list
 * load its rows (oracle_list_resize), oracle_stream_scan it and drop the rows again
 * (oracle_list_set_count); finish writes the partials and frees the stream. */
typedef struct oracle_stream oracle_stream;
oracle_stream* oracle_stream_begin(oracle_ivf* h, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k);
uint32_t oracle_stream_probed(const oracle_stream* st, uint32_t list);
void oracle_stream_scan(oracle_stream* st, uint32_t list, int threads);
void oracle_stream_finish(oracle_stream* st, const uint8_t* owned, float* distances, uint64_t* indices);
void oracle_merge_ranks(const float* dist, const uint64_t* ids, uint32_t nranks, uint32_t n,
                        uint32_t k, float* out_dist, uint64_t* out_ids);

/* select_nprobe_lists (ivf_flat_index.cpp:298-336): writes min(nprobe, nlist) ids. */
void oracle_select_nprobe(oracle_ivf* h, const float* query, uint32_t nprobe, uint32_t* out);
/* assign_to_lists (ivf_flat_index.cpp:259-295). */
void oracle_assign(oracle_ivf* h, const float* vectors, uint64_t n, uint32_t* out);
/* The same, rows over `threads` OpenMP threads (0: all): bit-identical per row. */
void oracle_assign_mt(oracle_ivf* h, const float* vectors, uint64_t n, uint32_t* out, int threads);

void oracle_get_centroids(oracle_ivf* h, float* out);
void oracle_set_centroids(oracle_ivf* h, const float* centroids);
uint64_t oracle_list_count(oracle_ivf* h, uint32_t list);
void oracle_get_list(oracle_ivf* h, uint32_t list, float* vectors, uint64_t* ids);
/* Replace list contents (used to mirror an index built elsewhere). */
void oracle_set_list(oracle_ivf* h, uint32_t list, const float* vectors, const uint64_t* ids,
                     uint64_t count);
/* Resize list storage and hand back pointers so a caller can fill it in place. */
/* Count-only list (stored on another shard): emptiness is kept, no rows. */
void oracle_list_set_count(oracle_ivf* h, uint32_t list, uint64_t count);
void oracle_list_resize(oracle_ivf* h, uint32_t list, uint64_t count, float** vectors,
                        uint64_t** ids);
uint64_t oracle_total_vectors(oracle_ivf* h);

/* std::mt19937(seed) + std::normal_distribution<float>(0,1), n draws in order
 * (test/gpu_vs_cpu_test.cpp:83-94, test/simple_test.cpp:127-135,
 * bench/benchmark.cpp:132-138). Same libstdc++ as the reference build. */
void oracle_gen_normal(uint32_t seed, uint64_t n, float* out);

#ifdef __cplusplus
}
#endif
