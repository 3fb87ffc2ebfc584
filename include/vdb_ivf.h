/*
 * vdb_ivf.h — C ABI of the MI355X-native IVF-Flat engine (libvdb_ivf.so).
 *
 * This is the drop-in boundary for the reference's search path. Each entry point
 * names the reference interface it replaces (paths relative to the reference
 * repository, wedevxer/CUDA-AcceleratedVectorDatabaseEngine):
 *
 *   vdb_ivf_create        IVFFlatIndex::IVFFlatIndex(const Config&, TransferManager*)   engine/ivf_flat_index.h:44, .cpp:13-33
 *   vdb_ivf_destroy       IVFFlatIndex::~IVFFlatIndex()                                 engine/ivf_flat_index.h:45, .cpp:36-46
 *   vdb_ivf_train         IVFFlatIndex::train(const float*, uint64_t)                   engine/ivf_flat_index.h:47, .cpp:49-145
 *   vdb_ivf_add           IVFFlatIndex::add(const float*, const uint64_t*, uint64_t)    engine/ivf_flat_index.h:49, .cpp:148-202
 *   vdb_ivf_search        IVFFlatIndex::search(const float*, uint32_t, const SearchParams&, float*, uint64_t*)
 *                                                                                       engine/ivf_flat_index.h:51-53, .cpp:205-256
 *   vdb_ivf_warmup        IVFFlatIndex::warmup_lists(const std::vector<uint32_t>&)      engine/ivf_flat_index.h:60
 *   vdb_ivf_evict         IVFFlatIndex::evict_list(uint32_t)                            engine/ivf_flat_index.h:61
 *   vdb_ivf_gpu_bytes     IVFFlatIndex::get_gpu_memory_usage()                          engine/ivf_flat_index.h:63, .cpp:707-709
 *   vdb_ivf_ntotal        IVFFlatIndex::get_total_vectors()                             engine/ivf_flat_index.h:64
 *
 * The remaining entry points have no single reference counterpart; they expose the
 * device-resident and multi-GPU forms of the same path (the reference searches one
 * query and one list at a time on device 0, ivf_flat_index.cpp:214-255).
 *
 * Conventions: every call returns 0 on success and a negative code on failure;
 * vdb_last_error() then describes the failure (thread-local). Host buffers are
 * caller-owned and row-major (queries n x dim fp32; outputs n x k). Metric
 * ordinals follow kernels::Metric (engine/kernels.cuh:24-28): L2 = 0 (squared
 * L2), InnerProduct = 1 (negated dot), Cosine = 2 (the reference CPU path leaves
 * its distance at 0.0f, ivf_flat_index.cpp:351-362; mirrored exactly).
 * Unfilled result slots are (FLT_MAX, UINT64_MAX) as in ivf_flat_index.cpp:513-517.
 * Results are bit-identical to the reference CPU path (ids and distance bits).
 * No torch or HIP types appear in these signatures; streams are passed as void*.
 */
#ifndef VDB_IVF_H
#define VDB_IVF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    VDB_OK = 0,
    VDB_ERR_INVALID_ARGUMENT = -1,
    VDB_ERR_DEVICE = -2,
    VDB_ERR_OUT_OF_MEMORY = -3,
    VDB_ERR_UNSUPPORTED = -4,
    VDB_ERR_STATE = -5
};

enum { VDB_METRIC_L2 = 0, VDB_METRIC_INNER_PRODUCT = 1, VDB_METRIC_COSINE = 2 };

typedef struct vdb_ivf vdb_ivf;

/* Mirrors IVFFlatIndex::Config (engine/ivf_flat_index.h:16-22) plus the device. */
typedef struct vdb_ivf_config {
    uint32_t dimension;
    uint32_t nlist;
    int32_t metric;
    int32_t use_gpu;          /* accepted for API parity; the engine always runs on the GPU */
    uint64_t max_gpu_memory;  /* HBM cap on resident list bytes (count * (dim * 4 + 8) per list, the
                                 reference's gpu_memory_used_, ivf_flat_index.cpp:398-402). Once an add
                                 takes the lists above it, the handle switches to the list-cache tier
                                 with an HBM cache of this many bytes (lists home in page-locked host
                                 memory; results unchanged); lifting or raising the cap above the lists
                                 brings them back. Only list bytes count: the screen's bf16 shadow
                                 (about half the list bytes) is not list data. 0 = no cap: every list
                                 HBM-resident (288 GB per GPU). The reference searches lists that do
                                 not fit on the CPU; here an exact-path search (k > 64, Cosine, screen
                                 off) whose single query probes more than the cap fails with
                                 VDB_ERR_OUT_OF_MEMORY; the screened tier loads no list. */
    int32_t device;           /* HIP device ordinal */
} vdb_ivf_config;

/* Per-handle measurement, filled by vdb_ivf_profile_read (see DESIGN.md "Measurement"). */
typedef struct vdb_ivf_profile {
    uint64_t batches;          /* search batches executed since the last reset */
    uint64_t scan_launches;    /* ivf_scan kernel launches */
    double scan_ms;            /* summed ivf_scan durations (HIP events on the search stream) */
    double coarse_ms;          /* summed coarse-quantiser durations (distance + select) */
    double total_ms;           /* summed per-batch durations (first to last kernel) */
    uint64_t scan_vectors;     /* sum over batches of sum_{distinct probed local lists} n_l */
    uint64_t distinct_lists;   /* sum over batches of distinct probed local lists */
    uint64_t work_items;       /* sum over batches of scan work items */
    uint64_t scan_bytes;       /* algorithmic bytes read by ivf_scan: 4 * dim * scan_vectors */
    uint64_t pair_vectors;     /* sum over batches and (query, probe) pairs of n_l: distances computed */
    uint64_t exact_reranks;    /* screened / bounded scan: (query, vector) distances recomputed exactly (option bounded_stats) */
    uint64_t bounded_blocks;   /* screened / bounded scan: 64-vector blocks bounded on the matrix cores (option bounded_stats) */
    uint64_t computed_vectors; /* query slots the scan streams per vector: pair_vectors plus one per
                                  odd wide group (its last query runs alone, on scalar ops) */
    double local_merge_ms;     /* summed per-batch merges after the scan (segment, slot, query top-k) */
    uint64_t exchanges;        /* multi-GPU: exchanges timed below */
    double exchange_ms;        /* summed: this rank's results ready -> all-gather done (the wait for the
                                  slowest rank plus the collective itself) */
    double rank_merge_ms;      /* summed: all-gather done -> final results merged */
    uint64_t screen_collected; /* deferred screened scan: (query, vector) pairs collected against the
                                  upper-bound thresholds (option bounded_stats); exact_reranks counts
                                  the survivors of each pair's final threshold, recomputed exactly */
    double collect_ms;         /* deferred screened scan: summed durations of its collect kernel (the
                                  stream of the bf16 shadow; scan_ms covers it and the re-check kernels) */
    double recheck_ms;         /* ... and of the final thresholds, selection and exact re-checks after it */
    uint64_t screen_floor_batches; /* batches the run-time floor ran on the exact scan */
    uint64_t screen_floor_trips;   /* screened batches that tripped the floor */
    uint32_t screen_shadow;        /* the screen's shadow now: 0 none, 1 bf16, 2 int8 (option screen_i8) */
    uint32_t reserved0;
} vdb_ivf_profile;

const char* vdb_last_error(void);
const char* vdb_version(void);
/* Hash of the sources that shape the scan kernels and their launches (16 hex digits):
 * measurements (PMC traffic) are tied to the library they were taken on. */
const char* vdb_build_id(void);
int vdb_device_count(int* count);

int vdb_ivf_create(const vdb_ivf_config* config, vdb_ivf** out);
int vdb_ivf_destroy(vdb_ivf* index);

/* Training (k-means++ seeded with mt19937(42), then 10 Lloyd iterations), exactly
 * the reference algorithm; distances run on the GPU. */
int vdb_ivf_train(vdb_ivf* index, const float* vectors, uint64_t n);
int vdb_ivf_train_device(vdb_ivf* index, const float* d_vectors, uint64_t n);
int vdb_ivf_set_centroids(vdb_ivf* index, const float* centroids);  /* nlist x dim, host */
int vdb_ivf_get_centroids(vdb_ivf* index, float* centroids);        /* nlist x dim, host */

/* add: exact nearest-centroid assignment, lists appended in input order. */
int vdb_ivf_add(vdb_ivf* index, const float* vectors, const uint64_t* ids, uint64_t n);
int vdb_ivf_add_device(vdb_ivf* index, const float* d_vectors, const uint64_t* d_ids, uint64_t n);

/* Append rows to explicitly given lists (no assignment), input order kept per list.
 * Used by vdb_ivf_load and for indexes whose assignment was computed elsewhere. */
int vdb_ivf_add_to_lists(vdb_ivf* index, const float* vectors, const uint64_t* ids, const uint32_t* lists,
                         uint64_t n);
/* Exact assignment only (assign_to_lists, engine/ivf_flat_index.cpp:259-295): one list id
 * per row into a device array, nothing stored. With add_to_lists_device it splits `add`
 * (cpp:148-202) into two passes, so a sharded build can learn the final list sizes first. */
int vdb_ivf_assign_device(vdb_ivf* index, const float* d_vectors, uint64_t n, uint32_t* d_lists);
int vdb_ivf_add_to_lists_device(vdb_ivf* index, const float* d_vectors, const uint64_t* d_ids,
                                const uint32_t* d_lists, uint64_t n);
/* Persist / restore centroids and lists (IVFFlatIndex::save/load, engine/ivf_flat_index.h:66-67,
 * declared but never defined in the reference; this engine's own file format). */
int vdb_ivf_save(vdb_ivf* index, const char* path);
int vdb_ivf_load(vdb_ivf* index, const char* path);

/* search: host buffers in and out (PCIe included). nprobe is clamped to nlist.
 * Thread-safe: concurrent callers are coalesced into shared device batches (calls with
 * the same nprobe and k), each call keeping exactly the results it would get alone
 * (option "coalesce" = 0 serialises calls instead). */
int vdb_ivf_search(vdb_ivf* index, const float* queries, uint32_t n, uint32_t nprobe, uint32_t k,
                   float* distances, uint64_t* ids);
/* search on device buffers, enqueued on `stream` (NULL = the handle's stream),
 * asynchronous. When a shard is set (vdb_ivf_set_shard with world > 1) the outputs
 * are this rank's partial results, to be combined with vdb_merge_ranks_device. */
int vdb_ivf_search_device(vdb_ivf* index, const float* d_queries, uint32_t n, uint32_t nprobe,
                          uint32_t k, float* d_distances, uint64_t* d_ids, void* stream);

/* Multi-GPU: restrict this handle to the lists rank `rank` owns out of `world`
 * (size-balanced LPT over list lengths, identical on every rank), and free the
 * rest of the list arena. Emptiness of non-owned lists is still tracked. */
int vdb_ivf_set_shard(vdb_ivf* index, uint32_t rank, uint32_t world);
/* Sharded build of an index larger than one GPU (100M x 768 over 8 GPUs): on an empty,
 * trained index, fix this rank's lists from the final list sizes (the same LPT plan as
 * set_shard); later adds store only those lists' rows and count the others. */
int vdb_ivf_plan_shard(vdb_ivf* index, uint32_t rank, uint32_t world, const uint64_t* final_sizes);
/* Combine per-rank partials gathered as [nranks][n][k] into final [n][k]. */
int vdb_merge_ranks_device(const float* d_dist, const uint64_t* d_ids, uint32_t nranks, uint32_t n,
                           uint32_t k, float* d_out_dist, uint64_t* d_out_ids, void* stream);
/* One rank's partials as a single record for ONE collective per batch: f32 dist[n][k],
 * padded to 8 bytes, then u64 ids[n][k]. vdb_rank_record_bytes gives its size; a
 * search writes into it with d_distances = record, d_ids = record + that padding. */
uint64_t vdb_rank_record_bytes(uint32_t n, uint32_t k);
/* Combine gathered records [nranks][record] into final [n][k]. */
int vdb_merge_ranks_packed_device(const void* d_records, uint32_t nranks, uint32_t n, uint32_t k,
                                  float* d_out_dist, uint64_t* d_out_ids, void* stream);
/* Host-only: the LPT owner of every list for `world` ranks (no GPU needed). */
int vdb_shard_plan(const uint64_t* list_sizes, uint32_t nlist, uint32_t world, uint32_t* owner);
/* Host-only: LPT over each list's expected scan cost per batch of `batch` queries, from a
 * probe census (probe_counts[l] of n_sample query-like rows probe list l): the list is
 * streamed once per group of 16 queries that probe it (binomial expectation) plus the
 * per-query distance arithmetic. Balances the ranks' scan time where list popularity, not
 * only list size, differs. Identical on every rank for the same inputs. */
int vdb_shard_plan_probe_weighted(const uint64_t* list_sizes, const uint64_t* probe_counts, uint64_t n_sample,
                                  uint32_t batch, uint32_t nlist, uint32_t world, uint32_t* owner);
/* counts[l] = how many of the n device rows d_rows (n x dim) probe list l with `nprobe`
 * (the exact probe selection of search; nlist entries written). */
int vdb_ivf_probe_census(vdb_ivf* index, const float* d_rows, uint64_t n, uint32_t nprobe, uint64_t* counts);
/* set_shard / plan_shard with an explicit plan (owner[l] = rank of list l, the same array
 * on every rank), e.g. from vdb_shard_plan_probe_weighted. */
int vdb_ivf_set_shard_owners(vdb_ivf* index, uint32_t rank, uint32_t world, const uint32_t* owner);
int vdb_ivf_plan_shard_owners(vdb_ivf* index, uint32_t rank, uint32_t world, const uint64_t* final_sizes,
                              const uint32_t* owner);

/* ---- Multi-GPU inside the engine (RCCL over xGMI) ----
 * One process per GPU: rank 0 draws a communicator id (vdb_comm_unique_id) and shares it
 * with the other ranks (any channel); every rank, after set_shard / plan_shard with the
 * same (rank, world), calls vdb_ivf_attach_comm. From then on vdb_ivf_search_device /
 * vdb_ivf_search on that handle all-gather every batch's per-rank partials (ONE RCCL
 * all-gather per batch of vdb_rank_record_bytes per rank) and merge them on the device,
 * so every rank receives the FINAL results. Every rank must issue the same search calls
 * (same n, nprobe, k and batch option) in the same order; on such a handle vdb_ivf_search
 * does not coalesce concurrent callers (the grouping would depend on each rank's timing):
 * calls run one at a time. At world > 1 a call ends in ONE all-gather of the whole call's
 * partials (not one per batch): a rank's own state (its list-cache tier, which its shard's
 * size may switch on, and what its cache holds) shapes its batches, so only per-call
 * exchanges are the same on every rank. */
#define VDB_COMM_ID_BYTES 128
int vdb_comm_unique_id(void* id); /* VDB_COMM_ID_BYTES bytes (ncclGetUniqueId) */
int vdb_ivf_attach_comm(vdb_ivf* index, const void* id, uint32_t rank, uint32_t world);
int vdb_ivf_detach_comm(vdb_ivf* index);
/* The communicator's deadline (option "comm_timeout_ms", default 120000): init is
 * non-blocking and polled, so a rank that never joins makes vdb_ivf_attach_comm fail with
 * VDB_ERR_DEVICE naming this rank; at attach every rank's dimension, nlist, metric, batch,
 * stale_slots and list sizes are compared, and the ranks' stored lists must
 * partition the non-empty lists (VDB_ERR_STATE otherwise). Each exchange's completion is watched; one
 * still pending after the deadline marks the communicator failed (later searches fail with
 * the message). vdb_ivf_comm_status returns VDB_OK, or VDB_ERR_DEVICE with that message,
 * and the exchanges issued / completed so far (either pointer may be NULL): a caller
 * waiting on its streams polls it to stop waiting on a stalled peer. After a failure the
 * process is expected to exit; vdb_ivf_detach_comm then aborts the communicator. */
int vdb_ivf_comm_status(vdb_ivf* index, uint64_t* exchanges_issued, uint64_t* exchanges_done);
/* One process driving several GPUs: a group handle with one member index per device
 * (devices[0] holds the host-API staging; device pointers passed to the group's calls
 * live on devices[0]). The group is used through every call of this header like a
 * single-device handle: train runs on devices[0] and its centroids are copied to every
 * member; add places each list on a member when the list first receives vectors
 * (largest first on the least-loaded member: the LPT plan of vdb_shard_plan for a bulk
 * add) and every member stores its lists; a search broadcasts the queries (RCCL), runs
 * each member's shard and all-gathers + merges per batch, with results bit-identical to
 * one device. Members on distinct devices use ncclCommInitAll; members sharing a device
 * (a one-GPU rehearsal) exchange through device copies. The list-cache tier and the
 * max_gpu_memory cap act per member (per GPU); a call on a group with tiered members ends
 * in one exchange for the whole call. Not available on a group: set_shard, plan_shard,
 * open_lists. */
int vdb_ivf_create_group(const vdb_ivf_config* config, const int* devices, uint32_t ndevices, vdb_ivf** out);
uint32_t vdb_ivf_group_size(const vdb_ivf* index); /* members; 1 for a single-device handle */
/* Per list the member (group) or rank (sharded handle) storing it; UINT32_MAX: none. */
int vdb_ivf_list_owners(vdb_ivf* index, uint32_t* owner);

/* List residency. By default the whole index is HBM-resident (288 GB per GPU) and
 * these keep the API. With the list-cache tier (option "list_cache_bytes" > 0) the
 * lists live in page-locked host memory and HBM caches whole lists under that byte
 * cap, like the reference's load_list_to_gpu / evict_list_from_gpu
 * (engine/ivf_flat_index.cpp:387-471, ivf_flat_index.h:60-61): warmup loads lists
 * (one that cannot fit is skipped), evict drops one, and a search loads the lists
 * each batch probes first (least recently used lists make room). Results are the
 * same in both modes. */
int vdb_ivf_warmup(vdb_ivf* index, const uint32_t* lists, uint32_t n);
int vdb_ivf_evict(vdb_ivf* index, uint32_t list);
typedef struct vdb_ivf_cache_stats_t {
    uint64_t capacity_bytes;  /* 0: tier off */
    uint64_t resident_bytes;
    uint64_t resident_lists;
    uint64_t loads;           /* lists copied host -> HBM */
    uint64_t evictions;       /* lists evicted to make room (not counting vdb_ivf_evict) */
    uint64_t bytes_loaded;
    uint64_t file_bytes_read; /* lists served from a file: bytes read from it */
    uint64_t subbatches;      /* sub-batches searched through the tier (cut to fit the cache) */
    uint64_t prefetches;      /* sub-batches whose lists were loaded while the previous one scanned */
    uint64_t sync_loads;      /* sub-batches whose lists were loaded before their own scan */
    int32_t io_uring;         /* 1: the file home is read through io_uring (0: pread fallback) */
    int32_t o_direct;         /* 1: the file home is read with O_DIRECT */
    /* The screen in the tier (L2 / IP, k <= 64): the lists' bf16 shadow, norms and ids stay in
     * HBM and only the exact re-checks' rows are read from the home, per batch. */
    int32_t screen_resident;      /* 1: the shadow of every stored list is HBM-resident */
    int32_t reserved;
    uint64_t screen_bytes;        /* HBM of the resident shadow, norms and ids */
    uint64_t screen_batches;      /* batches the screen served in the tier */
    uint64_t screen_rows_fetched; /* survivors' rows read from the file home (host home: read over PCIe) */
    uint64_t screen_row_bytes;
    uint64_t screen_reruns;       /* batches re-run after overflowing the candidate buffer */
    uint64_t screen_rows_cached;  /* survivor rows read from the HBM cache instead of the file
                                     (option tier_row_cache: the largest lists' rows kept there) */
    uint64_t screen_fallbacks;    /* batches whose candidates would exceed "tier_cand_max": served
                                     by the exact list-cache path instead */
} vdb_ivf_cache_stats_t;
int vdb_ivf_cache_stats(vdb_ivf* index, vdb_ivf_cache_stats_t* out);
/* The screened tier's row cache (file home, option tier_row_cache): refill the HBM list
 * cache with the lists that save the most survivor-row reads per cached byte, by
 * weights[l] / count[l] (weights: per list its expected survivor rows, e.g. the histogram of
 * the batches served so far from vdb_ivf_survivor_histogram), or by list size when weights is
 * null (the default). The order is kept for later fills (a rebuilt screen). */
int vdb_ivf_fill_row_cache(vdb_ivf* index, const uint64_t* weights);
/* Per list (nlist entries): the survivor rows the screened tier's batches needed so far. */
int vdb_ivf_survivor_histogram(vdb_ivf* index, uint64_t* out);
/* Diagnostics (option "collect_stamps" = N records): the screened collect kernel's timeline,
 * 4 x u64 per record {batch << 40 | item << 16 | workgroup, start, end (wall clock ticks),
 * queries | segments << 8 | kind << 16 (0 wide item, 1 narrow item, 2 workgroup start) |
 * list << 32}; copies min(cap, *n) records, *clock_hz = the wall clock's rate, and resets the
 * buffer. Synchronises the handle. */
int vdb_ivf_collect_stamps(vdb_ivf* index, uint64_t* out, uint64_t cap, uint64_t* n, uint64_t* clock_hz);
/* The tier's home on disk (ListPrefetcher::register_list_file / prefetch_lists,
 * engine/prefetcher.h:139-183; list files of format/storage.h): serve this handle's lists
 * from an index file written by vdb_ivf_save, without reading them into memory.
 * Centroids and list sizes are read at once; a list is read (pread -> pinned staging ->
 * HBM -> pad + interleave on the device) when a batch first probes it or on
 * vdb_ivf_warmup, and evicted like any cached list. Needs "list_cache_bytes" > 0 set
 * first; the handle becomes read-only (add fails with VDB_ERR_STATE). A shard file
 * (vdb_ivf_save of a handle with world > 1: every list's count, only the rank's own lists'
 * rows) makes this handle that rank's shard: rank and world come from the file and the lists
 * it stores define the shard (any plan; nothing is checked against a plan here, only
 * vdb_ivf_attach_comm's partition check across the ranks); vdb_ivf_attach_comm then serves a
 * sharded index larger than the node's HBM from every rank's own file.
 * With the screen (L2 / IP, k <= 64) the first search streams the file once to build the
 * lists' bf16 shadow, norms and ids in HBM; later searches read only the exact re-checks'
 * rows from the file (one O_DIRECT read each, option "tier_row_direct" 0: buffered). */
int vdb_ivf_open_lists(vdb_ivf* index, const char* path);

/* get_gpu_memory_usage's definition: count * (dim * 4 + 8) bytes per GPU-resident list. */
uint64_t vdb_ivf_gpu_bytes(const vdb_ivf* index);
/* Device memory this handle really holds: the lists in every layout it keeps (row-major
 * fp32 copy, bf16 shadow and norms while the screen serves; the interleaved arena otherwise
 * or when an exact-path search rebuilt it; the whole cache in the list-cache tier), ids,
 * centroids, directories, every search workspace and staging buffer. */
uint64_t vdb_ivf_gpu_bytes_allocated(const vdb_ivf* index);
uint64_t vdb_ivf_ntotal(const vdb_ivf* index);
uint32_t vdb_ivf_dimension(const vdb_ivf* index);
uint32_t vdb_ivf_nlist(const vdb_ivf* index);
int vdb_ivf_list_sizes(const vdb_ivf* index, uint64_t* sizes);  /* nlist entries */
/* Copy list `list` out row-major (count x dim) with its ids, in add order. */
int vdb_ivf_get_list(vdb_ivf* index, uint32_t list, float* vectors, uint64_t* ids);

/* Queries per internal batch (default 256; bounded so batch * nprobe <= 8192). */
int vdb_ivf_set_batch(vdb_ivf* index, uint32_t batch);
/* Reference quirk A1: an empty probed list leaves the previous query's
 * slot content in the merge. 1 (default) reproduces it; 0 drops empty slots. */
int vdb_ivf_set_stale_slots(vdb_ivf* index, int enable);

/* Coarse-quantiser mode: 1 (default) = MFMA distance bounds + exact re-rank of the
 * lists that can reach the top nprobe (same probe sets as mode 0); 0 = exact VALU
 * distances of every centroid. Cosine always uses mode 0. */
int vdb_ivf_set_coarse_mode(vdb_ivf* index, int mode);
/* Engine tuning knobs by name (results never change, only speed): "coarse_mode"
 * (0/1, as above), "wide_scan" (0/1: large lists as multi-query workgroup items),
 * "wide_stride" (prime dispatch stride of wide items; 1 = plan order), "batch",
 * "stale_slots" (as vdb_ivf_set_batch / vdb_ivf_set_stale_slots), "seg_vectors" (0 = auto, or
 * 64/128/256/512/1024: list vectors per scan segment), "coalesce" (0/1), "coalesce_max_queries",
 * "coalesce_window_us" (0: no waiting; calls arriving while the device is busy batch up),
 * "fused_scan" (1, default: one persistent scan grid takes both the wide and the narrow
 * items; 0: narrow items on a second stream), "screen" (1, default: the screened scan — bf16
 * matrix-core distance bounds from a shadow of the lists, exact fp32 sums only for pairs that can
 * reach a list's top-k; L2/IP, k <= 64; the lists are then held as a row-major fp32 copy plus the
 * bf16 shadow and norms, ~1.5x the list bytes, for every k: exact-path searches, k > 64, scan
 * the row-major copy; in the list-cache tier the shadow alone stays
 * in HBM and the rows at home; 0: the exact VALU scan of every pair), "screen_group" (16,
 * default, or 32: queries per screened wide item; with the deferred scan every shadow tile
 * then feeds two 16-query A operands, inline: two wave halves), "screen_defer" (1, default:
 * the screen collects candidates against upper-bound thresholds and re-checks afterwards only
 * the survivors of each (query, list) pair's final threshold; 0: re-checks inline as
 * candidates appear), "screen_recheck2" (1, default: the survivors are re-checked in two passes —
 * each pair's k smallest lower bounds first, then only the others not above their k-th exact
 * distance; in the file-home tier as two read phases; 0: every survivor in one pass; results are
 * identical), "screen_cand_cap" (collected candidates per batch, default 4M; a pair
 * beyond it is recomputed over its whole list, a file-home tier batch re-run with more, up to
 * "tier_cand_max" (32M: beyond it that batch is served by the exact list-cache path)),
 * "tier_row_direct" (1, default: the screened tier reads survivors' rows with O_DIRECT),
 * "tier_row_qd" (256: survivor-row reads in flight), "tier_row_cache" (1, default: a file-home
 * screened tier fills its idle HBM cache with the largest lists, whose survivors' rows are then
 * copied from HBM instead of read from the file), "screen_i8" (2, default: automatic —
 * int8 for lists in HBM unless the build's calibration batch vetoes it (survivors beyond k above
 * 1.5 % of the pairs, or an overflow), bf16 in the list-cache tier; 1: int8 with a per-vector
 * scale, a quarter of the fp32 bytes, a wider bound; 0: bf16, half the fp32 bytes), "screen_thr_every" (0 = automatic: blocks
 * between the collect kernel's re-reads of the shared thresholds; 4 for 32-query items, else 1),
 * "screen_floor_ppm" (50000, default: a screened batch of at least "screen_floor_min" (4M)
 * (query, vector) pairs that overflowed its candidate buffer, or whose survivors beyond k per
 * (query, list) pair exceed this many per million of its pairs, sends the next
 * "screen_floor_skip" (32) batches to the exact scan, twice as many after each further trip in
 * a row (at most 32x), then the screen is tried again; 0: never; lists in HBM only),
 * "list_cache_bytes" (0 = every list HBM-resident; > 0 = the list-cache tier above with an
 * HBM cache of that many bytes; a search whose single query probes more fails with
 * VDB_ERR_OUT_OF_MEMORY, a batch probing more is split; setting it replaces the
 * max_gpu_memory cap), "max_gpu_memory" (the Config cap, applied at once), "bounded_stats"
 * (0/1: count the screened / bounded scan's exact re-checks and blocks in vdb_ivf_profile). Timing experiments
 * that change results exist only as separate builds (VDB_SCAN_DIAG), never as options. */
int vdb_ivf_set_option(vdb_ivf* index, const char* name, int64_t value);
/* Host-API coalescing counters: device batches run and search() calls they served. */
int vdb_ivf_coalesce_stats(vdb_ivf* index, uint64_t* batches, uint64_t* requests);

int vdb_ivf_profile_enable(vdb_ivf* index, int enable);
int vdb_ivf_profile_reset(vdb_ivf* index);
int vdb_ivf_profile_read(vdb_ivf* index, vdb_ivf_profile* out);  /* synchronises the stream */

/* Wait for all work the handle enqueued on its own stream. */
int vdb_ivf_synchronize(vdb_ivf* index);
/* The handle's stream (hipStream_t as void*). */
void* vdb_ivf_stream(vdb_ivf* index);

/* Deterministic N(0,1) fp32 generator on the device (synthetic benchmark data):
 * element e of the stream (seed, offset + i) is written to d_out[i]. */
int vdb_gen_normal_device(float* d_out, uint64_t n, uint64_t seed, uint64_t offset, void* stream);
/* Gaussian-mixture rows (synthetic clustered data, balanced IVF lists): row row0 + r
 * belongs to a component drawn from (seed, row), x = d_centers[comp] (ncomp x dim,
 * device) + sigma * N(0,1). Independent of how the rows are split into calls. */
int vdb_gen_mixture_device(float* d_out, uint64_t rows, uint32_t dim, const float* d_centers, uint32_t ncomp,
                           float sigma, uint64_t seed, uint64_t row0, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VDB_IVF_H */
