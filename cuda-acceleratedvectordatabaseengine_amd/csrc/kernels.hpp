// kernels.hpp — launchers for the gfx950 IVF-Flat kernels (kernels.hip).
//
// HBM layouts (DESIGN.md "Data layout"):
//   * list arena: vectors in blocks of 64, each block [D4][64 lanes][float4]
//     (D4 = ceil(dim/4), zero-padded dims), so one wave-instruction reads 1 KiB
//     contiguous; ids [block*64 + lane] uint64.
//   * centroids: the same interleaved layout (coarse step), plus a zero-padded
//     row-major copy [nlist][Dp] (training).
//   * queries: zero-padded row-major [B][Dp], Dp = 4*D4. Zero pads add +0.0f to
//     sums that can never be -0.0f, so distances keep the reference's bits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vdbk {

constexpr int kMaxSegBlocks = 16;          // 64-vector blocks per scan segment (the runtime
                                           // size is 1..8, chosen per shard size by the engine)
constexpr int kTilePipe = 16;              // float4 tiles of a list vector in flight per lane (scan)
constexpr uint32_t kMfmaBlockedRows = 1024;  // coarse bounds: 2x2-blocked MFMA kernel from this many rows
#ifndef VDB_MERGE_BLOCKS
#define VDB_MERGE_BLOCKS 1024  // measured: 53 -> 27 us per batch vs 256, throughput unchanged
#endif
constexpr uint32_t kMergeBlocks = VDB_MERGE_BLOCKS;  // level-1 partial merge: workgroups (grid-stride)
#ifndef VDB_TILE_PIPE_NARROW
#define VDB_TILE_PIPE_NARROW 4
#endif
constexpr int kTilePipeNarrow = VDB_TILE_PIPE_NARROW;  // the same for narrow items (queries held in SGPRs)
// Scan timing experiments (a separate build, tools/build_variant.sh; never a runtime option):
// 1 skip top-k upkeep, 2 one query pair per wave, 4 no insertion on a segment's first block,
// 8 insertions on its first block only, 16 no LDS reads of query pairs in the wide loop (tile
// 0's pairs reused), 32 no list reads in the loop (the first tiles reused). Every non-zero
// value makes search results INVALID.
#ifndef VDB_SCAN_DIAG
#define VDB_SCAN_DIAG 0
#endif
constexpr int kTileAlign = kTilePipe;      // D4 is padded to whole pipeline rounds
constexpr int kMergeFan = 32;              // segment partials folded per level-1 merge wave
constexpr int kWideGroup = 16;             // max queries per wide scan item (4-wave items)
constexpr int kWaveQueries = 16;           // max queries one wave of a wide item computes (8 pairs)
constexpr int kWideMinSeg = 4;             // lists with >= 4 segments are scanned by wide items
constexpr int kNarrowMax = 4;              // pairs per narrow scan item
constexpr int kPlanMaxPairs = 8192;        // batch * nprobe per plan launch
constexpr int kMaxK = 1024;                // top-k capacity (16 registers x 64 lanes)
constexpr size_t kLdsBytes = 160 * 1024;   // LDS per CU (gfx950)
constexpr uint32_t kPersistentBlocks = 512; // scan grid: 2 workgroups per CU on 256 CUs
// per-batch counters (the plan kernel's [0, 8), then the deferred screened scan's)
constexpr int kCtrValid = 8;   // valid (query, probe) pairs of the batch (sorted pairs [0, n))
constexpr int kCtrCand = 9;    // candidates the screen collected (may exceed the buffer)
constexpr int kCtrSurv = 10;   // survivors of the final thresholds
constexpr int kCtrPairs = 11;  // (query, vector) pairs of the batch (saturating at 2^32 - 1)
constexpr int kCtrOvf = 12;    // 1 when a collected candidate fell beyond the buffer (its pair marked in ovf)
constexpr int kCtrReal = 13;   // candidates the screen collected (kCtrCand counts reserved slots: padded chunks)
constexpr uint32_t kCandChunk = 128;  // candidate slots a collect wave reserves at once (screen.hip)
constexpr int kCounters = 16;
constexpr int kUbLists = 128;   // deferred screened scan: upper-bound lists kept per (query, list) pair

struct ScanItem {
    uint32_t list;
    uint32_t seg;
    uint32_t pair_start;
    uint32_t npairs;
};

// Number of lane registers for a list of capacity k, and the query-group size the
// scan kernel uses for that register count.
inline int topk_regs(uint32_t k) {
    int r = 1;
    while (r * 64 < (int)k) r <<= 1;
    return r;
}
__host__ __device__ constexpr int scan_group_max(int regs) { return regs == 1 ? 4 : (regs == 2 ? 2 : 1); }
inline int scan_group(int regs) { return scan_group_max(regs); }

// ---- search ----
void launch_pad_rows(const float* src, uint64_t n, uint32_t dim, uint32_t dp, float* dst, hipStream_t s);
void launch_coarse(int metric, const float4* cent_il, uint32_t nlist, uint32_t d4, const float* qpad,
                   uint32_t B, float* cd, hipStream_t s);
// Coarse step on the matrix cores (L2 / IP): bounds-carrying approximate distances
// [B][nlist] + their error bounds, then exact re-rank of the lists that can reach the
// top P (bit-identical probe sets to the exact path).
void launch_coarse_mfma(int metric, const float* cent_rm, uint32_t nlist, uint32_t dp, const float* qpad,
                        uint32_t B, float* approx, float* delta, hipStream_t s);
// LDS rows per re-rank chunk for padded dimension dp (0: dp too large for the MFMA path).
uint32_t rerank_rows(uint32_t dp, int regs);
void launch_select_rerank(int metric, int regs, const float* approx, const float* delta, const float* cent_rm,
                          uint32_t nlist, uint32_t dp, const float* qpad, uint32_t B, uint32_t P, uint32_t* cand,
                          uint32_t* probes, hipStream_t s);
// assign_to_lists from the MFMA bounds: exact argmin (ties to the lowest centroid).
void launch_assign_rerank(int metric, const float* approx, const float* delta, const float* cent_rm,
                          uint32_t nlist, uint32_t dp, const float* rows, uint32_t n, uint32_t* out, hipStream_t s);
void launch_select(int regs, const float* cd, uint32_t nlist, uint32_t B, uint32_t P, uint32_t* probes,
                   hipStream_t s);
void launch_plan(const uint32_t* probes, const uint32_t* nseg_local, const uint32_t* count_local,
                 uint32_t B, uint32_t P, uint32_t group, int wide, uint32_t segs_item, ScanItem* items, ScanItem* items_w,
                 uint32_t* counters, uint32_t* sorted_pair, uint32_t* part_base_sorted, uint32_t* part_base_qp,
                 uint32_t* nseg_qp, uint32_t* l1base_qp, uint2* l1_items, unsigned long long* stats,
                 uint32_t* thr, uint32_t mfma_min, hipStream_t s);
void launch_merge_partials(int regs, uint32_t grid_items, const uint32_t* probes, const uint32_t* count_global,
                           const uint32_t* nseg_qp, const uint32_t* part_base_qp, const uint32_t* l1base_qp,
                           const uint2* l1_items, const uint32_t* counters, const float* part_d,
                           const uint64_t* part_i, uint32_t k, float* l1_d, uint64_t* l1_i, hipStream_t s);
// Fine scan of one batch (kernels.hip): small lists as narrow items (one wave each),
// large lists as wide items (one workgroup: 4 segments x <= 16 queries in LDS).
struct ScanArgs {
    const float4* __restrict__ arena;
    const uint64_t* __restrict__ ids;
    const uint64_t* __restrict__ block_off;
    const uint32_t* __restrict__ count;
    const float* __restrict__ qpad;
    const ScanItem* __restrict__ items;
    const ScanItem* __restrict__ items_w;
    const uint32_t* __restrict__ counters;
    const uint32_t* __restrict__ sorted_pair;
    const uint32_t* __restrict__ part_base_sorted;
    float* __restrict__ part_d;
    uint64_t* __restrict__ part_i;
    uint32_t d4;
    uint32_t k;
    uint32_t wide_stride;  // wide-item dispatch stride (prime; 0/1 = plan order)
    uint32_t* work;        // [3] item queues (narrow, wide, bounded), reset by the plan kernel
    uint32_t seg_blocks;   // 64-vector blocks per list segment (one wave's unit of a scan item)
    uint32_t segs_item;   // segments per wide item (>= 4; the 4 waves take them dynamically)
    uint32_t fused;        // ivf_scan_wide also drains the narrow queue (R = 1); the last `fused`
                           // workgroups start on narrow items (0: narrow items on their own kernel)
    uint32_t* thr;         // per sorted (query, probe) pair: the best k-th distance any wave has
                           // reached on that list so far (order-preserving uint encoding, reset
                           // by the plan kernel); candidates strictly worse are never inserted
    uint32_t mfma_min;     // wide items of >= this many queries run the bounded (MFMA) waves (0: never)
    unsigned long long* mstats;  // bounded-scan statistics (option bounded_stats; null by default):
                                 // [0] exact re-ranks, [1] bounded blocks
    // Screened scan (screen.hip): the lists' bf16 residual shadow in MFMA B-operand order,
    // their fp32 rows in slot order (exact re-checks) and per-slot norms; per (query, probe)
    // pair (q * P + p) the bf16 A rows [B * P][dp] and their norms.
    const uint4* __restrict__ shadow = nullptr;
    const float* __restrict__ rows = nullptr;
    const float4* __restrict__ meta = nullptr;
    const uint16_t* __restrict__ qres = nullptr;
    const float4* __restrict__ pst = nullptr;
    const float* __restrict__ sscale = nullptr;  // int8 shadow (deferred screen): per slot s_b (null: bf16)
    const float* __restrict__ qscale = nullptr;  // ... per (query, probe) pair s_a
    uint32_t dp = 0;
    uint32_t P = 0;
    uint32_t wide_q = 16;  // queries per screened wide item at most (16 or 32)
    uint32_t thr_every = 1;  // deferred screen: blocks between re-reads of the shared (global) thresholds
    uint32_t* thr4 = nullptr;  // per sorted pair, 4 quarter-list thresholds (screen.hip)
    // Deferred screened scan: collected (sorted pair, slot, lower bound, rank) entries, their
    // capacity, the collection counter (counters + kCtrCand) and per sorted pair the overflow mark.
    uint4* cand = nullptr;
    uint32_t cand_cap = 0;
    uint32_t* ccount = nullptr;
    uint32_t* ovf = nullptr;
    uint4* floor_out = nullptr; // (page-locked, mapped) {survivors, pairs, sequence, 1} of the batch: the run-time floor
    uint32_t floor_seq = 0;
    float* ublist = nullptr;    // per sorted pair kUbLists lists of k upper bounds (the waves' running lists)
    uint32_t* ubcnt = nullptr;  // ... and how many were offered
    // The exact scans (ivf_scan_narrow / ivf_scan_wide, 4-wave items) read `arena` as the
    // lists' row-major fp32 copy ([slot][dp], one slack block) instead of the interleaved
    // layout: the arena released while the screen serves (one fp32 copy in HBM).
    uint32_t rows_layout = 0;
    // (option collect_stamps, diagnostics) per collect item a record of 4 u64 {batch << 40 |
    // item << 16 | workgroup, wall clock at its start, at its end, nq | segments << 8 | kind
    // << 16 | list << 32} (kind 0 wide item, 1 narrow item, 2 workgroup start); stamps[0]
    // counts records, stamps_cap bounds them
    unsigned long long* stamps = nullptr;
    uint32_t stamps_cap = 0;
    uint32_t stamp_batch = 0;
};
size_t scan_wide_lds(uint32_t d4, uint32_t k, int waves);   // dynamic LDS of a wide-item block
bool scan_wide_fits(uint32_t d4, uint32_t k, int waves);
void launch_scan_narrow(int metric, int regs, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s);
// L2 / IP only (Cosine, whose CPU-path distance is always 0.0f, scans narrow items).
// waves 4: items of <= 16 queries, two workgroups per CU; 8: items of <= 32, one per CU.
void launch_scan_wide(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s, int waves = 4);
// wide items of >= a.mfma_min queries (L2 / IP): bounded on the matrix cores, exact re-rank
size_t scan_bounded_lds(uint32_t d4, uint32_t k);
bool scan_bounded_fits(uint32_t d4, uint32_t k);
void launch_scan_bounded(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s);
// ---- screened scan (screen.hip): L2 / IP, k <= 64, lists in HBM ----
bool scan_screen_fits(uint32_t k, uint32_t dp, uint32_t wq, bool deferred);
size_t screen_exact_lds(uint32_t d4);  // dynamic LDS of the LDS-staged exact re-check (screen_post.hip)
void launch_gather_cache_rows(const float4* cache, uint32_t d4, const ulonglong2* src, uint32_t n, float* rows,
                              hipStream_t s);
size_t screen_shadow_u4(uint64_t blocks, uint32_t d4, bool i8 = false);  // shadow size (uint4) incl. the prefetch slack
void launch_screen_build(const float4* arena, uint64_t blocks, uint32_t d4, const uint32_t* block_list,
                         const float* cent_rm, uint4* shadow, float* rows, float4* meta, hipStream_t s, float* sscale = nullptr);
// scnt / ovf / counters (the deferred scan; null for the inline one) are reset too.
void launch_screen_pairs(int metric, const float* q, uint32_t B, uint32_t P, const uint32_t* probes,
                         const float* cent_rm, uint32_t dp, uint16_t* qres, float4* pst, uint32_t* thr4, hipStream_t s,
                         uint32_t* scnt = nullptr, uint32_t* ovf = nullptr, uint32_t* counters = nullptr,
                         uint32_t* ubcnt = nullptr, float* qscale = nullptr);
void launch_scan_screen(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s);
// Deferred screened scan: collect (a.cand), then select (each pair's final threshold, the
// survivors of it grouped per pair in surv with offsets soff[0 .. nvalid] and their count in
// counters[kCtrSurv]), then the exact re-check of the survivors into each pair's only partial.
void launch_screen_collect(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s);
// slb (optional): the survivors' lower bounds beside surv (the two-pass re-check reads them)
void launch_screen_select(const ScanArgs& a, uint32_t BP, uint32_t* scnt, uint32_t* soff, uint2* surv,
                          const uint32_t* ovf, hipStream_t s, float* slb = nullptr);
// surv: (slot, sorted pair) per survivor; fetched: null = rows from a.rows by slot, else the
// survivors' rows [survivor][dp] (tier); sdist: their exact distances (max_surv entries).
void launch_screen_recheck(int metric, const ScanArgs& a, uint32_t BP, const uint32_t* probes, uint32_t* nseg_qp,
                           const uint32_t* soff, const uint32_t* scnt, const uint2* surv, const uint32_t* ovf,
                           const float* fetched, float* sdist, uint32_t max_surv, uint32_t smax, hipStream_t s,
                           const float* slb = nullptr);  // slb: the two-pass re-check (rows in HBM)
// The screened tier's two-pass re-check from the index file (screen_post.hip): phase 0 marks
// each pair's pass-A survivors (mark 1), phase 1 computes their exact distances from the compact
// fetched rows (rowmap: survivor -> row) and marks pass B (mark 2), phase 2 computes pass B and
// writes each pair's exact top-k as its only partial.
void launch_tier_recheck(int phase, int metric, const ScanArgs& a, uint32_t BP, uint32_t* nseg_qp, const uint32_t* soff,
                         const uint32_t* scnt, const uint2* surv, const float* slb, uint8_t* mark, const uint32_t* rowmap,
                         const float* fetched, float* sdist, hipStream_t s);
void launch_slot_merge(int regs, const uint32_t* probes, const uint32_t* count_global,
                       const uint32_t* nseg_qp, const uint32_t* part_base_qp, const uint32_t* l1base_qp,
                       const float* part_d, const uint64_t* part_i, const float* l1_d, const uint64_t* l1_i,
                       uint32_t BP, uint32_t k, float* slot_d, uint64_t* slot_i, hipStream_t s);
// req_start (device, per call-global query: its request's first query; null = one
// request) keeps the stale-slot semantics per coalesced request.
void launch_query_merge(int regs, const uint32_t* probes, const uint32_t* count_global, const float* slot_d,
                        const uint64_t* slot_i, const float* carry_d, const uint64_t* carry_i,
                        uint32_t B, uint32_t P, uint32_t k, int stale, const uint32_t* req_start, uint32_t b0,
                        float* out_d, uint64_t* out_i, hipStream_t s);
void launch_carry(const uint32_t* probes, const uint32_t* count_global, uint32_t B, uint32_t P, uint32_t k,
                  const float* slot_d, const uint64_t* slot_i, const uint32_t* req_start, uint32_t b0,
                  float* carry_d, uint64_t* carry_i, hipStream_t s);
// The four merges above in one launch (one workgroup per query): effective slots (own
// fold of every segment partial, stale source recomputed, or carry) into slot_d/i, the
// unique-id top-k into out, and the next batch's carry into carry_nd/ni (ping-pong).
void launch_merge_fused(int regs, const uint32_t* probes, const uint32_t* count_global, const uint32_t* nseg_qp,
                        const uint32_t* part_base_qp, const float* part_d, const uint64_t* part_i, uint32_t B,
                        uint32_t P, uint32_t k, int stale, const uint32_t* req_start, uint32_t b0, const float* carry_d,
                        const uint64_t* carry_i, float* slot_d, uint64_t* slot_i, float* carry_nd, uint64_t* carry_ni,
                        float* out_d, uint64_t* out_i, hipStream_t s);
void launch_rank_merge(int regs, const float* d, const uint64_t* i, uint64_t d_stride, uint64_t i_stride,
                       uint32_t nranks, uint32_t n, uint32_t k, float* out_d, uint64_t* out_i, hipStream_t s);
void launch_fill_empty(uint64_t n, float* d, uint64_t* i, hipStream_t s);

// ---- build (train / add / layout) ----
void launch_interleave(const float* rows, uint64_t n, uint32_t dp, float4* blocks, hipStream_t s);
void launch_scatter_rows(const float* rows, const uint64_t* row_ids, const uint32_t* order, uint64_t n,
                         uint32_t dp, const uint64_t* dest_slot, float4* arena, uint64_t* arena_ids,
                         hipStream_t s);
void launch_copy_lists(const float4* old_arena, const uint64_t* old_ids, const uint64_t* old_off,
                       const uint64_t* new_off, const uint32_t* nblocks, uint32_t nlist, uint32_t d4,
                       float4* new_arena, uint64_t* new_ids, hipStream_t s);
void launch_export_list(const float4* arena, const uint64_t* ids, uint64_t block_off, uint32_t count,
                        uint32_t dim, uint32_t d4, float* out, uint64_t* out_ids, hipStream_t s);
void launch_assign(int metric, const float* vpad, uint64_t n, uint32_t dp, const float4* cent_il,
                   uint32_t nlist, uint32_t* out, hipStream_t s);
void launch_histogram(const uint32_t* keys, uint64_t n, uint32_t* counts, hipStream_t s);
void launch_mindist_init(float* mind, uint64_t n, hipStream_t s);
void launch_mindist_update(const float4* v_il, uint64_t n, uint32_t d4, const float* centroid_row,
                           float* mind, hipStream_t s);
void launch_centroid_update(const float* vpad, uint32_t dp, const uint32_t* order, const uint32_t* offsets,
                            const uint32_t* counts, uint32_t nlist, uint32_t dim, float* cent_rm,
                            hipStream_t s);
void launch_iota(uint32_t* out, uint64_t n, hipStream_t s);
void launch_slots_from_order(const uint32_t* sorted_keys, uint64_t n, const uint64_t* group_start,
                             const uint64_t* list_base_slot, uint64_t* dest_slot, hipStream_t s);
void launch_gen_normal(float* out, uint64_t n, uint64_t seed, uint64_t offset, hipStream_t s);
void launch_gen_mixture(float* out, uint64_t rows, uint32_t dim, const float* centers, uint32_t ncomp, float sigma,
                        uint64_t seed, uint64_t row0, hipStream_t s);

// Stable key/value radix sort (hipCUB). temp == nullptr queries temp_bytes.
hipError_t radix_sort_pairs(void* temp, size_t& temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                            const uint32_t* vals_in, uint32_t* vals_out, uint64_t n, int end_bit,
                            hipStream_t s);

}  // namespace vdbk
