// screen_post.hip — the deferred screened scan after its collect kernel (screen.hip): each
// (query, list) pair's final threshold, the survivors of it grouped per pair, and their exact
// re-check with the reference's sequential fp32 sum (search_list_cpu, ivf_flat_index.cpp:
// 339-384) into the pair's only partial. Its own translation unit: these kernels change
// without recompiling the collect kernel's many instantiations.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <stdexcept>
#include <type_traits>

#include "kernels.hpp"
#include "scan_common.hpp"
#include "wave_topk.hpp"

namespace vdbk {

// One wave per valid sorted pair: the k-th smallest of the union of its contributed upper-
// bound lists (k vectors of the list have exact distances at or below it) lowers a.thr.
// (Latency-bound: the contributions are read four 64-element chunks at a time, all loads in
// flight together, and only values below the running k-th are inserted — a wave top-k keyed
// (value, element) — instead of sorting and merging every chunk.)
__global__ __launch_bounds__(256) void ivf_screen_tfinal(ScanArgs a) {
    chain_prio();
    const int lane = lane_id();
    const uint32_t nvalid = a.counters[kCtrValid];
    const int k = (int)a.k;
    for (uint32_t s = blockIdx.x * 4 + wave_index(); s < nvalid; s += gridDim.x * 4) {
        const uint32_t nl = min(a.ubcnt[s], (uint32_t)kUbLists);
        const uint32_t n = nl * (uint32_t)k;
        const float* src = a.ublist + (size_t)s * kUbLists * k;
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        for (uint32_t e0 = 0; e0 < n; e0 += 4 * 64) {
            float d[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t e = e0 + 64 * u + (uint32_t)lane;
                d[u] = e < n ? src[e] : __builtin_inff();
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t e = e0 + 64 * u + (uint32_t)lane;
                offer_lanes<1>(tk, e < n && key_less(d[u], e, kd, ki), d[u], (uint64_t)e, k, kd, ki);
            }
        }
        if (lane == 0 && kd < ord_dec(a.thr[s])) a.thr[s] = ord_enc(kd);
    }
}

// Per collected pair: keep it if its lower bound is not above its pair's final threshold;
// its rank among its pair's survivors into .w (~0: dropped). The collect kernel appends a
// ballot's candidates in lane order, so consecutive entries come in runs of one pair (up to
// 16): each wave takes 64 consecutive entries and does one atomic per run (segmented by equal
// pairs across its lanes) instead of one per survivor on the pair's counter. (Latency-bound:
// each wave takes kFilterU 64-entry chunks a grid pass apart at once, every load of one kind
// in flight together: the entries, then their thresholds, then the run atomics.)
constexpr int kFilterU = 4;
__global__ __launch_bounds__(256) void ivf_screen_filter(uint4* __restrict__ cand, const uint32_t* __restrict__ counters,
                                                         uint32_t cap, const uint32_t* __restrict__ thr,
                                                         const uint32_t* __restrict__ thr4,
                                                         const uint32_t* __restrict__ ovf, uint32_t* __restrict__ scnt) {
    chain_prio();
    const uint32_t n = min(counters[kCtrCand], cap);
    const int lane = lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u; i0 < n; i0 += kFilterU * stride) {
        uint4 c[kFilterU];
#pragma unroll
        for (int u = 0; u < kFilterU; ++u) {
            const uint32_t i = i0 + u * stride + (uint32_t)lane;
            c[u] = i < n ? cand[i] : make_uint4(~0u, 0u, 0u, ~0u);
        }
        uint4 t4[kFilterU];
        uint32_t tg[kFilterU], ov[kFilterU];
#pragma unroll
        for (int u = 0; u < kFilterU; ++u) {
            const bool act = c[u].x != ~0u;  // (sentinel: the padding of a collect wave's candidate chunk)
            const uint32_t sp = act ? c[u].x : 0u;
            t4[u] = act ? *(const uint4*)(thr4 + (size_t)sp * 4) : make_uint4(0u, 0u, 0u, 0u);
            tg[u] = act ? thr[sp] : 0u;
            ov[u] = act ? ovf[sp] : 1u;
        }
        uint32_t base[kFilterU];
        bool keep[kFilterU];
        uint64_t runm[kFilterU], keeps[kFilterU];
        int endl[kFilterU];
#pragma unroll
        for (int u = 0; u < kFilterU; ++u) {
            const bool act = c[u].x != ~0u;
            const uint32_t sp = c[u].x;
            const float T = fminf(ord_dec(tg[u]), fmaxf(fmaxf(ord_dec(t4[u].x), ord_dec(t4[u].y)),
                                                         fmaxf(ord_dec(t4[u].z), ord_dec(t4[u].w))));
            keep[u] = act && !ov[u] && !(__uint_as_float(c[u].z) > T);
            // runs of equal pairs: a run starts where the previous lane's pair differs
            const uint32_t prev = __shfl_up(sp, 1);
            const uint64_t heads = __ballot(lane == 0 || prev != sp);
            keeps[u] = __ballot(keep[u]);
            const int start = 63 - __builtin_clzll(heads & (below | (1ull << lane)));  // this lane's run start
            const uint64_t after = heads & ~(below | (1ull << lane));                   // later run starts
            endl[u] = after ? __builtin_ctzll(after) - 1 : 63;                           // this lane's run end
            runm[u] = (endl[u] == 63 ? ~0ull : ((1ull << (endl[u] + 1)) - 1ull)) & ~((1ull << start) - 1ull);
            base[u] = 0;
            if (lane == endl[u] && act && (keeps[u] & runm[u])) base[u] = atomicAdd(&scnt[sp], (uint32_t)__popcll(keeps[u] & runm[u]));
        }
#pragma unroll
        for (int u = 0; u < kFilterU; ++u) {
            const uint32_t bs = __shfl(base[u], endl[u]);
            const uint32_t i = i0 + u * stride + (uint32_t)lane;
            if (c[u].x != ~0u && i < n) cand[i].w = keep[u] ? bs + (uint32_t)__popcll(keeps[u] & runm[u] & below) : ~0u;
        }
    }
}

// Exclusive scan of the survivor counts of the batch's valid sorted pairs (one workgroup):
// soff[0 .. nvalid], the total into counters[kCtrSurv].
__global__ __launch_bounds__(1024) void ivf_screen_offsets(const uint32_t* __restrict__ scnt,
                                                           uint32_t* __restrict__ counters,
                                                           uint32_t* __restrict__ soff, uint4* __restrict__ floor_out,
                                                           uint32_t floor_seq, uint32_t cap, uint32_t k) {
    chain_prio();
    __shared__ uint32_t wsum[16];
    const uint32_t n = counters[kCtrValid];
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t c0 = min(n, threadIdx.x * per), c1 = min(n, c0 + per);
    uint32_t s = 0;
    for (uint32_t i = c0; i < c1; ++i) s += scnt[i];
    // inclusive scan of s over the workgroup
    uint32_t x = s;
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (uint32_t w = 0; w < (blockDim.x >> 6); ++w) {
        if (w < (threadIdx.x >> 6)) wbase += wsum[w];
        total += wsum[w];
    }
    uint32_t o = wbase + x - s;
    for (uint32_t i = c0; i < c1; ++i) {
        soff[i] = o;
        o += scnt[i];
    }
    if (threadIdx.x == 0) {
        soff[n] = total;
        counters[kCtrSurv] = total;
        // (the run-time floor's report into its ring entry of page-locked host memory:
        // {survivors or ~0 after an overflow, (query, vector) pairs, sequence, k x valid pairs}.
        // The counts first, then a system-scope release fence, then the sequence number: the
        // host reads the sequence before and after the counts and keeps only a match (floor.hpp))
        if (floor_out) {
            volatile uint32_t* f = (volatile uint32_t*)floor_out;
            f[0] = counters[kCtrOvf] ? ~0u : total;
            f[1] = counters[kCtrPairs];
            f[3] = (uint32_t)min(0xFFFFFFFFull, (unsigned long long)k * n);
            __threadfence_system();
            f[2] = floor_seq;
        }
    }
}

__global__ __launch_bounds__(256) void ivf_screen_scatter(const uint4* __restrict__ cand,
                                                          const uint32_t* __restrict__ counters, uint32_t cap,
                                                          const uint32_t* __restrict__ soff,
                                                          uint2* __restrict__ surv, float* __restrict__ slb) {
    chain_prio();
    const uint32_t n = min(counters[kCtrCand], cap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint4 c = cand[i];
        if (c.w != ~0u) {
            surv[soff[c.x] + c.w] = make_uint2(c.y, c.x);  // (slot, sorted pair)
            if (slb) slb[soff[c.x] + c.w] = __uint_as_float(c.z);  // (its lower bound: the two-pass re-check)
        }
    }
}

// The exact sequential distance of `slot` for query row qr: from the interleaved arena
// ([block][d4][64 lanes] float4; device or page-locked host memory) or a row-major row.
template <int M, bool ROWS>
__device__ __forceinline__ float exact_dist(const float4* __restrict__ src, uint64_t row_or_slot, uint32_t d4,
                                            const float4* __restrict__ qr) {
    constexpr int kP = 8;
    const float4* base;
    size_t stride;
    if (ROWS) {
        base = src + row_or_slot * d4;
        stride = 1;
    } else {
        base = src + (row_or_slot >> 6) * (uint64_t)d4 * 64 + (row_or_slot & 63);
        stride = 64;
    }
    float acc = 0.0f;
    float4 xb[kP], qb[kP];
#pragma unroll
    for (int i = 0; i < kP; ++i) {
        xb[i] = i < (int)d4 ? base[(size_t)i * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
        qb[i] = i < (int)d4 ? qr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (uint32_t t0 = 0; t0 < d4; t0 += kP) {
#pragma unroll
        for (int i = 0; i < kP; ++i) {
            if (t0 + i < d4) acc = acc4<M>(acc, qb[i], xb[i]);
            const uint32_t tn = t0 + kP + i;
            if (tn < d4) {
                xb[i] = base[(size_t)tn * stride];
                qb[i] = qr[tn];
            }
        }
    }
    return dist_finish<M>(acc);
}

// Exact distances of the survivors (one 64-thread workgroup per kExactRows of them, in
// their per-pair order): the rows are loaded into LDS together, kExactRows x 1 KiB
// contiguous wave-loads per 256 dims, all in flight at once, from the row-major fp32 copy
// of the lists (SRC 0, slot-indexed), from rows fetched from the tier's file home (SRC 1,
// [survivor][dp]), or from the interleaved arena in page-locked host memory (SRC 2, the
// tier's host home, read over PCIe);
// then one lane per row runs the reference's sequential sum over its LDS row (row stride
// d4 + 1 float4: the lanes' rows fall on distinct banks) against its pair's query.
#ifndef VDB_EXACT_LANE
#define VDB_EXACT_LANE 1
#endif
constexpr bool kExactLane = VDB_EXACT_LANE != 0;  // (A/B builds: 0 = the LDS-staged kernel for HBM rows too)
constexpr uint32_t kExactLaneMin = 16384;
constexpr int kExactRows = 16;
constexpr int kExactChunks = 3;  // 64-float4 chunks of a row loaded per pass (768 dims)
__host__ __device__ constexpr size_t exact_lds(uint32_t d4) { return ((size_t)kExactRows * (d4 + 1) + 64) * 16; }
size_t screen_exact_lds(uint32_t d4) { return exact_lds(d4); }

template <int M, int SRC>
__global__ __launch_bounds__(64) void ivf_screen_exact(ScanArgs a, const uint2* __restrict__ surv,
                                                       const float* __restrict__ fetched,
                                                       float* __restrict__ sdist) {
    extern __shared__ __attribute__((aligned(16))) float4 rlds[];
    const int lane = lane_id();
    const uint32_t total = a.counters[kCtrSurv];
    if (SRC != 2 && kExactLane && total >= kExactLaneMin) return;  // (ivf_screen_exact_lane's)
    const uint32_t d4 = a.d4, rs = d4 + 1;
    const float4* src = SRC == 1 ? (const float4*)fetched : SRC == 0 ? (const float4*)a.rows : a.arena;
    for (uint32_t base = blockIdx.x * kExactRows; base < total; base += gridDim.x * kExactRows) {
        const uint32_t ng = min((uint32_t)kExactRows, total - base);
        const uint2 my = lane < (int)ng ? surv[base + lane] : make_uint2(0u, 0u);
        // every load unconditional (clamped to valid rows and dims) so that all of them are in
        // flight together; writes of clamped elements go to the LDS dump row kExactRows
        for (uint32_t c0 = 0; c0 < d4; c0 += 64 * kExactChunks) {
            float4 v[kExactRows][kExactChunks];
#pragma unroll
            for (int r = 0; r < kExactRows; ++r) {
                const uint32_t rr = min((uint32_t)r, ng - 1);
                const uint64_t row = SRC == 1 ? (uint64_t)(base + rr) : (uint64_t)__builtin_amdgcn_readlane(my.x, (int)rr);
#pragma unroll
                for (int c = 0; c < kExactChunks; ++c) {
                    const uint32_t t = min(c0 + 64 * c + lane, d4 - 1);
                    v[r][c] = SRC == 2 ? src[((row >> 6) * d4 + t) * 64 + (row & 63)] : src[row * d4 + t];
                }
            }
#pragma unroll
            for (int r = 0; r < kExactRows; ++r)
#pragma unroll
                for (int c = 0; c < kExactChunks; ++c) {
                    const uint32_t t = c0 + 64 * c + lane;
                    rlds[(r < (int)ng && t < d4) ? r * rs + t : kExactRows * rs + lane] = v[r][c];
                }
        }
        __syncthreads();
        if (lane < (int)ng) {
            const uint32_t q = a.sorted_pair[my.y] >> 16;
            const float4* qr = (const float4*)(a.qpad + (size_t)q * a.dp);
            const float4* xr = rlds + (size_t)lane * rs;
            float acc = 0.0f;
#pragma unroll 8
            for (uint32_t t = 0; t < d4; ++t) acc = acc4<M>(acc, qr[t], xr[t]);
            sdist[base + lane] = dist_finish<M>(acc);
        }
        __syncthreads();  // (the next rows overwrite the LDS)
    }
}

// The same exact distances for rows in HBM (SRC 0: the row-major copy by slot; SRC 1: the
// tier's fetched rows [survivor][dp]) when a batch has many survivors (at least
// kExactLaneMin: the LDS-staged kernel, one round trip per 16 rows, is faster for a few
// thousand), 64 survivors per wave, one lane each (the reference's
// sequential sum needs one lane per (query, row) pair): every lane streams its own row and
// its query (a few distinct queries per wave: the survivors are grouped per pair, so those
// loads are mostly one address) kLaneRowPipe float4 ahead of its sum, without LDS. All 64
// lanes sum (the LDS-staged kernel above keeps 48 idle and holds 50 KB of LDS per 16 rows).
constexpr int kLaneRowPipe = 16;                  // (d4 is a multiple of 16 for the screen)
template <int M, int SRC>
__global__ __launch_bounds__(256) void ivf_screen_exact_lane(ScanArgs a, const uint2* __restrict__ surv,
                                                             const float* __restrict__ fetched,
                                                             float* __restrict__ sdist) {
    const int lane = lane_id();
    const uint32_t total = a.counters[kCtrSurv];
    if (total < kExactLaneMin) return;  // (ivf_screen_exact's)
    const uint32_t d4 = a.d4;
    const float4* src = SRC == 1 ? (const float4*)fetched : (const float4*)a.rows;
    for (uint32_t i0 = (blockIdx.x * 4 + wave_index()) * 64; i0 < total; i0 += gridDim.x * 256) {
        const uint32_t i = min(i0 + (uint32_t)lane, total - 1);
        const uint2 my = surv[i];
        const float4* xr = src + (SRC == 1 ? (uint64_t)i : (uint64_t)my.x) * d4;
        const float4* qr = (const float4*)(a.qpad + (size_t)(a.sorted_pair[my.y] >> 16) * a.dp);
        float4 xb[kLaneRowPipe], qb[kLaneRowPipe];
#pragma unroll
        for (int p = 0; p < kLaneRowPipe; ++p) {
            xb[p] = xr[p];
            qb[p] = qr[p];
        }
        float acc = 0.0f;
        for (uint32_t t0 = 0; t0 < d4; t0 += kLaneRowPipe) {
            const bool more = t0 + kLaneRowPipe < d4;  // (wave-uniform)
#pragma unroll
            for (int p = 0; p < kLaneRowPipe; ++p) {
                acc = acc4<M>(acc, qb[p], xb[p]);
                if (more) {
                    xb[p] = xr[t0 + kLaneRowPipe + p];
                    qb[p] = qr[t0 + kLaneRowPipe + p];
                }
            }
        }
        if (i0 + (uint32_t)lane < total) sdist[i0 + lane] = dist_finish<M>(acc);
    }
}

// One wave per valid sorted (query, list) pair: the exact top-k of its survivors' distances,
// written as the pair's only partial. A pair that overflowed the candidate buffer keeps its
// planned segments instead: one wave per (pair, segment) recomputes the segment lane =
// vector from the row-major copy and writes the segment's partial (neighbouring waves take
// the same segment of one list for neighbouring queries: its rows are shared in L2), so a
// batch in the cancellation regime costs a parallel dense pass, not one wave per pair.
template <int M>
__global__ __launch_bounds__(256) void ivf_screen_pair_topk(ScanArgs a, const uint32_t* __restrict__ probes,
                                                            uint32_t* __restrict__ nseg_qp,
                                                            const uint32_t* __restrict__ soff,
                                                            const uint32_t* __restrict__ scnt,
                                                            const uint2* __restrict__ surv,
                                                            const float* __restrict__ sdist,
                                                            const uint32_t* __restrict__ ovf, uint32_t smax) {
    const int lane = lane_id();
    const uint32_t nvalid = a.counters[kCtrValid];
    const int k = (int)a.k;
    const uint32_t wv = blockIdx.x * 4 + wave_index(), nw = gridDim.x * 4;
    unsigned long long rechecked = 0;
    for (uint32_t s = wv; s < nvalid; s += nw) {
        if (ovf[s]) continue;
        const uint32_t pr = a.sorted_pair[s];
        const uint32_t q = pr >> 16, p = pr & 0xFFFFu;
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        const uint32_t n = scnt[s], o = soff[s];
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool act = i < n;
            const float dist = act ? sdist[o + i] : __builtin_inff();
            const uint64_t id = act ? a.ids[surv[o + i].x] : kNoId;
            offer_lanes<1>(tk, act && key_less(dist, id, kd, ki), dist, id, k, kd, ki);
        }
        rechecked += n;
        // the pair's exact top-k is its only partial: the merge reads the first of its segments
        const uint32_t part = a.part_base_sorted[s];
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk.d[0];
            a.part_i[(size_t)part * k + lane] = tk.id[0];
        }
        if (lane == 0) nseg_qp[(size_t)q * a.P + p] = 1u;
    }
    // (no pair overflowed unless the batch collected more candidates than the buffer holds)
    const uint64_t tasks = a.counters[kCtrOvf] ? (uint64_t)nvalid * smax : 0;
    const uint32_t segv = a.seg_blocks * 64;
    for (uint64_t t = wv; t < tasks; t += nw) {
        const uint32_t s = (uint32_t)(t % nvalid), j = (uint32_t)(t / nvalid);
        if (!ovf[s]) continue;
        const uint32_t pr = a.sorted_pair[s];
        const uint32_t q = pr >> 16, p = pr & 0xFFFFu;
        if (j >= nseg_qp[(size_t)q * a.P + p]) continue;  // (the planned segments: untouched above)
        const uint32_t list = probes[(size_t)q * a.P + p];
        const uint32_t n = min(a.count[list], (j + 1) * segv);
        const uint64_t lbase = a.block_off[list] * 64;
        const float4* qr = (const float4*)(a.qpad + (size_t)q * a.dp);
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        for (uint32_t i0 = j * segv; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool act = i < n;
            float dist = __builtin_inff();
            uint64_t id = kNoId;
            if (act) {  // (the row-major copy, or the tier's host arena; a file home never overflows)
                dist = a.rows ? exact_dist<M, true>((const float4*)a.rows, lbase + i, a.d4, qr)
                              : exact_dist<M, false>(a.arena, lbase + i, a.d4, qr);
                id = a.ids[lbase + i];
            }
            offer_lanes<1>(tk, act && key_less(dist, id, kd, ki), dist, id, k, kd, ki);
        }
        rechecked += n > j * segv ? n - j * segv : 0;
        const uint32_t part = a.part_base_sorted[s] + j;
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk.d[0];
            a.part_i[(size_t)part * k + lane] = tk.id[0];
        }
    }
    if (a.mstats && lane == 0 && rechecked) atomicAdd(&a.mstats[2], rechecked);
}

// The reference's sequential sum of one row-major row against the query row, kLaneRowPipe
// float4 of both in flight per lane (ivf_screen_exact_lane's loop).
template <int M>
__device__ __forceinline__ float lane_row_dist(const float4* __restrict__ xr, const float4* __restrict__ qr,
                                               uint32_t d4) {
    float4 xb[kLaneRowPipe], qb[kLaneRowPipe];
#pragma unroll
    for (int p = 0; p < kLaneRowPipe; ++p) {
        xb[p] = xr[p];
        qb[p] = qr[p];
    }
    float acc = 0.0f;
    for (uint32_t t0 = 0; t0 < d4; t0 += kLaneRowPipe) {
        const bool more = t0 + kLaneRowPipe < d4;  // (wave-uniform)
#pragma unroll
        for (int p = 0; p < kLaneRowPipe; ++p) {
            acc = acc4<M>(acc, qb[p], xb[p]);
            if (more) {
                xb[p] = xr[t0 + kLaneRowPipe + p];
                qb[p] = qr[t0 + kLaneRowPipe + p];
            }
        }
    }
    return dist_finish<M>(acc);
}

// TWO-PASS exact re-check (default for rows in HBM; option screen_recheck2), in place of
// ivf_screen_exact_lane + ivf_screen_pair_topk. One wave per valid sorted (query, list) pair
// with n survivors of its final upper-bound threshold T (ivf_screen_filter):
//  * n <= k: all of them, one round (one lane per survivor: the reference's sequential sum);
//  * else pass A: the k survivors with the smallest lower bounds (key (lb, index), a wave
//    top-k), one round; their k-th exact distance kd is a valid threshold (k vectors of the
//    list are at or below it) and, on iid 768-D data, far below T (the k-th smallest UPPER
//    bound: about one bound width, delta, above the k-th distance, so T admits a window of 2
//    delta above it and kd one of delta);
//  * pass B: every other survivor whose lower bound is not above the current kd (NaN bounds
//    always), compacted 64 at a time through the wave's LDS ring; kd tightens with every
//    round and each entry is tested again when its round starts.
// A skipped survivor has lb > kd, i.e. an exact distance strictly above k distances of its
// list: it cannot be in the list's multiset top-k (the exact scan's pruning rule), so the
// pair's exact top-k — written as its only partial, as ivf_screen_pair_topk does — is the
// same. Re-checks at the headline: ~37 per pair instead of ~110 (a CPU model of the int8
// bound; the bench reports the measured count). Overflowed pairs: ivf_screen_pair_topk's
// recomputation over their planned segments, unchanged.
// The same sum with the query row read from LDS (one pair per wave: every lane has the same
// query) and KP float4 of the lane's row in flight: twice the loads in flight per lane of
// lane_row_dist for the same registers, so a round of re-checks costs half the round trips.
template <int M, int KP>
__device__ __forceinline__ float lane_row_dist_lq(const float4* __restrict__ xr, const float4* ql, uint32_t d4) {
    float4 xb[KP];
#pragma unroll
    for (int p = 0; p < KP; ++p) xb[p] = xr[p];
    float acc = 0.0f;
    for (uint32_t t0 = 0; t0 < d4; t0 += KP) {
        const bool more = t0 + KP < d4;  // (wave-uniform)
#pragma unroll
        for (int p = 0; p < KP; ++p) {
            acc = acc4<M>(acc, ql[t0 + p], xb[p]);
            if (more) xb[p] = xr[t0 + KP + p];
        }
    }
    return dist_finish<M>(acc);
}

constexpr uint32_t kR2Ring = 128;
constexpr uint32_t kR2MaxD4 = 512;  // (query rows staged in LDS up to 2048 dims: 32 KB; wider: from global memory)
template <int M, int KP>
__global__ __launch_bounds__(256) void ivf_screen_recheck2(ScanArgs a, const uint32_t* __restrict__ probes,
                                                           uint32_t* __restrict__ nseg_qp,
                                                           const uint32_t* __restrict__ soff,
                                                           const uint32_t* __restrict__ scnt,
                                                           const uint2* __restrict__ surv,
                                                           const float* __restrict__ slb,
                                                           const uint32_t* __restrict__ ovf, uint32_t smax) {
    chain_prio();
    __shared__ uint32_t s_ring[4][kR2Ring];
    extern __shared__ __attribute__((aligned(16))) float4 s_qrow[];  // (KP > 0: per wave its pair's query row)
    const int lane = lane_id();
    const uint32_t wl = wave_index();
    uint32_t* ring = s_ring[wl];
    float4* ql = s_qrow + (size_t)wl * a.d4;
    const uint32_t nvalid = a.counters[kCtrValid];
    const int k = (int)a.k;
    const uint32_t d4 = a.d4;
    const float4* rows = (const float4*)a.rows;
    const uint32_t wv = blockIdx.x * 4 + wl, nw = gridDim.x * 4;
    unsigned long long rechecked = 0;
    for (uint32_t s = wv; s < nvalid; s += nw) {
        if (ovf[s]) continue;
        const uint32_t pr = a.sorted_pair[s];
        const uint32_t q = pr >> 16, p = pr & 0xFFFFu;
        const uint32_t n = scnt[s], o = soff[s];
        const float4* qr = (const float4*)(a.qpad + (size_t)q * a.dp);
        if constexpr (KP > 0) {  // (the previous pair's reads of the row are done: in order within the wave)
            for (uint32_t t = (uint32_t)lane; t < d4; t += 64) ql[t] = qr[t];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        // Every round of re-checks goes through the wave's LDS ring and ONE call site (the
        // row-stream registers are allocated once): pass A's entries (all n when n <= k) are
        // queued first; then the scan of the others (pass B) queues those not above the
        // current k-th, and a round runs whenever 64 are queued or the scan is done. Each
        // entry is tested again against the k-th when its round starts (pass A's: kd is +inf).
        uint32_t head = 0, tail = 0;  // (wave-uniform ring cursors)
        float sk = __builtin_inff();
        uint64_t si = kNoId;
        uint32_t scan = n;  // (pass B's next survivor; n: no pass B)
        if (n <= (uint32_t)k) {
            if ((uint32_t)lane < n) ring[lane] = (uint32_t)lane;
            tail = n;
        } else {
            // pass A: the k smallest keys (lb, index); NaN bounds first
            WaveTopK<1> sel;
            sel.init();
            for (uint32_t i0 = 0; i0 < n; i0 += 64) {
                const uint32_t i = i0 + (uint32_t)lane;
                const bool act = i < n;
                const float lb = act ? slb[o + i] : __builtin_inff();
                const float lk = lb == lb ? lb : -__builtin_inff();
                offer_lanes<1>(sel, act && key_less(lk, i, sk, si), lk, (uint64_t)i, k, sk, si);
            }
            if (lane < k) ring[lane] = (uint32_t)sel.id[0];
            tail = (uint32_t)k;
            scan = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        for (;;) {
            if (scan < n && tail - head < 64 && head != 0) {  // (pass B scans after pass A's round)
                const uint32_t i = scan + (uint32_t)lane;
                const bool act = i < n;
                const float lb = act ? slb[o + i] : __builtin_inff();
                const float lk = lb == lb ? lb : -__builtin_inff();
                const bool in_a = !key_less(sk, si, lk, (uint64_t)i);  // (lk, i) <= the k-th key of pass A
                const bool want = act && !in_a && !(lb > kd);
                const uint64_t m = __ballot(want);
                if (want)
                    ring[(tail + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))) &
                         (kR2Ring - 1)] = i;
                tail += (uint32_t)__popcll(m);
                scan += 64;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                continue;
            }
            if (tail == head) break;
            // one round: up to 64 queued survivors, one lane each (inactive lanes read the first
            // active lane's row: no extra traffic, every load unconditional)
            const uint32_t cnt = min(64u, tail - head);
            const bool in = (uint32_t)lane < cnt;
            const uint32_t idx = ring[(head + (in ? (uint32_t)lane : 0u)) & (kR2Ring - 1)];
            head += cnt;
            const bool act = in && !(slb[o + idx] > kd);
            const uint64_t m = __ballot(act);
            if (!m) continue;
            const int first = __ffsll((long long)m) - 1;
            const uint32_t ie = act ? idx : (uint32_t)__builtin_amdgcn_readlane((int)idx, first);
            const uint64_t slot = surv[o + ie].x;
            float dist;
            if constexpr (KP > 0) dist = lane_row_dist_lq<M, KP>(rows + slot * d4, ql, d4);
            else dist = lane_row_dist<M>(rows + slot * d4, qr, d4);
            const uint64_t id = a.ids[slot];
            offer_lanes<1>(tk, act && key_less(dist, id, kd, ki), dist, id, k, kd, ki);
            rechecked += (unsigned long long)__popcll(m);
        }
        // the pair's exact top-k is its only partial: the merge reads the first of its segments
        const uint32_t part = a.part_base_sorted[s];
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk.d[0];
            a.part_i[(size_t)part * k + lane] = tk.id[0];
        }
        if (lane == 0) nseg_qp[(size_t)q * a.P + p] = 1u;
    }
    // overflowed pairs: as ivf_screen_pair_topk (its planned segments recomputed)
    const uint64_t tasks = a.counters[kCtrOvf] ? (uint64_t)nvalid * smax : 0;
    const uint32_t segv = a.seg_blocks * 64;
    for (uint64_t t = wv; t < tasks; t += nw) {
        const uint32_t s = (uint32_t)(t % nvalid), j = (uint32_t)(t / nvalid);
        if (!ovf[s]) continue;
        const uint32_t pr = a.sorted_pair[s];
        const uint32_t q = pr >> 16, p = pr & 0xFFFFu;
        if (j >= nseg_qp[(size_t)q * a.P + p]) continue;
        const uint32_t list = probes[(size_t)q * a.P + p];
        const uint32_t n = min(a.count[list], (j + 1) * segv);
        const uint64_t lbase = a.block_off[list] * 64;
        const float4* qr = (const float4*)(a.qpad + (size_t)q * a.dp);
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        for (uint32_t i0 = j * segv; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool act = i < n;
            float dist = __builtin_inff();
            uint64_t id = kNoId;
            if (act) {
                dist = exact_dist<M, true>(rows, lbase + i, d4, qr);
                id = a.ids[lbase + i];
            }
            offer_lanes<1>(tk, act && key_less(dist, id, kd, ki), dist, id, k, kd, ki);
        }
        rechecked += n > j * segv ? n - j * segv : 0;
        const uint32_t part = a.part_base_sorted[s] + j;
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk.d[0];
            a.part_i[(size_t)part * k + lane] = tk.id[0];
        }
    }
    if (a.mstats && lane == 0 && rechecked) atomicAdd(&a.mstats[2], rechecked);
}

// Screened tier: survivor rows whose list is in the HBM cache ({row index, cache slot}: one wave
// each) copied from the cache's block layout into the batch's row-major rows [n][dp].
__global__ __launch_bounds__(256) void ivf_gather_cache_rows(const float4* __restrict__ cache, uint32_t d4,
                                                             const ulonglong2* __restrict__ src, uint32_t n,
                                                             float4* __restrict__ rows) {
    const int lane = lane_id();
    for (uint32_t i = blockIdx.x * 4 + wave_index(); i < n; i += gridDim.x * 4) {
        const ulonglong2 e = src[i];
        const uint64_t blk = e.y >> 6, vl = e.y & 63;
        for (uint32_t t = lane; t < d4; t += 64) rows[e.x * d4 + t] = cache[(blk * d4 + t) * 64 + vl];
    }
}

void launch_gather_cache_rows(const float4* cache, uint32_t d4, const ulonglong2* src, uint32_t n, float* rows,
                              hipStream_t s) {
    if (!n) return;
    const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(4096, (n + 3) / 4));
    ivf_gather_cache_rows<<<g, 256, 0, s>>>(cache, d4, src, n, (float4*)rows);
}

void launch_screen_select(const ScanArgs& a, uint32_t BP, uint32_t* scnt, uint32_t* soff, uint2* surv,
                          const uint32_t* ovf, hipStream_t s, float* slb) {
    if (!BP) return;
    uint32_t* ctr = const_cast<uint32_t*>(a.counters);
    ivf_screen_tfinal<<<std::max<uint32_t>(1, std::min<uint32_t>(2048, (BP + 3) / 4)), 256, 0, s>>>(a);
    const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(1024, (a.cand_cap + 255) / 256));
    ivf_screen_filter<<<g, 256, 0, s>>>(a.cand, a.counters, a.cand_cap, a.thr, a.thr4, ovf, scnt);
    ivf_screen_offsets<<<1, 1024, 0, s>>>(scnt, ctr, soff, a.floor_out, a.floor_seq, a.cand_cap, a.k);
    ivf_screen_scatter<<<g, 256, 0, s>>>(a.cand, a.counters, a.cand_cap, soff, surv, slb);
}

void launch_screen_recheck(int metric, const ScanArgs& a, uint32_t BP, const uint32_t* probes, uint32_t* nseg_qp,
                           const uint32_t* soff, const uint32_t* scnt, const uint2* surv, const uint32_t* ovf,
                           const float* fetched, float* sdist, uint32_t max_surv, uint32_t smax, hipStream_t s,
                           const float* slb) {
    if (!BP) return;
    if (slb && !fetched && a.rows) {  // the two-pass re-check (rows in HBM)
        const uint32_t gp = std::max<uint32_t>(512, std::min<uint32_t>(2048, (BP + 3) / 4));
        // (the pair's query row in LDS, 16 float4 of each lane's row in flight: 220 VGPRs, two
        // waves per SIMD; 32 in flight spilled)
        const int kp = a.d4 <= kR2MaxD4 ? 16 : 0;
        const size_t lds = kp ? (size_t)4 * a.d4 * sizeof(float4) : 0;
        auto go = [&](auto m_c, auto kp_c) {
            constexpr int Mm = decltype(m_c)::value, KPc = decltype(kp_c)::value;
            ivf_screen_recheck2<Mm, KPc><<<gp, 256, lds, s>>>(a, probes, nseg_qp, soff, scnt, surv, slb, ovf, smax);
        };
        auto go_m = [&](auto m_c) {
            if (kp == 16) go(m_c, std::integral_constant<int, 16>{});
            else go(m_c, std::integral_constant<int, 0>{});
        };
        if (metric == kL2) go_m(std::integral_constant<int, kL2>{});
        else go_m(std::integral_constant<int, kIP>{});
        return;
    }
    static const bool raised = [] {
        for (const void* fn : {(const void*)ivf_screen_exact<kL2, 0>, (const void*)ivf_screen_exact<kIP, 0>,
                               (const void*)ivf_screen_exact<kL2, 1>, (const void*)ivf_screen_exact<kIP, 1>,
                               (const void*)ivf_screen_exact<kL2, 2>, (const void*)ivf_screen_exact<kIP, 2>})
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytes / 2));
        (void)hipGetLastError();
        return true;
    }();
    (void)raised;
    // (a grid-stride loop: 2048 workgroups of one wave cover 32K survivors per pass; a grid
    // sized to the buffer's capacity launched 16384, nearly all of which found nothing to do)
    const uint32_t ge = std::max<uint32_t>(1, std::min<uint32_t>(2048, (max_surv + kExactRows - 1) / kExactRows));
    const size_t lds = exact_lds(a.d4);
    // (a wave per pair, and at least 2048 waves for the (pair, segment) tasks of overflowed pairs)
    const uint32_t gp = std::max<uint32_t>(512, std::min<uint32_t>(2048, (BP + 3) / 4));
    const int src = fetched ? 1 : (a.rows ? 0 : 2);
    // (rows in HBM: 64 survivors per wave, 4 waves per workgroup; the host arena over PCIe:
    // 16 rows per workgroup)
    const uint32_t gl = std::max<uint32_t>(1, std::min<uint32_t>(2048, (max_surv + 255) / 256));
    auto exact = [&](auto m_c) {
        constexpr int Mm = decltype(m_c)::value;
        // (both kernels for rows in HBM: each serves the batch whose survivor count is its
        // regime and returns at once otherwise; the count is known only on the device)
        if (src == 0 && kExactLane && max_surv >= kExactLaneMin)
            ivf_screen_exact_lane<Mm, 0><<<gl, 256, 0, s>>>(a, surv, fetched, sdist);
        else if (src == 1 && kExactLane && max_surv >= kExactLaneMin)
            ivf_screen_exact_lane<Mm, 1><<<gl, 256, 0, s>>>(a, surv, fetched, sdist);
        if (src == 0) ivf_screen_exact<Mm, 0><<<ge, 64, lds, s>>>(a, surv, fetched, sdist);
        else if (src == 1) ivf_screen_exact<Mm, 1><<<ge, 64, lds, s>>>(a, surv, fetched, sdist);
        else ivf_screen_exact<Mm, 2><<<ge, 64, lds, s>>>(a, surv, fetched, sdist);
        ivf_screen_pair_topk<Mm><<<gp, 256, 0, s>>>(a, probes, nseg_qp, soff, scnt, surv, sdist, ovf, smax);
    };
    if (metric == kL2) exact(std::integral_constant<int, kL2>{});
    else exact(std::integral_constant<int, kIP>{});
}

// ============================================================================
// The screened tier's two-pass re-check (file home): the survivors' rows are read from the
// index file by the host, so the two passes of ivf_screen_recheck2 become two read phases —
// only the rows each pass needs are read. Rows arrive compact ([j][dp], j =
// rowmap[survivor]); mark[survivor]: 1 pass A, 2 pass B, 0 not needed.
//  1. ivf_tier_pass_a: per pair its k survivors of smallest lower bound (all of them when
//     n <= k) marked 1;
//  2. (host: read the marked rows) ivf_tier_pass_b: their exact distances into sdist, the
//     pair's k-th of them kd, and every other survivor whose lower bound is not above kd
//     (NaN always) marked 2 — strictly worse ones cannot be in the list's top-k;
//  3. (host: read those rows) ivf_tier_finish: their exact distances, then the pair's exact
//     top-k over both marks, written as its only partial.
// ============================================================================
__device__ __forceinline__ void select_k_smallest_lb(const float* __restrict__ lbp, uint32_t n, int k, float& sk,
                                                     uint64_t& si) {
    WaveTopK<1> sel;
    sel.init();
    sk = __builtin_inff();
    si = kNoId;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane_id();
        const bool act = i < n;
        const float lb = act ? lbp[i] : __builtin_inff();
        const float lk = lb == lb ? lb : -__builtin_inff();
        offer_lanes<1>(sel, act && key_less(lk, i, sk, si), lk, (uint64_t)i, k, sk, si);
    }
}

__global__ __launch_bounds__(256) void ivf_tier_pass_a(ScanArgs a, const uint32_t* __restrict__ soff,
                                                       const uint32_t* __restrict__ scnt, const float* __restrict__ slb,
                                                       uint8_t* __restrict__ mark) {
    const int lane = lane_id();
    const uint32_t nvalid = a.counters[kCtrValid];
    const int k = (int)a.k;
    for (uint32_t s = blockIdx.x * 4 + wave_index(); s < nvalid; s += gridDim.x * 4) {
        const uint32_t n = scnt[s], o = soff[s];
        if (n <= (uint32_t)k) {
            if ((uint32_t)lane < n) mark[o + lane] = 1;
            continue;
        }
        float sk;
        uint64_t si;
        select_k_smallest_lb(slb + o, n, k, sk, si);
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + (uint32_t)lane;
            if (i >= n) continue;
            const float lb = slb[o + i];
            const float lk = lb == lb ? lb : -__builtin_inff();
            mark[o + i] = key_less(sk, si, lk, (uint64_t)i) ? 0 : 1;  // (lk, i) <= the k-th key: pass A
        }
    }
}

// exact distances of the pair's survivors marked `want`, from the compact fetched rows
template <int M>
__device__ __forceinline__ void tier_exact_marked(const ScanArgs& a, uint32_t o, uint32_t n, uint8_t want,
                                                  const uint8_t* __restrict__ mark, const uint32_t* __restrict__ rowmap,
                                                  const float4* __restrict__ rows, const float4* __restrict__ qr,
                                                  float* __restrict__ sdist) {
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane_id();
        const bool act = i < n && mark[o + i] == want;
        const uint64_t m = __ballot(act);
        if (!m) continue;
        const int first = __ffsll((long long)m) - 1;
        const uint32_t ie = act ? i : (uint32_t)__builtin_amdgcn_readlane((int)i, first);
        const float dist = lane_row_dist<M>(rows + (uint64_t)rowmap[o + ie] * a.d4, qr, a.d4);
        if (act) sdist[o + i] = dist;
    }
}

template <int M>
__global__ __launch_bounds__(256) void ivf_tier_pass_b(ScanArgs a, const uint32_t* __restrict__ soff,
                                                       const uint32_t* __restrict__ scnt, const uint2* __restrict__ surv,
                                                       const float* __restrict__ slb, uint8_t* __restrict__ mark,
                                                       const uint32_t* __restrict__ rowmap, const float* __restrict__ fetched,
                                                       float* __restrict__ sdist) {
    const int lane = lane_id();
    const uint32_t nvalid = a.counters[kCtrValid];
    const int k = (int)a.k;
    for (uint32_t s = blockIdx.x * 4 + wave_index(); s < nvalid; s += gridDim.x * 4) {
        const uint32_t n = scnt[s], o = soff[s];
        const float4* qr = (const float4*)(a.qpad + (size_t)(a.sorted_pair[s] >> 16) * a.dp);
        tier_exact_marked<M>(a, o, n, 1, mark, rowmap, (const float4*)fetched, qr, sdist);
        if (n <= (uint32_t)k) continue;  // (every survivor was in pass A)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + (uint32_t)lane;
            const bool act = i < n && mark[o + i] == 1;
            const float d = act ? sdist[o + i] : __builtin_inff();
            const uint64_t id = act ? a.ids[surv[o + i].x] : kNoId;
            offer_lanes<1>(tk, act && key_less(d, id, kd, ki), d, id, k, kd, ki);
        }
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + (uint32_t)lane;
            if (i < n && mark[o + i] == 0 && !(slb[o + i] > kd)) mark[o + i] = 2;
        }
    }
}

template <int M>
__global__ __launch_bounds__(256) void ivf_tier_finish(ScanArgs a, uint32_t* __restrict__ nseg_qp,
                                                       const uint32_t* __restrict__ soff, const uint32_t* __restrict__ scnt,
                                                       const uint2* __restrict__ surv, const uint8_t* __restrict__ mark,
                                                       const uint32_t* __restrict__ rowmap, const float* __restrict__ fetched,
                                                       float* __restrict__ sdist) {
    const int lane = lane_id();
    const uint32_t nvalid = a.counters[kCtrValid];
    const int k = (int)a.k;
    unsigned long long rechecked = 0;
    for (uint32_t s = blockIdx.x * 4 + wave_index(); s < nvalid; s += gridDim.x * 4) {
        const uint32_t pr = a.sorted_pair[s];
        const uint32_t q = pr >> 16, p = pr & 0xFFFFu;
        const uint32_t n = scnt[s], o = soff[s];
        const float4* qr = (const float4*)(a.qpad + (size_t)q * a.dp);
        if (n > (uint32_t)k) tier_exact_marked<M>(a, o, n, 2, mark, rowmap, (const float4*)fetched, qr, sdist);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        WaveTopK<1> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + (uint32_t)lane;
            const bool act = i < n && mark[o + i] != 0;
            const float d = act ? sdist[o + i] : __builtin_inff();
            const uint64_t id = act ? a.ids[surv[o + i].x] : kNoId;
            offer_lanes<1>(tk, act && key_less(d, id, kd, ki), d, id, k, kd, ki);
            rechecked += (unsigned long long)__popcll(__ballot(act));
        }
        const uint32_t part = a.part_base_sorted[s];
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk.d[0];
            a.part_i[(size_t)part * k + lane] = tk.id[0];
        }
        if (lane == 0) nseg_qp[(size_t)q * a.P + p] = 1u;
    }
    if (a.mstats && lane == 0 && rechecked) atomicAdd(&a.mstats[2], rechecked);
}

void launch_tier_recheck(int phase, int metric, const ScanArgs& a, uint32_t BP, uint32_t* nseg_qp, const uint32_t* soff,
                         const uint32_t* scnt, const uint2* surv, const float* slb, uint8_t* mark, const uint32_t* rowmap,
                         const float* fetched, float* sdist, hipStream_t s) {
    if (!BP) return;
    const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(2048, (BP + 3) / 4));
    if (phase == 0) {
        ivf_tier_pass_a<<<g, 256, 0, s>>>(a, soff, scnt, slb, mark);
    } else if (phase == 1) {
        if (metric == kL2) ivf_tier_pass_b<kL2><<<g, 256, 0, s>>>(a, soff, scnt, surv, slb, mark, rowmap, fetched, sdist);
        else ivf_tier_pass_b<kIP><<<g, 256, 0, s>>>(a, soff, scnt, surv, slb, mark, rowmap, fetched, sdist);
    } else {
        if (metric == kL2) ivf_tier_finish<kL2><<<g, 256, 0, s>>>(a, nseg_qp, soff, scnt, surv, mark, rowmap, fetched, sdist);
        else ivf_tier_finish<kIP><<<g, 256, 0, s>>>(a, nseg_qp, soff, scnt, surv, mark, rowmap, fetched, sdist);
    }
}

}  // namespace vdbk
