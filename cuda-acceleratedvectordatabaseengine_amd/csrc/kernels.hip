// kernels.hip — hand-written gfx950 kernels of the IVF-Flat search path.
//
// Exactness: every distance is the reference's sequential fp32 sum
// (ivf_flat_index.cpp:308-318, 352-362): diff = a - b rounded, diff*diff rounded,
// acc + term rounded, d = 0..D-1. This file is compiled with -ffp-contract=off and
// the pragma below, so no multiply-add is ever fused; v_sub/v_mul/v_add_f32 are
// IEEE round-to-nearest with denormals kept (the default gfx950 float mode), the
// same results the x86 SSE path produces.
#pragma clang fp contract(off)

#include <stdexcept>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>

#include <algorithm>
#include <type_traits>

#include "kernels.hpp"
#include "scan_common.hpp"
#include "wave_topk.hpp"


namespace vdbk {

// Grid-stride helpers. An HSA dispatch packet holds the grid size in work-items as
// 32 bits, so every element-wise launch caps its grid (launch_grid) and strides.
__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return (uint64_t)gridDim.x * blockDim.x; }

// ============================================================================
// Query padding: [n][dim] -> [n][dp] with +0.0f pads.
// ============================================================================
__global__ void ivf_pad_queries(const float* __restrict__ src, uint64_t n, uint32_t dim, uint32_t dp,
                           float* __restrict__ dst) {
    for (uint64_t e = gtid(); e < n * dp; e += gstride()) {
        const uint64_t r = e / dp;
        const uint32_t c = (uint32_t)(e - r * dp);
        dst[e] = c < dim ? src[r * dim + c] : 0.0f;
    }
}

// ============================================================================
// Coarse quantiser, distance part (select_nprobe_lists, cpp:302-321).
// One lane = one centroid of an interleaved 64-centroid block; each wave takes
// 4 queries whose dims are wave-uniform (scalar loads). Exact sequential sums.
// ============================================================================
template <int M>
__global__ __launch_bounds__(256) void ivf_coarse_distances(const float4* __restrict__ cent, uint32_t nlist, uint32_t d4,
                                                const float* __restrict__ qpad, uint32_t B,
                                                float* __restrict__ cd) {
    constexpr int G = 4;
    const int lane = lane_id();
    const uint32_t cb = blockIdx.x;
    const uint32_t q0 = (blockIdx.y * 4 + wave_index()) * G;
    if (q0 >= B) return;
    const uint32_t dp = d4 * 4;
    const float4* q[G];
#pragma unroll
    for (int g = 0; g < G; ++g) q[g] = (const float4*)(qpad + (size_t)min(q0 + g, B - 1) * dp);
    const float4* vb = cent + (size_t)cb * d4 * 64 + lane;
    float acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = 0.0f;
#pragma unroll 4
    for (uint32_t t = 0; t < d4; ++t) {
        const float4 x = vb[(size_t)t * 64];
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = acc4<M>(acc[g], q[g][t], x);
    }
    const uint32_t c = cb * 64 + lane;
    if (c < nlist) {
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (q0 + g < B) cd[(size_t)(q0 + g) * nlist + c] = dist_finish<M>(acc[g]);
    }
}

// NaN distances order after every number (the reference's comparisons leave them
// unordered); keeps every selected list id valid.
__device__ __forceinline__ float nan_last(float d) { return d == d ? d : __builtin_inff(); }

// Order-preserving float <-> uint32 map (a < b as floats <=> enc(a) < enc(b) as
// unsigned), so shared thresholds can be lowered with integer atomic minimum.


// ============================================================================
// Coarse quantiser, selection part: the first min(nprobe, nlist) lists by
// (dist, list_id) — partial_sort on std::pair (cpp:324-333). One wave per query.
// ============================================================================
template <int R>
__global__ __launch_bounds__(256) void ivf_select_probes(const float* __restrict__ cd, uint32_t nlist, uint32_t B,
                                                uint32_t P, uint32_t* __restrict__ probes) {
    const uint32_t q = blockIdx.x * 4 + wave_index();
    if (q >= B) return;
    const int lane = lane_id();
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    const float* row = cd + (size_t)q * nlist;
    for (uint32_t c0 = 0; c0 < nlist; c0 += 64) {
        const uint32_t c = c0 + lane;
        const bool valid = c < nlist;
        const float d = valid ? nan_last(row[c]) : __builtin_inff();
        offer_lanes<R>(tk, valid && d <= kd, d, (uint64_t)c, (int)P, kd, ki);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t e = r * 64 + lane;
        if (e < P) probes[(size_t)q * P + e] = (uint32_t)tk.id[r];
    }
}

// ============================================================================
// Coarse quantiser on the matrix cores (L2 / IP): the batch x centroid-table
// product is the path's one real contraction, so it runs on v_mfma_f32_16x16x4_f32
// (f32 in, f32 accumulate). Its sums run in a different order from the reference's
// sequential loop, so they only bound the exact distance: with u = 2^-24 and
// n = padded dimension, |mfma - exact| <= 4 (n + 4) u (|q| + |c|)^2 for L2
// (|q| |c| for IP), counting the exact sum's own error against the real value.
// ivf_select_rerank then keeps every centroid whose interval can reach the P-th
// smallest upper bound, recomputes those exactly and selects by (dist, list).
// One wave = one 16-query x 16-centroid tile over all dimensions. Lane (r, h):
// row r = lane & 15 of each operand, dims d0 + 4h .. d0 + 4h + 3 of every
// 16-dim step, fed to four MFMAs (k index h <-> dim d0 + 4h + s in step s).
// The operand norms are summed from the same registers on the way.
// ============================================================================
typedef float f4v __attribute__((ext_vector_type(4)));

template <int M, int G>
__global__ __launch_bounds__(256) void ivf_coarse_mfma(const float* __restrict__ cent_rm, uint32_t nlist,
                                                       uint32_t dp, const float* __restrict__ qpad, uint32_t B,
                                                       float* __restrict__ approx, float* __restrict__ delta) {
    chain_prio();
    const int lane = lane_id();
    const uint32_t ct = blockIdx.x * 4 + wave_index();  // centroid tile
    const uint32_t qt = blockIdx.y;                      // query tile
    if (ct * 16 >= nlist) return;
    const int r = lane & 15, h = lane >> 4;
    const uint32_t qrow = qt * 16 + r, crow = ct * 16 + r;
    const bool qok = qrow < B, cok = crow < nlist;
    const float4* qa = (const float4*)(qpad + (size_t)(qok ? qrow : 0) * dp) + h;
    const float4* cb = (const float4*)(cent_rm + (size_t)(cok ? crow : 0) * dp) + h;
    f4v acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};  // two chains hide the MFMA latency
    float qn = 0.f, cn = 0.f;
    const uint32_t steps = dp / 16;  // a multiple of G (the launcher picks G = 8 or 4)
    float4 a[G], b[G];
#pragma unroll
    for (int g = 0; g < G; ++g) a[g] = qa[(size_t)g * 4], b[g] = cb[(size_t)g * 4];
    for (uint32_t s0 = 0; s0 < steps; s0 += G) {
        float4 an[G], bn[G];
        const uint32_t nx = s0 + G < steps ? s0 + G : s0;  // the last group re-loads itself
#pragma unroll
        for (int g = 0; g < G; ++g) an[g] = qa[(size_t)(nx + g) * 4], bn[g] = cb[(size_t)(nx + g) * 4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float4 x = qok ? a[g] : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 y = cok ? b[g] : make_float4(0.f, 0.f, 0.f, 0.f);
            f4v& ac = acc[g & 1];
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, ac, 0, 0, 0);
            qn = qn + (x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w);
            cn = cn + (y.x * y.x + y.y * y.y) + (y.z * y.z + y.w * y.w);
            a[g] = an[g];
            b[g] = bn[g];
        }
    }
    acc[0] = acc[0] + acc[1];
    // row norms: lanes r, r+16, r+32, r+48 hold the four dim quarters of row r
    qn += __shfl_xor(qn, 16);
    qn += __shfl_xor(qn, 32);
    cn += __shfl_xor(cn, 16);
    cn += __shfl_xor(cn, 32);
    // C/D layout (16x16): col = lane & 15 (centroid), row = (lane >> 4) * 4 + reg (query)
    const uint32_t c = ct * 16 + (lane & 15);
    const float ca = sqrtf(cn);
    const float K = 4.0f * (float)(dp + 4) * 5.9604645e-8f;  // 4 (n + 4) u
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int row = (lane >> 4) * 4 + reg;
        const float qrn = __shfl(qn, row);  // lane `row` (< 16) holds query row `row`'s norm
        const uint32_t q = qt * 16 + row;
        if (q < B && c < nlist) {
            const float qa_ = sqrtf(qrn);
            float ap, dl;
            if constexpr (M == kL2) {
                ap = (qrn + cn) - 2.0f * acc[0][reg];
                dl = K * ((qa_ + ca) * (qa_ + ca)) + 1e-30f;
            } else {
                ap = -acc[0][reg];
                dl = K * (qa_ * ca) + 1e-30f;
            }
            approx[(size_t)q * nlist + c] = ap;
            delta[(size_t)q * nlist + c] = dl;
        }
    }
}

// The same bounds for large row counts (assignment at add / Lloyd, big search batches),
// register-blocked: one wave computes a 32-row x 32-centroid output as 2 x 2 MFMA tiles,
// so every float4 it loads feeds 8 MFMAs instead of 4 (the 16 x 16 wave above is bound
// by L1 traffic, not by the matrix cores). A workgroup's 4 waves share the 32 rows and
// take 4 adjacent 32-centroid tiles. Lane (r, h) holds dims 4h .. 4h + 3 of each
// 16-dim step of rows r and 16 + r of both operands, as above.
template <int M>
__global__ __launch_bounds__(256) void ivf_coarse_mfma2x2(const float* __restrict__ cent_rm, uint32_t nlist,
                                                          uint32_t dp, const float* __restrict__ qpad, uint32_t B,
                                                          float* __restrict__ approx, float* __restrict__ delta) {
    constexpr int G = 4;  // 16-dim steps per prefetch group (dp / 16 is a multiple of 4)
    const int lane = lane_id();
    const uint32_t ct = blockIdx.x * 4 + wave_index();  // 32-centroid tile
    const uint32_t qt = blockIdx.y;                      // 32-row tile
    if (ct * 32 >= nlist) return;
    const int r = lane & 15, h = lane >> 4;
    const float4* qa[2];
    const float4* cb[2];
    bool qok[2], cok[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t qrow = qt * 32 + i * 16 + r, crow = ct * 32 + i * 16 + r;
        qok[i] = qrow < B;
        cok[i] = crow < nlist;
        qa[i] = (const float4*)(qpad + (size_t)(qok[i] ? qrow : 0) * dp) + h;
        cb[i] = (const float4*)(cent_rm + (size_t)(cok[i] ? crow : 0) * dp) + h;
    }
    f4v acc[2][2];
    float qn[2] = {0.f, 0.f}, cn[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    const uint32_t steps = dp / 16;
    float4 a[2][G], b[2][G];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i][g] = qa[i][(size_t)g * 4], b[i][g] = cb[i][(size_t)g * 4];
    for (uint32_t s0 = 0; s0 < steps; s0 += G) {
        float4 an[2][G], bn[2][G];
        const uint32_t nx = s0 + G < steps ? s0 + G : s0;  // the last group re-loads itself
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < 2; ++i) an[i][g] = qa[i][(size_t)(nx + g) * 4], bn[i][g] = cb[i][(size_t)(nx + g) * 4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float4 x[2], y[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                x[i] = qok[i] ? a[i][g] : make_float4(0.f, 0.f, 0.f, 0.f);
                y[i] = cok[i] ? b[i][g] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f4v& ac = acc[i][j];
                    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x[i].x, y[j].x, ac, 0, 0, 0);
                    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x[i].y, y[j].y, ac, 0, 0, 0);
                    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x[i].z, y[j].z, ac, 0, 0, 0);
                    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(x[i].w, y[j].w, ac, 0, 0, 0);
                }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                qn[i] = qn[i] + (x[i].x * x[i].x + x[i].y * x[i].y) + (x[i].z * x[i].z + x[i].w * x[i].w);
                cn[i] = cn[i] + (y[i].x * y[i].x + y[i].y * y[i].y) + (y[i].z * y[i].z + y[i].w * y[i].w);
                a[i][g] = an[i][g];
                b[i][g] = bn[i][g];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        qn[i] += __shfl_xor(qn[i], 16);
        qn[i] += __shfl_xor(qn[i], 32);
        cn[i] += __shfl_xor(cn[i], 16);
        cn[i] += __shfl_xor(cn[i], 32);
    }
    const float K = 4.0f * (float)(dp + 4) * 5.9604645e-8f;  // 4 (n + 4) u, as ivf_coarse_mfma
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t c = ct * 32 + j * 16 + (lane & 15);
        const float ca = sqrtf(cn[j]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int row = (lane >> 4) * 4 + reg;
                const float qrn = __shfl(qn[i], row);
                const uint32_t q = qt * 32 + i * 16 + row;
                if (q < B && c < nlist) {
                    const float qa_ = sqrtf(qrn);
                    float ap, dl;
                    if constexpr (M == kL2) {
                        ap = (qrn + cn[j]) - 2.0f * acc[i][j][reg];
                        dl = K * ((qa_ + ca) * (qa_ + ca)) + 1e-30f;
                    } else {
                        ap = -acc[i][j][reg];
                        dl = K * (qa_ * ca) + 1e-30f;
                    }
                    approx[(size_t)q * nlist + c] = ap;
                    delta[(size_t)q * nlist + c] = dl;
                }
            }
    }
}

// Sequential exact distance of wave-uniform query row q against this lane's centroid
// row (the reference's loop order, cpp:308-318). Rows are zero padded to dp.
template <int M>
__device__ __forceinline__ float exact_row(const float* __restrict__ qrow, const float* __restrict__ crow,
                                           uint32_t dp) {
    const float4* q4 = (const float4*)qrow;
    const float4* c4 = (const float4*)crow;
    float acc = 0.0f;
#pragma unroll 8
    for (uint32_t t = 0; t < dp / 4; ++t) acc = acc4<M>(acc, q4[t], c4[t]);
    return dist_finish<M>(acc);
}

// Per query (one workgroup of 4 waves): tau = P-th smallest upper bound;
// candidates = lists whose lower bound is <= tau (this always contains the exact
// top-P: P lists have exact distance <= tau); exact distances of the candidates;
// top-P by (dist, list) as the reference's partial_sort on std::pair
// (cpp:324-333). Non-finite bounds make a list a candidate; NaN distances order
// last. One lane per candidate runs the reference's sequential sum over its centroid
// row, read from the table with the loads issued well ahead (`ch`: only checked).
template <int R, int M>
__global__ __launch_bounds__(256) void ivf_select_rerank(const float* __restrict__ approx,
                                                         const float* __restrict__ delta,
                                                         const float* __restrict__ cent_rm, uint32_t nlist,
                                                         uint32_t dp, const float* __restrict__ qpad, uint32_t B,
                                                         uint32_t P, uint32_t ch, uint32_t* __restrict__ cand,
                                                         uint32_t* __restrict__ probes) {
    chain_prio();
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    __shared__ float s_top_d[4 * R * 64];
    __shared__ uint32_t s_top_i[4 * R * 64];
    __shared__ float s_tau;
    __shared__ uint32_t s_n;
    const uint32_t q = blockIdx.x;
    if (q >= B) return;
    // (LDS audit: s_top_* hold 4 R x 64 entries; the host launch checks P and the query
    // row's LDS (ch > 0), this early-out is the device's last line)
    if (P > 64u * R || ch > 64u || ch == 0u) return;
    const int lane = lane_id();
    const uint32_t w = wave_index();
    const float* ar = approx + (size_t)q * nlist;
    const float* dr = delta + (size_t)q * nlist;
    if (threadIdx.x == 0) s_n = 0;
    // pass 1: tau, an upper bound on the P-th smallest upper bound. Lists are read in
    // rounds of kPre per lane (c = w*64 + 256 j + lane), every load issued up front.
    constexpr int kPre = 16;
    if constexpr (R == 1) {
        // P <= 64: the P-th smallest of the block's 256 lane minima. P lanes hold a
        // value <= it, so at least P upper bounds are <= it; no top-P list is needed.
        float lm = __builtin_inff();
        for (uint32_t r0 = w * 64; r0 < nlist; r0 += 256 * kPre) {
            float hv[kPre];
#pragma unroll
            for (int j = 0; j < kPre; ++j) {
                const uint32_t c = r0 + j * 256 + lane;
                hv[j] = c < nlist ? nan_last(ar[c] + dr[c]) : __builtin_inff();
            }
#pragma unroll
            for (int j = 0; j < kPre; ++j) lm = hv[j] < lm ? hv[j] : lm;
        }
        uint64_t li = (uint64_t)(w * 64 + lane);
        bitonic_sort64(lm, li);
        s_top_d[w * 64 + lane] = lm;
        s_top_i[w * 64 + lane] = (uint32_t)li;
        __syncthreads();
        if (w == 0) {
            float a = s_top_d[lane];
            uint64_t ai = s_top_i[lane];
            for (int v = 1; v < 4; ++v) bitonic_merge64(a, ai, s_top_d[v * 64 + lane], s_top_i[v * 64 + lane]);
            const float t = rd_lane(a, (int)P - 1);
            if (lane == 0) s_tau = t;
        }
        __syncthreads();
    } else {
        // P > 64: each wave's top-P upper bounds, then the P-th smallest of their union
        WaveTopK<R> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        for (uint32_t r0 = w * 64; r0 < nlist; r0 += 256 * kPre) {
            float hv[kPre];
#pragma unroll
            for (int j = 0; j < kPre; ++j) {
                const uint32_t c = r0 + j * 256 + lane;
                hv[j] = c < nlist ? nan_last(ar[c] + dr[c]) : __builtin_inff();
            }
#pragma unroll
            for (int j = 0; j < kPre; ++j) {
                const uint32_t c = r0 + j * 256 + lane;
                offer_lanes<R>(tk, c < nlist && hv[j] <= kd, hv[j], (uint64_t)c, (int)P, kd, ki);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            s_top_d[(w * R + r) * 64 + lane] = tk.d[r];
            s_top_i[(w * R + r) * 64 + lane] = (uint32_t)tk.id[r];
        }
        __syncthreads();
        if (w == 0) {
            WaveTopK<R> tk2;
            tk2.init();
            float kd2 = __builtin_inff();
            uint64_t ki2 = kNoId;
            for (uint32_t e0 = 0; e0 < 4 * R * 64; e0 += 64) {
                const float d = s_top_d[e0 + lane];
                const uint32_t id = s_top_i[e0 + lane];
                const bool valid = id != 0xFFFFFFFFu;
                offer_lanes<R>(tk2, valid && d <= kd2, d, (uint64_t)id, (int)P, kd2, ki2);
            }
            if (lane == 0) s_tau = kd2;
        }
        __syncthreads();
    }
    const float tau = s_tau;
    // pass 2: candidates, appended through one LDS counter per wave-iteration
    uint32_t* cl = cand + (size_t)q * nlist;
    const uint64_t below = (1ull << lane) - 1;
    for (uint32_t r0 = w * 64; r0 < nlist; r0 += 256 * kPre) {
        bool want[kPre];
#pragma unroll
        for (int j = 0; j < kPre; ++j) {
            const uint32_t c = r0 + j * 256 + lane;
            want[j] = c < nlist && !(ar[c] - dr[c] > tau);
        }
#pragma unroll
        for (int j = 0; j < kPre; ++j) {
            const uint64_t m = __ballot(want[j]);
            if (!m) continue;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&s_n, (uint32_t)__popcll(m));
            base = __shfl(base, 0);
            if (want[j]) cl[base + __popcll(m & below)] = r0 + j * 256 + lane;
        }
    }
    __threadfence_block();
    __syncthreads();
    const uint32_t n = s_n;
    // pass 3: exact sequential distances of the candidates. Candidate j: wave (j / 64) % 4,
    // lane j % 64, its row read straight from the centroid table (L2 / MALL: the coarse step
    // just read it) 16 to 32 float4 ahead of the dependent add chain; the query row in LDS.
    // (Round 6: the rows were staged in LDS in chunks of 19 rows that only wave 0 summed, so a
    // query's ~40 candidates took 2 - 3 chunk rounds of load, barrier and 768-step chain.)
    const uint32_t n4 = dp / 4;  // (a multiple of 16)
    float4* q_l = smem;          // the query row (broadcast reads)
    for (uint32_t e = threadIdx.x; e < n4; e += 256) q_l[e] = ((const float4*)(qpad + (size_t)q * dp))[e];
    __syncthreads();
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    for (uint32_t j0 = w * 64; j0 < n; j0 += 256) {
        const uint32_t j = j0 + lane;
        const bool valid = j < n;
        const uint32_t c = valid ? cl[j] : 0u;
        const float4* x = (const float4*)(cent_rm + (size_t)c * dp);
        const uint32_t last = n4 - 1;
        float acc = 0.0f;
        float4 xa[16], xb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) xa[u] = x[min((uint32_t)u, last)], xb[u] = x[min(16u + u, last)];
        uint32_t t0 = 0;
        for (; t0 + 32 <= n4; t0 += 32) {
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = acc4<M>(acc, q_l[t0 + u], xa[u]);
#pragma unroll
            for (int u = 0; u < 16; ++u) xa[u] = x[min(t0 + 32 + u, last)];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = acc4<M>(acc, q_l[t0 + 16 + u], xb[u]);
#pragma unroll
            for (int u = 0; u < 16; ++u) xb[u] = x[min(t0 + 48 + u, last)];
        }
        if (t0 < n4) {  // (n4 = 32 m + 16: the last 16 are in xa)
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = acc4<M>(acc, q_l[t0 + u], xa[u]);
        }
        const float d = valid ? nan_last(dist_finish<M>(acc)) : __builtin_inff();
        offer_lanes<R>(tk, valid && d <= kd, d, (uint64_t)c, (int)P, kd, ki);
    }
    if (n > 64) {  // (more than one wave's candidates: the top-P of the four waves' lists)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            s_top_d[(w * R + r) * 64 + lane] = tk.d[r];
            s_top_i[(w * R + r) * 64 + lane] = (uint32_t)tk.id[r];
        }
        __syncthreads();
        if (w == 0) {
            tk.init();
            kd = __builtin_inff();
            ki = kNoId;
            for (uint32_t e0 = 0; e0 < 4 * R * 64; e0 += 64) {
                const float dd = s_top_d[e0 + lane];
                const uint32_t id = s_top_i[e0 + lane];
                offer_lanes<R>(tk, id != 0xFFFFFFFFu && dd <= kd, dd, (uint64_t)id, (int)P, kd, ki);
            }
        }
    }
    if (w == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t e = r * 64 + lane;
            if (e < P) probes[(size_t)q * P + e] = (uint32_t)tk.id[r];
        }
    }
}

// assign_to_lists (cpp:259-295) from the MFMA bounds: one wave per row. tau = the
// smallest upper bound; every centroid whose lower bound is <= tau may be the exact
// minimum (usually one or two); each such candidate's exact sequential distance is
// computed by one lane, and the row goes to the smallest (dist, centroid) — the first
// strict '<' winner of the reference loop. NaN distances order last (an all-NaN row
// goes to list 0, as the reference's FLT_MAX start does).
template <int M>
__global__ __launch_bounds__(256) void ivf_assign_rerank(const float* __restrict__ approx,
                                                         const float* __restrict__ delta,
                                                         const float* __restrict__ cent_rm, uint32_t nlist,
                                                         uint32_t dp, const float* __restrict__ rows, uint32_t n,
                                                         uint32_t* __restrict__ out) {
    const uint32_t r = blockIdx.x * 4 + wave_index();
    if (r >= n) return;
    const int lane = lane_id();
    const float* ar = approx + (size_t)r * nlist;
    const float* dr = delta + (size_t)r * nlist;
    constexpr int kPre = 8;
    float lm = __builtin_inff();
    for (uint32_t c0 = 0; c0 < nlist; c0 += 64 * kPre) {
        float hv[kPre];
#pragma unroll
        for (int j = 0; j < kPre; ++j) {
            const uint32_t c = c0 + j * 64 + lane;
            hv[j] = c < nlist ? nan_last(ar[c] + dr[c]) : __builtin_inff();
        }
#pragma unroll
        for (int j = 0; j < kPre; ++j) lm = hv[j] < lm ? hv[j] : lm;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float x = __shfl_xor(lm, o);
        lm = x < lm ? x : lm;
    }
    const float tau = lm;
    float bd = __builtin_inff();
    uint32_t bc = 0xFFFFFFFFu;
    const float4* x4 = (const float4*)(rows + (size_t)r * dp);  // wave-uniform row
    for (uint32_t c0 = 0; c0 < nlist; c0 += 64) {
        const uint32_t c = c0 + lane;
        const bool cand = c < nlist && !(ar[c] - dr[c] > tau);
        if (__ballot(cand) == 0) continue;
        if (cand) {
            const float4* c4 = (const float4*)(cent_rm + (size_t)c * dp);
            float acc = 0.0f;
            for (uint32_t t0 = 0; t0 < dp / 4; t0 += 8) {  // dp / 4 is a multiple of 16
                float4 xv[8], cv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = x4[t0 + u], cv[u] = c4[t0 + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc = acc4<M>(acc, xv[u], cv[u]);
            }
            const float d = nan_last(dist_finish<M>(acc));
            if (d < bd || (d == bd && c < bc)) {
                bd = d;
                bc = c;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float od = __shfl_xor(bd, o);
        const uint32_t oc = (uint32_t)__shfl_xor((int)bc, o);
        if (od < bd || (od == bd && oc < bc)) {
            bd = od;
            bc = oc;
        }
    }
    if (lane == 0) out[r] = bc < nlist ? bc : 0u;
}

// ============================================================================
// Probe inversion (one workgroup): sort the batch's (query, probe) pairs by list,
// give every pair its range of partial-result slots, and emit scan work items
// (list, segment, group of <= G pairs). Items of one list are ordered
// (segment, group) so the groups that re-read a segment sit in one workgroup.
// ============================================================================
constexpr uint32_t kInvalidKey = 0xFFFFFFFFu;
#ifndef VDB_SEED_LEVELS
#define VDB_SEED_LEVELS 1  // wide-item queue levels by quad index (0: plan order)
#endif

__device__ uint32_t plan_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
    const int lane = lane_id();
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t w = threadIdx.x < nw ? sh[threadIdx.x] : 0u;
        uint32_t s = w;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(s, off);
            if (lane >= off) s += y;
        }
        if (threadIdx.x < nw) sh[threadIdx.x] = s - w;
        if (threadIdx.x == nw - 1) sh[32] = s;
    }
    __syncthreads();
    const uint32_t res = sh[wid] + x - v;
    total = sh[32];
    __syncthreads();
    return res;
}

// Exclusive block scans of NB counters at once (one barrier pair): v[b] -> ex[b],
// tot[b] = block total. sh holds NB * 17 words.
template <int NB>
__device__ void plan_excl_scan_multi(const uint32_t* v, uint32_t* ex, uint32_t* tot, uint32_t* sh) {
    const int lane = lane_id();
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t nw = blockDim.x >> 6;  // <= 16
    uint32_t x[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        x[b] = v[b];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x[b], off);
            if (lane >= off) x[b] += y;
        }
        if (lane == 63) sh[b * 17 + wid] = x[b];
    }
    __syncthreads();
    if (threadIdx.x < NB) {  // one thread per counter walks the wave totals
        const uint32_t b = threadIdx.x;
        uint32_t run = 0;
        for (uint32_t w = 0; w < nw; ++w) {
            const uint32_t t = sh[b * 17 + w];
            sh[b * 17 + w] = run;
            run += t;
        }
        sh[b * 17 + 16] = run;
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        ex[b] = sh[b * 17 + wid] + x[b] - v[b];
        tot[b] = sh[b * 17 + 16];
    }
    __syncthreads();
}

// Query groups of one list with m (query, probe) pairs and ns segments. A list of at
// least kWideMinSeg segments (with top-k in one register) is scanned by wide items:
// ceil(m / wg) balanced groups x ceil(ns / segs_item) segment ranges, so each list is
// read ceil(m / wg) times per batch (wg = 16, or 32 with 8-wave workgroups; 0 = no wide
// items). Other lists: narrow items of <= gn pairs x ns.
struct ListGroups {
    uint32_t wide, narrow;
};
__device__ __forceinline__ ListGroups list_groups(uint32_t m, uint32_t ns, uint32_t gn, uint32_t wg) {
    ListGroups g;
    if (wg && ns >= (uint32_t)kWideMinSeg) {
        g.wide = (m + wg - 1) / wg;
        g.narrow = 0;
    } else {
        g.wide = 0;
        g.narrow = (m + gn - 1) / gn;
    }
    return g;
}

// Last index d in [0, n) with base[d] <= x (base non-decreasing, base[0] == 0).
__device__ __forceinline__ uint32_t find_owner(const uint32_t* base, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;  // answer in [lo, hi)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (base[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(1024) void ivf_plan_probes(const uint32_t* __restrict__ probes,
                                                        const uint32_t* __restrict__ nseg_local,
                                                        const uint32_t* __restrict__ count_local, uint32_t B,
                                                        uint32_t P, uint32_t NP, uint32_t gn, uint32_t wide_on,
                                                        uint32_t segs_item, uint32_t mfma_min,
                                                        ScanItem* __restrict__ items_n, ScanItem* __restrict__ items_w,
                                                        uint32_t* __restrict__ counters,
                                                        uint32_t* __restrict__ sorted_pair,
                                                        uint32_t* __restrict__ part_base_sorted,
                                                        uint32_t* __restrict__ part_base_qp,
                                                        uint32_t* __restrict__ nseg_qp,
                                                        uint32_t* __restrict__ l1base_qp,
                                                        uint2* __restrict__ l1_items,
                                                        unsigned long long* __restrict__ stats,
                                                        uint32_t* __restrict__ thr) {
    chain_prio();
    // keys, starts, base_n, base_w: dynamic LDS sized by the batch (NP = B x P rounded up to a
    // power of two; 4 NP + 1 words, at most kPlanMaxPairs), not by kPlanMaxPairs: the 128 KB
    // static arrays of round 5 fit no CU that held a collect workgroup, so with batches in flight
    // a batch's plan waited for a CU to drain (round 6; the headline batch takes 32 KB)
    extern __shared__ uint32_t plan_lds[];
    uint32_t* const keys = plan_lds;
    uint32_t* const starts = keys + NP;
    uint32_t* const base_n = starts + NP + 1;
    uint32_t* const base_w = base_n + NP;
    __shared__ uint32_t sh[33];
    __shared__ uint32_t sh_multi[(VDB_SEED_LEVELS + 2) * 17];
    __shared__ unsigned long long s_pairs;
    const uint32_t tid = threadIdx.x;
    const uint32_t BP = B * P;
    const uint32_t wide = wide_on;  // wide group size (0: no wide items)
    // (LDS audit, VERDICT r5: the arrays above hold kPlanMaxPairs keys. launch_plan refuses a
    // larger batch on the host; should one arrive anyway the kernel plans nothing — no items,
    // no valid pairs — instead of writing past them)
    if (NP > (uint32_t)kPlanMaxPairs || BP > NP) {
        if (tid < (uint32_t)kCounters) counters[tid] = 0u;
        return;
    }

    if (tid == 0) {
        s_pairs = 0;
    }
    for (uint32_t i = tid; i < BP; i += blockDim.x) thr[i] = kThrInf;  // the scan's shared thresholds
    // The valid pairs' keys (probed lists this shard stores) compacted to keys[0, nvalid), then
    // only those sorted: a 1/8 shard's batch has ~1/8 of its pairs valid, so its sort is 8x
    // shorter (round 6; at one GPU nothing changes). Each thread keys up to kPlanMaxPairs / 1024
    // pairs i = tid + 1024 j, counted, scanned, written.
    constexpr int kPer = kPlanMaxPairs / 1024;
    uint32_t kv[kPer];
    uint32_t nmine = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t i = tid + 1024u * (uint32_t)j;
        kv[j] = kInvalidKey;
        if (i < BP) {
            const uint32_t l = probes[i];
            const uint32_t ns = nseg_local[l];
            nseg_qp[i] = ns;
            if (ns) {
                kv[j] = (l << 13) | i;
                ++nmine;
            }
        }
    }
    uint32_t nvalid;
    uint32_t wpos = plan_excl_scan(nmine, sh, nvalid);
#pragma unroll
    for (int j = 0; j < kPer; ++j)
        if (kv[j] != kInvalidKey) keys[wpos++] = kv[j];
    uint32_t NS = 1;  // (the sort's size: a power of two >= nvalid)
    while (NS < nvalid) NS <<= 1;
    for (uint32_t i = nvalid + tid; i < NS; i += blockDim.x) keys[i] = kInvalidKey;
    __syncthreads();

    // Bitonic sort in LDS, one compare-exchange per thread and step: pair p is (i, i + j)
    // with i = 2j (p / j) + p % j. A wave's 64 pairs then lie inside one 128-key block for
    // every j <= 64, so those steps need no workgroup barrier (a wave's LDS operations
    // complete in order); only the steps with j >= 128 (and the step before one) do.
    const uint32_t npairs = NS >> 1;
    for (uint32_t kk = 2; kk <= NS; kk <<= 1) {
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t p = tid; p < npairs; p += blockDim.x) {
                const uint32_t i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), x = i + j;
                const uint32_t a = keys[i], b = keys[x];
                if ((a > b) == ((i & kk) == 0)) {
                    keys[i] = b;
                    keys[x] = a;
                }
            }
            const uint32_t jn = j > 1 ? j >> 1 : kk;  // the next step's distance
            if (j >= 128 || jn >= 128) {
                __syncthreads();
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
    __syncthreads();

    // Each thread owns a contiguous chunk of sorted positions.
    const uint32_t per = (nvalid + blockDim.x - 1) / blockDim.x;
    const uint32_t c0 = min(nvalid, tid * per), c1 = min(nvalid, c0 + per);
    auto list_of = [&](uint32_t s) { return keys[s] >> 13; };
    auto is_head = [&](uint32_t s) { return s == 0 || list_of(s - 1) != list_of(s); };
    auto fan_of = [&](uint32_t ns) { return ns > (uint32_t)kMergeFan ? (ns + kMergeFan - 1) / kMergeFan : 0u; };

    uint32_t hsum = 0, nsum = 0, fsum = 0;
    unsigned long long vsum = 0;
    for (uint32_t s = c0; s < c1; ++s) {
        hsum += is_head(s) ? 1u : 0u;
        const uint32_t ns = nseg_local[list_of(s)];
        nsum += ns;
        fsum += fan_of(ns);
        vsum += count_local[list_of(s)];
    }
    // (diagnostic counters: one atomic per wave, not per thread or list, below)
    uint32_t nd, nparts, nl1;
    const uint32_t dl_base = plan_excl_scan(hsum, sh, nd);
    const uint32_t pb_base = plan_excl_scan(nsum, sh, nparts);
    const uint32_t fb_base = plan_excl_scan(fsum, sh, nl1);
    {
        int cur = (int)dl_base - 1;
        uint32_t pb = pb_base, fb = fb_base;
        for (uint32_t s = c0; s < c1; ++s) {
            const uint32_t l = list_of(s);
            if (is_head(s)) starts[++cur] = s;
            const uint32_t i = keys[s] & 8191u;
            const uint32_t ns = nseg_local[l];
            sorted_pair[s] = ((i / P) << 16) | (i % P);
            part_base_sorted[s] = pb;
            part_base_qp[i] = pb;
            l1base_qp[i] = fb;
            const uint32_t nf = fan_of(ns);
            for (uint32_t j = 0; j < nf; ++j) l1_items[fb + j] = make_uint2(i, j);
            pb += ns;
            fb += nf;
        }
    }
    if (tid == 0) starts[nd] = nvalid;
    __syncthreads();

    // Item counts per list: narrow = groups x segments, wide = groups x segment quads.
    uint32_t nsum_n = 0, nsum_w = 0;
    {
        int cur = (int)dl_base - 1;
        for (uint32_t s = c0; s < c1; ++s) {
            if (!is_head(s)) continue;
            ++cur;
            const uint32_t ns = nseg_local[list_of(s)];
            const ListGroups g = list_groups(starts[cur + 1] - starts[cur], ns, gn, wide);
            nsum_n += g.narrow * ns;
            nsum_w += g.wide * ((ns + segs_item - 1) / segs_item);
        }
    }
    uint32_t n_narrow, n_wide;
    const uint32_t bn_base = plan_excl_scan(nsum_n, sh, n_narrow);
    const uint32_t bw_base = plan_excl_scan(nsum_w, sh, n_wide);
    unsigned long long lsum = 0, csum = 0;
    {
        int cur = (int)dl_base - 1;
        uint32_t bn = bn_base, bw = bw_base;
        for (uint32_t s = c0; s < c1; ++s) {
            if (!is_head(s)) continue;
            ++cur;
            const uint32_t l = list_of(s);
            const uint32_t ns = nseg_local[l];
            const ListGroups g = list_groups(starts[cur + 1] - starts[cur], ns, gn, wide);
            base_n[cur] = bn;
            base_w[cur] = bw;
            bn += g.narrow * ns;
            bw += g.wide * ((ns + segs_item - 1) / segs_item);
            lsum += count_local[l];
            // query slots streamed: wide items run query pairs (an odd group's last query
            // runs alone on scalar ops, but holds a pair slot)
            const uint32_t m = starts[cur + 1] - starts[cur];
            csum += (unsigned long long)count_local[l] * (g.wide ? 2 * ((m + 1) / 2) : m);
        }
    }
    __syncthreads();

    // Emit items in parallel. Items of one list are ordered (segment or quad, group):
    // the groups re-reading one stretch of the list are adjacent in the grid.
    // Each thread emits a contiguous range of items with a cursor (list, group, segment):
    // one binary search per thread, then O(1) per item (no per-item search or division).
    struct Cur {
        uint32_t dl, st, m, l, ng, nitems, off, gi, seg;
    };
    auto cur_open = [&](Cur& c, uint32_t dl, uint32_t off, bool is_wide) {
        c.dl = dl;
        c.st = starts[dl];
        c.m = starts[dl + 1] - c.st;
        c.l = list_of(c.st);
        const uint32_t ns = nseg_local[c.l];
        const ListGroups g = list_groups(c.m, ns, gn, wide);
        c.ng = is_wide ? g.wide : g.narrow;  // groups (0: the list has no items of this kind)
        c.nitems = is_wide ? g.wide * ((ns + segs_item - 1) / segs_item) : g.narrow * ns;
        c.off = off;
        c.gi = c.ng ? off % c.ng : 0;
        c.seg = c.ng ? off / c.ng : 0;
    };
    auto cur_next = [&](Cur& c, bool is_wide) {  // the next item in plan order
        if (++c.off < c.nitems) {
            if (++c.gi == c.ng) c.gi = 0, ++c.seg;
            return;
        }
        uint32_t dl = c.dl;
        do cur_open(c, ++dl, 0, is_wide);
        while (c.nitems == 0 && dl + 1 < nd);
    };
    {
        const uint32_t per_n = (n_narrow + blockDim.x - 1) / blockDim.x;
        const uint32_t x0 = min(n_narrow, tid * per_n), x1 = min(n_narrow, x0 + per_n);
        Cur c;
        if (x0 < x1) {
            const uint32_t dl = find_owner(base_n, nd, x0);
            cur_open(c, dl, x0 - base_n[dl], false);
            while (c.off >= c.nitems) cur_next(c, false);  // (lists without narrow items share a base)
        }
        for (uint32_t x = x0; x < x1; ++x) {
            ScanItem it;
            it.list = c.l;
            it.seg = c.seg;
            it.pair_start = c.st + c.gi * gn;
            it.npairs = min(gn, c.m - c.gi * gn);
            items_n[x] = it;
            if (x + 1 < x1) cur_next(c, false);
        }
    }
    // groups balanced in query PAIRS (a wave computes two queries per packed op): all
    // even-sized but the last, so the list costs ceil(m / 2) pair passes, not one more per
    // odd group (40 queries: 12 + 14 + 14, not 14 + 13 + 13)
    auto wide_item = [&](const Cur& c) {
        const uint32_t m2 = (c.m + 1) / 2;
        const uint32_t p0 = min(2 * (c.gi * m2 / c.ng), c.m), p1 = min(2 * ((c.gi + 1) * m2 / c.ng), c.m);
        ScanItem it;
        it.list = c.l;
        it.seg = c.seg;
        it.pair_start = c.st + p0;
        it.npairs = p1 - p0;
        return it;
    };
    auto wide_cursor = [&](Cur& c, uint32_t x0) {
        const uint32_t dl = find_owner(base_w, nd, x0);
        cur_open(c, dl, x0 - base_w[dl], true);
        while (c.off >= c.nitems) cur_next(c, true);
    };
    // Queue order of the wide items (a stable bucket sort over contiguous per-thread
    // ranges): the exact items in list order, then the items of >= mfma_min queries, which
    // the bounded scan kernel takes. (List order interleaves VALU-heavy hub items with
    // HBM-bound ones all through the grid; heaviest-first made the scan alone 8 % faster at
    // a 1/8 shard but two scans in flight 4 % slower at one GPU: both then run their heavy
    // items at the same time.)
    // First quads first (VDB_SEED_LEVELS): every list's first quad is queued ahead of the
    // other quads of all lists (with L levels: quads 0, .., L-1 each as a level, then the rest). Items of one list are otherwise taken within a fraction
    // of an item's duration, so all of a hub list's segments would start from the cold
    // (infinite) shared threshold; queued behind the first quads they start from the k-th
    // distance of the list's first quad (a.thr), and most insertions never happen.
    constexpr int kLevels = VDB_SEED_LEVELS;
    constexpr int kBuckets = kLevels + 2;
    auto bucket_of = [&](const ScanItem& it) -> uint32_t {
        if (mfma_min && it.npairs >= mfma_min) return kLevels + 1;
        return min(it.seg, (uint32_t)kLevels);
    };
    const uint32_t wper = (n_wide + blockDim.x - 1) / blockDim.x;
    const uint32_t w0 = min(n_wide, tid * wper), w1 = min(n_wide, w0 + wper);
    uint32_t bcnt[kBuckets], bex[kBuckets], btot[kBuckets];
#pragma unroll
    for (int b = 0; b < kBuckets; ++b) bcnt[b] = 0;
    {
        Cur c;
        if (w0 < w1) wide_cursor(c, w0);
        for (uint32_t x = w0; x < w1; ++x) {
            const uint32_t b = bucket_of(wide_item(c));
#pragma unroll
            for (int bb = 0; bb < kBuckets; ++bb) bcnt[bb] += b == (uint32_t)bb ? 1u : 0u;
            if (x + 1 < w1) cur_next(c, true);
        }
    }
    plan_excl_scan_multi<kBuckets>(bcnt, bex, btot, sh_multi);
    uint32_t n_exact = 0;
#pragma unroll
    for (int b = 0; b <= kLevels; ++b) n_exact += btot[b];
    const uint32_t n_bounded = btot[kLevels + 1];
    {
        uint32_t base = 0;
#pragma unroll
        for (int b = 0; b < kBuckets; ++b) {  // bucket base + this thread's offset in it
            const uint32_t t = btot[b];
            bex[b] += base;
            base += t;
        }
        Cur c;
        if (w0 < w1) wide_cursor(c, w0);
        for (uint32_t x = w0; x < w1; ++x) {
            const ScanItem it = wide_item(c);
            const uint32_t b = bucket_of(it);
            uint32_t dst = 0;
#pragma unroll
            for (int bb = 0; bb < kBuckets; ++bb)
                if (b == (uint32_t)bb) dst = bex[bb]++;
            items_w[dst] = it;
            if (x + 1 < w1) cur_next(c, true);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        vsum += __shfl_xor(vsum, off);
        lsum += __shfl_xor(lsum, off);
        csum += __shfl_xor(csum, off);
    }
    if ((tid & 63) == 0 && vsum) atomicAdd(&s_pairs, vsum);
    if ((tid & 63) == 0) {
        if (vsum) atomicAdd(&stats[4], vsum);
        if (lsum) atomicAdd(&stats[1], lsum);
        if (csum) atomicAdd(&stats[7], csum);
    }
    if (tid == 0) {
        counters[0] = n_narrow;
        counters[1] = nparts;
        counters[2] = nl1;
        counters[3] = n_exact;
        counters[4] = 0;  // work queues of the persistent scan kernels (narrow waves, wide and
        counters[5] = 0;  // bounded workgroups)
        counters[6] = 0;
        counters[7] = n_bounded;  // bounded items: items_w[n_exact, n_exact + n_bounded)
        counters[kCtrValid] = nvalid;  // (sorted pairs [0, nvalid) are the batch's valid pairs)
    }
    __syncthreads();  // (s_pairs complete)
    if (tid == 0) {
        counters[kCtrPairs] = (uint32_t)min(s_pairs, 0xFFFFFFFFull);
        atomicAdd(&stats[0], (unsigned long long)nd);  // (the per-wave sums follow)
        atomicAdd(&stats[2], (unsigned long long)(n_narrow + n_wide));
        atomicAdd(&stats[3], 1ull);
    }
}

// ============================================================================
// ivf_scan: the fine scan of one list segment for a group of <= G queries
// (search_list_cpu, cpp:347-370). One lane = one list vector; one wave-load reads
// 1 KiB of the interleaved block; query dims are wave-uniform (scalar loads).
// Each query keeps a wave top-k of (dist, id); the segment's top-k becomes one
// partial result of that (query, probe) pair.
// ============================================================================


// Stream nb 64-vector blocks of one list segment through a wave as a tile pipeline:
// T float4 registers per lane hold the next T tiles, and each tile's register is
// refilled with the tile T ahead right after it is consumed, so T-1 wave-loads
// (1 KiB each) stay in flight while the wave computes. Tiles of consecutive blocks
// are contiguous ([block][D4][64] float4) and T divides D4 (the layout pads D4), so
// every load is unconditional: the pipeline runs T tiles (and one id block) past
// the segment, which the arena's slack block keeps in bounds.
//   compute(x, t): consume tile t (0 <= t < d4) of the current block
//   finish(j, id): block j done; id = this lane's id slot in block j

//
// ROWS: the same segment read from the lists' row-major fp32 copy ([slot][dp], the screen's
// rows, then the lists' only fp32 copy; one slack block past the last list) instead of the
// interleaved arena: lane = vector still, tile t of block j at base + 64 d4 j + t, so one
// wave-load touches 64 rows (16 B each) and the row's next tiles are the same lines (plain
// loads, which keep them in the L1/L2 for those tiles). Exact-path searches on an index
// whose arena was released (k > 64, the run-time floor) run on it without rebuilding it.
template <bool ROWS>
__device__ __forceinline__ const float4* lane_base(const float4* lists, uint64_t b0, uint32_t d4, int lane) {
    return ROWS ? lists + (b0 * 64 + (uint64_t)lane) * d4 : lists + b0 * d4 * 64 + lane;
}

template <int T, bool ROWS = false, class Compute, class Finish>
__device__ __forceinline__ void stream_blocks(const float4* __restrict__ base, const uint64_t* __restrict__ ids,
                                              uint32_t d4, uint32_t nb, Compute&& compute, Finish&& finish) {
    constexpr size_t TS = ROWS ? 1 : 64;  // float4 between a lane's consecutive tiles
    auto ld = [](const float4* q) -> float4 {
        if constexpr (ROWS) return *q;
        else return load_nt(q);
    };
    float4 x[T];
    const float4* p = base;
#pragma unroll
    for (int t = 0; t < T; ++t) x[t] = ld(p + (size_t)t * TS);
    uint64_t id_next = __builtin_nontemporal_load(ids);
    for (uint32_t j = 0; j < nb; ++j) {
        const uint64_t id = id_next;
        id_next = __builtin_nontemporal_load(ids + (size_t)(j + 1) * 64);
        for (uint32_t t0 = 0; t0 < d4; t0 += T) {
            // the next round's first tile (row-major: past the row's end, the next block's row)
            const float4* pn = p + (size_t)T * TS;
            if (ROWS && t0 + T == d4) pn += (size_t)63 * d4;
            static_for<0, T>([&](auto u) {
                constexpr int t = decltype(u)::value;
                compute(x[t], t0 + t, u);
                if (!(VDB_SCAN_DIAG & 32)) x[t] = ld(pn + (size_t)t * TS);  // (DIAGNOSTIC 32: no list reads)
            });
            p = pn;
        }
        finish(j, id);
    }
}

// One narrow wave-item: one segment of a small list against G <= 4 queries whose
// dims are wave-uniform scalar loads; each query's top-k lives in registers.
template <int R, int G, int M, bool ROWS>
__device__ __forceinline__ void scan_item(const ScanArgs& a, const ScanItem it) {
    const int lane = lane_id();
    const uint32_t count = a.count[it.list];
    const uint32_t seg_vectors = a.seg_blocks * 64;
    const uint64_t b0 = a.block_off[it.list] + (uint64_t)it.seg * a.seg_blocks;
    const uint32_t v0 = it.seg * seg_vectors;
    const uint32_t nv = min(count - v0, seg_vectors);
    const uint32_t nb = (nv + 63) >> 6;
    const uint32_t d4 = a.d4;
    const int k = (int)a.k;
    const int np = (int)it.npairs;  // <= G; slots g >= np recompute query np-1 and are dropped

    const float4* q[G];
    uint32_t part[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int gg = g < np ? g : np - 1;
        const uint32_t pr = a.sorted_pair[it.pair_start + gg];
        q[g] = (const float4*)(a.qpad + (size_t)(pr >> 16) * d4 * 4);
        part[g] = a.part_base_sorted[it.pair_start + gg] + it.seg;
    }
    WaveTopK<R> tk[G];
    float kd[G];
    uint64_t ki[G];
    float acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        tk[g].init();
        kd[g] = __builtin_inff();
        ki[g] = kNoId;
        acc[g] = 0.0f;
    }
    // one HBM read of a list vector feeds G distance chains, each summed in d order
    auto compute = [&](const float4 x, uint32_t t, auto) {
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = acc4<M>(acc[g], q[g][t], x);
    };
    auto finish = [&](uint32_t j, uint64_t id) {
        const bool valid = j * 64 + lane < nv;
        bool want[G];
        bool any = false;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            acc[g] = dist_finish<M>(acc[g]);
            want[g] = g < np && valid && acc[g] <= kd[g];
            any |= want[g];
        }
        if (__ballot(any)) {
            const uint64_t vid = valid ? id : kNoId;
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (g < np) offer_lanes<R>(tk[g], want[g], acc[g], vid, k, kd[g], ki[g]);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = 0.0f;
    };
    // (row-major: 8 tiles, half a row's 128-byte line pair, in flight per lane)
    stream_blocks<ROWS ? 8 : kTilePipeNarrow, ROWS>(lane_base<ROWS>(a.arena, b0, d4, lane), a.ids + b0 * 64 + lane, d4,
                                                    nb, compute, finish);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (g >= np) break;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = r * 64 + lane;
            if (e < k) {
                a.part_d[(size_t)part[g] * k + e] = tk[g].d[r];
                a.part_i[(size_t)part[g] * k + e] = tk[g].id[r];
            }
        }
    }
}

typedef float f2 __attribute__((ext_vector_type(2)));

// Packed term for two queries q = (qa, qb) against one list value held in half H of
// the aligned register pair x (H = 0: x.lo, 1: x.hi). The broadcast is an op_sel on
// the pair the value was loaded into, so a float4 of list data is consumed in place
// (the compiler would otherwise copy the odd halves into fresh pairs and, with them,
// wait on a prefetch it just issued). Sub, mul, add stay separate instructions:
// each half rounds exactly like the scalar diff = a - b; acc = acc + diff * diff.
template <int H>
__device__ __forceinline__ f2 pk_sub_bcast(f2 q, f2 x) {
    f2 r;
    if constexpr (H == 0)
        asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(q), "v"(x));
    else
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(q), "v"(x));
    return r;
}
template <int H>
__device__ __forceinline__ f2 pk_mul_bcast(f2 q, f2 x) {
    f2 r;
    if constexpr (H == 0)
        asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(q), "v"(x));
    else
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(q), "v"(x));
    return r;
}

template <int M, int H>
__device__ __forceinline__ f2 dist_term2(f2 acc, f2 q, f2 x) {
    if constexpr (M == kL2) {
        const f2 diff = pk_sub_bcast<H>(q, x);
        return acc + diff * diff;
    } else if constexpr (M == kIP) {
        return acc + pk_mul_bcast<H>(q, x);
    } else {
        return acc;
    }
}

// One wave of a wide item: segment `seg` of list it.list against GP query pairs read
// from LDS as interleaved pairs (q[2p][d], q[2p+1][d]): the item's pairs are staged
// tile-major with `pstride` pairs per tile, and this wave takes the GP pairs starting at
// qlds (its queries are the item's q0 .. q0 + np - 1). Two queries run per packed
// instruction (v_pk_add_f32 / v_pk_mul_f32 round each half exactly like the scalar
// ops); every query's sum still runs in d order. Per query only the k-th distance
// lives in registers; the top-k lists live in LDS (tk_d / tk_i), and the insertion
// code exists once, looping over the queries that have candidates.
#ifndef VDB_BIG_GROUP_PREFETCH
#define VDB_BIG_GROUP_PREFETCH 0  // 1 spills ~100 VGPRs in the 16-pair instantiation (measured with -Rpass-analysis)
#endif
constexpr bool kBigGroupPrefetch = VDB_BIG_GROUP_PREFETCH != 0;

// Shared thresholds (exact): a candidate strictly worse than a k-th distance that some
// wave has already reached on the same (query, list) cannot be in that list's top-k —
// those k candidates are in that wave's segment partial and beat it — so it is never
// inserted. Partials may then hold fewer than k entries; the merges take the top-min(k,
// n_l) of the union, which is unchanged. Ties (equal distance) are always kept.
// ODD: the wave's last pair holds one query (an odd query count): that query runs on
// plain v_sub/v_mul/v_add on the pair's low halves instead of a padded packed pair,
// which costs the same per lane-op, so the padding half's work is not done at all.
#ifndef VDB_ODD_PAIRS
#define VDB_ODD_PAIRS 1
#endif
constexpr bool kOddPairs = VDB_ODD_PAIRS != 0;
template <int GP, int M, bool SPLIT, bool ODD, bool ROWS>
__device__ __forceinline__ void scan_wide_wave(const ScanArgs& a, const ScanItem it, const float4* qlds,
                                               const uint32_t pstride_rt, const int q0, const int np, float* tk_d,
                                               uint64_t* tk_i, uint32_t* s_thr, const uint32_t seg) {
    constexpr int G = 2 * GP;
    // pairs per staged tile row: the wave's own pair count unless the item's queries are
    // split between two halves of the workgroup (a wave-uniform scalar either way)
    const uint32_t pstride = SPLIT ? pstride_rt : (uint32_t)GP;
    const uint32_t d4 = a.d4;
    const int lane = lane_id();
    const uint32_t count = a.count[it.list];
    const uint32_t seg_vectors = a.seg_blocks * 64;
    const uint64_t b0 = a.block_off[it.list] + (uint64_t)seg * a.seg_blocks;
    const uint32_t v0 = seg * seg_vectors;
    const uint32_t nv = min(count - v0, seg_vectors);
    const uint32_t nb = (nv + 63) >> 6;
    const int k = (int)a.k;

    for (int e = lane; e < G * k; e += 64) {
        tk_d[e] = __builtin_inff();
        tk_i[e] = kNoId;
    }
    float kd[G];
    f2 acc[GP];
    float acc1 = 0.0f;  // ODD: the single query of the last pair
#pragma unroll
    for (int g = 0; g < G; ++g) kd[g] = __builtin_inff();
#pragma unroll
    for (int p = 0; p < GP; ++p) acc[p] = f2{0.0f, 0.0f};
    // query g's running sum (g wave-uniform and unrolled: a register, no indexing)
    auto qsum = [&](int g) -> float {
        if (ODD && g == 2 * (GP - 1)) return acc1;
        return (g & 1) ? acc[g >> 1].y : acc[g >> 1].x;
    };
    // pair p's four terms of tile (lo, hi) against list values x
    auto pair_terms = [&](int p, const float4 lo, const float4 hi, const f2 xlo, const f2 xhi, const float4 x) {
        if (ODD && p == GP - 1) {  // query 2p's dims sit in the low halves: lo.x, lo.z, hi.x, hi.z
            acc1 = dist_term<M>(acc1, lo.x, x.x);
            acc1 = dist_term<M>(acc1, lo.z, x.y);
            acc1 = dist_term<M>(acc1, hi.x, x.z);
            acc1 = dist_term<M>(acc1, hi.z, x.w);
        } else {
            acc[p] = dist_term2<M, 0>(acc[p], f2{lo.x, lo.y}, xlo);
            acc[p] = dist_term2<M, 1>(acc[p], f2{lo.z, lo.w}, xlo);
            acc[p] = dist_term2<M, 0>(acc[p], f2{hi.x, hi.y}, xhi);
            acc[p] = dist_term2<M, 1>(acc[p], f2{hi.z, hi.w}, xhi);
        }
    };

    // Query pairs of tile t sit at qlds[(t * GP + p) * 2 + {0, 1}]: one address per
    // tile, the pairs at immediate offsets. Each pair's registers are refilled with
    // the next tile's pair as soon as they are consumed, so every LDS read has a whole
    // tile of arithmetic to land in.
    // More than 8 pairs: the register copy of a tile's pairs takes 4·GP float4, so either
    // fewer list tiles stay in flight (kBigGroupPrefetch) or each pair is read from LDS
    // where it is used.
    constexpr bool kDirect = GP > 8 && !kBigGroupPrefetch;
    constexpr int QB = kDirect ? 1 : GP;
    float4 qb[QB][2];
    if constexpr (!kDirect) {
        const float4* src = qlds;
#pragma unroll
        for (int p = 0; p < GP; ++p) qb[p][0] = src[2 * p], qb[p][1] = src[2 * p + 1];
    }
    auto compute = [&](const float4 x, uint32_t t, auto) {
        const f2 xlo = {x.x, x.y}, xhi = {x.z, x.w};
        if constexpr (kDirect) {
            const float4* cur = qlds + (size_t)t * pstride * 2;
#pragma unroll
            for (int p = 0; p < GP; ++p) {
                const float4 lo = cur[2 * p], hi = cur[2 * p + 1];
                pair_terms(p, lo, hi, xlo, xhi, x);
            }
        } else {
            const float4* nxt = qlds + (size_t)(t + 1 == d4 ? 0 : t + 1) * pstride * 2;
#pragma unroll
            for (int p = 0; p < GP; ++p) {
                const float4 lo = qb[p][0], hi = qb[p][1];
                pair_terms(p, lo, hi, xlo, xhi, x);
                if (!(VDB_SCAN_DIAG & 16)) {  // (DIAGNOSTIC 16: no LDS reads of query pairs in the loop)
                    qb[p][0] = nxt[2 * p];
                    qb[p][1] = nxt[2 * p + 1];
                }
            }
        }
    };
    auto finish = [&](uint32_t j, uint64_t id) {
        const bool valid = j * 64 + lane < nv;
        // the item's shared thresholds (the other waves' progress on the same list)
        float th[G];
#pragma unroll
        for (int g = 0; g < G; ++g) th[g] = g < np ? fminf(kd[g], ord_dec(s_thr[g])) : kd[g];
        uint32_t pend = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float dist = dist_finish<M>(qsum(g));
            if (g < np && __ballot(valid && dist <= th[g])) pend |= 1u << g;
        }
        if (VDB_SCAN_DIAG & 1) pend = 0;  // DIAGNOSTIC: no top-k maintenance (results invalid)
        if ((VDB_SCAN_DIAG & 4) && j == 0) pend = 0;  // DIAGNOSTIC: no insertion on a segment's first block
        if ((VDB_SCAN_DIAG & 8) && j != 0) pend = 0;  // DIAGNOSTIC: insertions on the first block only
        if (pend) {
            const uint64_t vid = valid ? id : kNoId;
            do {
                const int gs = __builtin_ctz(pend);
                pend &= pend - 1;
                float dist = 0.0f, kdg = 0.0f;
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (g == gs) {
                        dist = dist_finish<M>(qsum(g));
                        kdg = th[g];
                    }
                float* sd = tk_d + gs * k;
                uint64_t* si = tk_i + gs * k;
                WaveTopK<1> tk;
                tk.d[0] = lane < k ? sd[lane] : __builtin_inff();
                tk.id[0] = lane < k ? si[lane] : kNoId;
                float nkd;
                uint64_t nki;
                tk.at(k - 1, nkd, nki);
                offer_lanes<1>(tk, valid && dist <= kdg, dist, vid, k, nkd, nki);
                if (lane < k) {
                    sd[lane] = tk.d[0];
                    si[lane] = tk.id[0];
                }
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (g == gs) kd[g] = nkd;
                // a full list's k-th below the shared threshold lowers it for the item's waves
                if (nkd < kdg && lane == 0) atomicMin(&s_thr[gs], ord_enc(nkd));
            } while (pend);
        }
#pragma unroll
        for (int p = 0; p < GP; ++p) acc[p] = f2{0.0f, 0.0f};
        acc1 = 0.0f;
    };
    // more than 8 pairs: fewer tiles in flight (the pairs' query registers take the rest)
    constexpr int T = GP <= 8 ? kTilePipe : (kBigGroupPrefetch ? kTilePipe / 4 : kTilePipe / 2);
    stream_blocks<T, ROWS>(lane_base<ROWS>(a.arena, b0, d4, lane), a.ids + b0 * 64 + lane, d4, nb, compute, finish);
    // the segment's k-th distances lower the list-wide thresholds for later items
#pragma unroll
    for (int g = 0; g < G; ++g)
        if (g < np && lane == 0 && kd[g] < __builtin_inff())
            atomicMin(&a.thr[it.pair_start + q0 + g], ord_enc(kd[g]));
    for (int g = 0; g < np; ++g) {
        const uint32_t part = a.part_base_sorted[it.pair_start + q0 + g] + seg;
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk_d[g * k + lane];
            a.part_i[(size_t)part * k + lane] = tk_i[g * k + lane];
        }
    }
}

// ============================================================================
// Bounded wide wave (L2 / IP, items of >= a.mfma_min queries): the item semantics of
// scan_wide_wave for up to 16 queries, with every (query, vector) distance first
// BOUNDED on the matrix cores and computed exactly only where it can reach the top-k.
//  * Stream: the segment's rows go through v_mfma_f32_16x16x1_4b_f32 (4 blocks of
//    16 x 16 x 1): A = this lane's list vector (lane = vector, the arena's float4 in
//    place), B = query (lane & 15) from the item's row-major staging [d4][16] float4.
//    D lane l, reg r holds <q_(l&15), x_v> for v = 16 (r >> 2) + 4 (l >> 4) + (r & 3)
//    (measured: tools/mfma_probe.hip). Vector and query norms ride along (VALU).
//  * Bounds: approx = |q|^2 + |x|^2 - 2 <q, x> (L2) or -<q, x> (IP) is within
//    delta = 4 (n + 4) u (|q| + |x|)^2 (L2; |q||x| for IP) of the reference's
//    sequential fp32 distance — the coarse step's bound (ivf_coarse_mfma above).
//  * Threshold per query: min(own k-th exact, the item's shared k-th, T_seg), where
//    T_seg is the smallest block bound so far: per block, each of a query's 4 lanes
//    takes the ceil(k/4)-th smallest upper bound of its 16 vectors and the block bound
//    is the largest of the 4 — at least k vectors of the segment have exact distances
//    <= it, so anything strictly above it is not in the segment's multiset top-k.
//  * Candidates (lower bound not above the threshold; non-finite bounds always) are
//    compacted into an LDS list and recomputed exactly in rounds of 64 (one lane per
//    candidate, the reference's sequential sum over the re-read vector), then offered
//    to the query's top-k exactly as scan_wide_wave does. Results are bit-identical:
//    only candidates strictly worse than k vectors of the same list are skipped.
// ============================================================================
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kBoundPipe = 8;  // list rows in flight per lane (x 2 waves per SIMD: 16 KiB per SIMD)
constexpr int kExactPipe = 4;  // rows in flight per lane of an exact re-rank round

// (A real call: inlined into ivf_scan_wide, its registers would add to the exact
// waves' and spill both; one call per segment costs nothing measurable.)
template <int M>
__device__ __forceinline__ void scan_wide_wave_mfma(const ScanArgs& a, const ScanItem it, const float4* qrow,
                                                    const int np, float* tk_d, uint64_t* tk_i, uint32_t* s_thr,
                                                    uint16_t* cand, const uint32_t seg) {
    const uint32_t d4 = a.d4;
    const int lane = lane_id();
    const int qj = lane & 15;  // this lane's query: the B column of every D register
    const bool qok = qj < np;
    const uint32_t count = a.count[it.list];
    const uint32_t seg_vectors = a.seg_blocks * 64;
    const uint64_t b0 = a.block_off[it.list] + (uint64_t)seg * a.seg_blocks;
    const uint32_t v0 = seg * seg_vectors;
    const uint32_t nv = min(count - v0, seg_vectors);
    const uint32_t nb = (nv + 63) >> 6;
    const int k = (int)a.k;
    const int cth = (k + 3) >> 2;  // lane rank of the block bound (k <= 16; larger k: no block bound)

    for (int e = lane; e < kWaveQueries * k; e += 64) {
        tk_d[e] = __builtin_inff();
        tk_i[e] = kNoId;
    }
    float kdl = __builtin_inff();   // query qj's k-th exact distance (its top-k lives in LDS)
    float tseg = __builtin_inff();  // query qj's smallest block bound in this segment
    const float K = 4.0f * (float)(d4 * 4 + 4) * 5.9604645e-8f;  // 4 (n + 4) u
    v16f acc = {};
    float xn = 0.0f, qn = 0.0f;
    float4 qb = qrow[qj];
    const float4* seg_base = a.arena + b0 * d4 * 64;
    auto compute = [&](const float4 x, uint32_t t, auto) {
        const float4 q = qb;
        qb = qrow[(size_t)(t + 1 == d4 ? 0 : t + 1) * 16 + qj];
        acc = __builtin_amdgcn_mfma_f32_16x16x1f32(x.x, q.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x1f32(x.y, q.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x1f32(x.z, q.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x1f32(x.w, q.w, acc, 0, 0, 0);
        xn = __builtin_fmaf(x.x, x.x, xn);
        xn = __builtin_fmaf(x.y, x.y, xn);
        xn = __builtin_fmaf(x.z, x.z, xn);
        xn = __builtin_fmaf(x.w, x.w, xn);
        qn = __builtin_fmaf(q.x, q.x, qn);
        qn = __builtin_fmaf(q.y, q.y, qn);
        qn = __builtin_fmaf(q.z, q.z, qn);
        qn = __builtin_fmaf(q.w, q.w, qn);
    };
    auto finish = [&](uint32_t j, uint64_t id) {
        const float xnl = xn, qnv = qn;
        xn = 0.0f;
        qn = 0.0f;
        const float qa = sqrtf(qnv);
        const float th = fminf(kdl, qok ? ord_dec(s_thr[qj]) : __builtin_inff());
        const uint32_t vb = j * 64;
        float lb[16];
        uint32_t vmask = 0;
        float m0 = __builtin_inff(), m1 = m0, m2 = m0, m3 = m0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int v = 16 * (r >> 2) + 4 * (lane >> 4) + (r & 3);
            const float xv = __shfl(xnl, v);
            const bool valid = vb + v < nv;
            vmask |= valid ? 1u << r : 0u;
            float ap, dl;
            if constexpr (M == kL2) {
                const float xa = sqrtf(xv);
                ap = (qnv + xv) - 2.0f * acc[r];
                dl = K * ((qa + xa) * (qa + xa)) + 1e-30f;
            } else {
                ap = -acc[r];
                dl = K * (qa * sqrtf(xv)) + 1e-30f;
            }
            lb[r] = ap - dl;
            float ub = ap + dl;
            ub = valid && ub == ub ? ub : __builtin_inff();
            m3 = fminf(m3, fmaxf(m2, ub));
            m2 = fminf(m2, fmaxf(m1, ub));
            m1 = fminf(m1, fmaxf(m0, ub));
            m0 = fminf(m0, ub);
        }
        float tb = cth == 1 ? m0 : cth == 2 ? m1 : cth == 3 ? m2 : cth == 4 ? m3 : __builtin_inff();
        tb = fmaxf(tb, xor_f<16>(tb));
        tb = fmaxf(tb, xor_f<32>(tb));
        tseg = fminf(tseg, tb);
        const float T = fminf(th, tseg);
        uint32_t bits = 0;
        if (qok) {
#pragma unroll
            for (int r = 0; r < 16; ++r) bits |= !(lb[r] > T) ? 1u << r : 0u;
            bits &= vmask;
        }
        if (VDB_SCAN_DIAG & 1) bits = 0;  // DIAGNOSTIC: no exact pass / top-k (results invalid)
        // compact the candidates: (vector << 4 | query) per entry, lanes in order
        const uint32_t cnt = (uint32_t)__builtin_popcount(bits);
        uint32_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            inc += lane >= o ? y : 0u;
        }
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        acc = v16f{};
        if (total == 0) return;
        uint32_t off = inc - cnt;
        while (bits) {
            const int r = __builtin_ctz(bits);
            bits &= bits - 1;
            const int v = 16 * (r >> 2) + 4 * (lane >> 4) + (r & 3);
            cand[off++] = (uint16_t)((v << 4) | qj);
        }
        __builtin_amdgcn_wave_barrier();
        if (a.mstats && lane == 0) atomicAdd(&a.mstats[0], (unsigned long long)total);
        const float4* blk = seg_base + (size_t)j * d4 * 64;
        for (uint32_t base = 0; base < total; base += 64) {
            const bool act = base + lane < total;
            const uint32_t ent = act ? cand[base + lane] : 0u;
            const int cv = (int)(ent >> 4), cq = (int)(ent & 15);
            // the reference's sequential sum for (query cq, vector cv), 8 rows in flight
            const float4* xp = blk + cv;
            const float4* qp = qrow + cq;
            float sum = 0.0f;
            for (uint32_t t0 = 0; t0 < d4; t0 += kExactPipe) {
                float4 xv[kExactPipe], qv[kExactPipe];
#pragma unroll
                for (int u = 0; u < kExactPipe; ++u) {
                    xv[u] = xp[(size_t)(t0 + u) * 64];
                    qv[u] = qp[(size_t)(t0 + u) * 16];
                }
#pragma unroll
                for (int u = 0; u < kExactPipe; ++u) sum = acc4<M>(sum, qv[u], xv[u]);
            }
            const float dist = dist_finish<M>(sum);
            const uint64_t cid = shfl_u64(id, cv);
            uint32_t qm = act ? 1u << cq : 0u;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) qm |= (uint32_t)__shfl_xor((int)qm, o);
            qm = __builtin_amdgcn_readfirstlane(qm);
            while (qm) {
                const int gs = __builtin_ctz(qm);
                qm &= qm - 1;
                const float kdg = fminf(rd_lane(kdl, gs), ord_dec(s_thr[gs]));
                float* sd = tk_d + gs * k;
                uint64_t* si = tk_i + gs * k;
                WaveTopK<1> tk;
                tk.d[0] = lane < k ? sd[lane] : __builtin_inff();
                tk.id[0] = lane < k ? si[lane] : kNoId;
                float nkd;
                uint64_t nki;
                tk.at(k - 1, nkd, nki);
                offer_lanes<1>(tk, act && cq == gs && dist <= kdg, dist, cid, k, nkd, nki);
                if (lane < k) {
                    sd[lane] = tk.d[0];
                    si[lane] = tk.id[0];
                }
                if (qj == gs) kdl = nkd;
                if (nkd < kdg && lane == 0) atomicMin(&s_thr[gs], ord_enc(nkd));
            }
        }
    };
    stream_blocks<kBoundPipe>(a.arena + b0 * d4 * 64 + lane, a.ids + b0 * 64 + lane, d4, nb, compute, finish);
    if (a.mstats && lane == 0) atomicAdd(&a.mstats[1], (unsigned long long)nb);
    // the segment's k-th distances lower the list-wide thresholds for later items
    if (lane < np && kdl < __builtin_inff()) atomicMin(&a.thr[it.pair_start + lane], ord_enc(kdl));
    for (int g = 0; g < np; ++g) {
        const uint32_t part = a.part_base_sorted[it.pair_start + g] + seg;
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = tk_d[g * k + lane];
            a.part_i[(size_t)part * k + lane] = tk_i[g * k + lane];
        }
    }
}

// One wave-item of a narrow list (<= 4 pairs of one segment).
template <int R, int M, bool ROWS>
__device__ __forceinline__ void scan_narrow(const ScanArgs& a, const ScanItem it) {
    constexpr int GMAX = scan_group_max(R);
    switch (it.npairs) {
        case 1: scan_item<R, 1, M, ROWS>(a, it); break;
        case 2: if constexpr (GMAX >= 2) scan_item<R, 2, M, ROWS>(a, it); break;
        case 3: if constexpr (GMAX >= 3) scan_item<R, 3, M, ROWS>(a, it); break;
        case 4: if constexpr (GMAX >= 4) scan_item<R, 4, M, ROWS>(a, it); break;
        default: break;
    }
}

// ivf_scan_narrow: the fine scan (search_list_cpu, cpp:347-370) of the batch's small
// lists: each wave takes one narrow item (one segment x <= 4 queries, queries via
// scalar loads, top-k in registers).
template <int R, int M, bool ROWS>
// Persistent: a grid sized to the machine, each wave pulling items from a queue
// (one device-scope atomic per item) until the batch's items run out.
__global__ __launch_bounds__(256) void ivf_scan_narrow(ScanArgs a) {
    const uint32_t n_narrow = a.counters[0];
    for (;;) {
        uint32_t idx = 0;
        if (lane_id() == 0) idx = atomicAdd(&a.work[0], 1u);
        idx = __builtin_amdgcn_readfirstlane(idx);
        if (idx >= n_narrow) break;
        scan_narrow<R, M, ROWS>(a, a.items[idx]);
    }
}

// Narrow items pulled by one wave until the queue is empty (the fused wide scan).
// (Inlined at both call sites: a real call would spill the wide path's registers.)
template <int M, bool ROWS>
__device__ __forceinline__ void drain_narrow(const ScanArgs& a) {
    const uint32_t n_narrow = a.counters[0];
    for (;;) {
        uint32_t idx = 0;
        if (lane_id() == 0) idx = atomicAdd(&a.work[0], 1u);
        idx = __builtin_amdgcn_readfirstlane(idx);
        if (idx >= n_narrow) break;
        scan_narrow<1, M, ROWS>(a, a.items[idx]);
    }
}

// ivf_scan_wide: the large lists. A workgroup takes one wide item at a time: a range of
// a list's segments x up to 4W of the list's queries, staged once in LDS as pairs.
//  * W = 4: two 4-wave workgroups per CU, items of up to 16 queries; the 4 waves take the
//    item's segments dynamically, each against all of the item's queries.
//  * W = 8: one 8-wave workgroup per CU, items of up to 32 queries, so a list probed by
//    17-32 queries of the batch is streamed from HBM once instead of twice. Up to 16
//    queries the 8 waves share the segments as above. Beyond 16 the waves split into
//    two halves of 4, each half taking the item's segments in the same order against
//    its half of the queries: the two waves streaming one segment run side by side on
//    the CU, so the second read is served on-chip, and every wave keeps at most 8 query
//    pairs in registers (the code path that does not spill).
template <int M, int W, bool ROWS>
__global__ __launch_bounds__(64 * W, 2 * 4 / W) void ivf_scan_wide(ScanArgs a) {
    constexpr int GW = 4 * W;  // queries per item at most
    // Dynamic LDS: [d4][gpv][2] float4 of staged query pairs (tile-major), then per wave
    // kWaveQueries x k top-k ids (u64), then the same for distances (f32).
    extern __shared__ __attribute__((aligned(16))) float4 qlds[];
    const uint32_t d4 = a.d4;
    const uint32_t wv = wave_index();
    uint64_t* tk_i = (uint64_t*)(qlds + (size_t)(GW / 2) * d4 * 2) + (size_t)wv * kWaveQueries * a.k;
    float* tk_d = (float*)((uint64_t*)(qlds + (size_t)(GW / 2) * d4 * 2) + (size_t)W * kWaveQueries * a.k) +
                  (size_t)wv * kWaveQueries * a.k;
    const uint32_t n_wide = a.counters[3];
    // Items of one list are adjacent in the plan; dispatching them in a strided order
    // mixes lists of many queries (VALU-heavy) with lists of few (HBM-heavy) on the
    // CUs at every moment. The stride is a prime that does not divide n_wide, so the
    // map is a permutation.
    uint32_t stride = a.wide_stride;
    if (stride > 1 && n_wide % stride == 0) stride = stride == 40009u ? 40013u : 40009u;
    // Fused launch: narrow items (HBM-bound) run beside the wide ones (often VALU-bound)
    // inside this one persistent grid, no second stream: the last a.fused workgroups
    // start on the narrow queue, and every wave drains it once the wide queue is empty.
    if (a.fused && blockIdx.x + a.fused >= gridDim.x) drain_narrow<M, ROWS>(a);
    __shared__ uint32_t s_next;
    __shared__ uint32_t s_seg[2];   // next segment of the current item (per query half)
    __shared__ uint32_t s_thr[GW];  // per query of the item: the best k-th distance reached
    for (;;) {
        // persistent workgroups pull items from a queue (one atomic per item)
        if (threadIdx.x == 0) s_next = atomicAdd(&a.work[1], 1u);
        __syncthreads();
        const uint32_t b = s_next;
        if (b >= n_wide) break;
        const uint32_t item = stride > 1 ? (uint32_t)(((uint64_t)b * stride) % n_wide) : b;
        ScanItem it = a.items_w[item];
        it.list = __builtin_amdgcn_readfirstlane(it.list);  // (wave-uniform: scalar address math)
        it.seg = __builtin_amdgcn_readfirstlane(it.seg);
        it.pair_start = __builtin_amdgcn_readfirstlane(it.pair_start);
        it.npairs = __builtin_amdgcn_readfirstlane(it.npairs);
        const int np = min((int)it.npairs, GW);  // (s_thr and the staged pairs hold GW queries: the plan's bound)
        const int gp = (np + 1) / 2;
        if (threadIdx.x < 2) s_seg[threadIdx.x] = 0;  // visible after the staging barrier below
        if (threadIdx.x < (uint32_t)np) s_thr[threadIdx.x] = a.thr[it.pair_start + threadIdx.x];
        const int gpv = (VDB_SCAN_DIAG & 2) ? 1 : gp;  // (DIAGNOSTIC diag&2: one pair only, results invalid)
        for (uint32_t e = threadIdx.x; e < (uint32_t)gpv * d4; e += blockDim.x) {
            const uint32_t t = e / gpv, p = e - t * gpv;
            const int ga = min((int)(2 * p), np - 1), gb = min((int)(2 * p + 1), np - 1);
            const float4 qa = ((const float4*)(a.qpad + (size_t)(a.sorted_pair[it.pair_start + ga] >> 16) * d4 * 4))[t];
            const float4 qb = ((const float4*)(a.qpad + (size_t)(a.sorted_pair[it.pair_start + gb] >> 16) * d4 * 4))[t];
            qlds[(t * gpv + p) * 2 + 0] = make_float4(qa.x, qb.x, qa.y, qb.y);
            qlds[(t * gpv + p) * 2 + 1] = make_float4(qa.z, qb.z, qa.w, qb.w);
        }
        __syncthreads();
        // This wave's queries: all of the item's (one group), or its half's (W = 8, more
        // than 8 pairs). Pairs [p0, p0 + gw) are queries 2 p0 .. 2 p0 + nq - 1.
        const bool split = W == 8 && gpv > 8;
        const uint32_t half = split ? wv >> 2 : 0u;
        const int gh = (gpv + 1) / 2;
        const int p0 = split ? (int)half * gh : 0;
        const int gw = split ? (half ? gpv - gh : gh) : gpv;
        const int q0 = 2 * p0;
        const int nq = split ? (half ? np - q0 : min(np, 2 * gh)) : ((VDB_SCAN_DIAG & 2) ? min(np, 2) : np);
        const float4* qw = qlds + (size_t)p0 * 2;
        // the item's segments [seg0, seg1) go to the waves (of each half) dynamically: a
        // wave that finishes early takes the next one, so waves idle only at the item's end
        const uint32_t seg_vectors = a.seg_blocks * 64;
        const uint32_t nseg = (a.count[it.list] + seg_vectors - 1) / seg_vectors;
        const uint32_t seg0 = it.seg * a.segs_item, seg1 = min(nseg, seg0 + a.segs_item);
        for (;;) {
            uint32_t sg = 0;
            if (lane_id() == 0) sg = atomicAdd(&s_seg[half], 1u);
            sg = seg0 + __builtin_amdgcn_readfirstlane(sg);
            if (sg >= seg1) break;
#define VDB_WW(GPN)                                                                       \
    case GPN:                                                                             \
        if (W == 8 && split) scan_wide_wave<GPN, M, true, false, ROWS>(a, it, qw, gpv, q0, nq, tk_d, tk_i, s_thr + q0, sg); \
        else if (kOddPairs && (nq & 1)) scan_wide_wave<GPN, M, false, true, ROWS>(a, it, qw, gpv, q0, nq, tk_d, tk_i, s_thr + q0, sg);  \
        else scan_wide_wave<GPN, M, false, false, ROWS>(a, it, qw, gpv, q0, nq, tk_d, tk_i, s_thr + q0, sg);            \
        break;
            switch (gw) {
                VDB_WW(1) VDB_WW(2) VDB_WW(3) VDB_WW(4) VDB_WW(5) VDB_WW(6) VDB_WW(7)
                default:
                    if (W == 8 && split) scan_wide_wave<8, M, true, false, ROWS>(a, it, qw, gpv, q0, nq, tk_d, tk_i, s_thr + q0, sg);
                    else if (kOddPairs && (nq & 1)) scan_wide_wave<8, M, false, true, ROWS>(a, it, qw, gpv, q0, nq, tk_d, tk_i, s_thr + q0, sg);
                    else scan_wide_wave<8, M, false, false, ROWS>(a, it, qw, gpv, q0, nq, tk_d, tk_i, s_thr + q0, sg);
                    break;
            }
#undef VDB_WW
        }
        __syncthreads();  // qlds is restaged by the next wide item
    }
    if (a.fused) drain_narrow<M, ROWS>(a);
}

// ivf_scan_bounded: the wide items of >= a.mfma_min queries (items_w[counters[3] ..
// counters[3] + counters[7])), one 4-wave workgroup per item at a time as in
// ivf_scan_wide, every wave a bounded wave (scan_wide_wave_mfma). Its own kernel: the
// bounded waves' registers inlined beside the exact waves' would spill both.
// Dynamic LDS: [d4][16] float4 of staged queries (row-major), then per wave
// kWaveQueries x k top-k ids (u64), then distances (f32).
template <int M>
__global__ __launch_bounds__(256, 2) void ivf_scan_bounded(ScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) float4 qlds[];
    const uint32_t d4 = a.d4;
    const uint32_t wv = wave_index();
    uint64_t* tk_i = (uint64_t*)(qlds + (size_t)16 * d4) + (size_t)wv * kWaveQueries * a.k;
    float* tk_d = (float*)((uint64_t*)(qlds + (size_t)16 * d4) + (size_t)4 * kWaveQueries * a.k) +
                  (size_t)wv * kWaveQueries * a.k;
    const uint32_t first = a.counters[3], n_bounded = a.counters[7];
    __shared__ uint32_t s_next;
    __shared__ uint32_t s_seg;
    __shared__ uint32_t s_thr[16];
    __shared__ uint16_t s_cand[4][1024];  // per wave: (vector << 4 | query) of one block's candidates
    for (;;) {
        if (threadIdx.x == 0) s_next = atomicAdd(&a.work[2], 1u);
        __syncthreads();
        const uint32_t b = s_next;
        if (b >= n_bounded) break;
        ScanItem it = a.items_w[first + b];
        it.list = __builtin_amdgcn_readfirstlane(it.list);
        it.seg = __builtin_amdgcn_readfirstlane(it.seg);
        it.pair_start = __builtin_amdgcn_readfirstlane(it.pair_start);
        it.npairs = __builtin_amdgcn_readfirstlane(it.npairs);
        const int np = min((int)it.npairs, 16);  // <= 16 (wide group 16; s_thr and s_cand hold 16)
        if (threadIdx.x == 0) s_seg = 0;
        if (threadIdx.x < (uint32_t)np) s_thr[threadIdx.x] = a.thr[it.pair_start + threadIdx.x];
        for (uint32_t e = threadIdx.x; e < 16 * d4; e += blockDim.x) {
            const uint32_t t = e >> 4, jq = e & 15;
            qlds[e] = jq < (uint32_t)np
                          ? ((const float4*)(a.qpad + (size_t)(a.sorted_pair[it.pair_start + jq] >> 16) * d4 * 4))[t]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
        const uint32_t seg_vectors = a.seg_blocks * 64;
        const uint32_t nseg = (a.count[it.list] + seg_vectors - 1) / seg_vectors;
        const uint32_t seg0 = it.seg * a.segs_item, seg1 = min(nseg, seg0 + a.segs_item);
        for (;;) {
            uint32_t sg = 0;
            if (lane_id() == 0) sg = atomicAdd(&s_seg, 1u);
            sg = seg0 + __builtin_amdgcn_readfirstlane(sg);
            if (sg >= seg1) break;
            scan_wide_wave_mfma<M>(a, it, qlds, np, tk_d, tk_i, s_thr, s_cand[wv], sg);
        }
        __syncthreads();  // qlds is restaged by the next item
    }
}

// Offer n contiguous (dist, id) entries to a wave top-k: 64 x kPre entries per round,
// every load of a round issued before the first offer (the offers are dependent
// wave-wide steps; a load between them would expose its latency each time).
// UNIQUE: merge_results semantics (cpp:481-504) — UINT64_MAX ids are not results and
// each id is kept once at its smallest (dist, id).
template <int R, bool UNIQUE>
__device__ __forceinline__ void offer_array(WaveTopK<R>& tk, const float* __restrict__ d,
                                            const uint64_t* __restrict__ id, uint32_t n, int k, float& kd,
                                            uint64_t& ki) {
    constexpr int kPre = 8;
    const int lane = lane_id();
    for (uint32_t r0 = 0; r0 < n; r0 += 64 * kPre) {
        float dv[kPre];
        uint64_t iv[kPre];
#pragma unroll
        for (int j = 0; j < kPre; ++j) {
            const uint32_t e = r0 + j * 64 + lane;
            const bool v = e < n;
            dv[j] = v ? d[e] : __builtin_inff();
            iv[j] = v ? id[e] : kNoId;
        }
#pragma unroll
        for (int j = 0; j < kPre; ++j) {
            const bool v = r0 + j * 64 + lane < n;
            if constexpr (UNIQUE) {
                uint64_t mask = __ballot(v && iv[j] != kNoId && dv[j] <= kd);
                while (mask) {
                    const int l = __ffsll((long long)mask) - 1;
                    mask &= mask - 1;
                    tk.offer_unique(rd_lane(dv[j], l), rd_lane(iv[j], l), k, kd, ki);
                }
            } else {
                offer_lanes<R>(tk, v && dv[j] <= kd, dv[j], iv[j], k, kd, ki);
            }
        }
    }
}

// ============================================================================
// Level-1 partial merge: one wave folds <= kMergeFan segment partials of one
// (query, probe) pair into one (multiset top-min(k, n_l), cpp:368-377), so a list
// of millions of vectors is never merged by a single wave.
// ============================================================================
template <int R>
__device__ __forceinline__ void merge_partial_item(const uint32_t* __restrict__ probes,
                                                   const uint32_t* __restrict__ count_global,
                                                   const uint32_t* __restrict__ nseg_qp,
                                                   const uint32_t* __restrict__ part_base_qp,
                                                   const uint32_t* __restrict__ l1base_qp, const uint2 w,
                                                   const float* __restrict__ part_d,
                                                   const uint64_t* __restrict__ part_i, uint32_t k,
                                                   float* __restrict__ l1_d, uint64_t* __restrict__ l1_i);

template <int R>
__global__ __launch_bounds__(256) void ivf_merge_partials(const uint32_t* __restrict__ probes,
                                                          const uint32_t* __restrict__ count_global,
                                                          const uint32_t* __restrict__ nseg_qp,
                                                          const uint32_t* __restrict__ part_base_qp,
                                                          const uint32_t* __restrict__ l1base_qp,
                                                          const uint2* __restrict__ l1_items,
                                                          const uint32_t* __restrict__ counters,
                                                          const float* __restrict__ part_d,
                                                          const uint64_t* __restrict__ part_i, uint32_t k,
                                                          float* __restrict__ l1_d, uint64_t* __restrict__ l1_i) {
    const uint32_t n_items = counters[2];
    for (uint32_t idx = blockIdx.x * 4 + wave_index(); idx < n_items; idx += gridDim.x * 4)
        merge_partial_item<R>(probes, count_global, nseg_qp, part_base_qp, l1base_qp, l1_items[idx], part_d, part_i, k,
                              l1_d, l1_i);
}

template <int R>
__device__ __forceinline__ void merge_partial_item(const uint32_t* __restrict__ probes,
                                                   const uint32_t* __restrict__ count_global,
                                                   const uint32_t* __restrict__ nseg_qp,
                                                   const uint32_t* __restrict__ part_base_qp,
                                                   const uint32_t* __restrict__ l1base_qp, const uint2 w,
                                                   const float* __restrict__ part_d,
                                                   const uint64_t* __restrict__ part_i, uint32_t k,
                                                   float* __restrict__ l1_d, uint64_t* __restrict__ l1_i) {
    const uint32_t i = w.x, j = w.y;
    const int lane = lane_id();
    const uint32_t ns = nseg_qp[i];
    const uint32_t cnt = min((uint32_t)kMergeFan, ns - j * kMergeFan);
    const size_t base = ((size_t)part_base_qp[i] + (size_t)j * kMergeFan) * k;
    const int kk = (int)min(k, count_global[probes[i]]);
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    offer_array<R, false>(tk, part_d + base, part_i + base, cnt * k, kk, kd, ki);
    float* od = l1_d + ((size_t)l1base_qp[i] + j) * k;
    uint64_t* oi = l1_i + ((size_t)l1base_qp[i] + j) * k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < (int)k) {
            od[e] = e < kk ? tk.d[r] : __builtin_inff();
            oi[e] = e < kk ? tk.id[r] : kNoId;
        }
    }
}

// ============================================================================
// Per (query, probe) pair: top-min(k, n_l) of the list's segment partials, as
// search_list_cpu's partial_sort yields for the whole list (cpp:368-377).
// ============================================================================
template <int R>
__global__ __launch_bounds__(256) void ivf_merge_slots(const uint32_t* __restrict__ probes,
                                                       const uint32_t* __restrict__ count_global,
                                                       const uint32_t* __restrict__ nseg_qp,
                                                       const uint32_t* __restrict__ part_base_qp,
                                                       const uint32_t* __restrict__ l1base_qp,
                                                       const float* __restrict__ part_d,
                                                       const uint64_t* __restrict__ part_i,
                                                       const float* __restrict__ l1_d,
                                                       const uint64_t* __restrict__ l1_i, uint32_t BP, uint32_t k,
                                                       float* __restrict__ slot_d, uint64_t* __restrict__ slot_i) {
    const uint32_t i = blockIdx.x * 4 + wave_index();
    if (i >= BP) return;
    const int lane = lane_id();
    const uint32_t ns = nseg_qp[i];
    float* od = slot_d + (size_t)i * k;
    uint64_t* oi = slot_i + (size_t)i * k;
    if (ns == 0) {
        for (uint32_t e = lane; e < k; e += 64) {
            od[e] = __builtin_inff();
            oi[e] = kNoId;
        }
        return;
    }
    const float* sd;
    const uint64_t* si;
    uint32_t nin;
    if (ns <= (uint32_t)kMergeFan) {
        sd = part_d + (size_t)part_base_qp[i] * k;
        si = part_i + (size_t)part_base_qp[i] * k;
        nin = ns;
    } else {
        sd = l1_d + (size_t)l1base_qp[i] * k;
        si = l1_i + (size_t)l1base_qp[i] * k;
        nin = (ns + kMergeFan - 1) / kMergeFan;
    }
    if (nin == 1) {
        for (uint32_t e = lane; e < k; e += 64) {
            od[e] = sd[e];
            oi[e] = si[e];
        }
        return;
    }
    const int kk = (int)min(k, count_global[probes[i]]);
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    offer_array<R, false>(tk, sd, si, nin * k, kk, kd, ki);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < (int)k) {
            od[e] = e < kk ? tk.d[r] : __builtin_inff();
            oi[e] = e < kk ? tk.id[r] : kNoId;
        }
    }
}

// Offer k slot entries to a de-duplicating list (merge_results, cpp:481-504):
// ids == UINT64_MAX are not results (cpp:486).
template <int R>
__device__ __forceinline__ void offer_slot_unique(WaveTopK<R>& tk, const float* sd, const uint64_t* si,
                                                  uint32_t k, float& kd, uint64_t& ki) {
    const int lane = lane_id();
    for (uint32_t c0 = 0; c0 < k; c0 += 64) {
        const uint32_t c = c0 + lane;
        const bool valid = c < k;
        const float d = valid ? sd[c] : __builtin_inff();
        const uint64_t id = valid ? si[c] : kNoId;
        uint64_t mask = __ballot(valid && id != kNoId && d <= kd);
        while (mask) {
            const int l = __ffsll((long long)mask) - 1;
            mask &= mask - 1;
            tk.offer_unique(rd_lane(d, l), rd_lane(id, l), (int)k, kd, ki);
        }
    }
}

template <int R>
__device__ __forceinline__ void write_final(const WaveTopK<R>& tk, uint32_t k, float* od, uint64_t* oi) {
    const int lane = lane_id();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < (int)k) {
            const bool real = tk.id[r] != kNoId;
            od[e] = real ? tk.d[r] : FLT_MAX;  // padding as cpp:513-517
            oi[e] = tk.id[r];
        }
    }
}

// ============================================================================
// Per query: merge the P slots (with the reference's stale-slot reuse for empty
// lists, cpp:210-233) into the unique-id top-k.
// ============================================================================
template <int R>
__global__ __launch_bounds__(256) void ivf_merge_query(const uint32_t* __restrict__ probes,
                                                     const uint32_t* __restrict__ count_global,
                                                     const float* __restrict__ slot_d,
                                                     const uint64_t* __restrict__ slot_i,
                                                     const float* __restrict__ carry_d,
                                                     const uint64_t* __restrict__ carry_i, uint32_t B, uint32_t P,
                                                     uint32_t k, int stale, const uint32_t* __restrict__ req_start,
                                                     uint32_t b0, float* __restrict__ out_d,
                                                     uint64_t* __restrict__ out_i) {
    const uint32_t q = blockIdx.x * 4 + wave_index();
    if (q >= B) return;
    // Coalesced calls: slots live per reference search() call (cpp:210-211), so a
    // stale-slot lookup never crosses into another request (req_start: first query of
    // this query's request, call-global; null = one request).
    const uint32_t qs = req_start ? req_start[b0 + q] : 0u;
    const uint32_t q_lo = qs > b0 ? qs - b0 : 0u;  // lowest in-batch query of the request
    const bool carry_ok = qs < b0 || b0 == 0;       // the carry is this request's (or the call's fresh one)
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    bool any_empty = false;
    for (uint32_t p0 = 0; p0 < P; p0 += 64) {
        const uint32_t p = p0 + lane_id();
        any_empty |= __ballot(p < P && count_global[probes[(size_t)q * P + p]] == 0) != 0;
    }
    if (!any_empty) {  // every probed list non-empty: the query's P slots are contiguous
        offer_array<R, true>(tk, slot_d + (size_t)q * P * k, slot_i + (size_t)q * P * k, P * k, (int)k, kd, ki);
        write_final<R>(tk, k, out_d + (size_t)q * k, out_i + (size_t)q * k);
        return;
    }
    for (uint32_t p = 0; p < P; ++p) {
        const float* sd = nullptr;
        const uint64_t* si = nullptr;
        if (count_global[probes[(size_t)q * P + p]] > 0) {
            sd = slot_d + ((size_t)q * P + p) * k;
            si = slot_i + ((size_t)q * P + p) * k;
        } else if (stale) {
            uint32_t q2 = q;
            bool found = false;
            while (q2 > q_lo) {
                --q2;
                if (count_global[probes[(size_t)q2 * P + p]] > 0) {
                    found = true;
                    break;
                }
            }
            if (found) {
                sd = slot_d + ((size_t)q2 * P + p) * k;
                si = slot_i + ((size_t)q2 * P + p) * k;
            } else if (carry_ok) {
                sd = carry_d + (size_t)p * k;
                si = carry_i + (size_t)p * k;
            }  // else: the request's slot p is still empty
        }
        if (sd) offer_slot_unique<R>(tk, sd, si, k, kd, ki);
    }
    write_final<R>(tk, k, out_d + (size_t)q * k, out_i + (size_t)q * k);
}

// Slot content that survives into the next batch of the same search call.
// The carry belongs to the request of the batch's last query: only that request's
// queries are searched; if that request began in this batch and never filled slot p,
// the carried slot is empty.
__global__ void ivf_carry_slots(const uint32_t* __restrict__ probes, const uint32_t* __restrict__ count_global,
                        uint32_t B, uint32_t P, uint32_t k, const float* __restrict__ slot_d,
                        const uint64_t* __restrict__ slot_i, const uint32_t* __restrict__ req_start, uint32_t b0,
                        float* __restrict__ carry_d, uint64_t* __restrict__ carry_i) {
    __shared__ int s_q;
    const uint32_t p = blockIdx.x;
    const uint32_t qs = req_start ? req_start[b0 + B - 1] : 0u;
    const int q_lo = qs > b0 ? (int)(qs - b0) : 0;
    if (threadIdx.x == 0) {
        int found = -1;
        for (int q = (int)B - 1; q >= q_lo; --q)
            if (count_global[probes[(size_t)q * P + p]] > 0) {
                found = q;
                break;
            }
        s_q = found;
    }
    __syncthreads();
    if (s_q < 0) {
        if (qs >= b0)  // a request that began in this batch: its slot p is empty
            for (uint32_t e = threadIdx.x; e < k; e += blockDim.x) carry_i[(size_t)p * k + e] = kNoId;
        return;
    }
    const size_t src = ((size_t)s_q * P + p) * k;
    for (uint32_t e = threadIdx.x; e < k; e += blockDim.x) {
        carry_d[(size_t)p * k + e] = slot_d[src + e];
        carry_i[(size_t)p * k + e] = slot_i[src + e];
    }
}

// Final combine of per-rank partials [nranks][n][k] (list-sharded multi-GPU).
template <int R>
// Rank r's partials sit at d + r * d_stride and ids + r * i_stride (elements), each
// [n][k]: back to back ([nranks][n][k]) or interleaved per rank in one packed record.
__global__ __launch_bounds__(256) void ivf_merge_ranks(const float* __restrict__ d, const uint64_t* __restrict__ ids,
                                                    uint64_t d_stride, uint64_t i_stride, uint32_t nranks,
                                                    uint32_t n, uint32_t k, float* __restrict__ out_d,
                                                    uint64_t* __restrict__ out_i) {
    chain_prio();
    const uint32_t q = blockIdx.x * 4 + wave_index();
    if (q >= n) return;
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    for (uint32_t r = 0; r < nranks; ++r)
        offer_slot_unique<R>(tk, d + r * d_stride + (size_t)q * k, ids + r * i_stride + (size_t)q * k, k, kd, ki);
    write_final<R>(tk, k, out_d + (size_t)q * k, out_i + (size_t)q * k);
}

// ============================================================================
// Fused batch merge (one workgroup of min(16, P) waves per query): the work of ivf_merge_partials,
// ivf_merge_slots, ivf_merge_query and ivf_carry_slots in ONE launch.
//  1. Each wave takes probes p = wave, wave + waves, ... and writes the query's EFFECTIVE
//     slot p into slot_d/i[q][p]: its own list's top-min(k, n_l) folded from all the
//     segment partials of that (query, probe) pair (search_list_cpu's partial_sort,
//     cpp:368-377), or, for an empty probed list (quirk A1, cpp:210-233), the same fold
//     for the nearest earlier query of its request whose probe p is non-empty —
//     recomputed from that pair's partials, the same bits that query's slot holds —
//     else the call's carried slot, else nothing.
//  2. After the workgroup barrier, wave 0 merges the P slots into the unique-id top-k
//     (merge_results, cpp:474-518).
//  3. The batch's last query's workgroup writes its effective slots — the last content
//     of every slot — as the carry of the call's next batch, into the other carry buffer
//     (ping-pong: other workgroups of this batch may still read the current one).
// ============================================================================
template <int R>
__device__ __forceinline__ void fold_pair_slot(uint32_t i, const uint32_t* __restrict__ probes,
                                               const uint32_t* __restrict__ count_global,
                                               const uint32_t* __restrict__ nseg_qp,
                                               const uint32_t* __restrict__ part_base_qp,
                                               const float* __restrict__ part_d, const uint64_t* __restrict__ part_i,
                                               uint32_t k, float* __restrict__ od, uint64_t* __restrict__ oi) {
    const int lane = lane_id();
    const uint32_t ns = nseg_qp[i];
    const size_t base = (size_t)part_base_qp[i] * k;
    if (ns <= 1) {  // not stored here (or empty): nothing; one segment: its partial is the list's top-k
        for (uint32_t e = lane; e < k; e += 64) {
            od[e] = ns ? part_d[base + e] : __builtin_inff();
            oi[e] = ns ? part_i[base + e] : kNoId;
        }
        return;
    }
    const int kk = (int)min(k, count_global[probes[i]]);
    WaveTopK<R> tk;
    tk.init();
    float kd = __builtin_inff();
    uint64_t ki = kNoId;
    offer_array<R, false>(tk, part_d + base, part_i + base, ns * k, kk, kd, ki);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < (int)k) {
            od[e] = e < kk ? tk.d[r] : __builtin_inff();
            oi[e] = e < kk ? tk.id[r] : kNoId;
        }
    }
}

template <int R>
__global__ __launch_bounds__(1024) void ivf_merge_fused(const uint32_t* __restrict__ probes,
                                                     const uint32_t* __restrict__ count_global,
                                                     const uint32_t* __restrict__ nseg_qp,
                                                     const uint32_t* __restrict__ part_base_qp,
                                                     const float* __restrict__ part_d,
                                                     const uint64_t* __restrict__ part_i, uint32_t B, uint32_t P,
                                                     uint32_t k, int stale, const uint32_t* __restrict__ req_start,
                                                     uint32_t b0, const float* __restrict__ carry_d,
                                                     const uint64_t* __restrict__ carry_i, float* __restrict__ slot_d,
                                                     uint64_t* __restrict__ slot_i, float* __restrict__ carry_nd,
                                                     uint64_t* __restrict__ carry_ni, float* __restrict__ out_d,
                                                     uint64_t* __restrict__ out_i) {
    chain_prio();
    const uint32_t q = blockIdx.x;
    const uint32_t wv = wave_index();
    const int lane = lane_id();
    // the query's request (coalesced calls; null = one request): stale lookups never cross it
    const uint32_t qs = req_start ? req_start[b0 + q] : 0u;
    const uint32_t q_lo = qs > b0 ? qs - b0 : 0u;
    const bool carry_ok = qs < b0 || b0 == 0;
    const uint32_t nwaves = blockDim.x >> 6;  // (up to 16: a query's slots fold in parallel)
    for (uint32_t p = wv; p < P; p += nwaves) {
        float* od = slot_d + ((size_t)q * P + p) * k;
        uint64_t* oi = slot_i + ((size_t)q * P + p) * k;
        uint32_t src = q;
        bool have = count_global[probes[(size_t)q * P + p]] > 0;
        if (!have && stale) {
            for (uint32_t q2 = q; q2 > q_lo;) {
                --q2;
                if (count_global[probes[(size_t)q2 * P + p]] > 0) {
                    src = q2;
                    have = true;
                    break;
                }
            }
        }
        if (have) {
            fold_pair_slot<R>(src * P + p, probes, count_global, nseg_qp, part_base_qp, part_d, part_i, k, od, oi);
        } else {
            const bool from_carry = stale && carry_ok;
            for (uint32_t e = lane; e < k; e += 64) {
                od[e] = from_carry ? carry_d[(size_t)p * k + e] : __builtin_inff();
                oi[e] = from_carry ? carry_i[(size_t)p * k + e] : kNoId;
            }
        }
    }
    __threadfence_block();
    __syncthreads();
    if (wv == 0) {
        WaveTopK<R> tk;
        tk.init();
        float kd = __builtin_inff();
        uint64_t ki = kNoId;
        offer_array<R, true>(tk, slot_d + (size_t)q * P * k, slot_i + (size_t)q * P * k, P * k, (int)k, kd, ki);
        write_final<R>(tk, k, out_d + (size_t)q * k, out_i + (size_t)q * k);
    }
    if (stale && q + 1 == B) {  // the carry of the call's next batch
        for (uint32_t e = threadIdx.x; e < P * k; e += blockDim.x) {
            carry_nd[e] = slot_d[(size_t)q * P * k + e];
            carry_ni[e] = slot_i[(size_t)q * P * k + e];
        }
    }
}

__global__ void ivf_fill_empty(uint64_t n, float* __restrict__ d, uint64_t* __restrict__ i) {
    for (uint64_t e = gtid(); e < n; e += gstride()) {
        d[e] = FLT_MAX;
        i[e] = kNoId;
    }
}

// ============================================================================
// Build-side kernels: layout, assignment (assign_to_lists, cpp:259-295),
// k-means++ seeding and Lloyd update (train, cpp:49-145).
// ============================================================================
// rows [n][dp] -> interleaved blocks [ceil(n/64)][d4][64] float4 (tail lanes zero).
__global__ void ivf_interleave_rows(const float* __restrict__ rows, uint64_t n, uint32_t d4, float4* __restrict__ out) {
    const uint64_t nb = (n + 63) / 64;
    for (uint64_t e = gtid(); e < nb * d4 * 64; e += gstride()) {  // (block, t, lane)
        const uint32_t lane = e & 63;
        const uint64_t bt = e >> 6;
        const uint64_t b = bt / d4;
        const uint32_t t = (uint32_t)(bt - b * d4);
        const uint64_t r = b * 64 + lane;
        out[e] = r < n ? ((const float4*)(rows + r * (uint64_t)d4 * 4))[t] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__global__ void ivf_scatter_rows(const float* __restrict__ rows, const uint64_t* __restrict__ row_ids,
                               const uint32_t* __restrict__ order, uint64_t n, uint32_t d4,
                               const uint64_t* __restrict__ dest_slot, float4* __restrict__ arena,
                               uint64_t* __restrict__ arena_ids) {
    for (uint64_t e = gtid(); e < n * d4; e += gstride()) {  // (j, t)
        const uint64_t j = e / d4;
        const uint32_t t = (uint32_t)(e - j * d4);
        const uint64_t slot = dest_slot[j];
        if (slot == ~0ull) continue;  // list stored on another shard
        const uint64_t row = order[j];
        arena[((slot >> 6) * d4 + t) * 64 + (slot & 63)] = ((const float4*)(rows + row * (uint64_t)d4 * 4))[t];
        if (t == 0) arena_ids[slot] = row_ids[row];
    }
}

// Move each list's first nblocks[l] blocks from old_off[l] to new_off[l].
__global__ void ivf_copy_lists(const float4* __restrict__ old_arena, const uint64_t* __restrict__ old_ids,
                             const uint64_t* __restrict__ old_off, const uint64_t* __restrict__ new_off,
                             const uint32_t* __restrict__ nblocks, uint32_t d4, float4* __restrict__ new_arena,
                             uint64_t* __restrict__ new_ids) {
    const uint32_t l = blockIdx.y;
    const uint64_t nvec4 = (uint64_t)nblocks[l] * d4 * 64;
    const float4* src = old_arena + old_off[l] * d4 * 64;
    float4* dst = new_arena + new_off[l] * d4 * 64;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nvec4; e += (uint64_t)gridDim.x * blockDim.x)
        dst[e] = src[e];
    const uint64_t nid = (uint64_t)nblocks[l] * 64;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nid; e += (uint64_t)gridDim.x * blockDim.x)
        new_ids[new_off[l] * 64 + e] = old_ids[old_off[l] * 64 + e];
}

__global__ void ivf_export_list(const float4* __restrict__ arena, const uint64_t* __restrict__ ids,
                              uint64_t block_off, uint32_t count, uint32_t dim, uint32_t d4,
                              float* __restrict__ out, uint64_t* __restrict__ out_ids) {
    for (uint64_t e = gtid(); e < (uint64_t)count * dim; e += gstride()) {  // (v, d)
        const uint32_t v = (uint32_t)(e / dim), d = (uint32_t)(e - (uint64_t)v * dim);
        const float* blk = (const float*)(arena + ((block_off + (v >> 6)) * d4 + (d >> 2)) * 64 + (v & 63));
        out[e] = blk[d & 3];
        if (d == 0 && out_ids) out_ids[v] = ids[(block_off << 6) + v];
    }
}

template <int M, int G>
__device__ __forceinline__ void assign_group(const float* __restrict__ vpad, uint64_t n, uint32_t d4,
                                             const float4* __restrict__ cent, uint32_t nlist,
                                             uint32_t* __restrict__ out, uint64_t v0, int lane);

// Exact argmin over centroids with the reference's strict '<' (lowest index wins
// ties; a distance must beat FLT_MAX to count, else list 0). Lane = centroid,
// 8 row vectors per wave whose dims are wave-uniform.
template <int M>
__global__ __launch_bounds__(256) void ivf_assign(const float* __restrict__ vpad, uint64_t n, uint32_t d4,
                                                const float4* __restrict__ cent, uint32_t nlist,
                                                uint32_t* __restrict__ out) {
    constexpr int G = 8;
    const int lane = lane_id();
    for (uint64_t v0 = ((uint64_t)blockIdx.x * 4 + wave_index()) * G; v0 < n; v0 += (uint64_t)gridDim.x * 4 * G)
        assign_group<M, G>(vpad, n, d4, cent, nlist, out, v0, lane);
}

template <int M, int G>
__device__ __forceinline__ void assign_group(const float* __restrict__ vpad, uint64_t n, uint32_t d4,
                                             const float4* __restrict__ cent, uint32_t nlist,
                                             uint32_t* __restrict__ out, uint64_t v0, int lane) {
    const float4* q[G];
#pragma unroll
    for (int g = 0; g < G; ++g) q[g] = (const float4*)(vpad + min(v0 + g, n - 1) * (uint64_t)d4 * 4);
    float bd[G];
    uint32_t bc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        bd[g] = FLT_MAX;
        bc[g] = 0;
    }
    const uint32_t ncb = (nlist + 63) / 64;
    for (uint32_t cb = 0; cb < ncb; ++cb) {
        const float4* vb = cent + (size_t)cb * d4 * 64 + lane;
        float acc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = 0.0f;
#pragma unroll 4
        for (uint32_t t = 0; t < d4; ++t) {
            const float4 x = vb[(size_t)t * 64];
#pragma unroll
            for (int g = 0; g < G; ++g) acc[g] = acc4<M>(acc[g], q[g][t], x);
        }
        const uint32_t c = cb * 64 + lane;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float d = dist_finish<M>(acc[g]);
            if (c < nlist && d < bd[g]) {
                bd[g] = d;
                bc[g] = c;
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float d = bd[g];
        uint32_t c = bc[g];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float od = __shfl_xor(d, off);
            const uint32_t oc = (uint32_t)__shfl_xor((int)c, off);
            if (od < d || (od == d && oc < c)) {
                d = od;
                c = oc;
            }
        }
        if (lane == 0 && v0 + g < n) out[v0 + g] = c;
    }
}

__global__ void ivf_histogram(const uint32_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ counts) {
    for (uint64_t e = gtid(); e < n; e += gstride()) atomicAdd(&counts[keys[e]], 1u);
}

__global__ void ivf_fill_f32(float* __restrict__ p, uint64_t n, float v) {
    for (uint64_t e = gtid(); e < n; e += gstride()) p[e] = v;
}

// k-means++: min_dist[v] = std::min(min_dist[v], L2(v, newest centroid)) (cpp:68-84).
// Lane = training vector (interleaved copy); centroid dims are wave-uniform.
__global__ __launch_bounds__(256) void kmeanspp_mindist(const float4* __restrict__ v_il, uint64_t n, uint32_t d4,
                                                        const float* __restrict__ crow,
                                                        float* __restrict__ mind) {
    const int lane = lane_id();
    const float4* c4 = (const float4*)crow;
    for (uint64_t blk = (uint64_t)blockIdx.x * 4 + wave_index(); blk * 64 < n; blk += (uint64_t)gridDim.x * 4) {
        const float4* vb = v_il + blk * d4 * 64 + lane;
        float acc = 0.0f;
#pragma unroll 8
        for (uint32_t t = 0; t < d4; ++t) acc = acc4<kL2>(acc, vb[(size_t)t * 64], c4[t]);
        const uint64_t v = blk * 64 + lane;
        if (v < n) {
            const float m = mind[v];
            mind[v] = (acc < m) ? acc : m;  // std::min(m, acc)
        }
    }
}

// Lloyd update (cpp:122-141): per (cluster, dim), sum members in input order,
// then divide by the count; empty clusters keep their centroid.
__global__ void lloyd_update(const float* __restrict__ vpad, uint32_t dp, const uint32_t* __restrict__ order,
                                  const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ counts,
                                  uint32_t dim, float* __restrict__ cent) {
    const uint32_t c = blockIdx.y;
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t cnt = counts[c];
    if (d >= dim || cnt == 0) return;
    const uint32_t off = offsets[c];
    float s = 0.0f;
    for (uint32_t j = 0; j < cnt; ++j) s = s + vpad[(uint64_t)order[off + j] * dp + d];
    cent[(uint64_t)c * dp + d] = s / (float)cnt;
}

__global__ void ivf_iota(uint32_t* __restrict__ out, uint64_t n) {
    for (uint64_t e = gtid(); e < n; e += gstride()) out[e] = (uint32_t)e;
}

__global__ void ivf_slots_from_order(const uint32_t* __restrict__ sorted_keys, uint64_t n,
                                   const uint64_t* __restrict__ group_start,
                                   const uint64_t* __restrict__ base_slot, uint64_t* __restrict__ dest) {
    for (uint64_t j = gtid(); j < n; j += gstride()) {
        const uint32_t l = sorted_keys[j];
        dest[j] = base_slot[l] == ~0ull ? ~0ull : base_slot[l] + (j - group_start[l]);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Counter-based Box-Muller normal draws (synthetic benchmark data only).
__global__ void synth_gen_normal(float* __restrict__ out, uint64_t n, uint64_t seed, uint64_t offset) {
    const uint64_t sk = splitmix64(seed);
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t h = splitmix64(sk ^ (offset + i));
        const float u1 = ((float)(h >> 40) + 1.0f) * (1.0f / 16777216.0f);       // (0, 1]
        const float u2 = (float)(h & 0xFFFFFFull) * (1.0f / 16777216.0f);          // [0, 1)
        out[i] = sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
    }
}

// Gaussian mixture (synthetic clustered data): row r belongs to component
// splitmix(seed') ^ r mod ncomp, and x[r][d] = centers[comp][d] + sigma * N(0,1), the
// noise being element r * dim + d of the same counter-based stream as above.
__global__ void synth_gen_mixture(float* __restrict__ out, uint64_t rows, uint32_t dim,
                                  const float* __restrict__ centers, uint32_t ncomp, float sigma, uint64_t seed,
                                  uint64_t row0) {
    const uint64_t sk = splitmix64(seed);
    const uint64_t ck = splitmix64(seed ^ 0x6D69787475726531ull);
    for (uint64_t e = gtid(); e < rows * dim; e += gstride()) {
        const uint64_t r = e / dim;
        const uint32_t d = (uint32_t)(e - r * dim);
        const uint64_t gr = row0 + r;
        const uint32_t comp = (uint32_t)(splitmix64(ck ^ gr) % ncomp);
        const uint64_t h = splitmix64(sk ^ (gr * dim + d));
        const float u1 = ((float)(h >> 40) + 1.0f) * (1.0f / 16777216.0f);
        const float u2 = (float)(h & 0xFFFFFFull) * (1.0f / 16777216.0f);
        out[e] = centers[(uint64_t)comp * dim + d] + sigma * (sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2));
    }
}

// ============================================================================
// Launchers
// ============================================================================
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
// Blocks for an element-wise launch of n items: at most 2^20 blocks of 256 (2^28 work-items).
static inline uint32_t launch_grid(uint64_t n, uint32_t block = 256) {
    const uint64_t b = (n + block - 1) / block;
    return (uint32_t)(b < (1ull << 20) ? (b ? b : 1) : (1ull << 20));
}

void launch_pad_rows(const float* src, uint64_t n, uint32_t dim, uint32_t dp, float* dst, hipStream_t s) {
    if (!n) return;
    ivf_pad_queries<<<launch_grid(n * dp), 256, 0, s>>>(src, n, dim, dp, dst);
}

void launch_coarse(int metric, const float4* cent, uint32_t nlist, uint32_t d4, const float* qpad, uint32_t B,
                   float* cd, hipStream_t s) {
    dim3 grid(cdiv(nlist, 64), cdiv(B, 16));
    if (metric == kL2) ivf_coarse_distances<kL2><<<grid, 256, 0, s>>>(cent, nlist, d4, qpad, B, cd);
    else if (metric == kIP) ivf_coarse_distances<kIP><<<grid, 256, 0, s>>>(cent, nlist, d4, qpad, B, cd);
    else ivf_coarse_distances<kCos><<<grid, 256, 0, s>>>(cent, nlist, d4, qpad, B, cd);
}

void launch_select(int regs, const float* cd, uint32_t nlist, uint32_t B, uint32_t P, uint32_t* probes,
                   hipStream_t s) {
    const uint32_t g = cdiv(B, 4);
    switch (regs) {
        case 1: ivf_select_probes<1><<<g, 256, 0, s>>>(cd, nlist, B, P, probes); break;
        case 2: ivf_select_probes<2><<<g, 256, 0, s>>>(cd, nlist, B, P, probes); break;
        case 4: ivf_select_probes<4><<<g, 256, 0, s>>>(cd, nlist, B, P, probes); break;
        case 8: ivf_select_probes<8><<<g, 256, 0, s>>>(cd, nlist, B, P, probes); break;
        default: ivf_select_probes<16><<<g, 256, 0, s>>>(cd, nlist, B, P, probes); break;
    }
}

void launch_coarse_mfma(int metric, const float* cent_rm, uint32_t nlist, uint32_t dp, const float* qpad,
                        uint32_t B, float* approx, float* delta, hipStream_t s) {
    if (B >= kMfmaBlockedRows) {  // enough 32-row tiles to fill the chip: the register-blocked kernel
        dim3 g2(cdiv(cdiv(nlist, 32), 4), cdiv(B, 32));
        if (metric == kL2) ivf_coarse_mfma2x2<kL2><<<g2, 256, 0, s>>>(cent_rm, nlist, dp, qpad, B, approx, delta);
        else ivf_coarse_mfma2x2<kIP><<<g2, 256, 0, s>>>(cent_rm, nlist, dp, qpad, B, approx, delta);
        return;
    }
    dim3 grid(cdiv(cdiv(nlist, 16), 4), cdiv(B, 16));
    const bool g8 = (dp / 16) % 8 == 0;  // dp is a multiple of 64, so steps are a multiple of 4
    if (metric == kL2) {
        if (g8) ivf_coarse_mfma<kL2, 8><<<grid, 256, 0, s>>>(cent_rm, nlist, dp, qpad, B, approx, delta);
        else ivf_coarse_mfma<kL2, 4><<<grid, 256, 0, s>>>(cent_rm, nlist, dp, qpad, B, approx, delta);
    } else {
        if (g8) ivf_coarse_mfma<kIP, 8><<<grid, 256, 0, s>>>(cent_rm, nlist, dp, qpad, B, approx, delta);
        else ivf_coarse_mfma<kIP, 4><<<grid, 256, 0, s>>>(cent_rm, nlist, dp, qpad, B, approx, delta);
    }
}

// Static LDS of ivf_select_rerank<R>: the four partial top-P lists, tau, n, the
// chunk's candidate ids (plus slack).
static constexpr size_t rerank_static_lds(int regs) { return (size_t)4 * regs * 64 * 8 + 512; }

// (rerank_rows: how many candidate rows of dp dims would fit a 64 KB workgroup beside the query
// row; > 0 is the exact coarse path's feasibility test. Since round 6 the kernel stages only
// the query row: the candidates' rows are read from the table by their lanes.)
constexpr size_t kRerankLds = 64 * 1024;
uint32_t rerank_rows(uint32_t dp, int regs) {
    const size_t fixed = (size_t)dp * 4 + rerank_static_lds(regs);
    const size_t row = ((size_t)dp + 4) * 4;
    const size_t budget = std::max(kRerankLds, fixed + 4 * row);  // (wide rows: at least 4 per chunk)
    if (fixed + row > kLdsBytes) return 0;
    return (uint32_t)std::min<size_t>(64, (std::min(budget, kLdsBytes) - fixed) / row);
}

void launch_select_rerank(int metric, int regs, const float* approx, const float* delta, const float* cent_rm,
                          uint32_t nlist, uint32_t dp, const float* qpad, uint32_t B, uint32_t P, uint32_t* cand,
                          uint32_t* probes, hipStream_t s) {
    const uint32_t ch = rerank_rows(dp, regs);
    // (the kernel's fixed LDS: s_top_* of 4 regs x 64 entries hold the partial top-P lists;
    // ch > 0: the query row fits beside them)
    if (P > 64u * (uint32_t)regs || ch == 0 || ch > 64)
        throw std::length_error("launch_select_rerank: nprobe above the top-P registers or no LDS chunk");
    const size_t lds = (size_t)dp / 4 * sizeof(float4);  // (the query row)
#define VDB_SR(R)                                                                                             \
    do {                                                                                                      \
        static const bool raised_ = [] {                                                                      \
            /* dynamic share = the CU's LDS minus this instantiation's static arrays */                       \
            const int dyn = (int)(kLdsBytes - rerank_static_lds(R));                                          \
            (void)hipFuncSetAttribute((const void*)ivf_select_rerank<R, kL2>,                                 \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, dyn);                       \
            (void)hipFuncSetAttribute((const void*)ivf_select_rerank<R, kIP>,                                 \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, dyn);                       \
            (void)hipGetLastError();                                                                          \
            return true;                                                                                      \
        }();                                                                                                  \
        (void)raised_;                                                                                        \
        if (metric == kL2)                                                                                    \
            ivf_select_rerank<R, kL2><<<B, 256, lds, s>>>(approx, delta, cent_rm, nlist, dp, qpad, B, P, ch,  \
                                                          cand, probes);                                      \
        else                                                                                                  \
            ivf_select_rerank<R, kIP><<<B, 256, lds, s>>>(approx, delta, cent_rm, nlist, dp, qpad, B, P, ch,  \
                                                          cand, probes);                                      \
    } while (0)
    switch (regs) {
        case 1: VDB_SR(1); break;
        case 2: VDB_SR(2); break;
        case 4: VDB_SR(4); break;
        case 8: VDB_SR(8); break;
        default: VDB_SR(16); break;
    }
#undef VDB_SR
}

void launch_assign_rerank(int metric, const float* approx, const float* delta, const float* cent_rm,
                          uint32_t nlist, uint32_t dp, const float* rows, uint32_t n, uint32_t* out, hipStream_t s) {
    const uint32_t g = cdiv(n, 4);
    if (!g) return;
    if (metric == kL2) ivf_assign_rerank<kL2><<<g, 256, 0, s>>>(approx, delta, cent_rm, nlist, dp, rows, n, out);
    else ivf_assign_rerank<kIP><<<g, 256, 0, s>>>(approx, delta, cent_rm, nlist, dp, rows, n, out);
}

void launch_plan(const uint32_t* probes, const uint32_t* nseg_local, const uint32_t* count_local, uint32_t B,
                 uint32_t P, uint32_t group, int wide, uint32_t segs_item, ScanItem* items, ScanItem* items_w,
                 uint32_t* counters,
                 uint32_t* sorted_pair, uint32_t* part_base_sorted, uint32_t* part_base_qp, uint32_t* nseg_qp,
                 uint32_t* l1base_qp, uint2* l1_items, unsigned long long* stats, uint32_t* thr, uint32_t mfma_min,
                 hipStream_t s) {
    // (the kernel sorts the batch's pairs in LDS arrays of kPlanMaxPairs: a larger batch would
    // write past them; the engine cuts batches by batch_cap, this is the last line)
    if ((uint64_t)B * P > (uint64_t)kPlanMaxPairs) throw std::length_error("launch_plan: batch x nprobe above kPlanMaxPairs");
    // (wide items carry at most `wide` queries: the scan kernels' per-item LDS holds 16 or 32)
    if (wide != 0 && wide != 16 && wide != 32) throw std::length_error("launch_plan: wide items of 16 or 32 queries only");
    uint32_t np = 1;
    while (np < B * P) np <<= 1;
    static const bool raised = [] {  // (up to 4 x kPlanMaxPairs + 1 words of dynamic LDS)
        (void)hipFuncSetAttribute((const void*)ivf_plan_probes, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)((4 * (size_t)kPlanMaxPairs + 1) * 4));
        (void)hipGetLastError();
        return true;
    }();
    (void)raised;
    const size_t lds = (4 * (size_t)np + 1) * 4;
    ivf_plan_probes<<<1, 1024, lds, s>>>(probes, nseg_local, count_local, B, P, np, group, (uint32_t)wide, segs_item,
                                       wide == 16 ? mfma_min : 0u, items,
                                       items_w, counters, sorted_pair, part_base_sorted, part_base_qp, nseg_qp,
                                       l1base_qp, l1_items, stats, thr);
}

void launch_merge_partials(int regs, uint32_t grid_items, const uint32_t* probes, const uint32_t* count_global,
                           const uint32_t* nseg_qp, const uint32_t* part_base_qp, const uint32_t* l1base_qp,
                           const uint2* l1_items, const uint32_t* counters, const float* part_d,
                           const uint64_t* part_i, uint32_t k, float* l1_d, uint64_t* l1_i, hipStream_t s) {
    // grid-stride over the batch's actual item count (counters[2]): a small grid, so a
    // merge issued while another batch's scan holds the CUs has few workgroups to place
    const uint32_t g = std::min<uint32_t>(launch_grid(grid_items, 4), kMergeBlocks);
    if (!grid_items) return;
#define VDB_MP(R) ivf_merge_partials<R><<<g, 256, 0, s>>>(probes, count_global, nseg_qp, part_base_qp, l1base_qp, l1_items, counters, part_d, part_i, k, l1_d, l1_i)
    switch (regs) {
        case 1: VDB_MP(1); break;
        case 2: VDB_MP(2); break;
        case 4: VDB_MP(4); break;
        case 8: VDB_MP(8); break;
        default: VDB_MP(16); break;
    }
#undef VDB_MP
}

// static LDS of ivf_scan_wide (queue slots, shared thresholds) and ivf_scan_bounded
// (the same plus the waves' candidate lists), rounded up
static constexpr size_t wide_static_lds(int waves) { return waves == 4 ? 256 : 256; }
static constexpr size_t kBoundedStaticLds = 256 + 4 * 2048;

size_t scan_wide_lds(uint32_t d4, uint32_t k, int waves) {
    const size_t gw = 4 * (size_t)waves;
    return (gw / 2) * d4 * 2 * sizeof(float4) + (size_t)waves * kWaveQueries * k * (sizeof(float) + sizeof(uint64_t));
}

bool scan_wide_fits(uint32_t d4, uint32_t k, int waves) {
    return k <= 64 && scan_wide_lds(d4, k, waves) <= kLdsBytes - wide_static_lds(waves);
}

void launch_scan_narrow(int metric, int regs, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s) {
    if (!grid_blocks) return;
    const uint32_t g = std::min<uint32_t>(grid_blocks, kPersistentBlocks);
    // (row-major lists exist only beside the screen: L2 / IP)
#define VDB_SN(R)                                                                                    \
    do {                                                                                             \
        if (a.rows_layout && metric == kL2) ivf_scan_narrow<R, kL2, true><<<g, 256, 0, s>>>(a);      \
        else if (a.rows_layout && metric == kIP) ivf_scan_narrow<R, kIP, true><<<g, 256, 0, s>>>(a); \
        else if (metric == kL2) ivf_scan_narrow<R, kL2, false><<<g, 256, 0, s>>>(a);                 \
        else if (metric == kIP) ivf_scan_narrow<R, kIP, false><<<g, 256, 0, s>>>(a);                 \
        else ivf_scan_narrow<R, kCos, false><<<g, 256, 0, s>>>(a);                                   \
    } while (0)
    switch (regs) {
        case 1: VDB_SN(1); break;
        case 2: VDB_SN(2); break;
        case 4: VDB_SN(4); break;
        case 8: VDB_SN(8); break;
        default: VDB_SN(16); break;
    }
#undef VDB_SN
}

size_t scan_bounded_lds(uint32_t d4, uint32_t k) {
    return (size_t)16 * d4 * sizeof(float4) + (size_t)4 * kWaveQueries * k * (sizeof(float) + sizeof(uint64_t));
}

bool scan_bounded_fits(uint32_t d4, uint32_t k) {
    return k <= 64 && scan_bounded_lds(d4, k) <= kLdsBytes - kBoundedStaticLds;
}

void launch_scan_bounded(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s) {
    if (!grid_blocks || (metric != kL2 && metric != kIP)) return;
    static const bool raised = [] {
        const int dyn = (int)(kLdsBytes - kBoundedStaticLds);
        (void)hipFuncSetAttribute((const void*)ivf_scan_bounded<kL2>, hipFuncAttributeMaxDynamicSharedMemorySize, dyn);
        (void)hipFuncSetAttribute((const void*)ivf_scan_bounded<kIP>, hipFuncAttributeMaxDynamicSharedMemorySize, dyn);
        (void)hipGetLastError();
        return true;
    }();
    (void)raised;
    const size_t lds = scan_bounded_lds(a.d4, a.k);
    const uint32_t g = std::min<uint32_t>(grid_blocks, kPersistentBlocks);
    if (metric == kL2) ivf_scan_bounded<kL2><<<g, 256, lds, s>>>(a);
    else ivf_scan_bounded<kIP><<<g, 256, lds, s>>>(a);
}

void launch_scan_wide(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s, int waves) {
    if (!grid_blocks) return;
    static const bool raised = [] {
        // wide items stage up to 16 (32) queries in LDS: allow the whole 160 KB of a CU
        const void* f4[] = {(const void*)ivf_scan_wide<kL2, 4, false>, (const void*)ivf_scan_wide<kIP, 4, false>,
                            (const void*)ivf_scan_wide<kL2, 4, true>, (const void*)ivf_scan_wide<kIP, 4, true>};
        const void* f8[] = {(const void*)ivf_scan_wide<kL2, 8, false>, (const void*)ivf_scan_wide<kIP, 8, false>};
        for (const void* f : f4)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytes - wide_static_lds(4)));
        for (const void* f : f8)
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytes - wide_static_lds(8)));
        (void)hipGetLastError();
        return true;
    }();
    (void)raised;
    // (row-major lists: 4-wave items only; the engine plans 16-query items for them)
    const size_t lds = scan_wide_lds(a.d4, a.k, waves);
    if (waves == 8 && !a.rows_layout) {  // one 8-wave workgroup per CU
        const uint32_t g = std::min<uint32_t>(grid_blocks, kPersistentBlocks / 2);
        if (metric == kL2) ivf_scan_wide<kL2, 8, false><<<g, 512, lds, s>>>(a);
        else ivf_scan_wide<kIP, 8, false><<<g, 512, lds, s>>>(a);
        return;
    }
    const uint32_t g = std::min<uint32_t>(grid_blocks, kPersistentBlocks);
    if (a.rows_layout) {
        if (metric == kL2) ivf_scan_wide<kL2, 4, true><<<g, 256, lds, s>>>(a);
        else ivf_scan_wide<kIP, 4, true><<<g, 256, lds, s>>>(a);
        return;
    }
    if (metric == kL2) ivf_scan_wide<kL2, 4, false><<<g, 256, lds, s>>>(a);
    else ivf_scan_wide<kIP, 4, false><<<g, 256, lds, s>>>(a);
}

void launch_slot_merge(int regs, const uint32_t* probes, const uint32_t* count_global, const uint32_t* nseg_qp,
                       const uint32_t* part_base_qp, const uint32_t* l1base_qp, const float* part_d,
                       const uint64_t* part_i, const float* l1_d, const uint64_t* l1_i, uint32_t BP, uint32_t k,
                       float* slot_d, uint64_t* slot_i, hipStream_t s) {
    const uint32_t g = cdiv(BP, 4);
    if (!g) return;
#define VDB_SLOT(R) ivf_merge_slots<R><<<g, 256, 0, s>>>(probes, count_global, nseg_qp, part_base_qp, l1base_qp, part_d, part_i, l1_d, l1_i, BP, k, slot_d, slot_i)
    switch (regs) {
        case 1: VDB_SLOT(1); break;
        case 2: VDB_SLOT(2); break;
        case 4: VDB_SLOT(4); break;
        case 8: VDB_SLOT(8); break;
        default: VDB_SLOT(16); break;
    }
#undef VDB_SLOT
}

void launch_query_merge(int regs, const uint32_t* probes, const uint32_t* count_global, const float* slot_d,
                        const uint64_t* slot_i, const float* carry_d, const uint64_t* carry_i, uint32_t B,
                        uint32_t P, uint32_t k, int stale, const uint32_t* req_start, uint32_t b0, float* out_d,
                        uint64_t* out_i, hipStream_t s) {
    const uint32_t g = cdiv(B, 4);
    if (!g) return;
#define VDB_QM(R) ivf_merge_query<R><<<g, 256, 0, s>>>(probes, count_global, slot_d, slot_i, carry_d, carry_i, B, P, k, stale, req_start, b0, out_d, out_i)
    switch (regs) {
        case 1: VDB_QM(1); break;
        case 2: VDB_QM(2); break;
        case 4: VDB_QM(4); break;
        case 8: VDB_QM(8); break;
        default: VDB_QM(16); break;
    }
#undef VDB_QM
}

void launch_carry(const uint32_t* probes, const uint32_t* count_global, uint32_t B, uint32_t P, uint32_t k,
                  const float* slot_d, const uint64_t* slot_i, const uint32_t* req_start, uint32_t b0,
                  float* carry_d, uint64_t* carry_i, hipStream_t s) {
    if (!P || !B) return;
    ivf_carry_slots<<<P, 64, 0, s>>>(probes, count_global, B, P, k, slot_d, slot_i, req_start, b0, carry_d, carry_i);
}

void launch_merge_fused(int regs, const uint32_t* probes, const uint32_t* count_global, const uint32_t* nseg_qp,
                        const uint32_t* part_base_qp, const float* part_d, const uint64_t* part_i, uint32_t B,
                        uint32_t P, uint32_t k, int stale, const uint32_t* req_start, uint32_t b0, const float* carry_d,
                        const uint64_t* carry_i, float* slot_d, uint64_t* slot_i, float* carry_nd, uint64_t* carry_ni,
                        float* out_d, uint64_t* out_i, hipStream_t s) {
    if (!B || !P) return;
    const uint32_t threads = 64 * std::min<uint32_t>(16, P);
#define VDB_MF(R) ivf_merge_fused<R><<<B, threads, 0, s>>>(probes, count_global, nseg_qp, part_base_qp, part_d, part_i, B, P, k, stale, req_start, b0, carry_d, carry_i, slot_d, slot_i, carry_nd, carry_ni, out_d, out_i)
    switch (regs) {
        case 1: VDB_MF(1); break;
        case 2: VDB_MF(2); break;
        case 4: VDB_MF(4); break;
        case 8: VDB_MF(8); break;
        default: VDB_MF(16); break;
    }
#undef VDB_MF
}

void launch_rank_merge(int regs, const float* d, const uint64_t* i, uint64_t d_stride, uint64_t i_stride,
                       uint32_t nranks, uint32_t n, uint32_t k, float* out_d, uint64_t* out_i, hipStream_t s) {
    const uint32_t g = cdiv(n, 4);
    if (!g) return;
#define VDB_RM(R) ivf_merge_ranks<R><<<g, 256, 0, s>>>(d, i, d_stride, i_stride, nranks, n, k, out_d, out_i)
    switch (regs) {
        case 1: VDB_RM(1); break;
        case 2: VDB_RM(2); break;
        case 4: VDB_RM(4); break;
        case 8: VDB_RM(8); break;
        default: VDB_RM(16); break;
    }
#undef VDB_RM
}

void launch_fill_empty(uint64_t n, float* d, uint64_t* i, hipStream_t s) {
    if (!n) return;
    ivf_fill_empty<<<launch_grid(n), 256, 0, s>>>(n, d, i);
}

void launch_interleave(const float* rows, uint64_t n, uint32_t dp, float4* blocks, hipStream_t s) {
    if (!n) return;
    const uint32_t d4 = dp / 4;
    const uint64_t total = (n + 63) / 64 * d4 * 64;
    ivf_interleave_rows<<<launch_grid(total), 256, 0, s>>>(rows, n, d4, blocks);
}

void launch_scatter_rows(const float* rows, const uint64_t* row_ids, const uint32_t* order, uint64_t n, uint32_t dp,
                         const uint64_t* dest_slot, float4* arena, uint64_t* arena_ids, hipStream_t s) {
    if (!n) return;
    const uint32_t d4 = dp / 4;
    ivf_scatter_rows<<<launch_grid(n * d4), 256, 0, s>>>(rows, row_ids, order, n, d4, dest_slot, arena, arena_ids);
}

void launch_copy_lists(const float4* old_arena, const uint64_t* old_ids, const uint64_t* old_off,
                       const uint64_t* new_off, const uint32_t* nblocks, uint32_t nlist, uint32_t d4,
                       float4* new_arena, uint64_t* new_ids, hipStream_t s) {
    if (!nlist) return;
    dim3 grid(16, nlist);
    ivf_copy_lists<<<grid, 256, 0, s>>>(old_arena, old_ids, old_off, new_off, nblocks, d4, new_arena, new_ids);
}

void launch_export_list(const float4* arena, const uint64_t* ids, uint64_t block_off, uint32_t count, uint32_t dim,
                        uint32_t d4, float* out, uint64_t* out_ids, hipStream_t s) {
    if (!count) return;
    ivf_export_list<<<launch_grid((uint64_t)count * dim), 256, 0, s>>>(arena, ids, block_off, count, dim, d4, out,
                                                                   out_ids);
}

void launch_assign(int metric, const float* vpad, uint64_t n, uint32_t dp, const float4* cent, uint32_t nlist,
                   uint32_t* out, hipStream_t s) {
    if (!n) return;
    const uint32_t grid = launch_grid(n, 32);
    const uint32_t d4 = dp / 4;
    if (metric == kL2) ivf_assign<kL2><<<grid, 256, 0, s>>>(vpad, n, d4, cent, nlist, out);
    else if (metric == kIP) ivf_assign<kIP><<<grid, 256, 0, s>>>(vpad, n, d4, cent, nlist, out);
    else ivf_assign<kCos><<<grid, 256, 0, s>>>(vpad, n, d4, cent, nlist, out);
}

void launch_histogram(const uint32_t* keys, uint64_t n, uint32_t* counts, hipStream_t s) {
    if (!n) return;
    ivf_histogram<<<launch_grid(n), 256, 0, s>>>(keys, n, counts);
}

void launch_mindist_init(float* mind, uint64_t n, hipStream_t s) {
    if (!n) return;
    ivf_fill_f32<<<launch_grid(n), 256, 0, s>>>(mind, n, FLT_MAX);
}

void launch_mindist_update(const float4* v_il, uint64_t n, uint32_t d4, const float* crow, float* mind,
                           hipStream_t s) {
    if (!n) return;
    kmeanspp_mindist<<<launch_grid((n + 63) / 64, 4), 256, 0, s>>>(v_il, n, d4, crow, mind);
}

void launch_centroid_update(const float* vpad, uint32_t dp, const uint32_t* order, const uint32_t* offsets,
                            const uint32_t* counts, uint32_t nlist, uint32_t dim, float* cent_rm, hipStream_t s) {
    dim3 grid(cdiv(dim, 256), nlist);
    lloyd_update<<<grid, 256, 0, s>>>(vpad, dp, order, offsets, counts, dim, cent_rm);
}

void launch_iota(uint32_t* out, uint64_t n, hipStream_t s) {
    if (!n) return;
    ivf_iota<<<launch_grid(n), 256, 0, s>>>(out, n);
}

void launch_slots_from_order(const uint32_t* sorted_keys, uint64_t n, const uint64_t* group_start,
                             const uint64_t* base_slot, uint64_t* dest, hipStream_t s) {
    if (!n) return;
    ivf_slots_from_order<<<launch_grid(n), 256, 0, s>>>(sorted_keys, n, group_start, base_slot, dest);
}

void launch_gen_normal(float* out, uint64_t n, uint64_t seed, uint64_t offset, hipStream_t s) {
    if (!n) return;
    synth_gen_normal<<<launch_grid(n), 256, 0, s>>>(out, n, seed, offset);
}

void launch_gen_mixture(float* out, uint64_t rows, uint32_t dim, const float* centers, uint32_t ncomp, float sigma,
                        uint64_t seed, uint64_t row0, hipStream_t s) {
    if (!rows || !dim) return;
    synth_gen_mixture<<<launch_grid(rows * dim), 256, 0, s>>>(out, rows, dim, centers, ncomp, sigma, seed, row0);
}

hipError_t radix_sort_pairs(void* temp, size_t& temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                            const uint32_t* vals_in, uint32_t* vals_out, uint64_t n, int end_bit, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                              end_bit, s);
}

}  // namespace vdbk
