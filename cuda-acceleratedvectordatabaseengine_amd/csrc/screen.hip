// screen.hip — the screened fine scan (search_list_cpu, ivf_flat_index.cpp:339-384), the
// default scan for L2 / IP with k <= 64 on lists held in HBM.
//
// Every (query, list vector) distance is first SCREENED on the matrix cores from a bf16
// shadow of the lists, and the reference's exact sequential fp32 sum is computed only
// for the pairs that can still reach the list's top-k. Results are bit-identical to the
// exact scan (kernels.hip ivf_scan_wide / ivf_scan_narrow):
//  * Shadow: each list block of 64 vectors is also stored as bf16 RESIDUALS b' = bf16(x - c)
//    against the list's centroid c, in the B-operand order of v_mfma_f32_16x16x32_bf16:
//    per k-step s (32 dims) and vector tile vt (16 vectors), lane l holds vector
//    16 vt + (l & 15), dims 32 s + 8 (l >> 4) .. + 8 — one 1 KiB wave-load per MFMA operand,
//    half the bytes of the fp32 stream. Residuals keep the bound proportional to the spread
//    of the list rather than to |x|, so clustered data screens as well as iid data.
//  * Screen: A = per (query, probed list) bf16 rows a' (L2: a = q - c; IP: a = q), so D lane l
//    holds <a', b'> for vector v = 16 vt + (l & 15) and queries g = 4 (l >> 4) + r.
//      L2: |q - x|^2 = |a|^2 + |b|^2 - 2 <a, b>,  approx = |a|^2 + |b|^2 - 2 <a', b'>
//      IP: -<q, x> = -(<q, c> + <q, b>),           approx = -(<q, c> + <q', b'>)
//    With e = b - b', f = a - a' (measured per vector / pair in double, rounded up),
//      |<a, b> - <a', b'>| <= (|a| + |f|) |e| + |f| (|b| + |e|) + |f| |e|   (Cauchy-Schwarz)
//    and the MFMA's f32 accumulation, the reference's own rounding (its sequential fp32 sum
//    is within 2 (n + 4) u of the real value relative to (|a| + |b|)^2, resp. |q| |x|), the
//    float rounding of the norms and of approx are all below (12 dp + 64) u S^2 (S: the sum
//    of every norm involved, u = 2^-24). delta is padded further (x 1.001, + 1e-6 |approx|,
//    + 1e-30) for its own rounding and for subnormals.
//  * A pair is a candidate unless approx - delta > th, th = min(the wave's own k-th, the
//    list-wide shared k-th, the block bound below): a pair above th is strictly worse than
//    k vectors of the same list and cannot be in the list's multiset top-k (the exact
//    scan's pruning rule). NaN / inf anywhere makes the test false, so such pairs are always
//    re-checked; vectors, centroids or queries with a non-finite or huge (> 2^50) value carry
//    |e| or |f| = inf.
//  * Candidates are compacted into a per-wave LDS ring and recomputed exactly in rounds
//    of 64 (one lane per pair: the reference's d = 0..D-1 sum over the fp32 row, from a
//    row-major copy of the lists in slot order), then offered to the query's top-k exactly
//    as the exact scan does (ties always kept). Every k-th reached is published to the
//    list-wide thresholds at once, and every block re-reads them.
// Items, partials and merges are the exact scan's (kernels.hip).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <cfloat>
#include <type_traits>

#include "kernels.hpp"
#include "scan_common.hpp"
#include "wave_topk.hpp"

namespace vdbk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr float kScreenHuge = 1125899906842624.0f;  // 2^50: larger magnitudes are never screened
constexpr int kRing = 512;                          // candidate ring entries per wave
#ifndef VDB_SCREEN_EXACT_PIPE
#define VDB_SCREEN_EXACT_PIPE 4
#endif
constexpr int kExactPipe = VDB_SCREEN_EXACT_PIPE;   // float4 of a row in flight per lane (re-checks mid-stream)
#ifndef VDB_SCREEN_EXACT_PIPE_END
#define VDB_SCREEN_EXACT_PIPE_END 8
#endif
constexpr int kExactPipeEnd = VDB_SCREEN_EXACT_PIPE_END;  // ... for a segment's last partial round
// Timing experiment (a separate build, never an option): 1 drops the candidates instead
// of re-checking them (the screen stream alone; results INVALID).
#ifndef VDB_SCREEN_DIAG
#define VDB_SCREEN_DIAG 0
#endif

// Nearest bf16, ties to even; +0 for |f| < 2^-126 (no bf16 subnormals reach the matrix
// cores, and |e| accounts for the flush). Non-finite inputs are flagged by the caller.
__device__ __forceinline__ uint32_t bf16_bits(float f) {
    const uint32_t b = __float_as_uint(f);
    const uint32_t ex = b & 0x7F800000u;
    if (ex == 0) return 0u;
    if (ex == 0x7F800000u) return 0x7FC0u;
    return (b + 0x7FFFu + ((b >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_val(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ uint4 pack_bf16x8(const float4 lo, const float4 hi) {
    uint4 r;
    r.x = bf16_bits(lo.x) | (bf16_bits(lo.y) << 16);
    r.y = bf16_bits(lo.z) | (bf16_bits(lo.w) << 16);
    r.z = bf16_bits(hi.x) | (bf16_bits(hi.y) << 16);
    r.w = bf16_bits(hi.z) | (bf16_bits(hi.w) << 16);
    return r;
}

// x - c rounded to float (the value the shadow's bf16 rounds), from the exact double difference
__device__ __forceinline__ float4 resid(const float4 x, const float4 c) {
    return make_float4((float)((double)x.x - c.x), (float)((double)x.y - c.y), (float)((double)x.z - c.z),
                       (float)((double)x.w - c.w));
}

// ---- build: the residual shadow, the row-major fp32 copy and the per-slot norms
// {|b|^2, |b| up, |b - b'| up, |x| up} of every arena block (one wave per block of 64
// vectors; lane = vector; block_list: the list each block belongs to).
__device__ __forceinline__ float ru(double v) { return __double2float_ru(v * (1.0 + 0x1p-30)); }

__global__ __launch_bounds__(256) void ivf_screen_build(const float4* __restrict__ arena, uint64_t blocks,
                                                        uint32_t d4, const uint32_t* __restrict__ block_list,
                                                        const float* __restrict__ cent_rm, uint4* __restrict__ shadow,
                                                        float* __restrict__ rows, float4* __restrict__ meta) {
    const int lane = lane_id();
    const uint32_t dp = d4 * 4, ks = dp / 32;
    for (uint64_t b = (uint64_t)blockIdx.x * 4 + wave_index(); b < blocks; b += (uint64_t)gridDim.x * 4) {
        const float4* blk = arena + b * d4 * 64;
        const float4* cen = (const float4*)(cent_rm + (size_t)block_list[b] * dp);
        const uint64_t slot = b * 64 + lane;
        float4* row = rows ? (float4*)(rows + slot * dp) : nullptr;
        double x2 = 0.0, b2 = 0.0, e2 = 0.0;
        bool huge = false;
        for (uint32_t t = 0; t < d4; ++t) {
            const float4 x = blk[(size_t)t * 64 + lane];
            const float4 c = cen[t];
            if (rows) row[t] = x;  // (the inline scan's row-major copy; null: deferred re-checks read the arena)
            const float xv[4] = {x.x, x.y, x.z, x.w}, cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double bd = (double)xv[i] - (double)cv[i];
                const double ed = bd - (double)bf16_val(bf16_bits((float)bd));
                huge |= !(fabs(bd) <= (double)kScreenHuge) || !(fabsf(xv[i]) <= kScreenHuge);
                x2 += (double)xv[i] * xv[i];
                b2 += bd * bd;
                e2 += ed * ed;
            }
        }
        meta[slot] = huge ? make_float4(__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff())
                          : make_float4((float)b2, ru(sqrt(b2)), ru(sqrt(e2)), ru(sqrt(x2)));
        uint4* sh = shadow + b * (uint64_t)d4 * 32;
        const int vv = lane & 15, h = lane >> 4;
        for (uint32_t s = 0; s < ks; ++s) {
            const float4 c0 = cen[8 * s + 2 * h], c1 = cen[8 * s + 2 * h + 1];
            for (int vt = 0; vt < 4; ++vt) {
                const float4 lo = blk[(size_t)(8 * s + 2 * h) * 64 + 16 * vt + vv];
                const float4 hi = blk[(size_t)(8 * s + 2 * h + 1) * 64 + 16 * vt + vv];
                sh[((size_t)s * 4 + vt) * 64 + lane] = pack_bf16x8(resid(lo, c0), resid(hi, c1));
            }
        }
    }
}

// ---- per batch: per (query, probe) pair i = q * P + p the MFMA A row a' (bf16, [BP][dp]) and
// its norms pst[i]: L2 (a = q - c): {|a|^2, |a| up, |a - a'| up, 0}; IP (a = q):
// {<q, c>, |q| up, |q - q'| up, |c| up}. One wave per pair; flagged (inf) when q, c or a
// holds a non-finite or huge value.
template <int M>
__global__ __launch_bounds__(256) void ivf_screen_pairs(const float* __restrict__ q, uint32_t BP, uint32_t P,
                                                        const uint32_t* __restrict__ probes,
                                                        const float* __restrict__ cent_rm, uint32_t dp,
                                                        uint16_t* __restrict__ qres, float4* __restrict__ pst,
                                                        uint32_t* __restrict__ thr4, uint32_t* __restrict__ scnt,
                                                        uint32_t* __restrict__ ovf, uint32_t* __restrict__ counters,
                                                        uint32_t* __restrict__ ubcnt) {
    chain_prio();
    const int lane = lane_id();
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < 4 * BP; e += gridDim.x * blockDim.x) thr4[e] = kThrInf;
    if (scnt)  // (the deferred scan: survivor counts, overflow marks and the candidate count)
        for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < BP; e += gridDim.x * blockDim.x) {
            scnt[e] = 0u;
            ovf[e] = 0u;
            ubcnt[e] = 0u;
            if (e == 0) counters[kCtrCand] = counters[kCtrOvf] = counters[kCtrReal] = 0u;
        }
    for (uint32_t i = blockIdx.x * 4 + wave_index(); i < BP; i += gridDim.x * 4) {
        const float* qr = q + (size_t)(i / P) * dp;
        const float* cr = cent_rm + (size_t)probes[i] * dp;
        double a2 = 0.0, f2 = 0.0, c2 = 0.0, qc = 0.0;
        bool huge = false;
        for (uint32_t d = lane; d < dp; d += 64) {
            const float qv = qr[d], cv = cr[d];
            const double ad = M == kL2 ? (double)qv - (double)cv : (double)qv;
            const uint32_t h = bf16_bits((float)ad);
            qres[(size_t)i * dp + d] = (uint16_t)h;
            const double fd = ad - (double)bf16_val(h);
            huge |= !(fabs(ad) <= (double)kScreenHuge) || !(fabsf(qv) <= kScreenHuge) || !(fabsf(cv) <= kScreenHuge);
            a2 += ad * ad;
            f2 += fd * fd;
            c2 += (double)cv * cv;
            qc += (double)qv * cv;
        }
        for (int m = 32; m >= 1; m >>= 1) {
            a2 += __shfl_xor(a2, m);
            f2 += __shfl_xor(f2, m);
            c2 += __shfl_xor(c2, m);
            qc += __shfl_xor(qc, m);
        }
        huge = __ballot(huge) != 0;
        if (lane == 0) {
            const float inf = __builtin_inff();
            if (huge) pst[i] = make_float4(inf, inf, inf, inf);
            else if (M == kL2) pst[i] = make_float4((float)a2, ru(sqrt(a2)), ru(sqrt(f2)), 0.0f);
            else pst[i] = make_float4((float)qc, ru(sqrt(a2)), ru(sqrt(f2)), ru(sqrt(c2)));
        }
    }
}

// ---- the int8 shadow (deferred screen, option screen_i8): per vector a scale
// s_b = max_i |x_i - c_i| / 127 (rounded up) and q_b = rint((x - c) / s_b) in [-127, 127], so
// b' = s_b q_b; in the B-operand order of v_mfma_i32_16x16x64_i8: per k-step s (64 dims) and
// vector tile vt, lane l holds vector 16 vt + (l & 15), dims 64 s + 16 (l >> 4) .. + 16 (A and B
// share the instruction's lane -> k map, so the same dims in the same slots of both make the
// full dot product whatever that map is). Half the bf16 shadow's bytes; |b - b'| is measured
// exactly (double) as for bf16 and is about 4.6x larger on Gaussian residuals. The integer
// products and sums are exact (|dot| <= 127^2 dp < 2^24, also exact as a float).
__device__ __forceinline__ float i8_scale(float mx) { return mx > 0.0f ? mx * (1.0f / 127.0f) * (1.0f + 0x1p-20f) : 0.0f; }
__device__ __forceinline__ int i8_q(float r, float inv) { return max(-127, min(127, (int)rintf(r * inv))); }

__global__ __launch_bounds__(256) void ivf_screen_build_i8(const float4* __restrict__ arena, uint64_t blocks,
                                                           uint32_t d4, const uint32_t* __restrict__ block_list,
                                                           const float* __restrict__ cent_rm, uint4* __restrict__ shadow,
                                                           float* __restrict__ rows, float4* __restrict__ meta,
                                                           float* __restrict__ sscale) {
    const int lane = lane_id();
    const uint32_t dp = d4 * 4, ks = dp / 64;
    for (uint64_t b = (uint64_t)blockIdx.x * 4 + wave_index(); b < blocks; b += (uint64_t)gridDim.x * 4) {
        const float4* blk = arena + b * d4 * 64;
        const float4* cen = (const float4*)(cent_rm + (size_t)block_list[b] * dp);
        const uint64_t slot = b * 64 + lane;
        float4* row = rows ? (float4*)(rows + slot * dp) : nullptr;
        double x2 = 0.0, b2 = 0.0;
        float mx = 0.0f;
        bool huge = false;
        for (uint32_t t = 0; t < d4; ++t) {  // pass 1 (lane = vector): norms and the scale
            const float4 x = blk[(size_t)t * 64 + lane];
            const float4 c = cen[t];
            if (rows) row[t] = x;
            const float xv[4] = {x.x, x.y, x.z, x.w}, cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double bd = (double)xv[i] - (double)cv[i];
                huge |= !(fabs(bd) <= (double)kScreenHuge) || !(fabsf(xv[i]) <= kScreenHuge);
                x2 += (double)xv[i] * xv[i];
                b2 += bd * bd;
                mx = fmaxf(mx, fabsf((float)bd));
            }
        }
        const float sc = huge ? 0.0f : i8_scale(mx);
        sscale[slot] = sc;
        // pass 2 (lane = (vector 16 vt + (l & 15), dims 16 (l >> 4) ..)): the quantized shadow and |b - b'|
        const int vv = lane & 15, h = lane >> 4;
        float svt[4], inv[4];
        double e2p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) {
            svt[vt] = __shfl(sc, 16 * vt + vv);
            inv[vt] = svt[vt] > 0.0f ? 1.0f / svt[vt] : 0.0f;
        }
        uint4* sh = shadow + b * (uint64_t)ks * 256;
        for (uint32_t s = 0; s < ks; ++s) {
            float4 c4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) c4[j] = cen[16 * s + 4 * h + j];
#pragma unroll
            for (int vt = 0; vt < 4; ++vt) {
                uint32_t w[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float4 x = blk[(size_t)(16 * s + 4 * h + j) * 64 + 16 * vt + vv];
                    const float xv[4] = {x.x, x.y, x.z, x.w}, cv[4] = {c4[j].x, c4[j].y, c4[j].z, c4[j].w};
                    uint32_t word = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const double bd = (double)xv[i] - (double)cv[i];
                        const int qv = i8_q((float)bd, inv[vt]);
                        const double ed = bd - (double)svt[vt] * (double)qv;
                        e2p[vt] += ed * ed;
                        word |= (uint32_t)(qv & 0xFF) << (8 * i);
                    }
                    w[j] = word;
                }
                sh[((size_t)s * 4 + vt) * 64 + lane] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) {
            e2p[vt] += __shfl_xor(e2p[vt], 16);
            e2p[vt] += __shfl_xor(e2p[vt], 32);
        }
        const int mv = lane >> 4;  // (this lane's vector 16 mv + (l & 15): its |b - b'|^2)
        const double e2 = mv == 0 ? e2p[0] : mv == 1 ? e2p[1] : mv == 2 ? e2p[2] : e2p[3];
        meta[slot] = huge ? make_float4(__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff())
                          : make_float4((float)b2, ru(sqrt(b2)), ru(sqrt(e2)), ru(sqrt(x2)));
    }
}

// Per (query, probe) pair: the int8 A row (L2: a = q - c; IP: a = q) with its scale s_a, and
// pst as for bf16 ({|a|^2 or <q, c>, |a| up, |a - a'| up, |c| up}).
template <int M>
__global__ __launch_bounds__(256) void ivf_screen_pairs_i8(const float* __restrict__ q, uint32_t BP, uint32_t P,
                                                           const uint32_t* __restrict__ probes,
                                                           const float* __restrict__ cent_rm, uint32_t dp,
                                                           int8_t* __restrict__ qres, float* __restrict__ qscale,
                                                           float4* __restrict__ pst, uint32_t* __restrict__ thr4,
                                                           uint32_t* __restrict__ scnt, uint32_t* __restrict__ ovf,
                                                           uint32_t* __restrict__ counters, uint32_t* __restrict__ ubcnt) {
    chain_prio();
    const int lane = lane_id();
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < 4 * BP; e += gridDim.x * blockDim.x) thr4[e] = kThrInf;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < BP; e += gridDim.x * blockDim.x) {
        scnt[e] = 0u;
        ovf[e] = 0u;
        ubcnt[e] = 0u;
        if (e == 0) counters[kCtrCand] = counters[kCtrOvf] = counters[kCtrReal] = 0u;
    }
    for (uint32_t i = blockIdx.x * 4 + wave_index(); i < BP; i += gridDim.x * 4) {
        const float* qr = q + (size_t)(i / P) * dp;
        const float* cr = cent_rm + (size_t)probes[i] * dp;
        double a2 = 0.0, c2 = 0.0, qc = 0.0;
        float mx = 0.0f;
        bool huge = false;
        for (uint32_t d = lane; d < dp; d += 64) {
            const float qv = qr[d], cv = cr[d];
            const double ad = M == kL2 ? (double)qv - (double)cv : (double)qv;
            huge |= !(fabs(ad) <= (double)kScreenHuge) || !(fabsf(qv) <= kScreenHuge) || !(fabsf(cv) <= kScreenHuge);
            a2 += ad * ad;
            c2 += (double)cv * cv;
            qc += (double)qv * cv;
            mx = fmaxf(mx, fabsf((float)ad));
        }
        for (int m = 32; m >= 1; m >>= 1) {
            a2 += __shfl_xor(a2, m);
            c2 += __shfl_xor(c2, m);
            qc += __shfl_xor(qc, m);
            mx = fmaxf(mx, __shfl_xor(mx, m));
        }
        huge = __ballot(huge) != 0;
        const float sc = huge ? 0.0f : i8_scale(mx);
        const float inv = sc > 0.0f ? 1.0f / sc : 0.0f;
        double f2 = 0.0;
        for (uint32_t d = lane; d < dp; d += 64) {
            const float qv = qr[d], cv = cr[d];
            const double ad = M == kL2 ? (double)qv - (double)cv : (double)qv;
            const int qi = i8_q((float)ad, inv);
            qres[(size_t)i * dp + d] = (int8_t)qi;
            const double fd = ad - (double)sc * (double)qi;
            f2 += fd * fd;
        }
        for (int m = 32; m >= 1; m >>= 1) f2 += __shfl_xor(f2, m);
        if (lane == 0) {
            const float inf = __builtin_inff();
            qscale[i] = sc;
            if (huge) pst[i] = make_float4(inf, inf, inf, inf);
            else if (M == kL2) pst[i] = make_float4((float)a2, ru(sqrt(a2)), ru(sqrt(f2)), 0.0f);
            else pst[i] = make_float4((float)qc, ru(sqrt(a2)), ru(sqrt(f2)), ru(sqrt(c2)));
        }
    }
}

// One compare-exchange stage of a bitonic sort of 64 values held as u[v] in the 16 lanes of
// a DPP row: element e = 4 (lane & 15) + v (strides 1, 2 within a lane, 4 .. 32 across lanes).
template <int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic64_step(float (&u)[4], int l) {
    if constexpr (STRIDE < 4) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            if (v & STRIDE) continue;
            const int w = v | STRIDE;
            const bool asc = ((4 * l + v) & SIZE) == 0;
            const float lo = fminf(u[v], u[w]), hi = fmaxf(u[v], u[w]);
            u[v] = asc ? lo : hi;
            u[w] = asc ? hi : lo;
        }
    } else {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const float p = xor_f<STRIDE / 4>(u[v]);
            const int e = 4 * l + v;
            const bool keep_min = ((e & SIZE) == 0) == ((e & STRIDE) == 0);
            u[v] = keep_min ? fminf(u[v], p) : fmaxf(u[v], p);
        }
    }
}
// The kk-th smallest (1 <= kk <= 64) of the 64 values u[0..3] x 16 lanes of each DPP row, in
// every lane of the row (u is sorted in place). Every lane of the wave must be active.
__device__ __forceinline__ float block_kth(float (&u)[4], int kk) {
    const int l = lane_id() & 15;
    bitonic64_step<2, 1>(u, l);
    bitonic64_step<4, 2>(u, l), bitonic64_step<4, 1>(u, l);
    bitonic64_step<8, 4>(u, l), bitonic64_step<8, 2>(u, l), bitonic64_step<8, 1>(u, l);
    bitonic64_step<16, 8>(u, l), bitonic64_step<16, 4>(u, l), bitonic64_step<16, 2>(u, l), bitonic64_step<16, 1>(u, l);
    bitonic64_step<32, 16>(u, l), bitonic64_step<32, 8>(u, l), bitonic64_step<32, 4>(u, l);
    bitonic64_step<32, 2>(u, l), bitonic64_step<32, 1>(u, l);
    bitonic64_step<64, 32>(u, l), bitonic64_step<64, 16>(u, l), bitonic64_step<64, 8>(u, l);
    bitonic64_step<64, 4>(u, l), bitonic64_step<64, 2>(u, l), bitonic64_step<64, 1>(u, l);
    const int e = kk - 1, v = e & 3;
    const float x = v == 0 ? u[0] : v == 1 ? u[1] : v == 2 ? u[2] : u[3];
    return __shfl(x, (lane_id() & ~15) + (e >> 2));
}

__device__ __forceinline__ uint4 ld_nt_u4(const uint4* p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ bf16x8 as_bf16x8(const uint4 v) {
    return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ i32x4 as_i32x4(const uint4 v) {
    return __builtin_bit_cast(i32x4, v);
}

// One wave: segment `seg` of list it.list against the nq (<= 16) queries of the item
// starting at sorted pair it.pair_start + q0. tk_d / tk_i: the per-query top-k lists (nq x k,
// LDS) this wave inserts into: its own, reset when `fresh` (narrow items), or the wide item's
// lists shared by its 4 waves under `locks` (one insertion at a time per query); kdl: their
// k-th distances; s_thr: the shared k-th of the item's queries (LDS, lowered with atomicMin);
// ring: the candidate ring (kRing); item_slot: the item's index (quarter-list thresholds).
// The caller writes the partials (screen_partials).
template <int M, int KD>
__device__ __forceinline__ void screen_segment(const ScanArgs& a, const ScanItem it, const int q0, const int nq,
                                               const uint32_t seg, float* tk_d, uint64_t* tk_i, float* kdl,
                                               uint32_t* s_thr, uint32_t* ring, const bool fresh,
                                               uint32_t* locks, const uint32_t item_slot) {
    const int lane = lane_id();
    const uint32_t dp = a.dp, ks = dp >> 5, d4 = a.d4;
    const uint32_t count = a.count[it.list];
    const uint32_t seg_vectors = a.seg_blocks * 64;
    const uint64_t b0 = a.block_off[it.list] + (uint64_t)seg * a.seg_blocks;
    const uint32_t v0 = seg * seg_vectors;
    const uint32_t nv = min(count - v0, seg_vectors);
    const uint32_t nb = (nv + 63) >> 6;
    const int k = (int)a.k;
    const uint32_t* pairs = a.sorted_pair + it.pair_start + q0;
    // rounding coefficients of the bound (u = 2^-24, 1 % margin): the MFMA's f32 sum of dp
    // exact bf16 products (4 (dp + 4) u, a 4x margin over sequential accumulation), the
    // reference's sequential sum ((dp + 2) u relative to its terms), the norms' and approx's
    // own roundings
    const float cm = (float)(4 * dp + 16) * 0x1.02p-24f;
    const float cr = (float)(dp + 2) * 0x1.02p-24f;
    const float cu = 0x1.02p-23f;

    if (fresh) {
        for (int e = lane; e < 16 * k; e += 64) {
            tk_d[e] = __builtin_inff();
            tk_i[e] = kNoId;
        }
        if (lane < 16) kdl[lane] = __builtin_inff();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }

    // (query, probe) pair index of the item's query g: the A rows and norms are per pair
    auto pair_of = [&](int g) -> uint32_t {
        const uint32_t pr = pairs[g];
        return (pr >> 16) * a.P + (pr & 0xFFFFu);
    };
    // the MFMA A row of this lane: query (lane & 15), its dims 8 (lane >> 4) .. + 8 of each k-step
    const int ga = min(lane & 15, nq - 1);
    const uint4* qa_row = (const uint4*)(a.qres + (size_t)pair_of(ga) * dp) + (lane >> 4);
    // the D rows of this lane: queries 4 (lane >> 4) + r (their norms are re-read per block:
    // L1 hits, and no registers held across the stream)
    const float4* pst_r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pst_r[r] = a.pst + pair_of(min(4 * (lane >> 4) + r, nq - 1));

    uint32_t head = 0, tail = 0;  // wave-uniform ring cursors

    // Exact re-check of up to 64 ring entries (one per lane), then the top-k offers.
    auto exact_round = [&](uint32_t n, auto pipe_c) {
        constexpr int kPipe = decltype(pipe_c)::value;
        const bool act = lane < (int)n;
        const uint32_t ent = ring[(head + (act ? (uint32_t)lane : 0u)) & (kRing - 1)];
        head += n;
        if (a.mstats && lane == 0) atomicAdd(&a.mstats[0], (unsigned long long)n);
        const int g = (int)(ent >> 16);
        const uint32_t v = ent & 0xFFFFu;
        const uint64_t slot = (b0 + (v >> 6)) * 64 + (v & 63);
        const float4* xr = (const float4*)(a.rows + slot * dp);
        const float4* qr = (const float4*)(a.qpad + (size_t)(pairs[g] >> 16) * dp);
        float acc = 0.0f;
        float4 xb[kPipe], qb[kPipe];
#pragma unroll
        for (int i = 0; i < kPipe; ++i) {
            xb[i] = xr[i];
            qb[i] = qr[i];
        }
        for (uint32_t t0 = 0; t0 < d4; t0 += kPipe) {
#pragma unroll
            for (int i = 0; i < kPipe; ++i) {
                acc = acc4<M>(acc, qb[i], xb[i]);
                if (t0 + kPipe < d4) {
                    xb[i] = xr[t0 + kPipe + i];
                    qb[i] = qr[t0 + kPipe + i];
                }
            }
        }
        const float dist = dist_finish<M>(acc);
        const uint64_t vid = a.ids[slot];
        uint32_t present = 0;
        for (int gq = 0; gq < nq; ++gq)
            if (__ballot(act && g == gq)) present |= 1u << gq;
        while (present) {
            const int gs = __builtin_ctz(present);
            present &= present - 1;
            if (locks) {  // lists shared by the item's waves: one insertion at a time per query
                if (lane == 0)
                    while (atomicCAS(&locks[gs], 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            const float kdg = fminf(kdl[gs], ord_dec(s_thr[gs]));
            float* sd = tk_d + gs * k;
            uint64_t* si = tk_i + gs * k;
            WaveTopK<1> tk;
            tk.d[0] = lane < k ? sd[lane] : __builtin_inff();
            tk.id[0] = lane < k ? si[lane] : kNoId;
            float nkd;
            uint64_t nki;
            tk.at(k - 1, nkd, nki);
            offer_lanes<1>(tk, act && g == gs && dist <= kdg, dist, vid, k, nkd, nki);
            if (lane < k) {
                sd[lane] = tk.d[0];
                si[lane] = tk.id[0];
            }
            if (lane == 0) kdl[gs] = nkd;
            // the list's ceil(k/4)-th into this item's quarter slot (see thr4 below)
            const float dj = rd_lane(tk.d[0], (k + 3) / 4 - 1);
            if (lane == 0 && dj < __builtin_inff()) {
                uint32_t* s4 = a.thr4 + (size_t)(it.pair_start + q0 + gs) * 4 + (item_slot & 3u);
                if (dj < ord_dec(*s4)) atomicMin(s4, ord_enc(dj));
            }
            if (nkd < kdg && lane == 0) {
                atomicMin(&s_thr[gs], ord_enc(nkd));
                uint32_t* gt = a.thr + it.pair_start + q0 + gs;
                if (nkd < ord_dec(*gt)) atomicMin(gt, ord_enc(nkd));
            }
            if (locks) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) atomicExch(&locks[gs], 0u);
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            }
        }
    };

    // the screen: stream the segment's shadow blocks through the matrix cores, KD k-steps
    // (4 x 1 KiB each) in flight; the pipeline runs KD steps past the segment (slack)
    const uint4* sp = a.shadow + b0 * (uint64_t)dp * 8 + lane;
    uint4 xa[KD][4], qa[KD];
#pragma unroll
    for (int u = 0; u < KD; ++u) {
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) xa[u][vt] = ld_nt_u4(sp + (size_t)(u * 4 + vt) * 64);
        qa[u] = qa_row[4 * (u % ks)];
    }
    for (uint32_t j = 0; j < nb; ++j) {
        f32x4 acc[4];
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) acc[vt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        for (uint32_t s0 = 0; s0 < ks; s0 += KD) {
            static_for<0, KD>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
                const bf16x8 A = as_bf16x8(qa[u]);
#pragma unroll
                for (int vt = 0; vt < 4; ++vt)
                    acc[vt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, as_bf16x8(xa[u][vt]), acc[vt], 0, 0, 0);
                const uint64_t nxt = (uint64_t)j * ks + s0 + u + KD;
#pragma unroll
                for (int vt = 0; vt < 4; ++vt) xa[u][vt] = ld_nt_u4(sp + (nxt * 4 + vt) * 64);
                qa[u] = qa_row[4 * ((s0 + u + KD) % ks)];
            });
        }
        // Bounds of the block's 64 x 16 pairs: lower bounds replace the dot products in acc,
        // upper bounds go to ubv (invalid vectors and NaN: +inf).
        float ubv[4][4];
        float4 pst[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pst[r] = *pst_r[r];
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) {
            const float4 mt = a.meta[(b0 + j) * 64 + 16 * vt + (lane & 15)];
            const bool valid = j * 64 + 16 * vt + (lane & 15) < nv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float dot = acc[vt][r];
                const float4 ps = pst[r];
                const float approx = M == kL2 ? (ps.x + mt.x) - 2.0f * dot : -(ps.x + dot);
                // Cauchy-Schwarz term of <a, b> - <a', b'>, and the MFMA's accumulation bound
                const float an = ps.y + ps.z, bn = mt.y + mt.z;
                const float cs = an * mt.z + ps.z * bn + ps.z * mt.z;
                float del;
                if (M == kL2) {
                    // |approx - |a - b|^2| <= rest; the reference's sum is within cr |a - b|^2
                    // <= cr (|approx| + rest) of the real value
                    const float rest = 2.0f * (cs + cm * (an * bn)) + cu * (ps.x + mt.x + fabsf(approx));
                    del = rest + cr * (fabsf(approx) + rest);
                } else {
                    // IP: -(<q, c> + <q', b'>); the reference's sum is within cr |q| |x| (mt.w),
                    // <q, c> rounded to float within u |q| |c| (ps.w)
                    del = cs + cm * (an * bn) + cr * (ps.y * mt.w) + cu * (ps.y * ps.w + an * bn + fabsf(approx));
                }
                del = del * 1.001f + 1e-30f;
                const float ub = approx + del;
                acc[vt][r] = approx - del;
                ubv[r][vt] = valid && ub == ub ? ub : __builtin_inff();
            }
        }
        // Block bound per query: the k-th smallest upper bound of the block's 64 vectors (a
        // bitonic sort over the query's 16 lanes x 4 registers). k vectors of the list have
        // exact distances at or below it, so it is a valid shared threshold: published to the
        // item's and the list-wide thresholds at once, so that every segment of the list that
        // starts later (or reads them at its next block) prunes against it.
        // (Published only where it improves on the current list-wide value: a hub list's
        // blocks would otherwise serialise on the same few addresses.)
        float tb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int g = 4 * (lane >> 4) + r;
            const uint32_t* gt = a.thr + it.pair_start + q0 + min(g, nq - 1);
            // thr4: per (query, list) the smallest ceil(k/4)-th distance any item of residue
            // s (item index mod 4) reached, for s = 0..3. Four distinct items hold ceil(k/4)
            // vectors each at or below the largest of the four: a valid shared threshold,
            // nearer the k-th of the union of the items' lists than the min of their k-ths
            // (a.thr) when several items of one list run at once. (m = 2, 4, 8 slots together
            // measured no better.)
            const uint4 t4 = *(const uint4*)(a.thr4 + (size_t)(it.pair_start + q0 + min(g, nq - 1)) * 4);
            const float th4 = fmaxf(fmaxf(ord_dec(t4.x), ord_dec(t4.y)), fmaxf(ord_dec(t4.z), ord_dec(t4.w)));
            const float cur = fminf(fminf(ord_dec(*gt), th4), ord_dec(s_thr[min(g, nq - 1)]));
            const float t = block_kth(ubv[r], k);
            if ((lane & 15) == 0 && g < nq && t < cur) {
                atomicMin(&s_thr[g], ord_enc(t));
                atomicMin((uint32_t*)gt, ord_enc(t));
            }
            tb[r] = fminf(t, cur);
        }
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) {
            const uint32_t v = j * 64 + 16 * vt + (lane & 15);
            const bool valid = v < nv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int g = 4 * (lane >> 4) + r;
                // (re-read per tile: the exact rounds of the previous tile lower them)
                const float th = g < nq ? fminf(tb[r], fminf(kdl[g], ord_dec(s_thr[g]))) : -__builtin_inff();
                const bool cand = valid && g < nq && !(acc[vt][r] > th);
                const uint64_t m = __ballot(cand);
                if (cand) {
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    ring[(tail + below) & (kRing - 1)] = ((uint32_t)g << 16) | v;
                }
                tail += (uint32_t)__popcll(m);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            // full rounds as they fill (the list registers in flight leave room for a shallow
            // load pipeline); the segment's remainder after the stream, with a deep one
            if (VDB_SCREEN_DIAG & 1) head = tail;
            while (tail - head >= 64) exact_round(64u, std::integral_constant<int, kExactPipe>{});
        }
    }
    while (tail != head) exact_round(min(64u, tail - head), std::integral_constant<int, kExactPipeEnd>{});
    if (a.mstats && lane == 0) atomicAdd(&a.mstats[1], (unsigned long long)nb);
}

// The partials of segment `seg` for the item's nq queries: the wave's top-k lists (`keep`),
// or empty (inf, no id) for a segment whose vectors live on in the wave's lists and reach
// the merge through a later segment's partial. Every vector the wave scanned is in exactly
// one partial, so the merge's multiset top-min(k, n_l) of the union is the list's.
__device__ __forceinline__ void screen_partials(const ScanArgs& a, const ScanItem it, const int q0, const int nq,
                                                const uint32_t seg, const float* tk_d, const uint64_t* tk_i,
                                                const bool keep) {
    const int lane = lane_id();
    const int k = (int)a.k;
    for (int g = 0; g < nq; ++g) {
        const uint32_t part = a.part_base_sorted[it.pair_start + q0 + g] + seg;
        if (lane < k) {
            a.part_d[(size_t)part * k + lane] = keep ? tk_d[g * k + lane] : __builtin_inff();
            a.part_i[(size_t)part * k + lane] = keep ? tk_i[g * k + lane] : kNoId;
        }
    }
}

// Per-wave dynamic LDS: tk_i [16 k] u64 | tk_d [16 k] f32 | kdl [16] f32 | s_thr [16] u32 | ring [kRing] u32.
__host__ __device__ constexpr size_t screen_wave_lds(uint32_t k) { return (size_t)16 * k * 12 + 64 + 64 + kRing * 4; }
// Per-workgroup dynamic LDS ahead of the waves' areas: the wide item's shared lists for up to
// wq (16 or 32) queries: tk_i [wq k] u64 | tk_d [wq k] f32 | kdl [wq] f32 | locks [wq] u32.
__host__ __device__ constexpr size_t screen_item_lds(uint32_t k, uint32_t wq) { return (size_t)wq * (k * 12 + 8); }

// ivf_scan_screen: persistent grid (two 4-wave workgroups per CU) over the plan's queues,
// like ivf_scan_wide: wide items (a list's segments x <= a.wide_q queries; the 4 waves take
// the segments dynamically and share the item's lists and thresholds), then narrow items
// (one wave each: one segment x <= 4 queries). The last a.fused workgroups start on the
// narrow queue. An item of 17-32 queries splits its waves in two halves of 16 queries that
// take the item's segments in the same order, side by side on the CU: the list's shadow is
// read from HBM once for both halves (the second read is served by the L2).
template <int M, int KD>
__global__ __launch_bounds__(256, 2) void ivf_scan_screen(ScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t slds[];
    const uint32_t wv = wave_index();
    // the wide item's lists, shared by its 4 waves (each query's top-k over every segment the
    // item's waves scan: its k-th tightens 4x faster than one wave's)
    const uint32_t wq = a.wide_q;
    uint64_t* it_i = slds;
    float* it_d = (float*)(slds + wq * a.k);
    float* it_kd = it_d + wq * a.k;
    uint32_t* it_lock = (uint32_t*)(it_kd + wq);
    char* base = (char*)slds + screen_item_lds(a.k, wq) + (size_t)wv * screen_wave_lds(a.k);
    uint64_t* tk_i = (uint64_t*)base;
    float* tk_d = (float*)(base + (size_t)16 * a.k * 8);
    float* kdl = tk_d + 16 * a.k;
    uint32_t* s_thr_w = (uint32_t*)(kdl + 16);
    uint32_t* ring = s_thr_w + 16;
    __shared__ uint32_t s_next, s_seg[2];
    __shared__ uint32_t s_thr[32];
    const int lane = lane_id();

    auto drain_narrow = [&]() {
        const uint32_t n_narrow = a.counters[0];
        for (;;) {
            uint32_t idx = 0;
            if (lane == 0) idx = atomicAdd(&a.work[0], 1u);
            idx = __builtin_amdgcn_readfirstlane(idx);
            if (idx >= n_narrow) break;
            ScanItem it = a.items[idx];
            it.list = __builtin_amdgcn_readfirstlane(it.list);
            it.seg = __builtin_amdgcn_readfirstlane(it.seg);
            it.pair_start = __builtin_amdgcn_readfirstlane(it.pair_start);
            it.npairs = __builtin_amdgcn_readfirstlane(it.npairs);
            if (lane < (int)it.npairs) s_thr_w[lane] = a.thr[it.pair_start + lane];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            screen_segment<M, KD>(a, it, 0, (int)it.npairs, it.seg, tk_d, tk_i, kdl, s_thr_w, ring, true, nullptr,
                                  it.seg);
            screen_partials(a, it, 0, (int)it.npairs, it.seg, tk_d, tk_i, true);
        }
    };

    const uint32_t n_wide = a.counters[3];
    uint32_t stride = a.wide_stride;
    if (stride > 1 && n_wide % stride == 0) stride = stride == 40009u ? 40013u : 40009u;
    if (a.fused && blockIdx.x + a.fused >= gridDim.x) drain_narrow();
    for (;;) {
        if (threadIdx.x == 0) s_next = atomicAdd(&a.work[1], 1u);
        __syncthreads();
        const uint32_t b = s_next;
        if (b >= n_wide) break;
        const uint32_t item = stride > 1 ? (uint32_t)(((uint64_t)b * stride) % n_wide) : b;
        ScanItem it = a.items_w[item];
        it.list = __builtin_amdgcn_readfirstlane(it.list);
        it.seg = __builtin_amdgcn_readfirstlane(it.seg);
        it.pair_start = __builtin_amdgcn_readfirstlane(it.pair_start);
        it.npairs = __builtin_amdgcn_readfirstlane(it.npairs);
        const int nq = (int)it.npairs;
        if (threadIdx.x < 2) s_seg[threadIdx.x] = 0;
        if (threadIdx.x < (uint32_t)nq) s_thr[threadIdx.x] = a.thr[it.pair_start + threadIdx.x];
        for (uint32_t e = threadIdx.x; e < (uint32_t)nq * a.k; e += blockDim.x) {
            it_d[e] = __builtin_inff();
            it_i[e] = kNoId;
        }
        if (threadIdx.x < (uint32_t)nq) {
            it_kd[threadIdx.x] = __builtin_inff();
            it_lock[threadIdx.x] = 0u;
        }
        __syncthreads();
        const uint32_t seg_vectors = a.seg_blocks * 64;
        const uint32_t nseg = (a.count[it.list] + seg_vectors - 1) / seg_vectors;
        const uint32_t seg0 = it.seg * a.segs_item, seg1 = min(nseg, seg0 + a.segs_item);
        // The item's waves insert into its shared lists; every segment gets empty partials,
        // then the item's first segment the lists (every scanned vector is in exactly one
        // partial, so the merge's multiset top-min(k, n_l) of the union is unchanged).
        const bool split = nq > 16;
        const uint32_t half = split ? wv >> 1 : 0u;
        const int nq0 = split ? (nq + 1) / 2 : nq;  // (balanced halves)
        const int q0 = half ? nq0 : 0, nqh = half ? nq - nq0 : nq0;
        const int ko = q0 * (int)a.k;
        for (;;) {
            uint32_t sg = 0;
            if (lane == 0) sg = atomicAdd(&s_seg[half], 1u);
            sg = seg0 + __builtin_amdgcn_readfirstlane(sg);
            if (sg >= seg1) break;
            screen_segment<M, KD>(a, it, q0, nqh, sg, it_d + ko, it_i + ko, it_kd + q0, s_thr + q0, ring, false,
                                  it_lock + q0, it.seg);
            screen_partials(a, it, q0, nqh, sg, it_d + ko, it_i + ko, false);
        }
        __syncthreads();
        if ((wv & 1) == 0 && (wv == 0 || split)) screen_partials(a, it, q0, nqh, seg0, it_d + ko, it_i + ko, true);
        // (the next item's first barrier orders this before the lists are reset)
    }
    if (a.fused) drain_narrow();
}

// ============================================================================
// The DEFERRED screened scan (default): screen every pair, re-check later, only what the
// list's final threshold leaves.
//
// The inline kernel above re-checks a candidate the moment it passes the threshold the
// wave knows at that point; early in a segment that threshold is loose, so most of its
// re-checks (~200 per (query, list) pair at the headline) are of vectors that later turn
// out to be far from the list's top-k. Here the scan only COLLECTS candidates:
//  * thresholds come from upper bounds alone: every wave keeps, per query, the 64
//    smallest upper bounds (approx + delta) of the vectors it has screened in its item as
//    a sorted list in registers (16 lanes x 4 of the query's DPP row; each block's 64 upper
//    bounds are bitonic-sorted and merged in). k vectors of the list have exact distances
//    at or below the list's k-th element, so it is a valid shared threshold: published to
//    the item (LDS) and list-wide (a.thr) like the inline scan's exact k-th, and its
//    ceil(k/4)-th into the quarter slot of the wave's residue (the 4 waves of a wide item
//    hold 4 distinct residues, so thr4's maximum is a valid threshold too);
//  * a pair is collected unless lower bound > th (the inline test): (sorted pair, slot,
//    lower bound) appended to a.cand (per-wave chunks reserved a block ahead); beyond the capacity the
//    pair is marked overflowed;
//  * every segment's partials are written empty.
// Then (ivf_screen_filter / _offsets / _scatter / _recheck) each collected pair is kept
// only if its lower bound is not above the pair's FINAL threshold (min of a.thr and thr4's
// maximum after the whole list was screened: still >= the list's exact k-th distance, so
// every member of the list's top-min(k, n) survives), the survivors are grouped per pair,
// and one wave per (query, list) pair recomputes them with the reference's sequential sum
// and writes the pair's exact top-k as its first segment partial. On iid 768-D data a
// pair then re-checks ~k + a few vectors (the vectors within 2 delta of its k-th
// distance) instead of ~200. An overflowed pair is recomputed exactly over its whole list.
// ============================================================================

// Ascending 64-element bitonic sort of u (the 16 lanes x 4 registers of each DPP row).
__device__ __forceinline__ void block_sort64(float (&u)[4]) {
    const int l = lane_id() & 15;
    bitonic64_step<2, 1>(u, l);
    bitonic64_step<4, 2>(u, l), bitonic64_step<4, 1>(u, l);
    bitonic64_step<8, 4>(u, l), bitonic64_step<8, 2>(u, l), bitonic64_step<8, 1>(u, l);
    bitonic64_step<16, 8>(u, l), bitonic64_step<16, 4>(u, l), bitonic64_step<16, 2>(u, l), bitonic64_step<16, 1>(u, l);
    bitonic64_step<32, 16>(u, l), bitonic64_step<32, 8>(u, l), bitonic64_step<32, 4>(u, l);
    bitonic64_step<32, 2>(u, l), bitonic64_step<32, 1>(u, l);
    bitonic64_step<64, 32>(u, l), bitonic64_step<64, 16>(u, l), bitonic64_step<64, 8>(u, l);
    bitonic64_step<64, 4>(u, l), bitonic64_step<64, 2>(u, l), bitonic64_step<64, 1>(u, l);
}
// rl (sorted ascending) <- the 64 smallest of rl and u (both sorted ascending), sorted:
// min(rl[e], u[63 - e]) is bitonic; one merge pass sorts it. Element e = 4 (lane & 15) + v;
// 63 - e is lane 15 - (lane & 15) (DPP row mirror), register 3 - v.
__device__ __forceinline__ void merge_sorted64(float (&rl)[4], const float (&u)[4]) {
    const int l = lane_id() & 15;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const float rv = __uint_as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)__float_as_uint(u[3 - v]), 0x140, 0xF,
                                                                            0xF, false));
        rl[v] = fminf(rl[v], rv);
    }
    bitonic64_step<64, 32>(rl, l), bitonic64_step<64, 16>(rl, l), bitonic64_step<64, 8>(rl, l);
    bitonic64_step<64, 4>(rl, l), bitonic64_step<64, 2>(rl, l), bitonic64_step<64, 1>(rl, l);
}
// Element e (wave-uniform, 0..63) of each DPP row's sorted list, in every lane of the row.
__device__ __forceinline__ float row_elem(const float (&u)[4], int e) {
    const int v = e & 3;
    const float x = v == 0 ? u[0] : v == 1 ? u[1] : v == 2 ? u[2] : u[3];
    return __shfl(x, (lane_id() & ~15) + (e >> 2));
}

// Candidate slots of one wave: a.cand entries are reserved in chunks of kCandChunk (one atomic
// on the batch's counter per chunk), the next chunk's atomic issued one block ahead of its use,
// so no block's epilogue waits on a returning global access (vmcnt is in order: it would wait
// for the next block's shadow prefetches too). A block's candidates fill the current chunk to
// its end and continue in the next (round 6: round 5 padded the rest of a chunk whenever a
// block's candidates did not fit, up to half the entries the filter then read); the wave's
// unused rest at its end is filled with sentinel entries {~0, 0, 0, ~0} (never kept).
// (kCandChunk: kernels.hpp.) Reserved slots (counters[kCtrCand]) therefore exceed the candidates
// (counters[kCtrReal], added once per wave at its end): the overflow, floor, calibration and
// re-run decisions read kCtrOvf / kCtrReal, never the reserved count.
struct CandChunk {
    uint32_t base = 0, left = 0;  // (wave-uniform) the current chunk's next entry and entries left
    uint32_t next = 0;            // (wave-uniform) the first entry of the chunk reserved ahead
    uint32_t real = 0;            // (wave-uniform) candidates this wave collected
    bool pending = false;
};
__device__ __forceinline__ void pad_cand(const ScanArgs& a, uint32_t base, uint32_t n) {
    for (uint32_t i = (uint32_t)lane_id(); i < n; i += 64)
        if (base + i < a.cand_cap) a.cand[base + i] = make_uint4(~0u, 0u, 0u, ~0u);
}
__device__ __forceinline__ void finish_cand(const ScanArgs& a, CandChunk& cc) {
    pad_cand(a, cc.base, cc.left);
    if (cc.pending) pad_cand(a, cc.next, kCandChunk);
    if (cc.real && lane_id() == 0) atomicAdd(a.ccount + (kCtrReal - kCtrCand), cc.real);
    cc.left = 0;
    cc.real = 0;
    cc.pending = false;
}

// One wave: collect the candidates of segment `seg` of list it.list for the nq (<= 16 NG)
// queries of the item starting at sorted pair it.pair_start + q0. NG = 2 (items of 17-32
// queries): every shadow B tile the wave loads feeds two A operands (queries 0-15 and
// 16-31: 8 MFMAs per k-step), so a list is streamed once per 32 queries, not per 16.
// rl_lds: the wave's running lists of upper bounds (NG x 4 query rows; reset by the caller
// per item); s_thr: the item's shared k-th (LDS); s_pst / s_qsc: the item's per-query pair
// norms and int8 scales (LDS, loaded by the caller); s_mt / s_vs: the wave's LDS scratch for
// one block's vector norms and scales; residue: the wave's quarter slot (0..3, distinct per
// wave of an item); cc: the wave's candidate chunk.
template <int M, int KD, int NG, bool I8, bool W2>
__device__ __forceinline__ void collect_segment(const ScanArgs& a, const ScanItem it, const int q0, const int nq,
                                                const uint32_t seg, float4* rl_lds, uint32_t* s_thr,
                                                const float4* s_pst, const float* s_qsc, float4* s_mt, float* s_vs,
                                                const uint32_t residue, CandChunk& cc) {
    const int lane = lane_id();
    const uint32_t dp = a.dp, ks = dp >> (I8 ? 6 : 5);  // (k-steps of 64 int8 or 32 bf16 dims)
    const uint32_t count = a.count[it.list];
    const uint32_t seg_vectors = a.seg_blocks * 64;
    const uint64_t b0 = a.block_off[it.list] + (uint64_t)seg * a.seg_blocks;
    const uint32_t v0 = seg * seg_vectors;
    const uint32_t nv = min(count - v0, seg_vectors);
    const uint32_t nb = (nv + 63) >> 6;
    const int k = (int)a.k, kq = ((int)a.k + 3) / 4;
    const uint32_t* pairs = a.sorted_pair + it.pair_start + q0;
    const float cm = (float)(4 * dp + 16) * 0x1.02p-24f;
    const float cr = (float)(dp + 2) * 0x1.02p-24f;
    const float cu = 0x1.02p-23f;
    auto pair_of = [&](int g) -> uint32_t {
        const uint32_t pr = pairs[g];
        return (pr >> 16) * a.P + (pr & 0xFFFFu);
    };
    // the MFMA A rows of this lane: query 16 gg + (lane & 15) of group gg, its dims 8 (lane >> 4) ..
    const uint4* qa_row[NG];
#pragma unroll
    for (int gg = 0; gg < NG; ++gg)
        qa_row[gg] = (const uint4*)((const char*)a.qres + (size_t)pair_of(min(16 * gg + (lane & 15), nq - 1)) * dp *
                                                              (I8 ? 1 : 2)) +
                     (lane >> 4);
    uint32_t collected = 0;
    // the shared thresholds (list-wide k-th, quarter slots) as last read, refreshed every
    // thr_every blocks (a stale value is larger, so only looser: still valid); the 32-query
    // variant also keeps them across blocks (its one workgroup per CU has the registers)
    float gthr[NG][4], gq4[NG][4];  // (and this wave's quarter slot)
#pragma unroll
    for (int gg = 0; gg < NG; ++gg)
#pragma unroll
        for (int r = 0; r < 4; ++r) gthr[gg][r] = gq4[gg][r] = __builtin_inff();
    const uint32_t thr_every = W2 ? a.thr_every : 1u;
    // the pair whose shared thresholds this lane fetches (query lane mod 16 NG of the item)
    const uint32_t spl = it.pair_start + q0 + min(lane & (16 * NG - 1), nq - 1);

    const uint4* sp = a.shadow + b0 * (uint64_t)ks * 256 + lane;
    uint4 xa[KD][4], qa[NG][KD];
#pragma unroll
    for (int u = 0; u < KD; ++u) {
#pragma unroll
        for (int vt = 0; vt < 4; ++vt) xa[u][vt] = ld_nt_u4(sp + (size_t)(u * 4 + vt) * 64);
#pragma unroll
        for (int gg = 0; gg < NG; ++gg) qa[gg][u] = qa_row[gg][4 * (u % ks)];
    }
    using AccT = std::conditional_t<I8, i32x4, f32x4>;
    for (uint32_t j = 0; j < nb; ++j) {
        // The block's epilogue operands are issued ahead of its k-steps, so the epilogue waits
        // on no global access: lane l's vector norms (and int8 scale), the shared thresholds
        // of query l mod 16 NG, and the wave's next candidate chunk when the current one runs low
        const uint64_t mslot = (b0 + j) * 64 + lane;
        const float4 mt_l = a.meta[mslot];
        float vs_l = 0.0f;
        if constexpr (I8) vs_l = a.sscale[mslot];
        const bool thr_now = j % thr_every == 0;
        uint32_t gt_l = 0u;
        uint4 t4_l = make_uint4(0u, 0u, 0u, 0u);
        if (thr_now) {
            gt_l = a.thr[spl];
            t4_l = *(const uint4*)(a.thr4 + (size_t)spl * 4);
        }
        // (its reply is read at this block's epilogue: a reply held across blocks made the
        // compiler wait for every load in flight before reading it)
        const bool reserve = !cc.pending && cc.left < kCandChunk / 2;
        uint32_t reply = 0;
        if (reserve && lane == 0) reply = atomicAdd(a.ccount, kCandChunk);
        AccT acc[NG][4];
#pragma unroll
        for (int gg = 0; gg < NG; ++gg)
#pragma unroll
            for (int vt = 0; vt < 4; ++vt) acc[gg][vt] = AccT{0, 0, 0, 0};
        for (uint32_t s0 = 0; s0 < ks; s0 += KD) {
            static_for<0, KD>([&](auto uu) {
                constexpr int u = decltype(uu)::value;
#pragma unroll
                for (int gg = 0; gg < NG; ++gg) {
                    if constexpr (I8) {
                        const i32x4 A = as_i32x4(qa[gg][u]);
#pragma unroll
                        for (int vt = 0; vt < 4; ++vt)
                            acc[gg][vt] =
                                __builtin_amdgcn_mfma_i32_16x16x64_i8(A, as_i32x4(xa[u][vt]), acc[gg][vt], 0, 0, 0);
                    } else {
                        const bf16x8 A = as_bf16x8(qa[gg][u]);
#pragma unroll
                        for (int vt = 0; vt < 4; ++vt)
                            acc[gg][vt] =
                                __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, as_bf16x8(xa[u][vt]), acc[gg][vt], 0, 0, 0);
                    }
                }
                const uint64_t nxt = (uint64_t)j * ks + s0 + u + KD;
#pragma unroll
                for (int vt = 0; vt < 4; ++vt) xa[u][vt] = ld_nt_u4(sp + (nxt * 4 + vt) * 64);
#pragma unroll
                for (int gg = 0; gg < NG; ++gg) qa[gg][u] = qa_row[gg][4 * ((s0 + u + KD) % ks)];
            });
        }
        // (vector 16 vt + (lane & 15)'s norms are read from the wave's scratch below)
        s_mt[lane] = mt_l;
        if constexpr (I8) s_vs[lane] = vs_l;
        if (reserve) {
            cc.next = __builtin_amdgcn_readfirstlane(reply);
            cc.pending = true;
        }
        float gthr_l = 0.0f, gq4_l = 0.0f;
        if (thr_now) {
            const float th4 =
                fmaxf(fmaxf(ord_dec(t4_l.x), ord_dec(t4_l.y)), fmaxf(ord_dec(t4_l.z), ord_dec(t4_l.w)));
            gthr_l = fminf(ord_dec(gt_l), th4);
            gq4_l = ord_dec(residue == 0 ? t4_l.x : residue == 1 ? t4_l.y : residue == 2 ? t4_l.z : t4_l.w);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int gg = 0; gg < NG; ++gg) {
            const int g0 = 16 * gg;  // this group's first query of the item
            // lower bounds into acc, upper bounds into ubv (the inline kernel's bound)
            float ubv[4][4];
            float4 pst[4];
            float qsc[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gc = min(g0 + 4 * (lane >> 4) + r, nq - 1);
                pst[r] = s_pst[gc];
                if constexpr (I8) qsc[r] = s_qsc[gc];
            }
#pragma unroll
            for (int vt = 0; vt < 4; ++vt) {
                const float4 mt = s_mt[16 * vt + (lane & 15)];
                float vsc = 0.0f;
                if constexpr (I8) vsc = s_vs[16 * vt + (lane & 15)];
                const bool valid = j * 64 + 16 * vt + (lane & 15) < nv;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // (int8: <a', b'> = s_a s_b <q_a, q_b>, the integer sum exact; the two float
                    // roundings are far inside the MFMA accumulation term cm below)
                    float dot;
                    if constexpr (I8) dot = (float)acc[gg][vt][r] * (qsc[r] * vsc);
                    else dot = acc[gg][vt][r];
                    const float4 ps = pst[r];
                    const float approx = M == kL2 ? (ps.x + mt.x) - 2.0f * dot : -(ps.x + dot);
                    const float an = ps.y + ps.z, bn = mt.y + mt.z;
                    const float cs = an * mt.z + ps.z * bn + ps.z * mt.z;
                    float del;
                    if (M == kL2) {
                        const float rest = 2.0f * (cs + cm * (an * bn)) + cu * (ps.x + mt.x + fabsf(approx));
                        del = rest + cr * (fabsf(approx) + rest);
                    } else {
                        del = cs + cm * (an * bn) + cr * (ps.y * mt.w) + cu * (ps.y * ps.w + an * bn + fabsf(approx));
                    }
                    del = del * 1.001f + 1e-30f;
                    const float ub = approx + del;
                    if constexpr (I8) acc[gg][vt][r] = __float_as_int(approx - del);  // (the lower bound, in place)
                    else acc[gg][vt][r] = approx - del;
                    ubv[r][vt] = valid && ub == ub ? ub : __builtin_inff();
                }
            }
            // per query row: the block's sorted upper bounds into the running list; its k-th
            // (and ceil(k/4)-th) published; th = the smallest valid threshold known. A block
            // none of whose upper bounds is below any row's current k-th cannot change those
            // rows' first k elements (the only ones used): its sort and merge are skipped (the
            // list's elements k .. 63 may then go stale; elements 0 .. k-1 stay exact)
            float th[4], pub_t[4], pub_q[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int g = g0 + 4 * (lane >> 4) + r;
                const int gc = min(g, nq - 1);
                float4* rlp = rl_lds + (gg * 4 + r) * 64 + lane;
                const float4 rv = *rlp;
                float rl[4] = {rv.x, rv.y, rv.z, rv.w};
                float tw = row_elem(rl, k - 1), tq = row_elem(rl, kq - 1);
                if (thr_now) {  // (lane gc fetched query gc's)
                    const float gn = __shfl(gthr_l, gc), qn = __shfl(gq4_l, gc);
                    if constexpr (W2) {
                        gthr[gg][r] = fminf(gthr[gg][r], gn);
                        gq4[gg][r] = fminf(gq4[gg][r], qn);
                    } else {
                        gthr[gg][r] = gn;
                        gq4[gg][r] = qn;
                    }
                }
                const float cur = fminf(gthr[gg][r], ord_dec(s_thr[gc]));
                // Only upper bounds below min(tw, cur) are kept: one at or above a valid shared
                // threshold cannot lower any threshold, and the union of the contributed lists
                // already holds k upper bounds at or below cur (those of the waves that
                // published it), so its k-th is unchanged (ivf_screen_tfinal). A block with
                // none skips its sort and merge.
                const float bmin = fminf(fminf(ubv[r][0], ubv[r][1]), fminf(ubv[r][2], ubv[r][3]));
                if (__ballot(bmin < fminf(tw, cur))) {
                    block_sort64(ubv[r]);
                    merge_sorted64(rl, ubv[r]);
                    *rlp = make_float4(rl[0], rl[1], rl[2], rl[3]);
                    tw = row_elem(rl, k - 1);
                    tq = row_elem(rl, kq - 1);
                }
                // (published below by the lane of query g: no per-row addresses held)
                pub_t[r] = tw < cur ? tw : __builtin_inff();
                pub_q[r] = tq < gq4[gg][r] ? tq : __builtin_inff();
                gthr[gg][r] = fminf(gthr[gg][r], tw);
                gq4[gg][r] = fminf(gq4[gg][r], tq);
                th[r] = g < nq ? fminf(tw, cur) : -__builtin_inff();
            }
            {  // lane 16 gg + q publishes query g0 + q's new k-th / quarter k-th (row q / 4, element q % 4)
                const int lq = lane & 15, src = 16 * (lq >> 2), rs = lq & 3;
                float pt = __builtin_inff(), pq = __builtin_inff();
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t = __shfl(pub_t[r], src), q = __shfl(pub_q[r], src);
                    if (rs == r) pt = t, pq = q;
                }
                if ((lane >> 4) == gg && g0 + lq < nq) {  // (then spl is this query's sorted pair)
                    if (pt < __builtin_inff()) {
                        atomicMin(&s_thr[g0 + lq], ord_enc(pt));
                        atomicMin(a.thr + spl, ord_enc(pt));
                    }
                    if (pq < __builtin_inff()) atomicMin(a.thr4 + (size_t)spl * 4 + residue, ord_enc(pq));
                }
            }
            // candidates: the wave's whole batch of them for this block and group into its chunk
            // (the ballots are recomputed for the writes rather than held: registers)
            auto lbv = [&](int vt, int r) -> float {
                if constexpr (I8) return __int_as_float(acc[gg][vt][r]);
                else return acc[gg][vt][r];
            };
            auto is_cand = [&](int vt, int r) {
                return j * 64 + 16 * vt + (lane & 15) < nv && g0 + 4 * (lane >> 4) + r < nq && !(lbv(vt, r) > th[r]);
            };
            uint32_t tot = 0;
#pragma unroll
            for (int vt = 0; vt < 4; ++vt)
#pragma unroll
                for (int r = 0; r < 4; ++r) tot += (uint32_t)__popcll(__ballot(is_cand(vt, r)));
            if (tot) {
                // the block's candidates take ranks 0 .. tot-1: the first cn0 go to [cb0, cb0 + cn0),
                // the rest to [cb1, ..): the current chunk is filled to its end and the next one
                // continues it, so no entry is left unused except at a wave's very end
                uint32_t cb0, cn0, cb1 = 0;  // (cb0: not the segment's first block b0)
                if (tot <= cc.left) {
                    cb0 = cc.base;
                    cn0 = tot;
                    cc.base += tot;
                    cc.left -= tot;
                } else if (tot > kCandChunk) {  // (a range of its own; the current chunk stays)
                    uint32_t v = 0;
                    if (lane == 0) v = atomicAdd(a.ccount, tot);
                    cb0 = __builtin_amdgcn_readfirstlane(v);
                    cn0 = tot;
                } else {  // the current chunk's rest, then the chunk reserved ahead
                    cb0 = cc.base;
                    cn0 = cc.left;
                    uint32_t v = 0;
                    if (cc.pending) {
                        cb1 = cc.next;
                        cc.pending = false;
                    } else {
                        if (lane == 0) v = atomicAdd(a.ccount, kCandChunk);
                        cb1 = __builtin_amdgcn_readfirstlane(v);
                    }
                    cc.base = cb1 + (tot - cn0);
                    cc.left = kCandChunk - (tot - cn0);
                }
                collected += tot;
                cc.real += tot;
                uint32_t rank = 0;
#pragma unroll
                for (int vt = 0; vt < 4; ++vt) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const bool c = is_cand(vt, r);
                        const uint64_t mm = __ballot(c);
                        if (c) {
                            const uint32_t rk = rank + __builtin_amdgcn_mbcnt_hi(
                                                           (uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                            const uint32_t idx = rk < cn0 ? cb0 + rk : cb1 + (rk - cn0);
                            const uint32_t spi = it.pair_start + q0 + g0 + 4 * (lane >> 4) + r;
                            const uint32_t slot = (uint32_t)((b0 + j) * 64 + 16 * vt + (lane & 15));
                            if (idx < a.cand_cap)
                                a.cand[idx] = make_uint4(spi, slot, __float_as_uint(lbv(vt, r)), 0u);
                            else {
                                a.ovf[spi] = 1u;  // (any store of 1: idempotent)
                                a.ccount[kCtrOvf - kCtrCand] = 1u;
                            }
                        }
                        rank += (uint32_t)__popcll(mm);
                    }
                }
            }
        }
    }
    if (a.mstats && lane == 0) {
        atomicAdd(&a.mstats[0], (unsigned long long)collected);
        atomicAdd(&a.mstats[1], (unsigned long long)nb);
    }
}

// (LDS audit) An item wider than the collect kernel's per-item LDS (s_thr, s_pst,
// s_qsc: 32 queries for a wide item, 16 per wave for a narrow one) is never planned (the
// plan kernel's items carry <= wide_q queries; launch_plan and launch_screen_collect check
// the widths on the host). Should one arrive anyway, its pairs are marked overflowed, which
// sends them to the exact recomputation over their planned segments (ivf_screen_pair_topk)
// instead of writing past the arrays: results stay exact.
__device__ __forceinline__ void overflow_item(const ScanArgs& a, uint32_t pair_start, uint32_t npairs, uint32_t t0,
                                              uint32_t nt) {
    for (uint32_t t = t0; t < npairs; t += nt) a.ovf[pair_start + t] = 1u;
    if (t0 == 0) a.ccount[kCtrOvf - kCtrCand] = 1u;
}

__device__ __forceinline__ void reset_rl(float4* rl_lds, int rows) {
    const int lane = lane_id();
    const float inf = __builtin_inff();
    for (int r = 0; r < rows; ++r) rl_lds[r * 64 + lane] = make_float4(inf, inf, inf, inf);
}

// The wave's running lists of the item's nq queries (the k smallest upper bounds of the
// vectors it screened) appended to their pairs' contributions (a.ublist: per sorted pair
// kUbLists lists of k; a.ubcnt: how many were offered). Every contribution covers vectors
// no other contribution covers, so the k-th smallest of their union is a valid threshold
// (ivf_screen_tfinal); a list beyond the capacity is dropped, which only loosens it.
__device__ __forceinline__ void contribute_rl(const ScanArgs& a, const ScanItem it, const int q0, const int nq,
                                              const float4* rl_lds) {
    const int lane = lane_id();
    const int k = (int)a.k;
    for (int r = 0; r < (nq + 15) / 16 * 4; ++r) {  // (query rows: 4 per group of 16)
        const int g = 16 * (r >> 2) + 4 * (lane >> 4) + (r & 3);
        const uint32_t spi = it.pair_start + q0 + min(g, nq - 1);
        uint32_t slot = 0;
        if ((lane & 15) == 0 && g < nq) slot = atomicAdd(&a.ubcnt[spi], 1u);
        slot = __shfl(slot, lane & ~15);
        const float4 rv = rl_lds[r * 64 + lane];
        const float rl[4] = {rv.x, rv.y, rv.z, rv.w};
        if (g < nq && slot < (uint32_t)kUbLists) {
            float* dst = a.ublist + ((size_t)spi * kUbLists + slot) * k;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int e = 4 * (lane & 15) + v;
                if (e < k) dst[e] = rl[v];
            }
        }
    }
}

// (option collect_stamps) one timeline record of the collect kernel
__device__ __forceinline__ void put_stamp(const ScanArgs& a, uint64_t w0, uint64_t t0, uint64_t w3) {
    const uint32_t i = atomicAdd((unsigned int*)a.stamps, 1u);
    if (i < a.stamps_cap) {
        unsigned long long* r = a.stamps + 2 + (size_t)i * 4;
        r[0] = ((uint64_t)a.stamp_batch << 40) | w0;
        r[1] = t0;
        r[2] = wall_clock64();
        r[3] = w3;
    }
}

// ivf_screen_collect: the persistent grid of ivf_scan_screen over the same queues (wide
// items: a list's segments x <= a.wide_q (16 or 32) queries, the 4 waves taking the
// segments dynamically; narrow items: one wave = one segment x <= 4 queries), collecting
// instead of re-checking. W2: items of up to 32 queries (two A operands per shadow tile: the
// registers of one workgroup per CU; otherwise two).
template <int M, int KD, bool W2, bool I8>
__global__ __launch_bounds__(256, W2 ? 1 : 2) void ivf_screen_collect(ScanArgs a) {
    __shared__ uint32_t s_next, s_seg;
    __shared__ uint32_t s_thr[32];
    __shared__ uint32_t s_thr_w[4][16];
    __shared__ float4 s_rl[4][8 * 64];  // each wave's running lists (up to 2 groups x 4 query rows x 64 lanes)
    __shared__ float4 s_pst[32], s_pst_w[4][16];  // the item's pair norms (wide: shared; narrow: per wave)
    __shared__ float s_qsc[32], s_qsc_w[4][16];   // ... and int8 scales
    __shared__ float4 s_mt[4][64];                // each wave's scratch: one block's vector norms
    __shared__ float s_vs[4][64];                 // ... and int8 scales
    const uint32_t wv = wave_index();
    const int lane = lane_id();
    float4* rl = s_rl[wv];
    CandChunk cc;
    // (per-query pair norms of the item starting at sorted pair ps, query t)
    auto pair_stats = [&](uint32_t ps, uint32_t t, float4* dp4, float* dsc) {
        const uint32_t pr = a.sorted_pair[ps + t];
        const uint32_t pi = (pr >> 16) * a.P + (pr & 0xFFFFu);
        dp4[t] = a.pst[pi];
        if (I8) dsc[t] = a.qscale[pi];
    };

    auto drain_narrow = [&]() {
        const uint32_t n_narrow = a.counters[0];
        for (;;) {
            uint32_t idx = 0;
            if (lane == 0) idx = atomicAdd(&a.work[0], 1u);
            idx = __builtin_amdgcn_readfirstlane(idx);
            if (idx >= n_narrow) break;
            ScanItem it = a.items[idx];
            it.list = __builtin_amdgcn_readfirstlane(it.list);
            it.seg = __builtin_amdgcn_readfirstlane(it.seg);
            it.pair_start = __builtin_amdgcn_readfirstlane(it.pair_start);
            it.npairs = __builtin_amdgcn_readfirstlane(it.npairs);
            if (it.npairs > 16u) {  // (never planned: see overflow_item)
                overflow_item(a, it.pair_start, it.npairs, (uint32_t)lane, 64u);
                continue;
            }
            if (lane < (int)it.npairs) {
                s_thr_w[wv][lane] = a.thr[it.pair_start + lane];
                pair_stats(it.pair_start, lane, s_pst_w[wv], s_qsc_w[wv]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const uint64_t t0 = a.stamps ? wall_clock64() : 0;
            reset_rl(rl, 4);
            collect_segment<M, KD, 1, I8, W2>(a, it, 0, (int)it.npairs, it.seg, rl, s_thr_w[wv], s_pst_w[wv],
                                              s_qsc_w[wv], s_mt[wv], s_vs[wv], it.seg & 3u, cc);
            contribute_rl(a, it, 0, (int)it.npairs, rl);
            if (a.stamps && lane == 0)
                put_stamp(a, ((uint64_t)idx << 16) | blockIdx.x, t0, it.npairs | (1u << 8) | (1u << 16) | ((uint64_t)it.list << 32));
        }
    };

    const uint32_t n_wide = a.counters[3];
    if (a.stamps && threadIdx.x == 0) put_stamp(a, blockIdx.x, wall_clock64(), 2u << 16);
    if (a.fused && blockIdx.x + a.fused >= gridDim.x) drain_narrow();
    for (;;) {
        if (threadIdx.x == 0) s_next = atomicAdd(&a.work[1], 1u);
        __syncthreads();
        const uint32_t b = s_next;
        if (b >= n_wide) break;
        const uint64_t t_item = a.stamps ? wall_clock64() : 0;
        ScanItem it = a.items_w[b];
        it.list = __builtin_amdgcn_readfirstlane(it.list);
        it.seg = __builtin_amdgcn_readfirstlane(it.seg);
        it.pair_start = __builtin_amdgcn_readfirstlane(it.pair_start);
        it.npairs = __builtin_amdgcn_readfirstlane(it.npairs);
        const int nq = (int)it.npairs;
        if (nq > (W2 ? 32 : 16)) {  // (never planned: see overflow_item; the barrier orders s_next)
            overflow_item(a, it.pair_start, (uint32_t)nq, threadIdx.x, blockDim.x);
            __syncthreads();
            continue;
        }
        if (threadIdx.x == 0) s_seg = 0;
        if (threadIdx.x < (uint32_t)nq) {
            s_thr[threadIdx.x] = a.thr[it.pair_start + threadIdx.x];
            pair_stats(it.pair_start, threadIdx.x, s_pst, s_qsc);
        }
        __syncthreads();
        const uint32_t seg_vectors = a.seg_blocks * 64;
        const uint32_t nseg = (a.count[it.list] + seg_vectors - 1) / seg_vectors;
        const uint32_t seg0 = it.seg * a.segs_item, seg1 = min(nseg, seg0 + a.segs_item);
        reset_rl(rl, nq > 16 ? 8 : 4);
        bool any = false;
        for (;;) {
            uint32_t sg = 0;
            if (lane == 0) sg = atomicAdd(&s_seg, 1u);
            sg = seg0 + __builtin_amdgcn_readfirstlane(sg);
            if (sg >= seg1) break;
            if (W2 && nq > 16)
                collect_segment<M, KD, 2, I8, W2>(a, it, 0, nq, sg, rl, s_thr, s_pst, s_qsc, s_mt[wv], s_vs[wv], wv, cc);
            else
                collect_segment<M, KD, 1, I8, W2>(a, it, 0, nq, sg, rl, s_thr, s_pst, s_qsc, s_mt[wv], s_vs[wv], wv, cc);
            any = true;
        }
        if (any) contribute_rl(a, it, 0, nq, rl);
        __syncthreads();  // (s_thr and s_seg are reset by the next item only after every wave is done)
        if (a.stamps && threadIdx.x == 0)
            put_stamp(a, ((uint64_t)b << 16) | blockIdx.x, t_item, (uint32_t)nq | ((seg1 - seg0) << 8) | ((uint64_t)it.list << 32));
    }
    if (a.fused) drain_narrow();
    finish_cand(a, cc);
}

bool scan_screen_fits(uint32_t k, uint32_t dp, uint32_t wq, bool deferred) {
    // (the deferred collect kernel's LDS is static and independent of k and the item width:
    // only the exact re-check's row staging counts; the inline kernel stages the item's
    // queries and its waves' top-k lists)
    return k >= 1 && k <= 64 && dp % 64 == 0 && (wq == 16 || wq == 32) && screen_exact_lds(dp / 4) <= kLdsBytes / 2 &&
           (deferred || screen_item_lds(k, wq) + 4 * screen_wave_lds(k) + 256 <= kLdsBytes / 2);
}

size_t screen_shadow_u4(uint64_t blocks, uint32_t d4, bool i8) {
    return (size_t)(blocks + 2) * d4 * (i8 ? 16 : 32);
}

void launch_screen_build(const float4* arena, uint64_t blocks, uint32_t d4, const uint32_t* block_list,
                         const float* cent_rm, uint4* shadow, float* rows, float4* meta, hipStream_t s, float* sscale) {
    if (!blocks) return;
    const uint32_t g = (uint32_t)std::min<uint64_t>((blocks + 3) / 4, 8192);
    if (sscale) ivf_screen_build_i8<<<g, 256, 0, s>>>(arena, blocks, d4, block_list, cent_rm, shadow, rows, meta, sscale);
    else ivf_screen_build<<<g, 256, 0, s>>>(arena, blocks, d4, block_list, cent_rm, shadow, rows, meta);
}

void launch_screen_pairs(int metric, const float* q, uint32_t B, uint32_t P, const uint32_t* probes,
                         const float* cent_rm, uint32_t dp, uint16_t* qres, float4* pst, uint32_t* thr4, hipStream_t s,
                         uint32_t* scnt, uint32_t* ovf, uint32_t* counters, uint32_t* ubcnt, float* qscale) {
    const uint32_t BP = B * P;
    if (!BP) return;
    const uint32_t g = std::min<uint32_t>((BP + 3) / 4, 2048);
    if (qscale) {  // (the int8 shadow: deferred scan only)
        if (metric == kL2)
            ivf_screen_pairs_i8<kL2><<<g, 256, 0, s>>>(q, BP, P, probes, cent_rm, dp, (int8_t*)qres, qscale, pst, thr4,
                                                       scnt, ovf, counters, ubcnt);
        else
            ivf_screen_pairs_i8<kIP><<<g, 256, 0, s>>>(q, BP, P, probes, cent_rm, dp, (int8_t*)qres, qscale, pst, thr4,
                                                       scnt, ovf, counters, ubcnt);
        return;
    }
    if (metric == kL2)
        ivf_screen_pairs<kL2><<<g, 256, 0, s>>>(q, BP, P, probes, cent_rm, dp, qres, pst, thr4, scnt, ovf, counters, ubcnt);
    else
        ivf_screen_pairs<kIP><<<g, 256, 0, s>>>(q, BP, P, probes, cent_rm, dp, qres, pst, thr4, scnt, ovf, counters, ubcnt);
}

#ifndef VDB_COLLECT_KD
#define VDB_COLLECT_KD 4
#endif
void launch_screen_collect(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s) {
    if (!grid_blocks) return;
    // (the kernel's per-item LDS holds 32 queries: wide items of 16 or 32 only)
    if (a.wide_q != 16 && a.wide_q != 32) throw std::length_error("launch_screen_collect: items of 16 or 32 queries only");
    const bool w2 = a.wide_q > 16;
    const uint32_t g = std::min<uint32_t>(grid_blocks, w2 ? kPersistentBlocks / 2 : kPersistentBlocks);
    auto go = [&](auto m_c, auto w_c, auto i_c) {
        constexpr int Mm = decltype(m_c)::value;
        constexpr bool Ww = decltype(w_c)::value;
        constexpr bool Ii = decltype(i_c)::value;
        // k-steps in flight per wave: a divisor of the row's k-steps (32 bf16 / 64 int8 dims
        // each); 32-query items run one workgroup per CU, so they keep more in flight (8 bf16,
        // 6 int8: as many bytes per CU as two workgroups of 4 bf16 k-steps, or nearly)
        constexpr int KW = Ii ? 6 : 8;
        const uint32_t ks = a.dp / (Ii ? 64 : 32);
        if (Ww && ks % KW == 0) ivf_screen_collect<Mm, KW, Ww, Ii><<<g, 256, 0, s>>>(a);
        else if (!Ww && VDB_COLLECT_KD != 4 && ks % VDB_COLLECT_KD == 0)  // (A/B builds of the 16-query depth)
            ivf_screen_collect<Mm, VDB_COLLECT_KD, Ww, Ii><<<g, 256, 0, s>>>(a);
        else if (ks % 4 == 0) ivf_screen_collect<Mm, 4, Ww, Ii><<<g, 256, 0, s>>>(a);
        else if (ks % 2 == 0) ivf_screen_collect<Mm, 2, Ww, Ii><<<g, 256, 0, s>>>(a);
        else ivf_screen_collect<Mm, 1, Ww, Ii><<<g, 256, 0, s>>>(a);
    };
    auto go_w = [&](auto m_c, auto i_c) {
        if (w2) go(m_c, std::true_type{}, i_c);
        else go(m_c, std::false_type{}, i_c);
    };
    auto go_i = [&](auto m_c) {
        if (a.sscale) go_w(m_c, std::true_type{});
        else go_w(m_c, std::false_type{});
    };
    if (metric == kL2) go_i(std::integral_constant<int, kL2>{});
    else go_i(std::integral_constant<int, kIP>{});
}

void launch_scan_screen(int metric, uint32_t grid_blocks, const ScanArgs& a, hipStream_t s) {
    if (!grid_blocks) return;
    static const bool raised = [] {  // up to half a CU's LDS per workgroup (k = 64: 70 KB)
        const void* f[] = {(const void*)ivf_scan_screen<kL2, 4>, (const void*)ivf_scan_screen<kL2, 2>,
                           (const void*)ivf_scan_screen<kIP, 4>, (const void*)ivf_scan_screen<kIP, 2>};
        for (const void* fn : f)
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytes / 2 - 256));
        (void)hipGetLastError();
        return true;
    }();
    (void)raised;
    const uint32_t g = std::min<uint32_t>(grid_blocks, kPersistentBlocks);
    const size_t lds = screen_item_lds(a.k, a.wide_q) + 4 * screen_wave_lds(a.k);
    const bool kd4 = (a.dp / 32) % 4 == 0;
    if (metric == kL2) {
        if (kd4) ivf_scan_screen<kL2, 4><<<g, 256, lds, s>>>(a);
        else ivf_scan_screen<kL2, 2><<<g, 256, lds, s>>>(a);
    } else {
        if (kd4) ivf_scan_screen<kIP, 4><<<g, 256, lds, s>>>(a);
        else ivf_scan_screen<kIP, 2><<<g, 256, lds, s>>>(a);
    }
}

}  // namespace vdbk
