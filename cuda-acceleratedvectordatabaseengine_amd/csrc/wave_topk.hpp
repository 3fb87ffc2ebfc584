// wave_topk.hpp — wave64 top-k selection primitives for gfx950.
//
// A candidate is the pair (dist, id) under the lexicographic order std::pair uses
// in the reference (ivf_flat_index.cpp:324, 368, 493): smaller dist first, ties by
// smaller id. A wave keeps the k best candidates spread over its 64 lanes and R
// registers: element e = r*64 + lane, ascending in e. Unused elements hold
// (+inf, UINT64_MAX), which no real candidate ranks below.
//
// Two insertion paths:
//   * insert(): one wave-uniform candidate, shifting the tail up by one element
//     (ballot + popcount for the position, shfl_up for the shift);
//   * merge_batch(): R == 1 only — bitonic-sort the 64 lane candidates and fold
//     them into the current list with one bitonic merge. Used when many lanes
//     pass the threshold at once (first blocks of a segment).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vdbk {

constexpr uint64_t kNoId = ~0ull;

__device__ __forceinline__ bool key_less(float d1, uint64_t i1, float d2, uint64_t i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

__device__ __forceinline__ float rd_lane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint64_t rd_lane(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rd_lane_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ float shfl_f(float v, int src) { return __shfl(v, src); }

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

template <int R>
struct WaveTopK {
    float d[R];
    uint64_t id[R];

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            d[r] = __builtin_inff();
            id[r] = kNoId;
        }
    }

    // (dist, id) of element e (wave-uniform e).
    __device__ __forceinline__ void at(int e, float& od, uint64_t& oi) const {
        const int rr = e >> 6, l = e & 63;
        float vd = d[0];
        uint64_t vi = id[0];
#pragma unroll
        for (int r = 1; r < R; ++r)
            if (r == rr) {
                vd = d[r];
                vi = id[r];
            }
        od = rd_lane(vd, l);
        oi = rd_lane(vi, l);
    }

    // Insert a wave-uniform candidate known to rank below element k-1.
    __device__ __forceinline__ void insert(float cd, uint64_t cid) {
        const int lane = lane_id();
        int pos = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) pos += __popcll(__ballot(key_less(d[r], id[r], cd, cid)));
        float carry_d = 0.f;
        uint64_t carry_i = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int src = lane == 0 ? 0 : lane - 1;
            float up_d = shfl_f(d[r], src);
            uint64_t up_i = shfl_u64(id[r], src);
            const float last_d = rd_lane(d[r], 63);
            const uint64_t last_i = rd_lane(id[r], 63);
            if (lane == 0) {
                up_d = carry_d;
                up_i = carry_i;
            }
            const int e = r * 64 + lane;
            if (e > pos) {
                d[r] = up_d;
                id[r] = up_i;
            } else if (e == pos) {
                d[r] = cd;
                id[r] = cid;
            }
            carry_d = last_d;
            carry_i = last_i;
        }
    }

    // Remove element e (wave-uniform), shifting the tail down; tail becomes empty.
    __device__ __forceinline__ void remove(int e) {
        const int lane = lane_id();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int src = lane == 63 ? 63 : lane + 1;
            float dn_d = shfl_f(d[r], src);
            uint64_t dn_i = shfl_u64(id[r], src);
            if (lane == 63) {
                if (r + 1 < R) {
                    dn_d = rd_lane(d[r + 1 < R ? r + 1 : r], 0);
                    dn_i = rd_lane(id[r + 1 < R ? r + 1 : r], 0);
                } else {
                    dn_d = __builtin_inff();
                    dn_i = kNoId;
                }
            }
            if (r * 64 + lane >= e) {
                d[r] = dn_d;
                id[r] = dn_i;
            }
        }
    }

    // Offer one wave-uniform candidate against a list of capacity k.
    __device__ __forceinline__ void offer(float cd, uint64_t cid, int k, float& kd, uint64_t& ki) {
        if (key_less(cd, cid, kd, ki)) {
            insert(cd, cid);
            at(k - 1, kd, ki);
        }
    }

    // Offer with id de-duplication (merge_results, cpp:495-504): the list keeps
    // each id once, at its smallest (dist, id); a larger duplicate is dropped.
    __device__ __forceinline__ void offer_unique(float cd, uint64_t cid, int k, float& kd, uint64_t& ki) {
        int where = -1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint64_t m = __ballot(id[r] == cid);
            if (m && where < 0) where = r * 64 + (__ffsll((long long)m) - 1);
        }
        if (where >= 0) {
            float od;
            uint64_t oi;
            at(where, od, oi);
            if (!(cd < od)) return;
            remove(where);
            insert(cd, cid);
            at(k - 1, kd, ki);
            return;
        }
        offer(cd, cid, k, kd, ki);
    }
};

// Bitonic sort of one (dist, id) per lane, ascending over lanes 0..63.
__device__ __forceinline__ void bitonic_sort64(float& d, uint64_t& id) {
    const int lane = lane_id();
#pragma unroll
    for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            const float od = __shfl_xor(d, j);
            const uint64_t oi = shfl_u64(id, lane ^ j);
            const bool asc = (lane & kk) == 0;
            const bool lower = (lane & j) == 0;
            const bool keep_min = (lower == asc);
            const bool take = keep_min ? key_less(od, oi, d, id) : key_less(d, id, od, oi);
            if (take) {
                d = od;
                id = oi;
            }
        }
    }
}

// Sorted-ascending list (one element per lane) merged with a sorted batch: keeps
// the 64 smallest of the union, sorted. min(A[i], B[63-i]) is bitonic.
__device__ __forceinline__ void bitonic_merge64(float& ad, uint64_t& ai, float bd, uint64_t bi) {
    const int lane = lane_id();
    const float rd = shfl_f(bd, 63 - lane);
    const uint64_t ri = shfl_u64(bi, 63 - lane);
    if (key_less(rd, ri, ad, ai)) {
        ad = rd;
        ai = ri;
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        const float od = __shfl_xor(ad, j);
        const uint64_t oi = shfl_u64(ai, lane ^ j);
        const bool lower = (lane & j) == 0;
        const bool take = lower ? key_less(od, oi, ad, ai) : key_less(ad, ai, od, oi);
        if (take) {
            ad = od;
            ai = oi;
        }
    }
}

// Fold this lane's candidate (cd, cid) — if `want` — into the list. Candidates
// must already be filtered to those that may rank below element k-1.
template <int R>
__device__ __forceinline__ void offer_lanes(WaveTopK<R>& tk, bool want, float cd, uint64_t cid, int k,
                                            float& kd, uint64_t& ki) {
    uint64_t mask = __ballot(want);
    if (!mask) return;
    if constexpr (R == 1) {
        if (__popcll(mask) > 6) {
            float bd = want ? cd : __builtin_inff();
            uint64_t bi = want ? cid : kNoId;
            bitonic_sort64(bd, bi);
            bitonic_merge64(tk.d[0], tk.id[0], bd, bi);
            tk.at(k - 1, kd, ki);
            return;
        }
    }
    while (mask) {
        const int l = __ffsll((long long)mask) - 1;
        mask &= mask - 1;
        const float c_d = rd_lane(cd, l);
        const uint64_t c_i = rd_lane(cid, l);
        tk.offer(c_d, c_i, k, kd, ki);
    }
}

}  // namespace vdbk
