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

#include <type_traits>

namespace vdbk {

constexpr uint64_t kNoId = ~0ull;

__device__ __forceinline__ bool key_less(float d1, uint64_t i1, float d2, uint64_t i2) {
    return (d1 < d2) | ((d1 == d2) & (i1 < i2));  // bitwise: no branch around the id compare
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

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// ---- lane exchanges without the LDS crossbar where gfx950 allows it ----------
// x ^ MASK for MASK in {1, 2, 4, 8}: DPP moves inside a 16-lane row; 16: ds_swizzle
// (bit mode, xor inside 32 lanes); 32: ds_bpermute. Callers run with every lane of
// the wave active (the top-k code is wave-uniform).
template <int MASK>
__device__ __forceinline__ uint32_t xor_u32(uint32_t v) {
    const int x = (int)v;
    if constexpr (MASK == 1) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    else if constexpr (MASK == 2) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    else if constexpr (MASK == 4)  // half-row mirror (i ^ 7), then quad_perm [3,2,1,0] (i ^ 3)
        return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF,
                                                  false);
    else if constexpr (MASK == 8) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false);  // row_ror:8
    else if constexpr (MASK == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle(x, 0x401F);  // and 0x1F, xor 0x10
    else return (uint32_t)__shfl_xor(x, MASK);
}
template <int MASK>
__device__ __forceinline__ float xor_f(float v) {
    return __uint_as_float(xor_u32<MASK>(__float_as_uint(v)));
}
template <int MASK>
__device__ __forceinline__ uint64_t xor_u64(uint64_t v) {
    return ((uint64_t)xor_u32<MASK>((uint32_t)(v >> 32)) << 32) | xor_u32<MASK>((uint32_t)v);
}
// lane i <- lane i - 1 (lane 0 <- fill) and lane i <- lane i + 1 (lane 63 <- fill):
// DPP wave_shr:1 / wave_shl:1.
__device__ __forceinline__ uint32_t up1_u32(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t down1_u32(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xF, 0xF, false);
}

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
            // lane i takes lane i-1's element; lane 0 takes the previous register's last
            const float up_d = __uint_as_float(up1_u32(__float_as_uint(d[r]), __float_as_uint(carry_d)));
            const uint64_t up_i = ((uint64_t)up1_u32((uint32_t)(id[r] >> 32), (uint32_t)(carry_i >> 32)) << 32) |
                                  up1_u32((uint32_t)id[r], (uint32_t)carry_i);
            const float last_d = rd_lane(d[r], 63);
            const uint64_t last_i = rd_lane(id[r], 63);
            const int e = r * 64 + lane;
            d[r] = e > pos ? up_d : (e == pos ? cd : d[r]);
            id[r] = e > pos ? up_i : (e == pos ? cid : id[r]);
            carry_d = last_d;
            carry_i = last_i;
        }
    }

    // Remove element e (wave-uniform), shifting the tail down; tail becomes empty.
    __device__ __forceinline__ void remove(int e) {
        const int lane = lane_id();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            // lane 63 takes the next register's first element (or the empty key)
            float nd = __builtin_inff();
            uint64_t ni = kNoId;
            if (r + 1 < R) {
                nd = rd_lane(d[r + 1 < R ? r + 1 : r], 0);
                ni = rd_lane(id[r + 1 < R ? r + 1 : r], 0);
            }
            const float dn_d = __uint_as_float(down1_u32(__float_as_uint(d[r]), __float_as_uint(nd)));
            const uint64_t dn_i = ((uint64_t)down1_u32((uint32_t)(id[r] >> 32), (uint32_t)(ni >> 32)) << 32) |
                                  down1_u32((uint32_t)id[r], (uint32_t)ni);
            const bool mv = r * 64 + lane >= e;
            d[r] = mv ? dn_d : d[r];
            id[r] = mv ? dn_i : id[r];
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

// One compare-exchange step of a bitonic network at lane distance J: keep the
// smaller key if keep_min, else the larger. Branch-free (selects, no exec masking).
template <int J>
__device__ __forceinline__ void cmpx(float& d, uint64_t& id, bool keep_min) {
    const float od = xor_f<J>(d);
    const uint64_t oi = xor_u64<J>(id);
    const bool take = keep_min ? key_less(od, oi, d, id) : key_less(d, id, od, oi);
    d = take ? od : d;
    id = take ? oi : id;
}

// Bitonic sort of one (dist, id) per lane, ascending over lanes 0..63.
__device__ __forceinline__ void bitonic_sort64(float& d, uint64_t& id) {
    const int lane = lane_id();
    static_for<1, 7>([&](auto ks) {  // kk = 2^ks = 2 .. 64
        constexpr int KK = 1 << decltype(ks)::value;
        const bool asc = (lane & KK) == 0;
        static_for<0, decltype(ks)::value>([&](auto js) {  // j = KK/2 .. 1
            constexpr int J = (KK >> 1) >> decltype(js)::value;
            const bool lower = (lane & J) == 0;
            cmpx<J>(d, id, lower == asc);
        });
    });
}

// Sorted-ascending list (one element per lane) merged with a sorted batch: keeps
// the 64 smallest of the union, sorted. min(A[i], B[63-i]) is bitonic.
__device__ __forceinline__ void bitonic_merge64(float& ad, uint64_t& ai, float bd, uint64_t bi) {
    const int lane = lane_id();
    const float rd = shfl_f(bd, 63 - lane);
    const uint64_t ri = shfl_u64(bi, 63 - lane);
    const bool t = key_less(rd, ri, ad, ai);
    ad = t ? rd : ad;
    ai = t ? ri : ai;
    static_for<0, 6>([&](auto js) {  // j = 32 .. 1
        constexpr int J = 32 >> decltype(js)::value;
        cmpx<J>(ad, ai, (lane & J) == 0);
    });
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
            if (kd == __builtin_inff() && ki == kNoId && rd_lane(tk.id[0], 0) == kNoId) {
                // empty list (a segment's first block): the sorted batch is the list
                tk.d[0] = bd;
                tk.id[0] = bi;
            } else {
                bitonic_merge64(tk.d[0], tk.id[0], bd, bi);
            }
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
