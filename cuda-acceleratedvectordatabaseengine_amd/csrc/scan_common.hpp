// scan_common.hpp — device helpers shared by the scan translation units (kernels.hip,
// screen.hip): the reference's distance arithmetic, the order-preserving threshold
// encoding and the streaming load.
//
// Exactness: every distance is the reference's sequential fp32 sum
// (ivf_flat_index.cpp:308-318, 352-362): diff = a - b rounded, diff*diff rounded,
// acc + term rounded, d = 0..D-1. Every including file is compiled with
// -ffp-contract=off and `#pragma clang fp contract(off)`, so no multiply-add is fused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave_topk.hpp"

namespace vdbk {

enum { kL2 = 0, kIP = 1, kCos = 2 };

template <int M>
__device__ __forceinline__ float dist_term(float acc, float a, float b) {
    if constexpr (M == kL2) {
        const float diff = a - b;
        return acc + diff * diff;
    } else if constexpr (M == kIP) {
        return acc + a * b;
    } else {
        return acc;  // Cosine: the CPU path never assigns a distance (cpp:351-362)
    }
}
template <int M>
__device__ __forceinline__ float dist_finish(float acc) {
    if constexpr (M == kIP) return -acc;
    return acc;
}

template <int M>
__device__ __forceinline__ float acc4(float acc, const float4 q, const float4 x) {
    acc = dist_term<M>(acc, q.x, x.x);
    acc = dist_term<M>(acc, q.y, x.y);
    acc = dist_term<M>(acc, q.z, x.z);
    acc = dist_term<M>(acc, q.w, x.w);
    return acc;
}

__device__ __forceinline__ uint32_t wave_index() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// Issue priority of the per-batch chain's short kernels (coarse step, re-rank, plan, pair
// rows, the screen's selection, re-check and merges) over the collect kernel's waves sharing
// their SIMDs (s_setprio; the collect keeps the hardware default 0). With batches in flight a
// batch's chain runs beside another batch's collect; raising it shortens the chain without
// slowing the stream: the 1/8 shard at 3 in flight 0.262 -> 0.251 ms per step at priority 2,
// every rank of the 8-GPU emulation 0.276-0.287 -> 0.266-0.270 ms, the headline unchanged;
// priority 3 (the highest) 1 % faster again at both, same box (round 6,
// tools/build_chain_prio_variant.sh A/B, profiles/r06_sweep_chain_prio.jsonl). Never changes
// results.
#ifndef VDB_CHAIN_PRIO
#define VDB_CHAIN_PRIO 3
#endif
__device__ __forceinline__ void chain_prio() {
    if constexpr (VDB_CHAIN_PRIO > 0) __builtin_amdgcn_s_setprio(VDB_CHAIN_PRIO);
}

// Order-preserving float <-> uint encoding of the shared k-th thresholds (atomicMin).
__device__ __forceinline__ uint32_t ord_enc(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord_dec(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
constexpr uint32_t kThrInf = 0xFF800000u;  // ord_enc(+inf)

// List data is read once per batch: non-temporal loads (nt) keep it from displacing
// reusable lines and stream measurably faster on gfx950 (tools/stream_probe.hip:
// 6.8 vs 6.25 TB/s for this access pattern).
typedef float v4f_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 load_nt(const float4* p) {
    const v4f_nt v = __builtin_nontemporal_load((const v4f_nt*)p);
    return make_float4(v.x, v.y, v.z, v.w);
}

}  // namespace vdbk
