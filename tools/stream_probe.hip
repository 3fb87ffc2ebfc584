// stream_probe.hip — HBM streaming ceiling for the scan's access pattern (diagnostic).
//
// Each wave streams one contiguous segment of `seg_kb` KiB (the scan's 512-vector
// list segment at 768 dims is 1.5 MiB), one 1 KiB wave-load per tile, with T tiles in
// flight, and optionally `work` packed-fp32 instructions per tile standing in for the
// distance math. Reports TB/s over a buffer far larger than the Infinity Cache.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
// run:   tools/stream_probe [GiB=24]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt(const float4* p) {
    const v4f v = __builtin_nontemporal_load((const v4f*)p);
    return make_float4(v.x, v.y, v.z, v.w);
}

template <int T, int WORK, bool NT = false>
__global__ __launch_bounds__(256) void seg_stream(const float4* __restrict__ buf, uint64_t seg_tiles, uint64_t nseg,
                                                  float* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    f2 acc = {0.f, 0.f};
    for (uint64_t s = wave; s < nseg; s += nwaves) {
        const float4* p = buf + s * seg_tiles * 64 + lane;
        float4 x[T];
#pragma unroll
        for (int t = 0; t < T; ++t) x[t] = NT ? ldnt(p + (size_t)t * 64) : p[(size_t)t * 64];
        for (uint64_t t0 = 0; t0 < seg_tiles; t0 += T) {
#pragma unroll
            for (int t = 0; t < T; ++t) {
                f2 a = {x[t].x, x[t].y}, b = {x[t].z, x[t].w};
#pragma unroll
                for (int w = 0; w < WORK; ++w) {
                    a = a * b + acc;
                    acc = acc + a;
                }
                acc = acc + a + b;
                // the last round prefetches up to T tiles into the next segment (or the slack)
                x[t] = NT ? ldnt(p + (size_t)(T + t) * 64) : p[(size_t)(T + t) * 64];
            }
            p += (size_t)T * 64;
        }
    }
    if (acc.x == 1234.5f) sink[0] = acc.y;
}

__global__ __launch_bounds__(256) void flat_stream(const float4* __restrict__ buf, uint64_t n4, float* __restrict__ sink) {
    float acc = 0.f;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const float4 v = buf[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) sink[0] = acc;
}

template <class F>
static double time_ms(F f) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    const int reps = 3;
    for (int r = 0; r < reps; ++r) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 24.0;
    const uint64_t seg_tiles = 8 * 192;  // 8 blocks x 192 tiles: 1.5 MiB per wave segment
    const uint64_t seg_bytes = seg_tiles * 64 * 16;
    const uint64_t nseg = (uint64_t)(gib * (1ull << 30)) / seg_bytes;
    const uint64_t bytes = nseg * seg_bytes;
    float4* buf;
    float* sink;
    CHECK(hipMalloc(&buf, bytes + (1 << 20)));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(buf, 0, bytes + (1 << 20)));
    printf("buffer %.2f GB, %llu segments of %.2f MB\n", bytes / 1e9, (unsigned long long)nseg, seg_bytes / 1e6);
    {
        const double ms = time_ms([&] { flat_stream<<<256 * 32, 256>>>(buf, bytes / 16, sink); });
        printf("flat grid-stride float4       : %.3f ms  %.2f TB/s\n", ms, bytes / ms / 1e9);
    }
#define RUN(T, W, WGS, NT)                                                                                     \
    {                                                                                                          \
        const uint32_t grid = 256 * (WGS);                                                                     \
        const double ms = time_ms([&] { seg_stream<T, W, NT><<<grid, 256>>>(buf, seg_tiles, nseg, sink); });   \
        printf("segments T=%2d work=%d wg/cu=%d nt=%d : %.3f ms  %.2f TB/s\n", T, W, WGS, (int)NT, ms,          \
               bytes / ms / 1e9);                                                                              \
    }
    RUN(16, 0, 2, true) RUN(16, 24, 2, true) RUN(16, 32, 2, true) RUN(16, 48, 2, true) RUN(8, 48, 2, true)
    RUN(8, 48, 3, true) RUN(8, 64, 2, true) RUN(8, 96, 2, true)
    CHECK(hipFree(buf));
    return 0;
}
