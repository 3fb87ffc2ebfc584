// mfma_probe.hip — layout and issue rate of the multi-block f32 MFMA forms on gfx950
// (v_mfma_f32_16x16x1_4b_f32 / 32x32x1_2b / 4x4x1_16b), used to design the bounded scan.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

// A = 1 at lane la only, B = 1 at lane lb only: D has a single 1 at the (row of la, col of
// lb) position of the block both lanes belong to; record which (lane, reg) holds it.
__global__ void layout16(int la, int lb, float* out) {
    const int l = threadIdx.x;
    const float a = l == la ? 1.f : 0.f, b = l == lb ? 1.f : 0.f;
    v16f c = {};
    c = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}

__global__ void rate16(float* out, int iters) {
    const int l = threadIdx.x;
    float a = l * 1e-3f, b = l * 2e-3f;
    v16f c0 = {}, c1 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x1f32(b, a, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, a, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x1f32(b, b, c1, 0, 0, 0);
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r];
    out[blockIdx.x * blockDim.x + l] = s;
}

__global__ void rate16dep(float* out, int iters) {  // one dependent chain
    const int l = threadIdx.x;
    float a = l * 1e-3f, b = l * 2e-3f;
    v16f c0 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(b, a, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, a, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x1f32(b, b, c0, 0, 0, 0);
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r];
    out[blockIdx.x * blockDim.x + l] = s;
}

int main() {
    float* d;
    hipMalloc(&d, 1 << 24);
    std::vector<float> h(64 * 16);
    // layout: for A lane la and B lane lb in the same 16-lane block
    printf("16x16x1_4b D layout (la, lb) -> (lane, reg):\n");
    int pairs[][2] = {{0, 0}, {1, 0}, {2, 0}, {5, 0}, {0, 1}, {0, 3}, {0, 7}, {0, 15}, {15, 15}, {16, 16}, {17, 16},
                      {16, 17}, {20, 21}, {32, 32}, {33, 40}, {48, 48}, {63, 63}, {4, 0}, {8, 0}, {12, 0}};
    for (auto& p : pairs) {
        layout16<<<1, 64>>>(p[0], p[1], d);
        hipMemcpy(h.data(), d, 64 * 16 * 4, hipMemcpyDeviceToHost);
        printf("  A lane %2d, B lane %2d:", p[0], p[1]);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r)
                if (h[l * 16 + r] != 0.f) printf(" (lane %d, reg %d)=%g", l, r, h[l * 16 + r]);
        printf("\n");
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096, blocks = 256 * 4 * 2;  // 2 waves per SIMD
    for (int dep = 0; dep < 2; ++dep) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (dep) rate16dep<<<blocks, 64>>>(d, iters);
            else rate16<<<blocks, 64>>>(d, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double macs = (double)blocks * iters * 4 * 1024;
            printf("%s: %.3f ms, %.1f TFLOP/s\n", dep ? "16x16x1 one chain" : "16x16x1 two chains", ms,
                   2 * macs / ms / 1e9);
        }
    }
    return 0;
}
