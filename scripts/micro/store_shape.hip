// Store rate of the MFMA accumulator's natural store shape against wider per-row segments
// (the training kernels write their activations / input gradients straight from
// 16 x 16 accumulator tiles: per wave-instruction 16 rows x 64 B). Writes a [R][256] fp32 buffer
// (R = 20480 * 16 rows, 336 MB), 512-thread workgroups, every CU busy:
//   seg64  : lane (i16, g) stores float4 at [row0 + i16][c0 + 4 g]       -> 16 rows x 64 B per instruction
//   seg128 : lane (i16, g) stores 2 x float4 at [row0 + i16][c0 + 8 g ..] -> 16 rows x 128 B per 2 instructions
//   row256 : lane l stores float4 at [row0 + l / 16][4 (l % 16)]       -> 4 rows x 256 B per instruction
// Build: hipcc --offload-arch=gfx950 -O3 -o store_shape store_shape.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int C = 256;

template <int MODE>
__global__ __launch_bounds__(512) void k_store(float* out, long long rows) {
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, i16 = l & 15, g = l >> 4;
    const f4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    // each workgroup: 80 rows (one 16-sample block's tokens) x 256 columns, like the training kernels
    const long long r0 = (long long)blockIdx.x * 80;
    if (r0 + 80 > rows) return;
    for (int t = 0; t < 5; ++t) {        // 5 token tiles of 16 rows
        const long long row = r0 + 16 * t + i16;
        if (MODE == 0) {                 // wave wv owns columns [32 wv, 32 wv + 32): two 16-col tiles
            for (int tile = 0; tile < 2; ++tile)
                *reinterpret_cast<f4*>(out + row * C + 32 * wv + 16 * tile + 4 * g) = v;
        } else if (MODE == 1) {          // the same 32 columns, each lane 8 consecutive floats
            *reinterpret_cast<f4*>(out + row * C + 32 * wv + 8 * g) = v;
            *reinterpret_cast<f4*>(out + row * C + 32 * wv + 8 * g + 4) = v;
        } else {                         // row-contiguous: 4 rows x 256 B per instruction
            for (int q = 0; q < 2; ++q) {
                const long long rr = r0 + 16 * t + 4 * (l >> 4) + 2 * q;  // rows of this wave's pair
                *reinterpret_cast<f4*>(out + (rr + (wv >> 2)) * C + 64 * (wv & 3) + 4 * i16) = v;
            }
        }
    }
}

int main() {
    const long long rows = 20480LL * 16;  // 327,680 rows x 1 KiB = 336 MB
    float* out;
    if (hipMalloc(&out, rows * C * sizeof(float)) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grid = (int)(rows / 80);
    const char* names[3] = {"seg64 (accumulator tiles)", "seg128 (8 floats per lane)", "row256 (row-contiguous)"};
    for (int mode = 0; mode < 3; ++mode) {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            (void)hipEventRecord(a, 0);
            if (mode == 0) hipLaunchKernelGGL(k_store<0>, dim3(grid), dim3(512), 0, 0, out, rows);
            if (mode == 1) hipLaunchKernelGGL(k_store<1>, dim3(grid), dim3(512), 0, 0, out, rows);
            if (mode == 2) hipLaunchKernelGGL(k_store<2>, dim3(grid), dim3(512), 0, 0, out, rows);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (r > 0 && ms < best) best = ms;
        }
        printf("%-28s %8.3f ms  %7.2f TB/s\n", names[mode], best, rows * C * 4.0 / (best * 1e-3) / 1e12);
    }
    return 0;
}
