// Per-CU L2 streaming bandwidth for the policy kernel's weight-load shape: 256 workgroups x 512
// threads all stream the same W (rows of 128 floats) as f32x4, 16 rows x 64 B per wave instruction
// (gemm_tile's A operand) or 1 KiB contiguous. Prints GB/s per CU and chip-wide.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE, int DEPTH>
__global__ __launch_bounds__(512) void k_stream(const float* __restrict__ W, int rows, float* out) {
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i16 = l & 15, g = l >> 4;
    f32x4 acc = {0, 0, 0, 0};
    // each wave sweeps a 16-row tile group: tiles wv, wv+8, ... ; per tile 8 k-blocks of 64 B per row
    for (int tile = wv; tile * 16 < rows; tile += 8) {
        const float* base = W + (size_t)tile * 16 * 128;
        f32x4 a[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            if (SHAPE == 0) a[p] = *reinterpret_cast<const f32x4*>(base + (size_t)i16 * 128 + 4 * g + 16 * p);
            else a[p] = *reinterpret_cast<const f32x4*>(base + (size_t)p * 256 + 4 * l);
        }
#pragma unroll
        for (int p = 0; p < 8; ++p) acc += a[p];
    }
    if (acc.x == 1234.5f) out[threadIdx.x] = acc.y + acc.z + acc.w;
}

template <int SHAPE, int DEPTH>
void run(const float* W, int rows, float* out, const char* name) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_stream<SHAPE, DEPTH>), dim3(256), dim3(512), 0, 0, W, rows, out);
    hipEventRecord(e0);
    const int N = 20;
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL((k_stream<SHAPE, DEPTH>), dim3(256), dim3(512), 0, 0, W, rows, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / N, bytes = (double)rows * 128 * 4;
    printf("%-28s rows=%6d  %.2f us/launch  per-CU %.1f GB/s  chip %.2f TB/s\n", name, rows, us, bytes / us / 1e3,
           bytes * 256 / us / 1e6);
}

int main() {
    const int rows = 3072;  // 1.5 MiB
    float *W, *out;
    hipMalloc(&W, (size_t)rows * 128 * 4 * 4);
    hipMalloc(&out, 4096);
    hipMemset(W, 0, (size_t)rows * 128 * 4 * 4);
    run<0, 8>(W, rows, out, "16 rows x 64 B (gemm A)");
    run<1, 8>(W, rows, out, "1 KiB contiguous");
    run<0, 8>(W, 768, out, "16x64B, 384 KiB");
    run<1, 8>(W, 768, out, "1 KiB, 384 KiB");
    return 0;
}
