// Per-CU L2 streaming rate of the rollout kernel's weight stream when every workgroup reads the
// SAME weights at the same time (the kernel's order: tile t, blocks 0..7 in order) against the same
// stream with each workgroup starting at a different place (tile order rotated by blockIdx, or the
// k-blocks of each tile rotated) -- does same-line contention in the L2 cap the 118 GB/s per CU of
// scripts/micro/l2bw.hip? Also the stream with 2 waves of 8 in flight per SIMD (DEPTH loads per wave
// before the first use). 256 workgroups x 512 threads, 1 KiB fragment loads (16 B per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ROT 0: every workgroup the same order; 1: tiles rotated by blockIdx; 2: k-blocks rotated by blockIdx
template <int ROT, int DEPTH>
__global__ __launch_bounds__(512) void k_stream(const float* __restrict__ W, int tiles, float* out) {
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    f32x4 acc = {0, 0, 0, 0};
    const int nt = tiles / 8;  // tiles per wave
    for (int j = 0; j < nt; ++j) {
        int tile = wv + 8 * j;
        if (ROT == 1) tile = (tile + 8 * (int)blockIdx.x) % tiles;
        const float* base = W + (size_t)tile * 8 * 256;
        f32x4 a[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int kb = ROT == 2 ? (p + (int)blockIdx.x) & 7 : p;
            a[p] = *reinterpret_cast<const f32x4*>(base + (size_t)kb * 256 + 4 * l);
            if (p >= DEPTH - 1) acc += a[p - DEPTH + 1];
        }
#pragma unroll
        for (int p = 8 - DEPTH + 1; p < 8; ++p) acc += a[p];
    }
    if (acc.x == 1234.5f) out[threadIdx.x] = acc.y + acc.z + acc.w;
}

template <int ROT, int DEPTH>
void run(const float* W, int tiles, float* out, const char* name) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_stream<ROT, DEPTH>), dim3(256), dim3(512), 0, 0, W, tiles, out);
    hipEventRecord(e0);
    const int N = 20;
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL((k_stream<ROT, DEPTH>), dim3(256), dim3(512), 0, 0, W, tiles, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / N, bytes = (double)tiles * 8 * 1024;
    printf("%-34s %5d KiB  %7.2f us/launch  per-CU %6.1f GB/s  chip %6.2f TB/s\n", name, (int)(bytes / 1024), us,
           bytes / us / 1e3, bytes * 256 / us / 1e6);
}

int main() {
    const int tiles = 192;  // 1.5 MiB: the rollout step's weights
    float *W, *out;
    hipMalloc(&W, (size_t)tiles * 8 * 1024);
    hipMalloc(&out, 4096);
    hipMemset(W, 0, (size_t)tiles * 8 * 1024);
    for (int r = 0; r < 2; ++r) {
        run<0, 2>(W, tiles, out, "same order, 2 in flight");
        run<0, 8>(W, tiles, out, "same order, 8 in flight");
        run<1, 2>(W, tiles, out, "tiles rotated, 2 in flight");
        run<1, 8>(W, tiles, out, "tiles rotated, 8 in flight");
        run<2, 2>(W, tiles, out, "k-blocks rotated, 2 in flight");
        run<2, 8>(W, tiles, out, "k-blocks rotated, 8 in flight");
    }
    return 0;
}
