// Kernel-boundary cost vs a grid barrier on MI355X (the minibatch-64 update: nine serial
// launches per optimizer step). Measures, with HIP events over a captured hipGraph:
//   (1) N dependent launches of a tiny kernel (G workgroups of 512 threads, one store each): time per
//       launch = the kernel-to-kernel cost inside a graph;
//   (2) one launch of G workgroups passing N grid barriers (an agent-scope counter: vector atomic add,
//       acquire loads with s_sleep between polls, bounded so a missing workgroup cannot hang the GPU).
// Build: hipcc --offload-arch=gfx950 -O3 -o launch_gap launch_gap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_tiny(float* out, int i) {
    if (threadIdx.x == 0) out[blockIdx.x] = (float)i;
}

// bounded grid barrier: returns false if the spin gave up (then *err is set)
__device__ bool grid_sync(unsigned* cnt, unsigned target, int* err) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        __atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE);
        int spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 22)) { atomicOr(err, 1); ok = false; break; }
        }
    }
    __syncthreads();
    return ok;
}

__global__ void k_barriers(unsigned* cnt, int n, float* out, int* err) {
    const unsigned G = gridDim.x;
    for (int i = 0; i < n; ++i) {
        if (threadIdx.x == 0) out[blockIdx.x] = (float)i;
        if (!grid_sync(cnt, (unsigned)(i + 1) * G, err)) return;
    }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 200;
    float* out; unsigned* cnt; int* err;
    CK(hipMalloc(&out, 4096 * sizeof(float)));
    CK(hipMalloc(&cnt, sizeof(unsigned)));
    CK(hipMalloc(&err, sizeof(int)));
    CK(hipMemset(err, 0, sizeof(int)));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grids[] = {1, 8, 40, 256};
    for (int G : grids) {
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_tiny, dim3(G), dim3(512), 0, st, out, i);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        printf("graph of %d dependent launches, %3d workgroups: %.2f us per launch\n", N, G, best * 1e3f / N);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    for (int G : grids) {
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipMemset(cnt, 0, sizeof(unsigned)));
            CK(hipEventRecord(a, st));
            hipLaunchKernelGGL(k_barriers, dim3(G), dim3(512), 0, st, cnt, N, out, err);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        int e = 0;
        CK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
        printf("one launch, %3d workgroups, %d grid barriers: %.2f us per barrier%s\n", G, N, best * 1e3f / N,
               e ? " (SPIN LIMIT HIT)" : "");
    }
    return 0;
}
