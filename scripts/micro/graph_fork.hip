// Do the parallel branches of a captured hipGraph run concurrently on MI355X? (the
// minibatch-64 update: the weight-gradient problems of the top layers could run beside the lower
// layers' backward launches, which use 20-40 of the 256 CUs, if a forked branch overlaps them.)
// Each "work" kernel is G workgroups that each spin for `us` microseconds (wall clock, s_memrealtime
// at 100 MHz). Measured with HIP events over 50 replays of:
//   serial: A ; B                      (one stream)
//   fork:   A || B                     (B captured on a second stream forked / joined with events)
//   chain:  A1 ; A2 ; A3  ||  B        (three dependent launches beside one long one)
// Build: hipcc --offload-arch=gfx950 -O3 -o graph_fork graph_fork.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_spin(float* out, int ticks) {  // ticks of the 100 MHz wall clock
    const unsigned long long t0 = wall_clock64();
    float acc = 0.f;
    while (wall_clock64() - t0 < (unsigned long long)ticks) acc += 1.f;
    if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

static float replay_us(hipGraphExec_t g, hipStream_t s, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipGraphLaunch(g, s));  // warm
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(g, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

int main() {
    float* out;
    CK(hipMalloc(&out, 4096 * sizeof(float)));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    const int G = 40, T20 = 2000, T5 = 500;  // 20 us, 5 us
    for (int mode = 0; mode < 3; ++mode) {
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        if (mode == 0) {
            hipLaunchKernelGGL(k_spin, dim3(G), dim3(512), 0, s, out, T20);
            hipLaunchKernelGGL(k_spin, dim3(G), dim3(512), 0, s, out + 1024, T20);
        } else {
            CK(hipEventRecord(fork, s));
            CK(hipStreamWaitEvent(s2, fork, 0));
            if (mode == 1) {
                hipLaunchKernelGGL(k_spin, dim3(G), dim3(512), 0, s, out, T20);
            } else {
                for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_spin, dim3(G), dim3(512), 0, s, out + 256 * i, T5);
            }
            hipLaunchKernelGGL(k_spin, dim3(G), dim3(512), 0, s2, out + 1024, mode == 1 ? T20 : T5 * 2);
            CK(hipEventRecord(join, s2));
            CK(hipStreamWaitEvent(s, join, 0));
        }
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        const float us = replay_us(ge, s, 50);
        const char* name[3] = {"serial A(20 us) ; B(20 us)        ", "fork   A(20 us) || B(20 us)       ",
                               "chain  3 x 5 us  || B(10 us)       "};
        printf("%s %8.2f us per replay\n", name[mode], us);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
    }
    return 0;
}
