// Grouped fp32 MFMA GEMM (csrc/gemm.hpp) at the PPO training-step shapes: correctness against a
// naive kernel and TFLOP/s per launch. Build: hipcc -O3 --offload-arch=gfx950 -o gemm_bench gemm_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../target-allocation-ppo-transformer_amd/csrc/gemm.hpp"
#include "rowgemm.hpp"

using namespace uavhip::tr;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// C[m][n] = sum_k A(m,k) B(k,n) for the three layouts
__global__ void k_ref(int layout, const float* A, int lda, const float* B, int ldb, float* C, int M, int N, int K) {
    const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double acc = 0;
    for (int k = 0; k < K; ++k) {
        const float a = layout == L_DW ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k];
        const float b = layout == L_FWD ? B[(size_t)n * ldb + k] : B[(size_t)k * ldb + n];
        acc += (double)a * b;
    }
    C[(size_t)m * N + n] = (float)acc;
}

float* dalloc(size_t n) {
    float* p; CK(hipMalloc(&p, n * 4));
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (float)((rand() % 2001) - 1000) / 1000.f;
    CK(hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice));
    return p;
}

template <int LAYOUT>
double time_it(const GemmBuilder& g, int reps = 20) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) launch_gemm<LAYOUT>(g, 0);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch_gemm<LAYOUT>(g, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}

double flops(const GemmBuilder& g) {
    double f = 0;
    for (int i = 0; i < g.gb.n; ++i) f += 2.0 * g.gb.p[i].M * g.gb.p[i].N * g.gb.p[i].K;
    return f;
}

template <int LAYOUT>
void check(const char* name, const GemmProb& P) {  // first problem, E_STORE / E_SPLIT slab 0 only
    float* ref; CK(hipMalloc(&ref, (size_t)P.M * P.N * 4));
    const int K = P.epi == E_SPLIT ? P.kchunk : P.K;
    hipLaunchKernelGGL(k_ref, dim3((P.N + 127) / 128, P.M), dim3(128), 0, 0, LAYOUT, P.A, P.lda, P.B, P.ldb, ref, P.M, P.N, K);
    CK(hipDeviceSynchronize());
    std::vector<float> a((size_t)P.M * P.N), b((size_t)P.M * P.N);
    CK(hipMemcpy(a.data(), ref, a.size() * 4, hipMemcpyDeviceToHost));
    std::vector<float> c((size_t)P.M * P.ldc);
    if (P.epi == E_SPLIT) CK(hipMemcpy(b.data(), P.C, b.size() * 4, hipMemcpyDeviceToHost));
    else {
        CK(hipMemcpy(c.data(), P.C, c.size() * 4, hipMemcpyDeviceToHost));
        for (int m = 0; m < P.M; ++m) for (int n = 0; n < P.N; ++n) b[(size_t)m * P.N + n] = c[(size_t)m * P.ldc + n];
    }
    double md = 0, ms = 0;
    for (size_t i = 0; i < a.size(); ++i) { md = fmax(md, fabs(a[i] - b[i])); ms = fmax(ms, fabs(a[i])); }
    printf("  check %-10s max|d| %.3e (scale %.3e)%s\n", name, md, ms, md > 1e-4 * ms ? "  MISMATCH" : "");
    CK(hipFree(ref));
}

int main() {
    const int R = 20480, Bm = 4096, D = 128, FF = 256;
    float* h = dalloc((size_t)R * D);
    float* h2 = dalloc((size_t)R * D);
    float* win = dalloc(3 * D * D);
    float* win2 = dalloc(3 * D * D);
    float* bias = dalloc(3 * D);
    float* qkv = dalloc((size_t)R * 3 * D);
    float* qkv2 = dalloc((size_t)R * 3 * D);
    float* w1 = dalloc(FF * D);
    float* w2 = dalloc(D * FF);
    float* u = dalloc((size_t)R * FF);
    float* f = dalloc((size_t)R * D);
    float* dh = dalloc((size_t)R * D);
    float* dh2 = dalloc((size_t)R * D);
    float* ws = dalloc((size_t)40 << 20);
    for (int bm : {64, 128}) {
    {
        GemmBuilder g(bm);
        g.add(h, D, win, D, qkv, 3 * D, R, 3 * D, D, E_STORE);
        g.add(h2, D, win2, D, qkv2, 3 * D, R, 3 * D, D, E_BIAS, bias);
        const double us = time_it<L_FWD>(g);
        printf("bm=%3d FWD qkv x2   (M=%d N=384 K=128): %7.1f us  %6.1f TF/s  tiles %d\n", bm, R, us, flops(g) / us / 1e6, g.tiles);
        check<L_FWD>("fwd", g.gb.p[0]);
    }
    {
        GemmBuilder g(bm);
        g.add(h, D, w1, D, u, FF, R, FF, D, E_BIAS_RELU, bias);
        g.add(h2, D, w1, D, u, FF, Bm, FF, D, E_BIAS_RELU, bias);
        const double us = time_it<L_FWD>(g);
        printf("bm=%3d FWD ffn1     (M=%d+%d N=256 K=128): %7.1f us  %6.1f TF/s\n", bm, R, Bm, us, flops(g) / us / 1e6);
    }
    {
        GemmBuilder g(bm);
        g.add(u, FF, w2, FF, f, D, R, D, FF, E_BIAS, bias);
        const double us = time_it<L_FWD>(g);
        printf("bm=%3d FWD ffn2     (M=%d N=128 K=256): %7.1f us  %6.1f TF/s\n", bm, R, us, flops(g) / us / 1e6);
    }
    {
        GemmBuilder g(bm);
        g.add(qkv, 3 * D, win, D, dh, D, R, D, 3 * D, E_STORE);
        g.add(qkv2, 3 * D, win2, D, dh2, D, R, D, 3 * D, E_ACCUM);
        const double us = time_it<L_DX>(g);
        printf("bm=%3d DX  win x2   (M=%d N=128 K=384): %7.1f us  %6.1f TF/s\n", bm, R, us, flops(g) / us / 1e6);
        check<L_DX>("dx", g.gb.p[0]);
    }
    {
        GemmBuilder g(bm);
        g.add(f, D, w2, FF, u, FF, R, FF, D, E_RELU_MASK, nullptr, u, FF);
        const double us = time_it<L_DX>(g);
        printf("bm=%3d DX  w2 relu  (M=%d N=256 K=128): %7.1f us  %6.1f TF/s\n", bm, R, us, flops(g) / us / 1e6);
    }
    {
        GemmBuilder g(bm);
        float* p = ws;
        const int kc = 2048;
        auto add = [&](const float* A, int lda, const float* B, int ldb, int M, int N, int K) {
            const int sp = (K + kc - 1) / kc;
            g.add(A, lda, B, ldb, p, N, M, N, K, E_SPLIT, nullptr, nullptr, 0, p + (size_t)sp * M * N, kc);
            p += (size_t)sp * ((size_t)M * N + M);
        };
        add(qkv, 3 * D, h, D, 3 * D, D, R);
        add(qkv2, 3 * D, h2, D, 3 * D, D, R);
        add(f, D, h, D, D, D, R);
        add(u, FF, h, D, FF, D, R);
        add(f, D, u, FF, D, FF, R);
        add(qkv, 3 * D, h2, D, 3 * D, D, R);
        add(f, D, h, D, D, D, Bm);
        add(u, FF, h, D, FF, D, Bm);
        add(f, D, u, FF, D, FF, Bm);
        const double us = time_it<L_DW>(g);
        printf("bm=%3d DW  9 probs  (split-K %d): %7.1f us  %6.1f TF/s  tiles %d\n", bm, kc, us, flops(g) / us / 1e6, g.tiles);
        check<L_DW>("dw", g.gb.p[0]);
    }
    }
    // ---- weights-resident row GEMM
    auto rtime = [&](const RowBuilder& g, int grid) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        for (int i = 0; i < 3; ++i) launch_rowgemm(g, 0, grid);
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; ++i) launch_rowgemm(g, 0, grid);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipGetLastError());
        return ms * 1e3 / 20;
    };
    auto rflops = [&](const RowBuilder& g) {
        double f = 0;
        for (int i = 0; i < g.rb.n; ++i) f += 2.0 * g.rb.p[i].M * g.rb.p[i].N * g.rb.p[i].K;
        return f;
    };
    float* xh = dalloc((size_t)R * D);
    float* rsd = dalloc(R);
    float* lnw = dalloc(D);
    for (int grid : {256, 512}) {
        {
            RowBuilder g; g.K = 128;
            RowProb p{}; p.A = h; p.lda = D; p.B = win; p.ldb = D; p.C = qkv; p.ldc = 3 * D; p.bias = bias;
            p.M = R; p.N = 3 * D; p.K = D; p.epi = R_BIAS; g.add(p);
            RowProb q = p; q.A = h2; q.B = win2; q.C = qkv2; g.add(q);
            const double us = rtime(g, grid);
            printf("grid %d ROW FWD qkv x2 (M=%d N=384 K=128): %7.1f us %6.1f TF/s valid %d\n", grid, R, us, rflops(g) / us / 1e6, (int)g.valid());
            if (grid == 256) {
                GemmProb c{}; c.A = h; c.lda = D; c.B = win; c.ldb = D; c.C = qkv; c.ldc = 3 * D; c.M = R; c.N = 3 * D; c.K = D; c.epi = E_STORE;
                // recompute with bias-free store for the check
                RowBuilder g2; g2.K = 128; RowProb p2 = p; p2.epi = R_STORE; g2.add(p2); launch_rowgemm(g2, 0, grid); CK(hipDeviceSynchronize());
                check<L_FWD>("row fwd", c);
            }
        }
        {
            RowBuilder g; g.K = 128;
            RowProb p{}; p.A = f; p.lda = D; p.B = win; p.ldb = D; p.C = dh; p.ldc = D; p.bias = bias; p.aux = h; p.ldaux = D;
            p.lnw = lnw; p.lnb = bias; p.xhat = xh; p.rstd = rsd; p.rmod = 1; p.rrem = 0;
            p.M = R; p.N = D; p.K = D; p.epi = R_BIAS_RES_LN; g.add(p);
            const double us = rtime(g, grid);
            printf("grid %d ROW FWD out+LN (M=%d N=128 K=128): %7.1f us %6.1f TF/s\n", grid, R, us, rflops(g) / us / 1e6);
        }
        {
            RowBuilder g; g.K = 128;
            RowProb p{}; p.A = h; p.lda = D; p.B = w1; p.ldb = D; p.C = u; p.ldc = FF; p.bias = bias;
            p.M = R; p.N = FF; p.K = D; p.epi = R_BIAS_RELU; g.add(p);
            const double us = rtime(g, grid);
            printf("grid %d ROW FWD ffn1 (M=%d N=256 K=128): %7.1f us %6.1f TF/s\n", grid, R, us, rflops(g) / us / 1e6);
        }
        {
            RowBuilder g; g.K = 256;
            RowProb p{}; p.A = u; p.lda = FF; p.B = w2; p.ldb = FF; p.C = f; p.ldc = D; p.bias = bias; p.aux = h; p.ldaux = D;
            p.lnw = lnw; p.lnb = bias; p.xhat = xh; p.rstd = rsd; p.rmod = 1; p.rrem = 0;
            p.M = R; p.N = D; p.K = FF; p.epi = R_BIAS_RES_LN; g.add(p);
            const double us = rtime(g, grid);
            printf("grid %d ROW FWD ffn2+LN (M=%d N=128 K=256): %7.1f us %6.1f TF/s\n", grid, R, us, rflops(g) / us / 1e6);
        }
        {
            RowBuilder g; g.K = 128; g.rb.bt = 1;
            RowProb p{}; p.A = f; p.lda = D; p.B = w2; p.ldb = FF; p.C = u; p.ldc = FF; p.aux = u; p.ldaux = FF;
            p.M = R; p.N = FF; p.K = D; p.epi = R_RELU_MASK; g.add(p);
            const double us = rtime(g, grid);
            printf("grid %d ROW DX w2 relu (M=%d N=256 K=128): %7.1f us %6.1f TF/s\n", grid, R, us, rflops(g) / us / 1e6);
            if (grid == 256) {
                RowBuilder g2; g2.K = 128; g2.rb.bt = 1; RowProb p2 = p; p2.epi = R_STORE; g2.add(p2); launch_rowgemm(g2, 0, grid); CK(hipDeviceSynchronize());
                GemmProb c{}; c.A = f; c.lda = D; c.B = w2; c.ldb = FF; c.C = u; c.ldc = FF; c.M = R; c.N = FF; c.K = D; c.epi = E_STORE;
                check<L_DX>("row dx", c);
            }
        }
        {
            RowBuilder g; g.K = 256; g.rb.bt = 1;
            RowProb p{}; p.A = u; p.lda = FF; p.B = w1; p.ldb = D; p.C = dh; p.ldc = D; p.aux = f; p.ldaux = D;
            p.M = R; p.N = D; p.K = FF; p.epi = R_ADD_RES; g.add(p);
            const double us = rtime(g, grid);
            printf("grid %d ROW DX w1 +res (M=%d N=128 K=256): %7.1f us %6.1f TF/s\n", grid, R, us, rflops(g) / us / 1e6);
        }
    }
    return 0;
}
