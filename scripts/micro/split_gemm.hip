// fp32-accurate GEMM on the f16 matrix cores: every fp32 operand x is carried as two fp16 planes,
// x1 = f16(x) and x2 = f16((x - x1) * 2^11), and Y = W X^T is summed as
//   hi += W1 X1,  lo += W1 X2 + W2 X1,  Y = hi + 2^-11 lo       (3 x v_mfma_f32_16x16x32_f16)
// against the 8 x v_mfma_f32_16x16x4_f32 the same 16 x 16 x 32 block takes in fp32 (16 vs 32 cycles
// per instruction: 48 vs 256 cycles). Shape of the rollout kernel's critic FFN1 phase: one
// 512-thread workgroup per CU, Y[80 tokens][256 features] = W[256][128] . X[80][128]^T, weights
// streamed from L2 in MFMA fragment order, activations in LDS; each wave owns 2 feature tiles x 5
// token tiles. Variants:
//   f32    : v_mfma_f32_16x16x4_f32, X fp32 in LDS (the production gemm_tile)
//   split  : fp16x3, weights as two fp16 planes, X as two fp16 planes in LDS (split by its producer)
//   otf    : fp16x3, weights as two fp16 planes, X fp32 in LDS split by each wave on the fly
// Prints us per GEMM phase (R phases per launch) and the max error against an fp64 host reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int TOK = 80, KD = 128, NOUT = 256, LDH = KD + 8, LDP = KD + 8;  // LDP: fp16 plane row stride

// fp32 fragment order (production): tile t, k-block kb (16): lane l -> W[16t + l%16][16kb + 4(l/16) + j]
// fp16 fragment order: tile t, k-block kb (32): lane l -> W[16t + l%16][32kb + 8(l/16) + j], per plane

__device__ __forceinline__ void split8(const f32x4 a, const f32x4 b, f16x8& h1, f16x8& h2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = j < 4 ? a[j] : b[j - 4];
        const _Float16 x1 = (_Float16)x;
        h1[j] = x1;
        h2[j] = (_Float16)((x - (float)x1) * 2048.f);
    }
}

template <int VAR>
__global__ __launch_bounds__(512) void k_gemm(const float* __restrict__ W32, const f16x8* __restrict__ W1,
                                              const f16x8* __restrict__ W2, const float* __restrict__ Xg, int R,
                                              float* __restrict__ Y, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) float xs[TOK * LDH];
    __shared__ __attribute__((aligned(16))) _Float16 xp[2][TOK * LDP];
    const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, i16 = l & 15, g = l >> 4;
    for (int i = tid; i < TOK * KD; i += 512) {
        const int t = i / KD, k = i % KD;
        const float x = Xg[i];
        xs[t * LDH + k] = x;
        const _Float16 x1 = (_Float16)x;
        xp[0][t * LDP + k] = x1;
        xp[1][t * LDP + k] = (_Float16)((x - (float)x1) * 2048.f);
    }
    __syncthreads();
    f32x4 acc[2][5], lo[2][5];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int c = 0; c < 5; ++c) acc[m][c] = lo[m][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
        // launder the operand bases each phase: without it LICM hoists every loop-invariant load
        const float* W32r = W32;
        const f16x8 *W1r = W1, *W2r = W2;
        int xo = 0;
        asm volatile("" : "+s"(W32r), "+s"(W1r), "+s"(W2r), "+v"(xo));
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int tile = 2 * wv + m;
            if (VAR == 0) {
                const float* wp = W32r + (size_t)tile * (KD / 16) * 256 + 4 * l;
                f32x4 a[KD / 16];
#pragma unroll
                for (int kb = 0; kb < KD / 16; ++kb) a[kb] = *reinterpret_cast<const f32x4*>(wp + 256 * kb);
#pragma unroll
                for (int kb = 0; kb < KD / 16; ++kb) {
                    f32x4 b[5];
#pragma unroll
                    for (int c = 0; c < 5; ++c)
                        b[c] = *reinterpret_cast<const f32x4*>(xs + xo + (16 * c + i16) * LDH + 16 * kb + 4 * g);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int c = 0; c < 5; ++c)
                            acc[m][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kb][j], b[c][j], acc[m][c], 0, 0, 0);
                }
            } else {
                const f16x8* w1 = W1r + (size_t)tile * (KD / 32) * 64 + l;
                const f16x8* w2 = W2r + (size_t)tile * (KD / 32) * 64 + l;
                f16x8 a1[KD / 32], a2[KD / 32];
#pragma unroll
                for (int kb = 0; kb < KD / 32; ++kb) { a1[kb] = w1[64 * kb]; a2[kb] = w2[64 * kb]; }
#pragma unroll
                for (int kb = 0; kb < KD / 32; ++kb) {
#pragma unroll
                    for (int c = 0; c < 5; ++c) {
                        f16x8 b1, b2;
                        if (VAR == 1) {
                            b1 = *reinterpret_cast<const f16x8*>(&xp[0][xo + (16 * c + i16) * LDP + 32 * kb + 8 * g]);
                            b2 = *reinterpret_cast<const f16x8*>(&xp[1][xo + (16 * c + i16) * LDP + 32 * kb + 8 * g]);
                        } else {
                            const float* xr = xs + xo + (16 * c + i16) * LDH + 32 * kb + 8 * g;
                            split8(*reinterpret_cast<const f32x4*>(xr), *reinterpret_cast<const f32x4*>(xr + 4), b1, b2);
                        }
                        acc[m][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[kb], b1, acc[m][c], 0, 0, 0);
                        lo[m][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[kb], b2, lo[m][c], 0, 0, 0);
                        lo[m][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[kb], b1, lo[m][c], 0, 0, 0);
                    }
                }
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    if (blockIdx.x == 0) {  // Y[tok][feature]: lane (i16, g) of tile (m, c) holds features 4g..4g+3 of token 16c + i16
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int c = 0; c < 5; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    Y[(16 * c + i16) * NOUT + 16 * (2 * wv + m) + 4 * g + j] = acc[m][c][j] + lo[m][c][j] * (1.f / 2048.f);
    }
}

int main() {
    std::vector<float> W(NOUT * KD), X(TOK * KD);
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    for (auto& w : W) w = 0.09f * rnd();
    for (auto& x : X) x = 2.f * rnd();
    // fragment orders
    std::vector<float> W32(NOUT * KD);
    std::vector<_Float16> P1(NOUT * KD), P2(NOUT * KD);
    for (int t = 0; t < NOUT / 16; ++t)
        for (int l = 0; l < 64; ++l) {
            for (int kb = 0; kb < KD / 16; ++kb)
                for (int j = 0; j < 4; ++j)
                    W32[((size_t)t * (KD / 16) + kb) * 256 + 4 * l + j] = W[(16 * t + l % 16) * KD + 16 * kb + 4 * (l / 16) + j];
            for (int kb = 0; kb < KD / 32; ++kb)
                for (int j = 0; j < 8; ++j) {
                    const float x = W[(16 * t + l % 16) * KD + 32 * kb + 8 * (l / 16) + j];
                    const _Float16 x1 = (_Float16)x;
                    P1[(((size_t)t * (KD / 32) + kb) * 64 + l) * 8 + j] = x1;
                    P2[(((size_t)t * (KD / 32) + kb) * 64 + l) * 8 + j] = (_Float16)((x - (float)x1) * 2048.f);
                }
        }
    float *dW32, *dX, *dY;
    f16x8 *dP1, *dP2;
    unsigned long long* dc;
    hipMalloc(&dW32, W32.size() * 4); hipMalloc(&dX, X.size() * 4); hipMalloc(&dY, TOK * NOUT * 4);
    hipMalloc(&dP1, P1.size() * 2); hipMalloc(&dP2, P2.size() * 2); hipMalloc(&dc, 256 * 8);
    hipMemcpy(dW32, W32.data(), W32.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dP1, P1.data(), P1.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dP2, P2.data(), P2.size() * 2, hipMemcpyHostToDevice);
    std::vector<double> ref(TOK * NOUT);
    double rmax = 0;
    for (int t = 0; t < TOK; ++t)
        for (int o = 0; o < NOUT; ++o) {
            double s = 0;
            for (int k = 0; k < KD; ++k) s += (double)W[o * KD + k] * X[t * KD + k];
            ref[t * NOUT + o] = s;
            rmax = fmax(rmax, fabs(s));
        }
    const char* names[3] = {"f32 16x16x4", "f16x3 split planes", "f16x3 on-the-fly split"};
    auto run = [&](auto kern, int var) {
        std::vector<float> Y(TOK * NOUT);
        hipLaunchKernelGGL(kern, dim3(1), dim3(512), 0, 0, dW32, dP1, dP2, dX, 1, dY, dc);
        hipMemcpy(Y.data(), dY, Y.size() * 4, hipMemcpyDeviceToHost);
        double emax = 0;
        for (int i = 0; i < TOK * NOUT; ++i) emax = fmax(emax, fabs(Y[i] - ref[i]));
        const int R = 400;
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, dW32, dP1, dP2, dX, R, dY, dc);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, dW32, dP1, dP2, dX, R, dY, dc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> c(256);
        hipMemcpy(c.data(), dc, 256 * 8, hipMemcpyDeviceToHost);
        double cm = 0;
        for (auto v : c) cm += v;
        cm /= 256;
        const double flop = 2.0 * TOK * NOUT * KD * R * 256;
        printf("%-26s %7.3f us/phase  %8.0f cycles/phase  %6.1f TFLOP/s fp32-equivalent   max|err| %.2e (%.2e of max|y|)\n",
               names[var], ms * 1e3 / R, cm / R, flop / (ms * 1e-3) / 1e12, emax, emax / rmax);
    };
    run(k_gemm<0>, 0);
    run(k_gemm<1>, 1);
    run(k_gemm<2>, 2);
    return 0;
}
