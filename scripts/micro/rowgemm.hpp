// rowgemm.hpp -- "weights resident" fp32 MFMA GEMM for the PPO training step: C[M][128-column
// block] = A[M][K] B[K][block] with the whole B block (a weight matrix slice, K <= 256) staged in
// LDS ONCE per workgroup and the activations A streamed from global memory straight into MFMA
// registers (each A element is read by one wave per column block). No barrier in the k-loop; a
// persistent workgroup walks row tiles. A wave owns 32 full rows of the 128-column block, so
// row-wise epilogues (bias, ReLU, residual add, LayerNorm forward) fuse.
#pragma once
#include <hip/hip_runtime.h>

namespace uavhip {
namespace tr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum RowEpi {
    R_STORE = 0,   // C = acc
    R_BIAS,        // C = acc + bias
    R_BIAS_RELU,   // C = relu(acc + bias)
    R_RELU_MASK,   // C = acc * (aux > 0)
    R_ADD_RES,     // C = acc + res (rows mapped by rmod / rrem as in gemm.hpp E_ADD_RES)
    R_BIAS_RES_LN, // z = acc + bias + res[row]; C = LN(z) * lnw + lnb, xhat / rstd saved (post-LN)
};

struct RowProb {
    const float* A;  // [M][K] rows (lda), row m at A + m * lda
    const float* B;  // BT = false: W[n][k] (ldb = k stride); BT = true: W[k][n] (ldb = n stride)
    float* C;        // [M][ldc], columns n0 .. n0 + 127
    const float* bias;
    const float* aux;   // R_RELU_MASK mask source [M][ldaux]; R_ADD_RES / R_*LN residual [.][ldaux]
    const float* lnw;   // R_BIAS_RES_LN: LayerNorm weight / bias
    const float* lnb;
    float* xhat;        // R_BIAS_RES_LN: [M][128] normalised rows (saved for the backward)
    float* rstd;        // [M]
    int M, N, K, lda, ldb, ldc, ldaux;
    int epi, rmod, rrem, nblocks_n, tile_begin;  // R_ADD_RES: rows m % rmod == rrem add res[m / rmod]
                                                 // (rmod 0: res[m]); R_BIAS_RES_LN: res row m * rmod + rrem
};
constexpr int kRowMaxProbs = 8;
struct RowBatch {
    RowProb p[kRowMaxProbs];
    int n, total, bt;
};

constexpr int RG_ROWS = 32;   // rows per wave
constexpr int RG_WAVES = 8;   // waves per workgroup (2 per SIMD)
constexpr int RG_TILE = RG_ROWS * RG_WAVES;  // 256 rows per workgroup tile
constexpr int RG_COLS = 128;

__device__ __forceinline__ int rg_lane() { return threadIdx.x & 63; }

__device__ __forceinline__ float rg_xor16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float rg_xor32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// K <= 256 and a multiple of 16; M a multiple of 32 (a wave's rows); N a multiple of 128.
template <int K>
__global__ __launch_bounds__(RG_WAVES * 64) void k_rowgemm(const RowBatch rb) {
    constexpr int LDW = K + 4;  // (K + 4) / 4 = odd number of 16-B slots: conflict-free b128 reads
    extern __shared__ __attribute__((aligned(16))) float Ws[];  // [128][LDW]
    const int l = rg_lane(), i16 = l & 15, g = l >> 4, wv = threadIdx.x >> 6;
    int cur_block = -1;  // (problem, column block) currently staged
    for (int tile = blockIdx.x; tile < rb.total; tile += gridDim.x) {
        int pi = 0;
        while (pi + 1 < rb.n && tile >= rb.p[pi + 1].tile_begin) ++pi;
        const RowProb& P = rb.p[pi];
        const int u = tile - P.tile_begin;
        const int nb = u % P.nblocks_n, rt = u / P.nblocks_n;
        const int key = pi * 64 + nb;
        if (key != cur_block) {  // stage W[n0 .. n0 + 127][0 .. K) as Ws[n][k]
            __syncthreads();
            const int n0 = nb * RG_COLS;
            if (!rb.bt) {
                for (int q = threadIdx.x; q < RG_COLS * K / 4; q += RG_WAVES * 64) {
                    const int n = q / (K / 4), k4 = (q % (K / 4)) * 4;
                    *reinterpret_cast<f32x4*>(Ws + n * LDW + k4) =
                        *reinterpret_cast<const f32x4*>(P.B + (size_t)(n0 + n) * P.ldb + k4);
                }
            } else {
                for (int q = threadIdx.x; q < RG_COLS * K / 4; q += RG_WAVES * 64) {
                    const int k = q / (RG_COLS / 4), n4 = (q % (RG_COLS / 4)) * 4;
                    const f32x4 v = *reinterpret_cast<const f32x4*>(P.B + (size_t)k * P.ldb + n0 + n4);
                    Ws[(n4 + 0) * LDW + k] = v.x;
                    Ws[(n4 + 1) * LDW + k] = v.y;
                    Ws[(n4 + 2) * LDW + k] = v.z;
                    Ws[(n4 + 3) * LDW + k] = v.w;
                }
            }
            __syncthreads();
            cur_block = key;
        }
        const int r0 = rt * RG_TILE + wv * RG_ROWS;
        if (r0 >= P.M) continue;
        const int n0 = nb * RG_COLS;
        // acc[a][b]: rows r0 + 16a + i16, columns n0 + 16b + 4g + (0..3) (C computed transposed)
        f32x4 acc[2][8];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* ap0 = P.A + (size_t)(r0 + i16) * P.lda + 4 * g;
        const float* ap1 = ap0 + (size_t)16 * P.lda;
        constexpr int KB = K / 16;
        f32x4 fa[KB][2];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {  // all of this wave's A fragments up front (K <= 256)
            fa[kb][0] = *reinterpret_cast<const f32x4*>(ap0 + 16 * kb);
            fa[kb][1] = *reinterpret_cast<const f32x4*>(ap1 + 16 * kb);
        }
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            f32x4 fb[8];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                fb[b] = *reinterpret_cast<const f32x4*>(Ws + (16 * b + i16) * LDW + 16 * kb + 4 * g);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[b][j], fa[kb][a][j], acc[a][b], 0, 0, 0);
        }
        // ---------------------------------------------------------------- epilogue
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int m = r0 + 16 * a + i16;
            float* crow = P.C + (size_t)m * P.ldc + n0;
            f32x4 v[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) v[b] = acc[a][b];
            const int col = 4 * g;  // + 16 b
            if (P.epi == R_BIAS || P.epi == R_BIAS_RELU || P.epi == R_BIAS_RES_LN) {
#pragma unroll
                for (int b = 0; b < 8; ++b) v[b] += *reinterpret_cast<const f32x4*>(P.bias + n0 + 16 * b + col);
            }
            if (P.epi == R_BIAS_RELU) {
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    v[b].x = fmaxf(v[b].x, 0.f); v[b].y = fmaxf(v[b].y, 0.f);
                    v[b].z = fmaxf(v[b].z, 0.f); v[b].w = fmaxf(v[b].w, 0.f);
                }
            } else if (P.epi == R_RELU_MASK) {
                const float* ar = P.aux + (size_t)m * P.ldaux + n0;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const f32x4 u4 = *reinterpret_cast<const f32x4*>(ar + 16 * b + col);
                    v[b].x = u4.x > 0.f ? v[b].x : 0.f; v[b].y = u4.y > 0.f ? v[b].y : 0.f;
                    v[b].z = u4.z > 0.f ? v[b].z : 0.f; v[b].w = u4.w > 0.f ? v[b].w : 0.f;
                }
            } else if (P.epi == R_ADD_RES) {
                if (P.rmod == 0 || m % P.rmod == P.rrem) {
                    const float* rr = P.aux + (size_t)(P.rmod ? m / P.rmod : m) * P.ldaux + n0;
#pragma unroll
                    for (int b = 0; b < 8; ++b) v[b] += *reinterpret_cast<const f32x4*>(rr + 16 * b + col);
                }
            } else if (P.epi == R_BIAS_RES_LN) {  // residual row m * rmod + rrem (token-4 rows if pruned)
                const float* rr = P.aux + (size_t)(m * P.rmod + P.rrem) * P.ldaux + n0;
#pragma unroll
                for (int b = 0; b < 8; ++b) v[b] += *reinterpret_cast<const f32x4*>(rr + 16 * b + col);
            }
            if (P.epi == R_BIAS_RES_LN) {  // full row = these 4 lanes (g) x 32 values
                float s = 0.f;
#pragma unroll
                for (int b = 0; b < 8; ++b) s += (v[b].x + v[b].y) + (v[b].z + v[b].w);
                s = rg_xor32(rg_xor16(s));
                const float mean = s * (1.0f / RG_COLS);
                float q = 0.f;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    v[b] -= mean;
                    q += (v[b].x * v[b].x + v[b].y * v[b].y) + (v[b].z * v[b].z + v[b].w * v[b].w);
                }
                q = rg_xor32(rg_xor16(q));
                const float rs = 1.0f / sqrtf(q * (1.0f / RG_COLS) + 1e-5f);
                float* xr = P.xhat + (size_t)m * RG_COLS;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    v[b] *= rs;
                    *reinterpret_cast<f32x4*>(xr + 16 * b + col) = v[b];
                    v[b] = v[b] * *reinterpret_cast<const f32x4*>(P.lnw + 16 * b + col) +
                           *reinterpret_cast<const f32x4*>(P.lnb + 16 * b + col);
                }
                if (g == 0) P.rstd[m] = rs;
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) *reinterpret_cast<f32x4*>(crow + 16 * b + col) = v[b];
        }
    }
}

struct RowBuilder {
    RowBatch rb{};
    int K = 0;
    void add(const RowProb& p) {
        RowProb& P = rb.p[rb.n++];
        P = p;
        P.nblocks_n = P.N / RG_COLS;
        P.tile_begin = rb.total;
        rb.total += ((P.M + RG_TILE - 1) / RG_TILE) * P.nblocks_n;
    }
    bool valid() const {
        for (int i = 0; i < rb.n; ++i) {
            const RowProb& P = rb.p[i];
            if (P.M % RG_ROWS || P.N % RG_COLS || P.K != K || P.lda % 4 || P.ldb % 4 || P.ldc % 4) return false;
        }
        return rb.n <= kRowMaxProbs && (K == 128 || K == 256);
    }
};

inline size_t rowgemm_lds(int K) { return (size_t)RG_COLS * (K + 4) * sizeof(float); }

inline void launch_rowgemm(const RowBuilder& g, hipStream_t st, int grid) {
    if (g.rb.n == 0) return;
    const int gr = g.rb.total < grid ? g.rb.total : grid;
    if (g.K == 128) hipLaunchKernelGGL((k_rowgemm<128>), dim3(gr), dim3(RG_WAVES * 64), rowgemm_lds(128), st, g.rb);
    else hipLaunchKernelGGL((k_rowgemm<256>), dim3(gr), dim3(RG_WAVES * 64), rowgemm_lds(256), st, g.rb);
}

}  // namespace tr
}  // namespace uavhip
