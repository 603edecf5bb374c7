// gemm.hpp -- grouped fp32 MFMA GEMM used by the PPO training step (train.hip): one launch runs a
// list of independent problems (the same layout), each tiled in BM x 64 output tiles (BM = 64 or
// 128), optionally split over K (weight gradients). Included by train.hip and by
// scripts/micro/gemm_bench.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace uavhip {
namespace tr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int gemm_lane() { return threadIdx.x & 63; }

enum Layout { L_FWD = 0, L_DX = 1, L_DW = 2 };
enum Epi { E_STORE = 0, E_BIAS, E_BIAS_RELU, E_ACCUM, E_RELU_MASK, E_SPLIT, E_ADD_RES };

struct GemmProb {
    const float* A;
    const float* B;
    float* C;            // output (E_SPLIT: partial slabs [splits][M][N])
    const float* bias;   // E_BIAS*: [N]
    const float* aux;    // E_RELU_MASK: C = acc * (aux[m][n] > 0); E_ADD_RES: C = acc + residual (below)
    float* bias_part;    // E_SPLIT: [splits][M] row sums of A over the split (the bias gradient)
    int M, N, K, lda, ldb, ldc, ldaux;
    int epi, kchunk, splits, tiles_n, tile_begin;
    int rmod, rrem;      // E_ADD_RES: rows m with m % rmod == rrem add aux[m / rmod] (rmod 0: every row, aux[m])
};
constexpr int kMaxProbs = 16;
struct GemmBatch {
    GemmProb p[kMaxProbs];
    int n, total;  // problems, tiles
};

constexpr int BN = 64, BK = 32, LDS_K = BK + 4;  // 36-float rows: conflict-free float4 operand reads

// A(m, k): L_FWD / L_DX row-major [M][K] (lda); L_DW "column" [K][M] (lda).
// B(k, n): L_FWD = W[n][k] (ldb = K-stride); L_DX / L_DW row-major [K][N] (ldb).
// LDS images are k-contiguous: As[m][k], Bs[n][k].
//
// Thread -> element maps. Row operands: float4 q covers row q >> 3, k-quad q & 7 and is stored
// as one float4. Transposed operands: float4 q covers 4 consecutive m / n at one k, stored as 4
// scalars; within a wave the 16 k and 4 quads it covers hit all 64 LDS banks once
// ((16 a + 36 i + k) mod 64 distinct).
template <int QUADS>
__device__ __forceinline__ void tmap(int q, int& quad, int& k) {
    const int lane = q & 63, w = q >> 6;
    quad = (lane >> 4) + 4 * (w % (QUADS / 4));
    k = (lane & 15) + 16 * (w / (QUADS / 4));
}

// One operand slab (ROWS x 32) in float4 registers: ROWS * 8 / 256 per thread.
template <bool TRANS, int ROWS>
__device__ __forceinline__ void load_op(const float* X, int ld, int r0, int k0, f32x4 (&r)[ROWS / 32]) {
#pragma unroll
    for (int h = 0; h < ROWS / 32; ++h) {
        const int q = threadIdx.x + 256 * h;
        if (TRANS) {
            int a, k;
            tmap<ROWS / 4>(q, a, k);
            r[h] = *reinterpret_cast<const f32x4*>(X + (size_t)(k0 + k) * ld + r0 + 4 * a);
        } else {
            const int m = q >> 3, kq = (q & 7) * 4;
            r[h] = *reinterpret_cast<const f32x4*>(X + (size_t)(r0 + m) * ld + k0 + kq);
        }
    }
}
template <bool TRANS, int ROWS>
__device__ __forceinline__ void store_op(float* Xs, const f32x4 (&r)[ROWS / 32]) {
#pragma unroll
    for (int h = 0; h < ROWS / 32; ++h) {
        const int q = threadIdx.x + 256 * h;
        if (TRANS) {
            int a, k;
            tmap<ROWS / 4>(q, a, k);
            Xs[(4 * a + 0) * LDS_K + k] = r[h].x;
            Xs[(4 * a + 1) * LDS_K + k] = r[h].y;
            Xs[(4 * a + 2) * LDS_K + k] = r[h].z;
            Xs[(4 * a + 3) * LDS_K + k] = r[h].w;
        } else {
            const int m = q >> 3, kq = (q & 7) * 4;
            *reinterpret_cast<f32x4*>(Xs + m * LDS_K + kq) = r[h];
        }
    }
}

struct TileInfo {
    int pi, m0, n0, kb, nslab, split, tni;
};
template <int BM>
__device__ __forceinline__ TileInfo decode_tile(const GemmBatch& gb, int tile) {
    TileInfo ti;
    int pi = 0;
    for (int hi = gb.n; hi - pi > 1;) {  // binary search: each probe is a kernarg load
        const int mid = (pi + hi) >> 1;
        if (tile >= gb.p[mid].tile_begin) pi = mid;
        else hi = mid;
    }
    const GemmProb& P = gb.p[pi];
    const int u = tile - P.tile_begin;
    const int tm_n = P.M / BM, tn_n = P.tiles_n, per_split = tm_n * tn_n;
    ti.pi = pi;
    // XCD-aware order (workgroup b runs on XCD b % 8, the persistent grid is a multiple of 8, so
    // tile u lands on XCD (tile_begin + u) % 8): the tiles that read the same operand slabs share
    // an XCD and its L2 -- all tiles of one K-split (split-K), or all column tiles of one row
    // block (the A slab). Groups of 8 splits / row blocks interleave over the 8 XCDs.
    int tmi;
    if (P.splits > 1) {
        const int g = u / (8 * per_split), r = u - g * 8 * per_split;
        const int gsz = min(8, P.splits - 8 * g);
        ti.split = 8 * g + r % gsz;
        const int j = r / gsz;
        tmi = j / tn_n;
        ti.tni = j - tmi * tn_n;
    } else {
        const int g = u / (8 * tn_n), r = u - g * 8 * tn_n;
        const int gsz = min(8, tm_n - 8 * g);
        ti.split = 0;
        tmi = 8 * g + r % gsz;
        ti.tni = r / gsz;
    }
    ti.m0 = tmi * BM;
    ti.n0 = ti.tni * BN;
    ti.kb = ti.split * P.kchunk;
    ti.nslab = (min(P.K, ti.kb + P.kchunk) - ti.kb) / BK;
    return ti;
}

// Persistent workgroups: workgroup w runs tiles w, w + grid, ... as one stream of 32-deep
// k-slabs (register-staged, LDS double buffer, one barrier per slab), so the first slab of its
// next tile is fetched while the last slab of the current one computes. One BM x 64 output tile
// at a time: wave w computes rows (BM / 2) (w & 1) + [0, BM / 2) and columns 32 (w >> 1) + [0, 32)
// as WTM x 2 MFMA 16 x 16 tiles (WTM = BM / 32). Both operands use the k permutation
// k = 16 h + 4 (lane >> 4) + j for MFMA j of float4 read h (as in policy.hip).
template <int LAYOUT, int WTM>
__global__ __launch_bounds__(256) void k_gemm(const GemmBatch gb) {
    constexpr int BM = 32 * WTM;
    constexpr bool TA = LAYOUT == L_DW, TB = LAYOUT != L_FWD;
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDS_K];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDS_K];
    int tile = blockIdx.x;
    if (tile >= gb.total) return;
    const int l = gemm_lane(), i16 = l & 15, g = l >> 4, wv = threadIdx.x >> 6;
    const int wm = (wv & 1) * (BM / 2), wn = (wv >> 1) * 32;
    TileInfo ti = decode_tile<BM>(gb, tile);

    f32x4 ra[BM / 32], rb[BN / 32];
    load_op<TA, BM>(gb.p[ti.pi].A, gb.p[ti.pi].lda, ti.m0, ti.kb, ra);
    load_op<TB, BN>(gb.p[ti.pi].B, gb.p[ti.pi].ldb, ti.n0, ti.kb, rb);
    store_op<TA, BM>(As[0], ra);
    store_op<TB, BN>(Bs[0], rb);
    __syncthreads();
    int buf = 0;
    while (true) {
        const GemmProb& P = gb.p[ti.pi];
        const int next = tile + (int)gridDim.x;
        const bool more = next < gb.total;
        TileInfo tn = ti;
        if (more) tn = decode_tile<BM>(gb, next);
        const bool rowsum = P.epi == E_SPLIT && P.bias_part && ti.tni == 0;
        float rs = 0.f;  // row sum of A for row m0 + threadIdx.x (threads < BM)
        f32x4 acc[WTM][2];
#pragma unroll
        for (int a = 0; a < WTM; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < ti.nslab; ++s) {
            const bool last = s + 1 == ti.nslab;
            if (!last) {
                load_op<TA, BM>(P.A, P.lda, ti.m0, ti.kb + (s + 1) * BK, ra);
                load_op<TB, BN>(P.B, P.ldb, ti.n0, ti.kb + (s + 1) * BK, rb);
            } else if (more) {
                const GemmProb& Q = gb.p[tn.pi];
                load_op<TA, BM>(Q.A, Q.lda, tn.m0, tn.kb, ra);
                load_op<TB, BN>(Q.B, Q.ldb, tn.n0, tn.kb, rb);
            }
            const float* as = As[buf];
            const float* bs = Bs[buf];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f32x4 fa[WTM], fb[2];
#pragma unroll
                for (int x = 0; x < WTM; ++x)
                    fa[x] = *reinterpret_cast<const f32x4*>(as + (wm + 16 * x + i16) * LDS_K + 16 * h + 4 * g);
#pragma unroll
                for (int x = 0; x < 2; ++x)
                    fb[x] = *reinterpret_cast<const f32x4*>(bs + (wn + 16 * x + i16) * LDS_K + 16 * h + 4 * g);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int a = 0; a < WTM; ++a)
#pragma unroll
                        for (int b = 0; b < 2; ++b)
                            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[b][j], fa[a][j], acc[a][b], 0, 0, 0);
            }
            if (rowsum && threadIdx.x < BM) {
                const float* row = as + threadIdx.x * LDS_K;
#pragma unroll
                for (int k = 0; k < BK; k += 4) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(row + k);
                    rs += (v.x + v.y) + (v.z + v.w);
                }
            }
            if (!last || more) {
                store_op<TA, BM>(As[buf ^ 1], ra);
                store_op<TB, BN>(Bs[buf ^ 1], rb);
            }
            __syncthreads();
            buf ^= 1;
        }
        if (rowsum && threadIdx.x < BM) P.bias_part[(size_t)ti.split * P.M + ti.m0 + threadIdx.x] = rs;

        // epilogue: the MFMA computed C^T (B-tile rows as its A operand), so lane (i16, g) of tile
        // (a, b) holds 4 consecutive columns C[m0 + wm + 16a + i16][n0 + wn + 16b + 4g + (0..3)]:
        // one float4 store per (a, b)
        float* C = P.epi == E_SPLIT ? P.C + (size_t)ti.split * P.M * P.N : P.C;
        const int ldc = P.epi == E_SPLIT ? P.N : P.ldc;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int n = ti.n0 + wn + 16 * b + 4 * g;
            f32x4 bv = {0.f, 0.f, 0.f, 0.f};
            if (P.epi == E_BIAS || P.epi == E_BIAS_RELU) bv = *reinterpret_cast<const f32x4*>(P.bias + n);
#pragma unroll
            for (int a = 0; a < WTM; ++a) {
                const int m = ti.m0 + wm + 16 * a + i16;
                f32x4 v = acc[a][b];
                f32x4* cp = reinterpret_cast<f32x4*>(C + (size_t)m * ldc + n);
                switch (P.epi) {
                    case E_BIAS: v = v + bv; break;
                    case E_BIAS_RELU:
                        v = v + bv;
                        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
                        break;
                    case E_ACCUM: v = *cp + v; break;
                    case E_ADD_RES:
                        if (P.rmod == 0 || m % P.rmod == P.rrem)
                            v = v + *reinterpret_cast<const f32x4*>(P.aux + (size_t)(P.rmod ? m / P.rmod : m) * P.ldaux + n);
                        break;
                    case E_RELU_MASK: {
                        const f32x4 u = *reinterpret_cast<const f32x4*>(P.aux + (size_t)m * P.ldaux + n);
                        v.x = u.x > 0.f ? v.x : 0.f; v.y = u.y > 0.f ? v.y : 0.f;
                        v.z = u.z > 0.f ? v.z : 0.f; v.w = u.w > 0.f ? v.w : 0.f;
                        break;
                    }
                    default: break;
                }
                *cp = v;
            }
        }
        if (!more) break;
        tile = next;
        ti = tn;
    }
}

// Resident workgroups per CU by LDS (2 x (BM + 64) x 36 floats each): 4 at BM = 64, 2 at 128.
constexpr int kCUs = 256;

struct GemmBuilder {
    GemmBatch gb{};
    int tiles = 0;
    int bm;
    explicit GemmBuilder(int bm_ = 64) : bm(bm_) {}
    void add(const float* A, int lda, const float* B, int ldb, float* C, int ldc, int M, int N, int K, int epi,
             const float* bias = nullptr, const float* aux = nullptr, int ldaux = 0, float* bias_part = nullptr,
             int kchunk = 0) {
        GemmProb& P = gb.p[gb.n++];
        P.A = A; P.B = B; P.C = C; P.bias = bias; P.aux = aux; P.bias_part = bias_part;
        P.M = M; P.N = N; P.K = K; P.lda = lda; P.ldb = ldb; P.ldc = ldc; P.ldaux = ldaux;
        P.epi = epi;
        P.kchunk = kchunk > 0 ? kchunk : K;
        P.splits = (K + P.kchunk - 1) / P.kchunk;
        P.tiles_n = N / BN;
        P.tile_begin = tiles;
        tiles += P.splits * (M / bm) * P.tiles_n;
        gb.total = tiles;
        P.rmod = P.rrem = 0;
    }
    // C = A B + residual rows of `res` (see E_ADD_RES)
    void add_res(const float* A, int lda, const float* B, int ldb, float* C, int ldc, int M, int N, int K,
                 const float* res, int ldres, int rmod, int rrem) {
        add(A, lda, B, ldb, C, ldc, M, N, K, E_ADD_RES, nullptr, res, ldres);
        gb.p[gb.n - 1].rmod = rmod;
        gb.p[gb.n - 1].rrem = rrem;
    }
    bool valid() const {  // the shapes the kernel assumes
        for (int i = 0; i < gb.n; ++i) {
            const GemmProb& P = gb.p[i];
            if (P.M % bm || P.N % BN || P.K % BK || P.kchunk % BK || P.lda % 4 || P.ldb % 4 || P.ldc % 4 ||
                P.ldaux % 4)
                return false;
        }
        return gb.n <= kMaxProbs;
    }
};

template <int LAYOUT>
void launch_gemm(const GemmBuilder& g, hipStream_t st) {
    if (g.gb.n == 0) return;
    const int per_cu = g.bm == 128 ? 2 : 4;
    const int grid = g.tiles < per_cu * kCUs ? g.tiles : per_cu * kCUs;
    if (g.bm == 128) hipLaunchKernelGGL((k_gemm<LAYOUT, 4>), dim3(grid), dim3(256), 0, st, g.gb);
    else hipLaunchKernelGGL((k_gemm<LAYOUT, 2>), dim3(grid), dim3(256), 0, st, g.gb);
}

}  // namespace tr
}  // namespace uavhip
