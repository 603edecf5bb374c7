// wgrad.hpp -- weight gradients of the PPO training step (train.hip): for a list of problems,
// dW[m][n] = sum_k dY[k][m] X[k][n] over the minibatch rows k, fp32 on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32). Bias gradients (sums of dY over k) come from k_policy_backward's
// per-workgroup partials, not from here.
//
// Operands. dY and X are the workspace's [row][feature] activations, so both are k-major: the LDS
// images are copies of the global rows ([64 k][128] per operand and slab), filled by
// global_load_lds_dwordx4 with no transposition and no register staging. MFMA fragments are read
// along m / n with ds_read_b128: lane (i, g) reads columns 4i..4i+3 of row k = 4 kk + g, which is
// row i of four 16 x 16 tiles at once (tile a holds the columns 4i + a). A quarter wave reads 256
// contiguous bytes: conflict-free. The epilogue undoes the column permutation with float4 stores.
//
// Workgroup: 512 threads = 8 waves, one 128 x 128 output tile; wave w computes the 64 x 64
// quadrant w & 3 over the k-steps of parity w >> 2 (4 x 4 MFMA tiles, 64 accumulator VGPRs), the
// two parities are added through LDS at the end. LDS: 2 stages x (A + B) x 64 x 128 floats = 128
// KiB, one workgroup per CU.
//
// Work split (stream-K over 64-deep k-slabs): the problems' 128 x 128 output tiles x K / 64 slabs
// form one list (problem-major, then tile, then k); workgroup w takes the contiguous range
// [w U / G, (w + 1) U / G) and accumulates each tile's slabs in registers, writing one partial
// tile per (workgroup, tile) run into slot kWgRuns w + j (j = the run's index within the
// workgroup). The host enumerates the same runs (WgPlan) to build the reduction segments: a tile's
// runs are slot kWgRuns w0 + j0, then kWgRuns w + 0 for w = w0 + 1 .. w1.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

namespace uavhip {
namespace tr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWgT = 128;                 // output tile edge
constexpr int kWgBK = 64;                 // k rows per slab
constexpr int kWgThreads = 512;
constexpr int kWgRuns = 3;                // partial slots per workgroup
constexpr int kWgSlot = kWgT * kWgT;      // floats per partial slot
constexpr int kWgMaxProbs = 16;
constexpr int kWgGrid = 256;              // one workgroup per CU

struct WgProb {
    const float* A;  // dY: row k at A + k * lda, columns m
    const float* B;  // X:  row k at B + k * ldb, columns n
    int M, N, K, lda, ldb;
    int tiles_n, tiles, slabs;  // per problem: column tiles, tiles, slabs per tile
    int unit_begin;             // first slab unit of this problem
};
struct WgBatch {
    WgProb p[kWgMaxProbs];
    int n;
    int units;
    float* part;  // [grid * kWgRuns][kWgSlot]
};

typedef __attribute__((address_space(3))) void wg_lds_void;
typedef __attribute__((address_space(1))) void wg_glob_void;

// Stamps (make TRACE=1 only): per workgroup, s_memtime at kernel start and, per run, after the
// first slab landed / after the k-loop / after the epilogue (uavhip_wgrad_trace copies them out).
#ifdef UAVHIP_POLICY_TRACE
__device__ unsigned long long g_wtrace[kWgGrid * 16];
#define WTR(slot)                                                                                   \
    do {                                                                                            \
        if (threadIdx.x == 0 && (slot) < 16) g_wtrace[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define WTR(slot) do {} while (0)
#endif

__device__ __forceinline__ int wg_find(const WgBatch& b, int u) {
    int lo = 0, hi = b.n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (u >= b.p[mid].unit_begin) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Issue the global_load_lds of one 64 x 128 slab of an operand (rows k0.., columns c0..) into
// `lds` ([64][128] floats): 32 row pairs (1 KiB each), 4 per wave. Columns >= ncols (a 64-wide
// problem) load column c0 instead; those products land in output rows that are never stored.
__device__ __forceinline__ void wg_load_slab(const float* X, int ld, int k0, int c0, int ncols, float* lds) {
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    int col = 4 * (l & 31);
    if (c0 + col >= ncols) col = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int rp = 4 * wv + q;
        const float* src = X + (size_t)(k0 + 2 * rp + (l >> 5)) * ld + c0 + col;
        __builtin_amdgcn_global_load_lds((wg_glob_void*)src, (wg_lds_void*)(lds + rp * 256), 16, 0, 0);
    }
}

__global__ __launch_bounds__(kWgThreads) void k_wgrad(const WgBatch wb) {
    // stage s: A at wg_smem + 2 s * kWgBK * kWgT, B right after it
    __shared__ __attribute__((aligned(16))) float wg_smem[4 * kWgBK * kWgT];
    constexpr int kStage = 2 * kWgBK * kWgT;
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, i16 = l & 15, g = l >> 4;
    const int quad = wv & 3, kp = wv >> 2;
    const int qm = 64 * (quad & 1), qn = 64 * (quad >> 1);
    const long long U = wb.units, G = gridDim.x;
    int u = (int)(blockIdx.x * U / G);
    const int u_end = (int)((blockIdx.x + 1) * U / G);
    int run = 0;
    WTR(0);
    while (u < u_end) {
        const int pi = wg_find(wb, u);
        const WgProb& P = wb.p[pi];
        const int local = u - P.unit_begin;
        const int tile = local / P.slabs, s0 = local - tile * P.slabs;
        const int n_slabs = min(u_end - u, P.slabs - s0);
        const int m0 = (tile / P.tiles_n) * kWgT, n0 = (tile % P.tiles_n) * kWgT;
        f32x4 acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        wg_load_slab(P.A, P.lda, s0 * kWgBK, m0, P.M, wg_smem);
        wg_load_slab(P.B, P.ldb, s0 * kWgBK, n0, P.N, wg_smem + kWgBK * kWgT);
        __syncthreads();  // waits vmcnt(0): the first slab has landed
        WTR(1 + 4 * run);
        for (int s = 0; s < n_slabs; ++s) {
            const int cur = s & 1;
            if (s + 1 < n_slabs) {
                float* nxt = wg_smem + (cur ^ 1) * kStage;
                wg_load_slab(P.A, P.lda, (s0 + s + 1) * kWgBK, m0, P.M, nxt);
                wg_load_slab(P.B, P.ldb, (s0 + s + 1) * kWgBK, n0, P.N, nxt + kWgBK * kWgT);
            }
            const float* as = wg_smem + cur * kStage + qm + 4 * i16;
            const float* bs = wg_smem + cur * kStage + kWgBK * kWgT + qn + 4 * i16;
#pragma unroll
            for (int h = 0; h < kWgBK / 8; ++h) {
                const int k = 4 * (2 * h + kp) + g;
                const f32x4 fa = *reinterpret_cast<const f32x4*>(as + k * kWgT);
                const f32x4 fb = *reinterpret_cast<const f32x4*>(bs + k * kWgT);
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a], fb[b], acc[a][b], 0, 0, 0);
            }
            __syncthreads();  // next slab landed (vmcnt(0)); everyone is done reading this one
        }
        WTR(2 + 4 * run);
        // k-parity 1 -> LDS, parity 0 adds and stores. Lane (i16, g) of tile (a, b) holds
        // dW[m0 + qm + 16 g + 4 r + a][n0 + qn + 4 i16 + b], r = 0..3.
        float* red = wg_smem + quad * 64 * 64;
        if (kp == 1) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<f32x4*>(red + (16 * g + 4 * r + a) * 64 + 4 * i16) =
                        f32x4{acc[a][0][r], acc[a][1][r], acc[a][2][r], acc[a][3][r]};
        }
        __syncthreads();
        if (kp == 0) {
            float* out = wb.part + (size_t)(blockIdx.x * kWgRuns + run) * kWgSlot;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ml = qm + 16 * g + 4 * r + a;
                    const f32x4 o = *reinterpret_cast<const f32x4*>(red + (16 * g + 4 * r + a) * 64 + 4 * i16);
                    *reinterpret_cast<f32x4*>(out + ml * kWgT + qn + 4 * i16) =
                        o + f32x4{acc[a][0][r], acc[a][1][r], acc[a][2][r], acc[a][3][r]};
                }
        }
        __syncthreads();  // LDS is reloaded by the next run
        WTR(3 + 4 * run);
        u += n_slabs;
        ++run;
    }
}

// Host side: problems, slab units, the static run schedule and its reduction map.
struct WgTileRuns {
    int prob, m0, n0, rows;  // output tile (rows = valid rows, <= 128)
    int first_slot;          // slot of the first run
    int rest_slot;           // slot of the second run; later runs every kWgRuns slots
    int runs;
};
struct WgPlan {
    WgBatch b{};
    int grid = 0;
    bool ok = true;
    void add(const float* A, int lda, const float* B, int ldb, int M, int N, int K) {
        if (b.n >= kWgMaxProbs || N % kWgT || K % kWgBK || (M % kWgT && M != 64) || lda % 4 || ldb % 4) {
            ok = false;
            return;
        }
        WgProb& P = b.p[b.n++];
        P.A = A; P.B = B; P.M = M; P.N = N; P.K = K; P.lda = lda; P.ldb = ldb;
        P.tiles_n = N / kWgT;
        P.tiles = ((M + kWgT - 1) / kWgT) * P.tiles_n;
        P.slabs = K / kWgBK;
        P.unit_begin = b.units;
        b.units += P.tiles * P.slabs;
    }
    // Workgroup w's unit range, as the kernel computes it.
    int w_begin(int w) const { return (int)((long long)w * b.units / grid); }
    // Enumerate every tile's runs (calls f(WgTileRuns)); false if a workgroup would need more than
    // kWgRuns slots.
    template <class F>
    bool tiles(F&& f) {
        grid = std::min(kWgGrid, b.units);
        for (int w = 0; w < grid; ++w) {  // runs per workgroup = tiles its range meets
            int u = w_begin(w), e = w_begin(w + 1), runs = 0;
            while (u < e) {
                int pi = 0;
                while (pi + 1 < b.n && u >= b.p[pi + 1].unit_begin) ++pi;
                const WgProb& P = b.p[pi];
                const int local = u - P.unit_begin, s0 = local % P.slabs;
                u += std::min(e - u, P.slabs - s0);
                ++runs;
            }
            if (runs > kWgRuns) return false;
        }
        for (int pi = 0; pi < b.n; ++pi) {
            const WgProb& P = b.p[pi];
            for (int t = 0; t < P.tiles; ++t) {
                const int t0 = P.unit_begin + t * P.slabs, t1 = t0 + P.slabs;  // the tile's units
                // workgroups meeting [t0, t1): w0 = the one holding t0, w1 = the one holding t1 - 1
                int w0 = (int)(((long long)t0 * grid) / b.units);
                while (w_begin(w0 + 1) <= t0) ++w0;
                while (w_begin(w0) > t0) --w0;
                int w1 = (int)(((long long)(t1 - 1) * grid) / b.units);
                while (w_begin(w1 + 1) <= t1 - 1) ++w1;
                while (w_begin(w1) > t1 - 1) --w1;
                // j0 = index of this tile among w0's runs = tiles started in w0's range before t0
                int j0 = 0;
                for (int u = w_begin(w0); u < t0;) {
                    int qi = 0;
                    while (qi + 1 < b.n && u >= b.p[qi + 1].unit_begin) ++qi;
                    const WgProb& Q = b.p[qi];
                    const int s0 = (u - Q.unit_begin) % Q.slabs;
                    u += Q.slabs - s0;
                    ++j0;
                }
                WgTileRuns tr;
                tr.prob = pi;
                tr.m0 = (t / P.tiles_n) * kWgT;
                tr.n0 = (t % P.tiles_n) * kWgT;
                tr.rows = std::min(kWgT, P.M - tr.m0);
                tr.first_slot = w0 * kWgRuns + j0;
                tr.rest_slot = (w0 + 1) * kWgRuns;
                tr.runs = w1 - w0 + 1;
                f(tr);
            }
        }
        return true;
    }
};

}  // namespace tr
}  // namespace uavhip
