// wgrad.hpp -- weight gradients of the PPO training step (train.hip): for a list of problems,
// dW[m][n] = sum_k dY[k][m] X[k][n] over the minibatch rows k, fp32-accurate split products on the
// f16 MFMA (v_mfma_f32_16x16x32_f16, see k_wgrad). Bias gradients (sums of dY over k) come from
// k_policy_backward's per-workgroup partials, not from here.
//
// Work split (stream-K over 32-deep k-slabs): the problems' 128 x 128 output tiles x K / 32 slabs
// form one list (problem-major, then tile, then k); workgroup w takes the contiguous range
// [w U / G, (w + 1) U / G) and accumulates each tile's slabs in registers, writing one partial
// tile per (workgroup, tile) run into slot kWgRuns w + j (j = the run's index within the
// workgroup). The host enumerates the same runs (WgPlan) to build the reduction segments: a tile's
// runs are slot kWgRuns w0 + j0, then kWgRuns w + 0 for w = w0 + 1 .. w1.
//
// Chunked mode (WgBatch::chunk > 0, large minibatches): every tile's k range is cut into chunks of
// WgProb::chunk slabs (shorter for the three-plane problems: WgPlan::chunked), and workgroup v takes
// exactly one (problem, chunk, tile) triple, numbered
// problem-major, then chunk, then tile -- so the tiles that share an operand slab (the m-tiles of
// in_proj / FFN1 share X, FFN2's two n-tiles share dY) are consecutive. v is the XCD-aware virtual
// index of blockIdx.x (workgroups are dealt to the 8 XCDs round-robin: v = (b % 8) G / 8 + b / 8), so
// consecutive v run at the same time on the same XCD and the second and third readers of a slab find
// it in that XCD's L2 instead of HBM. One run per workgroup: slot kWgRuns v; a tile's runs are
// slot kWgRuns (wg_begin + t), then every kWgRuns tiles slots.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "policy_layout.hpp"  // the operand range bounds (range_exp / range_bound / range_entry)

#ifndef UAVHIP_EXP
#define UAVHIP_EXP 0  // timing experiments (A/B builds, results wrong): 51 no loads after the first two
#endif                // slabs, 52 one MFMA of six, 53 no split arithmetic

namespace uavhip {
namespace tr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWgT = 128;                 // output tile edge
constexpr int kWgBK = 32;                 // k rows per slab (one 32-k MFMA block)
constexpr int kWgThreads = 512;
constexpr int kWgRuns = 3;                // partial slots per workgroup
constexpr int kWgSlot = kWgT * kWgT;      // floats per partial slot
constexpr int kWgMaxProbs = 24;
constexpr int kWgGrid = 256;              // one workgroup per CU

// X operands the training forward does not store: a LayerNorm output is formed from
// its stored x-hat as x-hat * gamma + beta (per column), a layer-0 input from the stored embedding as
// e + pos[s] (row k = b * 5 + s, or one fixed position s for the token-4 rows)
enum { kWgX = 0, kWgXAffine = 1, kWgXPosRow = 2, kWgXPosFixed = 3 };
struct WgProb {
    const float* A;  // dY: row k at A + k * lda, columns m
    const float* B;  // X:  row k at B + k * ldb, columns n (before the transform xmode)
    const float* xg;  // kWgXAffine: gamma [N] (other modes: read, unused; WgPlan::add points it at N valid floats)
    const float* xb;  // kWgXAffine: beta [N]; kWgXPosRow: pos [5][N]; kWgXPosFixed: pos row [N]; kWgX: X row 0
    int xmode;
    int M, N, K, lda, ldb;
    int tiles_n, tiles, slabs;  // per problem: column tiles, tiles, slabs per tile
    int unit_begin;             // first slab unit of this problem
    int tile_begin;             // first output tile of this problem (direct mode: its workgroup)
    int wg_begin;               // chunked mode: first workgroup (virtual index) of this problem
    int p3_tiles;               // bit t: tile t runs three-plane products (else two-plane)
    int chunk;                  // chunked mode: slabs per chunk of this problem's tiles
    int dst;                    // direct mode: float offset of dW [M][N] in `grads`
    // the X operand's range (policy_layout.hpp): X is staged as X 2^-s and the run's dW multiplied by
    // 2^s (exact), s from a bound on |X| -- rk: kWgRStatic (rarg = the forward's static operand: its
    // (2^-s, 2^s) pair), kWgRE / kWgRA0 (layer 0's input / attention output of trunk rarg: from the
    // run's rows' block maxima xmax, rpb rows each, and the forward's layer-0 constants)
    int rk, rarg, rpb;
    const float* xmax;
};
enum { kWgRNone = 0, kWgRStatic = 1, kWgRE = 3, kWgRA0 = 4 };
// Direct mode (small minibatches: every tile a few slabs): one workgroup per output tile runs all
// of its slabs and writes dW itself -- times `unscale` (BwdIO::gscale undone, exact) -- into the
// flat gradient, with the block's sum of squares in sq[blockIdx.x]; no partial tiles, no reduction.
struct WgBatch {
    WgProb p[kWgMaxProbs];
    int n;
    int units;
    float* part;  // [grid * kWgRuns][kWgSlot]
    int direct, tiles;
    int chunk, wgs;  // chunked mode: slabs per chunk (0: stream-K), workgroups holding work
    float* grads;
    float* sq;
    float unscale;
    const float* gsc;  // the critic's extra 2^k (heads_bwd): problems with dst >= crit_off
    int crit_off;
    const float* rt;   // the training forward's derived scales (TrainIO::rtab_out, policy_layout.hpp kRtOp ..)
};
constexpr int kWgDirectMaxSlabs = 12;  // direct mode only when no tile has more slabs (K <= 384 rows)


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

__device__ __forceinline__ int wg_find_tile(const WgBatch& b, int t) {
    int lo = 0, hi = b.n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (t >= b.p[mid].tile_begin) lo = mid;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int wg_find_wg(const WgBatch& b, int v) {
    int lo = 0, hi = b.n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (v >= b.p[mid].wg_begin) lo = mid;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int wg_find(const WgBatch& b, int u) {
    int lo = 0, hi = b.n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (u >= b.p[mid].unit_begin) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Split products with THREE fp16 planes: every operand element is staged as
// x = x1 + 2^-11 x2 + 2^-22 x3 (x1 = f16(x), x2 = f16((x - x1) 2^11), x3 = f16((x - x1 - 2^-11 x2) 2^22),
// exact to 2^-33) and dW = hi + 2^-11 mid + 2^-22 lo with hi += A1 B1, mid += A1 B2 + A2 B1,
// lo += A1 B3 + A3 B1 + A2 B2 on v_mfma_f32_16x16x32_f16 (6 x 16 cycles per 16 x 16 x 32 block
// against 8 x 32 for the f32 MFMA). The weight gradients sum thousands of rows whose terms
// largely cancel (the in_proj key rows: softmax removes the key bias), so the two-plane form's
// 2^-22 per product is not enough here; this one is more accurate than the f32 MFMA's fp32 sums.
//
// Operands. dY and X are the workspace's [row][feature] activations: k-major. Each thread loads its
// share of a 32 x 128 slab from global as float4 (registers, one slab ahead), splits it and writes
// the planes into the LDS stage as [k][128] fp16 images with 256-B rows whose 16-B chunks are
// XOR-swizzled (cdna_hip_programming.md T10 image (b)); the MFMA fragments -- 8 consecutive k of one
// m (A) or n (B) column per lane -- come out of ds_read_b64_tr_b16 (two per plane: rows 8g..8g+3
// and 8g+4..8g+7 of the slab), conflict-free with a 32-lane half's two row blocks 8 rows apart.
//
// Workgroup: 512 threads = 8 waves, one 128 x 128 output tile; wave w owns rows 64 (w & 1) .. + 63
// (4 m-tiles) x columns 32 (w >> 1) .. + 31 (2 n-tiles) over the whole k range (hi, mid, lo: 96
// accumulator VGPRs). LDS: 2 stages x 6 planes x 8 KiB = 96 KiB, one workgroup per CU.
typedef _Float16 wg_f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 wg_f16x8 __attribute__((ext_vector_type(8)));
typedef short wg_i16x4 __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) wg_i16x4 wg_lds_i16x4;
constexpr int kWgRowB = 2 * kWgT;              // bytes per plane row: 128 fp16
constexpr int kWgPlaneB = kWgBK * kWgRowB;     // 8 KiB: one plane of a 32 x 128 slab
constexpr int kWgStageB = 6 * kWgPlaneB;       // A x1 x2 x3 | B x1 x2 x3
static_assert(kWgBK == 32, "one 32-k MFMA block per slab");

__device__ __forceinline__ int wg_swz(int row, int ch) {
    return kWgRowB * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// this thread's share of a slab: rows (t >> 5) + 16 i, columns 4 (t & 31) .. + 3 of each operand.
// Columns >= M (a 64-wide problem) read column m0 instead; their products land in output rows
// that are never stored.
struct WgSlab {
    f32x4 a[2], b[2];
    f32x4 x[2];  // the X transform's additive term of each row: beta, or the row's pos
};
// Every load is unconditional (the host points xg / xb at valid memory for every mode), so the
// wait counts stay exact across the software pipeline; the mode only selects arithmetic.
__device__ __forceinline__ void wg_gload(WgSlab& r, const WgProb& P, int k0, int m0, int n0) {
    const int t = threadIdx.x, c = 4 * (t & 31);
    const int ca = m0 + c < P.M ? m0 + c : m0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = k0 + (t >> 5) + 16 * i;
        r.a[i] = *reinterpret_cast<const f32x4*>(P.A + (size_t)row * P.lda + ca);
        r.b[i] = *reinterpret_cast<const f32x4*>(P.B + (size_t)row * P.ldb + n0 + c);
        r.x[i] = *reinterpret_cast<const f32x4*>(P.xb + (P.xmode == kWgXPosRow ? (row % 5) * P.N : 0) + n0 + c);
    }
}
// gamma of this thread's 4 columns n0 + 4 (t & 31) .. + 3 (1 unless kWgXAffine), once per tile run
__device__ __forceinline__ f32x4 wg_xgamma(const WgProb& P, int n0) {
    const f32x4 g = *reinterpret_cast<const f32x4*>(P.xg + n0 + 4 * (threadIdx.x & 31));
    return P.xmode == kWgXAffine ? g : f32x4{1.f, 1.f, 1.f, 1.f};
}
template <bool P3>  // P3: the third plane (two-plane tiles neither write nor read it)
__device__ __forceinline__ void wg_split_store(const f32x4 v, char* plane, int off) {
    wg_f16x4 x1, x2, x3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        x1[j] = (_Float16)v[j];
        if constexpr (UAVHIP_EXP == 53) {
            x2[j] = x3[j] = x1[j];
            continue;
        }
        const float r1 = v[j] - (float)x1[j];                 // exact
        x2[j] = f16_lo(v[j], x1[j]);                          // = f16(r1 2^11)
        if constexpr (P3) x3[j] = (_Float16)((r1 - (float)x2[j] * (1.0f / 2048.0f)) * 4194304.f);  // exact
    }
    *reinterpret_cast<wg_f16x4*>(plane + off) = x1;
    *reinterpret_cast<wg_f16x4*>(plane + kWgPlaneB + off) = x2;
    if constexpr (P3) *reinterpret_cast<wg_f16x4*>(plane + 2 * kWgPlaneB + off) = x3;
}
// the X operand as the forward formed it: x-hat * gamma + beta (its LayerNorm epilogue's expression),
// e + pos[s] (gamma 1: exact), or x itself (applied at staging: the slab's loads have landed by then)
template <bool P3>
__device__ __forceinline__ void wg_stage_store(const WgSlab& r, char* stage, int xmode, const f32x4 xg, float xsc) {
    const int t = threadIdx.x, c4 = t & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int off = wg_swz((t >> 5) + 16 * i, c4 >> 1) + 8 * (c4 & 1);
        wg_split_store<P3>(r.a[i], stage, off);
        // X 2^-s (xsc, exact): every element inside fp16's range (wg_xrange). x-hat * gamma + beta as
        // one fma per element: the forward's (contracted) LayerNorm epilogue rounds it once too, so the
        // re-formed operand is its stored output bit for bit (this file itself stays uncontracted:
        // contracting all of it measured 2.5 us slower in k_wgrad, profiles/r06v_train_ab_contract.txt)
        f32x4 xv = r.b[i];
        if (xmode != kWgX) {
#pragma unroll
            for (int e = 0; e < 4; ++e) xv[e] = __builtin_fmaf(r.b[i][e], xg[e], r.x[i][e]);
        }
        wg_split_store<P3>(xv * xsc, stage + 3 * kWgPlaneB, off);
    }
}
// 16 columns (c16 .. c16 + 15) x 8 consecutive k (8 g ..) of a plane: lane (i16, g) gets column
// c16 + i16 -- the f16 MFMA operand -- from two transposed reads of 4 rows each
__device__ __forceinline__ wg_f16x8 wg_frag(const char* plane, int c16) {
    const int l = threadIdx.x & 63, g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    const int r0 = 8 * g + q, ch = (c16 >> 3) + (p >> 1), sub = 8 * (p & 1);
    const wg_i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((wg_lds_i16x4*)(plane + wg_swz(r0, ch) + sub));
    const wg_i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((wg_lds_i16x4*)(plane + wg_swz(r0 + 4, ch) + sub));
    const wg_f16x4 a = __builtin_bit_cast(wg_f16x4, lo), b = __builtin_bit_cast(wg_f16x4, hi);
    return wg_f16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// The exponent s of the X operand of rows [k0, k1) of problem P (WgProb::rk). Block-uniform; the
// dynamic kinds reduce the rows' block maxima over the workgroup (one barrier).
__device__ __forceinline__ float wg_dpp_max(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, true)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, true)));
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// (xsc, xinv) = (2^-s, 2^s) of the X operand of rows [k0, k1) of problem P (WgProb::rk), every
// operand a plain (vector) load issued behind the run's first slab loads: their in-order wait adds no
// round trip. Uniform over the workgroup; the dynamic kinds reduce many blocks with one barrier.
__device__ __forceinline__ void wg_xrange(const WgBatch& wb, const WgProb& P, int k0, int k1, float* wred, float& xsc,
                                          float& xinv) {
#pragma clang fp contract(off)
    xsc = xinv = 1.f;
    const float* rt = wb.rt;
    if (P.rk == kWgRNone || !rt) return;
    if (P.rk == kWgRStatic) {
        xsc = rt[pol::kRtOp + 2 * P.rarg];
        xinv = rt[pol::kRtOp + 2 * P.rarg + 1];
        return;
    }
    float m = 0.f;
    const int b0 = k0 / P.rpb, b1 = (k1 - 1) / P.rpb;  // the run's 16-sample blocks
    if (b1 - b0 < 32) {  // few: every thread takes them all (no barrier)
        for (int b = b0; b <= b1; ++b) m = fmaxf(m, P.xmax[b]);
    } else {
        for (int b = b0 + (int)threadIdx.x; b <= b1; b += kWgThreads) m = fmaxf(m, P.xmax[b]);
        m = wg_dpp_max(m);
        if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = m;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kWgThreads / 64; ++w) m = fmaxf(m, wred[w]);
    }
    const int t = P.rarg;
    float B = rt[pol::kRtE + 2 * t] * m + rt[pol::kRtE + 2 * t + 1];
    if (P.rk == kWgRA0) B = rt[pol::kRtA0 + 2 * t] * B + rt[pol::kRtA0 + 2 * t + 1];
    const int xs = pol::range_exp(B);
    xsc = ldexpf(1.0f, -xs);
    xinv = ldexpf(1.0f, xs);
}

// One tile run's k-loop: slabs s0 .. s0 + n_slabs - 1 of problem P into hi / mid / lo. P3: the
// three-plane products (6 MFMAs per block); otherwise two planes (x = x1 + 2^-11 x2, dropped terms
// 2^-22 of a product: hi += a1b1, mid += a1b2 + a2b1, lo += a2b2, 4 MFMAs), for the tiles whose sums
// do not cancel (WgProb::p3_tiles).
template <bool P3>
__device__ __forceinline__ void wg_kloop(char* wg_smem, const WgProb& P, int s0, int n_slabs, int m0, int n0, int mt0,
                                         int nt0, f32x4 (&hi)[4][2], f32x4 (&mid)[4][2], f32x4 (&lo)[4][2],
                                         [[maybe_unused]] int run, const WgBatch& wb, float* wred, float& xinv) {
        const int xmode = P.xmode;
        const f32x4 xg = wg_xgamma(P, n0);
        WgSlab nx;
        wg_gload(nx, P, s0 * kWgBK, m0, n0);
        // the X range behind the first slab's loads (its own loads then cost no extra round trip)
        float xsc;
        wg_xrange(wb, P, s0 * kWgBK, (s0 + n_slabs) * kWgBK, wred, xsc, xinv);
        wg_stage_store<P3>(nx, wg_smem, xmode, xg, xsc);
        if (n_slabs > 1) wg_gload(nx, P, (s0 + 1) * kWgBK, m0, n0);
        __syncthreads();
        WTR(1 + 4 * run);
        for (int s = 0; s < n_slabs; ++s) {
            const char* st = wg_smem + (s & 1) * kWgStageB;
            wg_f16x8 a1[4], a2[4], a3[4], b1[2], b2[2], b3[2];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                a1[a] = wg_frag(st, 16 * (mt0 + a));
                a2[a] = wg_frag(st + kWgPlaneB, 16 * (mt0 + a));
                if constexpr (P3) a3[a] = wg_frag(st + 2 * kWgPlaneB, 16 * (mt0 + a));
            }
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                b1[b] = wg_frag(st + 3 * kWgPlaneB, 16 * (nt0 + b));
                b2[b] = wg_frag(st + 4 * kWgPlaneB, 16 * (nt0 + b));
                if constexpr (P3) b3[b] = wg_frag(st + 5 * kWgPlaneB, 16 * (nt0 + b));
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    hi[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[a], b1[b], hi[a][b], 0, 0, 0);
                    if constexpr (UAVHIP_EXP == 52 && P3) {  // keep the operands live
                        mid[a][b] += __builtin_bit_cast(f32x4, a2[a]) + __builtin_bit_cast(f32x4, b2[b]);
                        lo[a][b] += __builtin_bit_cast(f32x4, a3[a]) + __builtin_bit_cast(f32x4, b3[b]);
                        continue;
                    }
                    mid[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[a], b2[b], mid[a][b], 0, 0, 0);
                    mid[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[a], b1[b], mid[a][b], 0, 0, 0);
                    if constexpr (P3) {
                        lo[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[a], b3[b], lo[a][b], 0, 0, 0);
                        lo[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a3[a], b1[b], lo[a][b], 0, 0, 0);
                    }
                    lo[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[a], b2[b], lo[a][b], 0, 0, 0);
                }
            if (s + 1 < n_slabs) {  // slab s + 1 (landed in registers meanwhile) -> the other stage
                wg_stage_store<P3>(nx, wg_smem + ((s + 1) & 1) * kWgStageB, xmode, xg, xsc);
                if (s + 2 < n_slabs && UAVHIP_EXP != 51) wg_gload(nx, P, (s0 + s + 2) * kWgBK, m0, n0);
            }
            __syncthreads();  // the next stage is written; everyone is done reading this one
        }
}

__global__ __launch_bounds__(kWgThreads) void k_wgrad(const WgBatch wb) {
    __shared__ __attribute__((aligned(16))) char wg_smem[2 * kWgStageB];
    __shared__ float wred[kWgThreads / 64];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, i16 = l & 15, g = l >> 4;
    const int mt0 = 4 * (wv & 1), nt0 = 2 * (wv >> 1);  // this wave's first m-tile / n-tile
    const long long U = wb.units, G = gridDim.x;
    int u = (int)(blockIdx.x * U / G);
    int u_end = (int)((blockIdx.x + 1) * U / G);
    int slot_wg = blockIdx.x;
    if (wb.chunk) {  // one (chunk, tile) per workgroup, siblings on one XCD (G % 8 == 0: host)
        slot_wg = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
        if (slot_wg >= wb.wgs) return;
        const WgProb& Q = wb.p[wg_find_wg(wb, slot_wg)];
        const int local = slot_wg - Q.wg_begin, c = local / Q.tiles, t = local - c * Q.tiles;
        const int s0 = c * Q.chunk;
        u = Q.unit_begin + t * Q.slabs + s0;
        u_end = u + min(Q.chunk, Q.slabs - s0);
    } else if (wb.direct) {  // workgroup = output tile: all of its slabs
        const WgProb& Q = wb.p[wg_find_tile(wb, blockIdx.x)];
        u = Q.unit_begin + (blockIdx.x - Q.tile_begin) * Q.slabs;
        u_end = u + Q.slabs;
    }
    int run = 0;
    WTR(0);
    while (u < u_end) {
        const int pi = wg_find(wb, u);
        const WgProb& P = wb.p[pi];
        const int local = u - P.unit_begin;
        const int tile = local / P.slabs, s0 = local - tile * P.slabs;
        const int n_slabs = min(u_end - u, P.slabs - s0);
        const int m0 = (tile / P.tiles_n) * kWgT, n0 = (tile % P.tiles_n) * kWgT;
        f32x4 hi[4][2], mid[4][2], lo[4][2];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) hi[a][b] = mid[a][b] = lo[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        float xinv;  // 2^s of the run's X operand (wg_xrange)
        if ((P.p3_tiles >> tile) & 1) wg_kloop<true>(wg_smem, P, s0, n_slabs, m0, n0, mt0, nt0, hi, mid, lo, run, wb, wred, xinv);
        else wg_kloop<false>(wg_smem, P, s0, n_slabs, m0, n0, mt0, nt0, hi, mid, lo, run, wb, wred, xinv);
        WTR(2 + 4 * run);
        // lane (i16, g) of tile (a, b) holds dW[m0 + 16 (mt0 + a) + 4 g + r][n0 + 16 (nt0 + b) + i16]
        if (wb.direct) {  // the whole tile: dW itself, unscaled, rows < M (a 64-row problem), and g^2
            float sq = 0.f;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const f32x4 v = (hi[a][b] + (mid[a][b] + lo[a][b] * (1.0f / 2048.0f)) * (1.0f / 2048.0f)) *
                                    (P.dst >= wb.crit_off ? wb.unscale * wb.gsc[0] : wb.unscale) * xinv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = m0 + 16 * (mt0 + a) + 4 * g + r;
                        if (row < P.M) {
                            wb.grads[P.dst + (size_t)row * P.N + n0 + 16 * (nt0 + b) + i16] = v[r];
                            sq += v[r] * v[r];
                        }
                    }
                }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) sq += __shfl_xor(sq, o);
            float* red = reinterpret_cast<float*>(wg_smem);  // the stages are dead after the last barrier
            if (l == 0) red[wv] = sq;
            __syncthreads();
            if (threadIdx.x == 0) {
                float t = 0.f;
                for (int w = 0; w < kWgThreads / 64; ++w) t += red[w];
                wb.sq[blockIdx.x] = t;
            }
            return;
        }
        float* out = wb.part + (size_t)(slot_wg * kWgRuns + run) * kWgSlot;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const f32x4 v = (hi[a][b] + (mid[a][b] + lo[a][b] * (1.0f / 2048.0f)) * (1.0f / 2048.0f)) * xinv;
#pragma unroll
                for (int r = 0; r < 4; ++r) out[(16 * (mt0 + a) + 4 * g + r) * kWgT + 16 * (nt0 + b) + i16] = v[r];
            }
        WTR(3 + 4 * run);
        u += n_slabs;
        ++run;
    }
}

// Host side: problems, slab units, the static run schedule and its reduction map.
struct WgTileRuns {
    int prob, m0, n0, rows;  // output tile (rows = valid rows, <= 128)
    int first_slot;          // slot of the first run
    int rest_slot;           // slot of the second run; later runs every run_stride slots
    int runs, run_stride;
};
struct WgPlan {
    WgBatch b{};
    int grid = 0;
    bool ok = true;
    void add(const float* A, int lda, const float* B, int ldb, int M, int N, int K, int xmode = kWgX,
             const float* xg = nullptr, const float* xb = nullptr) {
        if (b.n >= kWgMaxProbs || N % kWgT || K % kWgBK || (M % kWgT && M != 64) || lda % 4 || ldb % 4 ||
            (xmode == kWgXAffine && (!xg || !xb)) || (xmode >= kWgXPosRow && !xb)) {
            ok = false;
            return;
        }
        WgProb& P = b.p[b.n++];
        P.A = A; P.B = B; P.M = M; P.N = N; P.K = K; P.lda = lda; P.ldb = ldb;
        // xg / xb are read whatever the mode: unused ones point at N valid floats (X's row 0)
        P.xmode = xmode; P.xb = xb ? xb : B; P.xg = xg ? xg : P.xb;
        P.tiles_n = N / kWgT;
        P.tiles = ((M + kWgT - 1) / kWgT) * P.tiles_n;
        P.slabs = K / kWgBK;
        P.unit_begin = b.units;
        P.tile_begin = b.tiles;
        P.wg_begin = 0;
        P.p3_tiles = ~0;
        P.chunk = 0;
        P.dst = 0;
        P.rk = kWgRNone;
        P.rarg = 0;
        P.rpb = 1;
        P.xmax = nullptr;
        b.units += P.tiles * P.slabs;
        b.tiles += P.tiles;
    }
    int max_slabs() const {
        int m = 0;
        for (int i = 0; i < b.n; ++i) m = std::max(m, b.p[i].slabs);
        return m;
    }
    // Chunked mode: the smallest chunk ch (slabs) whose (problem, chunk, tile) triples fit kWgGrid
    // workgroups, where a problem with three-plane tiles gets chunks of ch * p3_ratio slabs (a
    // three-plane slab costs more: 6 MFMAs and three planes against 4 and two, so its workgroups
    // would otherwise finish last and set the launch's time); grid = the count rounded up to the 8
    // XCDs. False if none fits.
    bool chunked(float p3_ratio = 0.75f) {
        const int ms = max_slabs();
        for (int ch = 1; ch <= ms; ++ch) {
            const int ch3 = std::max(1, (int)(ch * p3_ratio + 0.5f));
            int wgs = 0;
            for (int i = 0; i < b.n; ++i) {
                WgProb& P = b.p[i];
                P.wg_begin = wgs;
                P.chunk = P.p3_tiles & ((1 << P.tiles) - 1) ? ch3 : ch;
                wgs += P.tiles * ((P.slabs + P.chunk - 1) / P.chunk);
            }
            if (wgs <= kWgGrid) {
                b.chunk = ch;
                b.wgs = wgs;
                grid = (wgs + 7) / 8 * 8;
                return true;
            }
        }
        return false;
    }
    // Workgroup w's unit range, as the kernel computes it.
    int w_begin(int w) const { return (int)((long long)w * b.units / grid); }
    // Enumerate every tile's runs (calls f(WgTileRuns)); false if a workgroup would need more than
    // kWgRuns slots.
    template <class F>
    bool tiles(F&& f) {
        if (b.chunk) {
            for (int pi = 0; pi < b.n; ++pi) {
                const WgProb& P = b.p[pi];
                for (int t = 0; t < P.tiles; ++t) {
                    WgTileRuns tr;
                    tr.prob = pi;
                    tr.m0 = (t / P.tiles_n) * kWgT;
                    tr.n0 = (t % P.tiles_n) * kWgT;
                    tr.rows = std::min(kWgT, P.M - tr.m0);
                    tr.first_slot = (P.wg_begin + t) * kWgRuns;
                    tr.rest_slot = (P.wg_begin + t + P.tiles) * kWgRuns;
                    tr.runs = (P.slabs + P.chunk - 1) / P.chunk;
                    tr.run_stride = P.tiles * kWgRuns;
                    f(tr);
                }
            }
            return true;
        }
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
                tr.run_stride = kWgRuns;
                f(tr);
            }
        }
        return true;
    }
};

}  // namespace tr
}  // namespace uavhip
