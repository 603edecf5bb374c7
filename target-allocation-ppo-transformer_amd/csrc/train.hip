// train.hip -- K5: one clipped-PPO minibatch step (agents/ppo.py:96-169) of TransformerActorCritic
// (networks/transformer_net.py) on gfx950, fp32-accurate throughout: every encoder GEMM (forward,
// input gradients, weight gradients) as split products on the f16 MFMA.
//
// Layout: a minibatch of Bm samples is R = 5 Bm token rows, row = b * 5 + s, features contiguous.
// One step is 5-7 launches on one stream (graph-capturable: no host sync, no allocation); minibatches
// of <= 256 samples run the position split instead (K7, policy.hip: 3 forward + 3 backward launches):
//    forward   k_policy_forward<TR> (policy.hip, the rollout's fused kernel writing activations),
//              with the heads and per-workgroup loss partials, then k_loss_sums (the four sums).
//              Minibatches of <= 2048 samples (2 Bm/16 workgroups fit one per CU) run trunk-split:
//              the actor's and the critic's workgroups side by side (the trunks are independent
//              until the loss), then k_loss_partials; the backward splits the same way
//    backward  k_policy_backward (K6, policy.hip: loss and head gradients, dX of the encoder
//              layers and embeddings, one workgroup per 16 samples), then every weight
//              gradient dW[out][in] = sum_row dY[row][out] X[row][in] as one stream-K launch of
//              three-plane split products (wgrad.hpp: per-workgroup partial tiles), and one k_reduce_grads over all
//              partials (weight tiles, K6's bias / LayerNorm / embedding / head partials)
//    update    k_adam (clip_grad_norm_ + Adam on the g^2 block partials of k_reduce_grads, or of
//              k_grad_norm after a data-parallel all-reduce)
// The last encoder layer of each trunk is pruned to the token the heads read (s = 4): K and V for
// all rows, everything else for Bm rows (compact [Bm][...] tensors), so its gradients are exactly
// the dense model's.
#include <cmath>
#include <cstdlib>

#include "common.hpp"
#include "policy_layout.hpp"
#include "wgrad.hpp"
#include "policy_train.hpp"

namespace uavhip {
namespace tr {
using namespace pol;

// ------------------------------------------------------------------ cross-lane sums (no LDS)
__device__ __forceinline__ float add_xor1(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ float add_xor2(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
}
__device__ __forceinline__ float add_ror4(float v) {  // row_ror:4 inside each row of 16
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, true));
}
__device__ __forceinline__ float add_ror8(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, true));
}
__device__ __forceinline__ float add_xor16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add_xor32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// sum over the 4 lanes of a quad / over the whole wave (same value in every lane)
__device__ __forceinline__ float quad_sum(float v) { return add_xor2(add_xor1(v)); }
__device__ __forceinline__ float wave_sum(float v) {
    return add_xor32(add_xor16(add_ror8(add_ror4(add_xor2(add_xor1(v))))));
}
template <int ctrl>
__device__ __forceinline__ float dpp_max(float v) {
    return fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, true)));
}
__device__ __forceinline__ float wave_max(float v) {  // the same value in every lane
    v = dpp_max<0x128>(dpp_max<0x124>(dpp_max<0x4E>(dpp_max<0xB1>(v))));
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// ================================================================== heads + loss
// 16 samples per 1024-thread block (one wave per sample). Head weights staged in LDS with a
// 129-float row stride (lane j reads row j: conflict-free).
constexpr int kHeadSamples = 16;
using pol::kHeadPart;

// Sum the per-workgroup loss partials of the training forward into loss_sums[4] (one wave, fixed order).
__global__ __launch_bounds__(64) void k_loss_sums(const float* __restrict__ part, int nblk, float* __restrict__ out) {
    const int l = lane_id();
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = l; i < nblk; i += 64)
        for (int c = 0; c < 4; ++c) s[c] += part[i * 4 + c];
    for (int c = 0; c < 4; ++c) {
        const float w = wave_sum(s[c]);
        if (l == 0) out[c] = w;
    }
}

// ================================================================== backward
// dX of the encoder layers + embeddings: k_policy_backward (policy.hip, K6), one fused kernel.
using pol::kEmbPart;

// ================================================================== gradient reduction + Adam
// Adam's per-step scalars, computed once by the block that advances the step counter (block 0 of
// k_reduce_grads or k_grad_norm): the bias corrections in double from the double hyper-parameters
// (torch's non-capturable single-tensor Adam), each coefficient rounded to float once.
struct AdamHyper {
    double lr_actor, lr_critic, beta1, beta2;
};
struct AdamScalars {
    float nss_a, nss_c, bc2s, pad;  // -lr / (1 - b1^t) per group, sqrt(1 - b2^t)
};
__device__ __forceinline__ void adam_advance(double* __restrict__ step, const AdamHyper& h, AdamScalars* __restrict__ sc) {
    const double t = step[0] + 1.0;
    step[0] = t;
    const double bc1 = 1.0 - pow(h.beta1, t), bc2 = 1.0 - pow(h.beta2, t);
    *sc = AdamScalars{(float)(-(h.lr_actor / bc1)), (float)(-(h.lr_critic / bc1)), (float)sqrt(bc2), 0.f};
}

// grads[dst + i] = sum_p src[p * part_stride + i] for each segment; block partial sums of g^2.
// Few parts (split-K slabs): one thread per element. Many parts (per-workgroup partials of K6 /
// the heads): a block takes 64 consecutive elements, each wave every 4th part, so every load is a
// coalesced 256 B row segment; the 4 wave sums combine in a fixed order (deterministic).
struct Segment {
    const float* src;       // part 0
    const float* src_rest;  // part p >= 1 at src_rest + (p - 1) * part_stride
    int dst, count, parts, part_stride, block_begin, tile_mode;
    int dst_ld;             // 0: dst + i; else a 128-wide weight tile, dst + (i / 128) * dst_ld + i % 128
    int vec4;               // element mode with 16-byte aligned rows: a thread sums 4 consecutive elements
};
constexpr int kMaxSegs = 64;
constexpr int kTileModeParts = 16;  // more parts than this: tile mode
struct SegBatch {
    Segment s[kMaxSegs];
    int n;
};
// unscale = 1 / BwdIO::gscale (a power of two: exact): the backward's partials carry the pre-scaled
// gradient, the flat buffer the loss's. The critic's segments (destinations from crit_off on: the
// critic trunk and head) carry gscale x 2^-k (heads_bwd): x gsc[0] = 2^k as well.
__global__ __launch_bounds__(256) void k_reduce_grads(const SegBatch sb, float* __restrict__ grads,
                                                      float* __restrict__ sq_part, double* __restrict__ step,
                                                      const AdamHyper h, AdamScalars* __restrict__ sc,
                                                      float unscale, const float* __restrict__ gsc, int crit_off,
                                                      float* __restrict__ range_m) {
    __shared__ float red[4];
    __shared__ float wsum[4][64];
    // segment of this block: lane l tests segment l (one round of kernarg loads, not a dependent
    // binary search); the segments are in block order, so the count of those begun is its index + 1
    static_assert(kMaxSegs <= 64, "one segment per lane");
    const int sl = lane_id();
    const bool begun = sl < sb.n && (int)blockIdx.x >= sb.s[sl].block_begin;
    const int si = __popcll(__ballot(begun)) - 1;
    const Segment S_ = sb.s[si];  // by value: one batch of scalar loads, not one per field use
    if (S_.dst >= crit_off) unscale *= gsc[0];
    const size_t ps = S_.part_stride;
    auto part = [&](int p) { return p == 0 ? S_.src : S_.src_rest + (size_t)(p - 1) * ps; };
    auto dsti = [&](int i) { return S_.dst + (S_.dst_ld ? (i >> 7) * S_.dst_ld + (i & 127) : i); };
    float sq = 0.f;
    if (S_.tile_mode) {
        const int wv = threadIdx.x >> 6, l = lane_id();
        const int i = (blockIdx.x - S_.block_begin) * 64 + l;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        if (i < S_.count) {  // uniform part stride in this mode (src_rest = src + part_stride)
            const float* src = S_.src + i;
            int p = wv;
#pragma unroll 4
            for (; p + 12 < S_.parts; p += 16) {
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] += src[(size_t)(p + 4 * u) * ps];
            }
            for (; p < S_.parts; p += 4) acc[0] += src[(size_t)p * ps];
        }
        wsum[wv][l] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        __syncthreads();
        if (wv == 0 && i < S_.count) {
            const float tot = ((wsum[0][l] + wsum[1][l]) + (wsum[2][l] + wsum[3][l])) * unscale;
            grads[dsti(i)] = tot;
            sq = tot * tot;
        }
    } else if (S_.vec4) {
        const int i = 4 * ((blockIdx.x - S_.block_begin) * 256 + threadIdx.x);
        if (i + 4 <= S_.count) {
            f32x4 acc[4] = {};
            int p = 0;
#pragma unroll 2
            for (; p + 4 <= S_.parts; p += 4) {
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] += *reinterpret_cast<const f32x4*>(part(p + u) + i);
            }
            for (; p < S_.parts; ++p) acc[0] += *reinterpret_cast<const f32x4*>(part(p) + i);
            const f32x4 tot = ((acc[0] + acc[1]) + (acc[2] + acc[3])) * unscale;
            *reinterpret_cast<f32x4*>(grads + dsti(i)) = tot;
            sq = (tot[0] * tot[0] + tot[1] * tot[1]) + (tot[2] * tot[2] + tot[3] * tot[3]);
        } else {
            for (int e = i; e < S_.count; ++e) {  // the ragged end of the segment
                float tot = 0.f;
                for (int p = 0; p < S_.parts; ++p) tot += part(p)[e];
                tot *= unscale;
                grads[dsti(e)] = tot;
                sq += tot * tot;
            }
        }
    } else {
        const int i = (blockIdx.x - S_.block_begin) * 256 + threadIdx.x;
        if (i < S_.count) {
            // four independent chains keep four loads in flight per thread
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            int p = 0;
#pragma unroll 4
            for (; p + 4 <= S_.parts; p += 4) {
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] += part(p + u)[i];
            }
            for (; p < S_.parts; ++p) acc[0] += part(p)[i];
            const float tot = ((acc[0] + acc[1]) + (acc[2] + acc[3])) * unscale;
            grads[dsti(i)] = tot;
            sq = tot * tot;
        }
    }
    sq = wave_sum(sq);
    if (lane_id() == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
        sq_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
        if (step && blockIdx.x == 0) adam_advance(step, h, sc);  // single-GPU step: these are the final grads
    }
    // the range table's maxima, ahead of k_adam's atomic maxima (nullable: no update in this call)
    if (range_m && blockIdx.x == 0 && threadIdx.x < kNumParams) range_m[threadIdx.x] = 0.f;
}

// Block partial sums of g^2 over the flat gradient after a cross-rank all-reduce (data-parallel
// UPDATE phase; a single-GPU step takes them from k_reduce_grads); advances Adam's step counter.
__global__ __launch_bounds__(256) void k_grad_norm(const float* __restrict__ grads, int n, float* __restrict__ sq_part,
                                                   double* __restrict__ step, const AdamHyper h,
                                                   AdamScalars* __restrict__ sc, float* __restrict__ range_m) {
    if (blockIdx.x == 0 && threadIdx.x < kNumParams) range_m[threadIdx.x] = 0.f;  // as k_reduce_grads'
    __shared__ float red[4];
    float s = 0.f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) s += grads[i] * grads[i];
    s = wave_sum(s);
    if (lane_id() == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        sq_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
        if (blockIdx.x == 0) adam_advance(step, h, sc);
    }
}
constexpr int kSqBlocks = 256;

// clip_grad_norm_(max_norm) + torch.optim.Adam (ppo.py:17-22 groups: actor params < critic trunk
// offset use lr_actor, the rest lr_critic), elementwise over the flat buffers, in the operation order
// and roundings of torch's single-tensor Adam (torch/optim/adam.py) -- the path torch takes for CPU
// tensors, where the reference's update ran when its fixtures were recorded (tests/golden/
// make_golden.py, no GPU). On a CUDA device (agents/ppo.py:14 when one is present) torch defaults to
// the foreach path, p + step * (m / denom): one rounding apart per element, inside the teacher-forced
// bound of tests/adam_bound.py; parity with that path is bounded, not bitwise:
//   m = lerp(m, g, 1 - b1)            = fma(w1, g - m, m)       (the vectorised lerp, weight < 0.5)
//   v = v * b2;  v = addcmul(v, g, g, 1 - b2) = v + ((1 - b2) g) g
//   denom = sqrt(v) / sqrt(1 - b2^t) + eps
//   p = addcdiv(p, m, denom, -lr / (1 - b1^t)) = p + ((-step) m) / denom
// with the step-dependent scalars from AdamScalars; no other contraction (explicit _rn operations).
//
// Work items: one float4 per thread, 256 per block; each parameter's items start a new block, so
// a block's parameter is a table lookup. A GEMM weight's block (kTileK != 0, flat [NR][NC]) covers
// 1024 / NC whole rows: after the update every thread writes its float4 into the forward's
// fragment-order copy (packed), and the block's tile goes through LDS so that every thread writes
// one float4 of the backward's transposed copy (packedT: four consecutive rows of one column) --
// k_policy_pack's mapping inverted, so an UPDATE leaves both current and the next FORWARD may
// skip the pack launch (UAVHIP_PPO_PACKED).
constexpr int kAdamMaxBlocks = 512;
struct AdamBlocks {
    int n;
    int param[kAdamMaxBlocks];  // parameter of the block
    int first[kAdamMaxBlocks];  // its first float4 within the parameter
    int tbase[kAdamMaxBlocks];  // packedT offset of the parameter's transposed copy, -1: none
    int sbase[kAdamMaxBlocks];  // packed offset of the parameter's split copy, -1: none
    int pbeg[kNumParams + 1];   // parameter q's blocks: [pbeg[q], pbeg[q + 1])
};
constexpr int adam_items(int q) { return pad4(kSizes[q]) / 4; }
constexpr int packedT_base(int q) {
    for (int li = 0; li < 3; ++li) {
        const int trunk = li == 0 ? kActorTrunk : kCriticTrunk, layer = li == 2 ? 1 : 0;
        if (q == layer_param(trunk, layer, INW)) return li * kLayerT + kTWin;
        if (q == layer_param(trunk, layer, OUTW)) return li * kLayerT + kTWo;
        if (q == layer_param(trunk, layer, L1W)) return li * kLayerT + kTW1;
        if (q == layer_param(trunk, layer, L2W)) return li * kLayerT + kTW2;
    }
    if (q == kActorHead) return kHeadT;
    if (q == kCriticHead) return kHeadT + D * HID;
    return -1;
}
constexpr AdamBlocks make_adam_blocks() {
    AdamBlocks b{};
    for (int q = 0; q < kNumParams; ++q) {
        b.pbeg[q] = b.n;
        for (int f = 0; f < adam_items(q); f += 256) {
            b.param[b.n] = q;
            b.first[b.n] = f;
            b.tbase[b.n] = packedT_base(q);
            b.sbase[b.n] = split_slot(q);
            ++b.n;
        }
    }
    b.pbeg[kNumParams] = b.n;
    return b;
}
constexpr AdamBlocks kAdamBlocks = make_adam_blocks();
constexpr bool adam_tiles_ok() {  // every tiled weight: whole blocks of whole rows, a transposed copy
    for (int q = 0; q < kNumParams; ++q)
        if (kTileK[q] && (kSizes[q] % 1024 || 1024 % kTileK[q] || (1024 / kTileK[q]) % 4 || packedT_base(q) < 0))
            return false;
    return true;
}
static_assert(kAdamBlocks.n <= kAdamMaxBlocks && adam_tiles_ok(), "Adam block table");

struct AdamArgs {
    float* params;
    float* grads;
    float* m;
    float* v;
    const AdamScalars* sc;
    const float* sq_part;
    int n_sq;
    double beta1, beta2, eps;
    float max_norm;
    float *packed, *packedT;  // nullable: refreshed with the updated params
};

__global__ __launch_bounds__(256) void k_adam(const AdamArgs a) {
    __shared__ float red[4];
    __shared__ __attribute__((aligned(16))) float tile[1024];
    const int q = kAdamBlocks.param[blockIdx.x];
    const int item = kAdamBlocks.first[blockIdx.x] + threadIdx.x;
    const int NC = kTileK[q], off = kOffs.o[q];
    const bool live = item < adam_items(q);
    const int f = off + 4 * item;
    // the update operands first, then the g^2 partials: both latencies overlap
    f32x4 g, m, v, p;
    if (live) {
        g = *reinterpret_cast<const f32x4*>(a.grads + f);
        m = *reinterpret_cast<const f32x4*>(a.m + f);
        v = *reinterpret_cast<const f32x4*>(a.v + f);
        p = *reinterpret_cast<const f32x4*>(a.params + f);
    }
    // the g^2 block partials (~2k): 8 independent loads in flight per thread, not a dependent chain
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < a.n_sq; i += 8 * 256) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i + 256 * u < a.n_sq) s8[u] += a.sq_part[i + 256 * u];
    }
    const AdamScalars sc = *a.sc;
    float s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    s = wave_sum(s);
    if (lane_id() == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    const float coef = fminf(a.max_norm / (norm + 1e-6f), 1.0f);
    const float nss = q < kCriticTrunk ? sc.nss_a : sc.nss_c;
    const float w1 = (float)(1.0 - a.beta1), b2 = (float)a.beta2, w2 = (float)(1.0 - a.beta2), epsf = (float)a.eps;
    if (live) {
        // no contraction here: __fmul_rn / __fadd_rn alone do not stop the compiler fusing a product
        // into the sum after it (this file builds with contraction on), the pragma does
#pragma clang fp contract(off)
        g = g * coef;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            m[j] = __fmaf_rn(w1, g[j] - m[j], m[j]);  // torch's vectorised lerp: one fma
            v[j] = v[j] * b2 + (w2 * g[j]) * g[j];
            const float denom = __fdiv_rn(__fsqrt_rn(v[j]), sc.bc2s) + epsf;
            p[j] = p[j] + __fdiv_rn(nss * m[j], denom);
        }
        *reinterpret_cast<f32x4*>(a.grads + f) = g;
        *reinterpret_cast<f32x4*>(a.m + f) = m;
        *reinterpret_cast<f32x4*>(a.v + f) = v;
        *reinterpret_cast<f32x4*>(a.params + f) = p;
    }
    if (!a.packed) return;
    {   // the packed range table (policy_layout.hpp) of the updated parameters: each block's max
        // |param| into its parameter's slot by an atomic max on the float bits (non-negative floats
        // order like their bits; the slots were zeroed by k_reduce_grads / k_grad_norm, earlier in
        // this step; order-free, so deterministic). The kernels derive every scale from these maxima.
        float am = live ? fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fmaxf(fabsf(p[2]), fabsf(p[3]))) : 0.f;
        am = wave_max(am);
        __shared__ float amw[4];
        if (lane_id() == 0) amw[threadIdx.x >> 6] = am;
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<unsigned*>(a.packed + kRangeOff + kRgMax + q),
                      __float_as_uint(fmaxf(fmaxf(amw[0], amw[1]), fmaxf(amw[2], amw[3]))));
    }
    if (!NC) {  // plain parameters are copied as they are
        if (live) *reinterpret_cast<f32x4*>(a.packed + f) = p;
        return;
    }
    // packed: row i of [NR][NC] in fragment order, float4 = columns j..j+3 (not for the weights the
    // training kernels read only through their split copies: policy_train.hpp kTrainF32LayerCopies)
    const int loc = 4 * item, i = loc / NC, j = loc - i * NC;
    const int sb = kAdamBlocks.sbase[blockIdx.x];
    if (kTrainF32LayerCopies || sb < 0)
        *reinterpret_cast<f32x4*>(a.packed + off + (((i >> 4) * (NC >> 4) + (j >> 4)) * 64 + (i & 15) +
                                                      16 * ((j & 15) >> 2)) * 4) = p;
    // the split copy (policy_layout.hpp kSplitParam): the fp16 planes of these four weights, lane
    // (i % 16) + 16 ((j % 32) / 8) of block (i / 16, j / 32), halves j % 8 .. + 3
    if (sb >= 0) {
        wg_f16x4 w1, w2;
        f16_split4(p, w1, w2);
        _Float16* sp = reinterpret_cast<_Float16*>(a.packed + sb) +
                       (((i >> 4) * (NC >> 5) + (j >> 5)) * 128 + (i & 15) + 16 * ((j & 31) >> 3)) * 8 + (j & 7);
        *reinterpret_cast<wg_f16x4*>(sp) = w1;
        *reinterpret_cast<wg_f16x4*>(sp + 64 * 8) = w2;
    }
    // packedT: W^T ([NC][NR]) in fragment order, float4 = rows it..it+3 of column jt
    *reinterpret_cast<f32x4*>(tile + 4 * threadIdx.x) = p;
    __syncthreads();
    const int NR = kSizes[q] / NC, i0 = 4 * kAdamBlocks.first[blockIdx.x] / NC;
    const int jt = threadIdx.x % NC, rq = threadIdx.x / NC, it = i0 + 4 * rq;
    const f32x4 col = {tile[(4 * rq) * NC + jt], tile[(4 * rq + 1) * NC + jt], tile[(4 * rq + 2) * NC + jt],
                       tile[(4 * rq + 3) * NC + jt]};
    const int tb = kAdamBlocks.tbase[blockIdx.x];
    if (kTrainF32LayerCopies || tb >= kHeadT)
        *reinterpret_cast<f32x4*>(a.packedT + tb + (((jt >> 4) * (NR >> 4) + (it >> 4)) * 64 + (jt & 15) +
                                                    16 * ((it & 15) >> 2)) * 4) = col;
    if (tb < kHeadT) {  // a layer weight: its transposed split copy (W^T[jt][it .. it + 3], halves it % 8 ..)
        wg_f16x4 w1, w2;
        f16_split4(col, w1, w2);
        _Float16* sp = reinterpret_cast<_Float16*>(a.packedT + kTSplit + tb) +
                       (((jt >> 4) * (NR >> 5) + (it >> 5)) * 128 + (jt & 15) + 16 * ((it & 31) >> 3)) * 8 + (it & 7);
        *reinterpret_cast<wg_f16x4*>(sp) = w1;
        *reinterpret_cast<wg_f16x4*>(sp + 64 * 8) = w2;
    }
}

// ================================================================== host orchestration
struct WS {  // workspace carve-up (floats), identical for sizing and for the step
    size_t off = 0;
    float* base = nullptr;
    float* take(size_t n) {
        float* p = base ? base + off : nullptr;
        off += (n + 63) & ~(size_t)63;
        return p;
    }
};

struct LayerBufs {  // one encoder layer (pruned: tail tensors are [Bm] rows)
    float *qkv, *o, *xhat1, *rstd1, *h1, *u, *xhat2, *rstd2, *h2;
    float *dqkv, *dz1, *du, *df;
    float *ln1_part, *ln2_part;
};

struct Plan {
    int Bm, R;
    float *xg, *mask, *tmax, *smp, *e_a, *h0_a, *e_c, *h0_c;
    LayerBufs la, lc0, lc1;
    float *z_a, *z_c, *dz_a, *dz_c, *fpart, *hpart, *epart, *sq_part;
    AdamScalars* adam_sc;  // Adam's step-dependent scalars (k_reduce_grads / k_grad_norm -> k_adam)
    float* vpart;          // [Bm/16] the forward's per-block value-error maxima (BwdIO::vpart)
    float* gsc;            // 2^k of the critic's gradient scale (heads_bwd -> k_reduce_grads)
    float* xmax;           // [Bm/16] the forward's per-block window-row maxima (k_wgrad's layer-0 X range)
    float* rt;             // [kRtN] the forward's derived scales (TrainIO::rtab_out -> k_wgrad)
    float* wg_part;  // weight-gradient partial tiles [kWgGrid * kWgRuns][kWgSlot]
    float* bpart;    // [prows][kBiasPart] bias partials of K6 / K7
    float* kvc;      // K7: [prows][80][256] each query position's share of every position's dk | dv
    int prows;       // partial rows: Bm/16, or 5 Bm/16 (position split: row b * 5 + s)
    float* packed;  // fragment-order copy of the parameters for the fused forward
    float* packedT; // transposed GEMM weights for the fused backward
    size_t total;   // workspace floats
};

inline void carve_layer(WS& w, LayerBufs& L, int R, int rows, int parts) {
    L.qkv = w.take((size_t)R * 3 * D);
    L.o = w.take((size_t)rows * D);
    L.xhat1 = w.take((size_t)rows * D);
    L.rstd1 = w.take(rows);
    L.h1 = w.take((size_t)rows * D);
    L.u = w.take((size_t)rows * FF);
    L.xhat2 = w.take((size_t)rows * D);
    L.rstd2 = w.take(rows);
    L.h2 = w.take((size_t)rows * D);
    L.dqkv = w.take((size_t)R * 3 * D);
    L.dz1 = w.take((size_t)rows * D);
    L.du = w.take((size_t)rows * FF);
    L.df = w.take((size_t)rows * D);
    L.ln1_part = w.take((size_t)parts * 2 * D);  // one partial row per workgroup of K6 / K7
    L.ln2_part = w.take((size_t)parts * 2 * D);
}

inline Plan make_plan(int Bm, float* base) {
    Plan p{};
    WS w;
    w.base = base;
    p.Bm = Bm;
    p.R = Bm * S;
    const int R = p.R;
    // partial rows: sized for the position split whenever this minibatch may run it (independent
    // of UAVHIP_POS_SPLIT, so the workspace size never depends on the environment)
    p.prows = (pol::ps_capable(Bm) ? S : 1) * (Bm / kHeadSamples);
    p.xg = w.take((size_t)R * 16);
    p.mask = w.take(R);
    p.tmax = w.take(R);
    p.xmax = w.take(Bm / kHeadSamples);
    static_assert(kRtN <= 32, "Plan::rt");
    p.rt = w.take(32);
    p.smp = w.take((size_t)Bm * 8);
    p.e_a = w.take((size_t)R * D);
    p.h0_a = w.take((size_t)R * D);
    p.e_c = w.take((size_t)R * D);
    p.h0_c = w.take((size_t)R * D);
    carve_layer(w, p.la, R, Bm, p.prows);
    carve_layer(w, p.lc0, R, R, p.prows);
    carve_layer(w, p.lc1, R, Bm, p.prows);
    p.z_a = w.take((size_t)Bm * HID);
    p.z_c = w.take((size_t)Bm * HID);
    p.dz_a = w.take((size_t)Bm * HID);
    p.dz_c = w.take((size_t)Bm * HID);
    p.fpart = w.take((size_t)(Bm / kHeadSamples) * 4);
    p.hpart = w.take((size_t)(Bm / kHeadSamples) * kHeadPart);
    p.epart = w.take((size_t)p.prows * 2 * kEmbPart);
    p.sq_part = w.take(1 << 16);
    p.adam_sc = reinterpret_cast<AdamScalars*>(w.take(4));
    p.vpart = w.take((size_t)(Bm / kHeadSamples));
    p.gsc = w.take(4);
    p.wg_part = w.take((size_t)kWgGrid * kWgRuns * kWgSlot);
    p.bpart = w.take((size_t)p.prows * pol::kBiasPart);
    p.kvc = pol::ps_capable(Bm) ? w.take((size_t)p.prows * S * kHeadSamples * 2 * D) : nullptr;  // [prows][80][256]
    p.packed = w.take(kPackedFloats);  // + the split copies (the training forward's split products)
    p.packedT = w.take(pol::kPackedTAllFloats);  // + the transposed split copies (K6's split products)
    p.total = w.off;
    return p;
}


// The backward's gradient pre-scale (BwdIO::gscale): the power of two >= the global minibatch
// (UAVHIP_GRAD_PRESCALE=0: 1, the unscaled backward, for the per-element precision test's A/B).
inline float grad_prescale(int Bg) {
    const char* e = std::getenv("UAVHIP_GRAD_PRESCALE");
    if (e && e[0] == '0') return 1.0f;
    int s = 1;
    while (s < Bg && s < (1 << 30)) s <<= 1;
    return (float)s;
}

inline const float* prm(const uavhip_ppo* c, int i) { return c->params + kOffs.o[i]; }
inline AdamHyper adam_hyper(const uavhip_ppo* c) { return AdamHyper{c->lr_actor, c->lr_critic, c->beta1, c->beta2}; }

// Position split (K7) for this minibatch size (UAVHIP_POS_SPLIT=0 turns it off: tests compare both ways).
inline bool pos_split(int Bm) {
    const char* e = std::getenv("UAVHIP_POS_SPLIT");
    return pol::ps_capable(Bm) && !(e && e[0] == '0');
}

// Weight gradients in direct mode (WgBatch::direct) only on request (UAVHIP_WGRAD_DIRECT=1, and
// only when no tile has more than kWgDirectMaxSlabs slabs): measured at minibatch 64 (r04b, same box,
// scripts/train_probe.py) the stream-K form with k_reduce_grads is faster, 0.098 against 0.113 ms
// per step -- one workgroup walking a tile's 10 slabs is a longer chain than spreading them over
// 148 workgroups and summing the partials.
inline bool wgrad_direct(int max_slabs) {
    const char* e = std::getenv("UAVHIP_WGRAD_DIRECT");
    return e && e[0] == '1' && max_slabs <= kWgDirectMaxSlabs;
}

// Weight gradients in chunked mode (WgBatch::chunk: one (chunk, tile) per workgroup, operand-sharing
// tiles on one XCD) for long k ranges (>= 64 slabs: 2048 rows); UAVHIP_WGRAD_CHUNK=0 / 1 forces
// stream-K / chunked.
inline bool wgrad_chunked(int max_slabs) {
    const char* e = std::getenv("UAVHIP_WGRAD_CHUNK");
    if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
    return max_slabs >= 64;
}

// K6's trunk order mixed across workgroups (BwdIO::mix; UAVHIP_BWD_MIX=0: every workgroup critic first)
inline int bwd_mix() {
    const char* e = std::getenv("UAVHIP_BWD_MIX");
    return !(e && e[0] == '0');
}

// The training forward's trunk order mixed across workgroups (TrainIO::mix; UAVHIP_FWD_MIX=0: actor first)
inline int fwd_mix() {
    const char* e = std::getenv("UAVHIP_FWD_MIX");
    return !(e && e[0] == '0');
}

// Chunk length of the three-plane problems relative to the two-plane ones in the chunked schedule
// (UAVHIP_WGRAD_P3_RATIO, default 0.75: the per-slab cost ratio of the two forms)
inline float wgrad_p3_ratio() {
    const char* e = std::getenv("UAVHIP_WGRAD_P3_RATIO");
    const float r = e ? (float)std::atof(e) : 0.75f;
    return r > 0.f && r <= 1.f ? r : 0.75f;
}

// Every weight-gradient tile on three-plane products (UAVHIP_WGRAD_PLANES=3; default: the key rows only)
inline bool wgrad_all_three_planes() {
    const char* e = std::getenv("UAVHIP_WGRAD_PLANES");
    return e && e[0] == '3';
}

// Trunk split for this minibatch size (UAVHIP_TRUNK_SPLIT=0 turns it off: tests compare both ways).
inline int split_blocks(int Bm) {
    const char* e = std::getenv("UAVHIP_TRUNK_SPLIT");
    return (pol::trunk_split(Bm) && !(e && e[0] == '0')) ? Bm / kHeadSamples : 0;
}

}  // namespace tr
}  // namespace uavhip

using namespace uavhip;
using namespace uavhip::tr;

#ifdef UAVHIP_POLICY_TRACE
extern "C" int uavhip_wgrad_trace(unsigned long long* out, int n) {  // k_wgrad stamps (TRACE build)
    const int total = kWgGrid * 16;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wtrace), sizeof(unsigned long long) * (n < total ? n : total), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int64_t uavhip_ppo_workspace_floats(int32_t minibatch) {
    if (minibatch <= 0 || minibatch % 64) return -1;
    return (int64_t)make_plan(minibatch, nullptr).total;
}

#define TR_CHECK(x)          \
    do {                     \
        const int rc_ = (x); \
        if (rc_) return rc_; \
    } while (0)

static int ppo_backward(const uavhip_ppo* c, const Plan& p, hipStream_t st, int Bg, double* step, int* n_sq,
                        bool fused_sums);

extern "C" int uavhip_ppo_step(const uavhip_ppo* c, const float* states, const int8_t* actions,
                               const float* old_logp, const float* old_values, const float* returns,
                               const float* advantages, const int32_t* idx, int32_t phases, uavhip_stream_t stream) {
    const bool fwd = phases & UAVHIP_PPO_FORWARD, bwd = phases & UAVHIP_PPO_BACKWARD, upd = phases & UAVHIP_PPO_UPDATE;
    if (!c || !c->params || !c->grads || !c->workspace || !c->loss_sums ||
        ((fwd || bwd) && (!states || !actions || !old_logp || !old_values || !returns || !advantages || !idx))) {
        set_error("uavhip_ppo_step: NULL pointer");
        return UAVHIP_EINVAL;
    }
    const int Bg = c->global_minibatch > 0 ? c->global_minibatch : c->minibatch;
    if (c->minibatch <= 0 || c->minibatch % 64 || Bg < c->minibatch || c->n_floats != kOffs.o[kNumParams] ||
        (phases & UAVHIP_PPO_FULL) == 0 || (phases & ~(UAVHIP_PPO_FULL | UAVHIP_PPO_PACKED)) ||
        (upd && (!c->adam_m || !c->adam_v || !c->adam_step))) {
        set_error("uavhip_ppo_step: minibatch %d (multiple of 64), global %d, n_floats %d (expected %d), phases %d",
                  c->minibatch, Bg, c->n_floats, kOffs.o[kNumParams], phases);
        return UAVHIP_EINVAL;
    }
    hipStream_t st = (hipStream_t)stream;
    const Plan p = make_plan(c->minibatch, c->workspace);
    const int Bm = p.Bm, nblk = Bm / kHeadSamples;
    const LayerBufs &A = p.la, &C0 = p.lc0, &C1 = p.lc1;

    // ---------------------------------------------------------------- forward
    // The rollout's fused forward kernel (policy.hip) in training mode: one workgroup per 16
    // samples, every activation the backward needs written to the workspace.
    if (fwd) {
        if (!(phases & UAVHIP_PPO_PACKED)) TR_CHECK(pol::policy_pack_train(c->params, p.packed, p.packedT, st));
        pol::TrainIO io{};
        io.idx = idx;
        io.act_in = actions;
        io.oldlp_in = old_logp;
        io.oldv_in = old_values;
        io.ret_in = returns;
        io.adv_in = advantages;
        io.smp = p.smp;
        io.xg = p.xg;
        io.mask = p.mask;
        io.tmax = p.tmax;
        io.xmax = p.xmax;
        io.rtab_out = p.rt;
        io.e[0] = p.e_a; io.e[1] = p.e_c;
        io.h0[0] = p.h0_a; io.h0[1] = p.h0_c;
        const LayerBufs* lb[3] = {&A, &C0, &C1};
        for (int i = 0; i < 3; ++i)
            io.L[i] = pol::TrainLayerIO{lb[i]->qkv, lb[i]->o, lb[i]->xhat1, lb[i]->rstd1, lb[i]->h1, lb[i]->u,
                                        lb[i]->xhat2, lb[i]->rstd2, lb[i]->h2};
        io.z[0] = p.z_a;
        io.z[1] = p.z_c;
        io.fpart = p.fpart;
        io.vpart = p.vpart;
        io.eps_clip = c->eps_clip;
        if (pos_split(Bm)) {  // K7: F1 / F2 / F3 (F3 writes the loss partials)
            TR_CHECK(pol::policy_forward_ps(p.packed, states, io, Bm, st));
        } else {
            io.split = split_blocks(Bm);
            io.mix = fwd_mix();
            TR_CHECK(pol::policy_forward_train(p.packed, states, io, Bm, st));
            if (io.split) TR_CHECK(pol::policy_loss_partials(io, Bm, st));
        }
        if (!bwd) {  // with BACKWARD in the same call, K6 sums the partials itself (one launch fewer)
            hipLaunchKernelGGL(k_loss_sums, dim3(1), dim3(64), 0, st, p.fpart, nblk, c->loss_sums);
            TR_CHECK(check_launch("k_loss_sums"));
        }
    }
    // single-GPU FULL step: the gradient reduction leaves the g^2 partials of the final grads;
    // otherwise (UPDATE after an all-reduce of grads) k_grad_norm computes them
    int n_sq = kSqBlocks;
    if (bwd) TR_CHECK(ppo_backward(c, p, st, Bg, upd ? c->adam_step : nullptr, &n_sq, fwd));
    if (upd) {
        if (!bwd) {
            hipLaunchKernelGGL(k_grad_norm, dim3(kSqBlocks), dim3(256), 0, st, c->grads, c->n_floats, p.sq_part,
                               c->adam_step, adam_hyper(c), p.adam_sc, p.packed + kRangeOff + kRgMax);
            TR_CHECK(check_launch("k_grad_norm"));
        }
        AdamArgs aa{c->params, c->grads, c->adam_m, c->adam_v, p.adam_sc, p.sq_part, n_sq, c->beta1, c->beta2,
                    c->adam_eps, c->max_grad_norm, p.packed, p.packedT};
        hipLaunchKernelGGL(k_adam, dim3(kAdamBlocks.n), dim3(256), 0, st, aa);
        TR_CHECK(check_launch("k_adam"));
    }
    return UAVHIP_OK;
}

// Backward + weight gradients of one minibatch (the workspace holds the forward's activations).
static int ppo_backward(const uavhip_ppo* c, const Plan& p, hipStream_t st, int Bg, double* step, int* n_sq,
                        bool fused_sums) {
    const int Bm = p.Bm, R = p.R, nblk = Bm / kHeadSamples;
    const LayerBufs &A = p.la, &C0 = p.lc0, &C1 = p.lc1;
    const int ta = kActorTrunk, tc = kCriticTrunk;
    // partial rows: K6 one per 16-sample workgroup; K7 one per (block, position), row b * 5 + s, the
    // per-block layers (actor L0, critic L1: their pruned tails) at row b * 5
    const bool ps = pos_split(Bm);
    const int rstep = ps ? S : 1;                 // rows from one block's per-block partial row to the next
    const int full_parts = ps ? p.prows : nblk;    // critic L0 and the embeddings (K7: every row)
    {
        pol::BwdIO io{};
        io.smp = p.smp;
        io.tot = c->loss_sums;
        if (fused_sums) {
            io.fpart = p.fpart;
            io.nfpart = nblk;
            io.tot_out = c->loss_sums;
        }
        io.z[0] = p.z_a;
        io.z[1] = p.z_c;
        io.dz[0] = p.dz_a;
        io.dz[1] = p.dz_c;
        io.hpart = p.hpart;
        io.stats = c->stats;
        io.eps_clip = c->eps_clip;
        io.value_coef = c->value_coef;
        io.entropy_coef = c->entropy_coef;
        io.Bg = Bg;
        io.gscale = grad_prescale(Bg);
        io.vpart = p.vpart;
        io.nvpart = nblk;
        io.gsc_out = p.gsc;
        io.xg = p.xg;
        io.mask = p.mask;
        io.e[0] = p.e_a;
        io.e[1] = p.e_c;
        io.epart = p.epart;
        io.split = ps ? 0 : split_blocks(Bm);
        io.mix = bwd_mix();
        const LayerBufs* lb[3] = {&A, &C0, &C1};
        for (int i = 0; i < 3; ++i)
            io.L[i] = pol::BwdLayerIO{lb[i]->qkv, lb[i]->xhat1, lb[i]->rstd1, lb[i]->u, lb[i]->xhat2, lb[i]->rstd2,
                                      lb[i]->dqkv, lb[i]->dz1, lb[i]->du, lb[i]->df, lb[i]->ln1_part,
                                      lb[i]->ln2_part, p.bpart + (size_t)i * pol::kBiasLayer};
        if (ps) TR_CHECK(pol::policy_backward_ps(p.packed, p.packedT, io, p.kvc, Bm, st));
        else TR_CHECK(pol::policy_backward_train(p.packed, p.packedT, io, Bm, st));
    }

    // ---------------------------------------------------------------- weight gradients
    SegBatch sb{};
    int seg_blocks = 0;
    int sq_base = 0;  // direct-mode k_wgrad's g^2 partials come first in sq_part
    auto seg = [&](const float* src, int dst, int count, int parts, int part_stride, const float* src_rest = nullptr,
                   int dst_ld = 0) {
        if (sb.n >= kMaxSegs) { ++sb.n; return; }
        Segment& s = sb.s[sb.n++];
        s.src = src; s.dst = dst; s.count = count; s.parts = parts; s.part_stride = part_stride;
        s.src_rest = src_rest ? src_rest : src + part_stride;
        s.dst_ld = dst_ld;
        s.block_begin = seg_blocks;
        s.tile_mode = parts > kTileModeParts && !src_rest;
        auto al16 = [](const float* q) { return ((uintptr_t)q & 15) == 0; };
        s.vec4 = !s.tile_mode && al16(s.src) && al16(s.src_rest) && part_stride % 4 == 0 && dst % 4 == 0 &&
                 dst_ld % 4 == 0;
        seg_blocks += s.tile_mode ? (count + 63) / 64 : s.vec4 ? (count + 1023) / 1024 : (count + 255) / 256;
    };
    {
        // dW[out][in] = sum_rows dY[row][out] X[row][in]; dst = the weight's float offset
        WgPlan wp;
        int dst[kWgMaxProbs];
        // X operands the fused forward does not store (wgrad.hpp kWgX*): a LayerNorm output from its
        // x-hat (x-hat * gamma + beta), a layer-0 input from the embedding (e + pos[s])
        // rk / rarg: the X operand's range for k_wgrad (WgProb::rk), as the forward bounds it
        struct XSrc {
            const float* x;
            int mode;
            const float *g, *b;
            int rk, rarg;
            XSrc at_token4() const {  // the token-4 rows (stride S D): one position of the pos table
                return XSrc{x + (S - 1) * D, mode == kWgXPosRow ? (int)kWgXPosFixed : mode, g,
                            mode == kWgXPosRow ? b + (S - 1) * D : b, rk, rarg};
            }
        };
        auto ln_out = [&](const float* xhat, int tr_, int ly, int w) {  // w = N1W or N2W (+1: bias)
            return XSrc{xhat, kWgXAffine, prm(c, layer_param(tr_, ly, w)), prm(c, layer_param(tr_, ly, w + 1)),
                        kWgRStatic, range_op(tr_, ly, w == N1W ? kOpLn1 : kOpLn2)};
        };
        auto emb_out = [&](const float* e, int tr_) {
            return XSrc{e, kWgXPosRow, nullptr, prm(c, tr_ + POS), kWgRE, trunk_index(tr_)};
        };
        // p3: the tiles that keep three-plane products (WgProb::p3_tiles): the key rows of in_proj,
        // whose sums cancel (softmax drops any per-query constant, so a sample's dk rows sum to
        // zero); every other tile is two-plane. UAVHIP_WGRAD_PLANES=3: every tile three-plane.
        const bool all3 = wgrad_all_three_planes();
        auto dw = [&](const float* dY, int ldy, const XSrc& X, int ldx, int M, int N, int K, int dst_w, int p3 = 0) {
            dst[wp.b.n] = dst_w;
            wp.add(dY, ldy, X.x, ldx, M, N, K, X.mode, X.g, X.b);
            if (wp.ok) {
                WgProb& Q = wp.b.p[wp.b.n - 1];
                Q.dst = dst_w;
                Q.p3_tiles = all3 ? ~0 : p3;
                Q.rk = X.rk;
                Q.rarg = X.rarg;
                Q.rpb = K == R ? S * kHeadSamples : kHeadSamples;  // rows per 16-sample block
                Q.xmax = p.xmax;
            }
        };
        auto layer_dw = [&](const LayerBufs& B, int tr_, int ly, const XSrc& hin, int rows) {
            const int pw = kOffs.o[layer_param(tr_, ly, INW)];
            // Q, K and V rows as problems of their own, so that the chunked schedule can give the
            // three-plane key rows shorter chunks (WgPlan::chunked)
            if (rows == R) {
                dw(B.dqkv, 3 * D, hin, D, D, D, R, pw);
                dw(B.dqkv + D, 3 * D, hin, D, D, D, R, pw + D * D, 1);
                dw(B.dqkv + 2 * D, 3 * D, hin, D, D, D, R, pw + 2 * D * D);
            } else {  // pruned: K / V rows over all R rows, Q rows over the Bm token-4 rows
                dw(B.dqkv + D, 3 * D, hin, D, D, D, R, pw + D * D, 1);
                dw(B.dqkv + 2 * D, 3 * D, hin, D, D, D, R, pw + 2 * D * D);
                dw(B.dqkv + (S - 1) * 3 * D, S * 3 * D, hin.at_token4(), S * D, D, D, Bm, pw);
            }
            const XSrc o = ly == 0 ? XSrc{B.o, kWgX, nullptr, nullptr, kWgRA0, trunk_index(tr_)}
                                   : XSrc{B.o, kWgX, nullptr, nullptr, kWgRStatic, range_op(tr_, ly, kOpAtt)};
            dw(B.dz1, D, o, D, D, D, rows, kOffs.o[layer_param(tr_, ly, OUTW)]);
            dw(B.du, FF, ln_out(B.xhat1, tr_, ly, N1W), D, FF, D, rows, kOffs.o[layer_param(tr_, ly, L1W)]);
            dw(B.df, D, XSrc{B.u, kWgX, nullptr, nullptr, kWgRStatic, range_op(tr_, ly, kOpHid)}, FF, D, FF, rows,
               kOffs.o[layer_param(tr_, ly, L2W)]);
        };
        layer_dw(C0, tc, 0, emb_out(p.e_c, tc), R);  // the long problems first
        layer_dw(A, ta, 0, emb_out(p.e_a, ta), Bm);
        layer_dw(C1, tc, 1, ln_out(C0.xhat2, tc, 0, N2W), Bm);
        dw(p.dz_a, HID, ln_out(A.xhat2, ta, 0, N2W), D, HID, D, Bm, kOffs.o[kActorHead]);
        dw(p.dz_c, HID, ln_out(C1.xhat2, tc, 1, N2W), D, HID, D, Bm, kOffs.o[kCriticHead]);
        wp.b.part = p.wg_part;
        wp.b.rt = p.rt;  // the forward's derived scales
        if (wp.ok && wgrad_direct(wp.max_slabs())) {
            // direct mode: one workgroup per output tile writes dW (unscaled) and its g^2 partial; the
            // reduction below covers the other gradients, its g^2 partials after these
            wp.b.direct = 1;
            wp.b.grads = c->grads;
            wp.b.sq = p.sq_part;
            wp.b.unscale = 1.0f / grad_prescale(Bg);
            wp.b.gsc = p.gsc;
            wp.b.crit_off = kOffs.o[kCriticTrunk];
            sq_base = wp.b.tiles;
            hipLaunchKernelGGL(k_wgrad, dim3(wp.b.tiles), dim3(kWgThreads), 0, st, wp.b);
            TR_CHECK(check_launch("k_wgrad"));
        } else {
            if (wp.ok && wgrad_chunked(wp.max_slabs()) && !wp.chunked(wgrad_p3_ratio())) wp.b.chunk = 0;
            const bool sched = wp.ok && wp.tiles([&](const WgTileRuns& t) {
                const WgProb& P = wp.b.p[t.prob];
                seg(p.wg_part + (size_t)t.first_slot * kWgSlot, dst[t.prob] + t.m0 * P.N + t.n0, t.rows * kWgT, t.runs,
                    t.run_stride * kWgSlot, p.wg_part + (size_t)t.rest_slot * kWgSlot, P.N);
            });
            if (!sched) {
                set_error("uavhip_ppo_step: weight-gradient problems do not fit the stream-K schedule");
                return UAVHIP_EINVAL;
            }
            hipLaunchKernelGGL(k_wgrad, dim3(wp.grid), dim3(kWgThreads), 0, st, wp.b);
            TR_CHECK(check_launch("k_wgrad"));
        }
    }
    // biases of the encoder layers (K6's per-workgroup sums of the dY rows)
    {
        const int lt[3][2] = {{ta, 0}, {tc, 0}, {tc, 1}};
        for (int i = 0; i < 3; ++i) {
            const float* bp = p.bpart + (size_t)i * pol::kBiasLayer;
            const int tr_ = lt[i][0], ly = lt[i][1];
            const int np = i == 1 ? full_parts : nblk;
            const int ps_ = (i == 1 && ps ? 1 : rstep) * pol::kBiasPart;
            seg(bp + pol::kBiasL1, kOffs.o[layer_param(tr_, ly, L1B)], FF, np, ps_);
            seg(bp + pol::kBiasL2, kOffs.o[layer_param(tr_, ly, L2B)], D, np, ps_);
            seg(bp + pol::kBiasOut, kOffs.o[layer_param(tr_, ly, OUTB)], D, np, ps_);
            seg(bp + pol::kBiasIn, kOffs.o[layer_param(tr_, ly, INB)], 3 * D, np, ps_);
        }
    }
    // LayerNorm weight | bias (adjacent parameters, as in the partial rows)
    const LayerBufs* lbs[3] = {&A, &C0, &C1};
    const int lts[3][2] = {{ta, 0}, {tc, 0}, {tc, 1}};
    for (int i = 0; i < 3; ++i) {
        const int np = i == 1 ? full_parts : nblk;
        const int ps_ = (i == 1 && ps ? 1 : rstep) * 2 * D;
        seg(lbs[i]->ln1_part, kOffs.o[layer_param(lts[i][0], lts[i][1], N1W)], 2 * D, np, ps_);
        seg(lbs[i]->ln2_part, kOffs.o[layer_param(lts[i][0], lts[i][1], N2W)], 2 * D, np, ps_);
    }
    // embeddings (pos | We | be per trunk, adjacent parameters; K7: one row per (block, position))
    for (int trunk = 0; trunk < 2; ++trunk)
        seg(p.epart + (size_t)trunk * kEmbPart, kOffs.o[(trunk ? kCriticTrunk : kActorTrunk) + POS], kEmbPart,
            full_parts, 2 * kEmbPart);
    // heads: head.2 weight | bias (adjacent), head.0 bias
    seg(p.hpart, kOffs.o[kActorHead + 2], 2 * HID + 2, nblk, kHeadPart);
    seg(p.hpart + 2 * HID + 2, kOffs.o[kCriticHead + 2], HID + 1, nblk, kHeadPart);
    seg(p.hpart + pol::kHeadB0, kOffs.o[kActorHead + 1], HID, nblk, kHeadPart);
    seg(p.hpart + pol::kHeadB0 + HID, kOffs.o[kCriticHead + 1], HID, nblk, kHeadPart);
    if (sb.n > kMaxSegs || seg_blocks > (1 << 16)) {
        set_error("uavhip_ppo_step: too many gradient segments (%d) / blocks (%d)", sb.n, seg_blocks);
        return UAVHIP_EINVAL;
    }
    // padding floats between parameters stay zero
    hipLaunchKernelGGL(k_reduce_grads, dim3(seg_blocks), dim3(256), 0, st, sb, c->grads, p.sq_part + sq_base, step,
                       adam_hyper(c), p.adam_sc, 1.0f / grad_prescale(Bg), static_cast<const float*>(p.gsc),
                       kOffs.o[kCriticTrunk], step ? p.packed + kRangeOff + kRgMax : nullptr);
    *n_sq = sq_base + seg_blocks;
    return check_launch("k_reduce_grads");
}
