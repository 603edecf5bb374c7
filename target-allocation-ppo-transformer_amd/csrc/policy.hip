// policy.hip -- K4: fused TransformerActorCritic forward (networks/transformer_net.py:15-144) on
// gfx950, fp32 end to end (the reference's dtype) on the f32-input MFMA (v_mfma_f32_16x16x4_f32,
// exact fp32 products, fp32 accumulation).
//
// Work decomposition (MI355X-first):
//  * one workgroup = 4 waves = 16 samples = 80 tokens, token index tok = s * 16 + p (s = window
//    position, p = sample): every 16-column MFMA tile is one window position of the 16 samples,
//    so the last position (the only one the heads read, transformer_net.py:106,114) is exactly
//    column tile 4. B = 4096 -> 256 workgroups = one per CU.
//  * GEMMs are computed transposed, Y^T = W . X^T: the weight rows (Linear's [out][in] layout,
//    contiguous in k) are the A operand, streamed from L2 as float4 (4 k per lane = 4 MFMAs);
//    activations live in LDS as [tok][feature] rows and are the B operand, read as float4; the
//    accumulator (feature rows x token columns) is stored back as one float4 per lane.
//    Both operands use the same k permutation (k = 16*i + 4*(lane>>4) + j for MFMA j), so the
//    sum is over every k exactly once.
//  * the four waves split the output features of every GEMM; attention (5 x 5 per sample and
//    head, far too small for MFMA), LayerNorm and the 128->64->{2,1} heads run on the VALU.
//  * last-layer pruning: in the final encoder layer of each trunk only K and V are formed for
//    all 80 tokens; Q, attention, out-projection, LayerNorms and the FFN run for column tile 4
//    only (2.45 instead of 4.04 MFLOP per sample; numerically identical outputs).
//  * sampling: a = (u < p0) ? 0 : 1 with u ~ Philox(seed, offset + b) (not torch's RNG stream;
//    parity is defined on logits / logp / value / entropy for given actions).
#include "common.hpp"

namespace uavhip {
namespace pol {

constexpr int S = 5, D = 128, NH = 8, HD = 16, FF = 256, IN = 14, HID = 64;
constexpr int SPW = 16;         // samples per workgroup
constexpr int TOK = S * SPW;    // 80
constexpr int NTHR = 256;
constexpr int LDH = D + 4;      // 132: row pad of 16 B -> conflict-free float4 column reads
constexpr int LDB = 3 * 64 + 4; // 196: [Q 64 | K 64 | V 64] for a chunk of 4 heads
constexpr int LDF = D + 4;

// ---- packed parameter table, in state_dict key order (transformer_net.py module order)
constexpr int kLayerParams = 12;
constexpr int kNumParams = 50;
constexpr int kSizes[kNumParams] = {
    // actor_net: pos_embedding, embedding.0.{weight,bias}, layers.0.*
    S * D, D * IN, D, 3 * D * D, 3 * D, D * D, D, FF * D, FF, D * FF, D, D, D, D, D,
    // actor_head.0.{weight,bias}, actor_head.2.{weight,bias}
    HID * D, HID, 2 * HID, 2,
    // critic_net: pos, embedding, layers.0.*, layers.1.*
    S * D, D * IN, D, 3 * D * D, 3 * D, D * D, D, FF * D, FF, D * FF, D, D, D, D, D,
    3 * D * D, 3 * D, D * D, D, FF * D, FF, D * FF, D, D, D, D, D,
    // critic_head.0.{weight,bias}, critic_head.2.{weight,bias}
    HID * D, HID, HID, 1};
constexpr int pad4(int x) { return (x + 3) & ~3; }
struct Offs { int o[kNumParams + 1]; };
constexpr Offs make_offs() {
    Offs r{};
    int acc = 0;
    for (int i = 0; i < kNumParams; ++i) { r.o[i] = acc; acc += pad4(kSizes[i]); }
    r.o[kNumParams] = acc;
    return r;
}
constexpr Offs kOffs = make_offs();
constexpr int kActorTrunk = 0, kActorHead = 15, kCriticTrunk = 19, kCriticHead = 46;
enum { POS = 0, EMB_W = 1, EMB_B = 2 };
enum { INW = 0, INB, OUTW, OUTB, L1W, L1B, L2W, L2B, N1W, N1B, N2W, N2B };
__host__ __device__ constexpr int layer_param(int trunk, int l, int which) { return trunk + 3 + kLayerParams * l + which; }

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Smem {
    float x[SPW * S * IN];      // input windows [p][s][k]
    float h[TOK * LDH];         // residual stream [tok][128]
    float big[TOK * LDB];       // QKV chunk / out-proj result / FFN hidden chunk
    float ctx[TOK * LDH];       // attention output / FFN output
    float z[SPW * HID];         // head hidden
    float logits[SPW * 2];
    float value[SPW];
    int mask[SPW * S];          // key padding mask (transformer_net.py:52-54)
};

// ------------------------------------------------------------------ GEMM building blocks
// acc[nt][ct] += W[wrow[nt] + i][kw0 + k] * X[xtok0 + 16 ct + j][k]  over k in [0, K)
template <int NT, int CT>
__device__ __forceinline__ void gemm_acc(f32x4 (&acc)[NT][CT], const float* __restrict__ W, int ldw,
                                         const int (&wrow)[NT], int kw0, int K, const float* X, int ldx,
                                         int xtok0) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4;
    const float* wp[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) wp[nt] = W + (size_t)(wrow[nt] + i16) * ldw + kw0 + 4 * g;
    const float* xp[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) xp[ct] = X + (xtok0 + 16 * ct + i16) * ldx + 4 * g;
#pragma unroll 2
    for (int kk = 0; kk < K; kk += 16) {
        f32x4 a[NT], b[CT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) a[nt] = *reinterpret_cast<const f32x4*>(wp[nt] + kk);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) b[ct] = *reinterpret_cast<const f32x4*>(xp[ct] + kk);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int ct = 0; ct < CT; ++ct)
                    acc[nt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nt][j], b[ct][j], acc[nt][ct], 0, 0, 0);
    }
}

template <int NT, int CT>
__device__ __forceinline__ void zero(f32x4 (&acc)[NT][CT]) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[nt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Y[ytok0 + 16 ct + j][ycol[nt] + i] = epi(acc + bias[brow[nt] + i])
template <int NT, int CT, bool RELU>
__device__ __forceinline__ void store_acc(const f32x4 (&acc)[NT][CT], const float* __restrict__ bias,
                                          const int (&brow)[NT], float* Y, int ldy, const int (&ycol)[NT],
                                          int ytok0) {
    const int l = lane_id(), i16 = l & 15, g = l >> 4;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + brow[nt] + 4 * g);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            f32x4 v = acc[nt][ct] + bb;
            if (RELU) {
                v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
            }
            *reinterpret_cast<f32x4*>(Y + (ytok0 + 16 * ct + i16) * ldy + ycol[nt] + 4 * g) = v;
        }
    }
}

// Y = epi(W[rows] . X^T + b) for one contiguous block of 64*NT... output features split over waves:
// wave w handles features [f0 + w*16*NT, f0 + (w+1)*16*NT).
template <int NT, int CT, bool RELU>
__device__ __forceinline__ void linear(const float* W, int ldw, int kw0, const float* bias, int f0, int K,
                                       const float* X, int ldx, int xtok0, float* Y, int ldy, int ycol0,
                                       int ytok0) {
    const int w = threadIdx.x >> 6;
    int rows[NT], cols[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        rows[nt] = f0 + (w * NT + nt) * 16;
        cols[nt] = ycol0 + (w * NT + nt) * 16;
    }
    f32x4 acc[NT][CT];
    zero(acc);
    gemm_acc<NT, CT>(acc, W, ldw, rows, kw0, K, X, ldx, xtok0);
    store_acc<NT, CT, RELU>(acc, bias, rows, Y, ldy, cols, ytok0);
}

// ------------------------------------------------------------------ VALU pieces
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// h[tok] = LN(h[tok] + a[tok]) * w + b for tok in [tok0, tok0 + ntok) (post-LN, eps 1e-5)
__device__ void add_layernorm(float* h, const float* a, int lda, int tok0, int ntok, const float* __restrict__ w,
                              const float* __restrict__ b) {
    const int l = lane_id(), wv = threadIdx.x >> 6;
    const float w0 = w[2 * l], w1 = w[2 * l + 1], b0 = b[2 * l], b1 = b[2 * l + 1];
    for (int t = tok0 + wv; t < tok0 + ntok; t += NTHR / kWave) {
        const float v0 = h[t * LDH + 2 * l] + a[t * lda + 2 * l];
        const float v1 = h[t * LDH + 2 * l + 1] + a[t * lda + 2 * l + 1];
        const float mean = wave_sum(v0 + v1) * (1.0f / D);
        const float d0 = v0 - mean, d1 = v1 - mean;
        const float var = wave_sum(d0 * d0 + d1 * d1) * (1.0f / D);
        const float rs = 1.0f / sqrtf(var + 1e-5f);
        h[t * LDH + 2 * l] = d0 * rs * w0 + b0;
        h[t * LDH + 2 * l + 1] = d1 * rs * w1 + b1;
    }
}

// scaled-dot-product attention for heads [4c, 4c+4) of the query positions [qs0, qs0 + nqs),
// keys/values of all 5 positions; reads sm.big (Q|K|V of the chunk), writes sm.ctx.
__device__ void attention_chunk(Smem& sm, int c, int qs0, int nqs) {
    const int ntask = nqs * SPW * 4;
    for (int task = threadIdx.x; task < ntask; task += NTHR) {
        const int hh = task & 3, rest = task >> 2, p = rest & 15, si = qs0 + (rest >> 4);
        const int ti = si * SPW + p;
        const float* qrow = sm.big + ti * LDB + hh * HD;
        float q[HD];
#pragma unroll
        for (int d = 0; d < HD; d += 4) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(qrow + d);
            q[d] = v.x; q[d + 1] = v.y; q[d + 2] = v.z; q[d + 3] = v.w;
        }
        float sc[S];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const float* krow = sm.big + (j * SPW + p) * LDB + 64 + hh * HD;
            float acc = 0.f;
#pragma unroll
            for (int d = 0; d < HD; d += 4) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(krow + d);
                acc += q[d] * v.x + q[d + 1] * v.y + q[d + 2] * v.z + q[d + 3] * v.w;
            }
            sc[j] = sm.mask[p * S + j] ? -INFINITY : acc * 0.25f;  // 1/sqrt(16)
            mx = fmaxf(mx, sc[j]);
        }
        float den = 0.f;
#pragma unroll
        for (int j = 0; j < S; ++j) {
            sc[j] = __expf(sc[j] - mx);
            den += sc[j];
        }
        const float inv = 1.0f / den;
        float o[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) o[d] = 0.f;
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const float pj = sc[j] * inv;
            const float* vrow = sm.big + (j * SPW + p) * LDB + 128 + hh * HD;
#pragma unroll
            for (int d = 0; d < HD; d += 4) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(vrow + d);
                o[d] += pj * v.x; o[d + 1] += pj * v.y; o[d + 2] += pj * v.z; o[d + 3] += pj * v.w;
            }
        }
        float* crow = sm.ctx + ti * LDH + (4 * c + hh) * HD;
#pragma unroll
        for (int d = 0; d < HD; d += 4) *reinterpret_cast<f32x4*>(crow + d) = f32x4{o[d], o[d + 1], o[d + 2], o[d + 3]};
    }
}

// embedding (transformer_net.py:57-59): h[s*16+p] = relu(W_e x[p][s] + b_e) + pos[s]
template <int trunk>
__device__ void embed(Smem& sm, const float* __restrict__ P) {
    const float* We = P + kOffs.o[trunk + EMB_W];
    const float* be = P + kOffs.o[trunk + EMB_B];
    const float* pos = P + kOffs.o[trunk + POS];
    const int f = threadIdx.x & (D - 1);
    float wr[IN];
#pragma unroll
    for (int k = 0; k < IN; ++k) wr[k] = We[f * IN + k];
    const float bf = be[f];
    for (int t = threadIdx.x >> 7; t < TOK; t += NTHR / D) {
        const int s = t / SPW, p = t - s * SPW;
        const float* xr = sm.x + (p * S + s) * IN;
        float acc = bf;
#pragma unroll
        for (int k = 0; k < IN; ++k) acc += wr[k] * xr[k];
        sm.h[t * LDH + f] = fmaxf(acc, 0.f) + pos[s * D + f];
    }
}

// One post-LN nn.TransformerEncoderLayer (relu FFN 256, 8 heads). last: prune to column tile 4.
template <int trunk, int layer, bool last>
__device__ void encoder_layer(Smem& sm, const float* __restrict__ P) {
    const float* Win = P + kOffs.o[layer_param(trunk, layer, INW)];
    const float* bin = P + kOffs.o[layer_param(trunk, layer, INB)];
    const float* Wo = P + kOffs.o[layer_param(trunk, layer, OUTW)];
    const float* bo = P + kOffs.o[layer_param(trunk, layer, OUTB)];
    const float* W1 = P + kOffs.o[layer_param(trunk, layer, L1W)];
    const float* b1 = P + kOffs.o[layer_param(trunk, layer, L1B)];
    const float* W2 = P + kOffs.o[layer_param(trunk, layer, L2W)];
    const float* b2 = P + kOffs.o[layer_param(trunk, layer, L2B)];
    const int wv = threadIdx.x >> 6;
    const int qtok0 = last ? (S - 1) * SPW : 0;   // first query token
    const int nqs = last ? 1 : S;                  // query positions

    // --- self-attention, in two chunks of 4 heads (LDS budget)
    for (int c = 0; c < 2; ++c) {
        // K, V of the chunk for all 80 tokens: 8 row tiles (K 4, V 4) -> 2 per wave
        {
            int rows[2], cols[2];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int tile = wv * 2 + nt;              // 0..7
                const int part = 1 + (tile >> 2);          // 1 = K, 2 = V
                rows[nt] = part * D + 64 * c + 16 * (tile & 3);
                cols[nt] = part * 64 + 16 * (tile & 3);
            }
            f32x4 acc[2][S];
            zero(acc);
            gemm_acc<2, S>(acc, Win, D, rows, 0, D, sm.h, LDH, 0);
            store_acc<2, S, false>(acc, bin, rows, sm.big, LDB, cols, 0);
        }
        // Q of the chunk for the query tokens: 4 row tiles -> 1 per wave
        {
            int rows[1] = {64 * c + 16 * wv};
            int cols[1] = {16 * wv};
            if constexpr (last) {
                f32x4 acc[1][1];
                zero(acc);
                gemm_acc<1, 1>(acc, Win, D, rows, 0, D, sm.h, LDH, qtok0);
                store_acc<1, 1, false>(acc, bin, rows, sm.big, LDB, cols, qtok0);
            } else {
                f32x4 acc[1][S];
                zero(acc);
                gemm_acc<1, S>(acc, Win, D, rows, 0, D, sm.h, LDH, 0);
                store_acc<1, S, false>(acc, bin, rows, sm.big, LDB, cols, 0);
            }
        }
        __syncthreads();
        attention_chunk(sm, c, last ? S - 1 : 0, nqs);
        __syncthreads();
    }
    // --- out projection -> big, then h = LN1(h + attn)
    if constexpr (last) linear<2, 1, false>(Wo, D, 0, bo, 0, D, sm.ctx, LDH, qtok0, sm.big, LDB, 0, qtok0);
    else linear<2, S, false>(Wo, D, 0, bo, 0, D, sm.ctx, LDH, 0, sm.big, LDB, 0, 0);
    __syncthreads();
    add_layernorm(sm.h, sm.big, LDB, qtok0, nqs * SPW, P + kOffs.o[layer_param(trunk, layer, N1W)],
                  P + kOffs.o[layer_param(trunk, layer, N1B)]);
    __syncthreads();
    // --- FFN: hidden 256 in two chunks of 128, second GEMM accumulated in registers
    if constexpr (last) {
        f32x4 acc2[2][1];
        zero(acc2);
        int rows2[2] = {32 * wv, 32 * wv + 16};
        for (int hc = 0; hc < 2; ++hc) {
            linear<2, 1, true>(W1, D, 0, b1, 128 * hc, D, sm.h, LDH, qtok0, sm.big, LDF, 0, qtok0);
            __syncthreads();
            gemm_acc<2, 1>(acc2, W2, FF, rows2, 128 * hc, 128, sm.big, LDF, qtok0);
            __syncthreads();
        }
        store_acc<2, 1, false>(acc2, b2, rows2, sm.ctx, LDH, rows2, qtok0);
    } else {
        f32x4 acc2[2][S];
        zero(acc2);
        int rows2[2] = {32 * wv, 32 * wv + 16};
        for (int hc = 0; hc < 2; ++hc) {
            linear<2, S, true>(W1, D, 0, b1, 128 * hc, D, sm.h, LDH, 0, sm.big, LDF, 0, 0);
            __syncthreads();
            gemm_acc<2, S>(acc2, W2, FF, rows2, 128 * hc, 128, sm.big, LDF, 0);
            __syncthreads();
        }
        store_acc<2, S, false>(acc2, b2, rows2, sm.ctx, LDH, rows2, 0);
    }
    __syncthreads();
    add_layernorm(sm.h, sm.ctx, LDH, qtok0, nqs * SPW, P + kOffs.o[layer_param(trunk, layer, N2W)],
                  P + kOffs.o[layer_param(trunk, layer, N2B)]);
    __syncthreads();
}

// 128 -> 64 -> relu -> nout on the last-position rows of sm.h (transformer_net.py:77-91)
template <int head, int nout>
__device__ void head_mlp(Smem& sm, const float* __restrict__ P, float* out) {
    const float* W0 = P + kOffs.o[head + 0];
    const float* b0 = P + kOffs.o[head + 1];
    const float* W2 = P + kOffs.o[head + 2];
    const float* b2 = P + kOffs.o[head + 3];
    for (int i = threadIdx.x; i < SPW * HID; i += NTHR) {
        const int p = i / HID, o = i - p * HID;
        const float* hr = sm.h + ((S - 1) * SPW + p) * LDH;
        const float* wr = W0 + o * D;
        float acc = 0.f;
        for (int k = 0; k < D; k += 4) {
            const f32x4 hv = *reinterpret_cast<const f32x4*>(hr + k);
            const f32x4 wv = *reinterpret_cast<const f32x4*>(wr + k);
            acc += hv.x * wv.x + hv.y * wv.y + hv.z * wv.z + hv.w * wv.w;
        }
        sm.z[p * HID + o] = fmaxf(acc + b0[o], 0.f);
    }
    __syncthreads();
    if (threadIdx.x < SPW * nout) {
        const int p = threadIdx.x / nout, a = threadIdx.x - p * nout;
        float acc = 0.f;
        for (int o = 0; o < HID; ++o) acc += W2[a * HID + o] * sm.z[p * HID + o];
        out[p * nout + a] = acc + b2[a];
    }
    __syncthreads();
}

__global__ __launch_bounds__(NTHR) void k_policy_forward(const float* __restrict__ P, const float* __restrict__ states,
                                                         int B, const int8_t* __restrict__ actions_in, uint64_t seed,
                                                         uint64_t offset, int8_t* __restrict__ action_out,
                                                         float* __restrict__ logp_out, float* __restrict__ value_out,
                                                         float* __restrict__ ent_out, float* __restrict__ logits_out) {
    __shared__ __attribute__((aligned(16))) Smem sm;
    const int b0 = blockIdx.x * SPW;
    // load 16 windows [p][s][k] (zero-fill the batch tail)
    for (int i = threadIdx.x; i < SPW * S * IN; i += NTHR) {
        const int p = i / (S * IN);
        sm.x[i] = (b0 + p < B) ? states[(size_t)b0 * S * IN + i] : 0.f;
    }
    __syncthreads();
    if (threadIdx.x < SPW * S) {  // key padding mask: all-zero rows, last row never masked
        const int p = threadIdx.x / S, s = threadIdx.x - p * S;
        bool z = true;
        for (int k = 0; k < IN; ++k) z = z && (sm.x[(p * S + s) * IN + k] == 0.f);
        sm.mask[p * S + s] = (s < S - 1) && z;
    }
    __syncthreads();
    // actor trunk (1 layer) + head
    embed<kActorTrunk>(sm, P);
    __syncthreads();
    encoder_layer<kActorTrunk, 0, true>(sm, P);
    head_mlp<kActorHead, 2>(sm, P, sm.logits);
    // critic trunk (2 layers) + head
    embed<kCriticTrunk>(sm, P);
    __syncthreads();
    encoder_layer<kCriticTrunk, 0, false>(sm, P);
    encoder_layer<kCriticTrunk, 1, true>(sm, P);
    head_mlp<kCriticHead, 1>(sm, P, sm.value);
    // Categorical(softmax(logits)): sample / log_prob / entropy (transformer_net.py:118-122)
    if (threadIdx.x < SPW) {
        const int p = threadIdx.x, b = b0 + p;
        if (b < B) {
            const float l0 = sm.logits[2 * p], l1 = sm.logits[2 * p + 1];
            const float m = fmaxf(l0, l1);
            const float lse = m + logf(expf(l0 - m) + expf(l1 - m));
            const float lp0 = l0 - lse, lp1 = l1 - lse;
            const float p0 = expf(lp0), p1 = expf(lp1);
            int a;
            if (actions_in) {
                a = actions_in[b] != 0;
            } else {
                const unsigned long long c = offset + (unsigned long long)b;
                const u32x4 r = philox(u32x4{(uint32_t)c, (uint32_t)(c >> 32), 0x5eedu, 0x9e37u}, (uint32_t)seed,
                                       (uint32_t)(seed >> 32));
                a = u01f(r.x) < p0 ? 0 : 1;
            }
            if (action_out) action_out[b] = (int8_t)a;
            if (logp_out) logp_out[b] = a ? lp1 : lp0;
            if (ent_out) ent_out[b] = -(p0 * lp0 + p1 * lp1);
            if (value_out) value_out[b] = sm.value[p];
            if (logits_out) { logits_out[2 * b] = l0; logits_out[2 * b + 1] = l1; }
        }
    }
}

}  // namespace pol
}  // namespace uavhip

using namespace uavhip;

extern "C" int32_t uavhip_policy_layout(int32_t* offsets, int32_t max_offsets) {
    if (offsets)
        for (int i = 0; i < pol::kNumParams && i < max_offsets; ++i) offsets[i] = pol::kOffs.o[i];
    return pol::kOffs.o[pol::kNumParams];
}

extern "C" int uavhip_policy_forward(const uavhip_policy* policy, const float* states, int32_t B,
                                     const int8_t* actions_in, uint64_t seed, uint64_t offset, int8_t* action_out,
                                     float* logp, float* value, float* entropy, float* logits,
                                     uavhip_stream_t stream) {
    if (!policy || !policy->weights || !states || B <= 0) {
        set_error("uavhip_policy_forward: NULL policy/weights/states or B=%d", B);
        return UAVHIP_EINVAL;
    }
    if (policy->n_floats != pol::kOffs.o[pol::kNumParams] || policy->d_model != pol::D || policy->n_heads != pol::NH ||
        policy->d_ff != pol::FF || policy->d_head_hidden != pol::HID || policy->actor_layers != 1 ||
        policy->critic_layers != 2) {
        set_error("uavhip_policy_forward: unsupported architecture / packed size %d (expected %d)", policy->n_floats,
                  pol::kOffs.o[pol::kNumParams]);
        return UAVHIP_EINVAL;
    }
    const int grid = (B + pol::SPW - 1) / pol::SPW;
    hipLaunchKernelGGL(pol::k_policy_forward, dim3(grid), dim3(pol::NTHR), 0, (hipStream_t)stream, policy->weights,
                       states, (int)B, actions_in, seed, offset, action_out, logp, value, entropy, logits);
    return check_launch("k_policy_forward");
}
