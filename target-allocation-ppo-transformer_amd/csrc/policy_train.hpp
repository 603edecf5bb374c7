// policy_train.hpp -- the training-mode view of the fused policy forward (policy.hip): the same
// kernel, instantiated with TR = true, gathers a minibatch of windows by row index and writes every
// activation the PPO backward (train.hip) reads, in its [row = b * 5 + s][feature] layout
// (pruned layers' tails as compact [b][feature] rows), runs the heads and writes per-workgroup
// partial sums of the PPO loss terms. Sampling is skipped.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "policy_layout.hpp"

namespace uavhip {
namespace pol {

struct TrainLayerIO {
    float *qkv, *o, *xhat1, *rstd1, *h1, *u, *xhat2, *rstd2, *h2;
};
struct TrainIO {
    const int32_t* idx;          // [Bm] rows of the trajectory buffers
    const int8_t* act_in;        // [n]
    const float *oldlp_in, *oldv_in, *ret_in, *adv_in;  // [n]
    float* smp;                  // [Bm][8]: action, old_logp, old_value, return, advantage
    float* xg;                   // [R][16]
    float* mask;                 // [R]
    float* tmax;                 // [R] max |x_k| of each window row (layer 0's operand range; K7 F2 reads it)
    float* xmax;                 // [Bm/16] max over each 16-sample block's window rows (the weight-gradient
                                 // GEMM's range of the layer-0 operands; nullable)
    float* rtab_out;             // [kRtN] the forward's derived scales (policy_layout.hpp kRtOp ..; nullable)
    float *e[2], *h0[2];         // [R][128] actor, critic embeddings (post-ReLU) and layer inputs
    TrainLayerIO L[3];           // actor L0 (pruned), critic L0 (full), critic L1 (pruned)
    float* z[2];                 // [Bm][64] relu(head.0) of the actor / critic head
    float* fpart;                // [Bm/16][4] per-workgroup loss partials: sum min(s1, s2),
                                 // sum (v-R)^2, sum (vc-R)^2, sum entropy (smp[5..7] = logits, value)
    float* vpart;                // [Bm/16] per-workgroup max(|v - R|, |vc - R|) (BwdIO::vpart)
    float eps_clip;
    // trunk split (small minibatches, 2 Bm/16 <= the CU count): workgroups [0, split) run the
    // actor trunk + head, [split, 2 split) the critic trunk + head of the same 16-sample blocks
    // (the two trunks are independent until the loss); the loss partials then come from
    // k_loss_partials. 0: both trunks in every workgroup.
    int split;
    int mix;    // no trunk split: every other group of 8 workgroups runs the critic trunk first
};

// ---- K6: fused backward of the three encoder layers + embeddings (policy.hip), one workgroup per
// 16 samples like the forward. Inputs are the forward's activations; outputs are the dY operands of
// the weight-gradient GEMMs and per-workgroup partials of the LayerNorm / embedding gradients.
struct BwdLayerIO {
    const float *qkv, *xhat1, *rstd1, *u, *xhat2, *rstd2;  // forward activations (TrainLayerIO)
    float *dqkv;                 // [R][384] (pruned layers: Q part on token-4 rows only)
    float *dz1, *du, *df;        // d(LN1 input), d(FFN hidden pre-ReLU), d(LN2 input) rows
    float *ln1_part, *ln2_part;  // [Bm/16][256]: dgamma | dbeta partials per workgroup
    float* bpart;                // this layer's [kBiasLayer] slice of rows [Bm/16][kBiasPart]
};
constexpr int kEmbPart = S * D + D * IN + D;  // 2560: pos [5][128] | We [128][14] | be [128]
// per-workgroup head partials: dW / db of actor_head.2 [0, 130) and critic_head.2 [130, 195), then
// db of actor_head.0 [196, 260) and critic_head.0 [260, 324)
constexpr int kHeadB0 = 196;
constexpr int kHeadPart = kHeadB0 + 2 * HID;
// per-workgroup bias partials of one encoder layer (sums over its rows of the dY operands)
constexpr int kBiasL1 = 0, kBiasL2 = FF, kBiasOut = FF + D, kBiasIn = FF + 2 * D, kBiasLayer = FF + 5 * D;
constexpr int kBiasPart = 3 * kBiasLayer;  // 2688: actor L0 | critic L0 | critic L1
struct BwdIO {
    // heads + loss (ppo.py:148-169): per-sample inputs / logits / value (TrainIO::smp), the loss
    // sums over the global minibatch (all-reduced when data parallel), relu(head.0) rows
    const float* smp;
    const float* tot;
    // FORWARD + BACKWARD in one call: the forward's per-workgroup loss partials [nfpart][4], summed
    // by every workgroup's wave 0 in k_loss_sums' order (tot unused; workgroup 0 writes tot_out)
    const float* fpart;
    int nfpart;
    float* tot_out;
    const float* z[2];
    float* dz[2];            // [Bm][64] d(head.0 pre-activation) (weight-gradient GEMM operand)
    float* hpart;            // [Bm/16][kHeadPart] head.2 weight / bias gradient partials
    double* stats;           // += loss_actor, loss_critic, entropy, 1 (workgroup 0)
    float eps_clip, value_coef, entropy_coef;
    int Bg;                  // samples in the global minibatch
    // every gradient the backward writes is pre-scaled by gscale = the power of two >= Bg (the
    // loss's 1/Bg folded in as gscale/Bg, exact): per-sample gradients O(1) instead of O(1/Bg), so
    // the dX GEMMs' fp16 operand planes stay above the fp16 subnormal range (x2 = f16((x - x1) 2^11)
    // loses relative accuracy below 2^-14); k_reduce_grads multiplies by 1/gscale (exact)
    float gscale;
    // the critic's gradients carry gscale x 2^-k, k from the minibatch's largest value error (the
    // forward's per-block maxima vpart[nvpart]; heads_bwd), and workgroup 0 writes 2^k to gsc_out
    // for the reductions (k_reduce_grads: critic segments x 2^k / gscale). k = 0 below |v - R| = 16.
    const float* vpart;
    int nvpart;
    float* gsc_out;
    const float* xg;         // [R][16] input windows (TrainIO::xg)
    const float* mask;       // [R] key padding mask
    const float* e[2];       // [R][128] embeddings after ReLU
    float* epart;            // [Bm/16][2][kEmbPart] embedding gradient partials
    BwdLayerIO L[3];         // actor L0 (pruned), critic L0 (full), critic L1 (pruned)
    int split;               // trunk split as in TrainIO (actor workgroups first)
    int mix;                 // K6 without the trunk split: every other group of 8 workgroups runs the actor first
};
// Transposed copies of each layer's GEMM weights in fragment order (the dX GEMMs' A operands):
// in_proj^T [128][384] | out_proj^T [128][128] | linear1^T [128][256] | linear2^T [256][128].
constexpr int kTWin = 0, kTWo = 3 * D * D, kTW1 = kTWo + D * D, kTW2 = kTW1 + FF * D;
constexpr int kLayerT = kTW2 + D * FF;  // 131072 floats per layer
// then head.0^T [128][64] of the actor and the critic head
constexpr int kHeadT = 3 * kLayerT;
constexpr int kPackedTFloats = kHeadT + 2 * D * HID;
// then the split copies of the three layers' transposed weights (the backward's dX GEMMs as split
// products): two fp16 planes per weight in split fragment order (policy_layout.hpp), at kTSplit +
// the weight's packedT offset
constexpr int kTSplit = kPackedTFloats;
constexpr int kPackedTAllFloats = kTSplit + kHeadT;
// The training kernels read the encoder GEMM weights only through their split copies (policy.hip
// kTrainSplit / kBwdSplit / kPsSplit): the trainer's fp32 fragment-order copies of those weights
// (packed at their kOffs slots, packedT below kHeadT) are dead. policy_pack_train fills them with
// NaN (a read would poison every output) and k_adam does not refresh them.
constexpr bool kTrainF32LayerCopies = false;

// flat parameters -> packed (forward) and packedT (backward) in one launch
int policy_pack_train(const float* flat, float* packed, float* packedT, hipStream_t st);
int policy_backward_train(const float* packed, const float* packedT, const BwdIO& io, int Bm, hipStream_t st);

// Launch the training-mode forward over Bm samples (multiple of 16) with fragment-order packed
// weights `packed` (uavhip_policy_pack) and trajectory windows `states` [n][5][14].
int policy_forward_train(const float* packed, const float* states, const TrainIO& io, int Bm, hipStream_t st);
// Trunk split: the per-workgroup loss partials from smp (k_loss_partials; the same terms and
// order as the fused forward's).
int policy_loss_partials(const TrainIO& io, int Bm, hipStream_t st);
// Position split (K7, policy.hip): small minibatches run every full encoder layer as one workgroup per
// (16-sample block, window position); partial rows per (block, position) = b * 5 + s, and kvc
// [Bm / 16 * 5][80][256] carries each query position's share of every position's dk / dv.
constexpr int kPsMaxBm = 256;
inline bool ps_capable(int Bm) { return Bm <= kPsMaxBm; }
int policy_forward_ps(const float* packed, const float* states, const TrainIO& io, int Bm, hipStream_t st);
int policy_backward_ps(const float* packed, const float* packedT, const BwdIO& io, float* kvc, int Bm, hipStream_t st);
// Whether a minibatch of Bm samples per step runs trunk-split (both trunks side by side on
// separate CUs): only while 2 Bm/16 workgroups fit one per CU.
inline bool trunk_split(int Bm) { return 2 * (Bm / 16) <= 256; }

}  // namespace pol
}  // namespace uavhip
