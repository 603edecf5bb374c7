// policy_layout.hpp -- parameter table of TransformerActorCritic (networks/transformer_net.py:67-144)
// shared by the rollout forward (policy.hip) and the PPO training step (train.hip): state_dict key
// order, sizes, float offsets (each parameter padded to a multiple of 4 floats) and which weights
// the rollout kernel keeps in MFMA fragment order.
#pragma once

namespace uavhip {
namespace pol {

constexpr int S = 5, D = 128, NH = 8, HD = 16, FF = 256, IN = 14, HID = 64;

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
// In-features K of the parameters stored in MFMA fragment order ([out][in] weights the kernel
// streams as the A operand: in_proj, out_proj, linear1, linear2 of every layer, head.0); 0 = plain.
// Fragment order of an [R][K] matrix: index ((r/16 * K/16 + k/16) * 64 + (r%16 + 16 * (k%16)/4)) * 4 + k%4.
constexpr int kTileK[kNumParams] = {
    0, 0, 0, D, 0, D, 0, D, 0, FF, 0, 0, 0, 0, 0,
    D, 0, 0, 0,
    0, 0, 0, D, 0, D, 0, D, 0, FF, 0, 0, 0, 0, 0,
    D, 0, D, 0, D, 0, FF, 0, 0, 0, 0, 0,
    D, 0, 0, 0};
constexpr int kActorTrunk = 0, kActorHead = 15, kCriticTrunk = 19, kCriticHead = 46;
enum { POS = 0, EMB_W = 1, EMB_B = 2 };
enum { INW = 0, INB, OUTW, OUTB, L1W, L1B, L2W, L2B, N1W, N1B, N2W, N2B };
__host__ __device__ constexpr int layer_param(int trunk, int l, int which) { return trunk + 3 + kLayerParams * l + which; }

// ---- split copies (inference forward only): the GEMM weights over all 80 tokens that run on the
// f16 matrix cores as fp32-accurate split products (policy.hip, hgemm_tile): the critic's layer-0
// out-projection and FFN, and its layer-1 in_proj (K / V of every token, Q of position 4); the
// layer-0 in_proj of both trunks for the rollout's window-row ring (the new row's Q | K | V); and the
// out-projection and FFN of both trunks' pruned top layers (the 16 tokens of position 4). Each weight
// W [R][K] is appended to the packed buffer as two fp16 planes, w1 = f16(w), w2 = f16((w - w1) 2^11),
// in split fragment order: per 16-row tile t and 32-k block kb, 1 KiB of plane 1 then 1 KiB of
// plane 2, lane l = r%16 + 16 ((k%32)/8) holding k%8 = 0..7 -- one float per weight, like the fp32
// copy. The split copies follow the 50 parameters.
constexpr int kNumSplit = 12;
constexpr int kSplitParam[kNumSplit] = {
    layer_param(kCriticTrunk, 0, L1W),  layer_param(kCriticTrunk, 0, L2W), layer_param(kCriticTrunk, 0, OUTW),
    layer_param(kCriticTrunk, 1, INW),  layer_param(kActorTrunk, 0, INW),  layer_param(kCriticTrunk, 0, INW),
    layer_param(kActorTrunk, 0, OUTW),  layer_param(kActorTrunk, 0, L1W),  layer_param(kActorTrunk, 0, L2W),
    layer_param(kCriticTrunk, 1, OUTW), layer_param(kCriticTrunk, 1, L1W), layer_param(kCriticTrunk, 1, L2W)};
struct SplitOffs { int o[kNumSplit + 1]; };
constexpr SplitOffs make_split_offs() {
    SplitOffs r{};
    int acc = kOffs.o[kNumParams];
    for (int i = 0; i < kNumSplit; ++i) { r.o[i] = acc; acc += kSizes[kSplitParam[i]]; }
    r.o[kNumSplit] = acc;
    return r;
}
constexpr SplitOffs kSplitOffs = make_split_offs();
constexpr int split_slot(int q) {
    for (int i = 0; i < kNumSplit; ++i)
        if (kSplitParam[i] == q) return kSplitOffs.o[i];
    return -1;
}

// ---- range table (DESIGN.md 4a "range"): after the split copies. The split products carry each
// activation operand as fp16 planes, exact to 2^-22 only for |x| in [2^-14, 65504], so every operand
// is multiplied by a power of two 2^-s before it is split and the consuming GEMM's output by 2^s
// (exact both ways: Y^T = W (2^-s X)^T 2^s). s comes from a rigorous bound B on the operand's
// magnitude: s = 0 while B is in [2^-4, 2^15) (every realistic weight set: the results are bitwise
// those without scaling), else B 2^-s lands in [2^14, 2^15), so no scaled value reaches fp16's
// overflow and the largest ones keep all 22 bits. The bounds (transformer_net.py's post-LN layers):
//   LayerNorm output  |x^ g + b| <= sqrt(D - 1) max|g| + max|b|            (|x^| <= sqrt(127))
//   FFN hidden        relu(W1 h + b1) <= D max|W1| B(h) + max|b1|
//   attention output  convex combination of V rows: <= D max|W_in| B(input) + max|b_in|
//   layer-0 input     e (+ pos) <= 14 max|W_e| max_k|x_k| + max|b_e| + max|pos| -- per token, from
//                     that token's window row (the kernels keep max_k|x_k| of every token in LDS)
// The packed buffer's table holds max|param| of every parameter (written by k_policy_range after a
// pack; after every update by k_adam, as atomic maxima) and zeros; each kernel derives the per-token
// constants of layer 0 and the (2^-s, 2^s) pairs of the operands whose bound depends on the weights
// alone from those maxima (range_entry: a few flops per entry, at kernel start), so a refresh is
// order-free and needs no second pass over the blocks' maxima. The host's range_derive fills the
// same entries into a full table (uavhip_policy_range_table).
constexpr int kRangeOff = kSplitOffs.o[kNumSplit];
constexpr int kRangeFloats = 96;
constexpr int kPackedFloats = kRangeOff + kRangeFloats;  // the inference forward's packed buffer
enum : int {
    kRgMax = 0,     // [q]: max |param q|, q < kNumParams
    kRgE = 52,      // + 2 t: 14 max|W_e|, + 2 t + 1: max|b_e| + max|pos| (trunk index t: 0 actor, 1 critic)
    kRgA0 = 56,     // + 2 t: D max|W_in(layer 0)|, + 2 t + 1: max|b_in(layer 0)|
    kRgOp = 64,     // + 2 op: 2^-s, + 2 op + 1: 2^s of static operand op
    kRgSpare = 84   // [kRgSpare, kRangeFloats): zero
};
// (in the packed buffer only the maxima [kRgMax, kRgMax + kNumParams) are stored; every other entry
// is what range_entry derives from them)
enum : int { kOpLn1 = 0, kOpHid = 1, kOpLn2 = 2, kOpAtt = 3 };  // static operand kinds
// static operand slot of (trunk, layer, kind): actor L0 {LN1 0, HID 1, LN2 8}; critic L0 {LN1 2,
// HID 3, LN2 4}; critic L1 {ATT 5, LN1 6, HID 7, LN2 9}; -1: not a static operand (layer 0's attention
// output, layer-0 input). The last layers' LN2 outputs (8, 9) are the heads' inputs: only the
// weight-gradient GEMM splits them (the heads run on the f32 MFMA).
__host__ __device__ constexpr int range_op(int trunk, int layer, int kind) {
    return trunk == kActorTrunk ? (layer == 0 && kind <= kOpHid ? kind : layer == 0 && kind == kOpLn2 ? 8 : -1)
           : layer == 0         ? (kind <= kOpLn2 ? 2 + kind : -1)
           : layer == 1         ? (kind == kOpAtt ? 5 : kind <= kOpHid ? 6 + kind : kind == kOpLn2 ? 9 : -1)
                                : -1;
}
constexpr int kNumRangeOps = 10;
static_assert(kRgOp + 2 * kNumRangeOps <= kRgSpare && kRgSpare <= kRangeFloats && kNumParams <= kRgE, "range table");
__host__ __device__ constexpr int trunk_index(int trunk) { return trunk == kActorTrunk ? 0 : 1; }
// The scales a kernel derives at start (policy.hip load_rtab -> Smem::rtab; the training forward
// exports them, TrainIO::rtab_out, for the weight-gradient GEMM): the static operands' (2^-s, 2^s)
// pairs, then layer 0's (14 max|W_e|, max|b_e| + max|pos|) and (D max|W_in|, max|b_in|) per trunk
constexpr int kRtOp = 0, kRtE = 2 * kNumRangeOps, kRtA0 = kRtE + 4, kRtN = kRtA0 + 4;

// The scale exponent of an operand bounded by B: 0 for B in [2^-4, 2^15) (and for 0 and NaN: a
// non-finite operand stays non-finite), else B 2^-s in [2^14, 2^15). frexp: B = f 2^e, f in [0.5, 1).
// A bound that overflowed fp32 (inf, or >= 2^115: the bounds are products of maxima and can overflow
// while the activations they bound stay finite) takes the largest exponent any finite fp32 operand
// needs, s = 113 (2^128 2^-113 = 2^15), instead of turning the scaling off; tiny bounds
// stop at s = -100. Weights are not range-scaled: their split copies hold f16(w), so a weight of
// 65520 or more is inf in the split products (non-finite outputs, never silently wrong;
// uavhip_policy_range_table reports max |param| for a caller that wants to check).
__host__ __device__ inline int range_exp(float B) {
    if (!(B > 0.f)) return 0;
    if (!(B < 0x1p115f)) return 113;
    int e = 0;
    (void)frexpf(B, &e);
    if (e >= -3 && e <= 15) return 0;
    const int s = e - 15;
    return s < -100 ? -100 : s;
}
// The bound of static operand op (range_op's numbering) from M = max|param q| (table[kRgMax ..]).
__host__ __device__ inline float range_bound(const float* M, int op) {
#pragma clang fp contract(off)
    constexpr float kLnMax = 11.5f;  // >= sqrt(D - 1): the largest |x^| of a D-feature LayerNorm
    const int tr = op < 2 || op == 8 ? kActorTrunk : kCriticTrunk, l = op < 5 || op == 8 ? 0 : 1;
    auto ln = [&](int layer, int w) { return kLnMax * M[layer_param(tr, layer, w)] + M[layer_param(tr, layer, w + 1)]; };
    auto hid = [&](int layer) {
        return (float)D * M[layer_param(tr, layer, L1W)] * ln(layer, N1W) + M[layer_param(tr, layer, L1B)];
    };
    switch (op) {
        case 0: case 2: case 6: return ln(l, N1W);     // LN1 outputs
        case 1: case 3: case 7: return hid(l);         // FFN hidden units
        case 4: case 8: return ln(0, N2W);             // layer-0 LN2 outputs (critic: layer 1's input)
        case 9: return ln(1, N2W);                     // the critic's layer-1 LN2 output
        default:                                       // 5: the critic's layer-1 attention output
            return (float)D * M[layer_param(tr, 1, INW)] * ln(0, N2W) + M[layer_param(tr, 1, INB)];
    }
}
// Derived entry k (kRgE <= k < kRangeFloats; 0 for the spare slots) from M. Host (range_derive:
// uavhip_policy_range_table) and device (load_rtab and the layer-0 constants of the forward
// kernels) evaluate the same fp32 operations without contraction: bitwise the same entries.
__host__ __device__ inline float range_entry(const float* M, int k) {
#pragma clang fp contract(off)
    if (k >= kRgE && k < kRgE + 4) {
        const int tr = k < kRgE + 2 ? kActorTrunk : kCriticTrunk;
        return (k & 1) ? M[tr + EMB_B] + M[tr + POS] : (float)IN * M[tr + EMB_W];
    }
    if (k >= kRgA0 && k < kRgA0 + 4) {
        const int tr = k < kRgA0 + 2 ? kActorTrunk : kCriticTrunk;
        return (k & 1) ? M[layer_param(tr, 0, INB)] : (float)D * M[layer_param(tr, 0, INW)];
    }
    if (k >= kRgOp && k < kRgOp + 2 * kNumRangeOps) {
        const int s = range_exp(range_bound(M, (k - kRgOp) >> 1));
        return ldexpf(1.0f, (k & 1) ? s : -s);
    }
    return 0.f;
}
static_assert(kRgE % 2 == 0 && kRgA0 % 2 == 0 && kRgOp % 2 == 0, "entry pairs start at even slots");
// table[kRgMax + q] (max|param q|) -> every derived entry (the host's table)
__host__ __device__ inline void range_derive(float* t) {
    for (int k = kRgE; k < kRangeFloats; ++k) t[k] = range_entry(t + kRgMax, k);
}

}  // namespace pol
}  // namespace uavhip
