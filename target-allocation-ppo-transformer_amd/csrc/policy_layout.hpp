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
constexpr int kPackedFloats = kSplitOffs.o[kNumSplit];  // the inference forward's packed buffer
constexpr int split_slot(int q) {
    for (int i = 0; i < kNumSplit; ++i)
        if (kSplitParam[i] == q) return kSplitOffs.o[i];
    return -1;
}

}  // namespace pol
}  // namespace uavhip
