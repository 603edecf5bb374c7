// policy_train.hpp -- the training-mode view of the fused policy forward (policy.hip): the same
// kernel, instantiated with TR = true, gathers a minibatch of windows by row index and writes every
// activation the PPO backward (train.hip) reads, in its [row = b * 5 + s][feature] layout
// (pruned layers' tails as compact [b][feature] rows). Heads and sampling are skipped.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
    float *e[2], *h0[2];         // [R][128] actor, critic embeddings (post-ReLU) and layer inputs
    TrainLayerIO L[3];           // actor L0 (pruned), critic L0 (full), critic L1 (pruned)
};

// Launch the training-mode forward over Bm samples (multiple of 16) with fragment-order packed
// weights `packed` (uavhip_policy_pack) and trajectory windows `states` [n][5][14].
int policy_forward_train(const float* packed, const float* states, const TrainIO& io, int Bm, hipStream_t st);

}  // namespace pol
}  // namespace uavhip
