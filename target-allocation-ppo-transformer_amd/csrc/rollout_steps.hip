// rollout_steps.hip -- k_rollout_steps (uavhip_rollout_steps): policy.hip's fused rollout step in a
// loop over the steps of one launch, compiled in a translation unit of its own so that every
// lane-index expression can be laundered per use (UAVHIP_TID_LAUNDER, common.hpp tid_x()) without
// touching the code of the single-step kernels.
#define UAVHIP_STEPS_TU 1
#define UAVHIP_TID_LAUNDER 1
#include "policy.hip"
