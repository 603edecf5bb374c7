/*
 * uavhip.h -- C ABI of libuavhip.so, the MI355X (gfx950) implementation of the PPO rollout
 * hot path of the UAV->target allocation reference (envs/uav_env.py, envs/mechanics.py,
 * networks/transformer_net.py, agents/ppo.py).
 *
 * The reference has no FFI layer: its boundary is the Python object API that main_train.py
 * calls (UAVEnv.reset/step, PPOAgent.select_action/store_transition/update). Each entry point
 * below replaces one piece of that API; the Python mirror in
 * target-allocation-ppo-transformer_amd/uavhip binds them with ctypes.
 *
 * Conventions
 *  - every pointer is CALLER-OWNED DEVICE memory (torch tensors), except the `const
 *    uavhip_env*` / `const uavhip_policy*` descriptors themselves, which live on the host and are
 *    copied into the launch; the library never allocates or frees on the hot path;
 *  - every call is asynchronous on `stream` (a hipStream_t; NULL = the legacy default stream)
 *    and never synchronises the device;
 *  - return 0 on success, a negative UAVHIP_E* code otherwise; uavhip_last_error() returns a
 *    thread-local message. No C++ exception crosses this boundary;
 *  - layouts are row-major, env index outermost ("[E][N][M]" = e*N*M + u*M + t).
 */
#ifndef UAVHIP_H
#define UAVHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* uavhip_stream_t; /* hipStream_t */

#define UAVHIP_SEQ_LEN 5    /* config.py:62 SEQ_LEN    */
#define UAVHIP_STATE_DIM 14 /* config.py:61 STATE_DIM  */
#define UAVHIP_OBS_FLOATS (UAVHIP_SEQ_LEN * UAVHIP_STATE_DIM)
#define UAVHIP_MAX_N 64     /* UAVs per env (one wave lane each)          */
#define UAVHIP_MAX_M 128    /* targets per env (<= 2 per wave lane)       */
#define UAVHIP_MAX_OBSTACLES 8
/* uavhip_env.flags */
#define UAVHIP_ENV_ONE_PER_WAVE 1  /* multi-step launches: never pack two envs into one wave */
#define UAVHIP_ENV_OBS_F16 2       /* obs_out of uavhip_env_reset / uavhip_env_step is IEEE binary16
                                      (round-to-nearest-even of the f32 window; BASELINE config 4)
                                      instead of f32; the env's own window stays f32          */
#define UAVHIP_ENV_NO_REPLAY 4     /* multi-step launches: never use the omega = 0 replay kernel
                                      (K2r, env_replay.hpp), always the step-by-step K2 / K2g.
                                      K2r assumes every tentative assign is accepted, which
                                      omega = 0 guarantees only when every target value is >= 0
                                      (J can then never drop, uav_env.py:317-338; pair
                                      probabilities are clipped to [0, 1] by construction). The
                                      generators never make a negative value; a caller loading
                                      host scenes that may must set this flag (VecUAVEnv.
                                      load_scenes does it).                                      */

enum uavhip_status {
    UAVHIP_OK = 0,
    UAVHIP_EINVAL = -1, /* bad argument / shape */
    UAVHIP_EHIP = -2,   /* HIP launch or runtime error */
};

/* Physics constants (config.py:7-12,53 / config0.py), passed by value. */
enum uavhip_param {
    UAVHIP_PRM_ZETA_D = 0, /* PARAM_ZETA_D, target distance scale (150)        */
    UAVHIP_PRM_K,          /* PARAM_K, speed ratio weight (1.2; 5.0 in config0)  */
    UAVHIP_PRM_C1,         /* PARAM_C1 */
    UAVHIP_PRM_C2,         /* PARAM_C2 */
    UAVHIP_PRM_C3,         /* PARAM_C3 */
    UAVHIP_PRM_C4,         /* PARAM_C4 */
    UAVHIP_PRM_OMEGA,      /* COST_WEIGHT_OMEGA */
    UAVHIP_PRM_ZETA_OBS,   /* obstacle distance scale, 10 (mechanics.py:79)      */
    UAVHIP_PRM_COUNT
};

/* On-device scene generator ranges (uav_env.py:65-173). */
enum uavhip_gen {
    UAVHIP_GEN_UAV_X0 = 0, UAVHIP_GEN_UAV_X1, /* UAV_GEN_X_RANGE            */
    UAVHIP_GEN_TGT_X0, UAVHIP_GEN_TGT_X1,     /* TARGET_GEN_X_RANGE         */
    UAVHIP_GEN_MAP_H,                         /* MAP_HEIGHT                 */
    UAVHIP_GEN_WEATHER_SPEED,                 /* WEATHER_SPEED_FACTOR       */
    UAVHIP_GEN_WEATHER_LOAD,                  /* WEATHER_LOAD_FACTOR        */
    UAVHIP_GEN_NFZ_X0, UAVHIP_GEN_NFZ_X1,     /* 120, 140 (uav_env.py:150)  */
    UAVHIP_GEN_ICP_X0, UAVHIP_GEN_ICP_X1,     /* 140, 160 (uav_env.py:160)  */
    UAVHIP_GEN_ICP_S0, UAVHIP_GEN_ICP_S1,     /* 0.30, 0.32 (uav_env.py:164)*/
    UAVHIP_GEN_COUNT = 16
};

/* Per-step diagnostics (uav_env.py:426-433 `info`), one row of doubles per env-step. */
enum uavhip_info {
    UAVHIP_INFO_J = 0,          /* J_val after the action (_calc_J_X)               */
    UAVHIP_INFO_NUM_ASSIGNED,   /* num_assigned = N0, covered targets                */
    UAVHIP_INFO_IS_VALID,       /* is_valid_action: 1/0, or -1 for None (action 0)   */
    UAVHIP_INFO_AVG_P_DMG,      /* avg_p_dmg over locked pairs                       */
    UAVHIP_INFO_AVG_P_FINAL,    /* avg_p_final over locked pairs                     */
    UAVHIP_INFO_UAV_IDX,        /* pointer after the action (before any auto-reset)  */
    UAVHIP_INFO_TARGET_IDX,
    UAVHIP_INFO_EPISODE,        /* 1-based episode index the step belonged to        */
    UAVHIP_INFO_COUNT
};

/* Integer per-env scalars, istate[E][UAVHIP_IST_COUNT]. */
enum uavhip_ist {
    UAVHIP_IST_UAV_IDX = 0, /* uav_env.py:33 self.uav_idx    */
    UAVHIP_IST_TARGET_IDX,  /* uav_env.py:34 self.target_idx */
    UAVHIP_IST_N_COVERED,   /* N0: targets with >= 1 lock    */
    UAVHIP_IST_N_ASSIGNED,  /* locked (uav, target) pairs    */
    UAVHIP_IST_EPISODE,     /* 1-based episode counter (main_train.py:77-79 cadence) */
    UAVHIP_IST_ERROR,       /* bit 0: a finished env was stepped without auto-reset;
                               bit 1: a full reset found no fresh spare scene (state-only reset done) */
    UAVHIP_IST_SCENE_SEL,   /* active scene buffer (0/1) when scene_buffers == 2 */
    UAVHIP_IST_SCENE_STALE, /* 1: the spare buffer still holds a used scene (uavhip_scene_refresh) */
    UAVHIP_IST_SCENE_GEN,   /* number of on-device scenes generated for this env (Philox counter) */
    UAVHIP_IST_PAD0, UAVHIP_IST_PAD1, UAVHIP_IST_PAD2,
    UAVHIP_IST_COUNT
};

/* Float64 per-env scalars, dstate[E][UAVHIP_DST_COUNT]. */
enum uavhip_dst {
    UAVHIP_DST_R = 0,      /* cached r(X) (_calculate_paper_reward of the current state) */
    UAVHIP_DST_J,          /* cached J(X)                                                */
    UAVHIP_DST_ASG_COST,   /* sum of costs of unavailable UAVs (chi_c numerator)         */
    UAVHIP_DST_COV_VALUE,  /* sum of values of covered targets (chi_v numerator)         */
    UAVHIP_DST_TOTAL_COST, /* total_swarm_cost (uav_env.py:118)                          */
    UAVHIP_DST_TOTAL_VALUE,/* sum of target values                                       */
    UAVHIP_DST_PD_CUR,     /* p_dmg of the current pointer pair (cached: no dependent load) */
    UAVHIP_DST_SUM_PDMG,   /* sum of p_dmg over locked pairs, in lock order (info avg_p_dmg)     */
    UAVHIP_DST_SUM_PFIN,   /* sum of p_final over locked pairs, in lock order (info avg_p_final) */
    UAVHIP_DST_PAD0, UAVHIP_DST_PAD1, UAVHIP_DST_PAD2,
    UAVHIP_DST_COUNT
};

/*
 * Vectorised env descriptor: E independent copies of UAVEnv (envs/uav_env.py:13) in SoA device
 * tensors. Replaces the Python objects `self.uavs / self.targets / self.nfz_list /
 * self.interceptors` (records of envs/entities.py:13-61) and the pointer/lock state.
 */
typedef struct uavhip_env {
    int32_t E, N, M, Kn, Ki;
    int32_t full_reset_period; /* auto-reset: switch to a fresh scene when episode % period == 0
                                  (200 in main_train.py:79); 0 = state-only resets. Needs
                                  scene_buffers == 2.                                         */
    int32_t scene_buffers;     /* 1, or 2 = every scene array and pair table below is
                                  [2][E]...: buffer istate[SCENE_SEL] is active, the other a
                                  pre-generated spare a full reset flips to                  */
    int32_t flags;              /* UAVHIP_ENV_* bits (0 = defaults)                    */
    uint64_t seed;             /* Philox key for on-device scene generation                 */
    uint64_t env_base;         /* global index of env 0: scene counters run on env_base + e, so
                                  a rank's shard [env_base, env_base + E) draws the scenes the
                                  same envs draw in one process over the union (0 on one GPU) */
    double prm[UAVHIP_PRM_COUNT];
    double gen[UAVHIP_GEN_COUNT];
    /* scene: entities.py records as SoA */
    double* uav_pos;   /* [E][N][2]  UAV.pos                                  */
    double* uav_vel;   /* [E][N][2]  UAV.velocity                             */
    double* uav_load;  /* [E][N]     UAV.load (weather-scaled)                */
    double* uav_cost;  /* [E][N]     UAV.cost (1.0 / 1.25)                    */
    int32_t* uav_type; /* [E][N]     UAV.uav_type                             */
    double* tgt_pos;   /* [E][M][2]  Target.pos, in LIST order (post-shuffle) */
    double* tgt_vel;   /* [E][M][2]  Target.velocity                          */
    double* tgt_value; /* [E][M]     Target.value                             */
    int32_t* tgt_id;   /* [E][M]     Target.id (pre-shuffle index)            */
    double* nfz_pos;   /* [E][Kn][2] NoFlyZone.pos                            */
    double* icp_pos;   /* [E][Ki][2] Interceptor.pos                          */
    double* icp_vel;   /* [E][Ki][2] Interceptor.velocity                     */
    /* pair tables (uavhip_score_pairs output) */
    double* p_dmg;     /* [E][N][M]  calc_damage_prob (mechanics.py:93)        */
    double* p_pen;     /* [E][N]     calc_penetration_prob (mechanics.py:118) */
    /* dynamic state */
    double* nh_final;  /* [E][M] prod over lockers of (1 - p_final), lock order  */
    double* nh_pure;   /* [E][M] prod over lockers of (1 - p_dmg)               */
    double* t_cost;    /* [E][M] sum of locker costs, lock order                */
    int32_t* n_lock;   /* [E][M] number of lockers                              */
    int32_t* assigned; /* [E][N] target LIST index or -1 (id = tgt_id[..])       */
    int32_t* istate;   /* [E][UAVHIP_IST_COUNT]                                */
    double* dstate;    /* [E][UAVHIP_DST_COUNT]                                */
    float* window;     /* [E][5][14] state_buffer deque (uav_env.py:37)        */
} uavhip_env;

/* ---------------------------------------------------------------- env (K1, K2, reset, gen) */

/* K1. Dense pair tables p_dmg[E][N][M], p_pen[E][N] of the ACTIVE scene buffer from the scene
 * arrays, for the envs with mask[e] != 0 (mask NULL = all). Replaces calc_advantage's per-call recomputation
 * (mechanics.py:93-181; called ~42x per env step by uav_env.py:184-435). */
int uavhip_score_pairs(const uavhip_env* env, const uint8_t* mask, uavhip_stream_t stream);

/* Philox4x32-10 scene generation on device (distribution of uav_env.py:65-173, not its
 * MT19937 stream) into the ACTIVE buffer of masked envs (and the spare, when scene_buffers == 2),
 * followed by K1 for them; the counter is (env, istate[SCENE_GEN]). */
int uavhip_scene_generate(const uavhip_env* env, const uint8_t* mask, uavhip_stream_t stream);

/* Regenerate (Philox + K1) the spare scene buffer of every env whose istate[SCENE_STALE] is set,
 * i.e. that flipped to its spare at a full reset. Call once per rollout iteration (full resets
 * are >= full_reset_period episodes apart). No-op unless scene_buffers == 2. */
int uavhip_scene_refresh(const uavhip_env* env, uavhip_stream_t stream);

/* UAVEnv.reset(full_reset=False) (uav_env.py:42-63,175-182) for masked envs: clears the
 * allocation, recomputes the scene totals, writes the first window to obs_out[E][5][14]
 * (nullable). episode >= 0 sets istate[EPISODE]; < 0 leaves it. */
int uavhip_env_reset(const uavhip_env* env, const uint8_t* mask, int32_t episode, float* obs_out,
                     uavhip_stream_t stream);

/* K2. UAVEnv.step (uav_env.py:295-435) for all E envs, T consecutive steps fused in one launch
 * (T = 1 for the per-step rollout). actions: int8 [T][E] (0 skip, 1 assign). Outputs (each
 * nullable): obs_out [T][E][5][14] f32, reward [T][E] f64, done [T][E] u8,
 * info [T][E][UAVHIP_INFO_COUNT] f64.
 * auto_reset != 0: a finished env is reset in-kernel (state-only, or a fresh on-device scene
 * every full_reset_period episodes) and obs_out carries the NEW episode's first window;
 * auto_reset == 0: obs_out is all zeros for a finished env (the reference returns zeros(14),
 * uav_env.py:188-189) and stepping it again only sets istate[ERROR]. */
int uavhip_env_step(const uavhip_env* env, const int8_t* actions, int32_t T, int32_t auto_reset,
                    float* obs_out, double* reward, uint8_t* done, double* info, uavhip_stream_t stream);

/* ---------------------------------------------------------------- PPO reductions (K3) */

/* GAE over a time-major [T][E] buffer (agents/ppo.py:70-91, fp32 arithmetic in the reference's
 * op order): next_v = v[t+1] (t < T-1) or last_value[e] (NULL -> 0, the reference's value at
 * an episode end); done zeroes the bootstrap and the carry. Writes returns and raw advantages
 * (returns - values), and per-block (sum, sum of squares) partials of the advantages to
 * partials[2 * uavhip_gae_partials(T, E)] (nullable) for uavhip_adv_normalize. */
int uavhip_gae(const double* reward, const uint8_t* done, const float* value, const float* last_value,
               int32_t T, int32_t E, double gamma, double lam, float* ret, float* adv, double* partials,
               uavhip_stream_t stream);
int32_t uavhip_gae_partials(int32_t T, int32_t E);

/* fp64 (sum, sum of squares) partials of adv[n] into partials[2 * n_partials] (one per block),
 * for buffers that did not come out of uavhip_gae. */
int uavhip_adv_partials(const float* adv, int64_t n, double* partials, int32_t n_partials, uavhip_stream_t stream);

/* adv <- (adv - mean) / (std_unbiased + 1e-7) over n elements (ppo.py:94), mean/std folded in
 * fp64 from partials[2 * n_partials] (uavhip_gae or uavhip_adv_partials) in a fixed order, then
 * rounded to fp32 as the reference's fp32 tensors are. n_total = element count the partials
 * describe (0 -> n); with data-parallel ranks pass all-reduced partials and the global count so
 * every rank normalises with the statistics of the whole gathered batch. stats_out[2] =
 * {mean, std} (nullable, device f64). */
int uavhip_adv_normalize(float* adv, int64_t n, const double* partials, int32_t n_partials, int64_t n_total,
                         double* stats_out, uavhip_stream_t stream);

/* Policy-input windows [blocks][T][E][5][14] of a trajectory from its compact all-gather form
 * (uavhip/dist.py pack_compact; the data-parallel exchange of SURVEY.md 8e): per block, first
 * windows first[e][70] (the window at step 0), rows[t][e][14] (the row pushed at step t = window
 * slot 4; row 0 is read from the first window) and done flags done[(t * E + e) * done_stride] (f32,
 * nonzero = the episode ended at step t, so step t + 1 starts from a zero window,
 * uav_env.py:42-63,241-242). Blocks are block_stride floats apart in all three arrays (one rank's
 * payload each). Replaces shipping 70 window floats per transition in the gather: the deque only
 * shifts, so a window is the last 5 rows of its episode. */
int uavhip_windows_from_rows(const float* first, const float* rows, const float* done, int32_t done_stride,
                             int64_t block_stride, int32_t blocks, int32_t T, int32_t E, float* out,
                             uavhip_stream_t stream);

/* ---------------------------------------------------------------- policy forward (K4) */

/* Packed fp32 weights of TransformerActorCritic (transformer_net.py:67-144), produced by
 * uavhip/policy.py pack_weights() from the 50-key state_dict: each parameter at its
 * uavhip_policy_layout() offset, flat or in MFMA fragment order (uavhip_policy_tiling()). */
typedef struct uavhip_policy {
    const float* weights; /* packed buffer, layout = uavhip_policy_layout() offsets + split copies */
                          /* (n_floats = uavhip_policy_split_layout()) */
    int32_t n_floats;
    int32_t d_model, n_heads, d_ff, d_head_hidden; /* 128, 8, 256, 64 */
    int32_t actor_layers, critic_layers;           /* 1, 2 */
} uavhip_policy;

/* Offsets (in floats) of every parameter in the packed buffer, in state_dict key order
 * (see policy.py). Returns the total number of floats; offsets may be NULL. */
int32_t uavhip_policy_layout(int32_t* offsets, int32_t max_offsets);

/* The inference forward's packed buffer (uavhip_policy.weights / n_floats) holds, after the
 * uavhip_policy_layout() parameters, split copies of the GEMM weights that run on the f16 matrix
 * cores as fp32-accurate split products: weight `params[i]` (state_dict index, [R][K]) at float
 * offset `offsets[i]`, as two fp16 planes w1 = f16(w), w2 = f16((w - w1) * 2^11) in split fragment
 * order (blocks of 16 rows x 32 k: 1 KiB of w1 then 1 KiB of w2, lane = r%16 + 16 ((k%32)/8)
 * holding k%8 = 0..7). Returns the packed buffer's total floats; params / offsets may be NULL. */
int32_t uavhip_policy_split_layout(int32_t* params, int32_t* offsets, int32_t max_entries);

/* flat (state_dict order, uavhip_policy_layout offsets, every parameter row-major) -> packed
 * (the same with the uavhip_policy_tiling weights in MFMA fragment order, the split copies and the
 * range table), on the device. */
int uavhip_policy_pack(const float* flat, float* packed, uavhip_stream_t stream);

/* The range table that ends the packed buffer (its last n floats, n = the return value): the
 * split products multiply every activation operand by a power of two 2^-s before splitting it into
 * fp16 planes and the GEMM output by 2^s, with s from a rigorous bound on the operand's magnitude
 * (0 on realistic weights), so no ACTIVATION operand the reference's fp32 can hold leaves fp16's
 * range (a bound that overflows fp32 takes the largest exponent, s = 113). The weights themselves
 * are not scaled: their split copies hold f16(w), so a parameter of magnitude >= 65520 makes the
 * outputs non-finite (never silently wrong); max_abs is the caller's check for that.
 * The packed buffer's table holds the maxima (max |param| of each state_dict tensor, floats 0..49;
 * the rest zero; uavhip_policy_pack writes them, an UPDATE step refreshes them) and every kernel
 * derives the scales from them. NaN elements do not count in a maximum (the device reduces with
 * fmaxf; the ctypes mirror drops them the same way), so host and device tables agree for any
 * parameters. Host side: max_abs[50] (key order) -> table[n]: the maxima, the
 * per-token constants of layer 0 and the static operands' (2^-s, 2^s) pairs -- bitwise what the
 * kernels derive. Either pointer NULL: only returns n. */
int32_t uavhip_policy_range_table(const float* max_abs, float* table);

/* Per parameter (state_dict key order): the in-features K of the weight matrices stored in MFMA
 * fragment order, 0 for parameters stored flat. An [R][K] matrix W in fragment order puts
 * W[r][k] at ((r/16 * K/16 + k/16) * 64 + r%16 + 16 * ((k%16)/4)) * 4 + k%4, so each 16 x 16
 * block the kernel streams is 1 KiB contiguous. Returns the number of parameters (50). */
int32_t uavhip_policy_tiling(int32_t* kcols, int32_t max_params);

/* get_action / evaluate (transformer_net.py:96-144) for B windows states[B][5][14]:
 * actions_in NULL -> sample a ~ Categorical(softmax(logits)) with Philox(seed, c), counter
 * c = offset + (offset_dev ? *offset_dev : 0) + b (offset_dev: device u64, lets a captured
 * hipGraph draw fresh numbers on every replay); else evaluate the given actions. Outputs
 * (nullable): action_out [B] int8, logp [B], value [B], entropy [B], logits [B][2] (all f32). */
int uavhip_policy_forward(const uavhip_policy* policy, const float* states, int32_t B, const int8_t* actions_in,
                          uint64_t seed, uint64_t offset, const uint64_t* offset_dev, int8_t* action_out,
                          float* logp, float* value, float* entropy, float* logits, uavhip_stream_t stream);

/* Rollout fast path of uavhip_policy_forward for a SEQUENCE of windows in which window g + 1 is
 * window g shifted by one row plus a new last row (the observation deque, uav_env.py:241-242;
 * after an episode end the earlier rows are zero padding). rowproj (caller-owned, size
 * uavhip_policy_rowproj_floats(B)) keeps, per window, the layer-0 in_proj of the embeddings of
 * its rows (a 5-slot ring indexed by step mod 5) and Win . pos of both trunks, so the forward of
 * step g projects only the new row (transformer_net.py:57-63 is linear up to the in_proj after
 * the embedding ReLU). step = g (>= 0, +1 per call along the sequence); fill != 0 rebuilds rows
 * 0-3 and the pos table from states and the current weights: required on the first call, after
 * the weights change, and whenever states is not the previous call's window advanced by one
 * row. Outputs as uavhip_policy_forward, equal to it within fp32 rounding (Win (e + pos) + b is
 * evaluated as (Win e + b) + Win pos). */
int64_t uavhip_policy_rowproj_floats(int32_t B);
int uavhip_policy_forward_rows(const uavhip_policy* policy, const float* states, int32_t B, float* rowproj,
                               int32_t step, int32_t fill, const int8_t* actions_in, uint64_t seed, uint64_t offset,
                               const uint64_t* offset_dev, int8_t* action_out, float* logp, float* value,
                               float* entropy, float* logits, uavhip_stream_t stream);

/* The value head alone on the window-row ring (the rollout's bootstrap V(s_T) after the last step,
 * ppo.py:70-94's next value): uavhip_policy_forward_rows' value output, bitwise, from the critic
 * trunk and head only (no actor trunk, no sampling: about 2/3 of the forward). The actor's ring row
 * of this step is not written, so the next call on the sequence must pass fill != 0. */
int uavhip_policy_value_rows(const uavhip_policy* policy, const float* states, int32_t B, float* rowproj,
                             int32_t step, int32_t fill, float* value, uavhip_stream_t stream);

/* One rollout step in ONE launch (main_train.py:109-117: select_action, then env.step): the
 * window-row forward of uavhip_policy_forward_rows with sampling, followed in the same
 * workgroups by the env step (uavhip_env_step, T = 1) of env e with the action sampled for
 * window b = e. B = env->E; the same outputs as the two calls in sequence, bitwise: action_out,
 * logp, value [E] of the forward, obs_out [E][5][14] (the next windows; f32, or binary16 under
 * UAVHIP_ENV_OBS_F16), reward [E], done [E], info [E][UAVHIP_INFO_COUNT] (nullable) of the step.
 * Needs N, M <= 64 (one env per wave). Saves the T = 1 env launch's fixed cost (dispatch, the
 * state-load round, the store drain: ~7 of its ~10 us at 4096 envs). */
int uavhip_rollout_step(const uavhip_policy* policy, const uavhip_env* env, const float* states, float* rowproj,
                        int32_t step, int32_t fill, uint64_t seed, uint64_t offset, const uint64_t* offset_dev,
                        int8_t* action_out, float* logp, float* value, int32_t auto_reset, float* obs_out,
                        double* reward, uint8_t* done, double* info, uavhip_stream_t stream);

/* n consecutive rollout steps in ONE launch (main_train.py:109-117 repeated n times): step t runs
 * uavhip_rollout_step on windows obs[t] with ring step `step` + t and sampling counters
 * offset + t * offset_stride + b, writing actions / logp / value / reward / done [t][E], info
 * [t][E][UAVHIP_INFO_COUNT] (nullable) and the next windows obs[t + 1]. obs is the time-major
 * [n + 1][E][5][14] f32 trajectory buffer (obs[0] = the current windows). Bitwise equal to n
 * uavhip_rollout_step calls. Every workgroup loops over the steps of its own 16 envs, so no
 * grid-wide synchronisation is involved; saves the per-launch tail and start-up of n - 1
 * launches. N, M <= 64; f32 observations (no UAVHIP_ENV_OBS_F16). */
int uavhip_rollout_steps(const uavhip_policy* policy, const uavhip_env* env, float* obs, float* rowproj,
                         int32_t step, int32_t n, int32_t fill, uint64_t seed, uint64_t offset,
                         uint64_t offset_stride, const uint64_t* offset_dev, int8_t* actions, float* logp,
                         float* value, int32_t auto_reset, double* reward, uint8_t* done, double* info,
                         uavhip_stream_t stream);

/* ---------------------------------------------------------------- PPO update (K5) */

/* One clipped-PPO minibatch step of agents/ppo.py:96-169 (evaluate -> surrogate / clipped value
 * / entropy loss -> backward -> clip_grad_norm_(1.0) -> Adam with the four parameter groups of
 * ppo.py:17-22), as hand-written kernels: fp32-accurate split-product GEMMs on the f16 MFMA for the
 * encoder layers (forward / input gradients two-plane, weight gradients three-plane) and f32 MFMA
 * GEMMs for the embeddings and heads
 * (forward, input gradients, split-K weight gradients), fused residual+LayerNorm, attention,
 * heads+loss, and a fused clip+Adam. Parameters, gradients and the Adam moments are FLAT
 * buffers in the plain (not fragment-order) uavhip_policy_layout() layout; the torch module's
 * parameters can be views of `params`. */
typedef struct uavhip_ppo {
    float* params;       /* [n_floats] */
    float* grads;        /* [n_floats] this rank's gradient contribution (written by BACKWARD) */
    float* adam_m;       /* [n_floats] exp_avg */
    float* adam_v;       /* [n_floats] exp_avg_sq */
    double* adam_step;   /* [1] device step counter (shared by all groups) */
    float* workspace;    /* [uavhip_ppo_workspace_floats(minibatch)], zero-filled before first use */
    float* loss_sums;    /* [4] written by FORWARD: sums over this rank's samples of min(s1, s2),
                            (v - R)^2, (v_clip - R)^2, entropy; BACKWARD reads them (all-reduced);
                            FORWARD | BACKWARD in one call: summed and written by the backward */
    double* stats;       /* [4] += loss_actor, loss_critic, entropy, 1 per step (nullable) */
    int32_t n_floats;
    int32_t minibatch;   /* samples per step on this rank, multiple of 64 */
    int32_t global_minibatch; /* samples per step over all ranks (0: = minibatch) */
    /* torch.optim.Adam's hyper-parameters as torch holds them (Python floats = doubles): the bias
       corrections and step size are formed in double and the per-element coefficients rounded to
       float once, as torch's single-tensor Adam does -- its path for CPU tensors, where the reference's
       fixtures were recorded (agents/ppo.py:17-22); torch's CUDA default (foreach) differs by one
       rounding per element (train.hip k_adam) */
    double lr_actor, lr_critic, beta1, beta2, adam_eps; /* 2e-4, 1e-3, 0.9, 0.999, 1e-8 */
    float eps_clip, max_grad_norm, value_coef, entropy_coef; /* 0.2, 1.0, 0.5, 0.01 */
} uavhip_ppo;

/* uavhip_ppo_step phases (bit mask). A data-parallel step over R ranks runs FORWARD,
 * all-reduces loss_sums (sum), runs BACKWARD (gradients scaled by 1 / global_minibatch, so their
 * sum over ranks is the global minibatch's gradient), all-reduces grads (sum), runs UPDATE. */
enum uavhip_ppo_phase {
    UAVHIP_PPO_FORWARD = 1,
    UAVHIP_PPO_BACKWARD = 2,
    UAVHIP_PPO_UPDATE = 4,   /* clip_grad_norm_ on grads + Adam */
    UAVHIP_PPO_FULL = 7,
    UAVHIP_PPO_PACKED = 8    /* with FORWARD: the workspace's packed weight copies are current (an
                                UPDATE on this workspace refreshes them with the new parameters,
                                and nothing changed the parameters since): skip the repack */
};

/* Floats of workspace one step needs at `minibatch` samples. */
int64_t uavhip_ppo_workspace_floats(int32_t minibatch);

/* Minibatch rows idx[minibatch] (int32, into the trajectory buffers) of states[n][5][14],
 * actions[n] (int8), old_logp / old_values / returns / advantages [n] (f32); idx[i] < 0 marks a
 * padding row that adds nothing to loss_sums or grads (a rank's share of a global minibatch drawn
 * over the ranks' own trajectory shards varies from step to step); `phases` a mask of
 * uavhip_ppo_phase (UAVHIP_PPO_FULL on one GPU; FORWARD | BACKWARD leaves the raw gradients in
 * ppo->grads). BACKWARD needs the workspace FORWARD filled for the same rows. */
int uavhip_ppo_step(const uavhip_ppo* ppo, const float* states, const int8_t* actions, const float* old_logp,
                    const float* old_values, const float* returns, const float* advantages, const int32_t* idx,
                    int32_t phases, uavhip_stream_t stream);

/* ---------------------------------------------------------------- episode metrics */

/* Per-episode sums main_train.py logs (:122-136, :161-195), one record per finished episode. */
enum uavhip_ep {
    UAVHIP_EP_ENV = 0,       /* env index                                              */
    UAVHIP_EP_EPISODE,       /* info EPISODE of the finishing step                     */
    UAVHIP_EP_STEPS,         /* ep_steps                                               */
    UAVHIP_EP_REWARD,        /* current_ep_reward (sum of rewards)                     */
    UAVHIP_EP_Q0,            /* value of the episode's first state (current_q0)        */
    UAVHIP_EP_J_SUM,         /* ep_total_J (sum of info J_val)                         */
    UAVHIP_EP_MAX_COV,       /* ep_max_cov (max num_assigned)                          */
    UAVHIP_EP_ACTION1,       /* ep_action1_cnt                                         */
    UAVHIP_EP_VALID,         /* ep_valid_cnt (action 1 and is_valid_action)            */
    UAVHIP_EP_PDMG_SUM,      /* ep_total_p_dmg (steps with num_assigned > 0)           */
    UAVHIP_EP_PFINAL_SUM,    /* ep_total_p_final                                       */
    UAVHIP_EP_ASSIGN_STEPS,  /* ep_steps_with_assign                                   */
    UAVHIP_EP_COUNT
};

/* Walk a [T][E] rollout chunk (reward f64, done u8, action i8, info [T][E][UAVHIP_INFO_COUNT],
 * value f32 = V(obs[t])) per env in time order, continuing the episodes in acc[E][UAVHIP_EP_COUNT]
 * (zero-initialised once; carries unfinished episodes across chunks). Every finished episode is
 * appended to records[max_records][UAVHIP_EP_COUNT] at slot atomicAdd(n_records, 1) (slots past
 * max_records are counted but dropped). Sums run in step order in fp64, as the reference's. */
int uavhip_episode_stats(const double* reward, const uint8_t* done, const int8_t* action, const double* info,
                         const float* value, int32_t T, int32_t E, double* acc, double* records,
                         int32_t max_records, uint32_t* n_records, uavhip_stream_t stream);

/* ---------------------------------------------------------------- N > 1 trajectory exchange
 * The all-gather of trajectories before the update (the reference has no multi-GPU
 * path, main_train.py:109-146 runs one process) as peer-to-peer copies beside the next rollout
 * (uavhip.dist.IpcAllGather). Host-side helpers over the HIP runtime:
 *   uavhip_device_pci_id: the PCI bus id of a device of this process (>= 13 bytes): the identity
 *                         the ranks exchange, since ordinals are local to a process
 *   uavhip_device_from_pci_id: this process's ordinal of the device with that bus id (-1: not
 *                         visible here)
 *   uavhip_peer_access  : can the current device read peer_device's memory (an ordinal of THIS
 *                         process)? enables peer access (an already enabled one is fine);
 *                         *can_access = 1 for the same device
 *   uavhip_ipc_export   : IPC handle (UAVHIP_IPC_HANDLE_BYTES) of the allocation holding ptr, and
 *                         ptr's offset inside it
 *   uavhip_ipc_open     : map a peer's exported allocation into the CURRENT device's address space
 *                         (no context on the exporter's device); *ptr = base + offset
 *   uavhip_ipc_close    : unmap (the base returned by open minus its offset)
 *   uavhip_copy_async   : device-to-device copy on `stream` (a mapped peer buffer as the source) */
#define UAVHIP_IPC_HANDLE_BYTES 64
int uavhip_device_pci_id(int32_t device, char* buf, int32_t len);
int uavhip_device_from_pci_id(const char* pci_id, int32_t* device);
int uavhip_peer_access(int32_t peer_device, int32_t* can_access);
int uavhip_ipc_export(const void* ptr, void* handle, uint64_t* offset);
int uavhip_ipc_open(const void* handle, uint64_t offset, void** ptr);
int uavhip_ipc_close(void* base);
int uavhip_copy_async(void* dst, const void* src, uint64_t bytes, uavhip_stream_t stream);

/* ---------------------------------------------------------------- misc */
const char* uavhip_last_error(void);
/* 4 since round 3 (struct uavhip_ppo: the Adam hyper-parameters are doubles; the inference packed
   buffer carries split weight copies, uavhip_policy_split_layout); 5 since round 5 (the packed
   buffer ends with the range table, uavhip_policy_range_table; N > 1 peers by PCI bus id); the
   ctypes binding refuses a library of another version */
int32_t uavhip_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* UAVHIP_H */
