// env.hip -- vectorised UAV->target allocation env on gfx950: K1 score_pairs, on-device scene
// generation / refresh, reset, K2 fused step. Reference: envs/uav_env.py, envs/mechanics.py,
// envs/entities.py. Device building blocks: env_device.hpp.
//
//  * K1: one workgroup per env, entity records + per-entity terms staged in LDS, pairs scored from
//    LDS with coalesced p_dmg stores; p_pen (target-independent, mechanics.py:118) per UAV. fp64 VALU.
//  * reset / step / generate / refresh: one wave per env (env_device.hpp).
//  * K2 keeps the whole env state in registers across T fused steps; T = 1 is the per-step
//    rollout call, T > 1 the env-only multi-step launch (BASELINE config 2). It never generates a
//    scene itself (register budget: 4 waves / SIMD); full resets flip to the spare buffer.
#include "env_device.hpp"
#include "env_group.hpp"
#include "env_replay.hpp"

#pragma clang fp contract(off)

namespace uavhip {
using namespace envdev;

namespace {
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWavesPerBlock * kWave;
}  // namespace

// ================================================================== K1: pair tables (active buffer)
// One workgroup per env (LDS-tiled pairwise scoring, BASELINE config 4). The per-UAV terms every
// pair reuses (common.hpp UavTerms: position, unit heading, speed and its reciprocal, load; 64 B)
// are staged in LDS once; each thread then owns ONE target t (its position and K * speed in
// registers) and walks the UAVs u = r, r + R, ... (R = 256 / M rows of M threads), reading the
// UAV's terms as LDS broadcasts (the lanes of a row read the same 64 B) -- no per-pair index
// division -- and storing p_dmg[u][t] coalesced (consecutive threads = consecutive targets).
// p_pen (target-independent, mechanics.py:118) by one thread per UAV. The pair math is damage_pair,
// which the per-wave scene scorer (score_scene_wave) runs too: bitwise the same tables.
constexpr int kScoreThreads = 256;
static_assert(UAVHIP_MAX_N + UAVHIP_MAX_M <= kScoreThreads && UAVHIP_MAX_M <= kScoreThreads,
              "one staging thread per entity; at least one row of targets");
__global__ __launch_bounds__(kScoreThreads) void k_score_pairs(uavhip_env env, const uint8_t* __restrict__ mask) {
    __shared__ __attribute__((aligned(16))) UavTerms s_u[UAVHIP_MAX_N];
    const int e = blockIdx.x;
    if (mask && !mask[e]) return;
    const int N = env.N, M = env.M, tid = threadIdx.x;
    const int sel = env.scene_buffers == 2 ? (env.istate[(long long)e * UAVHIP_IST_COUNT + UAVHIP_IST_SCENE_SEL] & 1) : 0;
    const long long sb = (long long)sel * env.E + e;
    // this thread's target: (row r, target t) of R = 256 / M rows; its loads issued before the barrier
    const int R = kScoreThreads / M, r = tid / M, t = tid - r * M;
    const bool tact = r < R;
    double tpx = 0.0, tpy = 0.0, tvx = 0.0, tvy = 0.0;
    if (tact) {
        const double* tp = env.tgt_pos + 2 * (sb * M + t);
        const double* tv = env.tgt_vel + 2 * (sb * M + t);
        tpx = tp[0];
        tpy = tp[1];
        tvx = tv[0];
        tvy = tv[1];
    }
    if (tid < N) {
        const double* up = env.uav_pos + 2 * (sb * N + tid);
        const double* uv = env.uav_vel + 2 * (sb * N + tid);
        s_u[tid] = uav_terms(up[0], up[1], uv[0], uv[1], env.uav_load[sb * N + tid]);
        env.p_pen[sb * N + tid] = penetration_prob(up[0], up[1], uv[0], uv[1], env.nfz_pos + 2 * sb * env.Kn, env.Kn,
                                                   env.icp_pos + 2 * sb * env.Ki, env.icp_vel + 2 * sb * env.Ki,
                                                   env.Ki, env.prm);
    }
    const PairConst pc = pair_const(env.prm);
    const double kts = env.prm[UAVHIP_PRM_K] * norm2(tvx, tvy);
    __syncthreads();
    if (!tact) return;
    double* out = env.p_dmg + sb * N * M + t;
    for (int u = r; u < N; u += R) out[(long long)u * M] = damage_pair(s_u[u], tpx, tpy, kts, pc);
}

// ================================================================== wave-per-env kernels
// LT (multi-step launches whose tables fit): each wave copies its env's p_dmg table to LDS once
// and the actions of 64 steps to one register, so nothing on the step-to-step dependency chain
// waits for global memory.
template <int TPL, bool LT>
__global__ __launch_bounds__(kBlock) void k_env_step(uavhip_env env, const int8_t* __restrict__ actions, int T,
                                                     int auto_reset, float* __restrict__ obs_out,
                                                     double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                     double* __restrict__ info_out) {
    extern __shared__ double s_tab[];
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock * 16];
    const int lane = lane_id();
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= env.E) return;
    EnvRegs<TPL> R;
    R.tab = s_tab + (threadIdx.x >> 6) * env.N * env.M;
    R.row = s_row + (threadIdx.x >> 6) * 16;
    load_regs<TPL>(R, env, e, lane);
    if (LT) load_table(R, env, lane);
    const long long E = env.E;
    for (int s0 = 0; s0 < T; s0 += kWave) {
        const int na = min(kWave, T - s0);
        // action == 1 (assign) bits of the next 64 steps in an SGPR pair: the wait for this load
        // happens here, not inside the step loop (where it would also wait for every store)
        const int av = lane < na ? actions[(long long)(s0 + lane) * E + e] : 0;
        const unsigned long long abits = ballot(av == 1);
        for (int i = 0; i < na; ++i) {
            const long long se = (long long)(s0 + i) * E + e;
            step_once<TPL, LT>(R, env, e, lane, (int)((abits >> i) & 1ull), auto_reset,
                               obs_out ? obs_at(obs_out, se, obs_f16(env)) : nullptr, reward_out ? reward_out + se : nullptr,
                               done_out ? done_out + se : nullptr,
                               info_out ? info_out + se * UAVHIP_INFO_COUNT : nullptr);
        }
    }
    store_regs(R, env, e, lane);
}
// Two envs per wave (env_group.hpp) for multi-step launches with N, M <= 32 and E even: the same
// step, half the VALU instructions per env-step (the wave-uniform fp64 work serves two envs).
__global__ __launch_bounds__(kBlock) void k_env_step_g(uavhip_env env, const int8_t* __restrict__ actions, int T,
                                                       int auto_reset, float* __restrict__ obs_out,
                                                       double* __restrict__ reward_out, uint8_t* __restrict__ done_out,
                                                       double* __restrict__ info_out) {
    extern __shared__ double s_tab[];  // [wave][group][N * M]
    __shared__ __attribute__((aligned(16))) float s_win[kWavesPerBlock * 2 * envgrp::kWin];
    const int lane = lane_id(), j = lane & 31, wv = threadIdx.x >> 6;
    const int slot = wv * 2 + (lane >> 5);
    const int e = blockIdx.x * kWavesPerBlock * 2 + slot;
    if (e >= env.E) return;  // E is even: both groups of a wave leave together
    envgrp::GRegs R;
    R.tab = s_tab + slot * env.N * env.M;
    R.win = s_win + slot * envgrp::kWin;
    envgrp::gload_regs(R, env, e, j);
    envgrp::gload_table(R, env, j);
    const long long E = env.E;
    for (int s0 = 0; s0 < T; s0 += envgrp::L) {
        const int na = min(envgrp::L, T - s0);
        // this env's action == 1 bits of the next 32 steps
        const int av = j < na ? actions[(long long)(s0 + j) * E + e] : 0;
        const unsigned abits = envgrp::gbits(ballot(av == 1));
        for (int i = 0; i < na; ++i) {
            const long long se = (long long)(s0 + i) * E + e;
            envgrp::gstep(R, env, e, j, (int)((abits >> i) & 1u), auto_reset,
                          obs_out ? obs_at(obs_out, se, obs_f16(env)) : nullptr, reward_out ? reward_out + se : nullptr,
                          done_out ? done_out + se : nullptr, info_out ? info_out + se * UAVHIP_INFO_COUNT : nullptr);
        }
    }
    envgrp::gstore_regs(R, env, e, j);
}

constexpr int kTableMinSteps = 4;                // below this the LDS table costs more than it saves
constexpr int kReplayMinSteps = 8;               // K2r: below this a chunk's walk / fold overhead does not pay
constexpr size_t kReplayMaxLds = 150 * 1024;     // per workgroup (4 envs), below the 160 KiB of a CU
constexpr int kGroupMinEnvs = 4096;
constexpr size_t kTableMaxBytes = 64 * 1024;     // per workgroup (4 envs)

template <int TPL>
__global__ __launch_bounds__(kBlock) void k_env_reset(uavhip_env env, const uint8_t* __restrict__ mask, int episode,
                                                      float* __restrict__ obs_out) {
    const int lane = lane_id();
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= env.E) return;
    if (mask && !mask[e]) return;
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock * 16];
    EnvRegs<TPL> R;
    R.row = s_row + (threadIdx.x >> 6) * 16;
    load_scene_index(env, e, R.sel, R.stale, R.gen, R.sb);
    const int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
    R.ep = episode >= 0 ? episode : is[UAVHIP_IST_EPISODE];
    R.err = 0;
    reset_regs(R, env, lane);
    store_regs(R, env, e, lane);
    if (obs_out) write_obs(obs_at(obs_out, e, obs_f16(env)), R.w0, R.w1, lane, obs_f16(env));
}

// Fresh scene(s) for masked envs: the active buffer, plus the spare when double-buffered.
template <int TPL>
__global__ __launch_bounds__(kBlock) void k_scene_generate(uavhip_env env, const uint8_t* __restrict__ mask) {
    const int lane = lane_id();
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= env.E) return;
    if (mask && !mask[e]) return;
    int sel, stale, gen;
    long long sb;
    load_scene_index(env, e, sel, stale, gen, sb);
    gen_scene_wave<TPL>(env, sb, e, gen++, lane);
    wave_global_fence();
    score_scene_wave(env, sb, lane);
    if (env.scene_buffers == 2) {
        const long long spare = (long long)(sel ^ 1) * env.E + e;
        gen_scene_wave<TPL>(env, spare, e, gen++, lane);
        wave_global_fence();
        score_scene_wave(env, spare, lane);
    }
    if (lane == 0) {
        int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
        is[UAVHIP_IST_SCENE_SEL] = sel;
        is[UAVHIP_IST_SCENE_STALE] = 0;
        is[UAVHIP_IST_SCENE_GEN] = gen;
    }
}

// Regenerate the spare of envs that flipped to it at a full reset.
template <int TPL>
__global__ __launch_bounds__(kBlock) void k_scene_refresh(uavhip_env env) {
    const int lane = lane_id();
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= env.E) return;
    int sel, stale, gen;
    long long sb;
    load_scene_index(env, e, sel, stale, gen, sb);
    if (!stale) return;
    const long long spare = (long long)(sel ^ 1) * env.E + e;
    gen_scene_wave<TPL>(env, spare, e, gen, lane);
    wave_global_fence();
    score_scene_wave(env, spare, lane);
    if (lane == 0) {
        int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
        is[UAVHIP_IST_SCENE_STALE] = 0;
        is[UAVHIP_IST_SCENE_GEN] = gen + 1;
    }
}

// ================================================================== C ABI
int validate_env(const uavhip_env* env, bool need_state) {
    if (!env) { set_error("env descriptor is NULL"); return UAVHIP_EINVAL; }
    if (env->E <= 0 || env->N <= 0 || env->N > UAVHIP_MAX_N || env->M <= 0 || env->M > UAVHIP_MAX_M ||
        env->Kn < 0 || env->Kn > UAVHIP_MAX_OBSTACLES || env->Ki < 0 || env->Ki > UAVHIP_MAX_OBSTACLES) {
        set_error("bad env dims E=%d N=%d M=%d Kn=%d Ki=%d (N<=%d, M<=%d, Kn,Ki<=%d)", env->E, env->N, env->M,
                  env->Kn, env->Ki, UAVHIP_MAX_N, UAVHIP_MAX_M, UAVHIP_MAX_OBSTACLES);
        return UAVHIP_EINVAL;
    }
    if (env->scene_buffers != 1 && env->scene_buffers != 2) {
        set_error("scene_buffers must be 1 or 2 (got %d)", env->scene_buffers);
        return UAVHIP_EINVAL;
    }
    if (env->full_reset_period > 0 && env->scene_buffers != 2) {
        set_error("full_reset_period > 0 needs scene_buffers == 2 (the step kernel flips to a pre-generated spare)");
        return UAVHIP_EINVAL;
    }
    if (!env->uav_pos || !env->uav_vel || !env->uav_load || !env->uav_cost || !env->tgt_pos || !env->tgt_vel ||
        !env->tgt_value || !env->tgt_id || (env->Kn && !env->nfz_pos) || (env->Ki && (!env->icp_pos || !env->icp_vel)) ||
        !env->p_dmg || !env->p_pen || !env->istate) {
        set_error("env scene / pair-table / istate pointer is NULL");
        return UAVHIP_EINVAL;
    }
    if (need_state && (!env->nh_final || !env->nh_pure || !env->t_cost || !env->n_lock || !env->assigned ||
                       !env->dstate || !env->window)) {
        set_error("env state pointer is NULL");
        return UAVHIP_EINVAL;
    }
    return UAVHIP_OK;
}
namespace {
int validate(const uavhip_env* env, bool need_state) { return validate_env(env, need_state); }
inline int wave_grid(int E) { return (E + kWavesPerBlock - 1) / kWavesPerBlock; }
}  // namespace

}  // namespace uavhip

using namespace uavhip;

#define UAVHIP_LAUNCH_TPL(kern, ...)                                                                       \
    do {                                                                                                   \
        if (env->M <= kWave)                                                                               \
            hipLaunchKernelGGL(kern<1>, dim3(wave_grid(env->E)), dim3(kBlock), 0, (hipStream_t)stream, __VA_ARGS__); \
        else                                                                                               \
            hipLaunchKernelGGL(kern<2>, dim3(wave_grid(env->E)), dim3(kBlock), 0, (hipStream_t)stream, __VA_ARGS__); \
    } while (0)

extern "C" int uavhip_score_pairs(const uavhip_env* env, const uint8_t* mask, uavhip_stream_t stream) {
    int rc = validate(env, false);
    if (rc) return rc;
    hipLaunchKernelGGL(k_score_pairs, dim3(env->E), dim3(kScoreThreads), 0, (hipStream_t)stream, *env, mask);
    return check_launch("k_score_pairs");
}

extern "C" int uavhip_scene_generate(const uavhip_env* env, const uint8_t* mask, uavhip_stream_t stream) {
    int rc = validate(env, false);
    if (rc) return rc;
    UAVHIP_LAUNCH_TPL(k_scene_generate, *env, mask);
    return check_launch("k_scene_generate");
}

extern "C" int uavhip_scene_refresh(const uavhip_env* env, uavhip_stream_t stream) {
    int rc = validate(env, false);
    if (rc) return rc;
    if (env->scene_buffers != 2) return UAVHIP_OK;
    UAVHIP_LAUNCH_TPL(k_scene_refresh, *env);
    return check_launch("k_scene_refresh");
}

extern "C" int uavhip_env_reset(const uavhip_env* env, const uint8_t* mask, int32_t episode, float* obs_out,
                                uavhip_stream_t stream) {
    int rc = validate(env, true);
    if (rc) return rc;
    UAVHIP_LAUNCH_TPL(k_env_reset, *env, mask, (int)episode, obs_out);
    return check_launch("k_env_reset");
}

#ifdef UAVHIP_POLICY_TRACE
extern "C" int uavhip_env_trace(unsigned long long* out, int n) {  // k_env_replay phase sums (TRACE build)
    const int total = envrep::kTraceEnvs * envrep::kTracePhases;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(envrep::g_etrace), sizeof(unsigned long long) * (n < total ? n : total),
                               0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int uavhip_env_step(const uavhip_env* env, const int8_t* actions, int32_t T, int32_t auto_reset,
                               float* obs_out, double* reward, uint8_t* done, double* info, uavhip_stream_t stream) {
    int rc = validate(env, true);
    if (rc) return rc;
    if (!actions || T <= 0) { set_error("actions NULL or T <= 0 (T=%d)", T); return UAVHIP_EINVAL; }
    const size_t tab = (size_t)kWavesPerBlock * env->N * env->M * sizeof(double);
    const bool lt = T >= kTableMinSteps && tab <= kTableMaxBytes;
    const dim3 grid(wave_grid(env->E)), block(kBlock);
    hipStream_t st = (hipStream_t)stream;
    // K2r (env_replay.hpp): with omega == 0 the walk is a function of the actions; replay it. Fastest
    // wherever it applies (T = 256, all outputs, G env-steps/s on MI355X: 1024 x 8 x 16 3.07 vs K2g
    // 1.09; 4096 x 8 x 16 3.60 vs 2.87; 4096 x 16 x 32 2.83 vs 2.77), so it is tried first.
    if (auto_reset && T >= kReplayMinSteps && env->prm[UAVHIP_PRM_OMEGA] == 0.0 && env->M <= envrep::kMaxM &&
        !(env->flags & UAVHIP_ENV_NO_REPLAY)) {
        const size_t l64 = (size_t)envrep::kWavesPerBlock * envrep::wave_doubles<64>(env->N, env->M) * sizeof(double);
        const size_t l32 = (size_t)envrep::kWavesPerBlock * envrep::wave_doubles<32>(env->N, env->M) * sizeof(double);
        const dim3 rgrid((env->E + envrep::kWavesPerBlock - 1) / envrep::kWavesPerBlock), rblock(envrep::kBlock);
        if (l64 <= kReplayMaxLds) {
            (void)hipFuncSetAttribute((const void*)envrep::k_env_replay<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l64);
            hipLaunchKernelGGL(envrep::k_env_replay<64>, rgrid, rblock, l64, st, *env, actions, (int)T, obs_out, reward,
                               done, info);
            return check_launch("k_env_replay");
        }
        if (l32 <= kReplayMaxLds) {
            (void)hipFuncSetAttribute((const void*)envrep::k_env_replay<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l32);
            hipLaunchKernelGGL(envrep::k_env_replay<32>, rgrid, rblock, l32, st, *env, actions, (int)T, obs_out, reward,
                               done, info);
            return check_launch("k_env_replay");
        }
    }
    // two envs per wave pays once there are >= 2 such waves per SIMD (E >= 4096 on 1024 SIMDs);
    // below that the launch is latency-bound and one env per wave keeps more waves in flight
    if (lt && env->N <= envgrp::L && env->M <= envgrp::L && env->E % 2 == 0 && env->E >= kGroupMinEnvs &&
        !(env->flags & UAVHIP_ENV_ONE_PER_WAVE)) {
        const int per_block = kWavesPerBlock * 2;
        hipLaunchKernelGGL(k_env_step_g, dim3((env->E + per_block - 1) / per_block), block, 2 * tab, st, *env, actions,
                           (int)T, (int)auto_reset, obs_out, reward, done, info);
        return check_launch("k_env_step_g");
    }
    // (the single-step load order with prefetched next-pair candidates, load_regs<TPL, true>, runs
    // inside the fused rollout launch; instantiating it here as well slowed the multi-step kernels
    // of this code object by ~9 % with byte-identical machine code for them: code placement)
    if (env->M <= kWave) {
        if (lt) hipLaunchKernelGGL((k_env_step<1, true>), grid, block, tab, st, *env, actions, (int)T, (int)auto_reset, obs_out, reward, done, info);
        else hipLaunchKernelGGL((k_env_step<1, false>), grid, block, 0, st, *env, actions, (int)T, (int)auto_reset, obs_out, reward, done, info);
    } else {
        if (lt) hipLaunchKernelGGL((k_env_step<2, true>), grid, block, tab, st, *env, actions, (int)T, (int)auto_reset, obs_out, reward, done, info);
        else hipLaunchKernelGGL((k_env_step<2, false>), grid, block, 0, st, *env, actions, (int)T, (int)auto_reset, obs_out, reward, done, info);
    }
    return check_launch("k_env_step");
}
