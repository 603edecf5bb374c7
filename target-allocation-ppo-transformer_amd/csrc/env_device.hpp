// env_device.hpp -- device building blocks of the vectorised UAV->target allocation env
// (envs/uav_env.py, envs/mechanics.py), shared by env.hip (standalone env kernels) and any kernel
// that steps envs in its epilogue.
//
// Mapping: ONE WAVE PER ENV. Lane l owns targets l and l+64 (list order) and UAV l. The sequential
// fp64 sums the reference performs (J(X) over targets in list order, uav_env.py:252-265; the info
// sums, :375-407) run as readlane chains in the reference order, so rewards / obs / info are
// bitwise what the reference's algorithm yields given the same pair probabilities. Per-target
// "not hit" products are cached and updated in lock order, the order the reference multiplies them
// in (:255-260). All control flow is wave-uniform.
//
// Scene storage: with scene_buffers == 2 every scene array and pair table is [2][E][...]; env e's
// active scene is buffer istate[SCENE_SEL]: element index base sb = sel * E + e. A full reset flips
// to the pre-generated spare (uavhip_scene_refresh regenerates spares off the step path).
#pragma once
#include "common.hpp"

#pragma clang fp contract(off)

namespace uavhip {
namespace envdev {

constexpr int kObs = UAVHIP_OBS_FLOATS;  // 70
constexpr int kDim = UAVHIP_STATE_DIM;   // 14

// ------------------------------------------------------------------ scene-level (rare path)

// Score all N*M pairs (+ N penetration terms) of scene buffer index sb with one wave.
__device__ inline void score_scene_wave(const uavhip_env& env, long long sb, int lane) {
    const int N = env.N, M = env.M, NM = N * M;
    for (int i = lane; i < NM + N; i += kWave) {
        const int u = i < NM ? i / M : i - NM;
        const double* up = env.uav_pos + 2 * (sb * N + u);
        const double* uv = env.uav_vel + 2 * (sb * N + u);
        if (i < NM) {
            const int t = i - u * M;
            const double* tp = env.tgt_pos + 2 * (sb * M + t);
            const double* tv = env.tgt_vel + 2 * (sb * M + t);
            env.p_dmg[sb * NM + i] =
                damage_prob(up[0], up[1], uv[0], uv[1], env.uav_load[sb * N + u], tp[0], tp[1], tv[0], tv[1], env.prm);
        } else {
            env.p_pen[sb * N + u] =
                penetration_prob(up[0], up[1], uv[0], uv[1], env.nfz_pos + 2 * sb * env.Kn, env.Kn,
                                 env.icp_pos + 2 * sb * env.Ki, env.icp_vel + 2 * sb * env.Ki, env.Ki, env.prm);
        }
    }
}

// Rank of this lane's key among the first n lanes (ties broken by lane index) -> a uniformly random
// permutation: the wave-parallel stand-in for random.shuffle / np.random.shuffle.
__device__ __forceinline__ int rank_in_wave(uint32_t key, int lane, int n) {
    int r = 0;
    for (int j = 0; j < n; ++j) {
        const uint32_t kj = readlane_u(key, j);
        r += (kj < key) || (kj == key && j < lane);
    }
    return r;
}

// uav_env.py:65-173 distribution into scene buffer index sb; Philox counter (lane, global env index
// env_base + e, gen, stream): a rank's shard draws the scenes of the same envs of the union.
template <int TPL>
__device__ void gen_scene_wave(const uavhip_env& env, long long sb, int e, int gen, int lane) {
    const int N = env.N, M = env.M;
    const uint32_t k0 = (uint32_t)env.seed, k1 = (uint32_t)(env.seed >> 32);
    const double* g = env.gen;
    const double H = g[UAVHIP_GEN_MAP_H];
    const uint32_t ue = (uint32_t)(env.env_base + (uint64_t)e), ug = (uint32_t)gen;
    {   // UAVs: N//4 of type 2 at random positions (random.shuffle(uav_types), :81-84)
        const u32x4 rk = philox(u32x4{(uint32_t)lane, ue, ug, 0u}, k0, k1);
        const u32x4 ru = philox(u32x4{(uint32_t)lane, ue, ug, 1u}, k0, k1);
        const u32x4 rv = philox(u32x4{(uint32_t)lane, ue, ug, 2u}, k0, k1);
        const int rank = rank_in_wave(rk.x, lane, N);
        if (lane < N) {
            const int type = rank < N / 4 ? 2 : 1;
            const double x = g[UAVHIP_GEN_UAV_X0] + (g[UAVHIP_GEN_UAV_X1] - g[UAVHIP_GEN_UAV_X0]) * u01(ru.x, ru.y);
            const double y = 0.0 + (H - 0.0) * u01(ru.z, ru.w);
            const double us = u01(rv.x, rv.y);
            const double base_speed = type == 1 ? 0.35 + (0.50 - 0.35) * us : 0.75 + (0.90 - 0.75) * us;
            const double speed = base_speed * g[UAVHIP_GEN_WEATHER_SPEED];
            const double load = (type == 1 ? 0.95 : 1.0) * g[UAVHIP_GEN_WEATHER_LOAD];
            const double deg = -15.0 + (15.0 - -15.0) * u01(rv.z, rv.w);
            const double ang = deg * (M_PI / 180.0);
            const long long o = sb * N + lane;
            env.uav_pos[2 * o] = x;
            env.uav_pos[2 * o + 1] = y;
            env.uav_vel[2 * o] = cos(ang) * speed;
            env.uav_vel[2 * o + 1] = sin(ang) * speed;
            env.uav_load[o] = load;
            env.uav_cost[o] = type == 1 ? 1.0 : 1.25;
            if (env.uav_type) env.uav_type[o] = type;
        }
    }
    {   // targets: values {4 x M//2, 6 x n2, 8 x n3, 16 x 1} shuffled, ids shuffled (:121-142,173)
        const int n1 = M / 2, n_remain = M - n1 - 1;
        const u32x4 rn = philox(u32x4{0u, ue, ug, 3u}, k0, k1);
        int n2 = 0;
        if (n_remain >= 1) n2 = min(n_remain, 1 + (int)(u01(rn.x, rn.y) * n_remain));
        const int n3 = n_remain - n2;
        uint32_t kid[TPL], kval[TPL];
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
            const u32x4 r = philox(u32x4{(uint32_t)(lane + kWave * k), ue, ug, 4u}, k0, k1);
            kid[k] = r.x;
            kval[k] = r.y;
        }
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
            const int t = lane + kWave * k;
            int rid = 0, rval = 0;
            for (int j = 0; j < M; ++j) {
                const int jl = j & 63;
                uint32_t a = readlane_u(kid[0], jl), b = readlane_u(kval[0], jl);
                if (TPL > 1 && j >= kWave) { a = readlane_u(kid[TPL - 1], jl); b = readlane_u(kval[TPL - 1], jl); }
                rid += (a < kid[k]) || (a == kid[k] && j < t);
                rval += (b < kval[k]) || (b == kval[k] && j < t);
            }
            if (t < M) {
                const u32x4 r = philox(u32x4{(uint32_t)t, ue, ug, 5u}, k0, k1);
                const u32x4 r2 = philox(u32x4{(uint32_t)t, ue, ug, 6u}, k0, k1);
                const long long o = sb * M + t;
                env.tgt_pos[2 * o] = g[UAVHIP_GEN_TGT_X0] + (g[UAVHIP_GEN_TGT_X1] - g[UAVHIP_GEN_TGT_X0]) * u01(r.x, r.y);
                env.tgt_pos[2 * o + 1] = 0.0 + (H - 0.0) * u01(r.z, r.w);
                env.tgt_vel[2 * o] = (u01(r2.x, r2.y) - 0.5) * 0.03;
                env.tgt_vel[2 * o + 1] = (u01(r2.z, r2.w) - 0.5) * 0.03;
                env.tgt_value[o] = rval < n1 ? 4.0 : (rval < n1 + n2 ? 6.0 : (rval < n1 + n2 + n3 ? 8.0 : 16.0));
                env.tgt_id[o] = rid;
            }
        }
    }
    if (lane < env.Kn) {  // no-fly zones (:146-153)
        const u32x4 r = philox(u32x4{(uint32_t)lane, ue, ug, 7u}, k0, k1);
        const long long o = sb * env.Kn + lane;
        env.nfz_pos[2 * o] = g[UAVHIP_GEN_NFZ_X0] + (g[UAVHIP_GEN_NFZ_X1] - g[UAVHIP_GEN_NFZ_X0]) * u01(r.x, r.y);
        env.nfz_pos[2 * o + 1] = 0.0 + (H - 0.0) * u01(r.z, r.w);
    }
    if (lane < env.Ki) {  // interceptors (:156-170)
        const u32x4 r = philox(u32x4{(uint32_t)lane, ue, ug, 8u}, k0, k1);
        const u32x4 r2 = philox(u32x4{(uint32_t)lane, ue, ug, 9u}, k0, k1);
        const long long o = sb * env.Ki + lane;
        env.icp_pos[2 * o] = g[UAVHIP_GEN_ICP_X0] + (g[UAVHIP_GEN_ICP_X1] - g[UAVHIP_GEN_ICP_X0]) * u01(r.x, r.y);
        env.icp_pos[2 * o + 1] = 0.0 + (H - 0.0) * u01(r.z, r.w);
        const double sp = g[UAVHIP_GEN_ICP_S0] + (g[UAVHIP_GEN_ICP_S1] - g[UAVHIP_GEN_ICP_S0]) * u01(r2.x, r2.y);
        const double ang = 0.0 + (2.0 * M_PI - 0.0) * u01(r2.z, r2.w);
        env.icp_vel[2 * o] = cos(ang) * sp;
        env.icp_vel[2 * o + 1] = sin(ang) * sp;
    }
}

// Make this wave's global writes visible to its own later loads (same CU: workgroup scope).
__device__ __forceinline__ void wave_global_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ------------------------------------------------------------------ register-resident env state
template <int TPL>
struct EnvRegs {
    // per target slot k (target t = lane + 64k, list order)
    double nhf[TPL], nhp[TPL], tc[TPL], val[TPL];
    int nlk[TPL];
    // per UAV lane
    int asg;                // target list index or -1
    double ucost, ppen;     // cost, p_pen
    // wave-uniform scalars
    int u, t, ncov, nasg, ep, err, sel, stale, gen;
    long long sb;           // active scene base index (sel * E + e)
    double r, J, asg_cost, cov_val, tot_cost, tot_val;
    double sum_pd, sum_pf;  // p_dmg / p_final summed over locked pairs in lock order (info)
    double pd_cur, pp_cur;  // pair probabilities of the current pointer (u, t)
    // observation window: element i (< 64) on lane i in w0, element 64 + i (i < 6) in w1
    float w0, w1;
    // multi-step launches (LT = true): this wave's LDS copy of the active scene's p_dmg table
    double* tab;
    // the wave's 16-float LDS scratch: the new observation row on its way to its lanes
    float* row;
    // loop-invariant divisors and their correctly rounded reciprocals (div_by)
    double den_c, rcp_c, den_v, rcp_v, rcp_m;
    double rcp_n;  // lane l: RN(1 / (l + 1)), the info averages' divisors 1..64
    // pair probabilities the first step of a launch can move the pointer to, loaded by load_regs
    // ahead of the step (p_dmg of (u, t + 1), (u + 1, 0) and (0, 0) of scene sb): one launch-start
    // load round instead of a dependent global load at the end of the step
    bool pc_ok = false;
    int pc_u, pc_t;
    long long pc_sb;
    double pc[3];
};

// a / b, correctly rounded, from y = RN(1 / b) (Markstein's theorem: q = RN(a y) is within 1 ulp
// of a / b, r = a - b q is exact by FMA, and RN(q + r y) = RN(a / b) without over/underflow). Three
// VALU ops instead of the ~10 of an IEEE fp64 division -- the step kernel is VALU-issue bound.
__device__ __forceinline__ double div_by(double a, double b, double y) {
    const double q = a * y;
    const double r = fma(-b, q, a);
    return fma(r, y, q);
}

template <int TPL>
__device__ __forceinline__ void set_scene_divisors(EnvRegs<TPL>& R) {
    R.den_c = R.tot_cost + 1e-6;
    R.rcp_c = 1.0 / R.den_c;
    R.den_v = R.tot_val + 1e-6;
    R.rcp_v = 1.0 / R.den_v;
}
template <int TPL>
__device__ __forceinline__ void set_step_divisors(EnvRegs<TPL>& R, const uavhip_env& env, int lane) {
    R.rcp_m = 1.0 / (double)env.M;
    R.rcp_n = 1.0 / (double)(lane + 1);
}

template <int TPL>
__device__ __forceinline__ double pick(const double (&a)[TPL], int k, int l) {
    double v = readlane_d(a[0], l);
    if (TPL > 1 && k == 1) v = readlane_d(a[TPL - 1], l);
    return v;
}
template <int TPL>
__device__ __forceinline__ int pick(const int (&a)[TPL], int k, int l) {
    int v = readlane_i(a[0], l);
    if (TPL > 1 && k == 1) v = readlane_i(a[TPL - 1], l);
    return v;
}

// Wait for this wave's outstanding memory operations. Called where register state was just
// loaded: a load still in flight at a loop back-edge makes the compiler wait for vmcnt(0) (all
// stores included) at every later use inside the step loop.
__device__ __forceinline__ void drain_loads() { __builtin_amdgcn_s_waitcnt(0); }

// Scene-dependent per-lane values (after a reset or a scene switch).
template <int TPL>
__device__ void load_scene_regs(EnvRegs<TPL>& R, const uavhip_env& env, int lane) {
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
        const int t = lane + kWave * k;
        R.val[k] = t < env.M ? env.tgt_value[R.sb * env.M + t] : 0.0;
    }
    R.ucost = lane < env.N ? env.uav_cost[R.sb * env.N + lane] : 0.0;
    R.ppen = lane < env.N ? env.p_pen[R.sb * env.N + lane] : 0.0;
    drain_loads();
}

// mechanics.py:185-241 get_state_vector + uav_env.py:194-237 (_get_obs context): the 14 floats of
// the observation row of pointer (u, t) -- UAV u's cost, target t's value, its locker-cost sum and
// not-hit products (tc, nhf, nhp), the allocation's cost / covered-value sums, the pair's p_dmg and
// p_pen, the scene divisors. The one definition of the row's arithmetic (push_obs, the replay kernel).
struct ObsRow {
    float v[14];
};
__device__ __forceinline__ ObsRow obs_row(double ucost, double val, double tc, double nhf, double nhp, double asg_cost,
                                          double cov_val, double pd, double pp, double den_c, double rcp_c,
                                          double den_v, double rcp_v) {
    const double chi_c = div_by(asg_cost, den_c, rcp_c);
    const double chi_v = div_by(cov_val, den_v, rcp_v);
    const double chi_mc = div_by(tc, den_c, rcp_c);
    const double pjp = 1.0 - nhf;
    const double pjp_pure = 1.0 - nhp;
    const double prev_rev = pjp * val;
    const double p_km = pd * pp;
    const double p_pure = pd;
    const double hat_p = 1.0 - (1.0 - pjp) * (1.0 - p_km);
    const double hat_pp = 1.0 - (1.0 - pjp_pure) * (1.0 - p_pure);
    const double hat_G = hat_p * val;
    const double d_pkm = p_pure - p_km;
    const double d_pm = hat_pp - hat_p;
    const double d_G = (hat_pp * val) - hat_G;
    return ObsRow{{(float)ucost / 2.0f, (float)val / 16.0f, (float)chi_c, (float)chi_v, (float)chi_mc, (float)p_km,
                   (float)pjp, (float)hat_p, (float)prev_rev / 16.0f, (float)hat_G / 16.0f, (float)d_pkm, (float)d_pm,
                   (float)d_G / 16.0f, 1.0f}};
}

// The current pointer's row (obs_row), pushed into the window (uav_env.py:241-242).
template <int TPL>
__device__ void push_obs(EnvRegs<TPL>& R, int lane) {
    const int tl = R.t & 63, tk = R.t >> 6;
    const ObsRow o = obs_row(readlane_d(R.ucost, R.u), pick(R.val, tk, tl), pick(R.tc, tk, tl), pick(R.nhf, tk, tl),
                             pick(R.nhp, tk, tl), R.asg_cost, R.cov_val, R.pd_cur, R.pp_cur, R.den_c, R.rcp_c, R.den_v,
                             R.rcp_v);
    // the new row goes through the wave's LDS scratch (lane 0 writes, lanes 56..63 and 0..5 read
    // their element): 6 LDS instructions instead of two 14-way VALU select chains. LDS operations
    // of one wave complete in order, so the reads see the write.
    if (lane == 0) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<f32x4*>(R.row) = f32x4{o.v[0], o.v[1], o.v[2], o.v[3]};
        *reinterpret_cast<f32x4*>(R.row + 4) = f32x4{o.v[4], o.v[5], o.v[6], o.v[7]};
        *reinterpret_cast<f32x4*>(R.row + 8) = f32x4{o.v[8], o.v[9], o.v[10], o.v[11]};
        *reinterpret_cast<f32x2*>(R.row + 12) = f32x2{o.v[12], o.v[13]};
    }
    // shift the deque by one row (14 floats) and append
    const float a = __shfl(R.w0, (lane + kDim) & 63);
    const float b = __shfl(R.w1, (lane + kDim - kWave) & 63);
    const float r0 = R.row[(lane - (kObs - kDim)) & 15];           // new row, elements 56..63
    const float r1 = R.row[(lane + kWave - (kObs - kDim)) & 15];   // new row, elements 64..69 (lane < 6)
    float nw0;
    if (lane < kWave - kDim) nw0 = a;             // elements 14..63 -> 0..49
    else if (lane < kObs - kDim) nw0 = b;         // elements 64..69 -> 50..55
    else nw0 = r0;
    R.w0 = nw0;
    R.w1 = lane < kObs - kWave ? r1 : 0.0f;
}

// Pair probabilities of the current pointer (u, t). LT: p_dmg from the wave's LDS table (a short
// LDS round trip instead of a global-memory one on the step-to-step dependency chain).
template <int TPL, bool LT = false>
__device__ __forceinline__ void load_cur_pair(EnvRegs<TPL>& R, const uavhip_env& env) {
    if (R.u < env.N) {
        if (LT) {
            R.pd_cur = R.tab[R.u * env.M + R.t];
        } else if (R.pc_ok && R.sb == R.pc_sb && R.t == 0 && (R.u == R.pc_u + 1 || R.u == 0)) {
            R.pd_cur = R.u == 0 ? R.pc[2] : R.pc[1];
        } else if (R.pc_ok && R.sb == R.pc_sb && R.u == R.pc_u && R.t == R.pc_t + 1) {
            R.pd_cur = R.pc[0];
        } else {
            R.pd_cur = env.p_dmg[(R.sb * env.N + R.u) * env.M + R.t];
        }
        R.pc_ok = false;
        R.pp_cur = readlane_d(R.ppen, R.u);
    } else {
        R.pd_cur = 0.0;
        R.pp_cur = 0.0;
    }
}

// Copy the active scene's p_dmg table [N][M] into the wave's LDS table (wave-private: LDS
// operations of one wave complete in order, so no barrier is needed before its own reads).
template <int TPL>
__device__ void load_table(EnvRegs<TPL>& R, const uavhip_env& env, int lane) {
    const int NM = env.N * env.M;
    const double* src = env.p_dmg + R.sb * NM;
    for (int i = lane; i < NM; i += kWave) R.tab[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// uav_env.py:42-63,175-182: reset allocation and window, first observation at (0, 0).
// scene: (re)load the scene-dependent registers and totals (after a scene switch or when starting
// from memory); a state-only reset within a launch keeps them.
template <int TPL, bool LT = false>
__device__ void reset_regs(EnvRegs<TPL>& R, const uavhip_env& env, int lane, bool scene = true) {
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
        R.nhf[k] = 1.0;
        R.nhp[k] = 1.0;
        R.tc[k] = 0.0;
        R.nlk[k] = 0;
    }
    R.asg = -1;
    R.u = 0; R.t = 0; R.ncov = 0; R.nasg = 0;
    R.r = 0.0; R.J = 0.0; R.asg_cost = 0.0; R.cov_val = 0.0;
    R.sum_pd = 0.0; R.sum_pf = 0.0;
    if (scene) {
        load_scene_regs(R, env, lane);
        // total_swarm_cost accumulated in generation order (uav_env.py:118); total value in list order (:198)
        double tc = 0.0;
        for (int j = 0; j < env.N; ++j) tc = tc + readlane_d(R.ucost, j);
        double tv = 0.0;
        for (int j = 0; j < env.M; ++j) {
            double v = readlane_d(R.val[0], j & 63);
            if (TPL > 1 && j >= kWave) v = readlane_d(R.val[TPL - 1], j & 63);
            tv = tv + v;
        }
        R.tot_cost = tc;
        R.tot_val = tv;
        set_scene_divisors(R);
    }
    R.w0 = 0.0f;
    R.w1 = 0.0f;
    load_cur_pair<TPL, LT>(R, env);
    push_obs(R, lane);
}

__device__ __forceinline__ void load_scene_index(const uavhip_env& env, int e, int& sel, int& stale, int& gen,
                                                 long long& sb) {
    const int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
    sel = env.scene_buffers == 2 ? (is[UAVHIP_IST_SCENE_SEL] & 1) : 0;
    stale = is[UAVHIP_IST_SCENE_STALE];
    gen = is[UAVHIP_IST_SCENE_GEN];
    sb = (long long)sel * env.E + e;
}

// Register state from memory. PF (single-step launches): ONE load round -- nothing waits for the
// active-scene index (the scene-dependent values are read from both buffers and selected
// afterwards) -- and then, without a wait, the pair probabilities the first step can move the
// pointer to (load_cur_pair). Multi-step launches load once per launch and keep the plain order
// (scene index, scene values, state): fewer live registers in their step loop.
template <int TPL, bool PF = false>
__device__ void load_regs(EnvRegs<TPL>& R, const uavhip_env& env, int e, int lane) {
    const int N = env.N, M = env.M;
    if constexpr (!PF) {
        load_scene_index(env, e, R.sel, R.stale, R.gen, R.sb);
        load_scene_regs(R, env, lane);
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
            const int t = lane + kWave * k;
            const long long o = (long long)e * M + t;
            const bool v = t < M;
            R.nhf[k] = v ? env.nh_final[o] : 1.0;
            R.nhp[k] = v ? env.nh_pure[o] : 1.0;
            R.tc[k] = v ? env.t_cost[o] : 0.0;
            R.nlk[k] = v ? env.n_lock[o] : 0;
        }
        R.asg = lane < N ? env.assigned[(long long)e * N + lane] : -1;
        const int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
        const double* ds = env.dstate + (long long)e * UAVHIP_DST_COUNT;
        R.u = is[UAVHIP_IST_UAV_IDX];
        R.t = is[UAVHIP_IST_TARGET_IDX];
        R.ncov = is[UAVHIP_IST_N_COVERED];
        R.nasg = is[UAVHIP_IST_N_ASSIGNED];
        R.ep = is[UAVHIP_IST_EPISODE];
        R.err = is[UAVHIP_IST_ERROR];
        R.r = ds[UAVHIP_DST_R];
        R.J = ds[UAVHIP_DST_J];
        R.asg_cost = ds[UAVHIP_DST_ASG_COST];
        R.cov_val = ds[UAVHIP_DST_COV_VALUE];
        R.tot_cost = ds[UAVHIP_DST_TOTAL_COST];
        R.tot_val = ds[UAVHIP_DST_TOTAL_VALUE];
        set_scene_divisors(R);
        set_step_divisors(R, env, lane);
        R.sum_pd = ds[UAVHIP_DST_SUM_PDMG];
        R.sum_pf = ds[UAVHIP_DST_SUM_PFIN];
        const float* w = env.window + (long long)e * kObs;
        R.w0 = w[lane];
        R.w1 = lane < kObs - kWave ? w[kWave + lane] : 0.0f;
        R.pd_cur = ds[UAVHIP_DST_PD_CUR];
        R.pp_cur = R.u < N ? readlane_d(R.ppen, R.u) : 0.0;
        drain_loads();
        return;
    }
    const int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
    const double* ds = env.dstate + (long long)e * UAVHIP_DST_COUNT;
    const int nb = env.scene_buffers;
    double valb[2][TPL], ucb[2], ppb[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const long long sb = (long long)(b < nb ? b : 0) * env.E + e;
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
            const int t = lane + kWave * k;
            valb[b][k] = t < M ? env.tgt_value[sb * M + t] : 0.0;
        }
        ucb[b] = lane < N ? env.uav_cost[sb * N + lane] : 0.0;
        ppb[b] = lane < N ? env.p_pen[sb * N + lane] : 0.0;
    }
    const int sel_raw = is[UAVHIP_IST_SCENE_SEL];
    R.stale = is[UAVHIP_IST_SCENE_STALE];
    R.gen = is[UAVHIP_IST_SCENE_GEN];
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
        const int t = lane + kWave * k;
        const long long o = (long long)e * M + t;
        const bool v = t < M;
        R.nhf[k] = v ? env.nh_final[o] : 1.0;
        R.nhp[k] = v ? env.nh_pure[o] : 1.0;
        R.tc[k] = v ? env.t_cost[o] : 0.0;
        R.nlk[k] = v ? env.n_lock[o] : 0;
    }
    R.asg = lane < N ? env.assigned[(long long)e * N + lane] : -1;
    R.u = is[UAVHIP_IST_UAV_IDX];
    R.t = is[UAVHIP_IST_TARGET_IDX];
    R.ncov = is[UAVHIP_IST_N_COVERED];
    R.nasg = is[UAVHIP_IST_N_ASSIGNED];
    R.ep = is[UAVHIP_IST_EPISODE];
    R.err = is[UAVHIP_IST_ERROR];
    R.r = ds[UAVHIP_DST_R];
    R.J = ds[UAVHIP_DST_J];
    R.asg_cost = ds[UAVHIP_DST_ASG_COST];
    R.cov_val = ds[UAVHIP_DST_COV_VALUE];
    R.tot_cost = ds[UAVHIP_DST_TOTAL_COST];
    R.tot_val = ds[UAVHIP_DST_TOTAL_VALUE];
    R.sum_pd = ds[UAVHIP_DST_SUM_PDMG];
    R.sum_pf = ds[UAVHIP_DST_SUM_PFIN];
    const float* w = env.window + (long long)e * kObs;
    R.w0 = w[lane];
    R.w1 = lane < kObs - kWave ? w[kWave + lane] : 0.0f;
    // the current pair's p_dmg was cached by the previous launch
    R.pd_cur = ds[UAVHIP_DST_PD_CUR];
    drain_loads();
    R.sel = nb == 2 ? (sel_raw & 1) : 0;
    R.sb = (long long)R.sel * env.E + e;
#pragma unroll
    for (int k = 0; k < TPL; ++k) R.val[k] = R.sel ? valb[1][k] : valb[0][k];
    R.ucost = R.sel ? ucb[1] : ucb[0];
    R.ppen = R.sel ? ppb[1] : ppb[0];
    if (R.u < N) {  // candidates for the first step's load_cur_pair, consumed after its compute
        const double* pt = env.p_dmg + R.sb * N * M;
        const int u = R.u, t = R.t;
        R.pc[0] = t + 1 < M ? pt[u * M + t + 1] : 0.0;
        R.pc[1] = u + 1 < N ? pt[(u + 1) * M] : 0.0;
        R.pc[2] = pt[0];
        R.pc_u = u;
        R.pc_t = t;
        R.pc_sb = R.sb;
        R.pc_ok = true;
    }
    set_scene_divisors(R);
    set_step_divisors(R, env, lane);
    R.pp_cur = R.u < N ? readlane_d(R.ppen, R.u) : 0.0;
}

template <int TPL>
__device__ void store_regs(const EnvRegs<TPL>& R, const uavhip_env& env, int e, int lane) {
    const int N = env.N, M = env.M;
#pragma unroll
    for (int k = 0; k < TPL; ++k) {
        const int t = lane + kWave * k;
        if (t < M) {
            const long long o = (long long)e * M + t;
            env.nh_final[o] = R.nhf[k];
            env.nh_pure[o] = R.nhp[k];
            env.t_cost[o] = R.tc[k];
            env.n_lock[o] = R.nlk[k];
        }
    }
    if (lane < N) env.assigned[(long long)e * N + lane] = R.asg;
    if (lane == 0) {
        int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
        double* ds = env.dstate + (long long)e * UAVHIP_DST_COUNT;
        is[UAVHIP_IST_UAV_IDX] = R.u;
        is[UAVHIP_IST_TARGET_IDX] = R.t;
        is[UAVHIP_IST_N_COVERED] = R.ncov;
        is[UAVHIP_IST_N_ASSIGNED] = R.nasg;
        is[UAVHIP_IST_EPISODE] = R.ep;
        is[UAVHIP_IST_ERROR] = R.err;
        is[UAVHIP_IST_SCENE_SEL] = R.sel;
        is[UAVHIP_IST_SCENE_STALE] = R.stale;
        is[UAVHIP_IST_SCENE_GEN] = R.gen;
        ds[UAVHIP_DST_R] = R.r;
        ds[UAVHIP_DST_J] = R.J;
        ds[UAVHIP_DST_ASG_COST] = R.asg_cost;
        ds[UAVHIP_DST_COV_VALUE] = R.cov_val;
        ds[UAVHIP_DST_TOTAL_COST] = R.tot_cost;
        ds[UAVHIP_DST_TOTAL_VALUE] = R.tot_val;
        ds[UAVHIP_DST_PD_CUR] = R.pd_cur;
        ds[UAVHIP_DST_SUM_PDMG] = R.sum_pd;
        ds[UAVHIP_DST_SUM_PFIN] = R.sum_pf;
    }
    float* w = env.window + (long long)e * kObs;
    w[lane] = R.w0;
    if (lane < kObs - kWave) w[kWave + lane] = R.w1;
}

// obs_out element type: f32, or IEEE binary16 (round to nearest even of the f32 window) under
// UAVHIP_ENV_OBS_F16 (BASELINE config 4: fp16 obs; the env's own window stays f32)
__device__ __forceinline__ bool obs_f16(const uavhip_env& env) { return (env.flags & UAVHIP_ENV_OBS_F16) != 0; }
__device__ __forceinline__ float* obs_at(float* base, long long i, bool h) {
    return h ? reinterpret_cast<float*>(reinterpret_cast<_Float16*>(base) + i * kObs) : base + i * kObs;
}
__device__ __forceinline__ void write_obs(float* o, float w0, float w1, int lane, bool h) {
    if (h) {
        _Float16* q = reinterpret_cast<_Float16*>(o);
        q[lane] = (_Float16)w0;
        if (lane < kObs - kWave) q[kWave + lane] = (_Float16)w1;
    } else {
        o[lane] = w0;
        if (lane < kObs - kWave) o[kWave + lane] = w1;
    }
}

// uav_env.py:369-433 diagnostics. The reference re-sums p_dmg / p_final over all locked pairs in
// (target list, lock) order every step; here they are running sums in lock (= time) order, which
// differ from it only by summation order (<= a few ulp, checked to 1e-12 against the reference).
template <int TPL>
__device__ void write_info(const EnvRegs<TPL>& R, const uavhip_env& env, double is_valid, double* o, int lane) {
    static_assert(UAVHIP_INFO_COUNT == 8 && UAVHIP_INFO_J == 0 && UAVHIP_INFO_NUM_ASSIGNED == 1 &&
                  UAVHIP_INFO_IS_VALID == 2 && UAVHIP_INFO_AVG_P_DMG == 3 && UAVHIP_INFO_AVG_P_FINAL == 4 &&
                  UAVHIP_INFO_UAV_IDX == 5 && UAVHIP_INFO_TARGET_IDX == 6 && UAVHIP_INFO_EPISODE == 7,
                  "info record layout");
    const int cnt = R.nasg;
    const double y = cnt > 0 ? readlane_d(R.rcp_n, cnt - 1) : 0.0;
    const double avg_d = cnt > 0 ? div_by(R.sum_pd, (double)cnt, y) : 0.0;
    const double avg_f = cnt > 0 ? div_by(R.sum_pf, (double)cnt, y) : 0.0;
    if (lane == 0) {  // the 64-byte record from one lane: 4 stores, no per-lane selection
        double2* q = reinterpret_cast<double2*>(o);
        q[0] = make_double2(R.J, (double)R.ncov);
        q[1] = make_double2(is_valid, avg_d);
        q[2] = make_double2(avg_f, (double)R.u);
        q[3] = make_double2((double)R.t, (double)R.ep);
    }
}

// One UAVEnv.step (uav_env.py:295-435) on register state. No scene generation on this path: a
// full reset flips to the pre-generated spare scene (scene_buffers == 2).
template <int TPL, bool LT = false>
__device__ void step_once(EnvRegs<TPL>& R, const uavhip_env& env, int e, int lane, int a, int auto_reset,
                          float* obs_o, double* rew_o, uint8_t* done_o, double* info_o) {
    const int N = env.N, M = env.M;
    if (R.u >= N) {  // stepping a finished env: the reference raises IndexError (:296)
        R.err |= 1;
        if (obs_o) write_obs(obs_o, 0.0f, 0.0f, lane, obs_f16(env));
        if (lane == 0) {
            if (rew_o) *rew_o = 0.0;
            if (done_o) *done_o = 1;
        }
        if (info_o && lane < UAVHIP_INFO_COUNT) info_o[lane] = 0.0;
        return;
    }
    const int u = R.u, t = R.t;
    const int tl = t & 63, tk = t >> 6;
    const double prev_r = R.r;  // :301 (cached r(X) of the current allocation)
    double reward = 0.0;
    if (a == 1) {  // :306-342 tentative assign, accept iff r(X') >= r(X)
        const double pd = R.pd_cur, pp = R.pp_cur;
        const double pf = pd * pp;
        const double nhf_t = pick(R.nhf, tk, tl);
        const int nlk_t = pick(R.nlk, tk, tl);
        const double nhf_new = nhf_t * (1.0 - pf);
        const int ncov_new = R.ncov + (nlk_t == 0 ? 1 : 0);
        // J(X') revenue: sum over targets in list order (:252-265); unlocked targets add +0.0
        double rev = 0.0;
#pragma unroll
        for (int k = 0; k < TPL; ++k) {
            const bool mine = (lane == tl) && (k == tk);
            const double nh = mine ? nhf_new : R.nhf[k];
            const double term = (1.0 - nh) * R.val[k];
            unsigned long long m = ballot(lane + kWave * k < M && (R.nlk[k] > 0 || mine));
            while (m) {
                const int j = ffs64(m);
                m &= m - 1;
                rev = rev + readlane_d(term, j);
            }
        }
        const double ucost_u = readlane_d(R.ucost, u);
        const double cost_all = R.asg_cost + ucost_u;  // exact for costs in {1, 1.25}
        const double J = rev - (env.prm[UAVHIP_PRM_OMEGA] * cost_all);
        const double new_r = (ncov_new == M) ? 2.0 * J : J * div_by((double)ncov_new, (double)M, R.rcp_m);
        if (new_r >= prev_r) {
            const double val_t = pick(R.val, tk, tl);
#pragma unroll
            for (int k = 0; k < TPL; ++k) {
                if (lane == tl && k == tk) {
                    R.nhf[k] = nhf_new;
                    R.nhp[k] = R.nhp[k] * (1.0 - pd);
                    R.tc[k] = R.tc[k] + ucost_u;
                    R.nlk[k] = R.nlk[k] + 1;
                }
            }
            if (lane == u) R.asg = t;
            R.sum_pd = R.sum_pd + pd;
            R.sum_pf = R.sum_pf + pf;
            R.asg_cost = cost_all;
            if (nlk_t == 0) R.cov_val = R.cov_val + val_t;
            R.ncov = ncov_new;
            R.nasg += 1;
            R.r = new_r;
            R.J = J;
            reward = new_r - prev_r;
            R.u = u + 1;
            R.t = 0;
        } else {
            reward = 0.0;
            R.t = t + 1;
            if (R.t >= M) { R.u += 1; R.t = 0; }
        }
    } else {  // :344-352 skip
        R.t = t + 1;
        if (R.t >= M) { R.u += 1; R.t = 0; }
    }
    const bool done = R.u >= N;       // :355-356
    if (done) reward = reward + R.r;  // :361-363 goal reward r(X_final)
    const double is_valid = a == 1 ? (reward != 0.0 ? 1.0 : 0.0) : -1.0;
    if (info_o) write_info(R, env, is_valid, info_o, lane);
    if (lane == 0) {
        if (rew_o) *rew_o = reward;
        if (done_o) *done_o = done ? 1 : 0;
    }
    if (!done) {
        load_cur_pair<TPL, LT>(R, env);
        push_obs(R, lane);
        if (obs_o) write_obs(obs_o, R.w0, R.w1, lane, obs_f16(env));
    } else if (auto_reset) {
        R.ep += 1;
        const int P = env.full_reset_period;
        bool flipped = false;
        if (P > 0 && (R.ep % P) == 0) {  // main_train.py:79 full_reset cadence
            if (env.scene_buffers == 2 && !R.stale) {
                R.sel ^= 1;
                R.stale = 1;
                R.sb = (long long)R.sel * env.E + e;
                if (LT) load_table(R, env, lane);
                flipped = true;
            } else {
                R.err |= 2;  // no fresh spare: keep the scene (state-only reset)
            }
        }
        reset_regs<TPL, LT>(R, env, lane, flipped);
        if (obs_o) write_obs(obs_o, R.w0, R.w1, lane, obs_f16(env));
    } else {
        if (obs_o) write_obs(obs_o, 0.0f, 0.0f, lane, obs_f16(env));  // _get_obs returns zeros when done (:188-189)
    }
}

}  // namespace envdev
}  // namespace uavhip
