// env_group.hpp -- the env step with TWO envs per wave (32 lanes each), for multi-step launches of
// envs with N, M <= 32 (env.hip k_env_step_g). Same algorithm, same fp64 operation order and the
// same state layout as env_device.hpp (whose one-env-per-wave kernels remain the general path);
// the point is throughput: the per-step scalar work (fp64 obs features, info, pointer logic) is
// wave-uniform there, so one VALU instruction did one env's work -- here it does two.
//
// Mapping: lane = 32 g + j; group g owns env e_g; lane j holds target j and UAV j of it. "Group-
// uniform" values (the pointer, r(X), sums ...) are VGPRs equal across a group. Values at a
// group-dependent lane index (target t, UAV u) are fetched with ds_bpermute inside the group;
// the revenue sum over locked targets (list order, the reference's fp64 order) walks the union of
// both groups' locked sets with readlanes of both halves. Control flow that differs between the
// two envs (assign / skip, accept / reject, done) runs under exec masks.
#pragma once
#include "env_device.hpp"

#pragma clang fp contract(off)

namespace uavhip {
namespace envgrp {
using namespace envdev;

constexpr int L = 32;  // lanes per env

// Attribution builds of the fused rollout's env step (make EXP=n, profiling only, WRONG results;
// scripts/profile_env_attrib.sh): each compiles out one group of the step's global accesses so its
// PMC bytes and time can be priced by difference against the product build.
//   21 scene values (tgt_value / uav_cost / p_pen of both buffers)   22 per-target / per-UAV state
//   23 istate / dstate rows    24 the env's own window    25 the state stores (gstore_regs)
//   26 the step's outputs (obs / reward / done / info)    27 the dependent p_dmg load of the new pair
#ifndef UAVHIP_EXP
#define UAVHIP_EXP 0
#endif
constexpr int kAttr = UAVHIP_EXP;
#ifndef GTR  // phase stamps inside gstep (policy.hip, make TRACE=1 ENVFINE=1 only)
#define GTR(id) do {} while (0)
#endif
// (24: the window registers take 1.0 instead of memory, so no later window row is padding: a zero
// window would turn the policy's ring loads of padded positions into reads of one hot row, policy.hip)
constexpr int kWin = 96;  // LDS scratch per env: window at [2, 72), new row at [72, 86)

struct GRegs {
    // lane j: target j (list order) and UAV j of this group's env
    double nhf, nhp, tc, val;
    int nlk, asg;
    double ucost, ppen;
    // group-uniform
    int u, t, ncov, nasg, ep, err, sel, stale, gen;
    long long sb;
    double r, J, asg_cost, cov_val, tot_cost, tot_val, sum_pd, sum_pf, pd_cur, pp_cur;
    double den_c, rcp_c, den_v, rcp_v, rcp_m;
    // single-step use (TAB = false, the fused rollout): which per-target / per-UAV entries the step
    // changed, so gstore_delta writes only those -- bit 0: all (a reset), bit 1: target ct and UAV cu
    // (an accepted assign); group-uniform
    int dmask, ct, cu;
    // window element j in w0, 32 + j in w1, 64 + j (j < 6) in w2
    float w0, w1, w2;
    double* tab;   // LDS p_dmg table of this env [N][M]
    float* win;    // LDS scratch [kWin] of this env
};

__device__ __forceinline__ int gbase() { return tid_env() & 32; }
__device__ __forceinline__ int gsh_i(int v, int j) { return __shfl(v, gbase() + j); }
__device__ __forceinline__ float gsh_f(float v, int j) { return __shfl(v, gbase() + j); }
__device__ __forceinline__ double gsh_d(double v, int j) {
    const int src = gbase() + j;
    const int lo = __shfl(__double2loint(v), src), hi = __shfl(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
// value at lane jj (wave-uniform index) of this lane's group: readlanes of both halves
__device__ __forceinline__ double grl_d(double v, int jj) {
    const double a = readlane_d(v, jj), b = readlane_d(v, L + jj);
    return gbase() ? b : a;
}
// this lane's group bits of a wave ballot
__device__ __forceinline__ unsigned gbits(unsigned long long m) { return (unsigned)(m >> gbase()); }

__device__ __forceinline__ void gset_scene_divisors(GRegs& R) {
    R.den_c = R.tot_cost + 1e-6;
    R.rcp_c = 1.0 / R.den_c;
    R.den_v = R.tot_val + 1e-6;
    R.rcp_v = 1.0 / R.den_v;
}

__device__ void gload_scene_regs(GRegs& R, const uavhip_env& env, int j) {
    R.val = j < env.M ? env.tgt_value[R.sb * env.M + j] : 0.0;
    R.ucost = j < env.N ? env.uav_cost[R.sb * env.N + j] : 0.0;
    R.ppen = j < env.N ? env.p_pen[R.sb * env.N + j] : 0.0;
    drain_loads();
}

// TAB = false (single-step use inside the fused rollout launch): pair probabilities are read from
// the global p_dmg table instead of an LDS copy. A compile-time choice: a global load that MAY be
// in flight in the step loop would make every later use wait for all the step's stores.
template <bool TAB = true>
__device__ void gload_table(GRegs& R, const uavhip_env& env, int j) {
    if (!TAB) return;
    const int NM = env.N * env.M;
    const double* src = env.p_dmg + R.sb * NM;
    for (int i = j; i < NM; i += L) R.tab[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool TAB = true>
__device__ __forceinline__ void gload_cur_pair(GRegs& R, const uavhip_env& env) {
    if (R.u < env.N) {
        R.pd_cur = TAB ? R.tab[R.u * env.M + R.t]
                       : (kAttr == 27 ? 0.5 : env.p_dmg[(R.sb * env.N + R.u) * env.M + R.t]);
        R.pp_cur = gsh_d(R.ppen, R.u);
    } else {
        R.pd_cur = 0.0;
        R.pp_cur = 0.0;
    }
}

// mechanics.py:185-241 + uav_env.py:194-242 for the current pointer (envdev::push_obs)
__device__ void gpush_obs(GRegs& R, int j) {
    const int t = R.t;
    const double val = gsh_d(R.val, t);
    const double tc = gsh_d(R.tc, t);
    const double nhf = gsh_d(R.nhf, t);
    const double nhp = gsh_d(R.nhp, t);
    const double ucost = gsh_d(R.ucost, R.u);
    const double chi_c = div_by(R.asg_cost, R.den_c, R.rcp_c);
    const double chi_v = div_by(R.cov_val, R.den_v, R.rcp_v);
    const double chi_mc = div_by(tc, R.den_c, R.rcp_c);
    const double pjp = 1.0 - nhf;
    const double pjp_pure = 1.0 - nhp;
    const double prev_rev = pjp * val;
    const double p_km = R.pd_cur * R.pp_cur;
    const double p_pure = R.pd_cur;
    const double hat_p = 1.0 - (1.0 - pjp) * (1.0 - p_km);
    const double hat_pp = 1.0 - (1.0 - pjp_pure) * (1.0 - p_pure);
    const double hat_G = hat_p * val;
    const double d_pkm = p_pure - p_km;
    const double d_pm = hat_pp - hat_p;
    const double d_G = (hat_pp * val) - hat_G;
    // the window shifted by one row through LDS: element i of the new window = win[16 + i]
    float* w = R.win;
    w[2 + j] = R.w0;
    w[2 + L + j] = R.w1;
    if (j < kObs - 2 * L) w[2 + 2 * L + j] = R.w2;
    if (j == 0) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<f32x4*>(w + 72) = f32x4{(float)ucost / 2.0f, (float)val / 16.0f, (float)chi_c, (float)chi_v};
        *reinterpret_cast<f32x4*>(w + 76) = f32x4{(float)chi_mc, (float)p_km, (float)pjp, (float)hat_p};
        *reinterpret_cast<f32x4*>(w + 80) =
            f32x4{(float)prev_rev / 16.0f, (float)hat_G / 16.0f, (float)d_pkm, (float)d_pm};
        // the constant feature materialised here: left to itself the compiler takes 1.0f from the high
        // half of a spilled register pair, a scratch round trip on the step's dependency chain (measured
        // -0.5 us per rollout step, same box)
        float one;
        asm volatile("v_mov_b32 %0, 1.0" : "=v"(one));
        *reinterpret_cast<f32x2*>(w + 84) = f32x2{(float)d_G / 16.0f, one};
    }
    R.w0 = w[16 + j];
    R.w1 = w[16 + L + j];
    R.w2 = j < kObs - 2 * L ? w[16 + 2 * L + j] : 0.0f;
}

__device__ __forceinline__ void gwrite_obs(float* o, const GRegs& R, int j, bool zero, bool h) {
    const float a = zero ? 0.0f : R.w0, b = zero ? 0.0f : R.w1, c = zero ? 0.0f : R.w2;
    if (h) {  // UAVHIP_ENV_OBS_F16
        _Float16* q = reinterpret_cast<_Float16*>(o);
        q[j] = (_Float16)a;
        q[L + j] = (_Float16)b;
        if (j < kObs - 2 * L) q[2 * L + j] = (_Float16)c;
    } else {
        o[j] = a;
        o[L + j] = b;
        if (j < kObs - 2 * L) o[2 * L + j] = c;
    }
}

__device__ void gwrite_info(const GRegs& R, double is_valid, double* o, int j) {
    const int cnt = R.nasg;
    const double y = cnt > 0 ? 1.0 / (double)cnt : 0.0;  // RN(1 / cnt): envdev's rcp_n[cnt - 1]
    const double avg_d = cnt > 0 ? div_by(R.sum_pd, (double)cnt, y) : 0.0;
    const double avg_f = cnt > 0 ? div_by(R.sum_pf, (double)cnt, y) : 0.0;
    if (j == 0) {
        double2* q = reinterpret_cast<double2*>(o);
        q[0] = make_double2(R.J, (double)R.ncov);
        q[1] = make_double2(is_valid, avg_d);
        q[2] = make_double2(avg_f, (double)R.u);
        q[3] = make_double2((double)R.t, (double)R.ep);
    }
}

// uav_env.py:42-63,175-182 (envdev::reset_regs)
template <bool TAB = true>
__device__ void greset_regs(GRegs& R, const uavhip_env& env, int j, bool scene) {
    R.nhf = 1.0;
    R.nhp = 1.0;
    R.tc = 0.0;
    R.nlk = 0;
    R.asg = -1;
    R.u = 0; R.t = 0; R.ncov = 0; R.nasg = 0;
    R.r = 0.0; R.J = 0.0; R.asg_cost = 0.0; R.cov_val = 0.0;
    R.sum_pd = 0.0; R.sum_pf = 0.0;
    if (scene) {
        gload_scene_regs(R, env, j);
        // total_swarm_cost in generation order (uav_env.py:118), total value in list order (:198)
        double tc = 0.0;
        for (int k = 0; k < env.N; ++k) tc = tc + grl_d(R.ucost, k);
        double tv = 0.0;
        for (int k = 0; k < env.M; ++k) tv = tv + grl_d(R.val, k);
        R.tot_cost = tc;
        R.tot_val = tv;
        gset_scene_divisors(R);
    }
    R.w0 = 0.0f;
    R.w1 = 0.0f;
    R.w2 = 0.0f;
    gload_cur_pair<TAB>(R, env);
    gpush_obs(R, j);
}

// Single-step use (the fused rollout launch): register state in one load round, scene-dependent
// values read from both scene buffers and selected after the wait (as envdev::load_regs<PF>).
// gload_issue only issues the loads (overlapped with the critic head); gload_finish consumes them.
// The per-env scalars (istate / dstate rows) arrive as one vector load each -- lane j of a group
// holds element j -- and are broadcast in gload_finish: 2 memory instructions instead of 18.
struct GPending {
    double valb[2], ucb[2], ppb[2];
    int isv;
    double dsv;
};
__device__ __forceinline__ int grl_i(int v, int jj) {
    const int a = __builtin_amdgcn_readlane(v, jj), b = __builtin_amdgcn_readlane(v, L + jj);
    return gbase() ? b : a;
}
__device__ __forceinline__ void gload_issue(GRegs& R, GPending& q, const uavhip_env& env, int e, int j) {
    const int N = env.N, M = env.M;
    const int* is = env.istate + (long long)e * UAVHIP_IST_COUNT;
    const double* ds = env.dstate + (long long)e * UAVHIP_DST_COUNT;
    const int nb = env.scene_buffers;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const long long sb = (long long)(b < nb ? b : 0) * env.E + e;
        if (kAttr == 21) {
            q.valb[b] = 4.0 + j;
            q.ucb[b] = 1.0;
            q.ppb[b] = 0.9;
            continue;
        }
        q.valb[b] = j < M ? env.tgt_value[sb * M + j] : 0.0;
        q.ucb[b] = j < N ? env.uav_cost[sb * N + j] : 0.0;
        q.ppb[b] = j < N ? env.p_pen[sb * N + j] : 0.0;
    }
    if (kAttr == 23) {
        q.isv = j == UAVHIP_IST_EPISODE ? 1 : 0;
        q.dsv = j == UAVHIP_DST_TOTAL_COST || j == UAVHIP_DST_TOTAL_VALUE ? 20.0 : 0.0;
    } else {
        q.isv = is[j < UAVHIP_IST_COUNT ? j : 0];
        q.dsv = ds[j < UAVHIP_DST_COUNT ? j : 0];
    }
    const long long o = (long long)e * M + j;
    const bool v = j < M;
    if (kAttr == 22) {
        R.nhf = 1.0; R.nhp = 1.0; R.tc = 0.0; R.nlk = 0; R.asg = -1;
    } else {
        R.nhf = v ? env.nh_final[o] : 1.0;
        R.nhp = v ? env.nh_pure[o] : 1.0;
        R.tc = v ? env.t_cost[o] : 0.0;
        R.nlk = v ? env.n_lock[o] : 0;
        R.asg = j < N ? env.assigned[(long long)e * N + j] : -1;
    }
    const float* w = env.window + (long long)e * kObs;
    if (kAttr == 24) {
        R.w0 = R.w1 = R.w2 = 1.0f;
    } else {
        R.w0 = w[j];
        R.w1 = w[L + j];
        R.w2 = j < kObs - 2 * L ? w[2 * L + j] : 0.0f;
    }
}
__device__ __forceinline__ void gload_finish(GRegs& R, const GPending& q, const uavhip_env& env, int e, int j) {
    const int N = env.N, M = env.M;
    const int sel_raw = grl_i(q.isv, UAVHIP_IST_SCENE_SEL);
    R.stale = grl_i(q.isv, UAVHIP_IST_SCENE_STALE);
    R.gen = grl_i(q.isv, UAVHIP_IST_SCENE_GEN);
    R.u = grl_i(q.isv, UAVHIP_IST_UAV_IDX);
    R.t = grl_i(q.isv, UAVHIP_IST_TARGET_IDX);
    R.ncov = grl_i(q.isv, UAVHIP_IST_N_COVERED);
    R.nasg = grl_i(q.isv, UAVHIP_IST_N_ASSIGNED);
    R.ep = grl_i(q.isv, UAVHIP_IST_EPISODE);
    R.err = grl_i(q.isv, UAVHIP_IST_ERROR);
    R.r = grl_d(q.dsv, UAVHIP_DST_R);
    R.J = grl_d(q.dsv, UAVHIP_DST_J);
    R.asg_cost = grl_d(q.dsv, UAVHIP_DST_ASG_COST);
    R.cov_val = grl_d(q.dsv, UAVHIP_DST_COV_VALUE);
    R.tot_cost = grl_d(q.dsv, UAVHIP_DST_TOTAL_COST);
    R.tot_val = grl_d(q.dsv, UAVHIP_DST_TOTAL_VALUE);
    R.sum_pd = grl_d(q.dsv, UAVHIP_DST_SUM_PDMG);
    R.sum_pf = grl_d(q.dsv, UAVHIP_DST_SUM_PFIN);
    R.pd_cur = grl_d(q.dsv, UAVHIP_DST_PD_CUR);
    R.sel = env.scene_buffers == 2 ? (sel_raw & 1) : 0;
    R.sb = (long long)R.sel * env.E + e;
    R.dmask = 0;
    R.ct = R.cu = -1;
    R.val = R.sel ? q.valb[1] : q.valb[0];
    R.ucost = R.sel ? q.ucb[1] : q.ucb[0];
    R.ppen = R.sel ? q.ppb[1] : q.ppb[0];
    gset_scene_divisors(R);
    R.rcp_m = 1.0 / (double)M;
    R.pp_cur = R.u < N ? gsh_d(R.ppen, R.u) : 0.0;
}
// Multi-step launches (once per launch): the plain order, scene index first (fewer live registers).
__device__ void gload_regs(GRegs& R, const uavhip_env& env, int e, int j) {
    const int N = env.N, M = env.M;
    load_scene_index(env, e, R.sel, R.stale, R.gen, R.sb);
    R.val = j < M ? env.tgt_value[R.sb * M + j] : 0.0;
    R.ucost = j < N ? env.uav_cost[R.sb * N + j] : 0.0;
    R.ppen = j < N ? env.p_pen[R.sb * N + j] : 0.0;
    const long long o = (long long)e * M + j;
    const bool v = j < M;
    R.nhf = v ? env.nh_final[o] : 1.0;
    R.nhp = v ? env.nh_pure[o] : 1.0;
    R.tc = v ? env.t_cost[o] : 0.0;
    R.nlk = v ? env.n_lock[o] : 0;
    R.asg = j < N ? env.assigned[(long long)e * N + j] : -1;
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
    R.sum_pd = ds[UAVHIP_DST_SUM_PDMG];
    R.sum_pf = ds[UAVHIP_DST_SUM_PFIN];
    R.pd_cur = ds[UAVHIP_DST_PD_CUR];
    const float* w = env.window + (long long)e * kObs;
    R.w0 = w[j];
    R.w1 = w[L + j];
    R.w2 = j < kObs - 2 * L ? w[2 * L + j] : 0.0f;
    drain_loads();
    gset_scene_divisors(R);
    R.rcp_m = 1.0 / (double)M;
    R.pp_cur = R.u < N ? gsh_d(R.ppen, R.u) : 0.0;
}

__device__ void gstore_regs(const GRegs& R, const uavhip_env& env, int e, int j) {
    const int N = env.N, M = env.M;
    if (kAttr == 25) return;
    if (j < M) {
        const long long o = (long long)e * M + j;
        env.nh_final[o] = R.nhf;
        env.nh_pure[o] = R.nhp;
        env.t_cost[o] = R.tc;
        env.n_lock[o] = R.nlk;
    }
    if (j < N) env.assigned[(long long)e * N + j] = R.asg;
    if (j == 0) {
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
    w[j] = R.w0;
    w[L + j] = R.w1;
    if (j < kObs - 2 * L) w[2 * L + j] = R.w2;
}

// gstore_regs for the single-step fused rollout: the per-target / per-UAV arrays only where the step
// changed them (R.dmask: after an accepted assign the one target's nh_final / nh_pure / t_cost / n_lock
// and the one UAV's assigned entry, after a reset all of them, else none) -- the same memory state as
// gstore_regs, with 8-20 instead of 960 bytes per env-step of those arrays on most steps.
__device__ void gstore_delta(const GRegs& R, const uavhip_env& env, int e, int j) {
    const int N = env.N, M = env.M;
    if (kAttr == 25) return;
    const bool all = (R.dmask & 1) != 0;
    const bool tgt = all ? j < M : ((R.dmask & 2) != 0 && j == R.ct);
    const bool uav = all ? j < N : ((R.dmask & 2) != 0 && j == R.cu);
    if (tgt) {
        const long long o = (long long)e * M + j;
        env.nh_final[o] = R.nhf;
        env.nh_pure[o] = R.nhp;
        env.t_cost[o] = R.tc;
        env.n_lock[o] = R.nlk;
    }
    if (uav) env.assigned[(long long)e * N + j] = R.asg;
    if (j == 0) {
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
    w[j] = R.w0;
    w[L + j] = R.w1;
    if (j < kObs - 2 * L) w[2 * L + j] = R.w2;
}

// One UAVEnv.step (uav_env.py:295-435) of this group's env (envdev::step_once).
template <bool TAB = true>
__device__ void gstep(GRegs& R, const uavhip_env& env, int e, int j, int a, int auto_reset, float* obs_o,
                      double* rew_o, uint8_t* done_o, double* info_o) {
    const int N = env.N, M = env.M;
    if (kAttr == 26) {  // the scalar outputs only: without the obs window the next inputs would be padding
        rew_o = nullptr; done_o = nullptr; info_o = nullptr;
    }
    if (R.u >= N) {  // stepping a finished env: the reference raises IndexError (:296)
        R.err |= 1;
        if (obs_o) gwrite_obs(obs_o, R, j, true, obs_f16(env));
        if (j == 0) {
            if (rew_o) *rew_o = 0.0;
            if (done_o) *done_o = 1;
        }
        if (info_o && j < UAVHIP_INFO_COUNT) info_o[j] = 0.0;
        return;
    }
    const int u = R.u, t = R.t;
    const double prev_r = R.r;  // :301
    double reward = 0.0;
    if (a == 1) {  // :306-342 tentative assign, accept iff r(X') >= r(X)
        const double pd = R.pd_cur, pp = R.pp_cur;
        const double pf = pd * pp;
        const double nhf_t = gsh_d(R.nhf, t);
        const int nlk_t = gsh_i(R.nlk, t);
        const double nhf_new = nhf_t * (1.0 - pf);
        const int ncov_new = R.ncov + (nlk_t == 0 ? 1 : 0);
        GTR(40);
        // J(X') revenue: sum over locked targets in list order (:252-265)
        const bool mine = j == t;
        const double nh = mine ? nhf_new : R.nhf;
        const double term = (1.0 - nh) * R.val;
        const unsigned long long m = ballot(j < M && (R.nlk > 0 || mine));
        const unsigned mine_bits = gbits(m);
        unsigned any = (unsigned)m | (unsigned)(m >> 32);  // both groups' locked targets
        double rev = 0.0;
        while (any) {
            const int jj = __ffs(any) - 1;
            any &= any - 1;
            const double tj = grl_d(term, jj);
            if ((mine_bits >> jj) & 1u) rev = rev + tj;
        }
        GTR(41);
        const double ucost_u = gsh_d(R.ucost, u);
        const double cost_all = R.asg_cost + ucost_u;  // exact for costs in {1, 1.25}
        const double J = rev - (env.prm[UAVHIP_PRM_OMEGA] * cost_all);
        const double new_r = (ncov_new == M) ? 2.0 * J : J * div_by((double)ncov_new, (double)M, R.rcp_m);
        if (new_r >= prev_r) {
            const double val_t = gsh_d(R.val, t);
            if (mine) {
                R.nhf = nhf_new;
                R.nhp = R.nhp * (1.0 - pd);
                R.tc = R.tc + ucost_u;
                R.nlk = R.nlk + 1;
            }
            if (j == u) R.asg = t;
            if (!TAB) {
                R.dmask |= 2;
                R.ct = t;
                R.cu = u;
            }
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
    GTR(42);
    const bool done = R.u >= N;       // :355-356
    if (done) reward = reward + R.r;  // :361-363 goal reward r(X_final)
    const double is_valid = a == 1 ? (reward != 0.0 ? 1.0 : 0.0) : -1.0;
    // the next observation row before the step's stores: with the stores ahead of the pair's load the
    // wait for the load is a wait for them too (one in-order vector memory counter)
    if (!done) {
        GTR(43);
        gload_cur_pair<TAB>(R, env);
        gpush_obs(R, j);
        GTR(44);
    }
    if (info_o) gwrite_info(R, is_valid, info_o, j);  // before a reset clears the registers
    if (j == 0) {
        if (rew_o) *rew_o = reward;
        if (done_o) *done_o = done ? 1 : 0;
    }
    if (!done) {
        if (obs_o) gwrite_obs(obs_o, R, j, false, obs_f16(env));
        GTR(45);
    } else if (auto_reset) {
        R.ep += 1;
        const int P = env.full_reset_period;
        bool flipped = false;
        if (P > 0 && (R.ep % P) == 0) {  // main_train.py:79 full_reset cadence
            if (env.scene_buffers == 2 && !R.stale) {
                R.sel ^= 1;
                R.stale = 1;
                R.sb = (long long)R.sel * env.E + e;
                gload_table<TAB>(R, env, j);
                flipped = true;
            } else {
                R.err |= 2;  // no fresh spare: keep the scene (state-only reset)
            }
        }
        greset_regs<TAB>(R, env, j, flipped);
        if (!TAB) R.dmask |= 1;
        if (obs_o) gwrite_obs(obs_o, R, j, false, obs_f16(env));
    } else {
        if (obs_o) gwrite_obs(obs_o, R, j, true, obs_f16(env));  // _get_obs returns zeros when done (:188-189)
    }
}

}  // namespace envgrp
}  // namespace uavhip
