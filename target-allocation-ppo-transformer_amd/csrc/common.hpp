// common.hpp -- shared device helpers for libuavhip.so (gfx950 / CDNA4, wave64).
//
// * fp64 mechanics (envs/mechanics.py) written as the reference evaluates them, one rounding
//   per numpy scalar op; the env translation units are built with -ffp-contract=off so no
//   product/sum is fused into an FMA (that would change the last bit of the rewards).
// * Philox4x32-10 counter RNG for on-device scene generation and action sampling.
// * wave-level helpers (readlane of doubles, ballots) for the one-wave-per-env kernels.
// * thread-local last-error plumbing for the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/uavhip.h"

#pragma clang fp contract(off)

namespace uavhip {

// ------------------------------------------------------------------ error plumbing (host)
void set_error(const char* fmt, ...);
int check_launch(const char* what);
int validate_env(const uavhip_env* env, bool need_state);  // env.hip: descriptor checks of the C ABI

// ------------------------------------------------------------------ wave helpers
constexpr int kWave = 64;

// threadIdx.x. In the multi-step rollout TU (rollout_steps.hip, UAVHIP_TID_LAUNDER) it is
// threadIdx.x + an LDS word that holds 0: every __syncthreads (a fence) makes that load opaque, so
// LICM cannot hoist the lane-index expressions of the step loop's body out of the loop (where they
// would be spilled), while GVN still shares them between the barriers of one phase.
#ifdef UAVHIP_TID_LAUNDER
__shared__ unsigned g_tid_zero;
__device__ __forceinline__ unsigned tid_x() { return threadIdx.x + g_tid_zero; }
#else
__device__ __forceinline__ unsigned tid_x() { return threadIdx.x; }
#endif
__device__ __forceinline__ unsigned tid_env() { return tid_x(); }
__device__ __forceinline__ int lane_id() { return tid_x() & (kWave - 1); }

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffull), l);
    const int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t readlane_u(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int ffs64(unsigned long long m) { return __ffsll((long long)m) - 1; }

// ------------------------------------------------------------------ split-product planes
// The second fp16 plane of a split operand, x2 = f16((x - x1) 2^11) with x1 = f16(x).
// Out of range: gfx950's f32 -> f16 conversions (v_cvt_pk_f16_f32 and v_cvt_f16_f32) round to inf at
// |x| >= 65520 (scripts/micro/f16_ovfl.hip: MODE.FP16_OVFL is 0 at kernel start), so x1 = inf and
// x2 = -inf, every product that reads them is +-inf or NaN, and the next LayerNorm turns the token
// row into NaN. What could hide that is a ReLU written as fmaxf (IEEE maxNum returns 0 for NaN):
// the GEMM epilogues use relu_nan (policy.hip) instead, so overflow reaches the outputs.
__device__ __forceinline__ _Float16 f16_lo(float x, _Float16 x1) { return (_Float16)((x - (float)x1) * 2048.f); }
// f16_lo's split four at a time as packed conversions: x1 = f16(x) once (v_cvt_pk_f16_f32), its fp32
// value from the packed halves -- element by element, the compiler converted every x twice (once for
// the store, once for the residual); the same RNE roundings, so bitwise the same planes
typedef float cm_f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 cm_f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void f16_split4(const cm_f32x4 x, cm_f16x4& x1, cm_f16x4& x2) {
    x1 = __builtin_convertvector(x, cm_f16x4);
    x2 = __builtin_convertvector((x - __builtin_convertvector(x1, cm_f32x4)) * 2048.f, cm_f16x4);
}

// ------------------------------------------------------------------ mechanics (fp64)
__device__ __forceinline__ double clipd(double x, double lo, double hi) {
    return x < lo ? lo : (x > hi ? hi : x);
}
__device__ __forceinline__ double norm2(double x, double y) { return sqrt(x * x + y * y); }

// mechanics.py:11-57 calc_angle_score(uav_pos, uav_vel, target_pos)
__device__ __forceinline__ double angle_score(double upx, double upy, double uvx, double uvy, double px,
                                              double py) {
    const double vx = px - upx, vy = py - upy;
    const double dist = norm2(vx, vy);
    if (dist < 1e-6) return 1.0;
    const double nx = vx / dist, ny = vy / dist;
    const double speed = norm2(uvx, uvy);
    double hx = 1.0, hy = 0.0;
    if (!(speed < 1e-6)) { hx = uvx / speed; hy = uvy / speed; }
    const double c = nx * hx + ny * hy;
    const double sigma = acos(clipd(c, -1.0, 1.0));
    double b = 0.002 * dist;
    if (b < 1e-6) b = 1e-6;
    const double q = sigma / (b * M_PI);
    return exp(-(q * q));
}

// mechanics.py:61-68
__device__ __forceinline__ double speed_score(double us, double ts, double K) {
    if (us < 1e-6) return 0.0;
    return clipd(1.0 - (K * ts / us), 0.0, 1.0);
}

// mechanics.py:72-89 (D_mid = 0)
__device__ __forceinline__ double dist_score(double d, double zeta) {
    const double q = (d - 0.0) / zeta;
    return exp(-(q * q));
}

// Per-UAV terms of angle_score / speed_score every pair of the UAV reuses: speed and unit heading
// ([1, 0] when the UAV is still, mechanics.py:37-41).
__device__ __forceinline__ void uav_heading(double uvx, double uvy, double& us, double& hx, double& hy) {
    us = norm2(uvx, uvy);
    hx = 1.0;
    hy = 0.0;
    if (!(us < 1e-6)) { hx = uvx / us; hy = uvy / us; }
}

// calc_damage_prob (mechanics.py:93-114) split into per-UAV, per-target and per-pair work, so the
// pair loop of K1 (and the scene scorer, which evaluates the same functions per pair: bitwise the same
// tables) does as little fp64 work per pair as the formula allows:
//  * per UAV: speed us, unit heading (hx, hy) ([1, 0] when still, mechanics.py:37-41), 1/us, load;
//  * per target: position and K * ts (speed_score's K ts / us evaluates (K ts) / us left to right);
//  * per pair: dist, ONE reciprocal 1/dist (v_rcp_f64 + two Newton steps) for the unit direction and
//    the angle's 1 / (b pi) = (1/dist) / (0.002 pi), acos, exp(-q^2), exp(-(dist / zeta)^2) with
//    1/zeta per kernel, the speed score as (K ts) (1/us).
// The products by reciprocals replace the reference's divisions: each differs from the quotient by
// at most an ulp or two (relative 2^-52 class), far inside the pair bars (5e-12 against the reference,
// tests/test_gpu_env.py); acos and exp are the same ocml functions as before.
struct UavTerms {
    double px, py, hx, hy, us, rus, load, pad;  // 64 B: four ds_read_b128 per UAV in K1's LDS table
};
__device__ __forceinline__ UavTerms uav_terms(double upx, double upy, double uvx, double uvy, double load) {
    UavTerms r;
    r.px = upx;
    r.py = upy;
    uav_heading(uvx, uvy, r.us, r.hx, r.hy);
    r.rus = r.us < 1e-6 ? 0.0 : 1.0 / r.us;
    r.load = load;
    r.pad = 0.0;
    return r;
}
struct PairConst {
    double rzeta, rb, rb0, c1, c2;  // 1/zeta_d, 1/(0.002 pi), 1/(1e-6 pi), C1, C2
};
__device__ __forceinline__ PairConst pair_const(const double* prm) {
    return PairConst{1.0 / prm[UAVHIP_PRM_ZETA_D], 1.0 / (0.002 * M_PI), 1.0 / (1e-6 * M_PI), prm[UAVHIP_PRM_C1],
                     prm[UAVHIP_PRM_C2]};
}
// 1/d for d in [1e-6, 1e30]: the hardware estimate plus two Newton steps (correct to about an ulp;
// no scaling needed in that range)
__device__ __forceinline__ double recip_d(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double damage_pair(const UavTerms& u, double tpx, double tpy, double kts, const PairConst& pc) {
    const double vx = tpx - u.px, vy = tpy - u.py;
    const double dist = norm2(vx, vy);
    double ea = 1.0;
    if (!(dist < 1e-6)) {
        const double rd = recip_d(dist);
        const double c = (vx * rd) * u.hx + (vy * rd) * u.hy;
        const double sigma = acos(clipd(c, -1.0, 1.0));
        // b = max(0.002 dist, 1e-6) (mechanics.py:52-54): sigma / (b pi)
        const double q = sigma * (0.002 * dist < 1e-6 ? pc.rb0 : rd * pc.rb);
        ea = exp(-(q * q));
    }
    const double qd = dist * pc.rzeta;  // dist_score, D_mid = 0
    const double ed = exp(-(qd * qd));
    const double es = u.us < 1e-6 ? 0.0 : clipd(1.0 - kts * u.rus, 0.0, 1.0);
    const double term = pc.c1 * ed + pc.c2 * es;
    const double p = ea * term * u.load;
    return clipd(p, 0.0, 1.0);
}

// mechanics.py:93-114 calc_damage_prob of one pair from the records (the per-wave scene scorer):
// the same per-UAV / per-target / per-pair functions as K1, so bitwise K1's tables
__device__ __forceinline__ double damage_prob(double upx, double upy, double uvx, double uvy, double load,
                                              double tpx, double tpy, double tvx, double tvy, const double* prm) {
    const UavTerms u = uav_terms(upx, upy, uvx, uvy, load);
    return damage_pair(u, tpx, tpy, prm[UAVHIP_PRM_K] * norm2(tvx, tvy), pair_const(prm));
}

// mechanics.py:118-163 calc_penetration_prob (independent of the target)
__device__ __forceinline__ double penetration_prob(double upx, double upy, double uvx, double uvy,
                                                   const double* nfz, int kn, const double* ip, const double* iv,
                                                   int ki, const double* prm) {
    double p = 1.0;
    const double us = norm2(uvx, uvy);
    for (int j = 0; j < kn; ++j) {
        const double ox = nfz[2 * j], oy = nfz[2 * j + 1];
        const double ea = angle_score(upx, upy, uvx, uvy, ox, oy);
        const double ed = dist_score(norm2(upx - ox, upy - oy), prm[UAVHIP_PRM_ZETA_OBS]);
        const double pn = (1.0 - ea) * (1.0 - ed);
        p *= clipd(pn, 0.0, 1.0);
    }
    for (int j = 0; j < ki; ++j) {
        const double ox = ip[2 * j], oy = ip[2 * j + 1];
        const double ea = angle_score(upx, upy, uvx, uvy, ox, oy);
        const double ed = dist_score(norm2(upx - ox, upy - oy), prm[UAVHIP_PRM_ZETA_OBS]);
        const double es = speed_score(us, norm2(iv[2 * j], iv[2 * j + 1]), prm[UAVHIP_PRM_K]);
        const double term = prm[UAVHIP_PRM_C3] * (1.0 - ed) + prm[UAVHIP_PRM_C4] * es;
        const double pi = (1.0 - ea) * term;
        p *= clipd(pi, 0.0, 1.0);
    }
    return p;
}

// ------------------------------------------------------------------ Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
// 53-bit uniform in [0, 1) from two words (numpy random_sample resolution)
__device__ __forceinline__ double u01(uint32_t a, uint32_t b) {
    const unsigned long long v = (((unsigned long long)a << 32) | b) >> 11;
    return (double)v * 0x1.0p-53;
}
// 24-bit uniform in [0, 1) for fp32 sampling
__device__ __forceinline__ float u01f(uint32_t a) { return (float)(a >> 8) * 0x1.0p-24f; }

}  // namespace uavhip
