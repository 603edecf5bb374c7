// env_replay.hpp -- K2r: the env-only multi-step launch (uavhip_env_step, T > 1, auto-reset) when
// COST_WEIGHT_OMEGA == 0, the reference's setting (config.py:53) and that of every BASELINE config.
//
// Why it can be replayed: with omega = 0 a tentative assign is always accepted (uav_env.py:317).
// J(X') >= J(X) because the lock multiplies one not-hit product by (1 - p) in [0, 1] and the
// list-order sum gains no negative term, and IEEE rounding is monotone; N0 never shrinks; so
// r(X') = J' N0' / M (or 2 J' at full coverage) >= r(X). The pointer walk, the lock sequence and the
// episode ends are then a function of the action stream alone, and K2's step-to-step dependency
// chain splits into a cheap integer walk and fp64 work that is independent across steps.
//
// One wave per env, chunks of up to C steps (lane i = step i of the chunk):
//   walk    lane = step, from the chunk's action bits alone (ballots and popcounts): pointer before /
//           after, assign, done, episode, full-reset scene flips -- a chunk ends right after a flip,
//           the rest runs on the new scene;
//   fold    lane = assign: the per-target not-hit products and locker costs, the info running sums
//           -- step_once's operations -- as ordered chains over lanes (round r settles chain
//           position r from position r - 1: bitwise the sequential values), lock counts and
//           coverage by popcounts over per-target ballots;
//   replay  lane = step: J(X) after its assign as the list-order sum over every target's current
//           not-hit product (gathered from the assign lanes; unlocked targets add +0.0, as in
//           _calc_J_X), r(X), reward, info and the observation row of the pointer after the step
//           (obs_row); rows -> LDS;
//   store   16 lanes per step, 4 steps at a time: each step's window out of the row table (an episode
//           start zeroes the older slots; rows before the chunk come from the carried window).
// A workgroup holds 4 envs: 4 compute waves (walk, fold, replay, rewards / info) and 4 store waves.
// Rows and the carried window of a chunk are double-buffered in LDS; after a workgroup barrier the
// store waves write chunk k's windows while the compute waves run chunk k + 1, so the window stores
// (80 % of the bytes) overlap the latency-bound fold instead of following it on the same wave.
// Every output and the carried state are bitwise those of step_once (tests: test_env_replay_*).
#pragma once
#include "env_device.hpp"

#pragma clang fp contract(off)

namespace uavhip {
namespace envrep {
using namespace envdev;

constexpr int kWavesPerBlock = 4;                 // envs (compute waves) per workgroup
constexpr int kBlock = 2 * kWavesPerBlock * kWave;  // + one store wave per env
constexpr int kRowStride = 18;   // floats per observation row in LDS (14 used): 8-byte aligned rows whose
                                 // stride (18 dwords) spreads 32 lanes' b64 reads over distinct banks
constexpr int kMaxM = 32;        // targets: the packed step record holds 7-bit pointers, ncov < 256
constexpr int kSeq = UAVHIP_SEQ_LEN;

// LDS per env, in doubles, every region an even count (16-byte aligned): p_dmg table [N][M], then
// twice (chunk k and k + 1): C observation rows, the carried window (70 floats).
__host__ __device__ constexpr size_t even(size_t x) { return (x + 1) & ~(size_t)1; }
template <int C>
__host__ __device__ constexpr size_t buf_doubles() { return (size_t)C * kRowStride / 2 + 36; }
template <int C>
__host__ __device__ constexpr size_t wave_doubles(int N, int M) {
    return even((size_t)N * M) + 2 * buf_doubles<C>();
}

__device__ __forceinline__ double shfl_d(double v, int src) {
    const int lo = __shfl(__double2loint(v), src), hi = __shfl(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
// old with lane i's element replaced by the wave-uniform v (a v_cndmask per dword)
template <class V>
__device__ __forceinline__ V put_lane(V v, int i, V old) {
    return lane_id() == i ? v : old;
}
__device__ __forceinline__ int top_bit(unsigned long long m) { return m ? 63 - __builtin_clzll(m) : -1; }
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
    return (unsigned long long)(unsigned)readlane_i((int)(unsigned)v, l) |
           ((unsigned long long)(unsigned)readlane_i((int)(unsigned)(v >> 32), l) << 32);
}
__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
    return (unsigned long long)(unsigned)__shfl((int)(unsigned)v, src) |
           ((unsigned long long)(unsigned)__shfl((int)(unsigned)(v >> 32), src) << 32);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// LDS written by some lanes and read by others of the same wave: complete and order them
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// packed step record (lane i): pointer before (ub, tb), after the action (ua, ta; ua == N at an
// episode end), assign, done
__device__ __forceinline__ int rec_pack(int ub, int tb, int ua, int ta, int a, int d) {
    return ub | (tb << 7) | (ua << 14) | (ta << 21) | (a << 28) | (d << 29);
}

#ifdef UAVHIP_POLICY_TRACE
// TRACE=1 builds: s_memtime cycles per phase summed over a wave's chunks (walk, fold, replay,
// carried state + flip, store, chunk count) for the first kTraceEnvs envs; uavhip_env_trace reads them
constexpr int kTraceEnvs = 4096, kTracePhases = 6;
__device__ unsigned long long g_etrace[kTraceEnvs * kTracePhases];
#define ETR_DECL unsigned long long etr[kTracePhases] = {0, 0, 0, 0, 0, 0}, etr_t = __builtin_amdgcn_s_memtime();
#define ETR(k)                                                  \
    do {                                                        \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        etr[k] += now_ - etr_t;                                 \
        etr_t = now_;                                           \
    } while (0)
#define ETR_END                                                                 \
    if (lane == 0 && e < kTraceEnvs)                                            \
        for (int k_ = 0; k_ < kTracePhases; ++k_) g_etrace[e * kTracePhases + k_] = etr[k_];
#else
#define ETR_DECL
#define ETR(k)
#define ETR_END
#endif

// The windows of one chunk (store waves): window slot j of step s holds the row of chunk step
// k = s - 4 + j: zero before the latest episode start d <= s (the reset row of step d opens the
// episode), from the carried window for k < 0 when the episode began before the chunk. 16 lanes per
// step write float pairs 16 k + j16 of its window: 3 instructions cover 4 steps, each touching 4
// runs of 128 contiguous bytes (one lane per step, 8 bytes each, touched 64 lines per instruction:
// 1.5x slower at configs[1]); the lane's pair, its window slot and column are fixed, and per group
// of 16 steps every LDS read is issued before the first store.
__device__ __forceinline__ void store_windows(float* __restrict__ obs_out, bool h, long long E, int e, int s0, int n,
                                              unsigned long long dbits, const float* rows, const float* carry) {
    const int lane = lane_id();
    const int g4 = lane >> 4, j16 = lane & 15;
    int jj[3], qq[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int p = 16 * k + j16;  // float pair of the 70-float window
        jj[k] = p / (kDim / 2);
        qq[k] = p - jj[k] * (kDim / 2);
    }
    const long long ostride = 4 * E * kObs;  // 4 steps, in elements
    for (int s16 = 0; s16 < n; s16 += 16) {
        float2 v[4][3];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int s = s16 + 4 * r + g4;
            const int d = top_bit(dbits & (s >= 63 ? ~0ull : (2ull << s) - 1));
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int kk = s - (kSeq - 1) + jj[k];  // chunk step whose row fills slot jj
                const float* src = kk >= 0 ? rows + kk * kRowStride : carry + (kSeq + kk) * kDim;
                v[r][k] = (s < n && 16 * k + j16 < kObs / 2) ? reinterpret_cast<const float2*>(src)[qq[k]]
                                                             : make_float2(0.0f, 0.0f);
                if (d >= 0 && kk < d) v[r][k] = make_float2(0.0f, 0.0f);
            }
        }
        const long long o0 = ((long long)(s0 + s16 + g4) * E + e) * kObs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int s = s16 + 4 * r + g4;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int p = 16 * k + j16;
                if (s < n && p < kObs / 2) {
                    const long long oi = o0 + r * ostride + 2 * p;
                    if (h) {  // binary16, round to nearest even (write_obs's conversion)
                        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
                        *reinterpret_cast<f16x2*>(reinterpret_cast<_Float16*>(obs_out) + oi) =
                            f16x2{(_Float16)v[r][k].x, (_Float16)v[r][k].y};
                    } else {
                        *reinterpret_cast<float2*>(obs_out + oi) = v[r][k];
                    }
                }
            }
        }
    }
}

template <int C>
__global__ __launch_bounds__(kBlock) void k_env_replay(uavhip_env env, const int8_t* __restrict__ actions, int T,
                                                       float* __restrict__ obs_out, double* __restrict__ reward_out,
                                                       uint8_t* __restrict__ done_out, double* __restrict__ info_out) {
    static_assert(C <= kWave, "one step per lane");
    extern __shared__ __attribute__((aligned(16))) double s_dyn[];
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock * 16];
    // per buffer and env: chunk start, steps, episode-end bits (lo, hi), more chunks follow
    __shared__ int s_meta[2][kWavesPerBlock][8];
    const int lane = lane_id(), wv = threadIdx.x >> 6, we = wv & (kWavesPerBlock - 1);
    const int e = blockIdx.x * kWavesPerBlock + we;
    const bool live = e < env.E;
    const int N = env.N, M = env.M;
    double* base = s_dyn + (size_t)we * wave_doubles<C>(N, M);
    float* const bufs = reinterpret_cast<float*>(base + even((size_t)N * M));  // [2][C rows | carried window]
    constexpr int kBufFloats = 2 * (int)buf_doubles<C>();
    const long long E = env.E;
    const bool h = obs_f16(env);
    if (wv >= kWavesPerBlock) {  // the store wave of env e: chunk k's windows after barrier k
        for (int k = 0;; ++k) {
            __syncthreads();
            const int* m = s_meta[k & 1][we];
            const int s0 = m[0], n = m[1];
            const unsigned long long db = (unsigned long long)(unsigned)m[2] | ((unsigned long long)(unsigned)m[3] << 32);
            bool more = false;
#pragma unroll
            for (int j = 0; j < kWavesPerBlock; ++j) more = more || s_meta[k & 1][j][4] != 0;
            if (obs_out && n > 0) {
                const float* rows = bufs + (k & 1) * kBufFloats;
                store_windows(obs_out, h, E, e, s0, n, db, rows, rows + C * kRowStride);
            }
            if (!more) return;
        }
    }
    EnvRegs<1> R;
    R.tab = base;
    R.row = s_row + we * 16;
    bool done = !live, stored = !live;
    if (live) {
        load_regs<1>(R, env, e, lane);
        load_table(R, env, lane);
        if (R.u >= N) {  // finished before the launch (a previous launch without auto-reset): K2's error path
            for (int s = 0; s < T; ++s) {
                const long long se = (long long)s * E + e;
                step_once<1, true>(R, env, e, lane, 0, 1, obs_out ? obs_at(obs_out, se, h) : nullptr,
                                   reward_out ? reward_out + se : nullptr, done_out ? done_out + se : nullptr,
                                   info_out ? info_out + se * UAVHIP_INFO_COUNT : nullptr);
            }
            store_regs(R, env, e, lane);
            done = stored = true;
        }
    }
    // window element handled by this lane for the carried window: element lane, and 64 + lane (lane < 6)
    const int j0 = lane / kDim, c0 = lane - j0 * kDim;
    const int j1 = (kWave + lane) / kDim, c1 = kWave + lane - j1 * kDim;
    // the actions of a chunk are loaded one chunk ahead: a load still in flight behind the chunk's
    // stores is waited for with a counted vmcnt, not a drain of every store
    int av = !done && lane < min(C, T) ? actions[(long long)lane * E + e] : 0;
    int s0 = 0;
    ETR_DECL
    for (int kc = 0;; ++kc) {
        float* const rows = bufs + (kc & 1) * kBufFloats;
        float* const carry = rows + C * kRowStride;
        const int cs0 = s0;
        int n = 0;
        unsigned long long dout = 0;
        if (!done) {
            // ------------------------------------------------------------ walk
            const int na = min(C, T - s0);
            const unsigned long long abits = ballot(av == 1 && lane < na);
            const int av_next = s0 + na + lane < T ? actions[(long long)(s0 + na + lane) * E + e] : 0;
            // Every lane works out its own step from the chunk's action bits (uav_env.py:306-356): the
            // pointer ADVANCES to the next UAV (t -> 0) on an assign, or on a skip of the last target.
            // Between two assigns the target index just counts skips modulo M, so step i's target is
            // (t at the run start + steps since) mod M, the run starting after the previous assign (at
            // the carried t for the chunk's first run). An episode is N advances: the UAV index is the
            // advance count modulo N, and it ends (u reaches N) on every N-th advance.
            const unsigned long long le = lane == 63 ? ~0ull : (2ull << lane) - 1, lt = (1ull << lane) - 1;
            const bool lin = lane < na;
            const int a_i = (int)((abits >> lane) & 1ull);
            const int p_as = top_bit(abits & lt);                     // previous assign in the chunk
            const int tb = (((p_as >= 0 ? 0 : R.t) + lane - (p_as + 1)) % M);
            const bool adv = lin && (a_i || tb + 1 == M);
            const unsigned long long advbits = ballot(adv);
            const int ub = (R.u + __popcll(advbits & lt)) % N;
            const int ua = ub + (adv ? 1 : 0), ta = adv ? 0 : tb + 1;
            const bool dn = adv && ua == N;                           // uav_env.py:355-356
            unsigned long long dbits = ballot(dn);
            const int epl = R.ep + __popcll(dbits & lt);              // the episode step i belongs to
            // main_train.py:79 full-reset cadence at the episode ends: the first one (spare fresh) flips
            // to the spare scene and ends the chunk; with the spare already used, a state-only reset
            const int P = env.full_reset_period;
            const unsigned long long frbits = ballot(dn && P > 0 && (epl + 1) % P == 0);
            n = na;
            bool flip = false;
            if (frbits) {
                if (env.scene_buffers == 2 && !R.stale) {
                    flip = true;
                    n = __builtin_ctzll(frbits) + 1;
                } else {
                    R.err |= 2;  // no fresh spare: state-only reset
                }
            }
            const unsigned long long nmask = n >= 64 ? ~0ull : (1ull << n) - 1;
            const int code = rec_pack(ub, tb, ua, ta, a_i, dn ? 1 : 0);
            // the walk's end state
            const int u = (R.u + __popcll(advbits & nmask)) % N;
            const int t = readlane_i(ta, n - 1);
            R.ep += __popcll(dbits & nmask);
            const unsigned long long amask = abits & nmask;
            dbits &= nmask;
            const bool act = lane < n;
            const bool la = act && a_i, ld = act && dn;
            // the pair each assign locks: p_dmg (this chunk's scene), p_pen and the UAV's cost
            const double pd_a = la ? R.tab[ub * M + tb] : 0.0;
            const double pp_a = shfl_d(R.ppen, ub);
            const double uc_a = shfl_d(R.ucost, ub);
            ETR(0);
            // ------------------------------------------------------------ fold (lane = assign)
            // step_once's per-assign updates (uav_env.py:306-325) as ordered chains over lanes: each
            // assign continues the chain of the previous assign of its episode (the running sums) and
            // of the previous assign of its episode to the same target (the not-hit products, the
            // locker costs); chain position r is settled in round r from the value of position r - 1,
            // with step_once's operations, so every value is bitwise the sequential one. The chains
            // of the episode the chunk started in begin from the carried state, later ones from the
            // fresh state of an episode-end reset (uav_env.py:175-182).
            const double c_r = R.r, c_J = R.J, c_spd = R.sum_pd, c_spf = R.sum_pf, c_ac = R.asg_cost, c_cv = R.cov_val;
            const int c_ncov = R.ncov, c_nasg = R.nasg;
            const double R0nhf = R.nhf[0], R0nhp = R.nhp[0], R0tc = R.tc[0];  // the chunk's starting targets
            carry[lane] = R.w0;
            if (lane < kObs - kWave) carry[kWave + lane] = R.w1;
            // lanes assigning the same target: tmask (assign lanes: those of its target), tm (lane t < M:
            // those of target t), one ballot per target hit in the chunk
            unsigned long long tmask = 0, tm = 0;
            for (unsigned long long rem = amask; rem;) {
                const int tk = readlane_i(tb, __builtin_ctzll(rem));
                const unsigned long long m = ballot(la && tb == tk);
                rem &= ~m;
                tmask = (la && tb == tk) ? m : tmask;
                tm = lane == tk ? m : tm;
            }
            const int dprev = top_bit(dbits & lt);           // latest episode end before this step
            const bool fresh = dprev >= 0;                   // the step's episode began inside the chunk
            const unsigned long long epm = fresh ? ~((2ull << dprev) - 1) : ~0ull;  // its steps
            const double pf_a = pd_a * pp_a;
            // per target: not-hit products and locker costs after each assign
            const unsigned long long tprev = tmask & lt & epm;
            const int tdep = __popcll(tprev), tsrc = top_bit(tprev);
            const double st_nhf = shfl_d(R.nhf[0], tb), st_nhp = shfl_d(R.nhp[0], tb), st_tc = shfl_d(R.tc[0], tb);
            const int st_nlk = __shfl(R.nlk[0], tb);
            double a_nhf = (fresh ? 1.0 : st_nhf) * (1.0 - pf_a);
            double a_nhp = (fresh ? 1.0 : st_nhp) * (1.0 - pd_a);
            double a_tc = (fresh ? 0.0 : st_tc) + uc_a;
            for (int r = 1; ballot(la && tdep >= r); ++r) {
                const int sl = tsrc < 0 ? lane : tsrc;
                const double p_nhf = shfl_d(a_nhf, sl), p_nhp = shfl_d(a_nhp, sl), p_tc = shfl_d(a_tc, sl);
                const bool now = la && tdep == r;
                a_nhf = now ? p_nhf * (1.0 - pf_a) : a_nhf;
                a_nhp = now ? p_nhp * (1.0 - pd_a) : a_nhp;
                a_tc = now ? p_tc + uc_a : a_tc;
            }
            // first lock of the target in the episode: covered (uav_env.py:255-259 N0, cov_val)
            const bool cov_new = la && tdep == 0 && (fresh || st_nlk == 0);
            const unsigned long long covbits = ballot(cov_new);
            const double v_tb = shfl_d(R.val[0], tb);  // (shuffles outside selects: the whole wave active)
            const double x_cv = cov_new ? v_tb : 0.0;  // + 0.0 keeps a sum >= +0 bitwise
            // the episode's running sums after each assign
            const unsigned long long aprv = amask & lt & epm;
            const int adep = __popcll(aprv), asrc = top_bit(aprv);
            double ev_spd = (fresh ? 0.0 : c_spd) + pd_a, ev_spf = (fresh ? 0.0 : c_spf) + pf_a;
            double ev_ac = (fresh ? 0.0 : c_ac) + uc_a, ev_cv = (fresh ? 0.0 : c_cv) + x_cv;
            for (int r = 1; ballot(la && adep >= r); ++r) {
                const int sl = asrc < 0 ? lane : asrc;
                const double p_spd = shfl_d(ev_spd, sl), p_spf = shfl_d(ev_spf, sl), p_ac = shfl_d(ev_ac, sl),
                             p_cv = shfl_d(ev_cv, sl);
                const bool now = la && adep == r;
                ev_spd = now ? p_spd + pd_a : ev_spd;
                ev_spf = now ? p_spf + pf_a : ev_spf;
                ev_ac = now ? p_ac + uc_a : ev_ac;
                ev_cv = now ? p_cv + x_cv : ev_cv;
            }
            const int ev_ncov = (fresh ? 0 : c_ncov) + __popcll(covbits & le & epm);
            const int ev_nasg = (fresh ? 0 : c_nasg) + __popcll(amask & le & epm);
            const int ev_cnt = (ev_ncov << 8) | ev_nasg;  // lane i: (ncov << 8) | nasg after step i's assign
            // the state the chunk hands on: that after the last assign of its last episode
            {
                const int dl = top_bit(dbits);
                const unsigned long long fm = dl >= 0 ? ~((2ull << dl) - 1) : ~0ull;
                const int jt = top_bit(tm & fm), ja = top_bit(amask & fm);
                const double e_nhf = shfl_d(a_nhf, jt < 0 ? 0 : jt), e_nhp = shfl_d(a_nhp, jt < 0 ? 0 : jt),
                             e_tc = shfl_d(a_tc, jt < 0 ? 0 : jt);
                const int nlk_f = __popcll(tm & fm);
                if (lane < M) {
                    R.nhf[0] = jt >= 0 ? e_nhf : (dl >= 0 ? 1.0 : R.nhf[0]);
                    R.nhp[0] = jt >= 0 ? e_nhp : (dl >= 0 ? 1.0 : R.nhp[0]);
                    R.tc[0] = jt >= 0 ? e_tc : (dl >= 0 ? 0.0 : R.tc[0]);
                    R.nlk[0] = nlk_f + (dl >= 0 ? 0 : R.nlk[0]);
                }
                if (ja >= 0) {
                    R.sum_pd = readlane_d(ev_spd, ja);
                    R.sum_pf = readlane_d(ev_spf, ja);
                    R.asg_cost = readlane_d(ev_ac, ja);
                    R.cov_val = readlane_d(ev_cv, ja);
                    const int cnt = readlane_i(ev_cnt, ja);
                    R.ncov = cnt >> 8;
                    R.nasg = cnt & 255;
                } else if (dl >= 0) {
                    R.sum_pd = R.sum_pf = R.asg_cost = R.cov_val = 0.0;
                    R.ncov = R.nasg = 0;
                }
                if (dl >= 0) R.asg = -1;
                for (unsigned long long q = amask & fm; q; q &= q - 1) {  // the last episode's locks per UAV
                    const int ci = readlane_i(code, __builtin_ctzll(q));
                    if (lane == (ci & 127)) R.asg = (ci >> 7) & 127;
                }
            }
            ETR(1);
            // ------------------------------------------------------------ replay (lane = step)
            // J(X), r(X) after this step's assign: the list-order revenue sum (uav_env.py:244-269) over
            // every target's not-hit product at this step -- that after the target's latest assign of
            // the episode up to here, else the episode's starting value (unlocked targets add +0.0)
            double Jv = 0.0, rv = 0.0;
            {
                double rev = 0.0;
                for (int k = 0; k < M; ++k) {
                    const unsigned long long tmk = readlane_u64(tm, k);
                    const int j = top_bit(tmk & le & epm);
                    const double hv = shfl_d(a_nhf, j < 0 ? 0 : j);
                    const double nh = j >= 0 ? hv : (fresh ? 1.0 : readlane_d(R0nhf, k));
                    rev = rev + (1.0 - nh) * readlane_d(R.val[0], k);
                }
                if (la) {
                    Jv = rev - (env.prm[UAVHIP_PRM_OMEGA] * ev_ac);
                    rv = (ev_ncov == M) ? 2.0 * Jv : Jv * div_by((double)ev_ncov, (double)M, R.rcp_m);
                }
            }
            // the state after this step (before an episode-end reset): that of the latest assign of its
            // episode, else the episode's fresh state (it began inside the chunk), else the chunk's start
            const int alast = top_bit(amask & le), aprev = top_bit(amask & lt);
            const bool has = alast > dprev, hasp = aprev > dprev;
            const int src = has ? alast : 0;
            const double s_r = shfl_d(rv, src), s_J = shfl_d(Jv, src), s_spd = shfl_d(ev_spd, src),
                         s_spf = shfl_d(ev_spf, src), s_ac = shfl_d(ev_ac, src), s_cv = shfl_d(ev_cv, src);
            const int s_cnt = __shfl(ev_cnt, src);
            const double p_r = shfl_d(rv, hasp ? aprev : 0);
            const double r_after = has ? s_r : (fresh ? 0.0 : c_r);
            const double J_after = has ? s_J : (fresh ? 0.0 : c_J);
            const double spd = has ? s_spd : (fresh ? 0.0 : c_spd);
            const double spf = has ? s_spf : (fresh ? 0.0 : c_spf);
            const double ac = has ? s_ac : (fresh ? 0.0 : c_ac);
            const double cv = has ? s_cv : (fresh ? 0.0 : c_cv);
            const int ncov = has ? (s_cnt >> 8) : (fresh ? 0 : c_ncov);
            const int nasg = has ? (s_cnt & 255) : (fresh ? 0 : c_nasg);
            const double r_before = hasp ? p_r : (fresh ? 0.0 : c_r);
            double reward = la ? r_after - r_before : 0.0;  // :321 R = r(X') - r(X)
            if (ld) reward = reward + r_after;              // :361-363 goal reward r(X_final)
            const double is_valid = la ? (reward != 0.0 ? 1.0 : 0.0) : -1.0;
            // (every cross-lane read with the whole wave active: ds_bpermute from an inactive lane reads 0)
            const double rn = shfl_d(R.rcp_n, nasg > 0 ? nasg - 1 : 0);
            const double y = nasg > 0 ? rn : 0.0;
            const double avg_d = nasg > 0 ? div_by(spd, (double)nasg, y) : 0.0;
            const double avg_f = nasg > 0 ? div_by(spf, (double)nasg, y) : 0.0;
            // the row pushed into the window: the pointer after the step, or at an episode end the new
            // episode's first row at (0, 0) on a fresh state (a flip's row is rebuilt on the new scene)
            {
                const int pu = ld ? 0 : ua, pt = ld ? 0 : ta;
                // target pt after the latest assign to it of this step's episode, else the episode's
                // starting value (fresh, or the chunk's carried state)
                const int j = top_bit(shfl_u64(tm, pt) & le & epm);
                const int jl = j < 0 ? 0 : j;
                const double g_nhf = shfl_d(a_nhf, jl), g_nhp = shfl_d(a_nhp, jl), g_tc = shfl_d(a_tc, jl);
                const double s_nhf = shfl_d(R0nhf, pt), s_nhp = shfl_d(R0nhp, pt), s_tc = shfl_d(R0tc, pt);
                const bool zero = ld || (j < 0 && fresh);
                const double nhf = zero ? 1.0 : (j >= 0 ? g_nhf : s_nhf);
                const double nhp = zero ? 1.0 : (j >= 0 ? g_nhp : s_nhp);
                const double tc = zero ? 0.0 : (j >= 0 ? g_tc : s_tc);
                const ObsRow row = obs_row(shfl_d(R.ucost, pu), shfl_d(R.val[0], pt), tc, nhf, nhp, ld ? 0.0 : ac,
                                           ld ? 0.0 : cv, R.tab[pu * M + pt], shfl_d(R.ppen, pu), R.den_c, R.rcp_c,
                                           R.den_v, R.rcp_v);
                if (act) {
                    float2* rw = reinterpret_cast<float2*>(rows + lane * kRowStride);
    #pragma unroll
                    for (int q = 0; q < kDim / 2; ++q) rw[q] = make_float2(row.v[2 * q], row.v[2 * q + 1]);
                }
            }
            if (act) {
                const long long se = (long long)(s0 + lane) * E + e;
                if (reward_out) reward_out[se] = reward;
                if (done_out) done_out[se] = ld ? 1 : 0;
                if (info_out) {  // uav_env.py:426-433 (write_info's layout)
                    double2* q = reinterpret_cast<double2*>(info_out + se * UAVHIP_INFO_COUNT);
                    q[0] = make_double2(J_after, (double)ncov);
                    q[1] = make_double2(is_valid, avg_d);
                    q[2] = make_double2(avg_f, (double)ua);
                    q[3] = make_double2((double)ta, (double)epl);
                }
            }
            ETR(2);
            // ------------------------------------------------------------ carried state
            {
                const int d_last = top_bit(dbits), a_last = top_bit(amask);
                if (a_last > d_last) {
                    R.r = readlane_d(rv, a_last);
                    R.J = readlane_d(Jv, a_last);
                } else if (d_last >= 0) {
                    R.r = 0.0;
                    R.J = 0.0;
                }
            }
            R.u = u;
            R.t = t;
            wave_lds_sync();
            if (flip) {  // the full reset at step n - 1 flips to the pre-generated spare scene
                R.sel ^= 1;
                R.stale = 1;
                R.sb = (long long)R.sel * env.E + e;
                load_table(R, env, lane);
                reset_regs<1, true>(R, env, lane, true);  // new scene values; its first row -> R.row
                wave_lds_sync();
                if (lane < kDim) rows[(n - 1) * kRowStride + lane] = R.row[lane];
                wave_lds_sync();
            } else {
                R.pd_cur = R.tab[R.u * M + R.t];
                R.pp_cur = readlane_d(R.ppen, R.u);
            }

            {   // the carried window: step n - 1's, element lane / 64 + lane
                const int s = n - 1;
                const int d = top_bit(dbits);
                auto elem = [&](int j, int c) -> float {
                    const int k = s - (kSeq - 1) + j;
                    if (d >= 0) return k >= d ? rows[k * kRowStride + c] : 0.0f;
                    return k >= 0 ? rows[k * kRowStride + c] : carry[(kSeq + k) * kDim + c];
                };
                R.w0 = elem(j0, c0);
                R.w1 = lane < kObs - kWave ? elem(j1, c1) : 0.0f;
            }
            s0 += n;
            dout = dbits;
            av = n == na ? av_next : (s0 + lane < T && lane < C ? actions[(long long)(s0 + lane) * E + e] : 0);
            done = s0 >= T;
        }
        ETR(3);
        if (lane == 0) {
            int* m = s_meta[kc & 1][we];
            m[0] = cs0;
            m[1] = n;
            m[2] = (int)(unsigned)dout;
            m[3] = (int)(unsigned)(dout >> 32);
            m[4] = done ? 0 : 1;
        }
        __syncthreads();  // chunk kc's rows to the store waves; they are done with chunk kc - 1's buffer
        bool more = false;
#pragma unroll
        for (int j = 0; j < kWavesPerBlock; ++j) more = more || s_meta[kc & 1][j][4] != 0;
        ETR(4);
#ifdef UAVHIP_POLICY_TRACE
        etr[5] += n > 0 ? 1 : 0;
#endif
        if (!more) break;
    }
    if (live) {
        ETR_END
    }
    if (!stored) store_regs(R, env, e, lane);
}

}  // namespace envrep
}  // namespace uavhip
