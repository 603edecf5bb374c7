/*
 * uav_oracle.c -- CPU ORACLE (test infrastructure, NOT product code).
 *
 * A literal, scalar, fp64 restatement of the reference's env hot path, used only by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker /
 * the timed CPU baseline. It deliberately follows the reference's from-scratch
 * algorithm (recompute J(X) over every locked pair on every call, calc_advantage per
 * pair on the fly) rather than the cached/incremental scheme the HIP kernels use, so
 * the two are independent.
 *
 * Pinned against the tests/golden fixtures, which were produced by running the reference
 * itself (tests/golden/make_golden.py).
 *
 * Reference citations (paths relative to the reference repo):
 *   angle score        envs/mechanics.py:11-57
 *   speed score        envs/mechanics.py:61-68
 *   dist score         envs/mechanics.py:72-89
 *   damage prob        envs/mechanics.py:93-114
 *   penetration prob   envs/mechanics.py:118-163
 *   advantage          envs/mechanics.py:167-181
 *   state vector       envs/mechanics.py:185-241
 *   _get_obs           envs/uav_env.py:184-242
 *   _calc_J_X          envs/uav_env.py:244-269
 *   paper reward       envs/uav_env.py:271-293
 *   step               envs/uav_env.py:295-435
 *   reset (state only) envs/uav_env.py:42-63,175-182
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off; no FMA contraction, so every
 * product/sum rounds exactly like the reference's numpy scalar ops).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* parameter vector layout, identical to include/uavhip.h UAVHIP_PRM_* */
enum { P_ZETA_D = 0, P_K, P_C1, P_C2, P_C3, P_C4, P_OMEGA, P_ZETA_OBS, P_COUNT };

#define SEQ_LEN 5
#define STATE_DIM 14

static double norm2(double x, double y) { return sqrt(x * x + y * y); }
static double clip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* mechanics.py:11-57 */
double uo_angle_score(const double* up, const double* uv, const double* pt) {
    double vx = pt[0] - up[0], vy = pt[1] - up[1];
    double dist = norm2(vx, vy);
    if (dist < 1e-6) return 1.0;
    double nx = vx / dist, ny = vy / dist;
    double speed = norm2(uv[0], uv[1]);
    double hx, hy;
    if (speed < 1e-6) { hx = 1.0; hy = 0.0; }
    else { hx = uv[0] / speed; hy = uv[1] / speed; }
    double c = nx * hx + ny * hy;
    double sigma = acos(clip(c, -1.0, 1.0));
    double b = 0.002 * dist;
    if (b < 1e-6) b = 1e-6;
    double q = sigma / (b * M_PI);
    return exp(-(q * q));
}

/* mechanics.py:61-68 */
double uo_speed_score(double us, double ts, const double* prm) {
    if (us < 1e-6) return 0.0;
    double s = 1.0 - (prm[P_K] * ts / us);
    return clip(s, 0.0, 1.0);
}

/* mechanics.py:72-89 (D_mid = 0 for both branches) */
double uo_dist_score(double d, int obstacle, const double* prm) {
    double zeta = obstacle ? prm[P_ZETA_OBS] : prm[P_ZETA_D];
    double q = (d - 0.0) / zeta;
    return exp(-(q * q));
}

/* mechanics.py:93-114 */
double uo_damage_prob(const double* up, const double* uv, double load, const double* tp, const double* tv,
                      const double* prm) {
    double dist = norm2(up[0] - tp[0], up[1] - tp[1]);
    double us = norm2(uv[0], uv[1]);
    double ts = norm2(tv[0], tv[1]);
    double ea = uo_angle_score(up, uv, tp);
    double ed = uo_dist_score(dist, 0, prm);
    double es = uo_speed_score(us, ts, prm);
    double term = prm[P_C1] * ed + prm[P_C2] * es;
    double p = ea * term * load;
    return clip(p, 0.0, 1.0);
}

/* mechanics.py:118-163 -- the target argument is never read, so it is not taken */
double uo_penetration_prob(const double* up, const double* uv, const double* nfz, int kn, const double* ip,
                           const double* iv, int ki, const double* prm) {
    double p = 1.0;
    double us = norm2(uv[0], uv[1]);
    for (int j = 0; j < kn; ++j) {
        double ea = uo_angle_score(up, uv, nfz + 2 * j);
        double dist = norm2(up[0] - nfz[2 * j], up[1] - nfz[2 * j + 1]);
        double ed = uo_dist_score(dist, 1, prm);
        double pn = (1.0 - ea) * (1.0 - ed);
        p *= clip(pn, 0.0, 1.0);
    }
    for (int j = 0; j < ki; ++j) {
        double ea = uo_angle_score(up, uv, ip + 2 * j);
        double dist = norm2(up[0] - ip[2 * j], up[1] - ip[2 * j + 1]);
        double ed = uo_dist_score(dist, 1, prm);
        double is = norm2(iv[2 * j], iv[2 * j + 1]);
        double es = uo_speed_score(us, is, prm);
        double term = prm[P_C3] * (1.0 - ed) + prm[P_C4] * es;
        double pi = (1.0 - ea) * term;
        p *= clip(pi, 0.0, 1.0);
    }
    return p;
}

/* dense pair tables for one scene, as main.py:35-45 builds them */
void uo_score_pairs(int N, int M, int kn, int ki, const double* uav_pos, const double* uav_vel,
                    const double* uav_load, const double* tgt_pos, const double* tgt_vel, const double* nfz_pos,
                    const double* icp_pos, const double* icp_vel, const double* prm, double* p_dmg, double* p_pen) {
    for (int u = 0; u < N; ++u) {
        p_pen[u] = uo_penetration_prob(uav_pos + 2 * u, uav_vel + 2 * u, nfz_pos, kn, icp_pos, icp_vel, ki, prm);
        for (int t = 0; t < M; ++t)
            p_dmg[u * M + t] = uo_damage_prob(uav_pos + 2 * u, uav_vel + 2 * u, uav_load[u], tgt_pos + 2 * t,
                                              tgt_vel + 2 * t, prm);
    }
}

/* ------------------------------------------------------------------------------ env */
typedef struct uo_env {
    int N, M, kn, ki;
    double prm[P_COUNT];
    /* scene (copied in) */
    double *uav_pos, *uav_vel, *uav_load, *uav_cost;
    double *tgt_pos, *tgt_vel, *tgt_value;
    int* tgt_id;
    double *nfz_pos, *icp_pos, *icp_vel;
    double total_swarm_cost;
    /* state */
    int uav_idx, target_idx;
    int* assigned_target_id; /* [N] reference target id or -1 */
    int* available;          /* [N] */
    int* locked;             /* [M][N] uav ids in lock (append) order */
    int* n_locked;           /* [M] */
    float window[SEQ_LEN][STATE_DIM];
} uo_env;

static double* dup(const double* p, size_t n) {
    double* q = (double*)malloc(n * sizeof(double) + 8);
    if (n) memcpy(q, p, n * sizeof(double));
    return q;
}

uo_env* uo_env_create(int N, int M, int kn, int ki, const double* uav_pos, const double* uav_vel,
                      const double* uav_load, const double* uav_cost, const double* tgt_pos, const double* tgt_vel,
                      const double* tgt_value, const int* tgt_id, const double* nfz_pos, const double* icp_pos,
                      const double* icp_vel, const double* prm) {
    uo_env* e = (uo_env*)calloc(1, sizeof(uo_env));
    e->N = N; e->M = M; e->kn = kn; e->ki = ki;
    memcpy(e->prm, prm, sizeof(e->prm));
    e->uav_pos = dup(uav_pos, 2 * N); e->uav_vel = dup(uav_vel, 2 * N);
    e->uav_load = dup(uav_load, N); e->uav_cost = dup(uav_cost, N);
    e->tgt_pos = dup(tgt_pos, 2 * M); e->tgt_vel = dup(tgt_vel, 2 * M); e->tgt_value = dup(tgt_value, M);
    e->tgt_id = (int*)malloc(sizeof(int) * (M + 1));
    memcpy(e->tgt_id, tgt_id, sizeof(int) * M);
    e->nfz_pos = dup(nfz_pos, 2 * kn); e->icp_pos = dup(icp_pos, 2 * ki); e->icp_vel = dup(icp_vel, 2 * ki);
    /* uav_env.py:118 -- accumulated in generation order */
    e->total_swarm_cost = 0.0;
    for (int u = 0; u < N; ++u) e->total_swarm_cost += uav_cost[u];
    e->assigned_target_id = (int*)malloc(sizeof(int) * N);
    e->available = (int*)malloc(sizeof(int) * N);
    e->locked = (int*)malloc(sizeof(int) * (size_t)M * N);
    e->n_locked = (int*)malloc(sizeof(int) * M);
    return e;
}

void uo_env_destroy(uo_env* e) {
    if (!e) return;
    free(e->uav_pos); free(e->uav_vel); free(e->uav_load); free(e->uav_cost);
    free(e->tgt_pos); free(e->tgt_vel); free(e->tgt_value); free(e->tgt_id);
    free(e->nfz_pos); free(e->icp_pos); free(e->icp_vel);
    free(e->assigned_target_id); free(e->available); free(e->locked); free(e->n_locked);
    free(e);
}

/* mechanics.py:167-181 */
static void advantage(const uo_env* e, int u, int t, double* p_final, double* p_dmg) {
    double pd = uo_damage_prob(e->uav_pos + 2 * u, e->uav_vel + 2 * u, e->uav_load[u], e->tgt_pos + 2 * t,
                               e->tgt_vel + 2 * t, e->prm);
    double pp = uo_penetration_prob(e->uav_pos + 2 * u, e->uav_vel + 2 * u, e->nfz_pos, e->kn, e->icp_pos,
                                    e->icp_vel, e->ki, e->prm);
    *p_final = pd * pp;
    *p_dmg = pd;
}

/* uav_env.py:244-269 */
static double calc_J(const uo_env* e) {
    double rev = 0.0, cost = 0.0;
    for (int t = 0; t < e->M; ++t) {
        double nh = 1.0;
        for (int k = 0; k < e->n_locked[t]; ++k) {
            int u = e->locked[t * e->N + k];
            double pf, pd;
            advantage(e, u, t, &pf, &pd);
            nh *= (1.0 - pf);
            cost += e->uav_cost[u];
        }
        double jp = 1.0 - nh;
        rev += jp * e->tgt_value[t];
    }
    return rev - (e->prm[P_OMEGA] * cost);
}

static int count_covered(const uo_env* e) {
    int n0 = 0;
    for (int t = 0; t < e->M; ++t) n0 += e->n_locked[t] > 0;
    return n0;
}

/* uav_env.py:271-293 */
static double paper_reward(const uo_env* e) {
    double J = calc_J(e);
    int n0 = count_covered(e);
    if (n0 == e->M) return 2.0 * J;
    return J * ((double)n0 / (double)e->M);
}

/* uav_env.py:184-242 + mechanics.py:185-241. Writes the (5,14) window; returns 0 if done. */
static int get_obs(uo_env* e, float* obs_out) {
    if (e->uav_idx >= e->N) {
        if (obs_out) memset(obs_out, 0, sizeof(float) * STATE_DIM);
        return 0;
    }
    const int u = e->uav_idx, t = e->target_idx;
    double asg = 0.0;
    for (int i = 0; i < e->N; ++i)
        if (!e->available[i]) asg += e->uav_cost[i];
    double chi_c = asg / (e->total_swarm_cost + 1e-6);
    double tot_v = 0.0, cov_v = 0.0;
    for (int i = 0; i < e->M; ++i) tot_v += e->tgt_value[i];
    for (int i = 0; i < e->M; ++i)
        if (e->n_locked[i] > 0) cov_v += e->tgt_value[i];
    double chi_v = cov_v / (tot_v + 1e-6);
    double tc = 0.0;
    for (int k = 0; k < e->n_locked[t]; ++k) tc += e->uav_cost[e->locked[t * e->N + k]];
    double chi_mc = tc / (e->total_swarm_cost + 1e-6);
    double nh = 1.0, nhp = 1.0;
    for (int k = 0; k < e->n_locked[t]; ++k) {
        double pf, pd;
        advantage(e, e->locked[t * e->N + k], t, &pf, &pd);
        nh *= (1.0 - pf);
        nhp *= (1.0 - pd);
    }
    double pjp = 1.0 - nh, pjp_pure = 1.0 - nhp;
    double val = e->tgt_value[t];
    double prev_rev = pjp * val;
    /* get_state_vector */
    double p_km, p_pure;
    advantage(e, u, t, &p_km, &p_pure);
    double hat_p = 1.0 - (1.0 - pjp) * (1.0 - p_km);
    double hat_pp = 1.0 - (1.0 - pjp_pure) * (1.0 - p_pure);
    double hat_G = hat_p * val;
    double d_pkm = p_pure - p_km;
    double d_pm = hat_pp - hat_p;
    double d_G = (hat_pp * val) - hat_G;
    float s[STATE_DIM] = {(float)e->uav_cost[u], (float)val, (float)chi_c, (float)chi_v, (float)chi_mc,
                          (float)p_km, (float)pjp, (float)hat_p, (float)prev_rev, (float)hat_G,
                          (float)d_pkm, (float)d_pm, (float)d_G, (float)(e->available[u] ? 1.0 : 0.0)};
    s[0] /= 2.0f; s[1] /= 16.0f; s[8] /= 16.0f; s[9] /= 16.0f; s[12] /= 16.0f;
    memmove(&e->window[0][0], &e->window[1][0], sizeof(float) * STATE_DIM * (SEQ_LEN - 1));
    memcpy(&e->window[SEQ_LEN - 1][0], s, sizeof(s));
    if (obs_out) memcpy(obs_out, e->window, sizeof(e->window));
    return 1;
}

/* uav_env.py:42-63 with full_reset=False (the scene was injected at create time) */
void uo_env_reset(uo_env* e, float* obs_out) {
    for (int u = 0; u < e->N; ++u) { e->available[u] = 1; e->assigned_target_id[u] = -1; }
    for (int t = 0; t < e->M; ++t) e->n_locked[t] = 0;
    e->uav_idx = 0; e->target_idx = 0;
    memset(e->window, 0, sizeof(e->window));
    get_obs(e, obs_out);
}

/*
 * uav_env.py:295-435. Returns 0 on success, -1 if the episode is already over (the
 * reference raises IndexError at :296). info[8] = {J_val, num_assigned, is_valid (-1 = None),
 * avg_p_dmg, avg_p_final, uav_idx, target_idx, 0}.
 * obs_out gets the (5,14) window, or 14 zeros followed by garbage-free zeros when done.
 */
int uo_env_step(uo_env* e, int action, float* obs_out, double* reward_out, int* done_out, double* info) {
    if (e->uav_idx >= e->N) return -1;
    const int u = e->uav_idx, t = e->target_idx;
    int done = 0;
    double prev_r = paper_reward(e);
    double reward = 0.0;
    if (action == 1) {
        e->assigned_target_id[u] = e->tgt_id[t];
        e->available[u] = 0;
        e->locked[t * e->N + e->n_locked[t]++] = u;
        double new_r = paper_reward(e);
        if (new_r >= prev_r) {
            reward = new_r - prev_r;
            e->uav_idx += 1;
            e->target_idx = 0;
        } else {
            e->assigned_target_id[u] = -1;
            e->available[u] = 1;
            e->n_locked[t]--;
            reward = 0.0;
            e->target_idx += 1;
            if (e->target_idx >= e->M) { e->uav_idx += 1; e->target_idx = 0; }
        }
    } else {
        reward = 0.0;
        e->target_idx += 1;
        if (e->target_idx >= e->M) { e->uav_idx += 1; e->target_idx = 0; }
    }
    if (e->uav_idx >= e->N) done = 1;
    if (done) reward += paper_reward(e);
    if (obs_out) memset(obs_out, 0, sizeof(float) * SEQ_LEN * STATE_DIM);
    get_obs(e, obs_out);
    double tot_d = 0.0, tot_f = 0.0;
    int count = 0;
    for (int tt = 0; tt < e->M; ++tt)
        for (int k = 0; k < e->n_locked[tt]; ++k) {
            double pf, pd;
            advantage(e, e->locked[tt * e->N + k], tt, &pf, &pd);
            tot_d += pd;
            count++;
        }
    for (int tt = 0; tt < e->M; ++tt)
        for (int k = 0; k < e->n_locked[tt]; ++k) {
            double pf, pd;
            advantage(e, e->locked[tt * e->N + k], tt, &pf, &pd);
            tot_f += pf;
        }
    if (info) {
        info[0] = calc_J(e);
        info[1] = (double)count_covered(e);
        info[2] = action == 1 ? (reward != 0.0 ? 1.0 : 0.0) : -1.0;
        info[3] = count > 0 ? tot_d / count : 0.0;
        info[4] = count > 0 ? tot_f / count : 0.0;
        info[5] = (double)e->uav_idx;
        info[6] = (double)e->target_idx;
        info[7] = 0.0;
    }
    *reward_out = reward;
    *done_out = done;
    return 0;
}

int uo_env_uav_idx(const uo_env* e) { return e->uav_idx; }
int uo_env_target_idx(const uo_env* e) { return e->target_idx; }
void uo_env_assigned(const uo_env* e, int* out) { memcpy(out, e->assigned_target_id, sizeof(int) * e->N); }

/*
 * Batched convenience for the CPU baseline: run `steps` env steps on a set of envs with
 * pre-drawn actions [steps][n_env]; auto-resets (state only) finished envs. Returns the
 * number of env-steps executed.
 */
long uo_envs_run(uo_env** envs, int n_env, const int8_t* actions, int steps, float* obs_scratch) {
    long n = 0;
    for (int s = 0; s < steps; ++s)
        for (int i = 0; i < n_env; ++i) {
            double r; int d; double info[8];
            if (uo_env_step(envs[i], actions[(size_t)s * n_env + i], obs_scratch, &r, &d, info) == 0) n++;
            if (d) uo_env_reset(envs[i], obs_scratch);
        }
    return n;
}
