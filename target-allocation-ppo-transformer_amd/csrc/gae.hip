// gae.hip -- K3: GAE + advantage normalisation over a time-major [T][E] rollout buffer.
// Reference: agents/ppo.py:70-94 (one Python iteration and a chain of 0-dim fp32 torch ops per
// transition). Here: one lane per env walks t = T-1..0 over inputs staged in LDS by its whole
// workgroup (the recurrence is the only serial part); fp32 arithmetic in the reference's op order,
// no FMA contraction, so returns are bitwise the reference's. The normalisation statistics are
// fp64 block partials (fixed reduction order -> run-to-run deterministic, no atomics).
#include "common.hpp"

#pragma clang fp contract(off)

namespace uavhip {
namespace {
constexpr int kGaeBlock = 64;     // envs per block (E = 4096 -> 64 blocks); one partial pair each
constexpr int kGaeThreads = 256;  // loaders / storers per block
constexpr int kGaeT = 64;         // steps staged in LDS per pass
constexpr int kGaeIt = kGaeT * kGaeBlock / kGaeThreads;  // staged items per thread and pass
constexpr int kRedBlock = 256;
constexpr int kNormPer = 4;  // k_adv_normalize: items per thread (uavhip_adv_normalize's grid covers n with 4)

// Deterministic fp64 block reduction of (a, b); result valid in thread 0.
template <int BLOCK>
__device__ __forceinline__ void block_sum2(double& a, double& b) {
    __shared__ double sa[BLOCK / kWave], sb[BLOCK / kWave];
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        a += __shfl_down(a, o);
        b += __shfl_down(b, o);
    }
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) { sa[w] = a; sb[w] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = 0.0; b = 0.0;
        for (int i = 0; i < BLOCK / kWave; ++i) { a += sa[i]; b += sb[i]; }
    }
}
}  // namespace

// One block per 64 envs: all 256 threads stage the [t][env] inputs of up to kGaeT steps in LDS
// (coalesced, 4 waves of loads in flight instead of one), wave 0 walks the recurrence from LDS --
// one lane per env, the serial part -- and all threads store the returns / advantages.
__global__ __launch_bounds__(kGaeThreads) void k_gae(const double* __restrict__ reward,
                                                     const uint8_t* __restrict__ done,
                                                     const float* __restrict__ value,
                                                     const float* __restrict__ last_value, int T, int E, float g,
                                                     float gl, float* __restrict__ ret, float* __restrict__ adv,
                                                     double* __restrict__ partials) {
    __shared__ float sr[kGaeT][kGaeBlock], sv[kGaeT][kGaeBlock], sret[kGaeT][kGaeBlock], sadv[kGaeT][kGaeBlock];
    __shared__ uint8_t sd[kGaeT][kGaeBlock];
    const int e0 = blockIdx.x * kGaeBlock, lane = threadIdx.x & (kGaeBlock - 1);
    const bool walker = threadIdx.x < kGaeBlock && e0 + lane < E;
    double s = 0.0, s2 = 0.0;
    float nv = 0.0f, gae = 0.0f;
    if (walker && last_value) nv = last_value[e0 + lane];  // ppo.py:77 next_values[-1] = 0
    for (int tend = T - 1; tend >= 0; tend -= kGaeT) {
        const int tbeg = tend - kGaeT + 1 > 0 ? tend - kGaeT + 1 : 0, nt = tend - tbeg + 1;
        // every load of the pass issued before the first LDS store (unconditional, clamped into the
        // buffer): one round of HBM latency instead of one per item (the loop form waited for each
        // item's load before its LDS store: 14.5 us per 4096 x 64 launch)
        float rr[kGaeIt], vv[kGaeIt];
        uint8_t dd[kGaeIt];
#pragma unroll
        for (int u = 0; u < kGaeIt; ++u) {
            const int it = threadIdx.x + u * kGaeThreads, k = it / kGaeBlock, j = it % kGaeBlock;
            const int kc = k < nt ? k : nt - 1, ec = e0 + j < E ? e0 + j : E - 1;
            const long long i = (long long)(tbeg + kc) * E + ec;
            rr[u] = (float)reward[i];  // python float promoted into the fp32 tensor op
            vv[u] = value[i];
            dd[u] = done[i];
        }
#pragma unroll
        for (int u = 0; u < kGaeIt; ++u) {
            const int it = threadIdx.x + u * kGaeThreads, k = it / kGaeBlock, j = it % kGaeBlock;
            if (k < nt && e0 + j < E) {
                sr[k][j] = rr[u];
                sv[k][j] = vv[u];
                sd[k][j] = dd[u];
            }
        }
        __syncthreads();
        if (walker) {
#pragma unroll 8
            for (int k = nt - 1; k >= 0; --k) {
                const float r = sr[k][lane], v = sv[k][lane];
                float delta;
                if (sd[k][lane]) {  // v_next = 0.0, carry cut (ppo.py:84-87)
                    delta = r - v;
                    gae = delta;
                } else {
                    delta = (r + g * nv) - v;
                    gae = delta + gl * gae;
                }
                const float R = gae + v;
                const float A = R - v;  // ppo.py:91 advantages = returns - values
                sret[k][lane] = R;
                sadv[k][lane] = A;
                s += (double)A;
                s2 += (double)A * (double)A;
                nv = v;
            }
        }
        __syncthreads();
        for (int it = threadIdx.x; it < nt * kGaeBlock; it += kGaeThreads) {
            const int k = it / kGaeBlock, j = it % kGaeBlock, e = e0 + j;
            if (e < E) {
                const long long i = (long long)(tbeg + k) * E + e;
                ret[i] = sret[k][j];
                adv[i] = sadv[k][j];
            }
        }
        __syncthreads();  // the next pass rewrites the LDS tiles
    }
    if (partials) {
        // waves 1-3 add zeros: the same value as the per-env-wave reduction of block_sum2<64>
        block_sum2<kGaeThreads>(s, s2);
        if (threadIdx.x == 0) {
            partials[2 * blockIdx.x] = s;
            partials[2 * blockIdx.x + 1] = s2;
        }
    }
}

__global__ __launch_bounds__(kRedBlock) void k_adv_partials(const float* __restrict__ adv, long long n,
                                                            double* __restrict__ partials) {
    double s = 0.0, s2 = 0.0;
    for (long long i = (long long)blockIdx.x * kRedBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kRedBlock) {
        const double a = adv[i];
        s += a;
        s2 += a * a;
    }
    block_sum2<kRedBlock>(s, s2);
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = s;
        partials[2 * blockIdx.x + 1] = s2;
    }
}

// Every block folds the (few) partials in the same fixed order, then normalises its slice.
__global__ __launch_bounds__(kRedBlock) void k_adv_normalize(float* __restrict__ adv, long long n,
                                                             const double* __restrict__ partials, int np,
                                                             long long n_total, double* __restrict__ stats) {
    __shared__ float sm[2];
    // this thread's advantages (kNormPer grid-stride items) loaded ahead of the partials' sum, so
    // both round trips overlap (unconditional: clamped into the buffer)
    float av[kNormPer];
    {
        const long long stride = (long long)gridDim.x * kRedBlock, i0 = (long long)blockIdx.x * kRedBlock + threadIdx.x;
#pragma unroll
        for (int u = 0; u < kNormPer; ++u) {
            const long long i = i0 + u * stride;
            av[u] = adv[i < n ? i : n - 1];
        }
    }
    double S = 0.0, S2 = 0.0;
    if (threadIdx.x < kWave) {
        // the partials arrive 64 at a time, one per lane (one load round instead of a chain of
        // dependent loads), and are added in index order as before; lane 0 finishes
        for (int c0 = 0; c0 < np; c0 += kWave) {
            const int i = c0 + threadIdx.x, m = np - c0 < kWave ? np - c0 : kWave;
            const double a = i < np ? partials[2 * i] : 0.0, b = i < np ? partials[2 * i + 1] : 0.0;
            for (int k = 0; k < m; ++k) {
                S += readlane_d(a, k);
                S2 += readlane_d(b, k);
            }
        }
    }
    if (threadIdx.x == 0) {
        const double mean = S / (double)n_total;
        double var = n_total > 1 ? (S2 - S * mean) / (double)(n_total - 1) : __builtin_nan("");
        if (var < 0.0) var = 0.0;
        const double sd = sqrt(var);
        sm[0] = (float)mean;
        sm[1] = (float)sd;
        if (stats && blockIdx.x == 0) { stats[0] = mean; stats[1] = sd; }
    }
    __syncthreads();
    const float mean = sm[0];
    const float den = sm[1] + 1e-7f;  // ppo.py:94 (std + 1e-7) in fp32
    const long long stride = (long long)gridDim.x * kRedBlock, i0 = (long long)blockIdx.x * kRedBlock + threadIdx.x;
#pragma unroll
    for (int u = 0; u < kNormPer; ++u) {
        const long long i = i0 + u * stride;
        if (i < n) adv[i] = (av[u] - mean) / den;
    }
    for (long long i = i0 + kNormPer * stride; i < n; i += stride) adv[i] = (adv[i] - mean) / den;  // n > grid x 4
}

// Trajectory windows from the compact all-gather format (uavhip/dist.py): thread per (block,
// step, env, window slot), 14 floats each. Slot s of step t holds the row pushed at step
// k = t - 4 + s if no episode ended in [k, t - 1] (else zeros, as after UAVEnv.reset); rows of
// steps k <= 0 come from the block's first window W(0).
__global__ __launch_bounds__(256) void k_windows_from_rows(const float* __restrict__ first,
                                                           const float* __restrict__ rows,
                                                           const float* __restrict__ done, int dstride,
                                                           long long bstride, int T, int E, float* __restrict__ out,
                                                           long long total) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int s = (int)(i % 5);
    long long r = i / 5;
    const int e = (int)(r % E);
    r /= E;
    const int t = (int)(r % T);
    const long long b = r / T;
    const int k = t - (4 - s);
    const float* dn = done + b * bstride;
    bool ok = true;
    for (int m = k > 0 ? k : 0; m < t; ++m) ok = ok && dn[((long long)m * E + e) * dstride] == 0.f;
    const float* src = k >= 1 ? rows + b * bstride + ((long long)k * E + e) * 14
                              : first + b * bstride + (long long)e * 70 + (k + 4) * 14;  // W(0) = first
    float2* dst = reinterpret_cast<float2*>(out + i * 14);
#pragma unroll
    for (int q = 0; q < 7; ++q) dst[q] = ok ? reinterpret_cast<const float2*>(src)[q] : make_float2(0.f, 0.f);
}

}  // namespace uavhip

using namespace uavhip;

extern "C" int uavhip_windows_from_rows(const float* first, const float* rows, const float* done, int32_t done_stride,
                                        int64_t block_stride, int32_t blocks, int32_t T, int32_t E, float* out,
                                        uavhip_stream_t stream) {
    if (!first || !rows || !done || !out || done_stride <= 0 || blocks <= 0 || T <= 0 || E <= 0 ||
        (block_stride & 1) || (((uintptr_t)first | (uintptr_t)rows | (uintptr_t)out) & 7)) {
        set_error("uavhip_windows_from_rows: bad args (blocks=%d T=%d E=%d stride=%lld; 8-byte aligned buffers)",
                  blocks, T, E, (long long)block_stride);
        return UAVHIP_EINVAL;
    }
    const long long total = (long long)blocks * T * E * 5;
    hipLaunchKernelGGL(k_windows_from_rows, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       first, rows, done, (int)done_stride, (long long)block_stride, (int)T, (int)E, out, total);
    return check_launch("k_windows_from_rows");
}

extern "C" int32_t uavhip_gae_partials(int32_t T, int32_t E) {
    (void)T;
    return (E + kGaeBlock - 1) / kGaeBlock;
}

extern "C" int uavhip_gae(const double* reward, const uint8_t* done, const float* value, const float* last_value,
                          int32_t T, int32_t E, double gamma, double lam, float* ret, float* adv, double* partials,
                          uavhip_stream_t stream) {
    if (!reward || !done || !value || !ret || !adv || T <= 0 || E <= 0) {
        set_error("uavhip_gae: NULL buffer or T=%d E=%d", T, E);
        return UAVHIP_EINVAL;
    }
    const float g = (float)gamma;
    const float gl = (float)(gamma * lam);  // cfg.GAMMA * cfg.GAE_LAMBDA is an f64 product (ppo.py:87)
    hipLaunchKernelGGL(k_gae, dim3((E + kGaeBlock - 1) / kGaeBlock), dim3(kGaeThreads), 0, (hipStream_t)stream, reward,
                       done, value, last_value, (int)T, (int)E, g, gl, ret, adv, partials);
    return check_launch("k_gae");
}

extern "C" int uavhip_adv_partials(const float* adv, int64_t n, double* partials, int32_t n_partials,
                                   uavhip_stream_t stream) {
    if (!adv || !partials || n <= 0 || n_partials <= 0) {
        set_error("uavhip_adv_partials: bad args n=%lld np=%d", (long long)n, n_partials);
        return UAVHIP_EINVAL;
    }
    hipLaunchKernelGGL(k_adv_partials, dim3(n_partials), dim3(kRedBlock), 0, (hipStream_t)stream, adv, (long long)n,
                       partials);
    return check_launch("k_adv_partials");
}

extern "C" int uavhip_adv_normalize(float* adv, int64_t n, const double* partials, int32_t n_partials,
                                    int64_t n_total, double* stats_out, uavhip_stream_t stream) {
    if (!adv || !partials || n <= 0 || n_partials <= 0) {
        set_error("uavhip_adv_normalize: bad args n=%lld np=%d", (long long)n, n_partials);
        return UAVHIP_EINVAL;
    }
    long long blocks = (n + kRedBlock * kNormPer - 1) / (kRedBlock * kNormPer);
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_adv_normalize, dim3((unsigned)blocks), dim3(kRedBlock), 0, (hipStream_t)stream, adv,
                       (long long)n, partials, (int)n_partials, (long long)(n_total > 0 ? n_total : n), stats_out);
    return check_launch("k_adv_normalize");
}
