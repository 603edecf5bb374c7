// metrics.hip -- per-episode training statistics of main_train.py:122-136 (the sums behind its CSV
// columns, :161-195) accumulated on device over rollout chunks: one thread per env walks the
// chunk in time order, so no per-step host sync is needed to log training curves.
#include "common.hpp"

namespace uavhip {

__global__ __launch_bounds__(256) void k_episode_stats(const double* __restrict__ reward,
                                                       const uint8_t* __restrict__ done,
                                                       const int8_t* __restrict__ action,
                                                       const double* __restrict__ info,
                                                       const float* __restrict__ value, int T, int E,
                                                       double* __restrict__ acc, double* __restrict__ records,
                                                       int max_records, uint32_t* __restrict__ n_records) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    double a[UAVHIP_EP_COUNT];
    double* ae = acc + (size_t)e * UAVHIP_EP_COUNT;
#pragma unroll
    for (int i = 0; i < UAVHIP_EP_COUNT; ++i) a[i] = ae[i];
    for (int t = 0; t < T; ++t) {
        const size_t te = (size_t)t * E + e;
        if (a[UAVHIP_EP_STEPS] == 0.0) a[UAVHIP_EP_Q0] = (double)value[te];  // episode start state
        const double* in = info + te * UAVHIP_INFO_COUNT;
        const double ncov = in[UAVHIP_INFO_NUM_ASSIGNED];
        a[UAVHIP_EP_STEPS] += 1.0;
        a[UAVHIP_EP_REWARD] = a[UAVHIP_EP_REWARD] + reward[te];
        a[UAVHIP_EP_J_SUM] = a[UAVHIP_EP_J_SUM] + in[UAVHIP_INFO_J];
        a[UAVHIP_EP_MAX_COV] = ncov > a[UAVHIP_EP_MAX_COV] ? ncov : a[UAVHIP_EP_MAX_COV];
        if (action[te] == 1) {
            a[UAVHIP_EP_ACTION1] += 1.0;
            if (in[UAVHIP_INFO_IS_VALID] == 1.0) a[UAVHIP_EP_VALID] += 1.0;
        }
        if (ncov > 0.0) {
            a[UAVHIP_EP_PDMG_SUM] = a[UAVHIP_EP_PDMG_SUM] + in[UAVHIP_INFO_AVG_P_DMG];
            a[UAVHIP_EP_PFINAL_SUM] = a[UAVHIP_EP_PFINAL_SUM] + in[UAVHIP_INFO_AVG_P_FINAL];
            a[UAVHIP_EP_ASSIGN_STEPS] += 1.0;
        }
        if (done[te]) {
            a[UAVHIP_EP_ENV] = (double)e;
            a[UAVHIP_EP_EPISODE] = in[UAVHIP_INFO_EPISODE];
            const uint32_t slot = atomicAdd(n_records, 1u);
            if ((int)slot < max_records) {
                double* r = records + (size_t)slot * UAVHIP_EP_COUNT;
#pragma unroll
                for (int i = 0; i < UAVHIP_EP_COUNT; ++i) r[i] = a[i];
            }
#pragma unroll
            for (int i = 0; i < UAVHIP_EP_COUNT; ++i) a[i] = 0.0;
        }
    }
#pragma unroll
    for (int i = 0; i < UAVHIP_EP_COUNT; ++i) ae[i] = a[i];
}

}  // namespace uavhip

extern "C" int uavhip_episode_stats(const double* reward, const uint8_t* done, const int8_t* action,
                                    const double* info, const float* value, int32_t T, int32_t E, double* acc,
                                    double* records, int32_t max_records, uint32_t* n_records,
                                    uavhip_stream_t stream) {
    using namespace uavhip;
    if (!reward || !done || !action || !info || !value || !acc || !n_records || (max_records > 0 && !records) ||
        T <= 0 || E <= 0 || max_records < 0) {
        set_error("uavhip_episode_stats: NULL pointer or bad sizes (T=%d, E=%d, max_records=%d)", T, E, max_records);
        return UAVHIP_EINVAL;
    }
    hipLaunchKernelGGL(k_episode_stats, dim3((E + 255) / 256), dim3(256), 0, (hipStream_t)stream, reward, done, action,
                       info, value, (int)T, (int)E, acc, records, (int)max_records, n_records);
    return check_launch("k_episode_stats");
}
