// Observation RunningMeanStd for VectorEnvNormObs (tianshou/env/venv_wrappers.py:65-112,
// tianshou/utils/statistics.py:69-114), kept on device.
//
// merge : batch (mean, var) from the env kernel's column partials (f64), then the Chan
//         parallel merge of RunningMeanStd.update, stored back as f32 like the reference.
// norm  : clip((x - mean) / sqrt(var + eps), +-clip) in f32, the reference's exact op order.
#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;

__global__ __launch_bounds__(TPB) void rms_merge_kernel(const double* partials, int64_t nblk,
                                                        int64_t dim, const uint8_t* mask,
                                                        int64_t k, float* mean, float* var,
                                                        double* count) {
    __shared__ double sh_cnt[TPB / kWave];
    // batch count
    double c = 0.0;
    if (mask) {
        for (int64_t r = threadIdx.x; r < k; r += TPB) c += mask[r] ? 1.0 : 0.0;
    } else if (threadIdx.x == 0) {
        c = (double)k;
    }
    c = wave_sum(c);
    if ((threadIdx.x & (kWave - 1)) == 0) sh_cnt[threadIdx.x / kWave] = c;
    __syncthreads();
    double bc = 0.0;
    for (int w = 0; w < TPB / kWave; ++w) bc += sh_cnt[w];
    if (bc == 0.0) return;  // nothing reset / stepped: no update (the reference skips it)
    const double old_count = *count;
    const double tot = old_count + bc;
    for (int64_t d = threadIdx.x; d < dim; d += TPB) {
        double s = 0.0, ss = 0.0;
        for (int64_t b = 0; b < nblk; ++b) {
            s += partials[(b * dim + d) * 2];
            ss += partials[(b * dim + d) * 2 + 1];
        }
        const double bm = s / bc;
        double bv = ss / bc - bm * bm;
        bv = bv < 0.0 ? 0.0 : bv;
        const double m0 = (double)mean[d];
        const double v0 = (double)var[d];
        const double delta = bm - m0;
        const double new_mean = m0 + delta * bc / tot;
        const double m2 = v0 * old_count + bv * bc + delta * delta * old_count * bc / tot;
        mean[d] = (float)new_mean;
        var[d] = (float)(m2 / tot);
    }
    __syncthreads();
    if (threadIdx.x == 0) *count = tot;
}

__device__ __forceinline__ float norm1(float x, float m, float v, float eps, float clip) {
    float y = (x - m) / __builtin_sqrtf(v + eps);
    if (clip > 0.0f) y = fminf(fmaxf(y, -clip), clip);
    return y;
}

__global__ __launch_bounds__(TPB) void rms_norm_kernel(const float* x, const uint8_t* mask,
                                                       int64_t k, int64_t dim,
                                                       const float* mean, const float* var,
                                                       float eps, float clip, float* out) {
    const int64_t total = k * dim;
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * TPB) {
        const int64_t r = i / dim;
        if (mask && !mask[r]) continue;
        const int64_t d = i - r * dim;
        out[i] = norm1(x[i], mean[d], var[d], eps, clip);
    }
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_rms_merge(const double* col_partials, int64_t nblk, int64_t dim,
                              const uint8_t* mask, int64_t k, float* mean, float* var,
                              double* count, void* stream) {
    TSRL_CHECK_ARG(col_partials && mean && var && count && dim > 0 && nblk >= 0 && k >= 0,
                   "tsrl_rms_merge: bad arguments");
    if (k == 0) return 0;
    hipLaunchKernelGGL(rms_merge_kernel, dim3(1), dim3(TPB), 0, as_stream(stream), col_partials,
                       nblk, dim, mask, k, mean, var, count);
    TSRL_LAUNCH_CHECK("tsrl_rms_merge");
    return 0;
}

extern "C" int tsrl_rms_norm_rows(const float* x, const uint8_t* mask, int64_t k, int64_t dim,
                                  const float* mean, const float* var, float eps, float clip,
                                  float* out, void* stream) {
    TSRL_CHECK_ARG(x && mean && var && out && dim > 0 && k >= 0, "tsrl_rms_norm_rows: bad args");
    if (k == 0) return 0;
    const int64_t total = k * dim;
    const int64_t grid = min((total + TPB - 1) / TPB, (int64_t)8192);
    hipLaunchKernelGGL(rms_norm_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream), x,
                       mask, k, dim, mean, var, eps, clip, out);
    TSRL_LAUNCH_CHECK("tsrl_rms_norm_rows");
    return 0;
}
