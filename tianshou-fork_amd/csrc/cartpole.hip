// CartPole-v1 for N envs in HBM (BASELINE config 1, test/discrete/test_ppo.py's task): the
// classic-control dynamics gymnasium publishes (cartpole.py: Euler integration, force +-10,
// x / theta thresholds 2.4 / 12 deg) behind TimeLimit(500), restated in f64 with no FMA
// contraction, in the order tianshou_amd/env/cartpole.py (host) and oracle/cartpole.py use.
// Resets draw U(-0.05, 0.05)^4 from a counter hash of (seed, env, episode, component).
#include "tsrl_common.h"

#pragma clang fp contract(off)

namespace tsrl {
namespace {

constexpr double kGravity = 9.8, kMassPole = 0.1, kTotalMass = 0.1 + 1.0, kLength = 0.5;
constexpr double kPoleMassLength = 0.1 * 0.5, kForceMag = 10.0, kTau = 0.02;
constexpr double kXThreshold = 2.4;

__device__ __forceinline__ bool beyond(double x, double theta, double th) {
    return x < -kXThreshold || x > kXThreshold || theta < -th || theta > th;
}

__global__ void cartpole_step_kernel(const int64_t* __restrict__ ids, int64_t k,
                                     const int64_t* __restrict__ act, int64_t max_steps,
                                     double theta_threshold, double* __restrict__ state,
                                     int64_t* __restrict__ ep_t, float* __restrict__ obs_out,
                                     double* __restrict__ rew_out, uint8_t* __restrict__ term_out,
                                     uint8_t* __restrict__ trunc_out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= k) return;
    const int64_t e = ids ? ids[r] : r;
    double* s = state + 4 * e;
    double x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
    // gymnasium's reward: 1 while the episode runs and on the terminating step, 0 on steps
    // taken after termination (steps_beyond_terminated) -- a function of the state
    const bool was_term = beyond(x, theta, theta_threshold);
    const double force = act[r] == 1 ? kForceMag : -kForceMag;
    const double costheta = cos(theta);
    const double sintheta = sin(theta);
    const double temp = (force + kPoleMassLength * (theta_dot * theta_dot) * sintheta) / kTotalMass;
    const double thetaacc = (kGravity * sintheta - costheta * temp) /
                            (kLength * (4.0 / 3.0 - kMassPole * (costheta * costheta) / kTotalMass));
    const double xacc = temp - kPoleMassLength * thetaacc * costheta / kTotalMass;
    x = x + kTau * x_dot;
    x_dot = x_dot + kTau * xacc;
    theta = theta + kTau * theta_dot;
    theta_dot = theta_dot + kTau * thetaacc;
    s[0] = x, s[1] = x_dot, s[2] = theta, s[3] = theta_dot;
    const bool term = beyond(x, theta, theta_threshold);
    const int64_t t = ep_t[e] + 1;
    ep_t[e] = t;
    float4 o = make_float4((float)x, (float)x_dot, (float)theta, (float)theta_dot);
    *reinterpret_cast<float4*>(obs_out + 4 * r) = o;
    rew_out[r] = was_term ? 0.0 : 1.0;
    term_out[r] = term;
    trunc_out[r] = t >= max_steps;
}

__global__ void cartpole_reset_kernel(const int64_t* __restrict__ ids,
                                      const uint8_t* __restrict__ mask, int64_t k, uint64_t seed,
                                      double* __restrict__ state, int64_t* __restrict__ ep_j,
                                      int64_t* __restrict__ ep_t, float* __restrict__ obs_out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= k || (mask && !mask[r])) return;
    const int64_t e = ids ? ids[r] : r;
    const int64_t j = ep_j[e] + 1;
    ep_j[e] = j;
    ep_t[e] = 0;
    const uint64_t key = sm64(sm64(sm64(seed) ^ (uint64_t)e) ^ (uint64_t)j);
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double u = (double)(sm64(key ^ (uint64_t)(i + 1)) >> 11) * (1.0 / 9007199254740992.0);
        v[i] = -0.05 + (0.05 - -0.05) * u;  // Generator.uniform: low + (high - low) * u
        state[4 * e + i] = v[i];
    }
    *reinterpret_cast<float4*>(obs_out + 4 * r) =
        make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_cartpole_step(const int64_t* ids, int64_t k, const int64_t* act,
                                  int64_t max_steps, double* state, int64_t* ep_t,
                                  float* obs_out, double* rew_out, uint8_t* term_out,
                                  uint8_t* trunc_out, void* stream) {
    TSRL_CHECK_ARG(k >= 0 && max_steps > 0, "tsrl_cartpole_step: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(act && state && ep_t && obs_out && rew_out && term_out && trunc_out &&
                       aligned16(obs_out),
                   "tsrl_cartpole_step: null / misaligned pointer");
    const double theta_threshold = 12 * 2 * 3.141592653589793 / 360;  // math.pi
    hipLaunchKernelGGL(cartpole_step_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0,
                       as_stream(stream), ids, k, act, max_steps, theta_threshold, state, ep_t,
                       obs_out, rew_out, term_out, trunc_out);
    TSRL_LAUNCH_CHECK("tsrl_cartpole_step");
    return 0;
}

extern "C" int tsrl_cartpole_reset(const int64_t* ids, const uint8_t* mask, int64_t k,
                                   uint64_t seed, double* state, int64_t* ep_j, int64_t* ep_t,
                                   float* obs_out, void* stream) {
    TSRL_CHECK_ARG(k >= 0, "tsrl_cartpole_reset: k < 0");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(state && ep_j && ep_t && obs_out && aligned16(obs_out),
                   "tsrl_cartpole_reset: null / misaligned pointer");
    hipLaunchKernelGGL(cartpole_reset_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0,
                       as_stream(stream), ids, mask, k, seed, state, ep_j, ep_t, obs_out);
    TSRL_LAUNCH_CHECK("tsrl_cartpole_reset");
    return 0;
}
