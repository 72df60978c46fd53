// torch.nn.utils.clip_grad_norm_ + torch.optim.Adam.step of the fused PPO minibatch
// (tianshou/policy/modelfree/ppo.py:143-151) as ONE launch over flat f32 storage: the fused
// MLP keeps every parameter, gradient and Adam moment of the actor-critic in flat buffers
// (policy/fused_mlp.py bind_adam), so torch's per-tensor foreach norm, scale and fused Adam
// kernels (~50-60 us per minibatch, launch- and latency-bound on 57 763 parameters) become
// one launch over 2048-element slices (each workgroup's squared slice norm, an in-kernel
// hand-off of the slice norms, Adam) plus, on the last minibatch only, the in-place gradient
// scaling.
//
//   norm  = ||g||_2 (f64 sum of squares), coef = max_norm / (norm + 1e-6) clamped at 1,
//   g    *= coef                                   (clip_grad_norm_, torch/nn/utils/clip_grad.py)
//   t    += 1
//   m     = beta1 m + (1 - beta1) g,  v = beta2 v + (1 - beta2) g^2
//   p    -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
// (torch's fused Adam formula, amsgrad / weight_decay / maximize off).  The step counter
// lives on device, so HIP-graph replays of whole epochs advance it.
#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr int OTPB = 256;
constexpr int OCHUNK = 2048;  // elements updated per workgroup

struct AdamArgs {
    float lr, beta1, beta2, eps, max_norm;
};

// Optional epilogue: the updated first-layer weights of both nets re-split into the bf16x6
// planes the next minibatch's tsrl_mlp_l1_fwd_x6 reads (the split_w kernel's layout:
// out[plane][f][k], f < 64 actor rows, >= 64 critic rows, k < kp; columns >= d stay zero).
struct SplitOut {
    __bf16* out;
    int64_t off_a, off_c, d, kp, plane;
};

__device__ __forceinline__ void split_store(const SplitOut& so, int64_t i, float x) {
    int64_t r = -1, f0 = 0;
    if (i >= so.off_a && i < so.off_a + 64 * so.d) {
        r = i - so.off_a;
    } else if (i >= so.off_c && i < so.off_c + 64 * so.d) {
        r = i - so.off_c;
        f0 = 64;
    }
    if (r < 0) return;
    const int64_t f = f0 + r / so.d, k = r - (r / so.d) * so.d;
    const __bf16 a0 = (__bf16)x;
    const float r1 = x - (float)a0;
    const __bf16 a1 = (__bf16)r1;
    __bf16* o = so.out + f * so.kp + k;
    o[0] = a0;
    o[so.plane] = a1;
    o[2 * so.plane] = (__bf16)(r1 - (float)a1);
}

// Sum of squares of each 2048-element gradient slice (f64), one workgroup per slice, in the
// order clip_adam_kernel's in-kernel form uses: the separate launch for grids too large to be
// resident at once (more than 256 slices, 2^19 parameters).
__global__ __launch_bounds__(OTPB) void norm_partials_kernel(const float* __restrict__ g,
                                                             int64_t n, double* partials) {
    __shared__ double red[OTPB / kWave];
    const int t = threadIdx.x;
    const int64_t i0 = (int64_t)blockIdx.x * OCHUNK;
    double ss = 0.0;
#pragma unroll
    for (int q = 0; q < OCHUNK / OTPB; ++q) {  // independent loads, all in flight together
        const int64_t i = i0 + q * OTPB + t;
        const double x = i < n ? (double)g[i] : 0.0;
        ss += x * x;
    }
    ss = wave_sum(ss);
    if ((t & (kWave - 1)) == 0) red[t / kWave] = ss;
    __syncthreads();
    if (t == 0) {
        double tot = 0.0;
        for (int w = 0; w < OTPB / kWave; ++w) tot += red[w];
        partials[blockIdx.x] = tot;
    }
}

// Each workgroup updates its own 2048-element slice with the clip coefficient of the slice
// norms.  Clipping: every workgroup first publishes its slice's f64 sum of squares (per thread
// the 8 elements in order, a wave reduction, the 4 waves in order) and arrives at ticket[1]
// (agent-scope release); it then waits until all have arrived (acquire; at most 29
// workgroups for the 57 763-parameter nets, all resident together) and folds the slice sums
// in the same fixed order in every workgroup.  This replaces round 3's separate
// norm_partials launch (5.5 us + a dependent boundary per minibatch) with a hand-off of one
// memory round trip.  The last workgroup to finish (ticket[0]) advances the device step
// counter and re-arms both tickets.
__global__ __launch_bounds__(OTPB) void clip_adam_kernel(float* __restrict__ p,
                                                         float* __restrict__ g,
                                                         float* __restrict__ m,
                                                         float* __restrict__ v, int64_t n,
                                                         float* __restrict__ step, int64_t nstep,
                                                         AdamArgs a, double* __restrict__ partials,
                                                         float* __restrict__ norm_out,
                                                         unsigned int* ticket, const float* __restrict__ lr_dev,
                                                         SplitOut so, int fused_norm) {
    __shared__ float s_scale;
    __shared__ int s_late;  // the slice-norm hand-off timed out
    const int t = threadIdx.x;
    const bool clip = a.max_norm > 0.0f;
    const float st = step[0] + 1.0f;
    const int64_t i0 = (int64_t)blockIdx.x * OCHUNK;
    // every element of this thread's slice loaded first, all in flight together and under the
    // fold of the partial norms (one memory latency per launch instead of one per element)
    constexpr int EPT = OCHUNK / OTPB;
    float gr[EPT], mr[EPT], vr[EPT], pr[EPT];
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
        const int64_t i = i0 + q * OTPB + t;
        const bool in = i < n;
        gr[q] = in ? g[i] : 0.0f;
        mr[q] = in ? m[i] : 0.0f;
        vr[q] = in ? v[i] : 0.0f;
        pr[q] = in ? p[i] : 0.0f;
    }
    if (t == 0) s_late = 0;
    if (clip && fused_norm) {
        __shared__ double red[OTPB / kWave];
        double ss = 0.0;
#pragma unroll
        for (int q = 0; q < EPT; ++q) {
            const double x = (double)gr[q];
            ss += x * x;
        }
        ss = wave_sum(ss);
        if ((t & (kWave - 1)) == 0) red[t / kWave] = ss;
        __syncthreads();
        if (t == 0) {
            double tot = 0.0;
            for (int w = 0; w < OTPB / kWave; ++w) tot += red[w];
            __hip_atomic_store(&partials[blockIdx.x], tot, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&ticket[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            // bounded wait: every workgroup of this small grid (<= the host's resident-slot
            // count) is resident, so the arrivals never depend on a workgroup that waits; if
            // the bound still runs out (e.g. another process holding the CUs), the norm is
            // poisoned with NaN below -- a loud NaN step (and norm_out NaN) instead of a
            // silently wrong clip coefficient from missing partials
            int late = 1;
            for (uint32_t spin = 0; spin < (1u << 24); ++spin) {
                if (__hip_atomic_load(&ticket[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >=
                    gridDim.x) {
                    late = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_late = late;
            // the late slice alone would step with a NaN coefficient while the others may
            // have seen every arrival: publish the timeout to a sticky device flag the host
            // checks (FlatAdam.check_handoff), so the whole step is rejected, not one slice
            if (late)
                __hip_atomic_store(&ticket[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (clip) {
        __syncthreads();
        // the slice sums folded by wave 0 in the same fixed order in every workgroup (so every
        // workgroup gets the identical coefficient)
        if (t < kWave) {
            double ss = 0.0;
            for (int64_t b = t; b < gridDim.x; b += kWave)
                ss += __hip_atomic_load(&partials[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ss = wave_sum(ss);
            if (t == 0) {
                const float norm = s_late ? __builtin_nanf("") : (float)sqrt(ss);
                // torch.clamp(coef, max=1.0): a NaN norm (a NaN or infinite gradient element)
                // gives a NaN coefficient that reaches every gradient, as in clip_grad_norm_
                // (fminf would return 1.0 and leave the finite gradients unclipped)
                const float coef = a.max_norm / (norm + 1e-6f);
                s_scale = coef > 1.0f ? 1.0f : coef;
                if (blockIdx.x == 0) {
                    norm_out[0] = norm;
                    norm_out[1] = s_scale;
                }
            }
        }
        __syncthreads();
    }
    const float scale = clip ? s_scale : 1.0f;
    const float bc1 = 1.0f - powf(a.beta1, st);
    const float bc2_sqrt = sqrtf(1.0f - powf(a.beta2, st));
    const float step_size = (lr_dev ? *lr_dev : a.lr) / bc1;
    // g is only read here (other workgroups are still summing it); the clipped gradient is
    // written back by clip_scale_kernel, the next launch on the stream
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
        const int64_t i = i0 + q * OTPB + t;
        if (i >= n) break;
        const float gi = gr[q] * scale;
        const float mi = a.beta1 * mr[q] + (1.0f - a.beta1) * gi;
        const float vi = a.beta2 * vr[q] + (1.0f - a.beta2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float pi = pr[q] - step_size * mi / (sqrtf(vi) / bc2_sqrt + a.eps);
        p[i] = pi;
        if (so.out) split_store(so, i, pi);
    }
    // the ticket orders only reads of step[0] (every wave's has returned: its value was used
    // above, and the barrier waits for all waves) before the last workgroup's write, so it is
    // relaxed: an acquire-release at agent scope would write back and invalidate this XCD's L2
    __syncthreads();
    if (t == 0) {
        const unsigned int done = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
        if (done == gridDim.x - 1) {  // every workgroup has read step[0] and the gradients
            for (int64_t i = 0; i < nstep; ++i) step[i] = st;
            // every workgroup has also passed the slice-norm wait (it precedes its ticket add)
            __hip_atomic_store(&ticket[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// clip_grad_norm_'s in-place scaling of the gradients (what p.grad holds after the step)
__global__ __launch_bounds__(OTPB) void clip_scale_kernel(float* __restrict__ g, int64_t n,
                                                          const float* __restrict__ norm_scale) {
    const float s = norm_scale[1];
    for (int64_t i = (int64_t)blockIdx.x * OTPB + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * OTPB)
        g[i] *= s;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_clip_adam_partials(int64_t n) { return (n + OCHUNK - 1) / OCHUNK; }

extern "C" int tsrl_clip_adam(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                              int64_t n, float* step, int64_t nstep, float lr, float beta1,
                              float beta2, float eps, float max_norm, double* partials,
                              float* norm_out, unsigned int* ticket, const float* lr_dev,
                              const tsrl_w1_split* split, int scale_grads, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && nstep >= 1, "tsrl_clip_adam: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && step && ticket,
                   "tsrl_clip_adam: null pointer");
    const int64_t grid = (n + OCHUNK - 1) / OCHUNK;
    TSRL_CHECK_ARG(max_norm <= 0.0f || (norm_out && partials),
                   "tsrl_clip_adam: clipping needs partials and norm_out[2]");
    // the in-kernel slice-norm hand-off needs every workgroup resident at once: up to one
    // slice per CU of this device (hipDeviceAttributeMultiprocessorCount, 256 on MI355X);
    // larger parameter sets take the separate norm launch
    const int fused_norm = grid <= n_cus();
    if (max_norm > 0.0f && !fused_norm) {
        hipLaunchKernelGGL(norm_partials_kernel, dim3((unsigned)grid), dim3(OTPB), 0,
                           as_stream(stream), grad, n, partials);
        TSRL_LAUNCH_CHECK("tsrl_clip_adam (norm)");
    }
    const AdamArgs a{lr, beta1, beta2, eps, max_norm};
    SplitOut so{nullptr, 0, 0, 1, 1, 0};
    if (split) {
        TSRL_CHECK_ARG(split->out && split->d > 0 && split->kp >= split->d &&
                           split->off_a >= 0 && split->off_c >= 0 &&
                           split->off_a + 64 * split->d <= n && split->off_c + 64 * split->d <= n,
                       "tsrl_clip_adam: bad first-layer split ranges");
        so = SplitOut{reinterpret_cast<__bf16*>(split->out), split->off_a, split->off_c,
                      split->d, split->kp, 128 * split->kp};
    }
    hipLaunchKernelGGL(clip_adam_kernel, dim3((unsigned)grid), dim3(OTPB), 0,
                       as_stream(stream), param, grad, exp_avg, exp_avg_sq, n, step, nstep, a,
                       partials, norm_out, ticket, lr_dev, so, fused_norm);
    TSRL_LAUNCH_CHECK("tsrl_clip_adam");
    if (max_norm > 0.0f && scale_grads) {
        const unsigned g2 = (unsigned)std::min<int64_t>((n + OTPB - 1) / OTPB, 1024);
        hipLaunchKernelGGL(clip_scale_kernel, dim3(g2), dim3(OTPB), 0, as_stream(stream), grad,
                           n, norm_out);
        TSRL_LAUNCH_CHECK("tsrl_clip_adam (scale)");
    }
    return 0;
}
