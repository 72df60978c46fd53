// Fused PPO clipped-surrogate + value + entropy loss with its analytic gradient
// (PPOPolicy.learn minibatch body, tianshou/policy/modelfree/ppo.py:106-151) for the
// Gaussian actor Independent(Normal(mu, exp(log_std)), 1) with state-independent log_std
// (ActorProb, utils/net/continuous.py:218-235; fixed_std_normal, utils/models.py:96-97).
//
// One pass over the minibatch rows: gathers act/logp_old/adv/returns/v_s through the
// minibatch index (no materialised minibatch copy), computes log-prob, ratio, the clipped
// objective (dual-clip optional), the value loss (value-clip optional), and writes
// d(mean loss)/d(mu) [b, A] and d/d(value) [b] directly; per-block partial sums of the loss
// terms and of d/d(log_std) are reduced deterministically (fixed order) afterwards.
// torch's tie rules are reproduced: min/max split the gradient in half on ties, clamp passes
// it on the closed interval.
#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int NW = TPB / kWave;
constexpr int MAX_ACT = 64;
constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;  // math.log(math.sqrt(2*pi))

struct Params {
    float lo, hi, eps_clip, dual, vf_coef, ent_coef, adv_eps;
    int value_clip, norm_adv, use_dual;
    double inv_b;
};

Params make_params(const tsrl_ppo_params& p) {
    Params q;
    q.lo = (float)(1.0 - p.eps_clip);
    q.hi = (float)(1.0 + p.eps_clip);
    q.eps_clip = (float)p.eps_clip;
    q.dual = (float)p.dual_clip;
    q.use_dual = p.dual_clip > 0.0;
    q.vf_coef = (float)p.vf_coef;
    q.ent_coef = (float)p.ent_coef;
    q.adv_eps = (float)p.adv_eps;
    q.value_clip = p.value_clip;
    q.norm_adv = p.norm_adv;
    q.inv_b = 1.0 / p.b_global;
    return q;
}

__global__ __launch_bounds__(TPB) void adv_moments_kernel(const float* adv, const int64_t* idx,
                                                          int64_t b, double* partials) {
    __shared__ double sh[NW][2];
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    double s = 0.0, ss = 0.0;
    if (r < b) {
        const double a = (double)adv[idx ? idx[r] : r];
        s = a;
        ss = a * a;
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        sh[w][0] = s;
        sh[w][1] = ss;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        double t = 0.0;
        for (int i = 0; i < NW; ++i) t += sh[i][threadIdx.x];
        partials[2 * blockIdx.x + threadIdx.x] = t;
    }
}

__global__ __launch_bounds__(TPB) void reduce_partials_kernel(const double* partials,
                                                              int64_t nblk, int64_t width,
                                                              double* out) {
    __shared__ double sh[TPB];
    for (int64_t c = 0; c < width; ++c) {
        double s = 0.0;
        for (int64_t i = threadIdx.x; i < nblk; i += TPB) s += partials[i * width + c];
        sh[threadIdx.x] = s;
        __syncthreads();
        for (int st = TPB / 2; st > 0; st >>= 1) {
            if (threadIdx.x < st) sh[threadIdx.x] += sh[threadIdx.x + st];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[c] = sh[0];
        __syncthreads();
    }
}

// Advantage moments of every minibatch of an epoch at once (one all-reduce per epoch under
// data parallelism instead of one per minibatch).  Segment g = rows [bounds[g], bounds[g+1])
// of idx; workgroup (p, g) folds a strided 1/nparts share of segment g into partials[g][p],
// then one workgroup per segment sums its partials in fixed order.
__global__ __launch_bounds__(TPB) void adv_moments_seg_kernel(const float* adv, const int64_t* idx,
                                                              const int64_t* bounds, int nparts,
                                                              double* partials) {
    __shared__ double sh[NW][2];
    const int g = blockIdx.y;
    const int64_t s0 = bounds[g], s1 = bounds[g + 1];
    double s = 0.0, ss = 0.0;
    for (int64_t r = s0 + (int64_t)blockIdx.x * TPB + threadIdx.x; r < s1;
         r += (int64_t)nparts * TPB) {
        const double a = (double)adv[idx ? idx[r] : r];
        s += a;
        ss += a * a;
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        sh[w][0] = s;
        sh[w][1] = ss;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        double t = 0.0;
        for (int i = 0; i < NW; ++i) t += sh[i][threadIdx.x];
        partials[((int64_t)g * nparts + blockIdx.x) * 2 + threadIdx.x] = t;
    }
}

__global__ __launch_bounds__(kWave) void adv_moments_seg_reduce_kernel(const double* partials,
                                                                       int nparts, double* out) {
    const int g = blockIdx.x;
    double s = 0.0, ss = 0.0;
    for (int i = threadIdx.x; i < nparts; i += kWave) {
        s += partials[((int64_t)g * nparts + i) * 2];
        ss += partials[((int64_t)g * nparts + i) * 2 + 1];
    }
    s = wave_sum(s);
    ss = wave_sum(ss);
    if (threadIdx.x == 0) {
        out[2 * g] = s;
        out[2 * g + 1] = ss;
    }
}

// One workgroup = 256 minibatch rows.  The [256, A] mu tile (contiguous) and the gathered
// act rows are staged through LDS with coalesced / row-contiguous loads, the per-row math
// reads LDS (row stride A: conflict-free for odd A), and grad_mu goes back out through the
// same LDS tile as one contiguous coalesced store.
__global__ __launch_bounds__(TPB) void gauss_fwd_bwd_kernel(
    const float* mu, const float* log_std, const float* value, const float* act,
    const float* logp_old, const float* adv, const float* ret, const float* v_s,
    const int64_t* idx, int64_t b, int64_t A, const double* adv_sums, Params p,
    float* grad_mu, float* grad_value, double* partials) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* s_mu = smem;             // [TPB * A]
    float* s_act = smem + TPB * A;  // [TPB * A]
    __shared__ float s_var[MAX_ACT], s_ls[MAX_ACT];
    __shared__ double red[NW][4 + MAX_ACT];
    const int w = threadIdx.x / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r0 = (int64_t)blockIdx.x * TPB;
    const int nrows = (int)min((int64_t)TPB, b - r0);
    for (int a = threadIdx.x; a < A; a += TPB) {
        const float sig = expf(log_std[a]);
        s_var[a] = sig * sig;
        s_ls[a] = logf(sig);
    }
    const int nel = nrows * (int)A;
    const float* mu_blk = mu + r0 * A;
    for (int f = threadIdx.x; f < nel; f += TPB) s_mu[f] = mu_blk[f];
    for (int f = threadIdx.x; f < nel; f += TPB) {
        const int row = f / (int)A;
        const int a = f - row * (int)A;
        const int64_t j = idx ? idx[r0 + row] : r0 + row;
        s_act[f] = act[j * A + a];
    }
    __syncthreads();
    float mean_f = 0.0f, std_f = 1.0f;
    if (p.norm_adv) {
        const double n = 1.0 / p.inv_b;
        const double m = adv_sums[0] / n;
        const double var = (adv_sums[1] - adv_sums[0] * m) / (n - 1.0);
        mean_f = (float)m;
        std_f = (float)sqrt(var > 0.0 ? var : 0.0);
    }
    const int t = threadIdx.x;
    const bool live = t < nrows;
    const int64_t r = r0 + t;
    const int64_t j = live ? (idx ? idx[r] : r) : 0;
    float* my_mu = s_mu + t * A;
    const float* my_act = s_act + t * A;
    float g_logp = 0.0f;
    double clip_term = 0.0, vf_term = 0.0;
    if (live) {
        float an = adv[j];
        if (p.norm_adv) an = (an - mean_f) / (std_f + p.adv_eps);
        float logp = 0.0f;
        for (int64_t a = 0; a < A; ++a) {
            const float diff = my_act[a] - my_mu[a];
            logp += -(diff * diff) / (2.0f * s_var[a]) - s_ls[a] - LOG_SQRT_2PI;
        }
        const float ratio = expf(logp - logp_old[j]);
        const float surr1 = ratio * an;
        const float rc = fminf(fmaxf(ratio, p.lo), p.hi);
        const float surr2 = rc * an;
        const float in_rng = (ratio >= p.lo && ratio <= p.hi) ? 1.0f : 0.0f;
        float clip1, d1;
        if (surr1 < surr2) {
            clip1 = surr1;
            d1 = an;
        } else if (surr2 < surr1) {
            clip1 = surr2;
            d1 = in_rng * an;
        } else {
            clip1 = surr1;
            d1 = 0.5f * an + 0.5f * in_rng * an;
        }
        float obj = clip1, dobj = d1;
        if (p.use_dual && an < 0.0f) {
            const float tt = p.dual * an;
            if (clip1 > tt) {
                obj = clip1;
            } else if (clip1 < tt) {
                obj = tt;
                dobj = 0.0f;
            } else {
                obj = clip1;
                dobj = 0.5f * d1;
            }
        }
        clip_term = -(double)obj;
        g_logp = (float)(-(double)dobj * (double)ratio * p.inv_b);

        const float v = value[r];
        const float rt = ret[j];
        float dv;
        if (p.value_clip) {
            const float vs = v_s[j];
            const float dlt = v - vs;
            const float dcl = fminf(fmaxf(dlt, -p.eps_clip), p.eps_clip);
            const float vcl = vs + dcl;
            const float e1 = rt - v, e2 = rt - vcl;
            const float vf1 = e1 * e1, vf2 = e2 * e2;
            const float g1 = -2.0f * e1;
            const float g2 = (dlt >= -p.eps_clip && dlt <= p.eps_clip) ? -2.0f * e2 : 0.0f;
            if (vf1 > vf2) {
                vf_term = vf1;
                dv = g1;
            } else if (vf2 > vf1) {
                vf_term = vf2;
                dv = g2;
            } else {
                vf_term = vf1;
                dv = 0.5f * g1 + 0.5f * g2;
            }
        } else {
            const float e1 = rt - v;
            vf_term = (double)(e1 * e1);
            dv = -2.0f * e1;
        }
        grad_value[r] = (float)((double)p.vf_coef * (double)dv * p.inv_b);
    }
    // d/d(mu) into the LDS tile (own row only), d/d(log_std) partials per dim
    for (int64_t a = 0; a < A; ++a) {
        double dls = 0.0;
        if (live) {
            const float diff = my_act[a] - my_mu[a];
            const float var = s_var[a];
            my_mu[a] = g_logp * diff / var;
            dls = (double)g_logp * ((double)(diff * diff) / (double)var - 1.0);
        }
        dls = wave_sum(dls);
        if (lane == 0) red[w][4 + a] = dls;
    }
    const double cs = wave_sum(clip_term);
    const double vs = wave_sum(vf_term);
    const double cnt = wave_sum(live ? 1.0 : 0.0);
    if (lane == 0) {
        red[w][0] = cs;
        red[w][1] = vs;
        red[w][2] = cnt;
        red[w][3] = 0.0;
    }
    __syncthreads();
    float* gm_blk = grad_mu + r0 * A;
    for (int f = threadIdx.x; f < nel; f += TPB) gm_blk[f] = s_mu[f];
    for (int c = threadIdx.x; c < 4 + A; c += TPB) {
        double tsum = 0.0;
        for (int i = 0; i < NW; ++i) tsum += red[i][c];
        partials[(int64_t)blockIdx.x * (4 + A) + c] = tsum;
    }
}

__global__ void gauss_finalize_kernel(const double* sums, int64_t A, const float* log_std,
                                      Params p, float* losses, float* grad_log_std) {
    if (threadIdx.x == 0) {
        float ent = 0.0f;
        for (int64_t a = 0; a < A; ++a) {
            const float sig = expf(log_std[a]);
            ent += 1.4189385332046727f + logf(sig);  // f32(0.5 + 0.5*log(2*pi)) + log(scale)
        }
        const float clip = (float)(sums[0] * p.inv_b);
        const float vf = (float)(sums[1] * p.inv_b);
        losses[0] = clip + p.vf_coef * vf - p.ent_coef * ent;
        losses[1] = clip;
        losses[2] = vf;
        losses[3] = ent;
    }
    for (int64_t a = threadIdx.x; a < A; a += blockDim.x)
        grad_log_std[a] = (float)(sums[4 + a] - (double)p.ent_coef);
}

__global__ __launch_bounds__(TPB) void gauss_logp_kernel(const float* mu, const float* log_std,
                                                         const float* act, int64_t b, int64_t A,
                                                         float* out) {
    __shared__ float s_var[MAX_ACT], s_ls[MAX_ACT];
    for (int a = threadIdx.x; a < A; a += TPB) {
        const float sig = expf(log_std[a]);
        s_var[a] = sig * sig;
        s_ls[a] = logf(sig);
    }
    __syncthreads();
    for (int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x; r < b;
         r += (int64_t)gridDim.x * TPB) {
        float lp = 0.0f;
        for (int64_t a = 0; a < A; ++a) {
            const float diff = act[r * A + a] - mu[r * A + a];
            lp += -(diff * diff) / (2.0f * s_var[a]) - s_ls[a] - LOG_SQRT_2PI;
        }
        out[r] = lp;
    }
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_ppo_num_partials(int64_t b) { return (b + TPB - 1) / TPB; }

extern "C" int tsrl_adv_moments(const float* adv, const int64_t* idx, int64_t b,
                                double* partials, void* stream) {
    TSRL_CHECK_ARG(b >= 0, "tsrl_adv_moments: b < 0");
    if (b == 0) return 0;
    TSRL_CHECK_ARG(adv && partials, "tsrl_adv_moments: null pointer");
    hipLaunchKernelGGL(adv_moments_kernel, dim3((unsigned)tsrl_ppo_num_partials(b)), dim3(TPB), 0,
                       as_stream(stream), adv, idx, b, partials);
    TSRL_LAUNCH_CHECK("tsrl_adv_moments");
    return 0;
}

extern "C" int64_t tsrl_adv_moments_seg_parts(int64_t max_seg) {
    const int64_t p = (max_seg + 4 * TPB - 1) / (4 * TPB);  // ~4 rows per thread
    return p < 1 ? 1 : (p > 256 ? 256 : p);
}

extern "C" int tsrl_adv_moments_seg(const float* adv, const int64_t* idx, const int64_t* bounds,
                                    int64_t nseg, int64_t max_seg, double* partials,
                                    double* out, void* stream) {
    TSRL_CHECK_ARG(nseg >= 0 && nseg <= 65535 && max_seg >= 0,
                   "tsrl_adv_moments_seg: nseg=%lld max_seg=%lld", (long long)nseg,
                   (long long)max_seg);
    if (nseg == 0) return 0;
    TSRL_CHECK_ARG(adv && bounds && partials && out, "tsrl_adv_moments_seg: null pointer");
    const int nparts = (int)tsrl_adv_moments_seg_parts(max_seg);
    hipLaunchKernelGGL(adv_moments_seg_kernel, dim3((unsigned)nparts, (unsigned)nseg), dim3(TPB),
                       0, as_stream(stream), adv, idx, bounds, nparts, partials);
    TSRL_LAUNCH_CHECK("adv_moments_seg_kernel");
    hipLaunchKernelGGL(adv_moments_seg_reduce_kernel, dim3((unsigned)nseg), dim3(kWave), 0,
                       as_stream(stream), partials, nparts, out);
    TSRL_LAUNCH_CHECK("adv_moments_seg_reduce_kernel");
    return 0;
}

extern "C" int tsrl_reduce_partials(const double* partials, int64_t nblk, int64_t width,
                                    double* out, void* stream) {
    TSRL_CHECK_ARG(partials && out && nblk >= 0 && width > 0, "tsrl_reduce_partials: bad args");
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(TPB), 0, as_stream(stream), partials,
                       nblk, width, out);
    TSRL_LAUNCH_CHECK("tsrl_reduce_partials");
    return 0;
}

extern "C" int tsrl_ppo_gauss_fwd_bwd(const float* mu, const float* log_std, const float* value,
                                      const float* act, const float* logp_old, const float* adv,
                                      const float* ret, const float* v_s, const int64_t* idx,
                                      int64_t b, int64_t act_dim, const double* adv_sums,
                                      tsrl_ppo_params p, float* grad_mu, float* grad_value,
                                      double* partials, void* stream) {
    TSRL_CHECK_ARG(b >= 0 && act_dim > 0 && act_dim <= MAX_ACT,
                   "tsrl_ppo_gauss_fwd_bwd: need 0 < act_dim <= %d", MAX_ACT);
    if (b == 0) return 0;
    TSRL_CHECK_ARG(mu && log_std && value && act && logp_old && adv && ret && grad_mu &&
                       grad_value && partials,
                   "tsrl_ppo_gauss_fwd_bwd: null pointer");
    TSRL_CHECK_ARG(!p.value_clip || v_s, "tsrl_ppo_gauss_fwd_bwd: value_clip needs v_s");
    TSRL_CHECK_ARG(!p.norm_adv || adv_sums, "tsrl_ppo_gauss_fwd_bwd: norm_adv needs adv_sums");
    TSRL_CHECK_ARG(p.b_global >= 1.0, "tsrl_ppo_gauss_fwd_bwd: b_global < 1");
    const size_t lds = 2 * (size_t)TPB * (size_t)act_dim * sizeof(float);
    hipLaunchKernelGGL(gauss_fwd_bwd_kernel, dim3((unsigned)tsrl_ppo_num_partials(b)), dim3(TPB),
                       lds, as_stream(stream), mu, log_std, value, act, logp_old, adv, ret, v_s,
                       idx, b, act_dim, adv_sums, make_params(p), grad_mu, grad_value, partials);
    TSRL_LAUNCH_CHECK("tsrl_ppo_gauss_fwd_bwd");
    return 0;
}

extern "C" int tsrl_ppo_gauss_finalize(const double* sums, int64_t act_dim, const float* log_std,
                                       tsrl_ppo_params p, float* losses, float* grad_log_std,
                                       void* stream) {
    TSRL_CHECK_ARG(sums && log_std && losses && grad_log_std && act_dim > 0 &&
                       act_dim <= MAX_ACT,
                   "tsrl_ppo_gauss_finalize: bad arguments");
    hipLaunchKernelGGL(gauss_finalize_kernel, dim3(1), dim3(64), 0, as_stream(stream), sums,
                       act_dim, log_std, make_params(p), losses, grad_log_std);
    TSRL_LAUNCH_CHECK("tsrl_ppo_gauss_finalize");
    return 0;
}

extern "C" int tsrl_gauss_logp(const float* mu, const float* log_std, const float* act,
                               int64_t b, int64_t act_dim, float* out, void* stream) {
    TSRL_CHECK_ARG(b >= 0 && act_dim > 0 && act_dim <= MAX_ACT, "tsrl_gauss_logp: bad sizes");
    if (b == 0) return 0;
    TSRL_CHECK_ARG(mu && log_std && act && out, "tsrl_gauss_logp: null pointer");
    const int64_t grid = std::min<int64_t>((b + TPB - 1) / TPB, 16384);
    hipLaunchKernelGGL(gauss_logp_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream),
                       mu, log_std, act, b, act_dim, out);
    TSRL_LAUNCH_CHECK("tsrl_gauss_logp");
    return 0;
}
