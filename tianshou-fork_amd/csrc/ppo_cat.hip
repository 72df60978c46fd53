// Fused PPO clipped-surrogate + value + entropy loss with its analytic gradient for
// Categorical policies (discrete actions; PPOPolicy.learn minibatch body,
// tianshou/policy/modelfree/ppo.py:106-151):
//   mode 0  Categorical(logits=x)  (examples/atari/atari_ppo.py:136-137, Actor with
//           softmax_output=False),
//   mode 1  Categorical(probs=x)   (test/discrete/test_ppo.py:95, Actor softmax output,
//           utils/net/discrete.py:69-70).
// torch's f32 formulation is followed step by step (torch/distributions/categorical.py,
// utils.py: logits = x - logsumexp(x); probs = softmax(logits) | probs = x / sum(x);
// logits = log(clamp(probs, eps, 1 - eps)); log_prob = logits[a]; entropy =
// -sum(clamp(logits, min=f32 min) * probs)), and its backward is written out: on ties min/max
// split the gradient in half and clamp passes it on the closed interval, as torch does.
// One workgroup = 256 minibatch rows; the [256, nA] tile of x (contiguous, minibatch order)
// is staged in LDS, the gathered rows of act/logp_old/adv/returns/v_s come through idx.
#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int NW = TPB / kWave;
constexpr int MAX_ACT = 64;
constexpr float F32_EPS = 1.1920928955078125e-07f;
constexpr float F32_MIN = -3.4028234663852886e+38f;

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

// Row quantities of the distribution: normalised logits l[] and probabilities q[] (in place
// over the LDS row), the sum S (probs mode), returns entropy.  clamp masks in m (probs mode).
struct Row {
    float H;
    float S;
};

__device__ __forceinline__ Row cat_row(float* x, float* l, int A, int mode, uint64_t* mask) {
    Row o;
    o.S = 1.0f;
    *mask = 0;
    if (mode == 0) {
        float mx = -INFINITY;
        for (int j = 0; j < A; ++j) mx = fmaxf(mx, x[j]);
        float se = 0.0f;
        for (int j = 0; j < A; ++j) se += expf(x[j] - mx);
        const float lse = mx + logf(se);
        float m2 = -INFINITY;
        for (int j = 0; j < A; ++j) {
            l[j] = x[j] - lse;
            m2 = fmaxf(m2, l[j]);
        }
        float s2 = 0.0f;
        for (int j = 0; j < A; ++j) {
            const float e = expf(l[j] - m2);
            x[j] = e;  // x now holds probs
            s2 += e;
        }
        for (int j = 0; j < A; ++j) x[j] = x[j] / s2;
    } else {
        float S = 0.0f;
        for (int j = 0; j < A; ++j) S += x[j];
        o.S = S;
        for (int j = 0; j < A; ++j) {
            const float q = x[j] / S;
            x[j] = q;
            const float qc = fminf(fmaxf(q, F32_EPS), 1.0f - F32_EPS);
            if (q >= F32_EPS && q <= 1.0f - F32_EPS) *mask |= 1ull << j;
            l[j] = logf(qc);
        }
    }
    float h = 0.0f;
    for (int j = 0; j < A; ++j) h += fmaxf(l[j], F32_MIN) * x[j];
    o.H = -h;
    return o;
}

__global__ __launch_bounds__(TPB) void cat_fwd_bwd_kernel(
    const float* xin, const float* value, const int64_t* act, const float* logp_old,
    const float* adv, const float* ret, const float* v_s, const int64_t* idx, int64_t b,
    int A, int mode, const double* adv_sums, Params p, float* grad_x, float* grad_value,
    double* partials) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* s_x = smem;             // [TPB * A]  x -> probs -> grad
    float* s_l = smem + TPB * A;   // [TPB * A]  normalised logits
    __shared__ double red[NW][4];
    const int w = threadIdx.x / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r0 = (int64_t)blockIdx.x * TPB;
    const int nrows = (int)min((int64_t)TPB, b - r0);
    const int nel = nrows * A;
    const float* x_blk = xin + r0 * A;
    for (int f = threadIdx.x; f < nel; f += TPB) s_x[f] = x_blk[f];
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
    double clip_term = 0.0, vf_term = 0.0, ent_term = 0.0;
    if (live) {
        const int64_t r = r0 + t;
        const int64_t j = idx ? idx[r] : r;
        float* q = s_x + t * A;
        float* l = s_l + t * A;
        uint64_t mask;
        const Row row = cat_row(q, l, A, mode, &mask);
        const int64_t a64 = act[j];
        const int a = (a64 >= 0 && a64 < A) ? (int)a64 : -1;  // invalid action -> NaN loss
        const float logp = a >= 0 ? l[a] : NAN;
        float an = adv[j];
        if (p.norm_adv) an = (an - mean_f) / (std_f + p.adv_eps);
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
        ent_term = (double)row.H;
        const float c_lp = (float)(-(double)dobj * (double)ratio * p.inv_b);
        const float c_h = (float)(-(double)p.ent_coef * p.inv_b);
        // d(loss)/dx in place over the probs row
        if (mode == 0) {
            for (int k = 0; k < A; ++k) {
                const float qk = q[k];
                const float g = c_lp * ((k == a ? 1.0f : 0.0f) - qk) + c_h * (-qk * (l[k] + row.H));
                l[k] = g;
            }
            for (int k = 0; k < A; ++k) q[k] = l[k];
        } else {
            float dot = 0.0f;
            for (int k = 0; k < A; ++k) {
                const float qk = q[k];
                const float dl = (k == a ? c_lp : 0.0f) - c_h * qk;
                const float g = ((mask >> k) & 1ull ? dl / qk : 0.0f) - c_h * l[k];
                l[k] = g;
                dot += g * qk;
            }
            for (int k = 0; k < A; ++k) q[k] = (l[k] - dot) / row.S;
        }
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
    const double cs = wave_sum(clip_term);
    const double vs = wave_sum(vf_term);
    const double cnt = wave_sum(live ? 1.0 : 0.0);
    const double es = wave_sum(ent_term);
    if (lane == 0) {
        red[w][0] = cs;
        red[w][1] = vs;
        red[w][2] = cnt;
        red[w][3] = es;
    }
    __syncthreads();
    float* g_blk = grad_x + r0 * A;
    for (int f = threadIdx.x; f < nel; f += TPB) g_blk[f] = s_x[f];
    if (threadIdx.x < 4) {
        double tsum = 0.0;
        for (int i = 0; i < NW; ++i) tsum += red[i][threadIdx.x];
        partials[(int64_t)blockIdx.x * 4 + threadIdx.x] = tsum;
    }
}

__global__ void cat_finalize_kernel(const double* sums, Params p, float* losses) {
    if (threadIdx.x == 0) {
        const float clip = (float)(sums[0] * p.inv_b);
        const float vf = (float)(sums[1] * p.inv_b);
        const float ent = (float)(sums[3] * p.inv_b);
        losses[0] = clip + p.vf_coef * vf - p.ent_coef * ent;
        losses[1] = clip;
        losses[2] = vf;
        losses[3] = ent;
    }
}

__global__ __launch_bounds__(TPB) void cat_logp_kernel(const float* xin, const int64_t* act,
                                                       int64_t b, int A, int mode, float* out) {
    float l[MAX_ACT], q[MAX_ACT];
    for (int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x; r < b;
         r += (int64_t)gridDim.x * TPB) {
        for (int j = 0; j < A; ++j) q[j] = xin[r * A + j];
        uint64_t mask;
        cat_row(q, l, A, mode, &mask);
        const int64_t a = act[r];
        out[r] = (a >= 0 && a < A) ? l[(int)a] : NAN;
    }
}

// Categorical(logits).sample() as one pass (Collector step, pg.py:133-171 -> dist.sample()):
// the Gumbel-max form argmax_a(logits[a] - log(-log(u[a]))) with u ~ U[0, 1) drawn by the
// caller (torch.rand_like: torch's own, graph-capturable stream), which samples exactly the
// categorical distribution of the logits (first index on ties; -inf logits are never drawn).
// Replaces torch's softmax + multinomial (exponential draw, argmax and its validity
// reductions): ~14 small kernels per collector step for Atari-sized batches.
__global__ __launch_bounds__(TPB) void cat_gumbel_argmax_kernel(const float* __restrict__ logits,
                                                                const float* __restrict__ u,
                                                                int64_t n, int64_t A,
                                                                int64_t* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r >= n) return;
    const float* lr = logits + r * A;
    const float* ur = u + r * A;
    float best = -INFINITY;
    int64_t arg = 0;
    for (int64_t a = 0; a < A; ++a) {
        const float g = lr[a] - logf(-logf(ur[a]));
        if (g > best) {
            best = g;
            arg = a;
        }
    }
    out[r] = arg;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_ppo_cat_fwd_bwd(const float* x, const float* value, const int64_t* act,
                                    const float* logp_old, const float* adv, const float* ret,
                                    const float* v_s, const int64_t* idx, int64_t b,
                                    int64_t num_actions, int mode, const double* adv_sums,
                                    tsrl_ppo_params p, float* grad_x, float* grad_value,
                                    double* partials, void* stream) {
    TSRL_CHECK_ARG(b >= 0 && num_actions > 0 && num_actions <= MAX_ACT,
                   "tsrl_ppo_cat_fwd_bwd: need 0 < num_actions <= %d", MAX_ACT);
    TSRL_CHECK_ARG(mode == 0 || mode == 1, "tsrl_ppo_cat_fwd_bwd: mode must be 0 or 1");
    if (b == 0) return 0;
    TSRL_CHECK_ARG(x && value && act && logp_old && adv && ret && grad_x && grad_value &&
                       partials,
                   "tsrl_ppo_cat_fwd_bwd: null pointer");
    TSRL_CHECK_ARG(!p.value_clip || v_s, "tsrl_ppo_cat_fwd_bwd: value_clip needs v_s");
    TSRL_CHECK_ARG(!p.norm_adv || adv_sums, "tsrl_ppo_cat_fwd_bwd: norm_adv needs adv_sums");
    TSRL_CHECK_ARG(p.b_global >= 1.0, "tsrl_ppo_cat_fwd_bwd: b_global < 1");
    const size_t lds = 2 * (size_t)TPB * (size_t)num_actions * sizeof(float);
    hipLaunchKernelGGL(cat_fwd_bwd_kernel, dim3((unsigned)((b + TPB - 1) / TPB)), dim3(TPB), lds,
                       as_stream(stream), x, value, act, logp_old, adv, ret, v_s, idx, b,
                       (int)num_actions, mode, adv_sums, make_params(p), grad_x, grad_value,
                       partials);
    TSRL_LAUNCH_CHECK("tsrl_ppo_cat_fwd_bwd");
    return 0;
}

extern "C" int tsrl_ppo_cat_finalize(const double* sums, tsrl_ppo_params p, float* losses,
                                     void* stream) {
    TSRL_CHECK_ARG(sums && losses, "tsrl_ppo_cat_finalize: null pointer");
    hipLaunchKernelGGL(cat_finalize_kernel, dim3(1), dim3(64), 0, as_stream(stream), sums,
                       make_params(p), losses);
    TSRL_LAUNCH_CHECK("tsrl_ppo_cat_finalize");
    return 0;
}

extern "C" int tsrl_cat_logp(const float* x, const int64_t* act, int64_t b, int64_t num_actions,
                             int mode, float* out, void* stream) {
    TSRL_CHECK_ARG(b >= 0 && num_actions > 0 && num_actions <= MAX_ACT,
                   "tsrl_cat_logp: need 0 < num_actions <= %d", MAX_ACT);
    TSRL_CHECK_ARG(mode == 0 || mode == 1, "tsrl_cat_logp: mode must be 0 or 1");
    if (b == 0) return 0;
    TSRL_CHECK_ARG(x && act && out, "tsrl_cat_logp: null pointer");
    const int64_t grid = std::min<int64_t>((b + TPB - 1) / TPB, 16384);
    hipLaunchKernelGGL(cat_logp_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream), x,
                       act, b, (int)num_actions, mode, out);
    TSRL_LAUNCH_CHECK("tsrl_cat_logp");
    return 0;
}

extern "C" int tsrl_cat_gumbel_argmax(const float* logits, const float* u, int64_t n,
                                      int64_t num_actions, int64_t* out, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && num_actions > 0, "tsrl_cat_gumbel_argmax: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(logits && u && out, "tsrl_cat_gumbel_argmax: null pointer");
    hipLaunchKernelGGL(cat_gumbel_argmax_kernel, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB),
                       0, as_stream(stream), logits, u, n, num_actions, out);
    TSRL_LAUNCH_CHECK("tsrl_cat_gumbel_argmax");
    return 0;
}
