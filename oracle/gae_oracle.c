/*
 * ORACLE (test infrastructure only) -- plain-C restatement of the reference GAE reverse scan.
 *
 * Follows tianshou/policy/base.py:453-497 (_gae_return) together with the value handling of
 * BasePolicy.compute_episodic_return (tianshou/policy/base.py:371-383), under the NumPy-2.2
 * promotion rules the container oracle pins:
 *
 *   f32 values  : delta = (double)rew + (double)(float)(v_next_masked * (float)gamma) - (double)v_s
 *   f64 values  : delta = rew + v_next_masked * gamma - v_s            (rew_norm path, a2c.py:98-100)
 *   discount    = (1.0 - end) * (gamma * gae_lambda)                   (f64)
 *   gae_i       = delta_i + discount_i * gae_{i+1}   (sequential, no FMA: build with
 *                                                      -ffp-contract=off)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.
 * It is the checker, never the product path.
 */
#include <stdint.h>

void oracle_gae_f32vals(const float *v_s, const float *v_next_masked, const double *rew,
                        const uint8_t *end, int64_t n, double gamma, double gae_lambda,
                        double *adv_out)
{
    const float g32 = (float)gamma;
    const double gl = gamma * gae_lambda;
    double gae = 0.0;
    for (int64_t i = n - 1; i >= 0; --i) {
        float t = v_next_masked[i] * g32;
        double delta = (rew[i] + (double)t) - (double)v_s[i];
        double disc = (1.0 - (double)(end[i] != 0)) * gl;
        gae = delta + disc * gae;
        adv_out[i] = gae;
    }
}

void oracle_gae_f64vals(const double *v_s, const double *v_next_masked, const double *rew,
                        const uint8_t *end, int64_t n, double gamma, double gae_lambda,
                        double *adv_out)
{
    const double gl = gamma * gae_lambda;
    double gae = 0.0;
    for (int64_t i = n - 1; i >= 0; --i) {
        double delta = (rew[i] + v_next_masked[i] * gamma) - v_s[i];
        double disc = (1.0 - (double)(end[i] != 0)) * gl;
        gae = delta + disc * gae;
        adv_out[i] = gae;
    }
}

/*
 * Sequential Fisher-Yates application of shuffle draws (NumPy legacy RandomState.shuffle,
 * mtrand.pyx _shuffle_raw: for i = n-1 .. 1, swap x[i] and x[draws[i]]) onto arange(n).
 * Checker for tsrl_np_shuffle_draws / tsrl_shuffle_apply.
 */
void oracle_shuffle_apply(const uint32_t *draws, int64_t n, int64_t *out)
{
    for (int64_t i = 0; i < n; ++i) out[i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        int64_t j = (int64_t)draws[i];
        int64_t t = out[i];
        out[i] = out[j];
        out[j] = t;
    }
}
