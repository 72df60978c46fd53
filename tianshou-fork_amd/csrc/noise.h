// Exploration noise of the fused Gaussian policy step (dist.sample() of pg.py:133-171): a
// counter-based standard normal pair per (seed, step, row, action pair).  Shared by
// policy.hip (tsrl_gauss_policy_act_rng) and collect.hip (the fused collect step).
#pragma once
#include "tsrl_common.h"

namespace tsrl {

// Two standard normals for (seed, step, row, pair): one splitmix64 counter hash gives two
// 24-bit uniforms -> Box-Muller (cos and sin branches).  Replaces torch.randn_like(mu) of the
// torch path (a separate launch).
__device__ __forceinline__ float2 counter_normal2(uint64_t seed, int64_t step, int64_t row,
                                                 int pair) {
    const uint64_t h = sm64(sm64(seed ^ (uint64_t)step) ^ (((uint64_t)row << 5) | (uint64_t)pair));
    const float u1 = ((float)(h >> 40) + 1.0f) * 0x1p-24f;                // (0, 1]
    const float u2 = (float)((h >> 16) & 0xFFFFFFu) * 0x1p-24f;          // [0, 1)
    const float r = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincospif(2.0f * u2, &sn, &cs);
    return make_float2(r * cs, r * sn);
}

}  // namespace tsrl
