// Counter-hash synthetic env of SURVEY.md §8d (oracle/synth_env.py restates it on the CPU):
// the per-(env, episode, time) key, the reward and the Box observation values.  Shared by the
// env kernels (env.hip) and the fused collect step (collect.hip), so both produce the same bits.
#pragma once
#include "tsrl_common.h"

namespace tsrl {
namespace synth {

constexpr uint64_t GOLD = 0x9E3779B97F4A7C15ull;
constexpr uint64_t REW_SALT = 0xD1B54A32D192ED03ull;

__device__ __forceinline__ uint64_t env_key(uint64_t s_seed, uint64_t e, int64_t j, int64_t t) {
    return sm64(sm64(sm64(s_seed ^ e) ^ (uint64_t)j) ^ (uint64_t)t);
}

__device__ __forceinline__ float box_val(uint64_t k, int64_t d) {
    const uint64_t h = sm64(k + (uint64_t)d * GOLD);
    return (float)(h >> 40) * 0x1p-23f - 1.0f;
}

// The action-coupled variant (SyntheticVectorEnv(act_coef=c), SURVEY.md §8d's env made to
// read its action like a MuJoCo env does): a step's observation value is
// f32(box_val + f32(c * a[d mod A])) with a the env's (remapped) action row; reset
// observations are box_val.  Its values are no longer multiples of 2^-23, so obs_rms moments
// of this env are general f64 sums.
__device__ __forceinline__ float coupled_val(uint64_t k, int64_t d, float a, float c) {
#pragma clang fp contract(off)
    const float ca = c * a;
    return box_val(k, d) + ca;
}

struct RowState {
    uint64_t key;
    int active;
};

}  // namespace synth
}  // namespace tsrl
