// Device synthetic vector env.  oracle/synth_env.py is the CPU restatement.
//
// Stands behind the BaseVectorEnv.step/reset surface (tianshou/env/venvs.py:260-381): one
// kernel steps every env of the shard and, while the raw observation rows are still in
// registers, accumulates the per-column (sum, sumsq) partials VectorEnvNormObs needs for its
// RunningMeanStd update (venv_wrappers.py:93-99), so the obs rows are read once.
#include "synth.h"

namespace tsrl {
namespace {

using synth::GOLD;
using synth::REW_SALT;
using synth::env_key;
using synth::box_val;
using synth::RowState;

constexpr int TPB = 256;
constexpr int ROWS = 16;  // env rows per workgroup

// Rows [r0, r0+ROWS): obs rows + column partials over active rows.  act (nullable): the
// rows' [k, act_dim] actions of the action-coupled env (synth.h coupled_val).
__device__ void box_rows(const RowState* rs, int64_t r0, int64_t k, int64_t dim, float* obs,
                         double* partials, const float* act = nullptr, int64_t act_dim = 1,
                         float act_coef = 0.0f) {
    const int nrows = (int)min((int64_t)ROWS, k - r0);
    for (int64_t d = threadIdx.x; d < dim; d += blockDim.x) {
        double s = 0.0, ss = 0.0;
        const int64_t ad = d % act_dim;
        for (int r = 0; r < nrows; ++r) {
            if (!rs[r].active) continue;
            const float x = act ? synth::coupled_val(rs[r].key, d, act[(r0 + r) * act_dim + ad],
                                                     act_coef)
                                : box_val(rs[r].key, d);
            obs[(r0 + r) * dim + d] = x;
            s += (double)x;
            ss += (double)x * (double)x;
        }
        if (partials) {
            double* pp = partials + ((int64_t)blockIdx.x * dim + d) * 2;
            pp[0] = s;
            pp[1] = ss;
        }
    }
}

__global__ __launch_bounds__(TPB) void box_step_kernel(const int64_t* ids, int64_t k,
                                                       int64_t dim, uint64_t s_seed,
                                                       int64_t ep_len, int64_t* ep_j,
                                                       int64_t* ep_t, float* obs, double* rew,
                                                       uint8_t* term, uint8_t* trunc,
                                                       double* partials, const float* act,
                                                       int64_t act_dim, float act_coef) {
    __shared__ RowState rs[ROWS];
    const int64_t r0 = (int64_t)blockIdx.x * ROWS;
    if (threadIdx.x < ROWS) {
        const int64_t r = r0 + threadIdx.x;
        RowState st = {0ull, 0};
        if (r < k) {
            const int64_t e = ids ? ids[r] : r;
            const int64_t j = ep_j[e];
            const int64_t t = ep_t[e] + 1;
            ep_t[e] = t;
            st.key = env_key(s_seed, (uint64_t)e, j, t);
            st.active = 1;
            const uint64_t h = sm64(st.key ^ REW_SALT);
            rew[r] = (double)(h >> 40) * 0x1p-24;
            const bool done = t >= ep_len;
            term[r] = (uint8_t)(done && (e % 2 == 0));
            trunc[r] = (uint8_t)(done && (e % 2 == 1));
        }
        rs[threadIdx.x] = st;
    }
    __syncthreads();
    box_rows(rs, r0, k, dim, obs, partials, act, act_dim, act_coef);
}

__global__ __launch_bounds__(TPB) void box_reset_kernel(const int64_t* ids, const uint8_t* mask,
                                                        int64_t k, int64_t dim, uint64_t s_seed,
                                                        int64_t ep_len, int64_t* ep_j,
                                                        int64_t* ep_t, float* obs,
                                                        double* partials) {
    __shared__ RowState rs[ROWS];
    const int64_t r0 = (int64_t)blockIdx.x * ROWS;
    if (threadIdx.x < ROWS) {
        const int64_t r = r0 + threadIdx.x;
        RowState st = {0ull, 0};
        if (r < k && (!mask || mask[r])) {
            const int64_t e = ids ? ids[r] : r;
            const int64_t j = ep_j[e] + 1;
            const int64_t t = (j == 0) ? (e % ep_len) : 0;
            ep_j[e] = j;
            ep_t[e] = t;
            st.key = env_key(s_seed, (uint64_t)e, j, t);
            st.active = 1;
        }
        rs[threadIdx.x] = st;
    }
    __syncthreads();
    box_rows(rs, r0, k, dim, obs, partials);
}

// Step + auto-reset in one launch (the Collector's step followed by reset of the finished
// envs, collector.py:310-361): raw step rows -> obs_out with partials P1 over every row;
// rows whose episode ended are reset at once -> reset_out with partials P2 over those rows
// only, and blk_done[block] counts them (the reset batch size of the second obs_rms update).
__global__ __launch_bounds__(1024) void box_step_reset_kernel(
    int64_t k, int64_t dim, uint64_t s_seed, int64_t ep_len, int64_t* ep_j, int64_t* ep_t,
    float* obs, float* reset_obs, double* rew, uint8_t* term, uint8_t* trunc, uint8_t* done,
    double* p_step, double* p_reset, double* blk_done, const float* act, int64_t act_dim,
    float act_coef) {
    __shared__ RowState rs[ROWS], rr[ROWS];
    __shared__ int nd;
    const int64_t r0 = (int64_t)blockIdx.x * ROWS;
    if (threadIdx.x == 0) nd = 0;
    __syncthreads();
    if (threadIdx.x < ROWS) {
        const int64_t r = r0 + threadIdx.x;
        RowState st = {0ull, 0}, sr = {0ull, 0};
        if (r < k) {
            const int64_t e = r;
            int64_t j = ep_j[e];
            int64_t t = ep_t[e] + 1;
            st.key = env_key(s_seed, (uint64_t)e, j, t);
            st.active = 1;
            const uint64_t h = sm64(st.key ^ REW_SALT);
            rew[r] = (double)(h >> 40) * 0x1p-24;
            const bool dn = t >= ep_len;
            term[r] = (uint8_t)(dn && (e % 2 == 0));
            trunc[r] = (uint8_t)(dn && (e % 2 == 1));
            done[r] = (uint8_t)dn;
            if (dn) {
                j += 1;
                t = (j == 0) ? (e % ep_len) : 0;
                ep_j[e] = j;
                sr.key = env_key(s_seed, (uint64_t)e, j, t);
                sr.active = 1;
                atomicAdd(&nd, 1);
            }
            ep_t[e] = t;
        }
        rs[threadIdx.x] = st;
        rr[threadIdx.x] = sr;
    }
    __syncthreads();
    box_rows(rs, r0, k, dim, obs, p_step, act, act_dim, act_coef);
    if (nd > 0) {
        box_rows(rr, r0, k, dim, reset_obs, p_reset);
    } else if (p_reset) {
        // no reset row in this block: the merge skips blocks with blk_done == 0
    }
    if (threadIdx.x == 0 && blk_done) blk_done[blockIdx.x] = (double)nd;
}

// u8 (Atari-shaped) observations: 4 bytes per thread-iteration, packed 32-bit stores.
// frame_stack S > 1 emulates gymnasium's FrameStack wrapper over a one-frame env: the
// observation is the last S frames, frame q of the obs at episode time t is the frame of
// time max(t - (S-1-q), t0) (t0 = the episode's first time step, whose frame a reset repeats
// S times).  fk[r][q] holds the key of that frame; S == 1 is the plain u8 observation.
constexpr int MAX_STACK = 8;
// u8 frame rows per workgroup: one row (28 KB of hashed bytes for 4x84x84) keeps 1024 env
// rows on 1024 workgroups; 16 rows per workgroup left 64 workgroups for 256 CUs
// (rocprofv3: 131 us per 1024-row step).
constexpr int U8_ROWS = 1;

__device__ void u8_rows(const RowState* rs, const uint64_t (*fk)[MAX_STACK], int64_t r0,
                        int64_t k, int64_t nbytes, int S, uint8_t* obs) {
    const int nrows = (int)min((int64_t)U8_ROWS, k - r0);
    const int64_t fbytes = nbytes / S;
    for (int r = 0; r < nrows; ++r) {
        if (!rs[r].active) continue;
        uint8_t* row = obs + (r0 + r) * nbytes;
        if ((fbytes & 3) == 0 && (((uintptr_t)row) & 3) == 0) {
            // frame by frame: no 64-bit division per word
            const int fw = (int)(fbytes / 4);
            for (int f = 0; f < S; ++f) {
                uint32_t* w = reinterpret_cast<uint32_t*>(row + f * fbytes);
                const uint64_t key = fk[r][f];
                for (int q = threadIdx.x; q < fw; q += TPB) {
                    const uint64_t i0 = 4ull * (uint64_t)q;
                    uint32_t v = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        v |= (uint32_t)(sm64(key + (i0 + b) * GOLD) & 0xFF) << (8 * b);
                    w[q] = v;
                }
            }
        } else {
            for (int64_t i = threadIdx.x; i < nbytes; i += TPB) {
                const int f = (int)(i / fbytes);
                row[i] = (uint8_t)(sm64(fk[r][f] + (uint64_t)(i - f * fbytes) * GOLD) & 0xFF);
            }
        }
    }
}

__device__ __forceinline__ void frame_keys(uint64_t s_seed, int64_t e, int64_t j, int64_t t,
                                           int64_t t0, int S, uint64_t* fk) {
    for (int q = 0; q < S; ++q) {
        const int64_t tq = max(t - (int64_t)(S - 1 - q), t0);
        fk[q] = env_key(s_seed, (uint64_t)e, j, tq);
    }
}

__device__ __forceinline__ int64_t episode_t0(int64_t e, int64_t j, int64_t ep_len) {
    return j == 0 ? e % ep_len : 0;
}

__global__ __launch_bounds__(TPB) void u8_step_kernel(const int64_t* ids, int64_t k,
                                                      int64_t nbytes, int S, uint64_t s_seed,
                                                      int64_t ep_len, int64_t* ep_j,
                                                      int64_t* ep_t, uint8_t* obs, double* rew,
                                                      uint8_t* term, uint8_t* trunc) {
    __shared__ RowState rs[U8_ROWS];
    __shared__ uint64_t fk[U8_ROWS][MAX_STACK];
    const int64_t r0 = (int64_t)blockIdx.x * U8_ROWS;
    if (threadIdx.x < U8_ROWS) {
        const int64_t r = r0 + threadIdx.x;
        RowState st = {0ull, 0};
        if (r < k) {
            const int64_t e = ids ? ids[r] : r;
            const int64_t j = ep_j[e];
            const int64_t t = ep_t[e] + 1;
            ep_t[e] = t;
            st.key = env_key(s_seed, (uint64_t)e, j, t);
            st.active = 1;
            frame_keys(s_seed, e, j, t, episode_t0(e, j, ep_len), S, fk[threadIdx.x]);
            const uint64_t h = sm64(st.key ^ REW_SALT);
            rew[r] = (double)(h >> 40) * 0x1p-24;
            const bool done = t >= ep_len;
            term[r] = (uint8_t)(done && (e % 2 == 0));
            trunc[r] = (uint8_t)(done && (e % 2 == 1));
        }
        rs[threadIdx.x] = st;
    }
    __syncthreads();
    u8_rows(rs, fk, r0, k, nbytes, S, obs);
}

__global__ __launch_bounds__(TPB) void u8_reset_kernel(const int64_t* ids, const uint8_t* mask,
                                                       int64_t k, int64_t nbytes, int S,
                                                       uint64_t s_seed, int64_t ep_len,
                                                       int64_t* ep_j, int64_t* ep_t,
                                                       uint8_t* obs) {
    __shared__ RowState rs[U8_ROWS];
    __shared__ uint64_t fk[U8_ROWS][MAX_STACK];
    const int64_t r0 = (int64_t)blockIdx.x * U8_ROWS;
    if (threadIdx.x < U8_ROWS) {
        const int64_t r = r0 + threadIdx.x;
        RowState st = {0ull, 0};
        if (r < k && (!mask || mask[r])) {
            const int64_t e = ids ? ids[r] : r;
            const int64_t j = ep_j[e] + 1;
            const int64_t t = episode_t0(e, j, ep_len);
            ep_j[e] = j;
            ep_t[e] = t;
            st.key = env_key(s_seed, (uint64_t)e, j, t);
            st.active = 1;
            frame_keys(s_seed, e, j, t, t, S, fk[threadIdx.x]);
        }
        rs[threadIdx.x] = st;
    }
    __syncthreads();
    u8_rows(rs, fk, r0, k, nbytes, S, obs);
}

inline unsigned blocks_for(int64_t k) { return (unsigned)((k + ROWS - 1) / ROWS); }
inline unsigned u8_blocks_for(int64_t k) { return (unsigned)((k + U8_ROWS - 1) / U8_ROWS); }

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_env_num_partials(int64_t k) { return (k + ROWS - 1) / ROWS; }

extern "C" int tsrl_synth_box_step_act(const int64_t* ids, int64_t k, int64_t dim,
                                       uint64_t seed, int64_t ep_len, int64_t* ep_j,
                                       int64_t* ep_t, float* obs_out, double* rew_out,
                                       uint8_t* term_out, uint8_t* trunc_out,
                                       double* col_partials, const float* act, int64_t act_dim,
                                       float act_coef, void* stream) {
    TSRL_CHECK_ARG(k >= 0 && dim > 0 && ep_len > 0 && (!act || act_dim > 0),
                   "tsrl_synth_box_step: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(ep_j && ep_t && obs_out && rew_out && term_out && trunc_out,
                   "tsrl_synth_box_step: null pointer");
    hipLaunchKernelGGL(box_step_kernel, dim3(blocks_for(k)), dim3(TPB), 0, as_stream(stream),
                       ids, k, dim, sm64(seed), ep_len, ep_j, ep_t, obs_out, rew_out, term_out,
                       trunc_out, col_partials, act, act ? act_dim : 1, act_coef);
    TSRL_LAUNCH_CHECK("tsrl_synth_box_step");
    return 0;
}

extern "C" int tsrl_synth_box_step(const int64_t* ids, int64_t k, int64_t dim, uint64_t seed,
                                   int64_t ep_len, int64_t* ep_j, int64_t* ep_t, float* obs_out,
                                   double* rew_out, uint8_t* term_out, uint8_t* trunc_out,
                                   double* col_partials, void* stream) {
    return tsrl_synth_box_step_act(ids, k, dim, seed, ep_len, ep_j, ep_t, obs_out, rew_out,
                                   term_out, trunc_out, col_partials, nullptr, 1, 0.0f, stream);
}

extern "C" int tsrl_synth_box_step_reset_act(int64_t k, int64_t dim, uint64_t seed,
                                             int64_t ep_len, int64_t* ep_j, int64_t* ep_t,
                                             float* obs_out, float* reset_out, double* rew_out,
                                             uint8_t* term_out, uint8_t* trunc_out,
                                             uint8_t* done_out, double* partials_step,
                                             double* partials_reset, double* blk_done,
                                             const float* act, int64_t act_dim, float act_coef,
                                             void* stream) {
    TSRL_CHECK_ARG(k >= 0 && dim > 0 && ep_len > 0 && (!act || act_dim > 0),
                   "tsrl_synth_box_step_reset: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(ep_j && ep_t && obs_out && reset_out && rew_out && term_out && trunc_out &&
                       done_out,
                   "tsrl_synth_box_step_reset: null pointer");
    TSRL_CHECK_ARG((partials_step == nullptr) == (partials_reset == nullptr) &&
                       (partials_step == nullptr) == (blk_done == nullptr),
                   "tsrl_synth_box_step_reset: partials / blk_done must be all set or all NULL");
    // one thread per observation column (up to 1024), so each thread's 16 rows are its
    // whole share of the block's work
    const unsigned tpb = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(64, (dim + 63) / 64 * 64));
    hipLaunchKernelGGL(box_step_reset_kernel, dim3(blocks_for(k)), dim3(tpb), 0,
                       as_stream(stream), k, dim, sm64(seed), ep_len, ep_j, ep_t, obs_out,
                       reset_out, rew_out, term_out, trunc_out, done_out, partials_step,
                       partials_reset, blk_done, act, act ? act_dim : 1, act_coef);
    TSRL_LAUNCH_CHECK("tsrl_synth_box_step_reset");
    return 0;
}

extern "C" int tsrl_synth_box_step_reset(int64_t k, int64_t dim, uint64_t seed, int64_t ep_len,
                                         int64_t* ep_j, int64_t* ep_t, float* obs_out,
                                         float* reset_out, double* rew_out, uint8_t* term_out,
                                         uint8_t* trunc_out, uint8_t* done_out,
                                         double* partials_step, double* partials_reset,
                                         double* blk_done, void* stream) {
    return tsrl_synth_box_step_reset_act(k, dim, seed, ep_len, ep_j, ep_t, obs_out, reset_out,
                                         rew_out, term_out, trunc_out, done_out, partials_step,
                                         partials_reset, blk_done, nullptr, 1, 0.0f, stream);
}

extern "C" int tsrl_synth_box_reset(const int64_t* ids, const uint8_t* mask, int64_t k,
                                    int64_t dim, uint64_t seed, int64_t ep_len, int64_t* ep_j,
                                    int64_t* ep_t, float* obs_out, double* col_partials,
                                    void* stream) {
    TSRL_CHECK_ARG(k >= 0 && dim > 0 && ep_len > 0, "tsrl_synth_box_reset: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(ep_j && ep_t && obs_out, "tsrl_synth_box_reset: null pointer");
    hipLaunchKernelGGL(box_reset_kernel, dim3(blocks_for(k)), dim3(TPB), 0, as_stream(stream),
                       ids, mask, k, dim, sm64(seed), ep_len, ep_j, ep_t, obs_out, col_partials);
    TSRL_LAUNCH_CHECK("tsrl_synth_box_reset");
    return 0;
}

extern "C" int tsrl_synth_u8_step(const int64_t* ids, int64_t k, int64_t obs_bytes,
                                  int64_t frame_stack, uint64_t seed, int64_t ep_len,
                                  int64_t* ep_j, int64_t* ep_t, uint8_t* obs_out,
                                  double* rew_out, uint8_t* term_out, uint8_t* trunc_out,
                                  void* stream) {
    TSRL_CHECK_ARG(k >= 0 && obs_bytes > 0 && ep_len > 0, "tsrl_synth_u8_step: bad sizes");
    TSRL_CHECK_ARG(frame_stack >= 1 && frame_stack <= MAX_STACK &&
                       obs_bytes % frame_stack == 0,
                   "tsrl_synth_u8_step: frame_stack must be 1..%d and divide obs_bytes",
                   MAX_STACK);
    if (k == 0) return 0;
    TSRL_CHECK_ARG(ep_j && ep_t && obs_out && rew_out && term_out && trunc_out,
                   "tsrl_synth_u8_step: null pointer");
    hipLaunchKernelGGL(u8_step_kernel, dim3(u8_blocks_for(k)), dim3(TPB), 0, as_stream(stream),
                       ids, k, obs_bytes, (int)frame_stack, sm64(seed), ep_len, ep_j, ep_t, obs_out,
                       rew_out, term_out, trunc_out);
    TSRL_LAUNCH_CHECK("tsrl_synth_u8_step");
    return 0;
}

extern "C" int tsrl_synth_u8_reset(const int64_t* ids, const uint8_t* mask, int64_t k,
                                   int64_t obs_bytes, int64_t frame_stack, uint64_t seed,
                                   int64_t ep_len, int64_t* ep_j, int64_t* ep_t,
                                   uint8_t* obs_out, void* stream) {
    TSRL_CHECK_ARG(k >= 0 && obs_bytes > 0 && ep_len > 0, "tsrl_synth_u8_reset: bad sizes");
    TSRL_CHECK_ARG(frame_stack >= 1 && frame_stack <= MAX_STACK &&
                       obs_bytes % frame_stack == 0,
                   "tsrl_synth_u8_reset: frame_stack must be 1..%d and divide obs_bytes",
                   MAX_STACK);
    if (k == 0) return 0;
    TSRL_CHECK_ARG(ep_j && ep_t && obs_out, "tsrl_synth_u8_reset: null pointer");
    hipLaunchKernelGGL(u8_reset_kernel, dim3(u8_blocks_for(k)), dim3(TPB), 0, as_stream(stream),
                       ids, mask, k, obs_bytes, (int)frame_stack, sm64(seed), ep_len, ep_j, ep_t,
                       obs_out);
    TSRL_LAUNCH_CHECK("tsrl_synth_u8_reset");
    return 0;
}
