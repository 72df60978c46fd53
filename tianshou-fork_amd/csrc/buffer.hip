// Device-resident VectorReplayBuffer storage operations.
//
// add    : ReplayBufferManager.add (tianshou/data/buffer/manager.py:104-161) for one vector
//          step -- the per-env `_add_index` loop (base.py:195-214) becomes one wave per env
//          row; episode statistics live on device.  The host keeps only the index
//          arithmetic (which it can do without reading device data).  The Collector's
//          obs_next normalisation (VectorEnvNormObs) is fused into the obs_next row copy.
// gather : fancy-index row gather (Batch.__getitem__, batch.py:446-460).
#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int ROWS_PER_BLOCK = TPB / kWave;  // one wave per row

__device__ __forceinline__ void copy_row(const void* src, void* dst, int64_t bytes, int lane) {
    const char* s = reinterpret_cast<const char*>(src);
    char* d = reinterpret_cast<char*>(dst);
    if ((bytes & 15) == 0 && aligned16(s) && aligned16(d)) {
        const int4* s4 = reinterpret_cast<const int4*>(s);
        int4* d4 = reinterpret_cast<int4*>(d);
        for (int64_t i = lane; i < bytes / 16; i += kWave) d4[i] = s4[i];
    } else if ((bytes & 3) == 0 && (((uintptr_t)s | (uintptr_t)d) & 3) == 0) {
        const int* s4 = reinterpret_cast<const int*>(s);
        int* d4 = reinterpret_cast<int*>(d);
        for (int64_t i = lane; i < bytes / 4; i += kWave) d4[i] = s4[i];
    } else {
        for (int64_t i = lane; i < bytes; i += kWave) d[i] = s[i];
    }
}

__device__ __forceinline__ float norm1(float x, float m, float v, float eps, float clip) {
    float y = (x - m) / __builtin_sqrtf(v + eps);
    if (clip > 0.0f) y = fminf(fmaxf(y, -clip), clip);
    return y;
}

__global__ __launch_bounds__(TPB) void buffer_add_kernel(tsrl_add_args a) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r = (int64_t)blockIdx.x * ROWS_PER_BLOCK + threadIdx.x / kWave;
    if (r >= a.k) return;
    const int64_t b = a.ids ? a.ids[r] : r;
    const int64_t ptr = a.ptr ? a.ptr[r] : a.offset[b] + a.uniform_rel;

    if (a.obs_src && a.obs_dst)
        copy_row((const char*)a.obs_src + r * a.obs_row_bytes,
                 (char*)a.obs_dst + ptr * a.obs_row_bytes, a.obs_row_bytes, lane);
    if (a.act_src && a.act_dst)
        copy_row((const char*)a.act_src + r * a.act_row_bytes,
                 (char*)a.act_dst + ptr * a.act_row_bytes, a.act_row_bytes, lane);
    if (a.obs_next_src_raw && a.obs_next_dst_raw)
        copy_row((const char*)a.obs_next_src_raw + r * a.obs_row_bytes,
                 (char*)a.obs_next_dst_raw + ptr * a.obs_row_bytes, a.obs_row_bytes, lane);
    if (a.obs_next_src && (a.obs_next_dst || a.cur_obs)) {
        const float* src = a.obs_next_src + r * a.obs_dim;
        float* dst = a.obs_next_dst ? a.obs_next_dst + ptr * a.obs_dim : nullptr;
        float* cur = a.cur_obs ? a.cur_obs + r * a.obs_dim : nullptr;
        const bool nrm = a.norm_mean != nullptr;
        for (int64_t d = lane; d < a.obs_dim; d += kWave) {
            float x = src[d];
            if (nrm) x = norm1(x, a.norm_mean[d], a.norm_var[d], a.norm_eps, a.norm_clip);
            if (dst) dst[d] = x;
            if (cur) cur[d] = x;
        }
    }
    if (lane == 0) {
        const double rew = a.rew ? a.rew[r] : 0.0;
        const uint8_t tm = a.term ? a.term[r] : 0;
        const uint8_t tr = a.trunc ? a.trunc[r] : 0;
        const uint8_t done = (uint8_t)((tm != 0) | (tr != 0));
        if (a.rew_dst) a.rew_dst[ptr] = rew;
        if (a.term_dst) a.term_dst[ptr] = (uint8_t)(tm != 0);
        if (a.trunc_dst) a.trunc_dst[ptr] = (uint8_t)(tr != 0);
        if (a.done_dst) a.done_dst[ptr] = done;
        if (a.env_id_dst) a.env_id_dst[ptr] = b;
        // ReplayBuffer._add_index episode bookkeeping (base.py:205-214)
        const double er = a.ep_rew[b] + rew;
        const int64_t el = a.ep_len[b] + 1;
        const int64_t ei = a.ep_idx[b] + a.offset[b];
        if (a.out_ep_rew) a.out_ep_rew[r] = done ? er : er * 0.0;
        if (a.out_ep_len) a.out_ep_len[r] = done ? el : 0;
        if (a.out_ep_idx) a.out_ep_idx[r] = ei;
        if (done) {
            if (a.stat_rew) a.stat_rew[ptr] = er;
            if (a.stat_len) a.stat_len[ptr] = el;
            if (a.stat_idx) a.stat_idx[ptr] = ei;
            a.ep_rew[b] = 0.0;
            a.ep_len[b] = 0;
            a.ep_idx[b] = a.next_rel ? a.next_rel[r] : a.uniform_next;
        } else {
            a.ep_rew[b] = er;
            a.ep_len[b] = el;
        }
    }
}

__global__ __launch_bounds__(TPB) void gather_rows_kernel(const char* src, int64_t row_bytes,
                                                          const int64_t* idx, int64_t k,
                                                          char* dst) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * ROWS_PER_BLOCK;
    for (int64_t r = (int64_t)blockIdx.x * ROWS_PER_BLOCK + threadIdx.x / kWave; r < k;
         r += nw) {
        copy_row(src + idx[r] * row_bytes, dst + r * row_bytes, row_bytes, lane);
    }
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_buffer_add(const tsrl_add_args* a, void* stream) {
    TSRL_CHECK_ARG(a != nullptr, "tsrl_buffer_add: null args");
    TSRL_CHECK_ARG(a->k >= 0, "tsrl_buffer_add: k < 0");
    if (a->k == 0) return 0;
    TSRL_CHECK_ARG(a->offset && a->ep_rew && a->ep_len && a->ep_idx,
                   "tsrl_buffer_add: offset/episode-state pointers are required");
    TSRL_CHECK_ARG(!a->obs_next_src || a->obs_dim > 0, "tsrl_buffer_add: obs_dim must be > 0");
    TSRL_CHECK_ARG(!a->norm_mean || a->norm_var, "tsrl_buffer_add: norm_var missing");
    const int64_t grid = (a->k + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
    hipLaunchKernelGGL(buffer_add_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream),
                       *a);
    TSRL_LAUNCH_CHECK("tsrl_buffer_add");
    return 0;
}

extern "C" int tsrl_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx,
                                int64_t k, void* dst, void* stream) {
    TSRL_CHECK_ARG(k >= 0 && row_bytes > 0, "tsrl_gather_rows: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(src && idx && dst, "tsrl_gather_rows: null pointer");
    const int64_t grid = std::min<int64_t>((k + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK, 16384);
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream),
                       (const char*)src, row_bytes, idx, k, (char*)dst);
    TSRL_LAUNCH_CHECK("tsrl_gather_rows");
    return 0;
}
