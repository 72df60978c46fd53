// One row of the VectorReplayBuffer add (ReplayBufferManager.add, tianshou/data/buffer/
// manager.py:104-161 + ReplayBuffer._add_index, base.py:195-214), used by buffer_add_kernel
// (csrc/buffer.hip).
// One wave per row: payload copies (obs, act, raw obs_next), the normalised obs_next / reset
// row into the buffer and the live obs, flags, env id and the episode bookkeeping.
#pragma once
#include "tsrl_common.h"

namespace tsrl {

__device__ __forceinline__ void copy_row(const void* src, void* dst, int64_t bytes, int lane,
                                         int nl = kWave) {
    const char* s = reinterpret_cast<const char*>(src);
    char* d = reinterpret_cast<char*>(dst);
    if ((bytes & 15) == 0 && aligned16(s) && aligned16(d)) {
        const int4* s4 = reinterpret_cast<const int4*>(s);
        int4* d4 = reinterpret_cast<int4*>(d);
        for (int64_t i = lane; i < bytes / 16; i += nl) d4[i] = s4[i];
    } else if ((bytes & 3) == 0 && (((uintptr_t)s | (uintptr_t)d) & 3) == 0) {
        const int* s4 = reinterpret_cast<const int*>(s);
        int* d4 = reinterpret_cast<int*>(d);
        for (int64_t i = lane; i < bytes / 4; i += nl) d4[i] = s4[i];
    } else {
        for (int64_t i = lane; i < bytes; i += nl) d[i] = s[i];
    }
}

__device__ __forceinline__ float norm1(float x, float m, float v, float eps, float clip) {
    float y = (x - m) / __builtin_sqrtf(v + eps);
    if (clip > 0.0f) y = fminf(fmaxf(y, -clip), clip);
    return y;
}
// norm1 with s = sqrt(v + eps) computed once per column by the caller (same bits)
__device__ __forceinline__ float norm1s(float x, float m, float s, float clip) {
    float y = (x - m) / s;
    if (clip > 0.0f) y = fminf(fmaxf(y, -clip), clip);
    return y;
}

// The payload copies of add_row (obs, act, raw obs_next rows) by nl lanes.
__device__ __forceinline__ void add_row_copies(const tsrl_add_args& a, int64_t r, int lane,
                                               int64_t ptr, int nl) {
    const int64_t obs_pitch = a.obs_src_pitch ? a.obs_src_pitch : a.obs_row_bytes;
    const int64_t next_pitch = a.obs_next_src_pitch ? a.obs_next_src_pitch : a.obs_row_bytes;
    const int64_t dst_pitch = a.obs_dst_pitch ? a.obs_dst_pitch : a.obs_row_bytes;
    if (a.obs_src && a.obs_dst)
        copy_row((const char*)a.obs_src + r * obs_pitch,
                 (char*)a.obs_dst + ptr * dst_pitch, a.obs_row_bytes, lane, nl);
    if (a.act_src && a.act_dst)
        copy_row((const char*)a.act_src + r * a.act_row_bytes,
                 (char*)a.act_dst + ptr * a.act_row_bytes, a.act_row_bytes, lane, nl);
    if (a.obs_next_src_raw && a.obs_next_dst_raw)
        copy_row((const char*)a.obs_next_src_raw + r * next_pitch,
                 (char*)a.obs_next_dst_raw + ptr * dst_pitch, a.obs_row_bytes, lane, nl);
}

// The lane-0 part of add_row: flags, env id and the episode bookkeeping of row r, split
// into its loads (RowTail::load) and the stores that use them (RowTail::apply), so a caller
// can issue the loads early and apply them later.
struct RowTail {
    double rew, ep_rew;
    int64_t ep_len, ep_idx, off, next_rel;
    uint8_t tm, tr;

    __device__ __forceinline__ void load(const tsrl_add_args& a, int64_t r, int64_t b) {
        rew = a.rew ? a.rew[r] : 0.0;
        tm = a.term ? a.term[r] : 0;
        tr = a.trunc ? a.trunc[r] : 0;
        ep_rew = a.ep_rew[b];
        ep_len = a.ep_len[b];
        ep_idx = a.ep_idx[b];
        off = a.offset[b];
        next_rel = a.next_rel ? a.next_rel[r] : 0;
    }
    __device__ __forceinline__ void apply(const tsrl_add_args& a, int64_t r, int64_t urel,
                                          int64_t b, int64_t ptr) const {
        const uint8_t done = (uint8_t)((tm != 0) | (tr != 0));
        if (a.rew_dst) a.rew_dst[ptr] = rew;
        if (a.term_dst) a.term_dst[ptr] = (uint8_t)(tm != 0);
        if (a.trunc_dst) a.trunc_dst[ptr] = (uint8_t)(tr != 0);
        if (a.done_dst) a.done_dst[ptr] = done;
        if (a.env_id_dst) a.env_id_dst[ptr] = b;
        // ReplayBuffer._add_index episode bookkeeping (base.py:205-214)
        const double er = ep_rew + rew;
        const int64_t el = ep_len + 1;
        const int64_t ei = ep_idx + off;
        if (a.out_ep_rew) a.out_ep_rew[r] = done ? er : er * 0.0;
        if (a.out_ep_len) a.out_ep_len[r] = done ? el : 0;
        if (a.out_ep_idx) a.out_ep_idx[r] = ei;
        if (done) {
            if (a.stat_rew) a.stat_rew[ptr] = er;
            if (a.stat_len) a.stat_len[ptr] = el;
            if (a.stat_idx) a.stat_idx[ptr] = ei;
            a.ep_rew[b] = 0.0;
            a.ep_len[b] = 0;
            a.ep_idx[b] = a.next_rel ? next_rel
                                     : (a.rel_dev ? (urel + 1) % a.ring_size : a.uniform_next);
        } else {
            a.ep_rew[b] = er;
            a.ep_len[b] = el;
        }
    }
};

__device__ __forceinline__ void add_row_tail(const tsrl_add_args& a, int64_t r, int lane,
                                             int64_t urel, int64_t b, int64_t ptr) {
    if (lane == 0) {
        RowTail rt;
        rt.load(a, r, b);
        rt.apply(a, r, urel, b, ptr);
    }
}

// Row r of one add (urel = the uniform ring position of this step) by nl lanes (lane < nl).
// lx (nullable): the new live obs row is also written to lx[col * lxp] (the fused collect step
// keeps it in LDS for the next policy step); cur_hbm = false then skips its HBM copy.
// STD: norm_var / reset_var hold sqrt(var + eps) per column already (norm1s; same bits).
template <bool STD = false>
__device__ __forceinline__ void add_row(const tsrl_add_args& a, int64_t r, int lane,
                                        int64_t urel, float* lx = nullptr, int lxp = 0,
                                        int nl = kWave, bool cur_hbm = true) {
    auto nrm1 = [&](float x, float m, float v) {
        return STD ? norm1s(x, m, v, a.norm_clip) : norm1(x, m, v, a.norm_eps, a.norm_clip);
    };
    const int64_t b = a.ids ? a.ids[r] : r;
    const int64_t ptr = a.ptr ? a.ptr[r] : a.offset[b] + urel;

    add_row_copies(a, r, lane, ptr, nl);
    if (a.obs_next_src && (a.obs_next_dst || a.cur_obs)) {
        const float* src = a.obs_next_src + r * a.obs_dim;
        const int64_t dpitch = a.obs_dst_pitch ? a.obs_dst_pitch / 4 : a.obs_dim;
        float* dst = a.obs_next_dst ? a.obs_next_dst + ptr * dpitch : nullptr;
        float* cur = a.cur_obs ? a.cur_obs + r * a.obs_dim : nullptr;
        const bool nrm = a.norm_mean != nullptr;
        const bool rst = a.reset_mask && a.reset_mask[r];
        // 16-byte path: a lane handles 4 consecutive columns (376 columns = 94 float4,
        // two passes of the wave instead of six); same per-element arithmetic
        const bool v4 = (a.obs_dim & 3) == 0 && aligned16(src) && (!dst || aligned16(dst)) &&
                        (!cur || aligned16(cur)) && (!nrm || (aligned16(a.norm_mean) &&
                                                             aligned16(a.norm_var))) &&
                        (!rst || (aligned16(a.reset_src + r * a.obs_dim) &&
                                  (!a.reset_mean || (aligned16(a.reset_mean) &&
                                                     aligned16(a.reset_var)))));
        if (v4) {
            // QB float4 per lane per pass, every load of a pass issued before its stores (the
            // stores may alias the loads, so without this each iteration waited out one full
            // load latency)
            const int64_t nq = a.obs_dim >> 2;
            constexpr int QB = 4;
            const float4* s4 = reinterpret_cast<const float4*>(src);
            const float4* r4 = rst ? reinterpret_cast<const float4*>(a.reset_src + r * a.obs_dim)
                                   : nullptr;
            const bool rnrm = rst && a.reset_mean;
            for (int64_t q0 = lane; q0 < nq; q0 += QB * nl) {
                float4 xs[QB], ms[QB], vs[QB], xr[QB], mr[QB], vr[QB];
#pragma unroll
                for (int j = 0; j < QB; ++j) {
                    const int64_t q = q0 + j * nl;
                    const int64_t qc = q < nq ? q : 0;  // in-bounds, branch-free
                    xs[j] = s4[qc];
                    if (nrm) {
                        ms[j] = reinterpret_cast<const float4*>(a.norm_mean)[qc];
                        vs[j] = reinterpret_cast<const float4*>(a.norm_var)[qc];
                    }
                    if (cur && rst) {
                        xr[j] = r4[qc];
                        if (rnrm) {
                            mr[j] = reinterpret_cast<const float4*>(a.reset_mean)[qc];
                            vr[j] = reinterpret_cast<const float4*>(a.reset_var)[qc];
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < QB; ++j) {
                    const int64_t q = q0 + j * nl;
                    if (q >= nq) break;
                    float4 x = xs[j];
                    if (nrm) {
                        x.x = nrm1(x.x, ms[j].x, vs[j].x);
                        x.y = nrm1(x.y, ms[j].y, vs[j].y);
                        x.z = nrm1(x.z, ms[j].z, vs[j].z);
                        x.w = nrm1(x.w, ms[j].w, vs[j].w);
                    }
                    if (dst) reinterpret_cast<float4*>(dst)[q] = x;
                    if (cur) {
                        if (rst) {
                            x = xr[j];
                            if (rnrm) {
                                x.x = nrm1(x.x, mr[j].x, vr[j].x);
                                x.y = nrm1(x.y, mr[j].y, vr[j].y);
                                x.z = nrm1(x.z, mr[j].z, vr[j].z);
                                x.w = nrm1(x.w, mr[j].w, vr[j].w);
                            }
                        }
                        if (cur_hbm) reinterpret_cast<float4*>(cur)[q] = x;
                        if (lx) {
                            lx[(4 * q) * lxp] = x.x;
                            lx[(4 * q + 1) * lxp] = x.y;
                            lx[(4 * q + 2) * lxp] = x.z;
                            lx[(4 * q + 3) * lxp] = x.w;
                        }
                    }
                }
            }
        } else
        for (int64_t d = lane; d < a.obs_dim; d += nl) {
            float x = src[d];
            if (nrm) x = nrm1(x, a.norm_mean[d], a.norm_var[d]);
            if (dst) dst[d] = x;
            if (cur) {
                if (rst) {
                    x = a.reset_src[r * a.obs_dim + d];
                    if (a.reset_mean)
                        x = nrm1(x, a.reset_mean[d], a.reset_var[d]);
                }
                if (cur_hbm) cur[d] = x;
                if (lx) lx[d * lxp] = x;
            }
        }
    }
    add_row_tail(a, r, lane, urel, b, ptr);
}

}  // namespace tsrl
