// One vector step of Collector.collect (tianshou/data/collector.py:258-361) as ONE launch, for
// the fused device path: a SyntheticVectorEnv with Box observations under VectorEnvNormObs
// (env/venv_wrappers.py:77-99, utils/statistics.py:93-114) and the MuJoCo Gaussian actor of
// utils/models.py:34-97 sampled as in pg.py:133-171.
//
// Before: four launches per step (tsrl_gauss_policy_act_rng -> tsrl_synth_box_step_reset ->
// tsrl_rms_merge2 -> tsrl_buffer_add), each a few microseconds of latency chain on 4096 rows.
// The add of step i needs the obs_rms state merged from ALL of step i's rows, so it cannot
// run in step i's launch without a grid barrier; it runs at the START of step i+1's launch
// instead (the step sequence rotated by one, "pending add"), and the caller issues the last
// step's add as a plain tsrl_buffer_add.  Per workgroup of R = 16 env rows, in order:
//   A. the pending add of step i-1 for these rows (add_row of buffer.hip: obs, act, the
//      normalised obs_next, reset rows, flags, episode statistics), the new live obs rows
//      also landing in LDS;
//   B. the actor on those rows (f32 MFMA 16x16x4: layer 1's K split over the 8 waves, layer 2
//      and the mu head over k halves / quarters, partials folded in fixed order), the noise
//      and map_action exactly as policy.hip;
//   C. the env step + auto-reset of these rows (synth.h, as env.hip's box_step_reset_kernel)
//      with the column moments of the step rows and of the reset rows;
//   D. obs_rms: the moments are folded deterministically without a grid barrier -- the last
//      of each group of GS workgroups to finish (agent-scope ticket) sums its group's partials
//      in index order, the last group sums the group partials in index order and applies both
//      RunningMeanStd updates (rms.hip's merge2 arithmetic), re-arming every ticket.  With
//      `totals` set (data parallel) it writes the step/reset moments instead and the caller
//      all-reduces them and runs tsrl_rms_merge2(nblk = 1).
#include "add_row.h"
#include "noise.h"
#include "synth.h"

namespace tsrl {
namespace {

using synth::box_val;
using synth::env_key;
using synth::REW_SALT;
using synth::RowState;

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int R = 16;          // env rows per workgroup
constexpr int NW = 8;          // waves per workgroup
constexpr int NT = NW * 64;
constexpr int H = 64;          // actor hidden width
constexpr int AMAX = 32;
constexpr int GS = 16;         // workgroups per obs_rms group
constexpr int KMAX = 512;      // observation columns handled (padded to 128)
constexpr int XP = 17;         // LDS pitch of the live-obs tile sX[col][row]
constexpr int HP = 16;         // h1 / h2 tiles [feature][row]
constexpr int WP = 68;         // W2 / W3 rows (4i + k banks: conflict-free A fragments)
// diagnostic builds only (tools/collect_step_bench.py): return after phase 1 (add), 2 (actor)
// or 3 (env); 0 = the whole step
#ifndef COLLECT_STOP
#define COLLECT_STOP 0
#endif
// diagnostic builds only: per-workgroup s_memrealtime stamps (100 MHz) after each phase,
// stored behind the workspace (tools/collect_step_bench.py --trace)
#ifndef COLLECT_TRACE
#define COLLECT_TRACE 0
#endif
#if COLLECT_TRACE
#define TSTAMP(i) \
    if (t == 0) ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memrealtime();
#else
#define TSTAMP(i)
#endif

__host__ __device__ inline int64_t kpad(int64_t dim) { return (dim + 127) / 128 * 128; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// packed[((w * SQ + sq) * 4 + ft) * 64 + lane][e] = W[16 ft + (lane & 15)][w * KW + 4 (4 sq + e)
// + (lane >> 4)] (0 beyond dim): wave w's A fragments of layer 1, one float4 load per
// (sq, ft), 1 KB contiguous per wave.
__global__ void pack_w1_kernel(const float* __restrict__ W, int64_t dim, float* __restrict__ out) {
    const int64_t Kp = kpad(dim), KW = Kp / NW, SQ = KW / 16;
    const int64_t total = (int64_t)H * Kp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const int64_t q = i >> 8;  // (w * SQ + sq) * 4 + ft
        const int ft = (int)(q & 3);
        const int64_t wsq = q >> 2, w = wsq / SQ, sq = wsq - w * SQ;
        const int64_t k = w * KW + 4 * (4 * sq + e) + (lane >> 4);
        out[i] = k < dim ? W[(int64_t)(16 * ft + (lane & 15)) * dim + k] : 0.0f;
    }
}

// Write-through (sc1) 16-byte stores and L1-bypassing (sc1) 16-byte loads of the handed-off
// obs_rms partials (buffer instructions, aux 16 = sc1), byte offsets into one descriptor.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st2_sc1(__amdgpu_buffer_rsrc_t r, int off, double x, double y) {
    const uint64_t a = __double_as_longlong(x), b = __double_as_longlong(y);
    u32x4 v;
    v.x = (unsigned)a;
    v.y = (unsigned)(a >> 32);
    v.z = (unsigned)b;
    v.w = (unsigned)(b >> 32);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
__device__ __forceinline__ double2 ld2_sc1(__amdgpu_buffer_rsrc_t r, int off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    return make_double2(__longlong_as_double(((uint64_t)v.y << 32) | v.x),
                        __longlong_as_double(((uint64_t)v.w << 32) | v.z));
}

struct Ws {
    unsigned int* tickets;  // [ngroups + 1]
    double* part;           // [nblk][PSTRIDE]
    double* gpart;          // [ngroups][PSTRIDE]
    int64_t pstride;        // 4 * dim + 4 (s1, q1, s2, q2 per column; reset-row count, pad)
    int64_t nblk;
    int ngroups;
    uint64_t* trace;
};
// Partial slab of one workgroup / group (doubles): [0, 2D) step rows (s, q) per column,
// [2D, 4D) reset rows (s, q) per column (zeros without reset rows), [4D] reset-row count.

__global__ __launch_bounds__(NT, 1) void collect_box_step_kernel(tsrl_collect_args a, Ws ws) {
#pragma clang fp contract(off)
    __shared__ float sX[KMAX * XP];
    __shared__ float sW2[H * WP], sW3[AMAX * WP];
    __shared__ float red[NW * 16 * 64];
    __shared__ float sH1[H * HP], sH2[H * HP];
    __shared__ float sb1[H], sb2[H], sb3[AMAX], ssig[AMAX], slo[AMAX], shi[AMAX];
    __shared__ float seps[R][AMAX + 1];
    __shared__ RowState rs[R], rr[R];
    __shared__ int s_nd, s_last;
    __shared__ int64_t s_row[R];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63;
    const int64_t k = a.k;
    const int D = (int)a.dim;
    const int A = (int)a.act_dim;
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int nrows = (int)min((int64_t)R, k - r0);
    const int Kp = (int)kpad(D), KW = Kp / NW, SQ = KW / 16;
    const int64_t rng_step = a.rng_ctr ? *a.rng_ctr : 0;
#if COLLECT_STOP == 9
    if (t >= 0) return;  // launch overhead only
#endif
#if COLLECT_TRACE
    if (t == 0) {
        unsigned xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 4] = 0;
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 5] = 0;
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 6] = xcc;
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 7] = hwid;
    }
#endif
    TSTAMP(0)

    // small actor weights: loads in flight during the add phase, LDS stores after it
    float4 w2r[2], w3r;
#pragma unroll
    for (int j = 0; j < 2; ++j) w2r[j] = reinterpret_cast<const float4*>(a.w2)[t + NT * j];
    w3r = reinterpret_cast<const float4*>(a.w3)[t < A * 16 ? t : 0];
    float vb1 = 0.f, vb2 = 0.f, vb3 = 0.f, vls = 0.f, vlo = -1.f, vhi = 1.f;
    if (t < H) {
        vb1 = a.b1[t];
        vb2 = a.b2[t];
    }
    if (t < A) {
        vb3 = a.b3[t];
        vls = a.log_std[t];
        if (a.low) {
            vlo = a.low[t];
            vhi = a.high[t];
        }
    }
    // layer-1 weight fragments of this wave (SQ <= KMAX / 128 = 4) and the env rows' episode
    // counters: independent of the add phase, so their latency hides behind it
    float4 wall[KMAX / 128][4];
    {
        const float4* wp = reinterpret_cast<const float4*>(a.w1p) + (int64_t)w * SQ * 4 * 64 + l;
#pragma unroll
        for (int sq = 0; sq < KMAX / 128; ++sq)
#pragma unroll
            for (int ft = 0; ft < 4; ++ft)
                wall[sq][ft] = wp[((sq < SQ ? sq : 0) * 4 + ft) * 64];
    }

    // ---- A. pending add of the previous step -> buffer rows + live obs (HBM and sX) ---------
    if (a.add.k > 0) {
        const int64_t urel = a.add.rel_dev ? *a.add.rel_dev : a.add.uniform_rel;
        // 32 lanes per row: all 16 rows' loads in flight at once
        const int rw = t >> 5;
        if (rw < nrows) add_row(a.add, r0 + rw, t & 31, urel, sX + rw, XP, 32, false);
        if (a.add.rel_next && blockIdx.x == 0 && t == 0)
            *a.add.rel_next = (urel + 1) % a.add.ring_size;
    } else {
        const int nq = D >> 2;
        for (int i = t; i < nrows * nq; i += NT) {
            const int rw = i / nq, q = i - rw * nq;
            const float4 x = reinterpret_cast<const float4*>(a.cur + (r0 + rw) * D)[q];
            sX[(4 * q) * XP + rw] = x.x;
            sX[(4 * q + 1) * XP + rw] = x.y;
            sX[(4 * q + 2) * XP + rw] = x.z;
            sX[(4 * q + 3) * XP + rw] = x.w;
        }
    }
    TSTAMP(1)
    // the env rows' episode counters: loaded now, used after the actor phase
    int64_t ej = 0, et = 0;
    if (t < nrows) {
        ej = a.ep_j[r0 + t];
        et = a.ep_t[r0 + t];
    }
    // zero padding: columns [D, Kp) and rows past the last env of a partial tile
    for (int i = t; i < (Kp - D) * R; i += NT) sX[(D + i / R) * XP + (i % R)] = 0.0f;
    if (nrows < R)
        for (int i = t; i < D * (R - nrows); i += NT) {
            const int c = i / (R - nrows), rw = nrows + i % (R - nrows);
            sX[c * XP + rw] = 0.0f;
        }
    // noise of this workgroup's rows: thread -> (row, pair of action dims)
    if (a.sample && t < R * 16) {
        const int er = t >> 4, pr = t & 15, a0 = 2 * pr;
        float2 z = make_float2(0.f, 0.f);
        if (er < nrows && a0 < A) z = counter_normal2(a.act_seed, rng_step, r0 + er, pr);
        seps[er][a0] = z.x;
        seps[er][a0 + 1] = z.y;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int e = 4 * (t + NT * j), rw = e >> 6, col = e & 63;
        float* d = sW2 + rw * WP + col;
        d[0] = w2r[j].x;
        d[1] = w2r[j].y;
        d[2] = w2r[j].z;
        d[3] = w2r[j].w;
    }
    {
        const int e = 4 * t, rw = e >> 6, col = e & 63;
        if (rw < AMAX) {
            const bool ok = rw < A;
            float* d = sW3 + rw * WP + col;
            d[0] = ok ? w3r.x : 0.f;
            d[1] = ok ? w3r.y : 0.f;
            d[2] = ok ? w3r.z : 0.f;
            d[3] = ok ? w3r.w : 0.f;
        }
    }
    if (t < H) {
        sb1[t] = vb1;
        sb2[t] = vb2;
    }
    if (t < AMAX) {
        sb3[t] = vb3;
        ssig[t] = t < A ? expf(vls) : 1.0f;
        slo[t] = vlo;
        shi[t] = vhi;
    }
    if (a.rng_next && blockIdx.x == 0 && t == 0) *a.rng_next = rng_step + 1;
    __syncthreads();
    // this step's stored obs rows (ReplayBuffer obs of step i = the live obs the actor sees):
    // written here from LDS, so the add of step i (next launch / flush) copies nothing and the
    // live obs never round-trips through HBM between fused steps
    if (t < nrows) {
        // with a pending add this launch's block 0 advances the device cursor concurrently,
        // so the position is the add's own plus one (the ring's uniform next)
        int64_t urel;
        if (a.add.k > 0) {
            const int64_t up = a.add.rel_dev ? *a.add.rel_dev : a.add.uniform_rel;
            urel = (up + 1) % a.add.ring_size;
        } else {
            urel = a.obs_rel_dev ? *a.obs_rel_dev : a.obs_uniform_rel;
        }
        s_row[t] = a.obs_offset[r0 + t] + urel;
    }
    __syncthreads();
    for (int i = t; i < nrows * D; i += NT) {
        const int rw = i / D, c = i - rw * D;
        a.obs_dst[s_row[rw] * D + c] = sX[c * XP + rw];
    }
#if COLLECT_STOP == 1
    return;
#endif

    // ---- B. actor: layer 1 (wave w: k in [w KW, (w+1) KW), all 64 features) -----------------
    {
        f32x4 acc[4];
#pragma unroll
        for (int ft = 0; ft < 4; ++ft) acc[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* xb = sX + (w * KW + (l >> 4)) * XP + (l & 15);
#pragma unroll
        for (int sq = 0; sq < KMAX / 128; ++sq) {
            if (sq >= SQ) break;
            const float* xs = xb + 16 * sq * XP;
            const float b0 = xs[0], b1 = xs[4 * XP], b2 = xs[8 * XP], b3 = xs[12 * XP];
#pragma unroll
            for (int ft = 0; ft < 4; ++ft) {
                acc[ft] = mfma4(wall[sq][ft].x, b0, acc[ft]);
                acc[ft] = mfma4(wall[sq][ft].y, b1, acc[ft]);
                acc[ft] = mfma4(wall[sq][ft].z, b2, acc[ft]);
                acc[ft] = mfma4(wall[sq][ft].w, b3, acc[ft]);
            }
        }
        // red[w][ft][r][lane]
#pragma unroll
        for (int ft = 0; ft < 4; ++ft)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((w * 4 + ft) * 4 + r) * 64 + l] = acc[ft][r];
    }
    __syncthreads();
    // h1 = tanh(sum over the 8 waves in order + b1) -> sH1[f][row]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = t + NT * j;  // (ft, r, lane)
        const int ln = i & 63, r = (i >> 6) & 3, ft = i >> 8;
        float z = red[i];
#pragma unroll
        for (int v = 1; v < NW; ++v) z += red[v * 16 * 64 + i];
        const int f = 16 * ft + 4 * (ln >> 4) + r;
        sH1[f * HP + (ln & 15)] = tanh_nb(z + sb1[f]);
    }
    __syncthreads();
    // layer 2: wave w -> feature tile w & 3 over k half w >> 2 (8 steps of 4)
    {
        const int ft = w & 3, kh = w >> 2;
        f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* wa = sW2 + (16 * ft + (l & 15)) * WP + 32 * kh + (l >> 4);
        const float* hb = sH1 + (32 * kh + (l >> 4)) * HP + (l & 15);
#pragma unroll
        for (int s = 0; s < 8; ++s) z = mfma4(wa[4 * s], hb[4 * s * HP], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(w * 4 + r) * 64 + l] = z[r];
    }
    __syncthreads();
    // h2 = tanh(half 0 + half 1 + b2) -> sH2
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = t + NT * j;  // (ft, r, lane) of 4 x 4 x 64
        const int ln = i & 63, r = (i >> 6) & 3, ft = i >> 8;
        const float z = red[(ft * 4 + r) * 64 + ln] + red[((ft + 4) * 4 + r) * 64 + ln];
        const int f = 16 * ft + 4 * (ln >> 4) + r;
        sH2[f * HP + (ln & 15)] = tanh_nb(z + sb2[f]);
    }
    __syncthreads();
    // mu head: wave w -> action tile w & 1 over k quarter w >> 1 (4 steps of 4)
    {
        const int at = w & 1, kq = w >> 1;
        f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* wa = sW3 + (16 * at + (l & 15)) * WP + 16 * kq + (l >> 4);
        const float* hb = sH2 + (16 * kq + (l >> 4)) * HP + (l & 15);
#pragma unroll
        for (int s = 0; s < 4; ++s) z = mfma4(wa[4 * s], hb[4 * s * HP], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(w * 4 + r) * 64 + l] = z[r];
    }
    __syncthreads();
    // mu = sum of the 4 quarters + b3; act = randn * sigma + mu; map_action -> act_remap
    {
        const int ln = t & 63, r = (t >> 6) & 3, at = t >> 8;  // 2 x 4 x 64 = 512 threads
        const int a_ = 16 * at + 4 * (ln >> 4) + r, rw = ln & 15;
        if (a_ < A && rw < nrows) {
            float mu = red[(at * 4 + r) * 64 + ln];
#pragma unroll
            for (int kq = 1; kq < 4; ++kq) mu += red[((at + 2 * kq) * 4 + r) * 64 + ln];
            const float m = mu + sb3[a_];
            float x = m;
            if (a.sample) x = seps[rw][a_] * ssig[a_] + m;  // contract(off): two roundings
            const int64_t row = r0 + rw;
            a.act[row * A + a_] = x;
            float y = x;
            if (a.bound_method == 1) y = y < -1.0f ? -1.0f : (y > 1.0f ? 1.0f : y);
            else if (a.bound_method == 2) y = tanh_nb(y);
            if (a.low) {
                const float lo = slo[a_], hi = shi[a_];
                y = lo + (hi - lo) * (y + 1.0f) / 2.0f;
            }
            a.act_remap[row * A + a_] = y;
        }
    }

#if COLLECT_STOP == 2
    return;
#endif
    // ---- C. env step + auto-reset of these rows (env.hip box_step_reset_kernel) -------------
    TSTAMP(2)
    if (t == 0) s_nd = 0;
    __syncthreads();
    if (t < R) {
        const int64_t r = r0 + t;
        RowState st = {0ull, 0}, sr = {0ull, 0};
        if (t < nrows) {
            const int64_t e = r;
            int64_t j = ej;
            int64_t tt = et + 1;
            st.key = env_key(a.env_seed, (uint64_t)e, j, tt);
            st.active = 1;
            const uint64_t h = sm64(st.key ^ REW_SALT);
            a.rew[r] = (double)(h >> 40) * 0x1p-24;
            const bool dn = tt >= a.ep_len;
            a.term[r] = (uint8_t)(dn && (e % 2 == 0));
            a.trunc[r] = (uint8_t)(dn && (e % 2 == 1));
            a.done[r] = (uint8_t)dn;
            if (dn) {
                j += 1;
                tt = (j == 0) ? (e % a.ep_len) : 0;
                a.ep_j[e] = j;
                sr.key = env_key(a.env_seed, (uint64_t)e, j, tt);
                sr.active = 1;
                atomicAdd(&s_nd, 1);
            }
            a.ep_t[e] = tt;
        }
        rs[t] = st;
        rr[t] = sr;
    }
    __syncthreads();
    const int nd = s_nd;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        ws.part + (int64_t)blockIdx.x * ws.pstride, 0, (int)(ws.pstride * 8), 0x00020000);
    for (int d = t; d < D; d += NT) {
        double s1 = 0.0, q1 = 0.0, s2 = 0.0, q2 = 0.0;
        for (int r = 0; r < nrows; ++r) {
            const float x = box_val(rs[r].key, d);
            a.raw[(r0 + r) * D + d] = x;
            s1 += (double)x;
            q1 += (double)x * (double)x;
        }
        if (nd > 0)
            for (int r = 0; r < nrows; ++r) {
                if (!rr[r].active) continue;
                const float x = box_val(rr[r].key, d);
                a.reset_raw[(r0 + r) * D + d] = x;
                s2 += (double)x;
                q2 += (double)x * (double)x;
            }
        st2_sc1(prs, 16 * d, s1, q1);
        st2_sc1(prs, 16 * (D + d), s2, q2);
    }
    if (t == 0) st2_sc1(prs, 32 * D, (double)nd, 0.0);

#if COLLECT_STOP == 3
    return;
#endif
    // ---- D. obs_rms: deterministic two-level fold by the last workgroups ---------------------
    // Hand-off (cdna_hip_programming.md Guideline 16, counter form with write-through data):
    // partials stored sc1 and drained by every wave, ONE relaxed agent-scope ticket add per
    // workgroup; the last arriver reads them with sc1 loads only (no L2 write-back / L1
    // invalidate fences: a __threadfence() in every thread cost ~100 us per step).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TSTAMP(3)
    const int g = (int)(blockIdx.x / GS);
    const int64_t gb0 = (int64_t)g * GS, gb1 = min(gb0 + GS, ws.nblk);
    if (t == 0) {
        const unsigned int prev = __hip_atomic_fetch_add(&ws.tickets[g], 1u, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (unsigned int)(gb1 - gb0 - 1);
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the group's slabs, every load of an entry issued before its (index-ordered) sum; entry
    // i < D: step column i, D <= i < 2D: reset column i - D, i = 2D: (reset-row count, 0)
    const int gn = (int)(gb1 - gb0);
    const int64_t sb = ws.pstride * 8;  // slab bytes
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
        ws.part + gb0 * ws.pstride, 0, (int)(sb * gn), 0x00020000);
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        ws.gpart + (int64_t)g * ws.pstride, 0, (int)sb, 0x00020000);
    for (int i = t; i <= 2 * D; i += NT) {
        double2 v[GS];
#pragma unroll
        for (int b = 0; b < GS; ++b)
            v[b] = b < gn ? ld2_sc1(grs, (int)(b * sb + 16 * i)) : make_double2(0.0, 0.0);
        double x = 0.0, y = 0.0;
#pragma unroll
        for (int b = 0; b < GS; ++b) {
            x += v[b].x;
            y += v[b].y;
        }
        st2_sc1(ors, 16 * i, x, y);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TSTAMP(4)
    if (t == 0) {
        __hip_atomic_store(&ws.tickets[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int prev = __hip_atomic_fetch_add(&ws.tickets[ws.ngroups], 1u,
                                                         __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (unsigned int)(ws.ngroups - 1);
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the last group: totals over the groups in index order, then both updates per column
    const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(
        ws.gpart, 0, (int)(ws.pstride * 8 * ws.ngroups), 0x00020000);
    const int64_t gsb = ws.pstride * 8;
    const double old_count = *a.count;
    const double bc1 = (double)k;
    double ND = 0.0;
    for (int d = t; d < D; d += NT) {  // D > 0: thread 0 always runs (its ND sets count)
        double S1 = 0.0, Q1 = 0.0, S2 = 0.0, Q2 = 0.0;
        const int dc = d;
        ND = 0.0;
        for (int g0 = 0; g0 < ws.ngroups; g0 += GS) {
            double2 v1[GS], v2[GS], vn[GS];
#pragma unroll
            for (int j = 0; j < GS; ++j) {
                const bool in = g0 + j < ws.ngroups;
                const int base = (int)((g0 + j) * gsb);
                v1[j] = in ? ld2_sc1(trs, base + 16 * dc) : make_double2(0.0, 0.0);
                v2[j] = in ? ld2_sc1(trs, base + 16 * (D + dc)) : make_double2(0.0, 0.0);
                vn[j] = in ? ld2_sc1(trs, base + 32 * D) : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (int j = 0; j < GS; ++j) {
                S1 += v1[j].x;
                Q1 += v1[j].y;
                S2 += v2[j].x;
                Q2 += v2[j].y;
                ND += vn[j].x;
            }
        }
        const double tot1 = old_count + bc1, tot2 = tot1 + ND;
        if (a.totals) {
            a.totals[2 * d] = S1;
            a.totals[2 * d + 1] = Q1;
            a.totals[2 * D + 2 * d] = S2;
            a.totals[2 * D + 2 * d + 1] = Q2;
            continue;
        }
        // rms.hip rms_merge2_kernel's arithmetic
        double m0 = (double)a.mean[d], v0 = (double)a.var[d];
        if (bc1 > 0.0) {
            const double bm = S1 / bc1;
            double bv = Q1 / bc1 - bm * bm;
            bv = bv < 0.0 ? 0.0 : bv;
            const double delta = bm - m0;
            const double nm = m0 + delta * bc1 / tot1;
            const double m2 = v0 * old_count + bv * bc1 + delta * delta * old_count * bc1 / tot1;
            m0 = (double)(float)nm;
            v0 = (double)(float)(m2 / tot1);
        }
        a.snap_mean[d] = (float)m0;
        a.snap_var[d] = (float)v0;
        if (ND > 0.0) {
            const double bm = S2 / ND;
            double bv = Q2 / ND - bm * bm;
            bv = bv < 0.0 ? 0.0 : bv;
            const double delta = bm - m0;
            const double nm = m0 + delta * ND / tot2;
            const double m2 = v0 * tot1 + bv * ND + delta * delta * tot1 * ND / tot2;
            m0 = (double)(float)nm;
            v0 = (double)(float)(m2 / tot2);
        }
        a.mean[d] = (float)m0;
        a.var[d] = (float)v0;
    }
    __syncthreads();  // every thread has read *count
    TSTAMP(5)
    if (t == 0) {
        if (a.totals) {
            a.totals[4 * D] = ND;
            a.totals[4 * D + 1] = bc1;
        } else {
            *a.count = old_count + bc1 + ND;
        }
        __hip_atomic_store(&ws.tickets[ws.ngroups], 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

inline int64_t nblk_for(int64_t k) { return (k + R - 1) / R; }
inline int ngroups_for(int64_t k) { return (int)((nblk_for(k) + GS - 1) / GS); }
inline int64_t ticket_bytes(int64_t k) { return ((ngroups_for(k) + 1) * 4 + 255) / 256 * 256; }
inline int64_t trace_bytes(int64_t k) { return COLLECT_TRACE ? 16 * nblk_for(k) * 64 : 0; }

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_collect_pack_floats(int64_t dim) { return dim > 0 ? H * kpad(dim) : 0; }

extern "C" int tsrl_collect_pack_w1(const float* W, int64_t dim, float* packed, void* stream) {
    TSRL_CHECK_ARG(W && packed && dim > 0 && dim <= KMAX, "tsrl_collect_pack_w1: bad arguments");
    const int64_t total = tsrl_collect_pack_floats(dim);
    const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(pack_w1_kernel, dim3(grid), dim3(256), 0, as_stream(stream), W, dim, packed);
    TSRL_LAUNCH_CHECK("tsrl_collect_pack_w1");
    return 0;
}

extern "C" int64_t tsrl_collect_workspace_bytes(int64_t k, int64_t dim) {
    if (k <= 0 || dim <= 0) return 0;
    return ticket_bytes(k) + (nblk_for(k) + ngroups_for(k)) * (4 * dim + 4) * 8 + trace_bytes(k);
}

extern "C" int tsrl_collect_box_step(const tsrl_collect_args* a, void* stream) {
    TSRL_CHECK_ARG(a != nullptr, "tsrl_collect_box_step: null args");
    const int64_t k = a->k, D = a->dim;
    TSRL_CHECK_ARG(k > 0 && D > 0 && D % 4 == 0 && D <= KMAX,
                   "tsrl_collect_box_step: need k > 0 and 0 < dim <= %d, dim %% 4 == 0", KMAX);
    TSRL_CHECK_ARG(a->act_dim > 0 && a->act_dim <= AMAX && a->bound_method >= 0 &&
                       a->bound_method <= 2,
                   "tsrl_collect_box_step: 0 < act_dim <= %d, bound_method 0..2", AMAX);
    TSRL_CHECK_ARG(a->obs_dst && a->obs_offset && (a->obs_rel_dev || a->obs_uniform_rel >= 0),
                   "tsrl_collect_box_step: obs_dst / obs_offset / this step's ring position");
    TSRL_CHECK_ARG(a->cur && a->w1p && a->b1 && a->w2 && a->b2 && a->w3 && a->b3 && a->log_std &&
                       a->act && a->act_remap && a->ep_j && a->ep_t && a->raw && a->reset_raw &&
                       a->rew && a->term && a->trunc && a->done && a->workspace && a->mean &&
                       a->var && a->count && (a->totals || (a->snap_mean && a->snap_var)),
                   "tsrl_collect_box_step: null pointer");
    // w1p / workspace are this library's layouts; cur, w2 and w3 are read with 16-byte loads
    // at 4-byte alignment (parameters may be views into a flat parameter buffer)
    TSRL_CHECK_ARG(aligned16(a->w1p) && aligned16(a->workspace) &&
                       ((reinterpret_cast<uintptr_t>(a->cur) | reinterpret_cast<uintptr_t>(a->w2) |
                         reinterpret_cast<uintptr_t>(a->w3)) & 3u) == 0,
                   "tsrl_collect_box_step: w1p / workspace must be 16-byte aligned, cur / w2 / w3 "
                   "4-byte aligned");
    TSRL_CHECK_ARG((a->low == nullptr) == (a->high == nullptr), "tsrl_collect_box_step: low/high");
    TSRL_CHECK_ARG(!a->sample || (a->rng_ctr && a->rng_next && a->rng_ctr != a->rng_next),
                   "tsrl_collect_box_step: sampling needs the rng counter pair");
    TSRL_CHECK_ARG(a->ep_len > 0, "tsrl_collect_box_step: ep_len <= 0");
    const tsrl_add_args& ad = a->add;
    if (ad.k != 0) {
        // the pending add runs row for row with this launch's env rows: same rows, identity
        // ids, f32 live-obs rows of dim columns, the live obs as cur_obs (its new rows are
        // the policy input)
        TSRL_CHECK_ARG(ad.k == k && ad.ids == nullptr && ad.obs_next_src && ad.cur_obs == a->cur &&
                           ad.obs_dim == D && ad.offset && ad.ep_rew && ad.ep_len && ad.ep_idx,
                       "tsrl_collect_box_step: pending add must cover the same k rows "
                       "(ids NULL, cur_obs == cur, obs_dim == dim)");
        TSRL_CHECK_ARG(!ad.rel_dev || (ad.ring_size > 0 && !ad.ptr),
                       "tsrl_collect_box_step: add.rel_dev needs ring_size and ptr == NULL");
        TSRL_CHECK_ARG(!ad.rel_next || (ad.rel_dev && ad.rel_next != ad.rel_dev),
                       "tsrl_collect_box_step: add.rel_next needs rel_dev (a different word)");
        TSRL_CHECK_ARG(!ad.reset_mask || ad.reset_src, "tsrl_collect_box_step: add reset_src");
        TSRL_CHECK_ARG(!ad.obs_src, "tsrl_collect_box_step: the pending add copies no obs (the "
                                    "launch that produced it stored them)");
    }
    Ws ws;
    ws.nblk = nblk_for(k);
    ws.ngroups = ngroups_for(k);
    ws.pstride = 4 * D + 4;
    char* base = reinterpret_cast<char*>(a->workspace);
    ws.tickets = reinterpret_cast<unsigned int*>(base);
    ws.part = reinterpret_cast<double*>(base + ticket_bytes(k));
    ws.gpart = ws.part + ws.nblk * ws.pstride;
    ws.trace = reinterpret_cast<uint64_t*>(ws.gpart + ws.ngroups * ws.pstride);
    tsrl_collect_args p = *a;
    p.act_seed = sm64(a->act_seed);
    p.env_seed = sm64(a->env_seed);
    hipLaunchKernelGGL(collect_box_step_kernel, dim3((unsigned)ws.nblk), dim3(NT), 0,
                       as_stream(stream), p, ws);
    TSRL_LAUNCH_CHECK("tsrl_collect_box_step");
    return 0;
}
