// Fused Gaussian policy step for the collector (Collector.collect -> policy.forward ->
// dist.sample -> map_action; tianshou/data/collector.py:286-303, policy/modelfree/pg.py:
// 133-171, policy/base.py:183-215) for the MuJoCo actor of utils/models.py:34-97:
//   mu  = Linear(64,A)(tanh(Linear(64,64)(tanh(Linear(D,64)(obs)))))   (unbounded)
//   act = eps * exp(log_std) + mu        (dist.sample() = torch.normal(mu, sigma))
//   act_remap = scale(bound(act))         (clip / tanh to [-1,1], then to [low, high])
// One workgroup = 32 env rows.  The first layer's K (= obs dim) is split over the 8 waves
// (f32 MFMA 32x32x2, batch rows on lanes, features on accumulator registers as in
// mlp.hip); layer 2 and the mu head are split over the 8 waves too (K quarters / eighths),
// every partial folded in fixed order through LDS.  The first-layer weight is pre-packed
// once per collect into the per-lane fragment order so every weight load is a contiguous
// 1 KB wave access.
#include "noise.h"

namespace tsrl {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int H = 64;
constexpr int AMAX = 32;
constexpr int WS = 65;

__device__ __forceinline__ int rho(int r) { return (r & 3) + 8 * (r >> 2); }
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.0f;
    return z;
}

// K padded to a multiple of 16; lane half h owns k in [h*S, (h+1)*S), S = Kp/2.
__host__ __device__ inline int64_t kpad(int64_t D) { return (D + 15) / 16 * 16; }

// packed[ot][g][lane][4] = W[32*ot + (lane&31)][(lane>>5)*S + 4*g + e]   (0 beyond D)
__global__ void pack_l1_kernel(const float* __restrict__ W, int64_t D, float* __restrict__ out) {
    const int64_t S = kpad(D) / 2, G = S / 4;
    const int64_t total = 2 * G * 64 * 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const int64_t g = (i >> 8) % G;
        const int ot = (int)((i >> 8) / G);
        const int64_t k = (lane >> 5) * S + 4 * g + e;
        out[i] = k < D ? W[(int64_t)(32 * ot + (lane & 31)) * D + k] : 0.0f;
    }
}

struct ActParams {
    int A, bound, scale, sample;
    uint64_t seed;  // rng mode (eps == NULL, sample): counter-based normals
};

constexpr int ANW = 8;  // waves per workgroup: the first layer's K is split 8 ways

__global__ __launch_bounds__(ANW * 64) void gauss_act_kernel(
    const float* __restrict__ obs, int64_t ldx, int64_t n, int64_t D,
    const float* __restrict__ w1p, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ w3, const float* __restrict__ b3,
    const float* __restrict__ log_std, const float* __restrict__ eps,
    const float* __restrict__ low, const float* __restrict__ high, ActParams p,
    float* __restrict__ act, float* __restrict__ act_remap, const int64_t* rng_ctr,
    int64_t* rng_next) {
#pragma clang fp contract(off)
    constexpr int NT = ANW * 64;
    __shared__ float sW2[H * WS], sW3[AMAX * WS];
    __shared__ float sb1[H], sb2[H], sb3[AMAX], ssig[AMAX], slo[AMAX], shi[AMAX];
    __shared__ float seps[32][AMAX + 1];
    __shared__ float red[ANW][2][16][64];
    __shared__ float sH[H * 32];  // h1, then h2: [feature][row]
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int A = p.A;
    const int64_t row0 = (int64_t)blockIdx.x * 32;
    const int64_t row = row0 + c;
    const bool live = row < n;
    const int64_t rng_step = rng_ctr ? *rng_ctr : 0;
    // small weights: loads issued now, LDS stores after the layer-1 loop (latency hidden)
    float4 w2r[2], w3r;
#pragma unroll
    for (int j = 0; j < 2; ++j) w2r[j] = reinterpret_cast<const float4*>(w2)[t + NT * j];
    w3r = reinterpret_cast<const float4*>(w3)[t < A * 16 ? t : 0];
    float vb1 = 0.f, vb2 = 0.f, vb3 = 0.f, vls = 0.f, vlo = -1.f, vhi = 1.f;
    if (t < H) {
        vb1 = b1[t];
        vb2 = b2[t];
    }
    if (t < A) {
        vb3 = b3[t];
        vls = log_std[t];
        if (p.scale) {
            vlo = low[t];
            vhi = high[t];
        }
    }
    // noise of this workgroup's 32 rows: thread -> (row, pair of action dims)
    if (p.sample) {
        const int er = t >> 4, pr = t & 15, a0 = 2 * pr;
        float2 z = make_float2(0.f, 0.f);
        if (row0 + er < n && a0 < A) {
            if (eps) {
                z.x = eps[(row0 + er) * A + a0];
                if (a0 + 1 < A) z.y = eps[(row0 + er) * A + a0 + 1];
            } else {
                z = counter_normal2(p.seed, rng_step, row0 + er, pr);
            }
        }
        seps[er][a0] = z.x;
        seps[er][a0 + 1] = z.y;
    }
    const int64_t S = kpad(D) / 2, G = S / 4;
    const int64_t g0 = G * w / ANW, g1 = G * (w + 1) / ANW;
    f32x16 acc0 = zero16(), acc1 = zero16();
    const float* xrow = obs + (live ? row : 0) * ldx;
    const float4* wp0 = reinterpret_cast<const float4*>(w1p) + l;
    const float4* wp1 = reinterpret_cast<const float4*>(w1p) + G * 64 + l;
    // rows of D % 4 != 0 columns (or a pitch that is not a multiple of 4) are read as four
    // scalars per group, each bounded by D
    const bool vec = (D & 3) == 0 && (ldx & 3) == 0;
    // batches of 6 groups: all loads of a batch are in flight before its first MFMA
    constexpr int GB = 6;
    for (int64_t gb = g0; gb < g1; gb += GB) {
        float4 xv[GB], a0[GB], a1[GB];
#pragma unroll
        for (int j = 0; j < GB; ++j) {
            const int64_t g = gb + j;
            const bool gin = g < g1;
            const int64_t k = h * S + 4 * (gin ? g : g0);
            const bool xin = gin && live && k < D;
            if (vec) {
                xv[j] = *reinterpret_cast<const float4*>(xrow + (xin ? k : 0));
            } else {
                xv[j].x = xrow[xin ? k : 0];
                xv[j].y = xin && k + 1 < D ? xrow[k + 1] : 0.0f;
                xv[j].z = xin && k + 2 < D ? xrow[k + 2] : 0.0f;
                xv[j].w = xin && k + 3 < D ? xrow[k + 3] : 0.0f;
            }
            a0[j] = wp0[(gin ? g : g0) * 64];
            a1[j] = wp1[(gin ? g : g0) * 64];
            if (!xin) xv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!gin) a0[j] = a1[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < GB; ++j) {
            acc0 = mfma(a0[j].x, xv[j].x, acc0);
            acc1 = mfma(a1[j].x, xv[j].x, acc1);
            acc0 = mfma(a0[j].y, xv[j].y, acc0);
            acc1 = mfma(a1[j].y, xv[j].y, acc1);
            acc0 = mfma(a0[j].z, xv[j].z, acc0);
            acc1 = mfma(a1[j].z, xv[j].z, acc1);
            acc0 = mfma(a0[j].w, xv[j].w, acc0);
            acc1 = mfma(a1[j].w, xv[j].w, acc1);
        }
    }
    // weights to LDS
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int e = 4 * (t + NT * j), rr = e >> 6, col = e & 63;
        float* d = sW2 + rr * WS + col;
        d[0] = w2r[j].x;
        d[1] = w2r[j].y;
        d[2] = w2r[j].z;
        d[3] = w2r[j].w;
    }
    {
        const int e = 4 * t, rr = e >> 6, col = e & 63;
        if (rr < AMAX) {
            const bool ok = rr < A;
            float* d = sW3 + rr * WS + col;
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
    // next step's noise counter into the other slot of a ping-pong pair (no atomics)
    if (rng_next && blockIdx.x == 0 && t == 0) *rng_next = rng_step + 1;
    // Every later stage is spread over all 8 waves (a serial chain of 96 dependent MFMAs in
    // one wave cost ~8 us of the ~17 us kernel).  Register slot j of the 32x64 C tile
    // (ot = j >> 4, r = j & 15) holds feature 32*ot + rho(r) + 4h of row c.
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        red[w][0][r][l] = acc0[r];
        red[w][1][r][l] = acc1[r];
    }
    __syncthreads();
    // layer-1 partials summed over the waves in fixed order; h1 -> sH[feature][row]
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int j = 4 * w + q, ot = j >> 4, r = j & 15;
        float z = red[0][ot][r][l];
#pragma unroll
        for (int v = 1; v < ANW; ++v) z += red[v][ot][r][l];
        const int f = 32 * ot + rho(r) + 4 * h;
        sH[f * 32 + c] = tanh_nb(z + sb1[f]);
    }
    __syncthreads();
    // layer 2: wave w -> output tile ot = w & 1 over k quarter kq = w >> 1 (16 k, 8 steps)
    {
        const int ot = w & 1, kq = w >> 1;
        f32x16 z = zero16();
        const float* wa = sW2 + (32 * ot + c) * WS + 16 * kq + h;
        const float* hb = sH + (16 * kq + h) * 32 + c;
#pragma unroll
        for (int st = 0; st < 8; ++st) z = mfma(wa[2 * st], hb[64 * st], z);
        float* rp = &red[0][0][0][0] + w * 16 * 64;
#pragma unroll
        for (int r = 0; r < 16; ++r) rp[r * 64 + l] = z[r];
    }
    __syncthreads();
    // h2 = tanh(sum of the 4 k quarters + b2) -> sH (h1 is dead)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int j = 4 * w + q, ot = j >> 4, r = j & 15;
        const float* rp = &red[0][0][0][0] + ot * 16 * 64 + r * 64 + l;
        float z = rp[0];
#pragma unroll
        for (int kq = 1; kq < 4; ++kq) z += rp[2 * kq * 16 * 64];
        const int f = 32 * ot + rho(r) + 4 * h;
        sH[f * 32 + c] = tanh_nb(z + sb2[f]);
    }
    __syncthreads();
    // mu head: wave w -> k eighth (8 k, 4 steps); rows of sW3 beyond A are zero
    {
        f32x16 z = zero16();
        const float* wa = sW3 + c * WS + 8 * w + h;
        const float* hb = sH + (8 * w + h) * 32 + c;
#pragma unroll
        for (int st = 0; st < 4; ++st) z = mfma(wa[2 * st], hb[64 * st], z);
        float* rp = &red[0][0][0][0] + w * 16 * 64;
#pragma unroll
        for (int r = 0; r < 16; ++r) rp[r * 64 + l] = z[r];
    }
    __syncthreads();
    if (!live) return;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int r = 2 * w + q;
        const int a = rho(r) + 4 * h;
        if (a >= A) continue;
        const float* rp = &red[0][0][0][0] + r * 64 + l;
        float mu = rp[0];
#pragma unroll
        for (int v = 1; v < ANW; ++v) mu += rp[v * 16 * 64];
        const float m = mu + sb3[a];
        float x = m;
        // randn * sigma + mu (two roundings, as torch's mul_ then add_)
        if (p.sample) x = seps[c][a] * ssig[a] + m;  // contract(off): two roundings
        act[row * A + a] = x;
        float y = x;
        if (p.bound == 1) y = y < -1.0f ? -1.0f : (y > 1.0f ? 1.0f : y);  // clamp, NaN passes
        else if (p.bound == 2) y = tanh_nb(y);
        if (p.scale) {
            const float lo = slo[a], hi = shi[a];
            y = lo + (hi - lo) * (y + 1.0f) / 2.0f;
        }
        act_remap[row * A + a] = y;
    }
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_policy_pack_floats(int64_t D) { return 2 * (kpad(D) / 2) * 64; }

extern "C" int tsrl_policy_pack_l1(const float* W, int64_t D, float* packed, void* stream) {
    TSRL_CHECK_ARG(W && packed && D > 0, "tsrl_policy_pack_l1: bad arguments");
    const int64_t total = tsrl_policy_pack_floats(D);
    const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(pack_l1_kernel, dim3(grid), dim3(256), 0, as_stream(stream), W, D, packed);
    TSRL_LAUNCH_CHECK("tsrl_policy_pack_l1");
    return 0;
}

extern "C" int tsrl_gauss_policy_act(const float* obs, int64_t ldx, int64_t n, int64_t D,
                                     const float* w1packed, const float* b1, const float* w2,
                                     const float* b2, const float* w3, const float* b3,
                                     const float* log_std, int64_t act_dim, const float* eps,
                                     int bound_method, const float* low, const float* high,
                                     float* act, float* act_remap, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && D > 0 && ldx >= D && act_dim > 0 && act_dim <= AMAX &&
                       bound_method >= 0 && bound_method <= 2,
                   "tsrl_gauss_policy_act: bad sizes (ldx >= D; 0 < act_dim <= %d)", AMAX);
    if (n == 0) return 0;
    TSRL_CHECK_ARG(obs && w1packed && b1 && w2 && b2 && w3 && b3 && log_std && act && act_remap,
                   "tsrl_gauss_policy_act: null pointer");
    TSRL_CHECK_ARG((aligned16(obs) || D % 4 || ldx % 4) && aligned16(w1packed),
                   "tsrl_gauss_policy_act: obs (rows read as float4) / packed weights must be "
                   "16-byte aligned");
    TSRL_CHECK_ARG((low == nullptr) == (high == nullptr), "tsrl_gauss_policy_act: low/high");
    ActParams p{(int)act_dim, bound_method, low != nullptr, eps != nullptr, 0ull};
    hipLaunchKernelGGL(gauss_act_kernel, dim3((unsigned)((n + 31) / 32)), dim3(ANW * 64), 0,
                       as_stream(stream), obs, ldx, n, D, w1packed, b1, w2, b2, w3, b3, log_std,
                       eps, low, high, p, act, act_remap, nullptr, nullptr);
    TSRL_LAUNCH_CHECK("tsrl_gauss_policy_act");
    return 0;
}

extern "C" int tsrl_gauss_policy_act_rng(const float* obs, int64_t ldx, int64_t n, int64_t D,
                                         const float* w1packed, const float* b1, const float* w2,
                                         const float* b2, const float* w3, const float* b3,
                                         const float* log_std, int64_t act_dim, uint64_t seed,
                                         const int64_t* rng_ctr, int64_t* rng_next,
                                         int bound_method, const float* low, const float* high,
                                         float* act, float* act_remap, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && D > 0 && ldx >= D && act_dim > 0 && act_dim <= AMAX &&
                       bound_method >= 0 && bound_method <= 2,
                   "tsrl_gauss_policy_act_rng: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(obs && w1packed && b1 && w2 && b2 && w3 && b3 && log_std && act && act_remap &&
                       rng_ctr && rng_next && rng_ctr != rng_next,
                   "tsrl_gauss_policy_act_rng: null pointer");
    TSRL_CHECK_ARG((aligned16(obs) || D % 4 || ldx % 4) && aligned16(w1packed),
                   "tsrl_gauss_policy_act_rng: obs (rows read as float4) / packed weights must "
                   "be 16-byte aligned");
    TSRL_CHECK_ARG((low == nullptr) == (high == nullptr), "tsrl_gauss_policy_act_rng: low/high");
    ActParams p{(int)act_dim, bound_method, low != nullptr, 1, sm64(seed)};
    hipLaunchKernelGGL(gauss_act_kernel, dim3((unsigned)((n + 31) / 32)), dim3(ANW * 64), 0,
                       as_stream(stream), obs, ldx, n, D, w1packed, b1, w2, b2, w3, b3, log_std,
                       nullptr, low, high, p, act, act_remap, rng_ctr, rng_next);
    TSRL_LAUNCH_CHECK("tsrl_gauss_policy_act_rng");
    return 0;
}
