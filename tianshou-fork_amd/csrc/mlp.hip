// Fused actor/critic MLP kernels for the PPO minibatch (PPOPolicy.learn, tianshou/policy/
// modelfree/ppo.py:106-151) on the MuJoCo network shape of tianshou/utils/models.py:34-97:
// actor  = Linear(D,64)-Tanh-Linear(64,64)-Tanh-Linear(64,A)      (ActorProb, unbounded)
// critic = Linear(D,64)-Tanh-Linear(64,64)-Tanh-Linear(64,1)      (Critic)
// with the state-independent log-std of fixed_std_normal.
//
// Three kernels per minibatch, all on v_mfma_f32_32x32x2_f32 (exact f32 fma chains, the
// f32 matrix rate of gfx950):
//   l1_fwd_kernel : H1^T = tanh(W1cat . X[idx]^T + b1) for both nets at once (W1cat = the
//                   two first-layer weights stacked, 128 features).  Minibatch rows are read
//                   through the permutation index (no gathered copy of the observations).
//   ppo_tail_kernel: layers 2-3 of both nets, the clipped-surrogate/value loss and its
//                   backward down to dZ1, plus the weight gradients of layers 2-3, per wave
//                   of 32 minibatch rows, without leaving registers/LDS.
//   dw_kernel     : dW1cat = dZ1^T . X[idx] (+ db1 through a ones column), split over the
//                   minibatch rows; dw_reduce_kernel folds the split partials.
//
// Orientation: every activation lives "feature-major" in the MFMA C layout, minibatch rows
// on the 32 lanes of a half-wave and features on the accumulator registers:
//   lane l, register r of a 32x32 tile hold  Z^T[f = rho(r) + 4*(l>>5)][b = l&31],
//   rho(r) = (r&3) + 8*(r>>2).
// A following product that sums over f takes that register as its B operand directly
// (B[k=l>>5][j=l&31]) when the A operand is read with the matching permuted k; so layer 2,
// the heads and the whole backward chain run without moving activations between lanes.
// Only the weight gradients (which sum over the minibatch rows) transpose through LDS.
#include "tsrl_common.h"

namespace tsrl {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int H = 64;           // hidden width of each net (fast path)
constexpr int HC = 2 * H;       // actor + critic first-layer features
constexpr int NT = HC / 32;     // feature tiles of the concatenated first layer
constexpr int AMAX = 32;        // action dims padded to one MFMA tile
constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;

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

// ---------------------------------------------------------------------------------------
// Layer 1 forward.  Workgroup = 128 minibatch rows x 128 features, 4 waves; wave w owns
// rows [32w, 32w+32) and all 4 feature tiles (64 accumulator registers).  K (= obs dim) is
// staged through LDS in 32-wide chunks, double buffered, rows padded to 34 floats so the
// 8-byte fragment reads (k = kk+2h, kk+2h+1 per lane) are bank-conflict free.
// ---------------------------------------------------------------------------------------
constexpr int L1_ROWS = 128;
constexpr int KC = 32;
constexpr int LS = 34;

__global__ __launch_bounds__(256, 2) void l1_fwd_kernel(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ idx, int64_t n, int D,
    const float* __restrict__ Wa, const float* __restrict__ ba, const float* __restrict__ Wc,
    const float* __restrict__ bc, int act_tanh, float* __restrict__ out, int frag_out) {
    __shared__ __attribute__((aligned(16))) float Xs[2][L1_ROWS][LS];
    __shared__ __attribute__((aligned(16))) float Ws[2][HC][LS];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int64_t row0 = (int64_t)blockIdx.x * L1_ROWS;
    // staging assignment: thread t moves float4 column (t&7) of rows (t>>3) + 32q
    const int sc = 4 * (t & 7);
    const float* xsrc[4];
    const float* wsrc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t r = row0 + (t >> 3) + 32 * q;
        xsrc[q] = r < n ? X + (idx ? idx[r] : r) * ldx : nullptr;
        const int f = (t >> 3) + 32 * q;
        wsrc[q] = f < H ? Wa + (int64_t)f * D : Wc + (int64_t)(f - H) * D;
    }
    const int nchunks = (D + KC - 1) / KC;
    float4 xr[4], wr[4];
    auto load = [&](int kc) {
        const int k = kc * KC + sc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), wv = xv;
            if (k + 3 < D) {
                if (xsrc[q]) xv = *reinterpret_cast<const float4*>(xsrc[q] + k);
                wv = *reinterpret_cast<const float4*>(wsrc[q] + k);
            } else if (k < D) {
                float xa[4] = {0.f, 0.f, 0.f, 0.f}, wa[4] = {0.f, 0.f, 0.f, 0.f};
                for (int e = 0; e < 4 && k + e < D; ++e) {
                    if (xsrc[q]) xa[e] = xsrc[q][k + e];
                    wa[e] = wsrc[q][k + e];
                }
                xv = make_float4(xa[0], xa[1], xa[2], xa[3]);
                wv = make_float4(wa[0], wa[1], wa[2], wa[3]);
            }
            xr[q] = xv;
            wr[q] = wv;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float* xd = &Xs[buf][(t >> 3) + 32 * q][sc];
            float* wd = &Ws[buf][(t >> 3) + 32 * q][sc];
            *reinterpret_cast<float2*>(xd) = make_float2(xr[q].x, xr[q].y);
            *reinterpret_cast<float2*>(xd + 2) = make_float2(xr[q].z, xr[q].w);
            *reinterpret_cast<float2*>(wd) = make_float2(wr[q].x, wr[q].y);
            *reinterpret_cast<float2*>(wd + 2) = make_float2(wr[q].z, wr[q].w);
        }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = zero16();
    load(0);
    store(0);
    __syncthreads();
    for (int kc = 0; kc < nchunks; ++kc) {
        const int buf = kc & 1;
        if (kc + 1 < nchunks) load(kc + 1);
#pragma unroll
        for (int kk = 0; kk < KC; kk += 4) {
            const float2 bx = *reinterpret_cast<const float2*>(&Xs[buf][32 * w + c][kk + 2 * h]);
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const float2 aw = *reinterpret_cast<const float2*>(&Ws[buf][32 * i + c][kk + 2 * h]);
                acc[i] = mfma(aw.x, bx.x, acc[i]);
                acc[i] = mfma(aw.y, bx.y, acc[i]);
            }
        }
        if (kc + 1 < nchunks) store(buf ^ 1);
        __syncthreads();
    }
    // epilogue: bias + tanh; frag layout [row tile][feature tile][lane][16] or row-major
    const int64_t bt = (row0 >> 5) + w;
    const int64_t brow = row0 + 32 * w + c;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * i + rho(r) + 4 * h;
            float z = acc[i][r] + (f < H ? ba[f] : bc[f - H]);
            v[r] = act_tanh ? tanhf(z) : z;
        }
        if (frag_out) {
            float4* o = reinterpret_cast<float4*>(out + ((bt * NT + i) * 64 + l) * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                o[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        } else if (brow < n) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(out + brow * HC + 32 * i + 8 * q + 4 * h) =
                    make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        }
    }
}

// ---------------------------------------------------------------------------------------
// Tail: layers 2-3 + loss + backward to dZ1 + layer-2/3 weight gradients.
// ---------------------------------------------------------------------------------------
struct TailParams {
    float lo, hi, eps_clip, dual, vf_coef, adv_eps;
    int value_clip, norm_adv, use_dual, A;
    float inv_b;
    double inv_b64;
};

constexpr int WS2 = 65;   // LDS row stride of the staged weights (odd: conflict-free reads)
constexpr int SS = 34;    // LDS row stride of the per-wave transpose scratch
// per-workgroup slab of weight-gradient partial sums (floats) and loss partial sums (doubles)
constexpr int SL_W2A = 0, SL_B2A = SL_W2A + H * H, SL_W2C = SL_B2A + H, SL_B2C = SL_W2C + H * H,
              SL_W3A = SL_B2C + H, SL_B3A = SL_W3A + AMAX * H, SL_W3C = SL_B3A + AMAX,
              SL_B3C = SL_W3C + H, SL_F = SL_B3C + 4;
constexpr int SL_D = 4 + AMAX;  // clip, vf, count, 0, d/dlog_std[AMAX]
constexpr int TAIL_TPB = 256;

struct TailWeights {
    const float *w2a, *b2a, *w2c, *b2c, *w3a, *b3a, *w3c, *b3c, *log_std;
};

// Sum of v[16] (one 32-feature tile in C layout) over the 32 lanes of each half-wave.
// Reduce-scatter: afterwards lane l holds the sum of register R(l) = 8*b4+4*b3+2*b2+b1 (the
// lane's bits 4..1) for feature rho(R)+4h; lanes l and l^1 hold the same value.
__device__ __forceinline__ float rs_sum16(const float (&v)[16], int l) {
    float a8[8], a4[4], a2[2];
    const bool b4 = l & 16, b3 = l & 8, b2 = l & 4, b1 = l & 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float keep = b4 ? v[i + 8] : v[i], send = b4 ? v[i] : v[i + 8];
        a8[i] = keep + __shfl_xor(send, 16, 64);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float keep = b3 ? a8[i + 4] : a8[i], send = b3 ? a8[i] : a8[i + 4];
        a4[i] = keep + __shfl_xor(send, 8, 64);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float keep = b2 ? a4[i + 2] : a4[i], send = b2 ? a4[i] : a4[i + 2];
        a2[i] = keep + __shfl_xor(send, 4, 64);
    }
    const float keep = b1 ? a2[1] : a2[0], send = b1 ? a2[0] : a2[1];
    float a1 = keep + __shfl_xor(send, 2, 64);
    return a1 + __shfl_xor(a1, 1, 64);
}
__device__ __forceinline__ int rs_reg(int l) {
    return 8 * ((l >> 4) & 1) + 4 * ((l >> 3) & 1) + 2 * ((l >> 2) & 1) + ((l >> 1) & 1);
}

__global__ __launch_bounds__(TAIL_TPB, 1) void ppo_tail_kernel(
    const float* __restrict__ h1f, int64_t n, const int64_t* __restrict__ idx, TailWeights wt,
    const float* __restrict__ act, const float* __restrict__ logp_old,
    const float* __restrict__ adv, const float* __restrict__ ret, const float* __restrict__ v_s,
    const double* __restrict__ adv_sums, TailParams p, float* __restrict__ dz1,
    float* __restrict__ slab_f, double* __restrict__ slab_d) {
    __shared__ float sW2a[H * WS2], sW2c[H * WS2], sW3a[AMAX * WS2];
    __shared__ float sb2a[H], sb2c[H], sb3a[AMAX], sw3c[H], svar[AMAX], sls[AMAX];
    __shared__ __attribute__((aligned(16))) float scr[4][2][H * SS];
    __shared__ double sred[4][SL_D];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int A = p.A;
    for (int i = t; i < H * H; i += TAIL_TPB) {
        const int o = i / H, f = i - o * H;
        sW2a[o * WS2 + f] = wt.w2a[i];
        sW2c[o * WS2 + f] = wt.w2c[i];
    }
    for (int i = t; i < AMAX * H; i += TAIL_TPB) {
        const int a = i / H, f = i - a * H;
        sW3a[a * WS2 + f] = a < A ? wt.w3a[i] : 0.0f;
    }
    if (t < H) {
        sb2a[t] = wt.b2a[t];
        sb2c[t] = wt.b2c[t];
        sw3c[t] = wt.w3c[t];
    }
    if (t < AMAX) {
        sb3a[t] = t < A ? wt.b3a[t] : 0.0f;
        const float sig = t < A ? expf(wt.log_std[t]) : 1.0f;
        svar[t] = sig * sig;
        sls[t] = logf(sig);
    }
    __syncthreads();
    const float b3c = wt.b3c[0];
    float mean_f = 0.0f, std_f = 1.0f;
    if (p.norm_adv) {
        const double nn = 1.0 / p.inv_b64;
        const double m = adv_sums[0] / nn;
        const double var = (adv_sums[1] - adv_sums[0] * m) / (nn - 1.0);
        mean_f = (float)m;
        std_f = (float)sqrt(var > 0.0 ? var : 0.0);
    }
    float* S1 = scr[w][0];
    float* S2 = scr[w][1];

    // persistent per-wave accumulators
    f32x16 gW2a[2][2], gW2c[2][2], gW3a[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        gW3a[i] = zero16();
#pragma unroll
        for (int j = 0; j < 2; ++j) gW2a[i][j] = gW2c[i][j] = zero16();
    }
    float gb2a[2] = {0.f, 0.f}, gb2c[2] = {0.f, 0.f}, gw3c[2] = {0.f, 0.f};
    float gb3a = 0.f, gb3c = 0.f;
    double dls_acc = 0.0, clip_acc = 0.0, vf_acc = 0.0, cnt_acc = 0.0;

    const int64_t ntiles = (n + 31) / 32;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w, nw = (int64_t)gridDim.x * 4;
    for (int64_t bt = gw; bt < ntiles; bt += nw) {
        const int64_t brow = bt * 32 + c;
        const bool live = brow < n;
        const int64_t j = live ? (idx ? idx[brow] : brow) : 0;
        // ---- H1 tiles (actor 0,1; critic 2,3) ------------------------------------------
        float h1[NT][16];
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const float4* src = reinterpret_cast<const float4*>(h1f + ((bt * NT + i) * 64 + l) * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = src[q];
                h1[i][4 * q] = v.x;
                h1[i][4 * q + 1] = v.y;
                h1[i][4 * q + 2] = v.z;
                h1[i][4 * q + 3] = v.w;
            }
        }
        // ---- layer 2 (both nets) ---------------------------------------------------------
        float h2a[2][16], h2c[2][16];
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
            f32x16 za = zero16(), zc = zero16();
            const float* wa = sW2a + (32 * ot + c) * WS2 + 4 * h;
            const float* wc = sW2c + (32 * ot + c) * WS2 + 4 * h;
#pragma unroll
            for (int it = 0; it < 2; ++it)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    za = mfma(wa[32 * it + rho(r)], h1[it][r], za);
                    zc = mfma(wc[32 * it + rho(r)], h1[2 + it][r], zc);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * ot + rho(r) + 4 * h;
                h2a[ot][r] = tanhf(za[r] + sb2a[f]);
                h2c[ot][r] = tanhf(zc[r] + sb2c[f]);
            }
        }
        // ---- heads ----------------------------------------------------------------------
        f32x16 mu = zero16();
        float vpart = 0.0f;
        {
            const float* wa = sW3a + c * WS2 + 4 * h;
#pragma unroll
            for (int it = 0; it < 2; ++it)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    mu = mfma(wa[32 * it + rho(r)], h2a[it][r], mu);
                    vpart += sw3c[32 * it + rho(r) + 4 * h] * h2c[it][r];
                }
        }
        const float value = vpart + __shfl_xor(vpart, 32, 64) + b3c;
        // ---- loss (both lanes of a row compute the row scalars) -------------------------
        float diff[16];
        float lp = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = rho(r) + 4 * h;
            const float m = mu[r] + sb3a[a];
            diff[r] = 0.0f;
            if (a < A && live) {
                diff[r] = act[j * A + a] - m;
                lp += -(diff[r] * diff[r]) / (2.0f * svar[a]) - sls[a] - LOG_SQRT_2PI;
            }
        }
        const float logp = lp + __shfl_xor(lp, 32, 64);
        float g_logp = 0.0f, gv = 0.0f;
        if (live) {
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
            g_logp = (float)(-(double)dobj * (double)ratio * p.inv_b64);
            const float rt = ret[j];
            float dv, vf;
            if (p.value_clip) {
                const float vs = v_s[j];
                const float dlt = value - vs;
                const float dcl = fminf(fmaxf(dlt, -p.eps_clip), p.eps_clip);
                const float vcl = vs + dcl;
                const float e1 = rt - value, e2 = rt - vcl;
                const float vf1 = e1 * e1, vf2 = e2 * e2;
                const float g1 = -2.0f * e1;
                const float g2 = (dlt >= -p.eps_clip && dlt <= p.eps_clip) ? -2.0f * e2 : 0.0f;
                if (vf1 > vf2) {
                    vf = vf1;
                    dv = g1;
                } else if (vf2 > vf1) {
                    vf = vf2;
                    dv = g2;
                } else {
                    vf = vf1;
                    dv = 0.5f * g1 + 0.5f * g2;
                }
            } else {
                const float e1 = rt - value;
                vf = e1 * e1;
                dv = -2.0f * e1;
            }
            gv = (float)((double)p.vf_coef * (double)dv * p.inv_b64);
            if (h == 0) {
                clip_acc += -(double)obj;
                vf_acc += (double)vf;
                cnt_acc += 1.0;
            }
        }
        // d/d(mu) in C layout (action a = rho(r)+4h), d/d(log_std) partials
        float dmu[16], dls[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = rho(r) + 4 * h;
            const float var = svar[a];
            dmu[r] = g_logp * diff[r] / var;
            dls[r] = (a < A && live) ? g_logp * (diff[r] * diff[r] / var - 1.0f) : 0.0f;
        }
        dls_acc += (double)rs_sum16(dls, l);
        gb3a += rs_sum16(dmu, l);
        {
            float gvh[16];
#pragma unroll
            for (int it = 0; it < 2; ++it) {
#pragma unroll
                for (int r = 0; r < 16; ++r) gvh[r] = gv * h2c[it][r];
                gw3c[it] += rs_sum16(gvh, l);
            }
        }
        {
            float gsum = h == 0 ? gv : 0.0f;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) gsum += __shfl_xor(gsum, off, 64);
            gb3c += gsum;
        }
        // ---- dW3a = dMu^T . H2a   (S1 = dMu^T [a][b], S2 = H2a^T [f][b]) ------------------
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            S1[(rho(r) + 4 * h) * SS + c] = dmu[r];
#pragma unroll
            for (int it = 0; it < 2; ++it) S2[(32 * it + rho(r) + 4 * h) * SS + c] = h2a[it][r];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float2 a2 = *reinterpret_cast<const float2*>(&S1[c * SS + 4 * s + 2 * h]);
#pragma unroll
            for (int ft = 0; ft < 2; ++ft) {
                const float2 b2 = *reinterpret_cast<const float2*>(&S2[(32 * ft + c) * SS + 4 * s + 2 * h]);
                gW3a[ft] = mfma(a2.x, b2.x, gW3a[ft]);
                gW3a[ft] = mfma(a2.y, b2.y, gW3a[ft]);
            }
        }
        // ---- dZ2 (actor: W3a^T dMu, critic: gv w3c) ---------------------------------------
        float dz2a[2][16], dz2c[2][16];
#pragma unroll
        for (int ft = 0; ft < 2; ++ft) {
            f32x16 d = zero16();
#pragma unroll
            for (int r = 0; r < 16; ++r)
                d = mfma(sW3a[(rho(r) + 4 * h) * WS2 + 32 * ft + c], dmu[r], d);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * ft + rho(r) + 4 * h;
                dz2a[ft][r] = d[r] * (1.0f - h2a[ft][r] * h2a[ft][r]);
                dz2c[ft][r] = gv * sw3c[f] * (1.0f - h2c[ft][r] * h2c[ft][r]);
            }
        }
        // ---- per net: dZ1 = (W2^T dZ2) * (1 - H1^2), dW2 = dZ2^T H1, db2 -----------------
#pragma unroll
        for (int net = 0; net < 2; ++net) {
            const float* sW2 = net ? sW2c : sW2a;
            float (&dz2)[2][16] = net ? dz2c : dz2a;
#pragma unroll
            for (int ft = 0; ft < 2; ++ft) {
                f32x16 d = zero16();
#pragma unroll
                for (int ot = 0; ot < 2; ++ot)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        d = mfma(sW2[(32 * ot + rho(r) + 4 * h) * WS2 + 32 * ft + c], dz2[ot][r], d);
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float hv = h1[2 * net + ft][r];
                    v[r] = live ? d[r] * (1.0f - hv * hv) : 0.0f;
                }
                if (live) {
                    float* o = dz1 + brow * HC + 64 * net + 32 * ft + 4 * h;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *reinterpret_cast<float4*>(o + 8 * q) =
                            make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
                }
            }
            // db2
#pragma unroll
            for (int ot = 0; ot < 2; ++ot) {
                const float s = rs_sum16(dz2[ot], l);
                if (net) gb2c[ot] += s; else gb2a[ot] += s;
            }
            // dW2 via LDS transposes (S1 = dZ2^T [o][b], S2 = H1^T [f][b])
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int it = 0; it < 2; ++it) {
                    S1[(32 * it + rho(r) + 4 * h) * SS + c] = dz2[it][r];
                    S2[(32 * it + rho(r) + 4 * h) * SS + c] = h1[2 * net + it][r];
                }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                float2 a2[2], b2[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    a2[i] = *reinterpret_cast<const float2*>(&S1[(32 * i + c) * SS + 4 * s + 2 * h]);
                    b2[i] = *reinterpret_cast<const float2*>(&S2[(32 * i + c) * SS + 4 * s + 2 * h]);
                }
#pragma unroll
                for (int ot = 0; ot < 2; ++ot)
#pragma unroll
                    for (int ft = 0; ft < 2; ++ft) {
                        f32x16& g = net ? gW2c[ot][ft] : gW2a[ot][ft];
                        g = mfma(a2[ot].x, b2[ft].x, g);
                        g = mfma(a2[ot].y, b2[ft].y, g);
                    }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
    }
    // ---- fold the 4 waves' accumulators (fixed order) into this workgroup's slab -------
    __syncthreads();
    float* red = &scr[0][0][0];  // 4 * 2 * H * SS floats >= 4 * H * H
    float* slab = slab_f + (int64_t)blockIdx.x * SL_F;
    auto fold_tile = [&](const f32x16 (&g)[2][2], int base, int rows) {
        // wave w writes its [o][f] matrix (C layout: o = 32ot+rho(r)+4h, f = 32ft+c)
#pragma unroll
        for (int ot = 0; ot < 2; ++ot)
#pragma unroll
            for (int ft = 0; ft < 2; ++ft)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int o = 32 * ot + rho(r) + 4 * h;
                    if (o < rows) red[w * H * H + o * H + 32 * ft + c] = g[ot][ft][r];
                }
        __syncthreads();
        for (int i = t; i < rows * H; i += TAIL_TPB)
            slab[base + i] = ((red[i] + red[H * H + i]) + red[2 * H * H + i]) + red[3 * H * H + i];
        __syncthreads();
    };
    fold_tile(gW2a, SL_W2A, H);
    fold_tile(gW2c, SL_W2C, H);
    {
        f32x16 g3[2][2] = {{gW3a[0], gW3a[1]}, {zero16(), zero16()}};
        fold_tile(g3, SL_W3A, AMAX);
    }
    // vectors: lanes with bit0 == 0 own feature rho(rs_reg(l)) + 4h of each tile
    float* vred = red;  // [4 waves][SL_F - SL_B2A region], reuse
    const int fr = rho(rs_reg(l)) + 4 * h;
    constexpr int VW = 4 * H + AMAX + 4;  // b2a, b2c, w3c(H) ... packed per wave
    if ((l & 1) == 0) {
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            vred[w * VW + 32 * it + fr] = gb2a[it];
            vred[w * VW + H + 32 * it + fr] = gb2c[it];
            vred[w * VW + 2 * H + 32 * it + fr] = gw3c[it];
        }
        vred[w * VW + 3 * H + fr] = gb3a;
    }
    if (l == 0) vred[w * VW + 3 * H + AMAX] = gb3c;
    __syncthreads();
    if (t < VW) {
        const float s = ((vred[t] + vred[VW + t]) + vred[2 * VW + t]) + vred[3 * VW + t];
        if (t < H) slab[SL_B2A + t] = s;
        else if (t < 2 * H) slab[SL_B2C + t - H] = s;
        else if (t < 3 * H) slab[SL_W3C + t - 2 * H] = s;
        else if (t < 3 * H + AMAX) slab[SL_B3A + t - 3 * H] = s;
        else if (t == 3 * H + AMAX) slab[SL_B3C] = s;
    }
    // doubles: loss sums (wave reduce) and d/dlog_std
    clip_acc = wave_sum(clip_acc);
    vf_acc = wave_sum(vf_acc);
    cnt_acc = wave_sum(cnt_acc);
    if ((l & 1) == 0) sred[w][4 + fr] = dls_acc;
    if (l == 0) {
        sred[w][0] = clip_acc;
        sred[w][1] = vf_acc;
        sred[w][2] = cnt_acc;
        sred[w][3] = 0.0;
    }
    __syncthreads();
    if (t < SL_D)
        slab_d[(int64_t)blockIdx.x * SL_D + t] =
            ((sred[0][t] + sred[1][t]) + sred[2][t]) + sred[3][t];
}

// Folds the per-workgroup slabs (fixed order) into the parameter gradients and the loss sums.
struct TailGrads {
    float *w2a, *b2a, *w2c, *b2c, *w3a, *b3a, *w3c, *b3c;
};

__global__ __launch_bounds__(256) void tail_reduce_kernel(const float* __restrict__ slab_f,
                                                          const double* __restrict__ slab_d,
                                                          int nslab, int A, TailGrads g,
                                                          double* __restrict__ sums) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < SL_F) {
        float s = 0.0f;
        for (int k = 0; k < nslab; ++k) s += slab_f[(int64_t)k * SL_F + i];
        if (i < SL_B2A) g.w2a[i] = s;
        else if (i < SL_W2C) g.b2a[i - SL_B2A] = s;
        else if (i < SL_B2C) g.w2c[i - SL_W2C] = s;
        else if (i < SL_W3A) g.b2c[i - SL_B2C] = s;
        else if (i < SL_B3A) { if (i - SL_W3A < A * H) g.w3a[i - SL_W3A] = s; }
        else if (i < SL_W3C) { if (i - SL_B3A < A) g.b3a[i - SL_B3A] = s; }
        else if (i < SL_B3C) g.w3c[i - SL_W3C] = s;
        else if (i == SL_B3C) g.b3c[0] = s;
    } else if (i < SL_F + SL_D) {
        const int k0 = i - SL_F;
        double s = 0.0;
        for (int k = 0; k < nslab; ++k) s += slab_d[(int64_t)k * SL_D + k0];
        if (k0 < 4 + A) sums[k0] = s;
    }
}

// ---------------------------------------------------------------------------------------
// dW1cat = dZ1^T . X[idx] and db1 (ones column at k = D), split over minibatch rows.
// Workgroup = 128 features x 128 input columns x one row range; wave w owns columns
// [32w, 32w+32) for all 4 feature tiles.  Rows are staged 32 at a time through LDS.
// ---------------------------------------------------------------------------------------
constexpr int DW_COLS = 128;
constexpr int DW_KB = 32;

__global__ __launch_bounds__(256, 2) void dw_kernel(
    const float* __restrict__ dz, const float* __restrict__ X, int64_t ldx,
    const int64_t* __restrict__ idx, int64_t n, int D, int64_t rows_per_split,
    int ncolpad, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float Zs[2][DW_KB][HC];
    __shared__ __attribute__((aligned(16))) float Xs[2][DW_KB][DW_COLS];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int col0 = blockIdx.x * DW_COLS;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
    const int64_t r1 = min(n, r0 + rows_per_split);
    // staging: thread t moves float4 (t & 31) of rows (t >> 5) + 8q, q = 0..3
    const int sc = 4 * (t & 31);
    float4 zr[4], xr[4];
    auto load = [&](int64_t rb) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t r = rb + (t >> 5) + 8 * q;
            float4 zv = make_float4(0.f, 0.f, 0.f, 0.f), xv = zv;
            if (r < r1) {
                zv = *reinterpret_cast<const float4*>(dz + r * HC + sc);
                const float* xrow = X + (idx ? idx[r] : r) * ldx;
                const int k = col0 + sc;
                if (k + 3 < D) {
                    xv = *reinterpret_cast<const float4*>(xrow + k);
                } else {
                    float xa[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        xa[e] = k + e < D ? xrow[k + e] : (k + e == D ? 1.0f : 0.0f);
                    xv = make_float4(xa[0], xa[1], xa[2], xa[3]);
                }
            }
            zr[q] = zv;
            xr[q] = xv;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            *reinterpret_cast<float4*>(&Zs[buf][(t >> 5) + 8 * q][sc]) = zr[q];
            *reinterpret_cast<float4*>(&Xs[buf][(t >> 5) + 8 * q][sc]) = xr[q];
        }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = zero16();
    const int64_t nchunk = r1 > r0 ? (r1 - r0 + DW_KB - 1) / DW_KB : 0;
    if (nchunk > 0) {
        load(r0);
        store(0);
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunk; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < nchunk) load(r0 + (ch + 1) * DW_KB);
#pragma unroll
        for (int s = 0; s < DW_KB / 2; ++s) {
            const float b = Xs[buf][2 * s + h][32 * w + c];
#pragma unroll
            for (int i = 0; i < NT; ++i) acc[i] = mfma(Zs[buf][2 * s + h][32 * i + c], b, acc[i]);
        }
        if (ch + 1 < nchunk) store(buf ^ 1);
        __syncthreads();
    }
    // partial [split][f][colpad]
    float* o = part + (int64_t)blockIdx.y * HC * ncolpad;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            o[(int64_t)(32 * i + rho(r) + 4 * h) * ncolpad + col0 + 32 * w + c] = acc[i][r];
}

__global__ __launch_bounds__(256) void dw_reduce_kernel(const float* __restrict__ part,
                                                        int nsplit, int ncolpad, int D,
                                                        float* __restrict__ gWa,
                                                        float* __restrict__ gba,
                                                        float* __restrict__ gWc,
                                                        float* __restrict__ gbc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)HC * ncolpad) return;
    const int f = (int)(i / ncolpad), k = (int)(i - (int64_t)f * ncolpad);
    if (k > D) return;
    float s = 0.0f;
    for (int sp = 0; sp < nsplit; ++sp) s += part[(int64_t)sp * HC * ncolpad + i];
    if (k == D) {
        if (f < H) gba[f] = s; else gbc[f - H] = s;
    } else {
        if (f < H) gWa[(int64_t)f * D + k] = s; else gWc[(int64_t)(f - H) * D + k] = s;
    }
}

TailParams make_tail_params(const tsrl_ppo_params& q, int A) {
    TailParams p;
    p.lo = (float)(1.0 - q.eps_clip);
    p.hi = (float)(1.0 + q.eps_clip);
    p.eps_clip = (float)q.eps_clip;
    p.dual = (float)q.dual_clip;
    p.use_dual = q.dual_clip > 0.0;
    p.vf_coef = (float)q.vf_coef;
    p.adv_eps = (float)q.adv_eps;
    p.value_clip = q.value_clip;
    p.norm_adv = q.norm_adv;
    p.A = A;
    p.inv_b = (float)(1.0 / q.b_global);
    p.inv_b64 = 1.0 / q.b_global;
    return p;
}

int tail_grid(int64_t n) {
    const int64_t tiles = (n + 31) / 32;
    const int64_t g = (tiles + 3) / 4;
    return (int)std::min<int64_t>(g, 256);
}

int dw_nsplit(int64_t n) {
    // ~512 resident workgroups on 256 CUs (3 column tiles at D=376), >= 64 rows per split
    int64_t s = std::max<int64_t>(1, std::min<int64_t>(170, n / 64));
    return (int)s;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_mlp_l1_fwd(const float* X, int64_t ldx, const int64_t* idx, int64_t n,
                               int64_t D, const float* Wa, const float* ba, const float* Wc,
                               const float* bc, int act_tanh, float* out, int frag_out,
                               void* stream) {
    TSRL_CHECK_ARG(n >= 0 && D > 0 && ldx >= D, "tsrl_mlp_l1_fwd: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(X && Wa && ba && Wc && bc && out, "tsrl_mlp_l1_fwd: null pointer");
    TSRL_CHECK_ARG(aligned16(X) && ldx % 4 == 0 && aligned16(Wa) && aligned16(Wc) && D % 4 == 0 &&
                       aligned16(out),
                   "tsrl_mlp_l1_fwd: X/W/out must be 16-byte aligned with D, ldx multiples of 4");
    const unsigned grid = (unsigned)((n + L1_ROWS - 1) / L1_ROWS);
    hipLaunchKernelGGL(l1_fwd_kernel, dim3(grid), dim3(256), 0, as_stream(stream), X, ldx, idx, n,
                       (int)D, Wa, ba, Wc, bc, act_tanh, out, frag_out);
    TSRL_LAUNCH_CHECK("tsrl_mlp_l1_fwd");
    return 0;
}

extern "C" int64_t tsrl_mlp_frag_floats(int64_t n) {
    return ((n + L1_ROWS - 1) / L1_ROWS) * L1_ROWS * HC;
}

extern "C" int64_t tsrl_ppo_tail_workspace_bytes(int64_t n) {
    const int g = tail_grid(n);
    return (int64_t)g * (SL_F * (int64_t)sizeof(float) + SL_D * (int64_t)sizeof(double)) + 256;
}

extern "C" int tsrl_ppo_tail(const float* h1frag, int64_t n, const int64_t* idx,
                             const tsrl_tail_weights* wt, int64_t act_dim, const float* act,
                             const float* logp_old, const float* adv, const float* ret,
                             const float* v_s, const double* adv_sums, tsrl_ppo_params prm,
                             float* dz1, const tsrl_tail_grads* grads, double* sums,
                             void* workspace, int64_t ws_bytes, void* stream) {
    TSRL_CHECK_ARG(n > 0 && act_dim > 0 && act_dim <= AMAX,
                   "tsrl_ppo_tail: need n > 0 and 0 < act_dim <= %d", AMAX);
    TSRL_CHECK_ARG(h1frag && wt && grads && act && logp_old && adv && ret && dz1 && sums &&
                       workspace,
                   "tsrl_ppo_tail: null pointer");
    TSRL_CHECK_ARG(!prm.value_clip || v_s, "tsrl_ppo_tail: value_clip needs v_s");
    TSRL_CHECK_ARG(!prm.norm_adv || adv_sums, "tsrl_ppo_tail: norm_adv needs adv_sums");
    TSRL_CHECK_ARG(prm.b_global >= 1.0, "tsrl_ppo_tail: b_global < 1");
    TSRL_CHECK_ARG(ws_bytes >= tsrl_ppo_tail_workspace_bytes(n), "tsrl_ppo_tail: workspace too small");
    TSRL_CHECK_ARG(aligned16(h1frag) && aligned16(dz1), "tsrl_ppo_tail: h1frag/dz1 not 16-byte aligned");
    const int g = tail_grid(n);
    float* slab_f = reinterpret_cast<float*>(workspace);
    uintptr_t dptr = reinterpret_cast<uintptr_t>(slab_f + (int64_t)g * SL_F);
    dptr = (dptr + 15) & ~(uintptr_t)15;
    double* slab_d = reinterpret_cast<double*>(dptr);
    TailWeights w{wt->w2a, wt->b2a, wt->w2c, wt->b2c, wt->w3a, wt->b3a, wt->w3c, wt->b3c,
                  wt->log_std};
    hipLaunchKernelGGL(ppo_tail_kernel, dim3(g), dim3(TAIL_TPB), 0, as_stream(stream), h1frag, n,
                       idx, w, act, logp_old, adv, ret, v_s, adv_sums,
                       make_tail_params(prm, (int)act_dim), dz1, slab_f, slab_d);
    TSRL_LAUNCH_CHECK("tsrl_ppo_tail");
    TailGrads gg{grads->w2a, grads->b2a, grads->w2c, grads->b2c, grads->w3a, grads->b3a,
                 grads->w3c, grads->b3c};
    hipLaunchKernelGGL(tail_reduce_kernel, dim3((SL_F + SL_D + 255) / 256), dim3(256), 0,
                       as_stream(stream), slab_f, slab_d, g, (int)act_dim, gg, sums);
    TSRL_LAUNCH_CHECK("tsrl_ppo_tail(reduce)");
    return 0;
}

extern "C" int64_t tsrl_mlp_dw_workspace_bytes(int64_t n, int64_t D) {
    const int ncolpad = (int)(((D + 1 + DW_COLS - 1) / DW_COLS) * DW_COLS);
    return (int64_t)dw_nsplit(n) * HC * ncolpad * (int64_t)sizeof(float);
}

extern "C" int tsrl_mlp_dw(const float* dz1, const float* X, int64_t ldx, const int64_t* idx,
                           int64_t n, int64_t D, float* gWa, float* gba, float* gWc, float* gbc,
                           void* workspace, int64_t ws_bytes, void* stream) {
    TSRL_CHECK_ARG(n > 0 && D > 0 && ldx >= D, "tsrl_mlp_dw: bad sizes");
    TSRL_CHECK_ARG(dz1 && X && gWa && gba && gWc && gbc && workspace, "tsrl_mlp_dw: null pointer");
    TSRL_CHECK_ARG(aligned16(dz1) && aligned16(X) && ldx % 4 == 0,
                   "tsrl_mlp_dw: dz1/X must be 16-byte aligned, ldx a multiple of 4");
    TSRL_CHECK_ARG(ws_bytes >= tsrl_mlp_dw_workspace_bytes(n, D), "tsrl_mlp_dw: workspace too small");
    const int ncolt = (int)((D + 1 + DW_COLS - 1) / DW_COLS);
    const int ncolpad = ncolt * DW_COLS;
    const int nsplit = dw_nsplit(n);
    const int64_t rps = ((n + nsplit - 1) / nsplit + DW_KB - 1) / DW_KB * DW_KB;
    float* part = reinterpret_cast<float*>(workspace);
    hipLaunchKernelGGL(dw_kernel, dim3(ncolt, nsplit), dim3(256), 0, as_stream(stream), dz1, X, ldx,
                       idx, n, (int)D, rps, ncolpad, part);
    TSRL_LAUNCH_CHECK("tsrl_mlp_dw");
    const int64_t outs = (int64_t)HC * ncolpad;
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((outs + 255) / 256)), dim3(256), 0,
                       as_stream(stream), part, nsplit, ncolpad, (int)D, gWa, gba, gWc, gbc);
    TSRL_LAUNCH_CHECK("tsrl_mlp_dw(reduce)");
    return 0;
}
