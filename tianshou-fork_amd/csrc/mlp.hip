// Fused actor/critic MLP kernels for the PPO minibatch (PPOPolicy.learn, tianshou/policy/
// modelfree/ppo.py:106-151) on the MuJoCo network shape of tianshou/utils/models.py:34-97:
// actor  = Linear(D,64)-Tanh-Linear(64,64)-Tanh-Linear(64,A)      (ActorProb, unbounded)
// critic = Linear(D,64)-Tanh-Linear(64,64)-Tanh-Linear(64,1)      (Critic)
// with the state-independent log-std of fixed_std_normal.
//
// Kernels of a minibatch (the production path runs the bf16x6 forms: exact three-way bf16
// splits of every f32 operand, x6.h; l1_fwd_kernel is the f32-input MFMA reference form):
//   l1_fwd_kernel / l1_ring_kernel (mlp_x6.hip): H1^T = tanh(W1cat . X[idx]^T + b1) for both nets at once (W1cat = the
//                   two first-layer weights stacked, 128 features).  Minibatch rows are read
//                   through the permutation index (no gathered copy of the observations).
//   ppo_tail_kernel: layers 2-3 of both nets, the clipped-surrogate/value loss and its
//                   backward down to dZ1, plus the weight gradients of layers 2-3, per wave
//                   of 32 minibatch rows, without leaving registers/LDS.
//   dw_x6_kernel  : dW1cat = dZ1^T . X[idx] (+ db1 through a ones column), split over the
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
#include "x6.h"

namespace tsrl {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
using x6::bf16x8;
using x6::mfma6;
using x6::NPL;
using x6::split1;
using x6::sw_off;

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
    __shared__ float sb[HC];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int64_t row0 = (int64_t)blockIdx.x * L1_ROWS;
    if (t < HC) sb[t] = t < H ? ba[t] : bc[t - H];
    // staging assignment: thread t moves float4 column (t&7) of rows (t>>3) + 32q.  Dead
    // rows read row 0 and are zeroed (branch-free loads; D % 4 == 0 so a float4 is either
    // wholly inside the row or wholly past its end).
    const int sc = 4 * (t & 7);
    const float* xsrc[4];
    const float* wsrc[4];
    bool xlive[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t r = row0 + (t >> 3) + 32 * q;
        xlive[q] = r < n;
        xsrc[q] = X + (xlive[q] ? (idx ? idx[r] : r) : 0) * ldx;
        const int f = (t >> 3) + 32 * q;
        wsrc[q] = f < H ? Wa + (int64_t)f * D : Wc + (int64_t)(f - H) * D;
    }
    const int nchunks = (D + KC - 1) / KC;
    float4 xr[4], wr[4];
    bool kin_ld = true;
    // loads go straight to registers; the masks are applied when the registers are
    // written to LDS (after the MFMA phase), so no wait sits between the loads
    auto load = [&](int kc) {
        const int k = kc * KC + sc;
        kin_ld = k < D;
        const int kk = kin_ld ? k : 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            xr[q] = *reinterpret_cast<const float4*>(xsrc[q] + kk);
            wr[q] = *reinterpret_cast<const float4*>(wsrc[q] + kk);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool xo = kin_ld && xlive[q];
            float* xd = &Xs[buf][(t >> 3) + 32 * q][sc];
            float* wd = &Ws[buf][(t >> 3) + 32 * q][sc];
            *reinterpret_cast<float2*>(xd) =
                make_float2(xo ? xr[q].x : 0.f, xo ? xr[q].y : 0.f);
            *reinterpret_cast<float2*>(xd + 2) =
                make_float2(xo ? xr[q].z : 0.f, xo ? xr[q].w : 0.f);
            *reinterpret_cast<float2*>(wd) =
                make_float2(kin_ld ? wr[q].x : 0.f, kin_ld ? wr[q].y : 0.f);
            *reinterpret_cast<float2*>(wd + 2) =
                make_float2(kin_ld ? wr[q].z : 0.f, kin_ld ? wr[q].w : 0.f);
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
    // epilogue: bias + tanh; fragment layout (x6::frag_off4) or row-major
    const int64_t bt = (row0 >> 5) + w;
    const int64_t brow = row0 + 32 * w + c;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * i + rho(r) + 4 * h;
            float z = acc[i][r] + sb[f];
            v[r] = act_tanh ? tanh_nb(z) : z;
        }
        if (frag_out) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(out + x6::frag_off4(bt * NT + i, l, q)) =
                    make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
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

// per-workgroup slab of weight-gradient partial sums (floats) and loss partial sums (doubles)
constexpr int SL_W2A = 0, SL_B2A = SL_W2A + H * H, SL_W2C = SL_B2A + H, SL_B2C = SL_W2C + H * H,
              SL_W3A = SL_B2C + H, SL_B3A = SL_W3A + AMAX * H, SL_W3C = SL_B3A + AMAX,
              SL_B3C = SL_W3C + H, SL_F = SL_B3C + 4;
constexpr int SL_D = 4 + AMAX;  // clip, vf, count, 0, d/dlog_std[AMAX]
struct TailWeights {
    const float *w2a, *b2a, *w2c, *b2c, *w3a, *b3a, *w3c, *b3c, *log_std;
};

// The actor (NET 0: layer 2, mu head, clipped surrogate, backward) and the critic (NET 1:
// layer 2, value head, value loss, backward) run as two launches: the loss gradient w.r.t.
// mu depends only on actor outputs and w.r.t. the value only on critic outputs.
// Feature-major weight-gradient scratch [feature][16 rows]: stride 20 floats (80 B) keeps the
// 8-row float4 reads of the bf16x6 weight gradients 16-byte aligned and spreads the 16 lanes
// of a read phase over all 16 bank groups (5 is odd).
constexpr int SH = 20;

// 32-row images (process_fn's eval_tail_kernel): the chain products (layer 2, mu head) run as
// bf16x6 (x6.h): their activation operand is the C-layout tile itself -- registers 8s..8s+7 of a 32x32 tile
// are the 8 k of k-step s on each lane half, element j of half h being feature
// 16s + 8(j>>2) + 4h + (j&3) of the tile -- split in registers, and the weight operand is an
// LDS image of the matrix, split once per workgroup into 3 bf16 planes whose rows hold the
// k in exactly that order.  Image of an [rows][32*nkc] matrix: plane p, 32-k chunk kc, row r
// at byte ((p*nkc + kc)*rows)*64 + sw_off(r, q), q = 2s + h the 16-byte chunk of (s, h).

__device__ __forceinline__ int img_off(int p, int kc, int row, int q, int nkc, int rows) {
    return (p * nkc + kc) * rows * 64 + sw_off(row, q);
}

// Split M(row, k) (k < 32*nkc) into the image; every thread writes whole 16-byte chunks.
template <int TPB, typename F>
__device__ __forceinline__ void build_img_n(char* img, int rows, int nkc, F val) {
    for (int i = threadIdx.x; i < rows * nkc * 4; i += TPB) {
        const int q = i & 3, kc = (i >> 2) % nkc, row = (i >> 2) / nkc;
        bf16x8 p0, p1, p2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 32 * kc + 16 * (q >> 1) + 8 * (j >> 2) + 4 * (q & 1) + (j & 3);
            __bf16 a, b, c;
            split1(val(row, k), a, b, c);
            p0[j] = a;
            p1[j] = b;
            p2[j] = c;
        }
        *reinterpret_cast<bf16x8*>(img + img_off(0, kc, row, q, nkc, rows)) = p0;
        *reinterpret_cast<bf16x8*>(img + img_off(1, kc, row, q, nkc, rows)) = p1;
        *reinterpret_cast<bf16x8*>(img + img_off(2, kc, row, q, nkc, rows)) = p2;
    }
}


// The 3 planes of one operand fragment: row `row`, 32-k chunk kc, k-step s, lane half h.
__device__ __forceinline__ void ld_img(const char* img, int nkc, int rows, int kc, int row,
                                       int s, int h, bf16x8 (&a)[NPL]) {
#pragma unroll
    for (int p = 0; p < NPL; ++p)
        a[p] = *reinterpret_cast<const bf16x8*>(img + img_off(p, kc, row, 2 * s + h, nkc, rows));
}

// B fragment of k-step s from registers 8s..8s+7 of a C-layout tile, split in registers.
__device__ __forceinline__ void split_frag(const float (&v)[16], int s, bf16x8 (&b)[NPL]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 x0, x1, x2;
        split1(v[8 * s + j], x0, x1, x2);
        b[0][j] = x0;
        b[1][j] = x1;
        b[2][j] = x2;
    }
}

// Accumulate D += A^T-in-LDS . B^T-in-LDS over 16 minibatch rows, bf16x6: one 16-deep k-step of v_mfma_f32_32x32x16_bf16 covers the 16
// rows; lane (c, h) reads rows 8h..8h+7 of feature c of each tile (two float4 reads) and
// splits them into the three planes in registers.  Both operands were written feature-major
// ([feature][row], stride SH) from the C layout; tiles ot x ft.
template <int NOT, int NFT>
__device__ __forceinline__ void acc_wgrad_x6(f32x16 (&g)[NOT][NFT], const float* S1,
                                             const float* S2, int c, int h) {
    bf16x8 b[NFT][NPL];
    auto ld8 = [&](const float* S, int tile, bf16x8 (&p)[NPL]) {
        const float4* src = reinterpret_cast<const float4*>(&S[(32 * tile + c) * SH + 8 * h]);
        const float4 u = src[0], v = src[1];
        const float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            __bf16 x0, x1, x2;
            split1(e[j], x0, x1, x2);
            p[0][j] = x0;
            p[1][j] = x1;
            p[2][j] = x2;
        }
    };
#pragma unroll
    for (int i = 0; i < NFT; ++i) ld8(S2, i, b[i]);
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
        bf16x8 a[NPL];
        ld8(S1, ot, a);
#pragma unroll
        for (int ft = 0; ft < NFT; ++ft) g[ot][ft] = mfma6(a, b[ft], g[ot][ft]);
    }
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------
// ppo_tail16_kernel: layers 2-3 of one net, the clipped-surrogate / value loss, the backward
// down to dZ1 and the layer-2/3 weight gradients, on 16-row tiles at TWO waves per SIMD.
// Round 5 replaced the round-2..4 32-row kernel, which ran one wave per SIMD (505 / 384
// VGPR+AGPR): its waves issued 54-56 % of their cycles and waited on their own dependent
// MFMA -> tanh -> MFMA chains the rest (profiles/r03_learn_sq_pmc.txt), and a quarter of its
// vector instructions moved values between VGPRs and AGPRs.  Here a wave owns 16 minibatch
// rows at a time: the chain products run on v_mfma_f32_16x16x32_bf16 (bf16x6, 16 cycles
// each, the same matrix-core time per row), so the per-tile activations take half the
// registers and the kernel fits 256 (8 waves per workgroup, one workgroup per CU, the weight
// images shared by all 8; no AGPR moves).  The weight gradients accumulate per wave on
// v_mfma_f32_32x32x16_bf16 over the tile's 16 rows (acc_wgrad_x6, one K step).  Measured
// (tools/mlp_kernel_bench.py --only tail, both nets + reduce, 262144 rows, A/B in one call,
// profiles/r05_tail16_ab.log): 188-197 vs 210-222 us for the 32-row kernel.
//
// Layouts (lane l: row b = l & 15 of the tile, lane group g = l >> 4):
//   H1: the 16 layer-1 features Fh1(g, r) = 32 (g >> 1) + rho(r) + 4 (g & 1), r = 0..15 --
//       one 64-byte run of the layer-1 kernel's 32x32 fragment (tile 2 net + (g >> 1), lane
//       (16 half + b) + 32 (g & 1)), so the load is four float4 reads;
//   16x16 C tiles (layer 2, heads, dZ2, dZ1): lane (b, g) holds rows 4g + r, r = 0..3, of
//       the tile's 16 features, column b;
//   B operands come straight from those registers: K chunk kc of a 64-feature activation is
//       register set 8 kc .. 8 kc + 7 (H1) or C tiles 2 kc, 2 kc + 1 (H2, dZ2), each lane
//       group supplying its own 8 k; the weight images hold the matching permuted k.
// Image of a [NTILE x 16 rows][NKC x 32 k] operand: plane p, tile, chunk kc, row i, group g
// -> 16 bytes at ((p NTILE + tile) NKC + kc) 1024 + 16 (16 g + i), the 8 bf16 k = 8 g + j:
// lane l = 16 g + i reads the chunk at + 16 l, 64 lanes, 1 KB contiguous, no bank conflicts.
// ---------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int T16_NW = 8;               // waves per workgroup (2 per SIMD)
constexpr int T16_TPB = 64 * T16_NW;

__device__ __forceinline__ int fh1(int g, int r) { return 32 * (g >> 1) + rho(r) + 4 * (g & 1); }
// feature of register (tile t, r) of a 16x16 C tile held by lane group g
__device__ __forceinline__ int fc16(int g, int t, int r) { return 16 * t + 4 * g + r; }
// k slot j of chunk kc of a B operand built from C tiles 2 kc, 2 kc + 1
__device__ __forceinline__ int fb16(int g, int kc, int j) { return fc16(g, 2 * kc + (j >> 2), j & 3); }

__device__ __forceinline__ f32x4 zero4() {
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    return z;
}

__device__ __forceinline__ f32x4 mfma6_16(const bf16x8 (&a)[NPL], const bf16x8 (&b)[NPL],
                                          f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
    return acc;
}

// Split an image: val(tile, kc, i, g, j) for tiles x nkc chunks; each thread writes whole
// 16-byte chunks of the three planes.
template <typename F>
__device__ __forceinline__ void build_img16(char* img, int ntile, int nkc, F val) {
    const int total = ntile * nkc * 64;
    for (int q = threadIdx.x; q < total; q += T16_TPB) {
        const int g = q & 3, i = (q >> 2) & 15, kc = (q >> 6) % nkc, tile = (q >> 6) / nkc;
        bf16x8 p0, p1, p2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            __bf16 a, b, c;
            split1(val(tile, kc, i, g, j), a, b, c);
            p0[j] = a;
            p1[j] = b;
            p2[j] = c;
        }
        const int off = (tile * nkc + kc) * 1024 + 16 * (16 * g + i);  // lane 16 g + i
        const int pl = ntile * nkc * 1024;
        *reinterpret_cast<bf16x8*>(img + off) = p0;
        *reinterpret_cast<bf16x8*>(img + pl + off) = p1;
        *reinterpret_cast<bf16x8*>(img + 2 * pl + off) = p2;
    }
}

__device__ __forceinline__ void ld_img16(const char* img, int ntile, int nkc, int tile, int kc,
                                         int l, bf16x8 (&a)[NPL]) {
    const int pl = ntile * nkc * 1024, off = (tile * nkc + kc) * 1024 + 16 * l;
#pragma unroll
    for (int p = 0; p < NPL; ++p) a[p] = *reinterpret_cast<const bf16x8*>(img + p * pl + off);
}

// B operand: 8 values split into the three planes
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&b)[NPL]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 x0, x1, x2;
        split1(v[j], x0, x1, x2);
        b[0][j] = x0;
        b[1][j] = x1;
        b[2][j] = x2;
    }
}

// Feature-major scratch [feature][16 rows] (stride SH) from 16 registers whose features are
// feat(reg): lane (b, g) writes column b.
template <int NV, typename F>
__device__ __forceinline__ void put16(float* S, const float (&v)[NV], int b, F feat) {
#pragma unroll
    for (int r = 0; r < NV; ++r) S[feat(r) * SH + b] = v[r];
}

// Sum of the 16 row values of scratch row S[0 .. 16) (fixed order).
__device__ __forceinline__ float rowsum16(const float* S) {
    const float4* q = reinterpret_cast<const float4*>(S);
    const float4 a = q[0], b = q[1], c = q[2], d = q[3];
    return ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w)) +
           (((c.x + c.y) + (c.z + c.w)) + ((d.x + d.y) + (d.z + d.w)));
}

constexpr int I16_W2 = 0;                          // W2: [4 out tiles][2 kc]
constexpr int I16_W2T = I16_W2 + NPL * 8 * 1024;   // W2^T: [4 f tiles][2 kc]
constexpr int I16_W3 = I16_W2T + NPL * 8 * 1024;   // W3: [2 a tiles][2 kc] (actor)
constexpr int I16_W3T = I16_W3 + NPL * 4 * 1024;   // W3^T: [4 out tiles][1 kc] (actor)
constexpr int I16_ACTOR = I16_W3T + NPL * 4 * 1024, I16_CRITIC = I16_W3;
// per-wave scratch: S1, S2 [64 features][SH]; reused by the final folds
constexpr int T16_SCR = T16_NW * 2 * H * SH;
static_assert(T16_SCR >= T16_NW * 32 * H, "fold scratch");
static_assert(T16_SCR >= T16_NW * 64 * 18, "vector fold scratch");
constexpr int T16_B2 = 0, T16_B3 = T16_B2 + H, T16_W3C = T16_B3 + AMAX,
              T16_LS = T16_W3C + H, T16_IV = T16_LS + AMAX, T16_IV2 = T16_IV + AMAX,
              T16_VEND = T16_IV2 + AMAX;

template <int NET>
__global__ __launch_bounds__(T16_TPB, 1) void ppo_tail16_kernel(
    const float* __restrict__ h1f, int64_t n, const int64_t* __restrict__ idx, TailWeights wt,
    const float* __restrict__ act, const float* __restrict__ logp_old,
    const float* __restrict__ adv, const float* __restrict__ ret, const float* __restrict__ v_s,
    const double* __restrict__ adv_sums, TailParams p, float* __restrict__ dz1,
    float* __restrict__ slab_f, double* __restrict__ slab_d) {
    constexpr bool actor = NET == 0;
    constexpr int net = NET;
    __shared__ __attribute__((aligned(16))) char img[actor ? I16_ACTOR : I16_CRITIC];
    __shared__ __attribute__((aligned(16))) float scr[T16_SCR];
    __shared__ float sv[T16_VEND];
    __shared__ double sred[T16_NW][SL_D];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, b = l & 15, g = l >> 4;
    const int A = p.A;
    {
        const float* w2 = actor ? wt.w2a : wt.w2c;
        const float* b2 = actor ? wt.b2a : wt.b2c;
        // layer 2: A = W2 [out 16 ot + i][k -> feature fh1(g, 8 kc + j)]
        build_img16(img + I16_W2, 4, 2, [=](int ot, int kc, int i, int gg, int j) {
            return w2[(16 * ot + i) * H + fh1(gg, 8 * kc + j)];
        });
        // dZ1: A = W2^T [f = fh1(i >> 2, 4 ft + (i & 3))][k -> out fb16(g, kc, j)]
        build_img16(img + I16_W2T, 4, 2, [=](int ft, int kc, int i, int gg, int j) {
            return w2[fb16(gg, kc, j) * H + fh1(i >> 2, 4 * ft + (i & 3))];
        });
        if (t < H) sv[T16_B2 + t] = b2[t];
        if (actor) {
            const float* w3 = wt.w3a;
            // mu head: A = W3 [a = 16 at + i][k -> h2 feature fb16(g, kc, j)]
            build_img16(img + I16_W3, 2, 2, [=](int at, int kc, int i, int gg, int j) {
                const int a = 16 * at + i;
                return a < A ? w3[a * H + fb16(gg, kc, j)] : 0.0f;
            });
            // dZ2: A = W3^T [out 16 ot + i][k -> a = fb16(g, 0, j)]
            build_img16(img + I16_W3T, 4, 1, [=](int ot, int, int i, int gg, int j) {
                const int a = fb16(gg, 0, j);
                return a < A ? w3[a * H + 16 * ot + i] : 0.0f;
            });
            if (t < AMAX) {
                sv[T16_B3 + t] = t < A ? wt.b3a[t] : 0.0f;
                const float sig = t < A ? expf(wt.log_std[t]) : 1.0f;
                sv[T16_LS + t] = logf(sig);
                sv[T16_IV + t] = 1.0f / (sig * sig);
                sv[T16_IV2 + t] = 1.0f / (2.0f * (sig * sig));
            }
        } else if (t < H) {
            sv[T16_W3C + t] = wt.w3c[t];
        }
    }
    __syncthreads();
    float* S1 = scr + w * 2 * H * SH;
    float* S2 = S1 + H * SH;
    const float b3c = wt.b3c[0];
    float mean_f = 0.0f, std_f = 1.0f;
    if (actor && p.norm_adv) {
        const double nn = 1.0 / p.inv_b64;
        const double m = adv_sums[0] / nn;
        const double var = (adv_sums[1] - adv_sums[0] * m) / (nn - 1.0);
        mean_f = (float)m;
        std_f = (float)sqrt(var > 0.0 ? var : 0.0);
    }
    // per-wave accumulators (32x32 C layout of acc_wgrad_x6) and per-lane column sums
    f32x16 gW2[2][2], gW3[1][actor ? 2 : 1];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) gW2[i][j] = zero16();
#pragma unroll
    for (int i = 0; i < (actor ? 2 : 1); ++i) gW3[0][i] = zero16();
    // column sums over the minibatch rows.  Each tile's are read off the feature-major
    // scratch the weight gradients stage anyway (one row of 16 values per lane): colA = db2
    // of feature l; colB (actor) = db3 of action l (l < 32) or d/dlog_std of action l - 32
    // (staged in S1 rows 32..63, which dW3 does not read).  Critic: dW3c and db3c as
    // per-lane partial sums (vl: 16 features of the lane's group, then gv).
    float colA = 0.f, colB = 0.f;
    constexpr int NV = actor ? 1 : 17;
    float vl[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) vl[i] = 0.f;
    double loss_acc = 0.0, cnt_acc = 0.0;
    const int c32 = l & 31, h32 = l >> 5;  // lane coordinates of the 32x32 weight-gradient tiles

    const int64_t ntiles = (n + 15) / 16;
    const int64_t gw = (int64_t)blockIdx.x * T16_NW + w, nw = (int64_t)gridDim.x * T16_NW;
    const uint32_t A_u = (uint32_t)A;
    for (int64_t tt = gw; tt < ntiles; tt += nw) {
        const int64_t row = tt * 16 + b;
        const bool live = row < n;
        const int64_t bt = tt >> 1;
        const int half = (int)(tt & 1);
        // ---- inputs ----------------------------------------------------------------------
        float h1[16];
        {
            const int64_t ftile = bt * NT + 2 * net + (g >> 1);
            const int flane = 16 * half + b + 32 * (g & 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v =
                    *reinterpret_cast<const float4*>(h1f + x6::frag_off4(ftile, flane, q));
                h1[4 * q] = v.x;
                h1[4 * q + 1] = v.y;
                h1[4 * q + 2] = v.z;
                h1[4 * q + 3] = v.w;
            }
        }
        const uint32_t j32 = live ? (uint32_t)(idx ? idx[row] : row) : 0u;
        float x0, x1;
        float av[8];
        if constexpr (actor) {
            const uint32_t ab = j32 * A_u;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t a = (uint32_t)fc16(g, r >> 2, r & 3);
                av[r] = act[ab + (a < A_u ? a : 0u)];
            }
            x0 = logp_old[j32];
            x1 = adv[j32];
        } else {
            x0 = ret[j32];
            x1 = p.value_clip ? v_s[j32] : 0.0f;
        }
        // ---- layer 2 ---------------------------------------------------------------------
        float h2[4][4];
        {
            f32x4 z[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
            for (int kc = 0; kc < 2; ++kc) {
                bf16x8 bb[NPL];
                float v8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v8[j] = h1[8 * kc + j];
                split8(v8, bb);
#pragma unroll
                for (int ot = 0; ot < 4; ++ot) {
                    bf16x8 aa[NPL];
                    ld_img16(img + I16_W2, 4, 2, ot, kc, l, aa);
                    z[ot] = mfma6_16(aa, bb, z[ot]);
                }
            }
#pragma unroll
            for (int ot = 0; ot < 4; ++ot)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    h2[ot][r] = tanh_nb(z[ot][r] + sv[T16_B2 + fc16(g, ot, r)]);
        }
        float dz2[4][4];
        if constexpr (actor) {
            // ---- mu head + clipped surrogate ---------------------------------------------
            f32x4 mu[2] = {zero4(), zero4()};
#pragma unroll
            for (int kc = 0; kc < 2; ++kc) {
                bf16x8 bb[NPL];
                float v8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v8[j] = h2[2 * kc + (j >> 2)][j & 3];
                split8(v8, bb);
#pragma unroll
                for (int at = 0; at < 2; ++at) {
                    bf16x8 aa[NPL];
                    ld_img16(img + I16_W3, 2, 2, at, kc, l, aa);
                    mu[at] = mfma6_16(aa, bb, mu[at]);
                }
            }
            float diff[8];
            float lp = 0.0f;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int a = fc16(g, r >> 2, r & 3);
                const bool in = a < A && live;
                const float d = av[r] - (mu[r >> 2][r & 3] + sv[T16_B3 + a]);
                const float term = -(d * d) * sv[T16_IV2 + a] - sv[T16_LS + a] - LOG_SQRT_2PI;
                diff[r] = in ? d : 0.0f;
                lp += in ? term : 0.0f;
            }
            const float lp2 = lp + __shfl_xor(lp, 16, 64);
            const float logp = lp2 + __shfl_xor(lp2, 32, 64);
            float g_logp = 0.0f;
            if (live) {
                float an = x1;
                if (p.norm_adv) an = (an - mean_f) / (std_f + p.adv_eps);
                const float ratio = expf(logp - x0);
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
                    const float tt2 = p.dual * an;
                    if (clip1 > tt2) {
                        obj = clip1;
                    } else if (clip1 < tt2) {
                        obj = tt2;
                        dobj = 0.0f;
                    } else {
                        obj = clip1;
                        dobj = 0.5f * d1;
                    }
                }
                g_logp = (float)(-(double)dobj * (double)ratio * p.inv_b64);
                if (g == 0) {
                    loss_acc += -(double)obj;
                    cnt_acc += 1.0;
                }
            }
            float dmu[8], dls[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int a = fc16(g, r >> 2, r & 3);
                const float iv = sv[T16_IV + a];
                dmu[r] = g_logp * diff[r] * iv;
                dls[r] = (a < A && live) ? g_logp * (diff[r] * diff[r] * iv - 1.0f) : 0.0f;
            }
            // dW3 = dMu^T . H2 over the tile's 16 rows; db3 and d/dlog_std from the scratch
            {
                float h2f[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) h2f[r] = h2[r >> 2][r & 3];
                wave_sync_lds();
                put16(S1, dmu, b, [=](int r) { return fc16(g, r >> 2, r & 3); });
                put16(S1, dls, b, [=](int r) { return 32 + fc16(g, r >> 2, r & 3); });
                put16(S2, h2f, b, [=](int r) { return fc16(g, r >> 2, r & 3); });
                wave_sync_lds();
                acc_wgrad_x6<1, 2>(gW3, S1, S2, c32, h32);
                colB += rowsum16(S1 + l * SH);
            }
            // dZ2 = (W3^T dMu) * (1 - H2^2)
            {
                bf16x8 bb[NPL];
                split8(dmu, bb);
#pragma unroll
                for (int ot = 0; ot < 4; ++ot) {
                    bf16x8 aa[NPL];
                    ld_img16(img + I16_W3T, 4, 1, ot, 0, l, aa);
                    const f32x4 d = mfma6_16(aa, bb, zero4());
#pragma unroll
                    for (int r = 0; r < 4; ++r) dz2[ot][r] = d[r] * (1.0f - h2[ot][r] * h2[ot][r]);
                }
            }
        } else {
            // ---- value head + value loss ---------------------------------------------------
            float vpart = 0.0f;
#pragma unroll
            for (int ot = 0; ot < 4; ++ot)
#pragma unroll
                for (int r = 0; r < 4; ++r) vpart += sv[T16_W3C + fc16(g, ot, r)] * h2[ot][r];
            const float v2 = vpart + __shfl_xor(vpart, 16, 64);
            const float value = v2 + __shfl_xor(v2, 32, 64) + b3c;
            float gv = 0.0f;
            if (live) {
                const float rt = x0;
                float dv, vf;
                if (p.value_clip) {
                    const float vs = x1;
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
                if (g == 0) loss_acc += (double)vf;
            }
#pragma unroll
            for (int ot = 0; ot < 4; ++ot)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    vl[4 * ot + r] += gv * h2[ot][r];
                    dz2[ot][r] = gv * sv[T16_W3C + fc16(g, ot, r)] * (1.0f - h2[ot][r] * h2[ot][r]);
                }
            vl[NV - 1] += g == 0 ? gv : 0.0f;
        }
        // ---- dZ1 = (W2^T dZ2) * (1 - H1^2) -> HBM (row-major [n][128]) -------------------
        {
            f32x4 d1[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
            for (int kc = 0; kc < 2; ++kc) {
                bf16x8 bb[NPL];
                float v8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v8[j] = dz2[2 * kc + (j >> 2)][j & 3];
                split8(v8, bb);
#pragma unroll
                for (int ft = 0; ft < 4; ++ft) {
                    bf16x8 aa[NPL];
                    ld_img16(img + I16_W2T, 4, 2, ft, kc, l, aa);
                    d1[ft] = mfma6_16(aa, bb, d1[ft]);
                }
            }
            if (live) {
                // register 4 ft + r holds feature fh1(g, 4 ft + r): four runs of 4 features
                float* o = dz1 + row * HC + 64 * net + 32 * (g >> 1) + 4 * (g & 1);
#pragma unroll
                for (int ft = 0; ft < 4; ++ft) {
                    const float4 v = make_float4(
                        d1[ft][0] * (1.0f - h1[4 * ft] * h1[4 * ft]),
                        d1[ft][1] * (1.0f - h1[4 * ft + 1] * h1[4 * ft + 1]),
                        d1[ft][2] * (1.0f - h1[4 * ft + 2] * h1[4 * ft + 2]),
                        d1[ft][3] * (1.0f - h1[4 * ft + 3] * h1[4 * ft + 3]));
                    *reinterpret_cast<float4*>(o + 8 * ft) = v;
                }
            }
        }
        // ---- db2, dW2 = dZ2^T . H1 over the tile's 16 rows ---------------------------------
        {
            float dzf[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) dzf[r] = dz2[r >> 2][r & 3];
            wave_sync_lds();
            put16(S1, dzf, b, [=](int r) { return fc16(g, r >> 2, r & 3); });
            put16(S2, h1, b, [=](int r) { return fh1(g, r); });
            wave_sync_lds();
            acc_wgrad_x6<2, 2>(gW2, S1, S2, c32, h32);
            colA += rowsum16(S1 + l * SH);
        }
    }
    // ---- fold the T16_NW waves (fixed order) into this workgroup's slab -------------------
    __syncthreads();
    float* red = scr;
    float* slab = slab_f + (int64_t)blockIdx.x * SL_F;
    auto fold = [&](const f32x16 (&gg)[2], int o0, int base) {
        // rows [o0, o0+32) of a [rows][64] matrix held as 32x32 C layout
#pragma unroll
        for (int ft = 0; ft < 2; ++ft)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                red[w * 32 * H + (rho(r) + 4 * h32) * H + 32 * ft + c32] = gg[ft][r];
        __syncthreads();
        for (int i = t; i < 32 * H; i += T16_TPB) {
            float v = red[i];
#pragma unroll
            for (int ww = 1; ww < T16_NW; ++ww) v += red[ww * 32 * H + i];
            slab[base + o0 * H + i] = v;
        }
        __syncthreads();
    };
    const int base2 = actor ? SL_W2A : SL_W2C;
    fold(gW2[0], 0, base2);
    fold(gW2[1], 32, base2);
    if constexpr (actor) fold(gW3[0], 0, SL_W3A);
    // column sums: [wave][lane][NF] = colA, colB, then (critic) the per-lane partials vl
    constexpr int NF = 2 + (actor ? 0 : NV);
    red[(w * 64 + l) * NF] = colA;
    red[(w * 64 + l) * NF + 1] = colB;
    if constexpr (!actor) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[(w * 64 + l) * NF + 2 + i] = vl[i];
    }
    loss_acc = wave_sum(loss_acc);
    cnt_acc = wave_sum(cnt_acc);
    if (l == 0) {
        sred[w][0] = loss_acc;
        sred[w][1] = cnt_acc;
    }
    __syncthreads();
    auto wsum = [&](int lane, int k) -> double {  // over the waves, fixed order
        double v = 0.0;
        for (int ww = 0; ww < T16_NW; ++ww) v += (double)red[(ww * 64 + lane) * NF + k];
        return v;
    };
    // critic per-lane partials: feature o of lane group (o >> 2) & 3, register
    // 4 (o >> 4) + (o & 3), over the group's 16 lanes (rows) and the waves
    auto gsum = [&](int gg, int k) -> double {
        double v = 0.0;
        for (int ww = 0; ww < T16_NW; ++ww) {
            float s = 0.f;
            for (int bb = 0; bb < 16; ++bb) s += red[(ww * 64 + 16 * gg + bb) * NF + k];
            v += (double)s;
        }
        return v;
    };
    double* sd = slab_d + (int64_t)blockIdx.x * SL_D;
    if (t < H) {
        slab[(actor ? SL_B2A : SL_B2C) + t] = (float)wsum(t, 0);
        if (!actor) slab[SL_W3C + t] = (float)gsum((t >> 2) & 3, 2 + 4 * (t >> 4) + (t & 3));
    } else if (actor && t < H + AMAX) {
        slab[SL_B3A + t - H] = (float)wsum(t - H, 1);
    } else if (actor && t < H + 2 * AMAX) {
        sd[4 + t - H - AMAX] = wsum(t - H, 1);  // lanes 32..63: d/dlog_std
    } else if (!actor && t == H) {
        slab[SL_B3C] = (float)gsum(0, 2 + NV - 1);
    } else if (t >= 3 * H && t < 3 * H + 2) {
        double v = 0.0;
#pragma unroll
        for (int ww = 0; ww < T16_NW; ++ww) v += sred[ww][t - 3 * H];
        if (actor) {
            if (t == 3 * H) sd[0] = v;  // clip sum
            else sd[2] = v;             // row count
        } else if (t == 3 * H) {
            sd[1] = v;                  // vf sum
        }
    }
    if (actor && t == 3 * H + 2) sd[3] = 0.0;
}

// ---------------------------------------------------------------------------------------
// Forward-only evaluation for PPOPolicy.process_fn: critic values V(s) (a2c.py:83-100) and,
// with LOGP, the Gaussian log-prob of the stored actions (logp_old, ppo.py:95-96), from the
// layer-1 activations of tsrl_mlp_l1_fwd.  One wave = 32 rows.
// ---------------------------------------------------------------------------------------
constexpr int E_B2A = 0, E_B2C = E_B2A + H, E_B3 = E_B2C + H, E_W3C = E_B3 + AMAX, E_VAR = E_W3C + H,
              E_LS = E_VAR + AMAX, E_END = E_LS + AMAX;

// Round 3: layer 2 and the mu head as bf16x6 products against split weight images (the
// 32-row image layout above) instead of v_mfma_f32_32x32x2_f32 with one LDS read
// per MFMA: 2.7x fewer matrix-core cycles per tile.
constexpr int EV_W2A = 0, EV_W2C = EV_W2A + NPL * 2 * H * 64, EV_W3 = EV_W2C + NPL * 2 * H * 64,
              EV_IMG = EV_W3 + NPL * 2 * AMAX * 64;  // 60 KB: two workgroups per CU

template <bool LOGP>
__global__ __launch_bounds__(256, 2) void eval_tail_kernel(const float* __restrict__ h1f,
                                                           int64_t n, TailWeights wt, int A,
                                                           const float* __restrict__ act,
                                                           float* __restrict__ value_out,
                                                           float* __restrict__ logp_out) {
    __shared__ float sm[E_END];
    __shared__ __attribute__((aligned(16))) char img[EV_IMG];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    build_img_n<256>(img + EV_W2C, H, 2, [=](int r, int k) { return wt.w2c[r * H + k]; });
    if (LOGP) {
        build_img_n<256>(img + EV_W2A, H, 2, [=](int r, int k) { return wt.w2a[r * H + k]; });
        build_img_n<256>(img + EV_W3, AMAX, 2,
                         [=](int r, int k) { return r < A ? wt.w3a[r * H + k] : 0.0f; });
    }
    if (t < H) {
        sm[E_B2C + t] = wt.b2c[t];
        sm[E_W3C + t] = wt.w3c[t];
        if (LOGP) sm[E_B2A + t] = wt.b2a[t];
    }
    if (LOGP && t < AMAX) {
        sm[E_B3 + t] = t < A ? wt.b3a[t] : 0.0f;
        const float sig = t < A ? expf(wt.log_std[t]) : 1.0f;
        sm[E_VAR + t] = sig * sig;
        sm[E_LS + t] = logf(sig);
    }
    __syncthreads();
    const float b3c = wt.b3c[0];
    const int64_t ntiles = (n + 31) / 32;
    // one net's two layer-1 tiles of row tile bt (fragment layout, 32 floats per lane)
    auto load_unit = [&](int64_t bt, int net, float (&h1)[2][16]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *reinterpret_cast<const float4*>(
                    h1f + x6::frag_off4(bt * NT + 2 * net + i, l, q));
                h1[i][4 * q] = v.x;
                h1[i][4 * q + 1] = v.y;
                h1[i][4 * q + 2] = v.z;
                h1[i][4 * q + 3] = v.w;
            }
        }
    };
    auto run_net = [&](int64_t bt, int net, const float (&h1)[2][16]) {
        const int64_t brow = bt * 32 + c;
        const bool live = brow < n;
        // the stored actions of the logp rows, loaded before the products they wait behind
        float av[16];
        if (net == 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int a = rho(r) + 4 * h;
                av[r] = 0.0f;
                if (a < A && live) av[r] = act[brow * A + a];
            }
        }
        const char* iw2 = img + (net ? EV_W2C : EV_W2A);
        const float* sb2 = sm + (net ? E_B2C : E_B2A);
        float h2[2][16];
        {
            f32x16 z0 = zero16(), z1 = zero16();
#pragma unroll
            for (int kc = 0; kc < 2; ++kc)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    bf16x8 b[NPL], a[NPL];
                    split_frag(h1[kc], s, b);
                    ld_img(iw2, 2, H, kc, c, s, h, a);
                    z0 = mfma6(a, b, z0);
                    ld_img(iw2, 2, H, kc, 32 + c, s, h, a);
                    z1 = mfma6(a, b, z1);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                h2[0][r] = tanh_nb(z0[r] + sb2[rho(r) + 4 * h]);
                h2[1][r] = tanh_nb(z1[r] + sb2[32 + rho(r) + 4 * h]);
            }
        }
        if (net == 1) {
            float vpart = 0.0f;
#pragma unroll
            for (int it = 0; it < 2; ++it)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    vpart += sm[E_W3C + 32 * it + rho(r) + 4 * h] * h2[it][r];
            const float value = vpart + __shfl_xor(vpart, 32, 64) + b3c;
            if (live && h == 0) value_out[brow] = value;
        } else {
            f32x16 mu = zero16();
#pragma unroll
            for (int kc = 0; kc < 2; ++kc)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    bf16x8 b[NPL], a[NPL];
                    split_frag(h2[kc], s, b);
                    ld_img(img + EV_W3, 2, AMAX, kc, c, s, h, a);
                    mu = mfma6(a, b, mu);
                }
            float lp = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int a = rho(r) + 4 * h;
                if (a < A && live) {
                    const float diff = av[r] - (mu[r] + sm[E_B3 + a]);
                    lp += -(diff * diff) / (2.0f * sm[E_VAR + a]) - sm[E_LS + a] - LOG_SQRT_2PI;
                }
            }
            const float logp = lp + __shfl_xor(lp, 32, 64);
            if (live && h == 0) logp_out[brow] = logp;
        }
    };
    const int64_t bstep = (int64_t)gridDim.x * 4;
    int64_t bt = (int64_t)blockIdx.x * 4 + w;
    if (LOGP) {
        // Round 5: one net's layer-1 tiles in flight while the other's products run (the
        // critic's of this row tile under the actor's, the next row tile's actor under this
        // critic's) instead of every wave waiting for its loads: 623 -> 542 us per 2M rows
        // (rocprof, profiles/r05_evtail_ab.log)
        float ua[2][16], ub[2][16];
        if (bt < ntiles) load_unit(bt, 0, ua);
        for (; bt < ntiles; bt += bstep) {
            load_unit(bt, 1, ub);
            __builtin_amdgcn_sched_barrier(0);
            run_net(bt, 0, ua);
            __builtin_amdgcn_sched_barrier(0);
            if (bt + bstep < ntiles) load_unit(bt + bstep, 0, ua);
            __builtin_amdgcn_sched_barrier(0);
            run_net(bt, 1, ub);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        for (; bt < ntiles; bt += bstep) {
            float h1[2][16];
            load_unit(bt, 1, h1);
            run_net(bt, 1, h1);
        }
    }
}

// Folds the per-workgroup slabs (fixed order) into the parameter gradients and the loss sums.
struct TailGrads {
    float *w2a, *b2a, *w2c, *b2c, *w3a, *b3a, *w3c, *b3c;
};

// Sum over `nslab` slabs (stride `stride` elements) of element i, fixed order: 4 lane groups
// of the workgroup take slabs g, g+4, ... with 4 independent accumulators each (loads stay in
// flight), then the groups combine in order through LDS.  Block = 64 outputs x 4 groups.
template <typename T>
__device__ __forceinline__ T slab_sum(const T* __restrict__ base, int64_t stride, int nslab,
                                      int64_t i, bool valid, T* sh) {
    const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
    T a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (valid) {
        int k = g;
        for (; k + 12 < nslab; k += 16) {
            a0 += base[(int64_t)k * stride + i];
            a1 += base[(int64_t)(k + 4) * stride + i];
            a2 += base[(int64_t)(k + 8) * stride + i];
            a3 += base[(int64_t)(k + 12) * stride + i];
        }
        for (; k < nslab; k += 4) a0 += base[(int64_t)k * stride + i];
    }
    sh[g * 64 + o] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    return ((sh[o] + sh[64 + o]) + sh[128 + o]) + sh[192 + o];
}

// Optional loss finalisation folded into the loss-sum block (tsrl_ppo_tail_fin): the work of
// ppo.hip's gauss_finalize_kernel (loss terms, the log-std gradient) on the sums this block
// just reduced, so the single-process minibatch needs no separate launch for it.
struct TailFin {
    const float* log_std;
    float* losses;        // NULL: no finalisation
    float* grad_log_std;
    float vf_coef, ent_coef;
    double inv_b;
};

__global__ __launch_bounds__(256) void tail_reduce_kernel(const float* __restrict__ slab_f,
                                                          const double* __restrict__ slab_d,
                                                          int nslab, int A, TailGrads g,
                                                          double* __restrict__ sums, TailFin fin) {
    __shared__ float shf[256];
    __shared__ double shd[256];
    const int nfb = (SL_F + 63) / 64;
    if ((int)blockIdx.x < nfb) {
        const int i = blockIdx.x * 64 + (threadIdx.x & 63);
        const float s = slab_sum(slab_f, SL_F, nslab, i, i < SL_F, shf);
        if (threadIdx.x >= 64 || i >= SL_F) return;
        if (i < SL_B2A) g.w2a[i] = s;
        else if (i < SL_W2C) g.b2a[i - SL_B2A] = s;
        else if (i < SL_B2C) g.w2c[i - SL_W2C] = s;
        else if (i < SL_W3A) g.b2c[i - SL_B2C] = s;
        else if (i < SL_B3A) { if (i - SL_W3A < A * H) g.w3a[i - SL_W3A] = s; }
        else if (i < SL_W3C) { if (i - SL_B3A < A) g.b3a[i - SL_B3A] = s; }
        else if (i < SL_B3C) g.w3c[i - SL_W3C] = s;
        else if (i == SL_B3C) g.b3c[0] = s;
    } else {
        const int k0 = threadIdx.x & 63;
        const double s = slab_sum(slab_d, SL_D, nslab, k0, k0 < SL_D, shd);
        if (threadIdx.x < 64 && k0 < 4 + A) sums[k0] = s;
        if (fin.losses) {
            __shared__ double fs[64];
            if (threadIdx.x < 64) fs[k0] = s;
            __syncthreads();
            if (threadIdx.x == 0) {
                float ent = 0.0f;
                for (int a = 0; a < A; ++a) {
                    const float sig = expf(fin.log_std[a]);
                    ent += 1.4189385332046727f + logf(sig);  // f32(0.5 + 0.5 log 2 pi) + log(scale)
                }
                const float clip = (float)(fs[0] * fin.inv_b);
                const float vf = (float)(fs[1] * fin.inv_b);
                fin.losses[0] = clip + fin.vf_coef * vf - fin.ent_coef * ent;
                fin.losses[1] = clip;
                fin.losses[2] = vf;
                fin.losses[3] = ent;
            }
            for (int a = threadIdx.x; a < A; a += blockDim.x)
                fin.grad_log_std[a] = (float)(fs[4 + a] - (double)fin.ent_coef);
        }
    }
}

// ---------------------------------------------------------------------------------------
// dW1cat = dZ1^T . X[idx] and db1 (ones column at k = D), split over minibatch rows.
// Workgroup = 128 features x 128 input columns x one row range; wave w owns columns
// [32w, 32w+32) for all 4 feature tiles.  Rows are staged 32 at a time through LDS.
// ---------------------------------------------------------------------------------------
constexpr int DW_COLS = 128;
constexpr int DW_KB = 32;

// bf16x6 (x6.h): every staged element is split once, by the thread that loads it, into three
// bf16 planes stored transposed ([feature or column][32 rows], x6::sw_off rows), so a
// lane's MFMA fragment (8 consecutive minibatch rows of one feature / column) is one
// ds_read_b128 per plane and the inner loop is 15 LDS reads + 24 bf16 MFMAs per 16 rows.
// Staging: thread t owns feature / column (t & 127) and the 8-row groups {rg, rg + 2} of the
// chunk (rg = t >> 7, wave-uniform, so the row indices come in through scalar loads); the
// next chunk's 32 values are loaded into registers during the current chunk's MFMAs.
// Round 3, measured and dropped: dZ1 handed over by the tail as split bf16 planes in this
// kernel's own LDS image (6 16-byte copies per thread per chunk instead of 16 loads + splits):
// dW1 217 -> 212 us but the tail's transpose + split of dZ1 221 vs 208 us -- a net loss.
// Also (tools/dw_ab.sh, 262144 rows, same box): one workgroup per
// CU covering all 384 columns, so each dZ1 element is loaded and split once instead of three
// times -- 4 waves with 12 accumulator tiles each 311-317 us vs 264-267 for this kernel; 8
// waves with 6 tiles each, MFMAs issued ahead of the next chunk's split 258-261 vs 246.
// Round 5 (tools/r05_ab.sh, profiles/r05_variant_ab.log): chunks fully inside the row range
// take their row indices eight at a time in one scalar load with 32-bit row offsets and are
// staged without row masks (static count of the per-chunk loop 700 -> 460 instructions, SALU
// 180 -> 42): dW1 + reduce 246.9 / 255.5 -> 237.0 / 235.8 us, minibatch 719 / 731 -> 695 /
// 680 us, two A/B rounds in one call -- now the only form.
#ifndef DWX6_OCC
#define DWX6_OCC 2
#endif
__global__ __launch_bounds__(256, DWX6_OCC) void dw_x6_kernel(
    const float* __restrict__ dz, const float* __restrict__ X, int64_t ldx,
    const int64_t* __restrict__ idx, int64_t n, int D, int64_t rows_per_split, int ncolpad,
    int ncolt, float* __restrict__ part) {
    constexpr int PL = 128 * 64;  // bytes per plane: 128 rows of 32 bf16
    __shared__ __attribute__((aligned(16))) char Zi[NPL * PL];
    __shared__ __attribute__((aligned(16))) char Xi[NPL * PL];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    // 1-D grid of ncolt x nsplit workgroups, remapped XCD-aware: blocks b and b + 8 share an
    // XCD (and its L2), so logical tile L = (b % 8) * (G / 8) + b / 8 puts the ncolt column
    // tiles of one row split on one XCD at about the same time and dZ1 (read once per column
    // tile) comes from HBM once (G % 8 == 0 by construction of dw_nsplit; otherwise L = b).
    const int G = gridDim.x, b = blockIdx.x;
    const int L = (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
    const int colt = L % ncolt, split = L / ncolt;
    const int col0 = colt * DW_COLS;
    const int64_t r0 = (int64_t)split * rows_per_split;
    const int64_t r1 = min(n, r0 + rows_per_split);
    const int fc = t & 127;                                  // staged feature / column
    const int rg = __builtin_amdgcn_readfirstlane(t >> 7);   // 8-row groups rg, rg + 2
    const int k = col0 + fc;
    const float ones = k == D ? 1.0f : 0.0f;  // db1 through a ones column at k == D
    const bool kin = k < D;
    const float* xcol = X + (kin ? k : 0);
    const uint64_t ldx32 = (uint32_t)ldx;
    float zr[16], xr[16];
#define DWX6_LOAD(rb)                                                                       \
    {                                                                                       \
        _Pragma("unroll") for (int q = 0; q < 16; ++q) {                                    \
            const int64_t r = (rb) + 8 * (rg + 2 * (q >> 3)) + (q & 7);                     \
            const int64_t rr = r < r1 ? r : r1 - 1;                                          \
            const int64_t ri = idx ? idx[rr] : rr;                                          \
            zr[q] = dz[rr * HC + fc];                                                       \
            xr[q] = xcol[ri * ldx];                                                         \
        }                                                                                   \
    }
    /* a whole chunk of gathered rows (rb + DW_KB <= r1): no clamps, so the 8 contiguous  */ \
    /* row indices of a group come in one scalar load and the dZ1 rows sit at immediate   */ \
    /* offsets of one base; the X row offset is a 32 x 32 -> 64-bit product of the row    */ \
    /* index (< 2^32, tsrl.h) and the pitch: 4 SALU per row instead of ~12 with the clamp  */ \
#define DWX6_LOAD_FULL(rb)                                                                  \
    {                                                                                       \
        _Pragma("unroll") for (int g_ = 0; g_ < 2; ++g_) {                                  \
            const int64_t rg0_ = (rb) + 8 * (rg + 2 * g_);                                  \
            const float* zb_ = dz + rg0_ * HC + fc;                                         \
            const int64_t* ib_ = idx + rg0_;                                                \
            _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_) {                              \
                zr[8 * g_ + j_] = zb_[j_ * HC];                                             \
                const uint64_t ri_ = (uint32_t)ib_[j_];                                     \
                xr[8 * g_ + j_] = xcol[ri_ * ldx32];                                        \
            }                                                                               \
        }                                                                                   \
    }
    /* masks applied at the LDS store, not next to the loads (a select on a loaded value */ \
    /* there would make the wave wait for the data before the chunk's MFMAs)           */ \
#define DWX6_STORE(rb, FULL)                                                                \
    {                                                                                       \
        _Pragma("unroll") for (int g = 0; g < 2; ++g) {                                     \
            bf16x8 zp[NPL], xp[NPL];                                                        \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                 \
                const bool lv = (FULL) || (rb) + 8 * (rg + 2 * g) + j < r1;                 \
                const float zv = lv ? zr[8 * g + j] : 0.0f;                                 \
                const float xv = lv ? (kin ? xr[8 * g + j] : ones) : 0.0f;                  \
                __bf16 a0, a1, a2;                                                          \
                split1(zv, a0, a1, a2);                                                     \
                zp[0][j] = a0;                                                              \
                zp[1][j] = a1;                                                              \
                zp[2][j] = a2;                                                              \
                split1(xv, a0, a1, a2);                                                     \
                xp[0][j] = a0;                                                              \
                xp[1][j] = a1;                                                              \
                xp[2][j] = a2;                                                              \
            }                                                                               \
            const int off = sw_off(fc, rg + 2 * g);                                         \
            _Pragma("unroll") for (int p = 0; p < NPL; ++p) {                               \
                *reinterpret_cast<bf16x8*>(Zi + p * PL + off) = zp[p];                      \
                *reinterpret_cast<bf16x8*>(Xi + p * PL + off) = xp[p];                      \
            }                                                                               \
        }                                                                                   \
    }
    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = zero16();
    const int64_t nchunk = r1 > r0 ? (r1 - r0 + DW_KB - 1) / DW_KB : 0;
    if (nchunk > 0) {
        DWX6_LOAD(r0)
        DWX6_STORE(r0, false)
    }
    __syncthreads();
    for (int64_t ch = 0; ch < nchunk; ++ch) {
        if (ch + 1 < nchunk) {
            const int64_t rb = r0 + (ch + 1) * DW_KB;
            if (idx && rb + DW_KB <= r1)
                DWX6_LOAD_FULL(rb)
            else
                DWX6_LOAD(rb)
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 b[NPL];
            const int xo = sw_off(32 * w + c, 2 * s + h);
#pragma unroll
            for (int p = 0; p < NPL; ++p) b[p] = *reinterpret_cast<const bf16x8*>(Xi + p * PL + xo);
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                bf16x8 a[NPL];
                const int zo = sw_off(32 * i + c, 2 * s + h);
#pragma unroll
                for (int p = 0; p < NPL; ++p)
                    a[p] = *reinterpret_cast<const bf16x8*>(Zi + p * PL + zo);
                acc[i] = mfma6(a, b, acc[i]);
            }
        }
        if (ch + 1 < nchunk) {
            __syncthreads();
            const int64_t rb = r0 + (ch + 1) * DW_KB;
            if (rb + DW_KB <= r1)
                DWX6_STORE(rb, true)  // no row masks in a whole chunk
            else
                DWX6_STORE(rb, false)
            __syncthreads();
        }
    }
#undef DWX6_LOAD
#undef DWX6_LOAD_FULL
#undef DWX6_STORE
    float* o = part + (int64_t)split * HC * ncolpad;
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
    __shared__ float sh[256];
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t total = (int64_t)HC * ncolpad;
    const int f = (int)(i / ncolpad), k = (int)(i - (int64_t)f * ncolpad);
    const bool valid = i < total && k <= D;
    const float s = slab_sum(part, total, nsplit, i, valid, sh);
    if (threadIdx.x >= 64 || !valid) return;
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
    // workgroups per net (one launch per net), one resident per CU
    const int64_t tiles = (n + 15) / 16;
    const int64_t g = (tiles + T16_NW - 1) / T16_NW;
    return (int)std::min<int64_t>(g, 256);
}

int dw_nsplit(int64_t n) {
    // ~512 resident workgroups on 256 CUs (3 column tiles at D=376), >= 64 rows per split.
    // Round 5 A/B of the cap (profiles/r05_learn_ab.log, dw + reduce per 262144 rows): 64 /
    // 96 / 128 / 168 / 208 / 256 splits -> 340 / 306 / 263 / 228-241 / 291-298 / 273-278 us
    int64_t s = std::max<int64_t>(1, std::min<int64_t>(170, n / 64));
    // a multiple of 8 (XCD-aware tile order in dw_x6_kernel) once there are 8 or more
    if (s >= 8) s &= ~int64_t(7);
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

static int ppo_tail_impl(const float* h1frag, int64_t n, const int64_t* idx,
                         const tsrl_tail_weights* wt, int64_t act_dim, const float* act,
                         const float* logp_old, const float* adv, const float* ret,
                         const float* v_s, const double* adv_sums, tsrl_ppo_params prm,
                         float* dz1, const tsrl_tail_grads* grads, double* sums,
                         void* workspace, int64_t ws_bytes, TailFin fin, int stages,
                         void* stream) {
    TSRL_CHECK_ARG((stages >= 1 && stages <= 3) || stages == 4 || stages == 8,
                   "tsrl_ppo_tail: stages must be 1, 2, 3, 4 or 8");
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
    const TailParams tp = make_tail_params(prm, (int)act_dim);
    // stages: 1 both nets' tails, 4 / 8 the actor's / the critic's alone (they write disjoint
    // slab entries and dZ1 halves, so two streams may run them side by side), 2 the reduction
    if (stages & (1 | 4)) {
        hipLaunchKernelGGL(ppo_tail16_kernel<0>, dim3(g), dim3(T16_TPB), 0, as_stream(stream),
                           h1frag, n, idx, w, act, logp_old, adv, ret, v_s, adv_sums, tp, dz1,
                           slab_f, slab_d);
        TSRL_LAUNCH_CHECK("tsrl_ppo_tail(actor)");
    }
    if (stages & (1 | 8)) {
        hipLaunchKernelGGL(ppo_tail16_kernel<1>, dim3(g), dim3(T16_TPB), 0, as_stream(stream),
                           h1frag, n, idx, w, act, logp_old, adv, ret, v_s, adv_sums, tp, dz1,
                           slab_f, slab_d);
        TSRL_LAUNCH_CHECK("tsrl_ppo_tail");
    }
    if (!(stages & 2)) return 0;
    TailGrads gg{grads->w2a, grads->b2a, grads->w2c, grads->b2c, grads->w3a, grads->b3a,
                 grads->w3c, grads->b3c};
    hipLaunchKernelGGL(tail_reduce_kernel, dim3((SL_F + 63) / 64 + 1), dim3(256), 0,
                       as_stream(stream), slab_f, slab_d, g, (int)act_dim, gg, sums, fin);
    TSRL_LAUNCH_CHECK("tsrl_ppo_tail(reduce)");
    return 0;
}

extern "C" int tsrl_ppo_tail(const float* h1frag, int64_t n, const int64_t* idx,
                             const tsrl_tail_weights* wt, int64_t act_dim, const float* act,
                             const float* logp_old, const float* adv, const float* ret,
                             const float* v_s, const double* adv_sums, tsrl_ppo_params prm,
                             float* dz1, const tsrl_tail_grads* grads, double* sums,
                             void* workspace, int64_t ws_bytes, void* stream) {
    const TailFin fin{nullptr, nullptr, nullptr, 0.f, 0.f, 0.0};
    return ppo_tail_impl(h1frag, n, idx, wt, act_dim, act, logp_old, adv, ret, v_s, adv_sums, prm,
                         dz1, grads, sums, workspace, ws_bytes, fin, 3, stream);
}

extern "C" int tsrl_ppo_tail_fin(const float* h1frag, int64_t n, const int64_t* idx,
                                 const tsrl_tail_weights* wt, int64_t act_dim, const float* act,
                                 const float* logp_old, const float* adv, const float* ret,
                                 const float* v_s, const double* adv_sums, tsrl_ppo_params prm,
                                 float* dz1, const tsrl_tail_grads* grads, double* sums,
                                 void* workspace, int64_t ws_bytes, const float* log_std,
                                 float* losses, float* grad_log_std, void* stream) {
    TSRL_CHECK_ARG(log_std && losses && grad_log_std, "tsrl_ppo_tail_fin: null pointer");
    const TailFin fin{log_std, losses, grad_log_std, (float)prm.vf_coef, (float)prm.ent_coef,
                      1.0 / prm.b_global};
    return ppo_tail_impl(h1frag, n, idx, wt, act_dim, act, logp_old, adv, ret, v_s, adv_sums, prm,
                         dz1, grads, sums, workspace, ws_bytes, fin, 3, stream);
}

extern "C" int tsrl_ppo_tail_stage(const float* h1frag, int64_t n, const int64_t* idx,
                                   const tsrl_tail_weights* wt, int64_t act_dim, const float* act,
                                   const float* logp_old, const float* adv, const float* ret,
                                   const float* v_s, const double* adv_sums, tsrl_ppo_params prm,
                                   float* dz1, const tsrl_tail_grads* grads, double* sums,
                                   void* workspace, int64_t ws_bytes, const float* log_std,
                                   float* losses, float* grad_log_std, int stages, void* stream) {
    TSRL_CHECK_ARG((log_std && losses && grad_log_std) || (!log_std && !losses && !grad_log_std),
                   "tsrl_ppo_tail_stage: log_std/losses/grad_log_std all set or all null");
    const TailFin fin{log_std, losses, grad_log_std, (float)prm.vf_coef, (float)prm.ent_coef,
                      1.0 / prm.b_global};
    return ppo_tail_impl(h1frag, n, idx, wt, act_dim, act, logp_old, adv, ret, v_s, adv_sums, prm,
                         dz1, grads, sums, workspace, ws_bytes, fin, stages, stream);
}

extern "C" int64_t tsrl_mlp_dw_workspace_bytes(int64_t n, int64_t D) {
    const int ncolpad = (int)(((D + 1 + DW_COLS - 1) / DW_COLS) * DW_COLS);
    const int nsplit = dw_nsplit(n);
    return (int64_t)nsplit * HC * ncolpad * (int64_t)sizeof(float);
}

extern "C" int tsrl_mlp_dw(const float* dz1, const float* X, int64_t ldx, const int64_t* idx,
                           int64_t n, int64_t D, float* gWa, float* gba, float* gWc, float* gbc,
                           void* workspace, int64_t ws_bytes, void* stream) {
    TSRL_CHECK_ARG(n > 0 && D > 0 && ldx >= D, "tsrl_mlp_dw: bad sizes");
    TSRL_CHECK_ARG(dz1 && X && gWa && gba && gWc && gbc && workspace, "tsrl_mlp_dw: null pointer");
    TSRL_CHECK_ARG(aligned16(dz1) && aligned16(X) && ldx % 4 == 0 && ldx >= (D + 3) / 4 * 4 && ldx < (int64_t(1) << 32),
                   "tsrl_mlp_dw: dz1/X must be 16-byte aligned, ldx a multiple of 4 and >= "
                   "roundup(D, 4) (columns D.. of the padding read as data-free)");
    TSRL_CHECK_ARG(ws_bytes >= tsrl_mlp_dw_workspace_bytes(n, D), "tsrl_mlp_dw: workspace too small");
    const int ncolt = (int)((D + 1 + DW_COLS - 1) / DW_COLS);
    const int ncolpad = ncolt * DW_COLS;
    const int nsplit = dw_nsplit(n);
    const int64_t rps = ((n + nsplit - 1) / nsplit + DW_KB - 1) / DW_KB * DW_KB;
    float* part = reinterpret_cast<float*>(workspace);
    hipLaunchKernelGGL(dw_x6_kernel, dim3(ncolt * nsplit), dim3(256), 0, as_stream(stream),
                       dz1, X, ldx, idx, n, (int)D, rps, ncolpad, ncolt, part);
    TSRL_LAUNCH_CHECK("tsrl_mlp_dw");
    const int64_t outs = (int64_t)HC * ncolpad;
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((outs + 63) / 64)), dim3(256), 0,
                       as_stream(stream), part, nsplit, ncolpad, (int)D, gWa, gba, gWc, gbc);
    TSRL_LAUNCH_CHECK("tsrl_mlp_dw(reduce)");
    return 0;
}

extern "C" int tsrl_ppo_eval(const float* h1frag, int64_t n, const tsrl_tail_weights* wt,
                             int64_t act_dim, const float* act, float* value_out,
                             float* logp_out, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && act_dim > 0 && act_dim <= AMAX, "tsrl_ppo_eval: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(h1frag && wt && value_out && (!logp_out || act),
                   "tsrl_ppo_eval: null pointer");
    TSRL_CHECK_ARG(aligned16(h1frag), "tsrl_ppo_eval: h1frag not 16-byte aligned");
    TailWeights w{wt->w2a, wt->b2a, wt->w2c, wt->b2c, wt->w3a, wt->b3a, wt->w3c, wt->b3c,
                  wt->log_std};
    const int64_t tiles = (n + 31) / 32;
    const unsigned g = (unsigned)std::min<int64_t>((tiles + 3) / 4, 1024);
    if (logp_out)
        hipLaunchKernelGGL(eval_tail_kernel<true>, dim3(g), dim3(256), 0, as_stream(stream), h1frag,
                           n, w, (int)act_dim, act, value_out, logp_out);
    else
        hipLaunchKernelGGL(eval_tail_kernel<false>, dim3(g), dim3(256), 0, as_stream(stream),
                           h1frag, n, w, (int)act_dim, act, value_out, logp_out);
    TSRL_LAUNCH_CHECK("tsrl_ppo_eval");
    return 0;
}
