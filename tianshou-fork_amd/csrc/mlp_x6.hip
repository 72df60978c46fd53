// First-layer GEMMs of the fused PPO MLP (mlp.hip) on the bf16 matrix cores with an exact
// three-way split of every f32 operand ("bf16x6" f32 emulation).
//
// An f32 x is split exactly into x = x0 + x1 + x2 with x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1) (round-to-nearest each time; the residuals are exact in f32 and the
// third piece holds the last 8 bits, so the split loses nothing).  A product a.b is
// accumulated as the six bf16 products of order <= 2,
//     a0b0 + (a0b1 + a1b0) + (a0b2 + a1b1 + a2b0),
// each exact in the f32 MFMA accumulator; the dropped terms (a1b2, a2b1, a2b2) are below
// 2^-24 |ab|, i.e. at the f32 rounding level of one product.  The sums accumulate in f32 as
// the f32-input MFMA path does, so the result carries f32 GEMM error (tests/test_gpu_mlp.py
// measures it against an fp64 product next to torch's own f32 GEMM).  Six bf16 MFMAs
// (v_mfma_f32_32x32x16_bf16, 32 cycles for 32x32x16) replace eight f32 ones
// (v_mfma_f32_32x32x2_f32, 64 cycles for 32x32x2): 2.7x the f32 matrix rate.
//
// l1_fwd_x6: H1^T = act(W1cat . X[idx]^T + b1) exactly as tsrl_mlp_l1_fwd (same output
// layouts); the weights are split once per parameter update (tsrl_mlp_split_w), the
// observation rows are staged as f32 and split by the wave that owns them, right before
// their MFMAs (each element is split once).  Measured (tools/mlp_kernel_bench.py, 262144
// gathered rows x 376): 250 us vs 336 us for the f32-input kernel.  Where the time goes
// (build variants timed on MI355X, since removed): without the global loads after chunk 0
// 171 us, without the MFMAs 223 us, X-row loads only 243 us, weight loads only 187 us; the
// matrix cores are 28 % busy (SQ_VALU_MFMA_BUSY_CYCLES).  The gathered X rows and the
// single-buffered chunk loop (two barriers per 32 k) bound it, not the MFMA rate; reading all
// of a step's LDS operands ahead of its MFMAs (sched_barrier) measured 6 % slower.
// Round 2 (tools/mlp_kernel_bench.py, 262144 rows): staging the X chunk with 8 consecutive
// lanes per 128-byte row segment (X6_COAL; two lanes per row before) takes the random-row
// gather from 285 to 245 us, the same as contiguous rows (240 us).  Tried and dropped: X
// straight to registers (no X LDS stage) with a 3-chunk register ring, double-buffered
// weight LDS and one barrier per chunk, paired v_cvt_pk splits: 243 / 280 us contiguous /
// random -- the LDS fragment reads right before their MFMAs (s_waitcnt per MFMA group) and
// the split VALU (~400 vector instructions per 48 MFMAs, SQ_INSTS_VALU) pace it, not the loads.
// Also tried in round 2 (same tool, one box, random rows; this kernel 241.7 us there): a
// generalised tiling of NW waves x RT 32-row tiles per wave, so each W fragment read from LDS
// feeds RT row tiles and each staged W chunk serves 32*NW*RT rows: 4x1 (the same tiling
// rewritten) 250 us, 8x1 (256 rows, W staging halved per row) 260 us, 4x2 (341 VGPR+AGPR,
// one wave per SIMD) 296 us -- fewer W bytes per row does not pay for the larger barrier
// group or the lost second wave per SIMD.  A two-register-set pipeline (each chunk's loads
// issued two chunks before its LDS store, 212 VGPRs, still 2 waves/SIMD) does not survive
// compilation: the IR passes sink the restrict-const loads next to their LDS stores (asm
// memory clobbers and sched_barrier do not pin them) and volatile loads get a vmcnt(0) each;
// it needs direct-to-LDS loads (global_load_lds_dwordx4) and an LDS ring instead.  Built and
// measured that way too (round 2): X rows and W planes by inline-asm LDS-DMA into a two-stage
// 2 x 40 KB ring, one barrier per chunk, the swizzles on the source addresses, explicit
// vmcnt(0) drains (hipcc's own LDS-DMA builtin makes every ds_read wait for the next stage):
// correct, 256-262 us vs 250-256 us for this kernel on the same box -- neither the staging
// instructions nor the second barrier are what bounds it.
#include "x6.h"

namespace tsrl {
namespace {

using x6::bf16x8;
using x6::f32x16;
using x6::mfma6;
using x6::NPL;
using x6::split1;
using x6::sw_off;

constexpr int H = 64;
constexpr int HC = 2 * H;   // actor + critic first-layer features
constexpr int NT = HC / 32;
constexpr int XR = 128;     // minibatch rows per workgroup
constexpr int KC = 32;      // k per staged chunk (two 16-k MFMA steps)
constexpr int ROWB = KC * 2;  // bytes per LDS row of one plane (32 bf16)

__device__ __forceinline__ int rho(int r) { return (r & 3) + 8 * (r >> 2); }

// f32 rows of KC floats (128 B, chunks q = 0..7): chunk index XOR row bits 1-3, so the
// 16-lane phases of a ds_read_b128 (rows r..r+15, one chunk) cover all banks.
constexpr int XROWB = KC * 4;
__device__ __forceinline__ int swf_off(int row, int q) {
    return row * XROWB + 16 * (q ^ ((row >> 1) & 7));
}

// v if keep else 0, per component (a whole-vector ternary becomes a scratch-indexed select)
__device__ __forceinline__ float4 keep4(bool keep, float4 v) {
    return make_float4(keep ? v.x : 0.f, keep ? v.y : 0.f, keep ? v.z : 0.f, keep ? v.w : 0.f);
}

// Elements o..o+3 of the three split planes from one float4.
__device__ __forceinline__ void split4(float4 v, bf16x8& p0, bf16x8& p1, bf16x8& p2, int o) {
    __bf16 a, b, c;
    split1(v.x, a, b, c);
    p0[o] = a, p1[o] = b, p2[o] = c;
    split1(v.y, a, b, c);
    p0[o + 1] = a, p1[o + 1] = b, p2[o + 1] = c;
    split1(v.z, a, b, c);
    p0[o + 2] = a, p1[o + 2] = b, p2[o + 2] = c;
    split1(v.w, a, b, c);
    p0[o + 3] = a, p1[o + 3] = b, p2[o + 3] = c;
}

// Split planes of the stacked first-layer weight: out[p][f][k] (f < 64 actor, >= 64 critic;
// k padded with zeros to Kp = roundup(D, 32)).
__global__ void split_w_kernel(const float* __restrict__ Wa, const float* __restrict__ Wc,
                               int64_t D, int64_t Kp, __bf16* __restrict__ out) {
    const int64_t total = (int64_t)HC * Kp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t f = i / Kp, k = i - f * Kp;
        float x = 0.0f;
        if (k < D) x = f < H ? Wa[f * D + k] : Wc[(f - H) * D + k];
        const __bf16 a0 = (__bf16)x;
        const float r1 = x - (float)a0;
        const __bf16 a1 = (__bf16)r1;
        out[i] = a0;
        out[total + i] = a1;
        out[2 * total + i] = (__bf16)(r1 - (float)a1);
    }
}

// Workgroup = 128 minibatch rows x 128 features, 4 waves; wave w owns rows [32w, 32w+32) and
// the 4 feature tiles.  K is staged 32 at a time: every thread loads 16 floats of one row
// (two threads per row, 128-byte row segments) and 16 pre-split weights per plane, both held
// in registers one chunk ahead and stored into the single-buffered LDS tiles after the
// chunk's MFMAs.  X6_IL interleaves the six products of two feature tiles; X6_OCC is the
// workgroups-per-CU bound (variants measured equal within 2 %, 2/1 kept).
#ifndef X6_OCC
#define X6_OCC 2
#endif
__global__ __launch_bounds__(256, X6_OCC) void l1_fwd_x6_kernel(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ idx, int64_t n,
    int D, int Kp, const __bf16* __restrict__ wsp, const float* __restrict__ ba,
    const float* __restrict__ bc, int act_tanh, float* __restrict__ out, int frag_out) {
    __shared__ __attribute__((aligned(16))) char Xs[XR * XROWB];  // f32 rows
    __shared__ __attribute__((aligned(16))) char Ws[NPL][HC * ROWB];
    __shared__ float sb[HC];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int64_t row0 = (int64_t)blockIdx.x * XR;
    if (t < HC) sb[t] = t < H ? ba[t] : bc[t - H];
    const int srow = t >> 1, sq = 2 * (t & 1);
    // X staging: thread t loads float4 (t & 7) of rows (t >> 3) + 32 i, i = 0..3: each load
    // instruction reads 8 whole 128-byte row segments (8 consecutive lanes per row)
    const int xq = t & 7, xr0 = t >> 3;
    const float* xs_[4];
    bool xl_[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t g_ = row0 + xr0 + 32 * i;
        xl_[i] = g_ < n;
        xs_[i] = X + (xl_[i] ? (idx ? idx[g_] : g_) : 0) * ldx;
    }
    const int64_t plane = (int64_t)HC * Kp;
    const __bf16* wsrc = wsp + (int64_t)srow * Kp + 8 * sq;
    const int nch = Kp / KC;
    // registers one chunk ahead: 16 floats of the row, 2 x 16 B per weight plane.  Loads are
    // branch-free (an out-of-range float4 reads k = 0 and is zeroed by a select: a load under
    // a runtime condition makes hipcc branch around it and drain vmcnt per element), and all
    // staging values are named scalars (no arrays or lambdas that end up in scratch).
    float4 x0, x1, x2, x3;
    uint4 w00, w01, w10, w11, w20, w21;
#define X6_XLOAD(kc)                                                                        \
    {                                                                                       \
        const int k_ = (kc) * KC + 4 * xq;                                                  \
        x0 = *reinterpret_cast<const float4*>(xs_[0] + (xl_[0] && k_ < D ? k_ : 0));        \
        x1 = *reinterpret_cast<const float4*>(xs_[1] + (xl_[1] && k_ < D ? k_ : 0));        \
        x2 = *reinterpret_cast<const float4*>(xs_[2] + (xl_[2] && k_ < D ? k_ : 0));        \
        x3 = *reinterpret_cast<const float4*>(xs_[3] + (xl_[3] && k_ < D ? k_ : 0));        \
    }
#define X6_XSTORE(kc)                                                                       \
    {                                                                                       \
        const int k_ = (kc) * KC + 4 * xq;                                                  \
        *reinterpret_cast<float4*>(&Xs[swf_off(xr0, xq)]) = keep4(xl_[0] && k_ < D, x0);     \
        *reinterpret_cast<float4*>(&Xs[swf_off(xr0 + 32, xq)]) = keep4(xl_[1] && k_ < D, x1);\
        *reinterpret_cast<float4*>(&Xs[swf_off(xr0 + 64, xq)]) = keep4(xl_[2] && k_ < D, x2);\
        *reinterpret_cast<float4*>(&Xs[swf_off(xr0 + 96, xq)]) = keep4(xl_[3] && k_ < D, x3);\
    }
#define X6_LOAD(kc)                                                                         \
    {                                                                                       \
        X6_XLOAD(kc)                                                                        \
        /* a float4 that starts inside the row is read whole: its columns >= D are the */    \
        /* caller's finite padding and meet zero weights (split_w pads W with zeros)  */    \
        const __bf16* wk_ = wsrc + (kc) * KC;                                                \
        w00 = *reinterpret_cast<const uint4*>(wk_);                                         \
        w01 = *reinterpret_cast<const uint4*>(wk_ + 8);                                     \
        w10 = *reinterpret_cast<const uint4*>(wk_ + plane);                                 \
        w11 = *reinterpret_cast<const uint4*>(wk_ + plane + 8);                             \
        w20 = *reinterpret_cast<const uint4*>(wk_ + 2 * plane);                             \
        w21 = *reinterpret_cast<const uint4*>(wk_ + 2 * plane + 8);                         \
    }
    const int off0 = sw_off(srow, sq), off1 = sw_off(srow, sq + 1);
    // f32 X rows, 16-B chunk qc = 4 * (t & 1) + i of row srow
// The out-of-range float4s are zeroed here, at the LDS store, not right after their loads:
// a select next to the load makes the wave wait for the data before the chunk's MFMAs (the
// whole fetch latency exposed once per chunk).
#define X6_STORE(kc)                                                                        \
    {                                                                                       \
        X6_XSTORE(kc)                                                                       \
        *reinterpret_cast<uint4*>(&Ws[0][off0]) = w00;                                      \
        *reinterpret_cast<uint4*>(&Ws[0][off1]) = w01;                                      \
        *reinterpret_cast<uint4*>(&Ws[1][off0]) = w10;                                      \
        *reinterpret_cast<uint4*>(&Ws[1][off1]) = w11;                                      \
        *reinterpret_cast<uint4*>(&Ws[2][off0]) = w20;                                      \
        *reinterpret_cast<uint4*>(&Ws[2][off1]) = w21;                                      \
    }
    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
    X6_LOAD(0)
    X6_STORE(0)
    __syncthreads();
    for (int kc = 0; kc < nch; ++kc) {
        if (kc + 1 < nch) X6_LOAD(kc + 1)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // this lane's 8 k of its row (f32), split here: every X element belongs to exactly
            // one wave's rows, so each is split once
            bf16x8 b[NPL];
            {
                const int xr = 32 * w + c;
                const float4 u = *reinterpret_cast<const float4*>(&Xs[swf_off(xr, 4 * s + 2 * h)]);
                const float4 v = *reinterpret_cast<const float4*>(
                    &Xs[swf_off(xr, 4 * s + 2 * h + 1)]);
                split4(u, b[0], b[1], b[2], 0);
                split4(v, b[0], b[1], b[2], 4);
            }
            // two feature tiles at a time, their six products interleaved (two independent
            // accumulation chains in flight)
#pragma unroll
            for (int ip = 0; ip < NT; ip += 2) {
                bf16x8 a0[NPL], a1[NPL];
                const int ao0 = sw_off(32 * ip + c, 2 * s + h);
                const int ao1 = sw_off(32 * (ip + 1) + c, 2 * s + h);
#pragma unroll
                for (int p = 0; p < NPL; ++p) {
                    a0[p] = *reinterpret_cast<const bf16x8*>(&Ws[p][ao0]);
                    a1[p] = *reinterpret_cast<const bf16x8*>(&Ws[p][ao1]);
                }
#define X6_PAIR(pa, pb)                                                                     \
    acc[ip] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[pa], b[pb], acc[ip], 0, 0, 0);     \
    acc[ip + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[pa], b[pb], acc[ip + 1], 0, 0, 0);
                X6_PAIR(0, 0)
                X6_PAIR(0, 1)
                X6_PAIR(1, 0)
                X6_PAIR(0, 2)
                X6_PAIR(1, 1)
                X6_PAIR(2, 0)
#undef X6_PAIR
            }
        }
        if (kc + 1 < nch) {
            __syncthreads();
            X6_STORE(kc + 1)
            __syncthreads();
        }
    }
#undef X6_LOAD
#undef X6_STORE
    // epilogue: bias + tanh; fragment layout (x6::frag_off4) or row-major
    const int64_t bt = (row0 >> 5) + w;
    const int64_t brow = row0 + 32 * w + c;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * i + rho(r) + 4 * h;
            const float z = acc[i][r] + sb[f];
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
// l1_ring_kernel: the same product (bit-identical accumulators: each accumulator sees the
// same k-steps and the same six-product order as l1_fwd_x6_kernel) with an LDS-DMA pipeline
// deep enough to keep the gathered rows streaming from HBM.
//
// Workgroup = 8 waves (2 per SIMD) x 32 rows = 256 rows per tile, all 128 features, up to
// RTPW tiles per workgroup (one row index per lane and piece loaded before the pipeline
// starts, so the K loop issues no ordinary global load).  Per 32-k chunk c (flattened over
// the workgroup's tiles):
//   X(c): every wave copies ITS OWN 32 rows x 128 B by global_load_lds_dwordx4 (4 wave-
//         instructions of 8 rows x 128 B; XOR swizzle applied on the source address, so the
//         lane-linear LDS image is swf_off's), into a 3-stage ring -- issued two chunks ahead
//         and waited for by the issuing wave only (nobody else reads them);
//   W(c): the three split-weight planes of the chunk (24 KB, 3 wave-instructions per wave,
//         x6::sw_off image), into a 2-stage ring -- issued one chunk ahead; one raw s_barrier
//         per chunk publishes them and retires the stage read in chunk c - 1.
// Waits are counted `s_waitcnt vmcnt(N)` in inline asm (the LDS-DMA loads are inline asm
// too, so the compiler inserts no drain of its own); the per-tile epilogue stores count in
// vmcnt and are skipped by the count of the wait that follows them.
// Round 6 (tools/r06_l1diag.sh, profiles/r06_l1_diag.log; diagnostic builds since removed,
// standalone 262144 gathered rows at pitch 384, two passes each): this kernel 224-235 us;
// without the X split (plane 0 reused) 218-223; without any MFMA 150-154; three of the six
// products 176-180; without the W reloads 221-222; without the X reloads 184-186; without the
// per-chunk barrier 223-225; LDS-DMA issue spread over the first MFMA pairs 226-228;
// s_setprio around the MFMAs 243-246.  SQ counters (profiles/r06_l1_pmc.txt): MFMA busy 43 %
// of the wave lifetime, waves issue-stalled 43 %, parked 32 %.  So neither the split VALU nor
// the weight stream nor the barrier bounds it; the MFMA time and the gathered X rows add
// rather than overlap.  A 16-k-chunk form with an 8-stage X ring (twice the chunks in flight,
// 112 KB per CU; bit-identical, 53 MLP / PPO tests green) measured SLOWER, 246-256 us gathered
// and 247-249 contiguous (profiles/r06_l1_deep_ab.log): in-flight depth is not the limit.
// ---------------------------------------------------------------------------------------
constexpr int RNW = 8;                   // waves per workgroup
constexpr int RROWS = 32 * RNW;          // rows per tile
constexpr int RTPW = 4;                  // tiles per workgroup (at most)
constexpr int RWS = 2;                   // W ring stages
constexpr int RXSTAGE = RROWS * XROWB;   // 32 KB
constexpr int RWSTAGE = NPL * HC * ROWB;  // 24 KB

// ---------------------------------------------------------------------------------------
// Fused process_fn evaluation (EVAL = true): the layer-1 ring with the evaluation of
// tsrl_ppo_eval (mlp.hip eval_tail_kernel: layer 2 of both nets, the critic's value head, the
// actor's mu head and the Gaussian log-prob of the stored action) run on each finished tile's
// activations in registers, so H1 never leaves the chip (round 6; the
// two-kernel form writes and re-reads 512 B per row, 1 GB per 2M-row chunk, past the 256 MB
// Infinity Cache).  LDS: a 2-stage X ring (measured as fast as 3 stages, tools/r06_rxs.sh,
// profiles/r06_fused_eval_ab.log), the W ring, and the two layer-2 images (48 KB) = 160 KB;
// the mu-head image and the small constants live in a global workspace built once per call
// (L1 / L2-resident), the layer-1 bias is read from global memory.  Same products in the same
// order as l1_ring_kernel + eval_tail_kernel: bit-identical values and log-probs.
constexpr int EH = 64, EAMAX = 32;
constexpr float E_LOG_SQRT_2PI = 0.91893853320467274178f;
constexpr int EV_W2 = NPL * 2 * EH * 64;         // one layer-2 image (2 chunks of 32 k)
constexpr int EV_W3 = NPL * 2 * EAMAX * 64;      // the mu-head image
// constants (floats): b2a, b2c, b3a (padded), w3c, sigma^2, log sigma
constexpr int EC_B2A = 0, EC_B2C = EC_B2A + EH, EC_B3 = EC_B2C + EH, EC_W3C = EC_B3 + EAMAX,
              EC_VAR = EC_W3C + EH, EC_LS = EC_VAR + EAMAX, EC_B1 = EC_LS + EAMAX,
              EC_END = EC_B1 + 2 * EH;  // + the layer-1 biases (actor, critic), 16-byte aligned
constexpr int EV_WS = EV_W3 + EC_END * 4;        // workspace bytes

template <bool EVAL>
struct RingLds {
    static constexpr int XS = EVAL ? 2 : 3;       // X ring stages
    static constexpr int WOFF = XS * RXSTAGE;
    static constexpr int BOFF = WOFF + RWS * RWSTAGE;  // layer-1 bias / layer-2 images
    static constexpr int SIZE = EVAL ? BOFF + 2 * EV_W2 : BOFF + HC * 4;
};
static_assert(RingLds<true>::SIZE <= 163840, "fused evaluation LDS");

struct EvalArgs {
    const float *w2a, *w2c, *b3c;  // raw layer-2 weights (images built per workgroup)
    const char* w3img;             // workspace: mu-head image, then the constants
    const float* act;              // stored actions [n][A] (null: values only)
    float *value_out, *logp_out;
    int A;
};

__device__ __forceinline__ int ev_img_off(int p, int kc, int row, int q, int nkc, int rows) {
    return (p * nkc + kc) * rows * 64 + sw_off(row, q);
}

// M(row, k) split into an image (layout of mlp.hip build_img_n); TPB threads
template <int TPB, typename F>
__device__ __forceinline__ void ev_build_img(char* img, int rows, int nkc, int t, F val) {
    for (int i = t; i < rows * nkc * 4; i += TPB) {
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
        *reinterpret_cast<bf16x8*>(img + ev_img_off(0, kc, row, q, nkc, rows)) = p0;
        *reinterpret_cast<bf16x8*>(img + ev_img_off(1, kc, row, q, nkc, rows)) = p1;
        *reinterpret_cast<bf16x8*>(img + ev_img_off(2, kc, row, q, nkc, rows)) = p2;
    }
}

__device__ __forceinline__ void ev_ld_img(const char* img, int nkc, int rows, int kc, int row,
                                          int s, int h, bf16x8 (&a)[NPL]) {
#pragma unroll
    for (int p = 0; p < NPL; ++p)
        a[p] = *reinterpret_cast<const bf16x8*>(img + ev_img_off(p, kc, row, 2 * s + h, nkc, rows));
}

__device__ __forceinline__ void ev_split_frag(const float (&v)[16], int s, bf16x8 (&b)[NPL]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 x0, x1, x2;
        split1(v[8 * s + j], x0, x1, x2);
        b[0][j] = x0;
        b[1][j] = x1;
        b[2][j] = x2;
    }
}

__device__ __forceinline__ f32x16 ev_zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.0f;
    return z;
}

// The workspace of a call: the mu-head image (zero rows past A) and the constants, exactly as
// eval_tail_kernel stages them in its LDS.
__global__ __launch_bounds__(256) void eval_ws_kernel(const float* __restrict__ w3a,
                                                      const float* __restrict__ b3a,
                                                      const float* __restrict__ w3c,
                                                      const float* __restrict__ b2a,
                                                      const float* __restrict__ b2c,
                                                      const float* __restrict__ log_std,
                                                      const float* __restrict__ b1a,
                                                      const float* __restrict__ b1c, int A,
                                                      char* __restrict__ ws) {
    const int t = threadIdx.x;
    ev_build_img<256>(ws, EAMAX, 2, t,
                      [=](int r, int k) { return (w3a && r < A) ? w3a[r * EH + k] : 0.0f; });
    float* ec = reinterpret_cast<float*>(ws + EV_W3);
    if (t < EH) {
        ec[EC_B2C + t] = b2c[t];
        ec[EC_W3C + t] = w3c[t];
        ec[EC_B2A + t] = b2a ? b2a[t] : 0.0f;
    }
    if (t < 2 * EH) ec[EC_B1 + t] = t < EH ? b1a[t] : b1c[t - EH];
    if (t < EAMAX) {
        ec[EC_B3 + t] = (b3a && t < A) ? b3a[t] : 0.0f;
        const float sig = (log_std && t < A) ? expf(log_std[t]) : 1.0f;
        ec[EC_VAR + t] = sig * sig;
        ec[EC_LS + t] = logf(sig);
    }
}

// One net of eval_tail_kernel's run_net on a wave's 32 rows: h1 = the net's two layer-1 tiles
// (C layout, after bias and tanh); iw2 = the net's layer-2 image (LDS).
__device__ __forceinline__ void ev_net(int net, const float (&h1a)[16], const float (&h1b)[16],
                                       int64_t brow, bool live, int c, int h, const char* iw2,
                                       const char* iw3, const float* __restrict__ ec,
                                       float b3c, const EvalArgs& ea) {
    const int A = ea.A;
    float av[16];
    if (net == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = rho(r) + 4 * h;
            av[r] = 0.0f;
            if (a < A && live) av[r] = ea.act[brow * A + a];
        }
    }
    const float* sb2 = ec + (net ? EC_B2C : EC_B2A);
    float h2[2][16];
    {
        f32x16 z0 = ev_zero16(), z1 = ev_zero16();
#pragma unroll
        for (int kc = 0; kc < 2; ++kc)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 b[NPL], a[NPL];
                ev_split_frag(kc == 0 ? h1a : h1b, s, b);
                ev_ld_img(iw2, 2, EH, kc, c, s, h, a);
                z0 = mfma6(a, b, z0);
                ev_ld_img(iw2, 2, EH, kc, 32 + c, s, h, a);
                z1 = mfma6(a, b, z1);
            }
        // constants of rows rho(r) + 4h, r = 4g..4g+3: 4 consecutive floats, one 16-byte load
        // (the workspace is 16-byte aligned)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 u = *reinterpret_cast<const float4*>(sb2 + 8 * g + 4 * h);
            const float4 v = *reinterpret_cast<const float4*>(sb2 + 32 + 8 * g + 4 * h);
            const float uu[4] = {u.x, u.y, u.z, u.w}, vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                h2[0][4 * g + e] = tanh_nb(z0[4 * g + e] + uu[e]);
                h2[1][4 * g + e] = tanh_nb(z1[4 * g + e] + vv[e]);
            }
        }
    }
    if (net == 1) {
        float w3[2][16];
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 u = *reinterpret_cast<const float4*>(ec + EC_W3C + 32 * it + 8 * g + 4 * h);
                w3[it][4 * g] = u.x, w3[it][4 * g + 1] = u.y, w3[it][4 * g + 2] = u.z,
                w3[it][4 * g + 3] = u.w;
            }
        float vpart = 0.0f;
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
            for (int r = 0; r < 16; ++r) vpart += w3[it][r] * h2[it][r];
        const float value = vpart + __shfl_xor(vpart, 32, 64) + b3c;
        if (live && h == 0) ea.value_out[brow] = value;
    } else {
        f32x16 mu = ev_zero16();
#pragma unroll
        for (int kc = 0; kc < 2; ++kc)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 b[NPL], a[NPL];
                ev_split_frag(h2[kc], s, b);
                ev_ld_img(iw3, 2, EAMAX, kc, c, s, h, a);
                mu = mfma6(a, b, mu);
            }
        float b3[16], vr[16], ls[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 u = *reinterpret_cast<const float4*>(ec + EC_B3 + 8 * g + 4 * h);
            const float4 v = *reinterpret_cast<const float4*>(ec + EC_VAR + 8 * g + 4 * h);
            const float4 q = *reinterpret_cast<const float4*>(ec + EC_LS + 8 * g + 4 * h);
            b3[4 * g] = u.x, b3[4 * g + 1] = u.y, b3[4 * g + 2] = u.z, b3[4 * g + 3] = u.w;
            vr[4 * g] = v.x, vr[4 * g + 1] = v.y, vr[4 * g + 2] = v.z, vr[4 * g + 3] = v.w;
            ls[4 * g] = q.x, ls[4 * g + 1] = q.y, ls[4 * g + 2] = q.z, ls[4 * g + 3] = q.w;
        }
        float lp = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = rho(r) + 4 * h;
            if (a < A && live) {
                const float diff = av[r] - (mu[r] + b3[r]);
                lp += -(diff * diff) / (2.0f * vr[r]) - ls[r] - E_LOG_SQRT_2PI;
            }
        }
        const float logp = lp + __shfl_xor(lp, 32, 64);
        if (live && h == 0) ea.logp_out[brow] = logp;
    }
}

// One LDS-DMA wave-instruction: lane l copies 16 bytes from src to LDS byte lds + 16 l (M0 is
// set and restored inside the statement; lds is wave-uniform).
__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lds)
        : "memory");
}

template <bool TANH, bool EVAL>
__global__ __launch_bounds__(RNW * 64, 1) void l1_ring_kernel(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ idx, int64_t n,
    int64_t ntiles, int Kp, int dq, const __bf16* __restrict__ wsp, const float* __restrict__ ba,
    const float* __restrict__ bc, float* __restrict__ out, int64_t frag_tiles, int tpw,
    EvalArgs ea) {
    using L = RingLds<EVAL>;
    constexpr int RXS = L::XS, RWOFF = L::WOFF, RBOFF = L::BOFF;
    __shared__ __attribute__((aligned(16))) char sm[L::SIZE];
    const int t = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int l = t & 63, h = l >> 5, c = l & 31;
    // tpw (<= RTPW) tiles per workgroup: RTPW once the grid fills the chip, fewer for small
    // row counts (more workgroups)
    const int64_t tile0 = (int64_t)blockIdx.x * tpw;
    const int ntl = (int)min((int64_t)tpw, ntiles - tile0);
    const int nch = Kp / KC;
    const int C = ntl * nch;
    float* sb = reinterpret_cast<float*>(sm + RBOFF);
    if constexpr (EVAL) {
        // the two layer-2 images (actor, critic), split once per workgroup
        ev_build_img<RNW * 64>(sm + RBOFF, EH, 2, t, [=](int r, int k) { return ea.w2a[r * EH + k]; });
        ev_build_img<RNW * 64>(sm + RBOFF + EV_W2, EH, 2, t,
                               [=](int r, int k) { return ea.w2c[r * EH + k]; });
    } else {
        if (t < HC) sb[t] = t < H ? ba[t] : bc[t - H];
    }
    // source rows of this lane's X pieces: tile tl, instruction i -> local row 32w + 8i + l/8
    // (rows past n, and tiles past ntl, read a real row; the index loads are unconditional)
    uint32_t rid[RTPW][4];
#pragma unroll
    for (int tl = 0; tl < RTPW; ++tl)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t g = (tile0 + tl) * RROWS + 32 * w + 8 * i + (l >> 3);
            rid[tl][i] = (uint32_t)(g < n ? g : n - 1);
        }
    if (idx) {
#pragma unroll
        for (int tl = 0; tl < RTPW; ++tl)
#pragma unroll
            for (int i = 0; i < 4; ++i) rid[tl][i] = (uint32_t)idx[rid[tl][i]];
    }
    __syncthreads();
    const uint32_t lds0 = (uint32_t)(uintptr_t)sm;
    // Issue cursors (wave-uniform): the next X chunk (tile px_tl, chunk px_kc, ring slot px_s)
    // and the next W chunk (chunk pw_kc, slot pw_s).  Per lane: the 4 row bases of the X
    // tile being issued and the lane's piece offsets (XOR swizzle on the source address, so
    // the lane-linear LDS image is swf_off's), the 3 weight-plane sources of the lane.
    int px_tl = 0, px_kc = 0, px_s = 0, pw_kc = 0, pw_s = 0;
    const float* xb[4];
    int xoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 32 * w + 8 * i + (l >> 3);
        xoff[i] = 4 * ((l & 7) ^ ((r >> 1) & 7));
        xb[i] = X;
    }
    const __bf16* wb[3];
    uint32_t wdst[3];
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
        const int j = 3 * w + jj;  // instruction j of the 24: plane j / 8, rows 16 (j % 8) ..
        const int p = j >> 3, row = 16 * (j & 7) + (l >> 2);
        const int q = (l & 3) ^ ((row >> 2) & 3);
        wb[jj] = wsp + p * (int64_t)HC * Kp + (int64_t)row * Kp + 8 * q;
        wdst[jj] = (uint32_t)(RWOFF + p * HC * ROWB + 16 * (j & 7) * ROWB);
    }
    auto issue_x = [&]() {
        if (px_kc == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t ri = 0;
#pragma unroll
                for (int u = 0; u < RTPW; ++u) ri = u == px_tl ? rid[u][i] : ri;
                xb[i] = X + (int64_t)ri * ldx;
            }
        }
        const uint32_t st = lds0 + (uint32_t)(px_s * RXSTAGE + (32 * w) * XROWB);
        const bool last = px_kc == nch - 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int k = px_kc * KC + xoff[i];
            // past the row's data (last chunk only; dq = roundup(D, 4)): column 0, a finite
            // value that meets zero weights -- a padded row pitch (ldx > dq) is never read
            if (last) k = k < dq ? k : 0;
            glds16(xb[i] + k, st + (uint32_t)(i * 8 * XROWB));
        }
        px_s = px_s == RXS - 1 ? 0 : px_s + 1;
        if (++px_kc == nch) {
            px_kc = 0;
            ++px_tl;
        }
    };
    auto issue_w = [&]() {
        const uint32_t st = lds0 + (uint32_t)(pw_s * RWSTAGE);
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) glds16(wb[jj] + pw_kc * KC, st + wdst[jj]);
        pw_s ^= 1;
        if (++pw_kc == nch) pw_kc = 0;
    };
    f32x16 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
    if (C > 0) {
        issue_w();
        issue_x();
        if (RXS > 2 && C > 1) issue_x();
    }
    bool epi_prev = false;
    int cs_x = 0, cs_w = 0;  // ring slots of the chunk being computed
    for (int cc = 0, tl = 0, kc = 0; cc < C; ++cc) {
        // retire W(cc) and X(cc): younger in flight are X(cc + 1) (4) and the previous tile's
        // epilogue stores (16), when they were issued
        // (EVAL: X(cc) is the youngest load -- X is issued one chunk ahead -- and the
        // evaluation epilogue drains everything it issued, so every wait is vmcnt(0))
        const bool nx = cc + 1 < C;
        if (RXS == 2 || !nx) {
            if (epi_prev) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (epi_prev) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        if (nx) issue_w();
        if (cc + RXS - 1 < C) issue_x();
        const char* Xs = sm + cs_x * RXSTAGE;
        const char* Ws = sm + RWOFF + cs_w * RWSTAGE;
        cs_x = cs_x == RXS - 1 ? 0 : cs_x + 1;
        cs_w ^= 1;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 b[NPL];
            {
                const int xr = 32 * w + c;
                const float4 u = *reinterpret_cast<const float4*>(&Xs[swf_off(xr, 4 * s + 2 * h)]);
                const float4 v = *reinterpret_cast<const float4*>(
                    &Xs[swf_off(xr, 4 * s + 2 * h + 1)]);
                split4(u, b[0], b[1], b[2], 0);
                split4(v, b[0], b[1], b[2], 4);
            }
#pragma unroll
            for (int ip = 0; ip < NT; ip += 2) {
                bf16x8 a0[NPL], a1[NPL];
                const int ao0 = sw_off(32 * ip + c, 2 * s + h);
                const int ao1 = sw_off(32 * (ip + 1) + c, 2 * s + h);
#pragma unroll
                for (int p = 0; p < NPL; ++p) {
                    a0[p] = *reinterpret_cast<const bf16x8*>(&Ws[p * HC * ROWB + ao0]);
                    a1[p] = *reinterpret_cast<const bf16x8*>(&Ws[p * HC * ROWB + ao1]);
                }
#define RX6_PAIR(pa, pb)                                                                    \
    acc[ip] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[pa], b[pb], acc[ip], 0, 0, 0);     \
    acc[ip + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[pa], b[pb], acc[ip + 1], 0, 0, 0);
                RX6_PAIR(0, 0)
                RX6_PAIR(0, 1)
                RX6_PAIR(1, 0)
                RX6_PAIR(0, 2)
                RX6_PAIR(1, 1)
                RX6_PAIR(2, 0)
#undef RX6_PAIR
            }
        }
        epi_prev = kc == nch - 1;
        if (EVAL && epi_prev) {
            // bias + tanh, then the evaluation of the wave's 32 rows (eval_tail_kernel's
            // run_net, actor then critic).  The loads issued here are younger than the ring's
            // LDS-DMA loads, so the compiler's waits for them also retire those (vmcnt retires
            // in order); the next chunk's wait is vmcnt(0) (epi_prev = false, X ring of 2)
            const int64_t bt = (tile0 + tl) * (RROWS / 32) + w;
            const int64_t brow = bt * 32 + c;
            const bool live = brow < n;
            const float* ec = reinterpret_cast<const float*>(ea.w3img + EV_W3);
            const float b3c = ea.b3c[0];
            // one net at a time (its two tiles' activations, then its accumulators are
            // free): the register peak of the epilogue
#pragma unroll
            for (int net = 0; net < 2; ++net) {
                float hv[2][16];
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 b4 = *reinterpret_cast<const float4*>(
                            ec + EC_B1 + 64 * net + 32 * ii + 8 * g + 4 * h);
                        const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float z = acc[2 * net + ii][4 * g + e] + bb[e];
                            hv[ii][4 * g + e] = TANH ? tanh_nb(z) : z;
                            acc[2 * net + ii][4 * g + e] = 0.0f;
                        }
                    }
                if (net == 1 || ea.logp_out)
                    ev_net(net, hv[0], hv[1], brow, live, c, h, sm + RBOFF + net * EV_W2,
                           ea.w3img, ec, b3c, ea);
            }
            epi_prev = false;
        } else if (epi_prev) {
            // bias + tanh -> fragment layout (x6::frag_off4)
            const int64_t bt = (tile0 + tl) * (RROWS / 32) + w;
            const bool keep = bt < frag_tiles;
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                float v[16];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 bb = *reinterpret_cast<const float4*>(&sb[32 * i + 8 * g + 4 * h]);
                    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float z = acc[i][4 * g + e] + bv[e];
                        v[4 * g + e] = TANH ? tanh_nb(z) : z;
                        acc[i][4 * g + e] = 0.0f;
                    }
                }
                if (keep) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *reinterpret_cast<float4*>(out + x6::frag_off4(bt * NT + i, l, q)) =
                            make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
                }
            }
            // a tile whose fragments lie past the buffer issues no stores: keep the counted
            // waits exact
            epi_prev = keep;
        }
        if (++kc == nch) {
            kc = 0;
            ++tl;
        }
    }
}

inline int64_t kpad32(int64_t D) { return (D + KC - 1) / KC * KC; }

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_mlp_split_bytes(int64_t D) {
    return D > 0 ? (int64_t)NPL * HC * kpad32(D) * 2 : 0;
}

extern "C" int tsrl_mlp_split_w(const float* Wa, const float* Wc, int64_t D, void* wsplit,
                                void* stream) {
    TSRL_CHECK_ARG(D > 0, "tsrl_mlp_split_w: D <= 0");
    TSRL_CHECK_ARG(Wa && Wc && wsplit, "tsrl_mlp_split_w: null pointer");
    const int64_t total = (int64_t)HC * kpad32(D);
    const unsigned g = (unsigned)std::min<int64_t>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(split_w_kernel, dim3(g), dim3(256), 0, as_stream(stream), Wa, Wc, D,
                       kpad32(D), reinterpret_cast<__bf16*>(wsplit));
    TSRL_LAUNCH_CHECK("tsrl_mlp_split_w");
    return 0;
}

extern "C" int tsrl_mlp_l1_fwd_x6(const float* X, int64_t ldx, const int64_t* idx, int64_t n,
                                  int64_t D, const void* wsplit, const float* ba,
                                  const float* bc, int act_tanh, float* out, int frag_out,
                                  void* stream) {
    TSRL_CHECK_ARG(n >= 0 && D > 0 && ldx >= D, "tsrl_mlp_l1_fwd_x6: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(X && wsplit && ba && bc && out, "tsrl_mlp_l1_fwd_x6: null pointer");
    TSRL_CHECK_ARG(aligned16(X) && ldx % 4 == 0 && ldx >= (D + 3) / 4 * 4 && aligned16(out) &&
                       aligned16(wsplit),
                   "tsrl_mlp_l1_fwd_x6: X/out/wsplit must be 16-byte aligned, ldx a multiple "
                   "of 4 and >= roundup(D, 4) (X columns D..roundup(D,4) finite: zero padding)");
    if (frag_out) {
        // the LDS-DMA pipelined kernel (fragment layout only); frag_tiles = the 32-row tiles
        // of tsrl_mlp_frag_floats(n)
        const int64_t ntiles = (n + RROWS - 1) / RROWS;
        const int64_t frag_tiles = (n + XR - 1) / XR * (XR / 32);
        // tiles per workgroup: RTPW when that still gives a workgroup per CU, fewer below
        // (config 2's 2048-row minibatches: 8 tiles on 8 workgroups instead of 2)
        const int64_t tpw = std::max<int64_t>(1, std::min<int64_t>(RTPW, ntiles / n_cus()));
        const unsigned grid = (unsigned)((ntiles + tpw - 1) / tpw);
        const EvalArgs none{};
        if (act_tanh)
            hipLaunchKernelGGL((l1_ring_kernel<true, false>), dim3(grid), dim3(RNW * 64), 0,
                               as_stream(stream), X, ldx, idx, n, ntiles, (int)kpad32(D),
                               (int)((D + 3) / 4 * 4), reinterpret_cast<const __bf16*>(wsplit),
                               ba, bc, out, frag_tiles, (int)tpw, none);
        else
            hipLaunchKernelGGL((l1_ring_kernel<false, false>), dim3(grid), dim3(RNW * 64), 0,
                               as_stream(stream), X, ldx, idx, n, ntiles, (int)kpad32(D),
                               (int)((D + 3) / 4 * 4), reinterpret_cast<const __bf16*>(wsplit),
                               ba, bc, out, frag_tiles, (int)tpw, none);
        TSRL_LAUNCH_CHECK("tsrl_mlp_l1_fwd_x6(ring)");
        return 0;
    }
    const unsigned grid = (unsigned)((n + XR - 1) / XR);
    hipLaunchKernelGGL(l1_fwd_x6_kernel, dim3(grid), dim3(256), 0, as_stream(stream), X, ldx,
                       idx, n, (int)D, (int)kpad32(D),
                       reinterpret_cast<const __bf16*>(wsplit), ba, bc, act_tanh, out,
                       frag_out);
    TSRL_LAUNCH_CHECK("tsrl_mlp_l1_fwd_x6");
    return 0;
}

extern "C" int64_t tsrl_ppo_eval_fused_workspace_bytes(void) { return EV_WS; }

extern "C" int tsrl_ppo_eval_fused(const float* X, int64_t ldx, const int64_t* idx, int64_t n,
                                   int64_t D, const void* wsplit, const float* ba,
                                   const float* bc, const tsrl_tail_weights* wt,
                                   int64_t act_dim, const float* act, float* value_out,
                                   float* logp_out, void* workspace, int64_t ws_bytes,
                                   void* stream) {
    TSRL_CHECK_ARG(n >= 0 && D > 0 && ldx >= D && act_dim > 0 && act_dim <= EAMAX,
                   "tsrl_ppo_eval_fused: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(X && wsplit && ba && bc && wt && value_out && (!logp_out || act) &&
                       workspace,
                   "tsrl_ppo_eval_fused: null pointer");
    TSRL_CHECK_ARG(wt->w2c && wt->b2c && wt->w3c && wt->b3c &&
                       (!logp_out || (wt->w2a && wt->b2a && wt->w3a && wt->b3a && wt->log_std)),
                   "tsrl_ppo_eval_fused: null weight");
    TSRL_CHECK_ARG(ws_bytes >= EV_WS && aligned16(workspace),
                   "tsrl_ppo_eval_fused: workspace too small or not 16-byte aligned");
    TSRL_CHECK_ARG(aligned16(X) && ldx % 4 == 0 && ldx >= (D + 3) / 4 * 4 && aligned16(wsplit),
                   "tsrl_ppo_eval_fused: X/wsplit must be 16-byte aligned, ldx a multiple of 4 "
                   "and >= roundup(D, 4)");
    hipLaunchKernelGGL(eval_ws_kernel, dim3(1), dim3(256), 0, as_stream(stream),
                       logp_out ? wt->w3a : nullptr, logp_out ? wt->b3a : nullptr, wt->w3c,
                       logp_out ? wt->b2a : nullptr, wt->b2c, logp_out ? wt->log_std : nullptr,
                       ba, bc, (int)act_dim, reinterpret_cast<char*>(workspace));
    TSRL_LAUNCH_CHECK("tsrl_ppo_eval_fused(workspace)");
    const int64_t ntiles = (n + RROWS - 1) / RROWS;
    const int64_t tpw = std::max<int64_t>(1, std::min<int64_t>(RTPW, ntiles / n_cus()));
    const unsigned grid = (unsigned)((ntiles + tpw - 1) / tpw);
    EvalArgs ea{logp_out ? wt->w2a : wt->w2c, wt->w2c, wt->b3c,
                reinterpret_cast<const char*>(workspace), act, value_out, logp_out,
                (int)act_dim};
    hipLaunchKernelGGL((l1_ring_kernel<true, true>), dim3(grid), dim3(RNW * 64), 0,
                       as_stream(stream), X, ldx, idx, n, ntiles, (int)kpad32(D),
                       (int)((D + 3) / 4 * 4), reinterpret_cast<const __bf16*>(wsplit), ba, bc,
                       nullptr, (int64_t)0, (int)tpw, ea);
    TSRL_LAUNCH_CHECK("tsrl_ppo_eval_fused");
    return 0;
}
