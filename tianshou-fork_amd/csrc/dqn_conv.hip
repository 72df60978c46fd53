// First convolution of the Nature-DQN trunk of BASELINE config 5
// (examples/atari/atari_network.py:53-90: Conv2d(4, 32, 8, stride 4) + ReLU over
// scale_obs(frames) = frames / 255, :18-30) straight from the uint8 frame stacks, as an
// implicit GEMM on the bf16 matrix cores.
//
// Exactness: a frame byte u (0..255) is exact in bf16, so the "input" operand needs ONE
// plane; every f32 weight is split exactly into three bf16 pieces (x6.h), so each of the
// three products w_p . u is exact in the f32 MFMA accumulator and the sum over k carries f32
// GEMM error of sum_k w_k u_k.  The output is relu(acc / scale + b): the same function as
// the reference's conv(f32(u / 255)) + b, whose own input rounding (2^-24 relative per
// element) is of the order of that accumulation error.  Three bf16 MFMAs per 16 k instead of
// the six of the f32-f32 split, and the u8 -> f32 frame conversion (and its 4x larger
// activation tensor) disappears from the forward path.
//
// GEMM view: D[32 channels][32 pixels] += W[32][16 k] . P[16 k][32 pixels] per MFMA
// (v_mfma_f32_32x32x16_bf16), k = c*64 + kh*8 + kw, so the 8 k of one lane half are the 8
// consecutive bytes x[c][4 oh + kh][4 ow .. 4 ow + 7] of one input row.  The three split
// planes of W (48 KB) are staged once per workgroup in LDS (rows of 512 B, 16-byte chunks
// XOR-swizzled by row so a ds_read_b128 phase hits distinct banks), each sample's frame stack
// too (dqn_conv1_fwd_lds_kernel below).  Epilogue: bias + ReLU, NHWC f32 output
// ([n][20][20][32], channels_last of [n,32,20,20]).
#include <algorithm>
#include <type_traits>

#include "x6.h"


namespace tsrl {
namespace {

using x6::bf16x8;
using x6::f32x16;
using x6::NPL;

__device__ __forceinline__ int rho(int r) { return (r & 3) + 8 * (r >> 2); }

constexpr int C1_CIN = 4, C1_HW = 84, C1_K = 8, C1_S = 4, C1_OUT = 20, C1_OC = 32;
constexpr int C1_KK = C1_CIN * C1_K * C1_K;       // 256
constexpr int C1_PIX = C1_OUT * C1_OUT;           // 400 output pixels per sample
constexpr int C1_FRAME = C1_CIN * C1_HW * C1_HW;  // 28224 bytes per frame stack
constexpr int C1_ROWB = C1_KK * 2;                // LDS bytes per weight row of one plane

// LDS byte offset of 16-byte chunk q (0..31) of weight row m (0..31) of one plane.
__device__ __forceinline__ int c1_off(int m, int q) { return m * C1_ROWB + 16 * (q ^ (m & 15)); }

// 8 bytes (two little-endian words) -> 8 bf16 (exact: integers 0..255).
__device__ __forceinline__ bf16x8 bytes_to_bf16(uint32_t lo, uint32_t hi) {
    bf16x8 b;
    b[0] = (__bf16)(float)(lo & 0xFF);
    b[1] = (__bf16)(float)((lo >> 8) & 0xFF);
    b[2] = (__bf16)(float)((lo >> 16) & 0xFF);
    b[3] = (__bf16)(float)(lo >> 24);
    b[4] = (__bf16)(float)(hi & 0xFF);
    b[5] = (__bf16)(float)((hi >> 8) & 0xFF);
    b[6] = (__bf16)(float)((hi >> 16) & 0xFF);
    b[7] = (__bf16)(float)(hi >> 24);
    return b;
}

// Round 6: each sample's frame stack staged in LDS.  The round-2..5 kernel (removed) gathered
// every B fragment from global memory: 8-byte loads whose 32 lanes overlap at a 4-byte stride
// (each frame byte fetched 4 times), so the address units, not the matrix cores, set its pace
// (0.45 ms per 8192 samples, 0.14 of the bf16 rate).  Here a workgroup (4 waves, 2 per
// CU: 48 KB weight planes + one 28224-byte frame stack) walks whole samples and a lane's B
// fragment is one ds_read2_b32 of the staged bytes.  The 400 output pixels of a sample are 13
// tiles of 32 (the last half-full): wave w owns tiles w, w + 4, w + 8 (and wave 0 tile 12),
// all of them accumulated together, k-step by k-step, so each weight fragment read from LDS
// serves 3-4 tiles.  The stack is staged in two halves, channels 0-1 (k-steps 0-7) and 2-3
// (8-15): the next sample's half h is loaded into registers (16-byte coalesced) while the
// current sample's products over half h run, and written to LDS after the barrier that ends
// them -- so every wait on those loads sits a half-sample of MFMAs after the loads AND after
// the previous sample's output stores (vmcnt counts both, in order), instead of exposing the
// stores' latency once per sample (the round-6 single-buffer form: 246 us per 8192 samples, of
// which 97 us went to the staging and 64 us to the output stores, tools/r06_dqm.sh).  Every
// accumulator sees the same products in the same order as the gathered kernel did (k-step j =
// 0..15, planes 0, 1, 2); the epilogue's division by scale is a reciprocal product with one fma
// correction (correctly rounded: bit-identical outputs to the gathered kernel at 37 and 8192
// samples, profiles/r06_atari_lds_ab.log), 3 VALU instead of the IEEE division's ~12.
// Measured (tools/atari_kernel_ab.py, 8192 samples, same box): 446-450 us gathered, 229-251
// single-buffer, 252-257 this form; counters (profiles/r06_atari_pmc.txt): MFMA busy 32 %, HBM
// traffic = the algorithmic 227 + 411 MB at 3.0 TB/s, waves parked 37 % and issue-stalled 36 %
// -- latency-bound at the 8 waves per CU that 77.5 KB of LDS per workgroup allow.
constexpr int C1L_HALF = C1_FRAME / 2;           // 14112 bytes: channels 0-1 or 2-3
constexpr int C1L_HV4 = C1L_HALF / 16;           // 882 16-byte pieces per half
constexpr int C1L_HPER = (C1L_HV4 + 255) / 256;  // 4 per thread
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool A16>
__global__ __launch_bounds__(256, 2) void dqn_conv1_fwd_lds_kernel(
    const uint8_t* __restrict__ X, int64_t n, const int64_t* __restrict__ rows,
    const float* __restrict__ W, int64_t sw0,
    int64_t sw1, int64_t sw2, int64_t sw3, const float* __restrict__ bias, float scale,
    int relu, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) char Ws[NPL][C1_OC * C1_ROWB];
    __shared__ __attribute__((aligned(16))) uint8_t Fs[C1_FRAME];
    __shared__ float sb[C1_OC];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    for (int i = t; i < C1_OC * C1_KK; i += 256) {
        const int m = i / C1_KK, k = i - m * C1_KK;
        const int ci = k >> 6, kh = (k >> 3) & 7, kw = k & 7;
        const float v = W[m * sw0 + ci * sw1 + kh * sw2 + kw * sw3];
        __bf16 a0, a1, a2;
        x6::split1(v, a0, a1, a2);
        const int o = c1_off(m, k >> 3) + 2 * (k & 7);
        *reinterpret_cast<__bf16*>(&Ws[0][o]) = a0;
        *reinterpret_cast<__bf16*>(&Ws[1][o]) = a1;
        *reinterpret_cast<__bf16*>(&Ws[2][o]) = a2;
    }
    if (t < C1_OC) sb[t] = bias ? bias[t] : 0.0f;
    const float inv_scale = 1.0f / scale;
    // half hf of a frame stack: 16-byte pieces t + 256 i held in registers (a frame base that
    // is only 4-byte aligned: copied word by word at the store instead); macros, not lambdas
    // over the array (a lambda capturing it put it in scratch memory), and a native vector
    // type (an array of HIP's uint4 stays in scratch too)
    u32x4 fr[C1L_HPER];
#define C1L_SRC(smp) (X + (rows ? rows[smp] : (smp)) * C1_FRAME)
#define C1L_LOAD(smp, hf)                                                                   \
    { if constexpr (A16) {                                                                  \
        const u32x4* src_ =                                                                 \
            reinterpret_cast<const u32x4*>(C1L_SRC(smp)) + (hf) * C1L_HV4;                  \
        _Pragma("unroll") for (int i = 0; i < C1L_HPER; ++i)                                \
            fr[i] = src_[t + 256 * i < C1L_HV4 ? t + 256 * i : 0];                          \
    } }
#define C1L_STORE(smp, hf)                                                                  \
    { if constexpr (A16) {                                                                  \
        _Pragma("unroll") for (int i = 0; i < C1L_HPER; ++i)                                \
            if (t + 256 * i < C1L_HV4)                                                      \
                reinterpret_cast<u32x4*>(Fs + (hf) * C1L_HALF)[t + 256 * i] = fr[i];        \
    } else {                                                                                \
        const uint32_t* src_ =                                                              \
            reinterpret_cast<const uint32_t*>(C1L_SRC(smp) + (hf) * C1L_HALF);              \
        for (int q = t; q < C1L_HALF / 4; q += 256)                                         \
            reinterpret_cast<uint32_t*>(Fs + (hf) * C1L_HALF)[q] = src_[q];                 \
    } }
    // the sample loop of a wave owning NT tiles (3, or 4 for wave 0)
    auto run = [&](auto nt_c) {
        constexpr int NT = decltype(nt_c)::value;
        int bo[NT];
        bool vt[NT];
        int pt[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            pt[i] = 32 * (w + 4 * i) + c;
            vt[i] = pt[i] < C1_PIX;
            const int q = vt[i] ? pt[i] : 0;
            const int oh = q / C1_OUT, ow = q - oh * C1_OUT;
            bo[i] = (C1_S * oh + h) * C1_HW + C1_S * ow;
        }
        f32x16 acc[NT];
        // k-steps j0 .. j0 + 7 (one half of the stack) into every tile's accumulator
        auto half = [&](int j0) {
#pragma unroll 2
            for (int j = j0; j < j0 + 8; ++j) {
                const int off = (j >> 2) * (C1_HW * C1_HW) + 2 * (j & 3) * C1_HW;
                const int ao = c1_off(c, 2 * j + h);
                const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(&Ws[0][ao]);
                const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(&Ws[1][ao]);
                const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(&Ws[2][ao]);
                bf16x8 b[NT];
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    const uint32_t* f = reinterpret_cast<const uint32_t*>(Fs + bo[i] + off);
                    b[i] = bytes_to_bf16(f[0], f[1]);
                }
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, b[i], acc[i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, b[i], acc[i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, b[i], acc[i], 0, 0, 0);
            }
        };
        for (int64_t smp = blockIdx.x; smp < n; smp += gridDim.x) {
            const int64_t nx = smp + gridDim.x;
            const bool more = nx < n;
#pragma unroll
            for (int i = 0; i < NT; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
            if (more) C1L_LOAD(nx, 0)
            half(0);
            __syncthreads();  // channels 0-1 of smp are done with
            if (more) C1L_STORE(nx, 0)
            if (more) C1L_LOAD(nx, 1)
            half(8);
            __syncthreads();  // channels 2-3 of smp are done with (and nx's 0-1 are staged)
            if (more) C1L_STORE(nx, 1)
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                if (vt[i]) {
                    float4* o_ = reinterpret_cast<float4*>(out + (smp * C1_PIX + pt[i]) * C1_OC);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float v_[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float x_ = acc[i][4 * q + e];
                            const float q0_ = x_ * inv_scale;
                            const float qt_ = fmaf(fmaf(-q0_, scale, x_), inv_scale, q0_);
                            const float z_ = qt_ + sb[8 * q + 4 * h + e];
                            v_[e] = relu ? fmaxf(z_, 0.0f) : z_;
                        }
                        o_[2 * q + h] = make_float4(v_[0], v_[1], v_[2], v_[3]);
                    }
                }
            }
        }
    };
    // the first sample of the workgroup, staged whole
    if (blockIdx.x < n) {
        C1L_LOAD((int64_t)blockIdx.x, 0)
        C1L_STORE((int64_t)blockIdx.x, 0)
        C1L_LOAD((int64_t)blockIdx.x, 1)
        C1L_STORE((int64_t)blockIdx.x, 1)
    }
    __syncthreads();
    if (w == 0)
        run(std::integral_constant<int, 4>{});
    else
        run(std::integral_constant<int, 3>{});
#undef C1L_SRC
#undef C1L_LOAD
#undef C1L_STORE
}

// ---------------------------------------------------------------------------------------
// Data gradient of the second convolution (Conv2d(32, 64, 4, stride 2): [n,32,20,20] ->
// [n,64,9,9]) as a bf16x6 implicit GEMM, the ReLU mask of its input (the first layer's
// output z1) fused into the epilogue: dX1 = (z1 > 0) * conv_transpose(gy2, W2).
// Input pixel (ih, iw) receives the 2x2 taps kh = ih%2 + 2 th, kw = iw%2 + 2 tw from output
// pixel (ih/2 - th, iw/2 - tw) when that lies inside the 9x9 map, so the pixels of one parity
// class (ih%2, iw%2) share one sub-kernel: D[32 ci][32 px] += Wc[32 ci][16 k] . G[16 k][32 px]
// with k = (tap, co), 4 taps x 64 channels = 256; every class's split sub-kernel is 3 planes
// of 48 KB (same swizzled rows as conv1).
constexpr int C2_CI = 32, C2_CO = 64, C2_IN = 20, C2_OUT = 9;
constexpr int C2_CPIX = (C2_IN / 2) * (C2_IN / 2);  // 100 input pixels per class per sample

// Round 6: each sample's gy2 staged in LDS, split once.  The round-2..5 kernel (removed)
// gathered 32 16-byte pieces of gy2 per lane and tile from global memory (each gy2 element
// fetched by 16 lanes across the 4 classes and taps) and split every piece it used; splitting
// gy2 into bf16 planes in a separate pass had measured slower for it (0.80 vs 0.60 ms).  Here a
// workgroup (4 waves per class it serves; its classes' 48 KB split sub-kernels + 31.5 KB of
// gy2 planes) walks whole samples: the next sample's 81 x 64 gy2 values are loaded into
// registers (16-byte coalesced) during the current sample's MFMAs, then split into the three
// bf16 planes of an LDS image [82 pixels][64 co] (row 81 stays zero: the taps that fall
// outside the 9 x 9 map read it) between two barriers.  A lane's B fragment is one
// ds_read_b128 per plane (16-byte chunks XOR-swizzled by pixel / 2: a 128-byte row spans half
// the 64 banks, so the 16 lanes of a read phase -- 16 different pixels -- hit distinct banks
// when both the row parity and the swizzled chunk differ).  The 100 input pixels of the class
// are 4 tiles of 32, one per wave (the last holds 4).  Every accumulator sees the same split
// values and products in the same order as the gathered kernel did: bit-identical outputs.
constexpr int C2L_PX = C2_OUT * C2_OUT;         // 81 gy2 pixels per sample
constexpr int C2L_ROW = C2_CO * 2;              // 128 bytes per image row (64 bf16)
constexpr int C2L_PLANE = (C2L_PX + 1) * C2L_ROW;
constexpr int C2L_V4 = C2L_PX * C2_CO / 4;      // 1296 float4 pieces per sample
typedef float f32x4n __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int c2l_off(int px, int q) {
    return px * C2L_ROW + 16 * (q ^ ((px >> 1) & 7));
}
__device__ __forceinline__ uint32_t bf2(__bf16 lo, __bf16 hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, lo) |
           ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
}

// NCL classes per workgroup (4 NCL waves, wave w: class NCL * blockIdx.y + w / 4, tile w % 4):
// the staged gy2 image serves NCL classes, so it is loaded and split 4 / NCL times per sample
// instead of 4.  NCL = 2: 96 KB of sub-kernels + the image, one 8-wave workgroup per CU.
template <int NCL>
__global__ __launch_bounds__(256 * NCL, 2 / NCL) void dqn_conv2_dgrad_lds_kernel(
    const float* __restrict__ gy, int64_t n, const float* __restrict__ W, int64_t sw0,
    int64_t sw1, int64_t sw2, int64_t sw3, const float* __restrict__ z1,
    float* __restrict__ dx) {
    constexpr int NTH = 256 * NCL;
    constexpr int PER = (C2L_V4 + NTH - 1) / NTH;
    __shared__ __attribute__((aligned(16))) char Ws[NCL][NPL][C2_CI * C1_ROWB];
    __shared__ __attribute__((aligned(16))) char Gs[NPL][C2L_PLANE];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    for (int i = t; i < NCL * C2_CI * 256; i += NTH) {
        const int cl = i / (C2_CI * 256), r = i - cl * (C2_CI * 256);
        const int cls = NCL * blockIdx.y + cl, ph = cls >> 1, pw = cls & 1;
        const int ci = r >> 8, k = r & 255;
        const int tap = k >> 6, co = k & 63;
        const int kh = ph + 2 * (tap >> 1), kw = pw + 2 * (tap & 1);
        const float v = W[co * sw0 + ci * sw1 + kh * sw2 + kw * sw3];
        __bf16 a0, a1, a2;
        x6::split1(v, a0, a1, a2);
        const int o = c1_off(ci, k >> 3) + 2 * (k & 7);
        *reinterpret_cast<__bf16*>(&Ws[cl][0][o]) = a0;
        *reinterpret_cast<__bf16*>(&Ws[cl][1][o]) = a1;
        *reinterpret_cast<__bf16*>(&Ws[cl][2][o]) = a2;
    }
    if (t < C2L_ROW / 4) {  // the zero row
#pragma unroll
        for (int p = 0; p < NPL; ++p)
            *reinterpret_cast<uint32_t*>(&Gs[p][C2L_PX * C2L_ROW + 4 * t]) = 0u;
    }
    // this wave's tile: class cls, input pixel p = 32 (w % 4) + c, the gy2 pixel of each tap
    const int wl = w >> 2;
    const int cls = NCL * blockIdx.y + wl, ph = cls >> 1, pw = cls & 1;
    const char* Wc = &Ws[wl][0][0];
    const int p = 32 * (w & 3) + c;
    const bool live = p < C2_CPIX;
    const int ih = 2 * ((live ? p : 0) / 10) + ph, iw = 2 * ((live ? p : 0) % 10) + pw;
    int tpx[4];
#pragma unroll
    for (int tap = 0; tap < 4; ++tap) {
        const int oh = (ih >> 1) - (tap >> 1), ow = (iw >> 1) - (tap & 1);
        const bool ok = live && oh >= 0 && oh < C2_OUT && ow >= 0 && ow < C2_OUT;
        tpx[tap] = ok ? oh * C2_OUT + ow : C2L_PX;
    }
    f32x4n gr[PER];
#define C2L_LOAD(smp)                                                                       \
    {                                                                                       \
        const f32x4n* src_ = reinterpret_cast<const f32x4n*>(gy + (smp) * (C2L_PX * C2_CO)); \
        _Pragma("unroll") for (int i = 0; i < PER; ++i)                                     \
            gr[i] = src_[t + NTH * i < C2L_V4 ? t + NTH * i : 0];                           \
    }
    /* piece i: pixel q / 16, channels 4 (q % 16) .. + 3 -> 8 bytes of each plane */        \
#define C2L_STORE()                                                                         \
    {                                                                                       \
        _Pragma("unroll") for (int i = 0; i < PER; ++i) {                                   \
            const int q_ = t + NTH * i;                                                     \
            if (q_ < C2L_V4) {                                                              \
                const int px_ = q_ >> 4, c4_ = q_ & 15;                                     \
                const int o_ = c2l_off(px_, c4_ >> 1) + 8 * (c4_ & 1);                      \
                uint32_t pk_[NPL][2];                                                       \
                _Pragma("unroll") for (int e = 0; e < 4; e += 2) {                          \
                    __bf16 x0_, x1_, x2_, y0_, y1_, y2_;                                    \
                    x6::split1(gr[i][e], x0_, x1_, x2_);                                    \
                    x6::split1(gr[i][e + 1], y0_, y1_, y2_);                                \
                    pk_[0][e >> 1] = bf2(x0_, y0_);                                         \
                    pk_[1][e >> 1] = bf2(x1_, y1_);                                         \
                    pk_[2][e >> 1] = bf2(x2_, y2_);                                         \
                }                                                                           \
                _Pragma("unroll") for (int pp = 0; pp < NPL; ++pp)                          \
                    *reinterpret_cast<uint2*>(&Gs[pp][o_]) = make_uint2(pk_[pp][0], pk_[pp][1]); \
            }                                                                               \
        }                                                                                   \
    }
    int64_t smp = blockIdx.x;
    if (smp < n) C2L_LOAD(smp)
    for (; smp < n; smp += gridDim.x) {
        __syncthreads();  // the previous sample's B reads are done (and, first, Ws / zero row)
        C2L_STORE()
        __syncthreads();
        if (smp + gridDim.x < n) C2L_LOAD(smp + gridDim.x)
        const int64_t o = ((smp * C2_IN + ih) * C2_IN + iw) * C2_CI;
        f32x4n zm[4];
        if (live && z1) {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
                zm[qq] = reinterpret_cast<const f32x4n*>(z1 + o)[2 * qq + h];
        }
        f32x16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
#pragma unroll 1
        for (int tap = 0; tap < 4; ++tap) {
          const int tp = tap == 0 ? tpx[0] : tap == 1 ? tpx[1] : tap == 2 ? tpx[2] : tpx[3];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * tap + jj;
            const int bo = c2l_off(tp, 2 * jj + h);
            const int ao = c1_off(c, 2 * j + h);
            bf16x8 a[NPL], b[NPL];
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) {
                b[pl] = *reinterpret_cast<const bf16x8*>(&Gs[pl][bo]);
                a[pl] = *reinterpret_cast<const bf16x8*>(Wc + pl * (C2_CI * C1_ROWB) + ao);
            }
            acc = x6::mfma6(a, b, acc);
          }
        }
        if (live) {
            float4* d = reinterpret_cast<float4*>(dx + o);
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                float4 v = make_float4(acc[4 * qq], acc[4 * qq + 1], acc[4 * qq + 2],
                                       acc[4 * qq + 3]);
                if (z1) {
                    v.x = zm[qq][0] > 0.0f ? v.x : 0.0f;
                    v.y = zm[qq][1] > 0.0f ? v.y : 0.0f;
                    v.z = zm[qq][2] > 0.0f ? v.z : 0.0f;
                    v.w = zm[qq][3] > 0.0f ? v.w : 0.0f;
                }
                d[2 * qq + h] = v;
            }
        }
    }
#undef C2L_LOAD
#undef C2L_STORE
}

// ---------------------------------------------------------------------------------------
// Weight and bias gradient of the first convolution straight from the uint8 frames:
// dW1[co][k] = (sum_p gy1[p][co] * u[p][k]) / scale, db1[co] = sum_p gy1[p][co], where p runs
// over every output pixel of the minibatch and u[p][k] is the frame byte under tap k of pixel
// p (k = ci*64 + kh*8 + kw, the NCHW order of W1).  The reference's weight gradient
// (loss.backward(), ppo.py:146, through scale_obs + Conv2d, atari_network.py:18-30,53-90)
// multiplies gy1 by f32(u / 255); here the bytes are exact bf16 values and gy1 is split exactly
// into three bf16 planes, so each product is exact in the f32 accumulator and the division
// by scale happens once per weight (f32 GEMM error, like the forward kernel above).  This also
// removes the u8 -> f32 frame conversion the MIOpen weight gradient needs.
// GEMM view: D[32 co][32 k] += G^T[32 co][16 px] . P[16 px][32 k] (v_mfma_f32_32x32x16_bf16,
// three per 16 pixels: one per plane of G).  A workgroup walks a contiguous range of
// 128-pixel chunks (flat pixel index over the batch; chunks may straddle samples).  Per chunk
// it stages the im2col bytes as Pb[k][128 px] (each thread copies the 8-byte runs
// u[p][ci][4oh+kh][4ow..+7] of 4 pixels and re-packs them as 4-pixel dwords of 8 k rows) and the
// gradient rows as split planes Gs[plane][co][128 px]; wave w owns the 64 taps of input channel
// w (two 32-k tiles).  Partial sums per workgroup, folded in fixed order by
// dqn_conv1_wgrad_reduce_kernel (f64).  32-pixel chunks: 345 us + a 147 us single-thread-per-
// output fold per 8192 rows; the chunk size amortises the two barriers per chunk.
constexpr int C1W_CH = 128;                   // pixels per chunk
constexpr int C1W_J = C1W_CH / 32;            // staging repeats per thread
constexpr int C1W_PR = C1W_CH + 8;            // Pb row pitch (bytes; 34 dwords at 128 px:
                                              // conflict-free b64 fragment reads)
constexpr int C1W_GR = 2 * C1W_CH + 16;       // Gs row pitch (bytes; 68 dwords: conflict-free
                                              // b128 phases)

__global__ __launch_bounds__(256, 2) void dqn_conv1_wgrad_kernel(
    const uint8_t* __restrict__ X, const int64_t* __restrict__ rows, const float* __restrict__ gy,
    int64_t npix, int64_t cpw, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) uint8_t Pb[C1_KK * C1W_PR];        // [k][px]
    __shared__ __attribute__((aligned(16))) uint8_t Gs[NPL][C1_OC * C1W_GR];   // [co][px] bf16
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int64_t nchunk = (npix + C1W_CH - 1) / C1W_CH;
    const int64_t c0 = (int64_t)blockIdx.x * cpw;
    const int64_t c1 = min(nchunk, c0 + cpw);
    // staging roles: im2col run q = t >> 3 (ci = q >> 3, kh = q & 7) of the pixel quads
    // 4 (pg + 8 j) .. + 3, pg = t & 7: 8 bytes per pixel, re-packed as 4-pixel dwords of the 8
    // rows k = 8q + kw; gradient float4s (channels 4gq..4gq+3, gq = (t >> 4) & 7) of the pixel
    // pairs 2 gp + 32 (2 jj + hf) + {0, 1}, gp = t & 15, hf = t >> 7, jj = 0, 1 -- so each
    // split plane takes one 4-byte store per channel and pair, and the 32 lanes of a store
    // phase (16 pairs x 2 channel groups) hit 32 distinct banks (round 6: the earlier 2-byte
    // store per pixel and plane, lanes spread over channels, made 52 % of this kernel's LDS
    // cycles bank conflicts, profiles/r06_atari_pmc.txt)
    const int q = t >> 3, pg = t & 7;
    const int gq = (t >> 4) & 7, gp = t & 15, hf = t >> 7;
    const int qoff = (q >> 3) * (C1_HW * C1_HW) + (q & 7) * C1_HW;  // channel + kernel row
    // A pixel quad 4m..4m+3 never straddles an output row or a sample (20 and 400 are
    // multiples of 4, and so is npix), so its 4 eight-byte runs are the 20-byte window
    // u[4 ow0 .. 4 ow0 + 19] of one input row: 5 dword loads, and kernel column kw of pixel i
    // is byte (kw & 3) of window dword (kw >> 2) + i.
    uint32_t rb[C1W_J][5];
    float4 gv[C1W_J];
    float db[4] = {0.f, 0.f, 0.f, 0.f};
#define C1W_LOAD(ch)                                                                        \
    {                                                                                       \
        _Pragma("unroll") for (int j = 0; j < C1W_J; ++j) {                                 \
            /* 32-bit pixel arithmetic (npix < 2^31, checked on the host): the divisions  */ \
            /* by the constants 400 and 20 become multiply-high + shift                   */ \
            const uint32_t p_ = (uint32_t)(ch) * C1W_CH + 4u * (pg + 8 * j);                \
            const uint32_t pp_ = p_ < (uint32_t)npix ? p_ : 0u;                             \
            const uint32_t s_ = pp_ / (uint32_t)C1_PIX;                                     \
            const uint32_t rr_ = pp_ - s_ * C1_PIX, oh_ = rr_ / (uint32_t)C1_OUT;           \
            const uint32_t ow_ = rr_ - oh_ * C1_OUT;                                        \
            const int64_t fs_ = rows ? rows[s_] : (int64_t)s_;                              \
            const uint32_t* a_ = reinterpret_cast<const uint32_t*>(                         \
                X + fs_ * C1_FRAME + qoff + C1_S * oh_ * C1_HW + C1_S * ow_);                \
            _Pragma("unroll") for (int d = 0; d < 5; ++d) rb[j][d] = a_[d];                 \
            const int64_t g_ = (ch) * C1W_CH + 2 * gp + 32 * (2 * (j >> 1) + hf) + (j & 1); \
            gv[j] = *reinterpret_cast<const float4*>(gy + (g_ < npix ? g_ : 0) * C1_OC + 4 * gq); \
        }                                                                                   \
    }
#define C1W_STORE(ch)                                                                       \
    {                                                                                       \
        _Pragma("unroll") for (int j = 0; j < C1W_J; ++j) {                                 \
            const int px0_ = 4 * (pg + 8 * j);                                              \
            const uint32_t m_ = (ch) * C1W_CH + px0_ < npix ? 0xFFFFFFFFu : 0u;              \
            _Pragma("unroll") for (int e = 0; e < 8; ++e) {                                 \
                const int k0_ = e >> 2;                                                     \
                const uint32_t b_ = (uint32_t)(e & 3);                                      \
                const uint32_t lo_ = __builtin_amdgcn_perm(                                 \
                    rb[j][k0_ + 1], rb[j][k0_], b_ | ((4u + b_) << 8) | 0x0C0C0000u);        \
                const uint32_t hi_ = __builtin_amdgcn_perm(                                 \
                    rb[j][k0_ + 3], rb[j][k0_ + 2], 0x00000C0Cu | (b_ << 16) | ((4u + b_) << 24)); \
                *reinterpret_cast<uint32_t*>(&Pb[(8 * q + e) * C1W_PR + px0_]) =            \
                    (lo_ | hi_) & m_;                                                       \
            }                                                                               \
        }                                                                                   \
        _Pragma("unroll") for (int jj = 0; jj < 2; ++jj) {                                  \
            const int px_ = 2 * gp + 32 * (2 * jj + hf);                                    \
            const bool ok0_ = (ch) * C1W_CH + px_ < npix;                                   \
            const bool ok1_ = (ch) * C1W_CH + px_ + 1 < npix;                               \
            const float4 u_ = gv[2 * jj], v_ = gv[2 * jj + 1];                              \
            const float ga_[4] = {ok0_ ? u_.x : 0.f, ok0_ ? u_.y : 0.f,                     \
                                  ok0_ ? u_.z : 0.f, ok0_ ? u_.w : 0.f};                    \
            const float gb_[4] = {ok1_ ? v_.x : 0.f, ok1_ ? v_.y : 0.f,                     \
                                  ok1_ ? v_.z : 0.f, ok1_ ? v_.w : 0.f};                    \
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                 \
                __bf16 a0_, a1_, a2_, b0_, b1_, b2_;                                        \
                x6::split1(ga_[e], a0_, a1_, a2_);                                          \
                x6::split1(gb_[e], b0_, b1_, b2_);                                          \
                const int o_ = (4 * gq + e) * C1W_GR + 2 * px_;                             \
                *reinterpret_cast<uint32_t*>(&Gs[0][o_]) = bf2(a0_, b0_);                   \
                *reinterpret_cast<uint32_t*>(&Gs[1][o_]) = bf2(a1_, b1_);                   \
                *reinterpret_cast<uint32_t*>(&Gs[2][o_]) = bf2(a2_, b2_);                   \
                db[e] += ga_[e] + gb_[e];                                                   \
            }                                                                               \
        }                                                                                   \
    }
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.0f;
    if (c0 < c1) {
        C1W_LOAD(c0)
        C1W_STORE(c0)
    }
    __syncthreads();
    for (int64_t ch = c0; ch < c1; ++ch) {
        if (ch + 1 < c1) C1W_LOAD(ch + 1)
#pragma unroll
        for (int s = 0; s < C1W_CH / 16; ++s) {
            const int po = 16 * s + 8 * h;
            bf16x8 a[NPL];
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl)
                a[pl] = *reinterpret_cast<const bf16x8*>(&Gs[pl][c * C1W_GR + 2 * po]);
            const uint2 u0 = *reinterpret_cast<const uint2*>(&Pb[(64 * w + c) * C1W_PR + po]);
            const uint2 u1 =
                *reinterpret_cast<const uint2*>(&Pb[(64 * w + 32 + c) * C1W_PR + po]);
            const bf16x8 b0 = bytes_to_bf16(u0.x, u0.y), b1 = bytes_to_bf16(u1.x, u1.y);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b1, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b1, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b1, acc1, 0, 0, 0);
        }
        if (ch + 1 < c1) {
            __syncthreads();
            C1W_STORE(ch + 1)
            __syncthreads();
        }
    }
#undef C1W_LOAD
#undef C1W_STORE
    // partial slab of this workgroup: [32 co][256 k] then db[32]
    float* o = part + (int64_t)blockIdx.x * (C1_OC * C1_KK + C1_OC);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int co = rho(r) + 4 * h;
        o[co * C1_KK + 64 * w + c] = acc0[r];
        o[co * C1_KK + 64 * w + 32 + c] = acc1[r];
    }
    // db: the 32 pixel slots of each channel, summed in slot order
    __syncthreads();
    float* red = reinterpret_cast<float*>(Pb);  // [32 slots][32 co]
#pragma unroll
    for (int e = 0; e < 4; ++e) red[(gp + 16 * hf) * C1_OC + 4 * gq + e] = db[e];
    __syncthreads();
    if (t < C1_OC) {
        float sacc = 0.0f;
        for (int i = 0; i < 32; ++i) sacc += red[i * C1_OC + t];
        o[C1_OC * C1_KK + t] = sacc;
    }
}

// Fixed-order fold of the per-workgroup slabs: block = 64 outputs x 4 lane groups; group g
// sums slabs g, g + 4, ... in f64 with 4 independent accumulators (loads stay in flight), then
// the groups combine in order through LDS.
__global__ __launch_bounds__(256) void dqn_conv1_wgrad_reduce_kernel(
    const float* __restrict__ part, int nslab, float inv_scale, float* __restrict__ gw,
    float* __restrict__ gb) {
    constexpr int W = C1_OC * C1_KK + C1_OC;
    __shared__ double sh[4][64];
    const int o = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + o;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (i < W) {
        int k = g;
        for (; k + 12 < nslab; k += 16) {
            a0 += (double)part[(int64_t)k * W + i];
            a1 += (double)part[(int64_t)(k + 4) * W + i];
            a2 += (double)part[(int64_t)(k + 8) * W + i];
            a3 += (double)part[(int64_t)(k + 12) * W + i];
        }
        for (; k < nslab; k += 4) a0 += (double)part[(int64_t)k * W + i];
    }
    sh[g][o] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (g != 0 || i >= W) return;
    const double s = ((sh[0][o] + sh[1][o]) + sh[2][o]) + sh[3][o];
    if (i < C1_OC * C1_KK) gw[i] = (float)(s * (double)inv_scale);
    else if (gb) gb[i - C1_OC * C1_KK] = (float)s;
}

// Bias + ReLU in place over NHWC rows (rows x C, C % 4 == 0): the epilogue of a library
// convolution run without bias, one pass instead of torch's bias add and ReLU (two passes
// over the activation).  y = max(y + b, 0) in f32, the same values as add then clamp_min.
__global__ __launch_bounds__(256) void bias_relu_rows_kernel(float4* __restrict__ y,
                                                             const float4* __restrict__ b,
                                                             int64_t n4, int c4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * 256) {
        const float4 bb = b ? b[i % c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 v = y[i];
        v.x = fmaxf(v.x + bb.x, 0.0f);
        v.y = fmaxf(v.y + bb.y, 0.0f);
        v.z = fmaxf(v.z + bb.z, 0.0f);
        v.w = fmaxf(v.w + bb.w, 0.0f);
        y[i] = v;
    }
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_dqn_conv1_fwd(const uint8_t* frames, int64_t n, const int64_t* rows,
                                  const float* w, int64_t sw0, int64_t sw1, int64_t sw2,
                                  int64_t sw3, const float* bias, float scale, int relu,
                                  float* out, void* stream) {
    TSRL_CHECK_ARG(n >= 0, "tsrl_dqn_conv1_fwd: n < 0");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(frames && w && out, "tsrl_dqn_conv1_fwd: null pointer");
    TSRL_CHECK_ARG((((uintptr_t)frames) & 3) == 0 && aligned16(out),
                   "tsrl_dqn_conv1_fwd: frames must be 4-byte and out 16-byte aligned");
    TSRL_CHECK_ARG(scale > 0.0f, "tsrl_dqn_conv1_fwd: scale must be > 0");
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // one persistent workgroup per sample up to two per CU
    const int64_t grid = std::min<int64_t>(n, (int64_t)ncu * 2);
    if (aligned16(frames))
        hipLaunchKernelGGL(dqn_conv1_fwd_lds_kernel<true>, dim3((unsigned)grid), dim3(256), 0,
                           as_stream(stream), frames, n, rows, w, sw0, sw1, sw2, sw3, bias,
                           scale, relu, out);
    else
        hipLaunchKernelGGL(dqn_conv1_fwd_lds_kernel<false>, dim3((unsigned)grid), dim3(256), 0,
                           as_stream(stream), frames, n, rows, w, sw0, sw1, sw2, sw3, bias,
                           scale, relu, out);
    TSRL_LAUNCH_CHECK("tsrl_dqn_conv1_fwd");
    return 0;
}

extern "C" int tsrl_dqn_conv2_dgrad(const float* gy, int64_t n, const float* w, int64_t sw0,
                                    int64_t sw1, int64_t sw2, int64_t sw3, const float* z1,
                                    float* dx, void* stream) {
    TSRL_CHECK_ARG(n >= 0, "tsrl_dqn_conv2_dgrad: n < 0");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(gy && w && dx, "tsrl_dqn_conv2_dgrad: null pointer");
    TSRL_CHECK_ARG(aligned16(gy) && aligned16(dx) && (!z1 || aligned16(z1)),
                   "tsrl_dqn_conv2_dgrad: gy / dx / z1 must be 16-byte aligned");
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // 4 / NCL class groups x gx persistent workgroups (samples bx, bx + gx, ...): 2 workgroups
    // of one class per CU, or one of two classes
    constexpr int NCL = 2;  // profiles/r06_atari_pmc.txt: 474-486 us vs 499-507 at NCL = 1
    const int64_t gx = std::max<int64_t>(1, std::min<int64_t>(n, (int64_t)ncu * NCL / 2));
    hipLaunchKernelGGL(dqn_conv2_dgrad_lds_kernel<NCL>, dim3((unsigned)gx, 4 / NCL),
                       dim3(256 * NCL), 0, as_stream(stream), gy, n, w, sw0, sw1, sw2, sw3, z1,
                       dx);
    TSRL_LAUNCH_CHECK("tsrl_dqn_conv2_dgrad");
    return 0;
}

extern "C" int64_t tsrl_dqn_conv1_wgrad_workspace_bytes(int64_t n) {
    if (n <= 0) return 0;
    const int64_t nchunk = (n * C1_PIX + C1W_CH - 1) / C1W_CH;
    const int64_t nwg = std::min<int64_t>(nchunk, 512);
    return nwg * (C1_OC * C1_KK + C1_OC) * (int64_t)sizeof(float);
}

extern "C" int tsrl_dqn_conv1_wgrad(const uint8_t* frames, int64_t n, const int64_t* rows,
                                    const float* gy, float scale, float* gw, float* gb,
                                    void* workspace, int64_t ws_bytes, void* stream) {
    TSRL_CHECK_ARG(n >= 0, "tsrl_dqn_conv1_wgrad: n < 0");
    TSRL_CHECK_ARG(frames && gy && gw && (n == 0 || workspace), "tsrl_dqn_conv1_wgrad: null pointer");
    TSRL_CHECK_ARG((((uintptr_t)frames) & 3) == 0 && aligned16(gy),
                   "tsrl_dqn_conv1_wgrad: frames must be 4-byte and gy 16-byte aligned");
    TSRL_CHECK_ARG(scale > 0.0f, "tsrl_dqn_conv1_wgrad: scale must be > 0");
    TSRL_CHECK_ARG(ws_bytes >= tsrl_dqn_conv1_wgrad_workspace_bytes(n),
                   "tsrl_dqn_conv1_wgrad: workspace too small");
    TSRL_CHECK_ARG(n * C1_PIX < ((int64_t)1 << 31), "tsrl_dqn_conv1_wgrad: n * 400 >= 2^31");
    constexpr int W = C1_OC * C1_KK + C1_OC;
    if (n == 0) {
        (void)hipMemsetAsync(gw, 0, C1_OC * C1_KK * sizeof(float), as_stream(stream));
        if (gb) (void)hipMemsetAsync(gb, 0, C1_OC * sizeof(float), as_stream(stream));
        TSRL_LAUNCH_CHECK("tsrl_dqn_conv1_wgrad");
        return 0;
    }
    const int64_t npix = n * C1_PIX;
    const int64_t nchunk = (npix + C1W_CH - 1) / C1W_CH;
    const int64_t nwg0 = std::min<int64_t>(nchunk, 512);
    const int64_t cpw = (nchunk + nwg0 - 1) / nwg0;
    const int64_t nwg = (nchunk + cpw - 1) / cpw;  // every workgroup has >= 1 chunk
    float* part = reinterpret_cast<float*>(workspace);
    hipLaunchKernelGGL(dqn_conv1_wgrad_kernel, dim3((unsigned)nwg), dim3(256), 0,
                       as_stream(stream), frames, rows, gy, npix, cpw, part);
    TSRL_LAUNCH_CHECK("tsrl_dqn_conv1_wgrad");
    hipLaunchKernelGGL(dqn_conv1_wgrad_reduce_kernel, dim3((W + 63) / 64), dim3(256), 0,
                       as_stream(stream), part, (int)nwg, 1.0f / scale, gw, gb);
    TSRL_LAUNCH_CHECK("tsrl_dqn_conv1_wgrad(reduce)");
    return 0;
}

// ReLU backward of the Conv2d + ReLU pairs fused with their bias gradient: gy = (z > 0) * gz
// over rows x C (NHWC rows) and, per workgroup of a contiguous row range, the column sums of gy
// (f32, LDS tree over the row lanes) into partials[blk][C]; relu_bwd_fold_kernel adds the
// partials in f64 in block order (deterministic).  One read of gz and z and one write of gy
// instead of threshold_backward plus a separate bias reduction over gy.
__global__ __launch_bounds__(256) void relu_bwd_rows_kernel(const float4* gz,
                                                            const float4* __restrict__ z,
                                                            float4* gy, int64_t rows, int c4,
                                                            int64_t rpb,
                                                            float4* __restrict__ part) {
    __shared__ float4 red[256];
    const int t = threadIdx.x;
    const int cg = t % c4, rl = t / c4, rstep = 256 / c4;
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    const int64_t r1 = std::min<int64_t>(rows, r0 + rpb);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t r = r0 + rl; r < r1; r += rstep) {
        const int64_t i = r * c4 + cg;
        const float4 g = gz[i], m = z[i];
        float4 v;
        v.x = m.x > 0.0f ? g.x : 0.0f;
        v.y = m.y > 0.0f ? g.y : 0.0f;
        v.z = m.z > 0.0f ? g.z : 0.0f;
        v.w = m.w > 0.0f ? g.w : 0.0f;
        gy[i] = v;
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    }
    if (!part) return;
    red[t] = acc;
    __syncthreads();
    for (int st = 128; st >= c4; st >>= 1) {
        if (t < st) {
            const float4 o = red[t + st];
            red[t].x += o.x;
            red[t].y += o.y;
            red[t].z += o.z;
            red[t].w += o.w;
        }
        __syncthreads();
    }
    if (t < c4) part[(int64_t)blockIdx.x * c4 + t] = red[t];
}

// one workgroup per column: strided f64 sums over the partial rows, then a fixed-order LDS tree
__global__ __launch_bounds__(256) void relu_bwd_fold_kernel(const float* __restrict__ part,
                                                            int64_t nblk, int64_t C,
                                                            float* __restrict__ gb) {
    __shared__ double red[256];
    const int t = threadIdx.x;
    const int64_t c = blockIdx.x;
    double s = 0.0;
    for (int64_t b = t; b < nblk; b += 256) s += (double)part[b * C + c];
    red[t] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (t < st) red[t] += red[t + st];
        __syncthreads();
    }
    if (t == 0) gb[c] = (float)red[0];
}

static int64_t relu_bwd_nblk(int64_t rows, int64_t C) {
    const int64_t rstep = 256 / (C / 4);
    // >= 16 workgroups per CU at the trunk's sizes (memory-level parallelism), ~10 rows each
    return std::max<int64_t>(1, std::min<int64_t>(4096, (rows + 4 * rstep - 1) / (4 * rstep)));
}

extern "C" int64_t tsrl_relu_bwd_rows_workspace_bytes(int64_t rows, int64_t C) {
    if (rows <= 0 || C <= 0 || C % 4 || C > 1024) return 0;
    return relu_bwd_nblk(rows, C) * C * 4;
}

extern "C" int tsrl_relu_bwd_rows(const float* gz, const float* z, float* gy, int64_t rows,
                                  int64_t C, float* gb, void* ws, int64_t ws_bytes,
                                  void* stream) {
    const int64_t c4 = C / 4;
    TSRL_CHECK_ARG(rows >= 0 && C > 0 && C % 4 == 0 && C <= 1024 && (c4 & (c4 - 1)) == 0,
                   "tsrl_relu_bwd_rows: need C %% 4 == 0, C / 4 a power of two, C <= 1024");
    if (rows == 0) {
        if (gb) (void)hipMemsetAsync(gb, 0, C * sizeof(float), as_stream(stream));
        return 0;
    }
    TSRL_CHECK_ARG(gz && z && gy, "tsrl_relu_bwd_rows: null pointer");
    TSRL_CHECK_ARG(aligned16(gz) && aligned16(z) && aligned16(gy),
                   "tsrl_relu_bwd_rows: gz / z / gy must be 16-byte aligned");
    const int64_t nblk = relu_bwd_nblk(rows, C);
    if (gb)
        TSRL_CHECK_ARG(ws && aligned16(ws) && ws_bytes >= nblk * C * 4,
                       "tsrl_relu_bwd_rows: workspace too small");
    const int64_t rpb = (rows + nblk - 1) / nblk;
    hipLaunchKernelGGL(relu_bwd_rows_kernel, dim3((unsigned)nblk), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(gz),
                       reinterpret_cast<const float4*>(z), reinterpret_cast<float4*>(gy), rows,
                       (int)c4, rpb, gb ? reinterpret_cast<float4*>(ws) : nullptr);
    TSRL_LAUNCH_CHECK("tsrl_relu_bwd_rows");
    if (gb) {
        hipLaunchKernelGGL(relu_bwd_fold_kernel, dim3((unsigned)C), dim3(256),
                           0, as_stream(stream), reinterpret_cast<const float*>(ws), nblk, C,
                           gb);
        TSRL_LAUNCH_CHECK("tsrl_relu_bwd_rows (fold)");
    }
    return 0;
}

extern "C" int tsrl_bias_relu_rows(float* y, const float* bias, int64_t rows, int64_t C,
                                   void* stream) {
    TSRL_CHECK_ARG(rows >= 0 && C > 0 && C % 4 == 0, "tsrl_bias_relu_rows: need C %% 4 == 0");
    if (rows == 0) return 0;
    TSRL_CHECK_ARG(y && aligned16(y) && (!bias || aligned16(bias)),
                   "tsrl_bias_relu_rows: y / bias must be 16-byte aligned");
    const int64_t n4 = rows * C / 4;
    const unsigned grid = (unsigned)std::min<int64_t>((n4 + 255) / 256, 8192);
    hipLaunchKernelGGL(bias_relu_rows_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<float4*>(y), reinterpret_cast<const float4*>(bias), n4,
                       (int)(C / 4));
    TSRL_LAUNCH_CHECK("tsrl_bias_relu_rows");
    return 0;
}
