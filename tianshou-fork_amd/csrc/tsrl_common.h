// Shared helpers for the libtsrl HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/tsrl.h"

namespace tsrl {

constexpr int kWave = 64;

// Thread-local last-error message, exposed through tsrl_last_error().
void set_error(const char* fmt, ...);

#define TSRL_CHECK_ARG(cond, ...)                                   \
    do {                                                            \
        if (!(cond)) {                                              \
            ::tsrl::set_error(__VA_ARGS__);                         \
            return (int)hipErrorInvalidValue;                       \
        }                                                           \
    } while (0)

#define TSRL_LAUNCH_CHECK(what)                                                     \
    do {                                                                            \
        hipError_t _e = hipGetLastError();                                          \
        if (_e != hipSuccess) {                                                     \
            ::tsrl::set_error("%s: launch failed: %s", what, hipGetErrorString(_e)); \
            return (int)_e;                                                         \
        }                                                                           \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Compute units of the current device (hipDeviceAttributeMultiprocessorCount: 256 on MI355X),
// queried once per process; 1 if the query fails.
inline int n_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0, cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cu = 1;
        n = cu > 0 ? cu : 1;
    }
    return n;
}

// splitmix64 finaliser of (x + golden gamma): the counter-based hash of the synthetic env
// (oracle/synth_env.py restates it on the CPU).
__host__ __device__ __forceinline__ uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// tanh without branches: both halves of ROCm's __ocml_tanh_f32 (the |x| < 0.625 polynomial
// and 1 - 2/(exp(2|x|) + 1)) are evaluated and selected, so unrolled MFMA code keeps one basic
// block (ocml's branch splits it per call).  Round 6: exp(2|x|) is one v_exp_f32 of
// 2|x| log2(e) instead of expf's range-reduced form -- within 1.6 ulp of tanh (emulated
// with correctly rounded exp2 / rcp over 3M points; expf's form 1.05 ulp), no longer
// bit-identical to tanhf; layer 1 222 -> 208 us per 262144-row minibatch, the evaluation
// of 2M rows 1800 -> 1688 us (tools/r06_tanh.sh, profiles/r06_tanh_ab.log).
__device__ __forceinline__ float tanh_nb(float x) {
    const float ax = __builtin_fabsf(x);
    const float x2 = x * x;
    float p = __builtin_fmaf(x2, -0x1.758e7ap-8f, 0x1.521192p-6f);
    p = __builtin_fmaf(x2, p, -0x1.b8389cp-5f);
    p = __builtin_fmaf(x2, p, 0x1.110704p-3f);
    p = __builtin_fmaf(x2, p, -0x1.555532p-2f);
    const float small = __builtin_fmaf(x2, ax * p, ax);
    const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);  // 2^(2|x| log2 e)
    const float large = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
    return __builtin_copysignf(ax < 0.625f ? small : large, x);
}

// Wave-wide sum of a double (64 lanes, xor butterfly).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

}  // namespace tsrl
