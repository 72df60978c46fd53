// bf16x6: f32 GEMM products on the bf16 matrix cores with an exact three-way operand split
// (mlp_x6.hip has the derivation).  An f32 x is split exactly into x = x0 + x1 + x2 (each the
// round-to-nearest bf16 of the remaining residual); a product a.b is accumulated as the six
// bf16 products of order <= 2 in the f32 MFMA accumulator, which carries f32 GEMM error.
#pragma once
#include "tsrl_common.h"

namespace tsrl {
namespace x6 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NPL = 3;  // split planes

// One f32 split exactly into three bf16 pieces.
__device__ __forceinline__ void split1(float x, __bf16& a0, __bf16& a1, __bf16& a2) {
    a0 = (__bf16)x;
    const float r1 = x - (float)a0;
    a1 = (__bf16)r1;
    a2 = (__bf16)(r1 - (float)a1);
}

// a.b accumulated as a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0 (v_mfma_f32_32x32x16_bf16).
__device__ __forceinline__ f32x16 mfma6(const bf16x8 (&a)[NPL], const bf16x8 (&b)[NPL],
                                        f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    return acc;
}

// Byte offset of 16-byte chunk q (0..3) of a 64-byte LDS row (32 bf16): chunks XOR-swizzled
// by row bits 2-3 so that the 16 lanes of a ds_read_b128 phase (rows c..c+15, one chunk)
// hit all 64 banks.
__device__ __forceinline__ int sw_off(int row, int q) {
    return row * 64 + 16 * (q ^ ((row >> 2) & 3));
}

// Layer-1 activations in MFMA-fragment order (l1 kernels -> tail / eval-tail kernels): 32x32
// fragment tile `tile` (= row tile * 4 + feature tile) holds lane l's 16 accumulator values
// as four float4 pieces q = 0..3, piece q of all 64 lanes contiguous ([tile][q][lane][4]), so
// each of the writer's four 16-byte stores covers one contiguous KB (round 6: the earlier
// [tile][lane][16] order wrote 64-byte-strided pieces; -9.5 us per 262144-row layer-1 launch).
__device__ __forceinline__ int64_t frag_off4(int64_t tile, int lane, int q) {
    return tile * 1024 + (int64_t)(q * 64 + lane) * 4;
}

}  // namespace x6
}  // namespace tsrl
