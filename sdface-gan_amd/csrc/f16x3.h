// f16x3.h -- the split-fp16 arithmetic shared by the MFMA kernels of libsdfr
// (field_f16x3.hip: the fused renderer's field stage; linear_f16x3.hip: the
// renderer MLP's training GEMMs).  An fp32 product W.x runs as three
// v_mfma_f32_16x16x32_f16 on round-to-nearest hi/lo fp16 splits of both
// operands, accumulated in fp32 (W_lo.x_lo, 2^-22 relative, is dropped):
//     W.x = W_hi.x_hi + W_hi.x_lo + W_lo.x_hi
// provided no lo part goes subnormal -- callers scale rows by powers of two.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sdfr {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ h8 as_h8(f4 v) { return __builtin_bit_cast(h8, v); }
__device__ __forceinline__ f4 mfma16(f4 a, f4 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(a), as_h8(b), c, 0, 0, 0);
}

// 8 fp32 -> (hi, lo) fp16x8, round-to-nearest both.  hi: v_cvt_pk_f16_f32 per
// pair.  x - hi is exact in fp32 (|x - hi| <= half an fp16 ulp of x), so
// lo = RN16(x - hi) is ONE v_fma_mix{lo,hi}_f16 per value: fma(hi, -1, x) with the
// packed f16 hi as a mixed-precision source, bit-identical to cvt(x - cvt(hi)) and
// half its VALU (the compiler canonicalises a written-out fma(-hi, 1, x) back to
// the sub, hence the asm).
__device__ __forceinline__ void split8(const float (&v)[8], f4 &hi, f4 &lo) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    uint32_t hp[4], lp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        h2 H;
        H[0] = (_Float16)v[2 * j];
        H[1] = (_Float16)v[2 * j + 1];
        hp[j] = __builtin_bit_cast(uint32_t, H);
        uint32_t l;
        asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(hp[j]), "v"(v[2 * j]));
        asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
            : "+v"(l) : "v"(hp[j]), "v"(v[2 * j + 1]));
        lp[j] = l;
    }
    hi = __builtin_bit_cast(f4, hp);
    lo = __builtin_bit_cast(f4, lp);
}

}  // namespace sdfr
