// Split-bf16 ("x3") helpers shared by the fp32-accurate MFMA kernels: an fp32 value is carried as
// three bf16 terms x = hi + mid + lo (exact for finite x), and a product as the six largest term
// products, folded into three v_mfma_f32_16x16x32_bf16 per 16 channels of K (see conv3x3_igemm.hip
// M16 and mbtrain.hip gemm_x3_kernel).
#pragma once
#include <hip/hip_runtime.h>

namespace ast_x3 {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// finite |x| above bf16's largest value would round hi to inf: hi is clamped to that value and the
// remainder stays exact. Non-finite x: hi = x, mid = lo = 0 (inf and NaN propagate through hi).
__device__ __forceinline__ void split3(float x, bf16& hi, bf16& mid, bf16& lo) {
  const bool finite = fabsf(x) <= 3.402823466e38f;
  hi = (bf16)x;
  if (finite && !(fabsf((float)hi) <= 3.402823466e38f)) hi = (bf16)copysignf(3.38953139e38f, x);
  const float r = finite ? x - (float)hi : 0.f;
  mid = (bf16)r;
  lo = (bf16)(r - (float)mid);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// Eight values at once into the three term planes, bit-identical to split3 value by value: the terms
// are round-to-nearest-even conversions of PAIRS (one v_cvt_pk_bf16_f32 per two values; the scalar
// casts of split3 each took their own conversion), unpacked to fp32 by a shift / mask. split3's
// clamp of a finite x whose hi overflows and its non-finite case are a rare path, taken per wave:
// for finite x with finite hi every remainder r = x - hi is finite (|r| <= 2^-8 |x|), so the sum of
// the eight remainders is finite unless one of them is not (r = NaN for a non-finite x, -+inf for an
// overflowed hi). ~6 VALU per value on the common path against ~20 for split3's expansion
// (the store phase between the K chunks' barriers).
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  float r[8], s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bf16x2 h = __builtin_convertvector((f32x2){x[2 * k], x[2 * k + 1]}, bf16x2);
    p0[2 * k] = h[0];
    p0[2 * k + 1] = h[1];
    r[2 * k] = x[2 * k] - (float)h[0];
    r[2 * k + 1] = x[2 * k + 1] - (float)h[1];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) s += fabsf(r[k]);
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(s <= 3.402823466e38f)) != 0, 0)) {
    // split3's hi and remainder, in place (the common tail below then forms mid and lo as split3)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool finite = fabsf(x[k]) <= 3.402823466e38f;
      bf16 hk = (bf16)x[k];
      if (finite && !(fabsf((float)hk) <= 3.402823466e38f)) hk = (bf16)copysignf(3.38953139e38f, x[k]);
      p0[k] = hk;
      r[k] = finite ? x[k] - (float)hk : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bf16x2 m = __builtin_convertvector((f32x2){r[2 * k], r[2 * k + 1]}, bf16x2);
    p1[2 * k] = m[0];
    p1[2 * k + 1] = m[1];
    const bf16x2 l = __builtin_convertvector((f32x2){r[2 * k] - (float)m[0], r[2 * k + 1] - (float)m[1]}, bf16x2);
    p2[2 * k] = l[0];
    p2[2 * k + 1] = l[1];
  }
}

}  // namespace ast_x3
