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

}  // namespace ast_x3
