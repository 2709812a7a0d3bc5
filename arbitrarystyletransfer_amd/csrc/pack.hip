// Side-by-side image packing for small-plane 3x3 convolutions (ops.conv3x3, zero padding).
// The implicit-GEMM conv kernel (conv3x3_igemm.hip) tiles each output row in 32-pixel MFMA M
// tiles, so a 20- or 10-pixel-wide plane leaves 38-69% of every tile idle (the AutoEncoder loss
// network's 512-channel layers at 160x160 input). G images placed side by side with `gap` zero
// columns between them form one wider plane whose zero-padded 3x3 conv equals the G separate
// zero-padded convs (a tap that leaves an image reads a gap zero, exactly like the padding);
// gap 2 keeps every image on an even column so the fused 2x2 max-pool never straddles two.
// Both kernels are pure copies (HBM-bound, one thread per destination element).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace {

constexpr int kT = 256;

// xp[gi][c][y][q], q = g*(w+gap) + j: image gi*G+g's pixel j (0 in gaps / missing images)
// IDX: the index type of the element decomposition -- 32-bit when the tensor allows it (the 64-bit
// divisions by runtime sizes cost several times the 32-bit ones, and this gather is all index math)
template <typename IDX>
__global__ __launch_bounds__(kT) void pack_kernel(const float* __restrict__ x, int n1, const float* __restrict__ x2,
                                                  int n, int c, int h, int w, int G, int gap, int wp,
                                                  float* __restrict__ xp, int64_t total) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const IDX ei = (IDX)e;
    const int q = (int)(ei % (IDX)wp);
    const IDX r = ei / (IDX)wp;  // (gi*c + ch)*h + y
    const int y = (int)(r % (IDX)h);
    const IDX r2 = r / (IDX)h;
    const int ch = (int)(r2 % (IDX)c);
    const int gi = (int)(r2 / (IDX)c);
    const int g = q / (w + gap), j = q - g * (w + gap);
    const int img = gi * G + g;
    float v = 0.f;
    if (j < w && img < n) {
      const float* src = img < n1 ? x + (int64_t)img * c * h * w : x2 + (int64_t)(img - n1) * c * h * w;
      v = src[((int64_t)ch * h + y) * w + j];
    }
    xp[e] = v;
  }
}

// out[i][c][y][x] = yp[i / G][c][y][(i % G) * sp + x]
template <typename IDX>
__global__ __launch_bounds__(kT) void unpack_kernel(const float* __restrict__ yp, int c, int h, int w, int G, int sp,
                                                    int wp, float* __restrict__ out, int64_t total) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const IDX ei = (IDX)e;
    const int xx = (int)(ei % (IDX)w);
    const IDX r = ei / (IDX)w;
    const int y = (int)(r % (IDX)h);
    const IDX r2 = r / (IDX)h;
    const int ch = (int)(r2 % (IDX)c);
    const int i = (int)(r2 / (IDX)c);
    out[e] = yp[(((int64_t)(i / G) * c + ch) * h + y) * wp + (i % G) * sp + xx];
  }
}

unsigned grid_for(int64_t n) {
  const int64_t b = (n + kT - 1) / kT;
  return (unsigned)(b < 1 ? 1 : (b > (1 << 20) ? (1 << 20) : b));
}

}  // namespace

extern "C" {

int ast_pack_images_f32(const float* x, int n1, const float* x2, int n2, int c, int h, int w, int G, int gap,
                        float* xp, void* stream) {
  if (!x || !xp || (n2 > 0 && !x2)) return AST_E_NULLPTR;
  if (n1 <= 0 || n2 < 0 || c <= 0 || h <= 0 || w <= 0 || G <= 0 || gap < 0) return AST_E_SHAPE;
  const int n = n1 + n2, ng = (n + G - 1) / G;
  const int wp = G * (w + gap) - gap;
  const int64_t total = (int64_t)ng * c * h * wp;
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(pack_kernel<unsigned>, dim3(grid_for(total)), dim3(kT), 0, (hipStream_t)stream, x, n1, x2, n, c,
                       h, w, G, gap, wp, xp, total);
  else
    hipLaunchKernelGGL(pack_kernel<int64_t>, dim3(grid_for(total)), dim3(kT), 0, (hipStream_t)stream, x, n1, x2, n, c,
                       h, w, G, gap, wp, xp, total);
  return (int)hipGetLastError();
}

int ast_unpack_images_f32(const float* yp, int n, int c, int h, int w, int G, int sp, int wp, float* out,
                          void* stream) {
  if (!yp || !out) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || h <= 0 || w <= 0 || G <= 0 || sp < w || (G - 1) * sp + w > wp) return AST_E_SHAPE;
  const int64_t total = (int64_t)n * c * h * w;
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(unpack_kernel<unsigned>, dim3(grid_for(total)), dim3(kT), 0, (hipStream_t)stream, yp, c, h, w, G,
                       sp, wp, out, total);
  else
    hipLaunchKernelGGL(unpack_kernel<int64_t>, dim3(grid_for(total)), dim3(kT), 0, (hipStream_t)stream, yp, c, h, w, G,
                       sp, wp, out, total);
  return (int)hipGetLastError();
}

}  // extern "C"
