// On-device image augmentation for the training data path (SURVEY §8f "next" #3): the
// get_transform pipeline of data_loader.py:110-135 (ToTensor, Random90Rot, horizontal/vertical
// flips, ColorJitter, Resize / RandomResizedCrop, GaussianBlur, RandomGrayscale) as HIP kernels on
// [C][H][W] fp32 images in HBM. The random draws stay on the host (data_loader.py); every kernel
// here is deterministic given its parameters. HBM-bound elementwise / stencil work: coalesced
// reads along x, one thread per output pixel.
//
// Semantics follow torchvision's tensor kernels (the reference applies its transforms after
// ToTensor, so the tensor code paths are the ones it runs):
//   rgb_to_grayscale  0.2989 r + 0.587 g + 0.114 b
//   _blend            clamp(ratio * a + (1 - ratio) * b, 0, 1)
//   adjust_hue        _rgb2hsv -> h = (h + f) mod 1 -> _hsv2rgb
//   resize            bilinear with antialias (torch's separable AA filter, align_corners=False)
//   gaussian_blur     separable normalised Gaussian, reflect padding
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "det.h"

namespace {

constexpr int kThreads = 256;

inline unsigned grid_for(int64_t n) {
  int64_t b = (n + kThreads - 1) / kThreads;
  return (unsigned)(b < 1 ? 1 : (b > 65535 * 8 ? 65535 * 8 : b));
}

// ToTensor: uint8 [H][W][cs] (cs >= 3, first 3 used) -> fp32 [3][H][W] / 255
__global__ void to_tensor_kernel(const uint8_t* __restrict__ src, int h, int w, int cs, float* __restrict__ dst) {
  const int64_t hw = (int64_t)h * w;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < hw; p += (int64_t)gridDim.x * kThreads) {
    const uint8_t* s = src + p * cs;
#pragma unroll
    for (int c = 0; c < 3; ++c) dst[c * hw + p] = (float)s[c] / 255.0f;
  }
}

// out[c][y][x] = in[c][ayy*y + ayx*x + ay0][axy*y + axx*x + ax0] (rot90 / flips: coefficients in {-1, 0, 1})
__global__ void remap_kernel(const float* __restrict__ src, int c, int hi, int wi, float* __restrict__ dst, int ho,
                             int wo, int ayy, int ayx, int ay0, int axy, int axx, int ax0) {
  const int64_t n = (int64_t)c * ho * wo;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < n; e += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(e % wo);
    const int64_t t = e / wo;
    const int y = (int)(t % ho), ch = (int)(t / ho);
    const int sy = ayy * y + ayx * x + ay0, sx = axy * y + axx * x + ax0;
    dst[e] = src[((int64_t)ch * hi + sy) * wi + sx];
  }
}

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }
__device__ __forceinline__ float gray(float r, float g, float b) { return 0.2989f * r + 0.587f * g + 0.114f * b; }

// sum of rgb_to_grayscale over an image (for adjust_contrast's mean), into the accumulator acc (det.h)
__global__ void gray_sum_kernel(const float* __restrict__ img, int64_t hw, float* acc) {
  __shared__ float sh[kThreads / 64];
  float s = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < hw; p += (int64_t)gridDim.x * kThreads)
    s += gray(img[p], img[hw + p], img[2 * hw + p]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  ast_det::loss_acc_commit(acc, (sh[0] + sh[1]) + (sh[2] + sh[3]));  // fixed-order sum over workgroups
}

// op: 0 brightness, 1 contrast (mean = *gsum / hw), 2 saturation, 3 hue, 4 grayscale (3 channels)
__global__ void color_kernel(const float* __restrict__ src, int64_t hw, int op, float f, const float* __restrict__ gsum,
                             float* __restrict__ dst) {
  const float mean = (op == 1 && gsum) ? *gsum / (float)hw : 0.f;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < hw; p += (int64_t)gridDim.x * kThreads) {
    float r = src[p], g = src[hw + p], b = src[2 * hw + p];
    if (op == 0) {
      r = clamp01(f * r); g = clamp01(f * g); b = clamp01(f * b);
    } else if (op == 1) {
      const float m = (1.0f - f) * mean;
      r = clamp01(f * r + m); g = clamp01(f * g + m); b = clamp01(f * b + m);
    } else if (op == 2) {
      const float l = (1.0f - f) * gray(r, g, b);
      r = clamp01(f * r + l); g = clamp01(f * g + l); b = clamp01(f * b + l);
    } else if (op == 4) {
      r = g = b = gray(r, g, b);
    } else {
      // torchvision _rgb2hsv
      const float maxc = fmaxf(fmaxf(r, g), b), minc = fminf(fminf(r, g), b);
      const bool eqc = maxc == minc;
      const float cr = maxc - minc;
      const float s = cr / (eqc ? 1.0f : maxc);
      const float crd = eqc ? 1.0f : cr;
      const float rc = (maxc - r) / crd, gc = (maxc - g) / crd, bc = (maxc - b) / crd;
      const float hr = (maxc == r) ? (bc - gc) : 0.f;
      const float hg = (maxc == g && maxc != r) ? (2.0f + rc - bc) : 0.f;
      const float hb = (maxc != g && maxc != r) ? (4.0f + gc - rc) : 0.f;
      float h = fmodf((hr + hg + hb) / 6.0f + 1.0f, 1.0f);
      // (h + f) % 1.0 with Python/torch remainder semantics (result in [0, 1))
      h = h + f;
      h = h - floorf(h);
      const float v = maxc;
      // torchvision _hsv2rgb
      const float fi = floorf(h * 6.0f);
      const float fr = h * 6.0f - fi;
      int i = (int)fi;
      const float pp = clamp01(v * (1.0f - s));
      const float qq = clamp01(v * (1.0f - s * fr));
      const float tt = clamp01(v * (1.0f - s * (1.0f - fr)));
      i = ((i % 6) + 6) % 6;
      switch (i) {
        case 0: r = v; g = tt; b = pp; break;
        case 1: r = qq; g = v; b = pp; break;
        case 2: r = pp; g = v; b = tt; break;
        case 3: r = pp; g = qq; b = v; break;
        case 4: r = tt; g = pp; b = v; break;
        default: r = v; g = pp; b = qq; break;
      }
    }
    dst[p] = r;
    dst[hw + p] = g;
    dst[2 * hw + p] = b;
  }
}

// torch's antialiased bilinear weights (upsample aa, align_corners=False): for output index i of a
// window [off, off + in) resized to out: scale = in/out, support = max(scale, 1), center =
// scale*(i+0.5), taps j in [xmin, xmin+xsize), w = max(0, 1 - |(j - center + 0.5)/max(scale,1)|),
// normalised by their sum.
__device__ __forceinline__ void aa_window(int i, int in, int out, int& xmin, int& xsize, float& scale, float& invs,
                                          float& center) {
  scale = (float)in / (float)out;
  const float support = scale >= 1.0f ? scale : 1.0f;
  invs = scale >= 1.0f ? 1.0f / scale : 1.0f;
  center = scale * ((float)i + 0.5f);
  xmin = max((int)(center - support + 0.5f), 0);
  xsize = min((int)(center + support + 0.5f), in) - xmin;
}

// horizontal pass: tmp[c][y][x] for y in the crop's rows, x in [0, wo)
__global__ void resize_h_kernel(const float* __restrict__ src, int c, int h, int w, int y0, int x0, int ch, int cw,
                                float* __restrict__ tmp, int wo) {
  const int64_t n = (int64_t)c * ch * wo;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < n; e += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(e % wo);
    const int64_t t = e / wo;
    const int y = (int)(t % ch), k = (int)(t / ch);
    int xmin, xsize;
    float scale, invs, center;
    aa_window(x, cw, wo, xmin, xsize, scale, invs, center);
    const float* row = src + ((int64_t)k * h + y0 + y) * w + x0;
    float tot = 0.f, acc = 0.f;
    for (int j = 0; j < xsize; ++j) {
      const float wt = fmaxf(0.f, 1.0f - fabsf(((float)(j + xmin) - center + 0.5f) * invs));
      tot += wt;
      acc = fmaf(wt, row[xmin + j], acc);
    }
    tmp[e] = tot != 0.f ? acc / tot : 0.f;
  }
}

// vertical pass: dst[c][y][x] from tmp[c][ch][wo]
__global__ void resize_v_kernel(const float* __restrict__ tmp, int c, int ch, int wo, float* __restrict__ dst, int ho) {
  const int64_t n = (int64_t)c * ho * wo;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < n; e += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(e % wo);
    const int64_t t = e / wo;
    const int y = (int)(t % ho), k = (int)(t / ho);
    int ymin, ysize;
    float scale, invs, center;
    aa_window(y, ch, ho, ymin, ysize, scale, invs, center);
    const float* col = tmp + (int64_t)k * ch * wo + x;
    float tot = 0.f, acc = 0.f;
    for (int j = 0; j < ysize; ++j) {
      const float wt = fmaxf(0.f, 1.0f - fabsf(((float)(j + ymin) - center + 0.5f) * invs));
      tot += wt;
      acc = fmaf(wt, col[(int64_t)(ymin + j) * wo], acc);
    }
    dst[e] = tot != 0.f ? acc / tot : 0.f;
  }
}

__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

struct BlurTaps {
  float w[15];
};

// separable Gaussian pass along x (dir 0) or y (dir 1); taps normalised (passed by value)
__global__ void blur_kernel(const float* __restrict__ src, int c, int h, int w, BlurTaps kern, int k, int dir,
                            float* __restrict__ dst) {
  const int64_t n = (int64_t)c * h * w;
  const int r = k / 2;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < n; e += (int64_t)gridDim.x * kThreads) {
    const int x = (int)(e % w);
    const int64_t t = e / w;
    const int y = (int)(t % h);
    const float* plane = src + (t / h) * (int64_t)h * w;
    float acc = 0.f;
    for (int j = 0; j < k; ++j) {
      const float v = dir == 0 ? plane[(int64_t)y * w + reflect_idx(x + j - r, w)]
                               : plane[(int64_t)reflect_idx(y + j - r, h) * w + x];
      acc = fmaf(kern.w[j], v, acc);
    }
    dst[e] = acc;
  }
}

}  // namespace

extern "C" {

int ast_aug_to_tensor(const unsigned char* src, int h, int w, int cs, float* dst, void* stream) {
  if (!src || !dst) return AST_E_NULLPTR;
  if (h <= 0 || w <= 0 || cs < 3) return AST_E_SHAPE;
  hipLaunchKernelGGL(to_tensor_kernel, dim3(grid_for((int64_t)h * w)), dim3(kThreads), 0, (hipStream_t)stream, src,
                     h, w, cs, dst);
  return (int)hipGetLastError();
}

int ast_aug_remap_f32(const float* src, int c, int hi, int wi, float* dst, int ho, int wo, const int* coef,
                      void* stream) {
  if (!src || !dst || !coef) return AST_E_NULLPTR;
  if (c <= 0 || hi <= 0 || wi <= 0 || ho <= 0 || wo <= 0) return AST_E_SHAPE;
  // the four corners must map inside the source (the map is affine)
  for (int cy = 0; cy < 2; ++cy)
    for (int cx = 0; cx < 2; ++cx) {
      const int y = cy ? ho - 1 : 0, x = cx ? wo - 1 : 0;
      const int sy = coef[0] * y + coef[1] * x + coef[2], sx = coef[3] * y + coef[4] * x + coef[5];
      if (sy < 0 || sy >= hi || sx < 0 || sx >= wi) return AST_E_SHAPE;
    }
  hipLaunchKernelGGL(remap_kernel, dim3(grid_for((int64_t)c * ho * wo)), dim3(kThreads), 0, (hipStream_t)stream, src,
                     c, hi, wi, dst, ho, wo, coef[0], coef[1], coef[2], coef[3], coef[4], coef[5]);
  return (int)hipGetLastError();
}

int ast_aug_gray_sum_f32(const float* img, int h, int w, float* acc, void* stream) {
  if (!img || !acc) return AST_E_NULLPTR;
  if (h <= 0 || w <= 0) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(acc, 0, sizeof(float), st);
  if (e != hipSuccess) return (int)e;
  const int64_t hw = (int64_t)h * w;
  unsigned g = grid_for(hw);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(gray_sum_kernel, dim3(g), dim3(kThreads), 0, st, img, hw, acc);
  return (int)hipGetLastError();
}

int ast_aug_color_f32(const float* src, int h, int w, int op, float factor, const float* gray_sum, float* dst,
                      void* stream) {
  if (!src || !dst) return AST_E_NULLPTR;
  if (h <= 0 || w <= 0) return AST_E_SHAPE;
  if (op < 0 || op > 4 || (op == 1 && !gray_sum)) return AST_E_UNSUPPORTED;
  const int64_t hw = (int64_t)h * w;
  hipLaunchKernelGGL(color_kernel, dim3(grid_for(hw)), dim3(kThreads), 0, (hipStream_t)stream, src, hw, op, factor,
                     gray_sum, dst);
  return (int)hipGetLastError();
}

size_t ast_aug_resize_workspace_floats(int c, int crop_h, int wo) { return (size_t)c * crop_h * wo; }

int ast_aug_resize_f32(const float* src, int c, int h, int w, int y0, int x0, int crop_h, int crop_w, float* dst,
                       int ho, int wo, float* tmp, void* stream) {
  if (!src || !dst || !tmp) return AST_E_NULLPTR;
  if (c <= 0 || h <= 0 || w <= 0 || ho <= 0 || wo <= 0 || crop_h <= 0 || crop_w <= 0) return AST_E_SHAPE;
  if (y0 < 0 || x0 < 0 || y0 + crop_h > h || x0 + crop_w > w) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(resize_h_kernel, dim3(grid_for((int64_t)c * crop_h * wo)), dim3(kThreads), 0, st, src, c, h, w,
                     y0, x0, crop_h, crop_w, tmp, wo);
  hipLaunchKernelGGL(resize_v_kernel, dim3(grid_for((int64_t)c * ho * wo)), dim3(kThreads), 0, st, tmp, c, crop_h, wo,
                     dst, ho);
  return (int)hipGetLastError();
}

int ast_aug_blur_f32(const float* src, int c, int h, int w, const float* taps, int k, float* dst, float* tmp,
                     void* stream) {
  if (!src || !dst || !tmp || !taps) return AST_E_NULLPTR;
  if (c <= 0 || h <= 0 || w <= 0 || k <= 0 || (k & 1) == 0 || k > 15) return AST_E_SHAPE;
  if (k / 2 >= h || k / 2 >= w) return AST_E_SHAPE;  // reflect padding needs pad < size
  BlurTaps bt{};
  for (int i = 0; i < k; ++i) bt.w[i] = taps[i];  // host array
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = grid_for((int64_t)c * h * w);
  hipLaunchKernelGGL(blur_kernel, dim3(g), dim3(kThreads), 0, st, src, c, h, w, bt, k, 0, tmp);
  hipLaunchKernelGGL(blur_kernel, dim3(g), dim3(kThreads), 0, st, tmp, c, h, w, bt, k, 1, dst);
  return (int)hipGetLastError();
}

}  // extern "C"
