// Per-(n,c) channel statistics and AdaIN for gfx950.
//
// channel_stats (model_util.py:3-8), calc_mean_std (models.py:54-62), mean_variance_norm
// (models.py:64-68), AdaIN.forward (models.py:43-51) and the alpha blend (models.py:471).
// HBM-bound: one workgroup per plane, two-pass statistics (sum, then sum of squared deviations:
// the second pass re-reads the plane from L1/L2, not HBM) with 64-lane shuffle + LDS reductions,
// then a fused normalise-affine-blend write. Algorithmic bytes: read content + style, write out.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the 256-thread block; every thread gets the total. `sh` holds kWaves floats.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) t += sh[i];
  return t;
}

__device__ __forceinline__ float plane_sum(const float* __restrict__ p, int64_t hw, float* sh) {
  float s = 0.f;
  if ((hw & 3) == 0 && ((uintptr_t)p & 15) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
    for (int64_t i = threadIdx.x; i < hw / 4; i += kThreads) {
      const float4 v = p4[i];
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    for (int64_t i = threadIdx.x; i < hw; i += kThreads) s += p[i];
  }
  return block_sum(s, sh);
}

__device__ __forceinline__ float plane_sqdev(const float* __restrict__ p, int64_t hw, float mean, float* sh) {
  float s = 0.f;
  if ((hw & 3) == 0 && ((uintptr_t)p & 15) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
    for (int64_t i = threadIdx.x; i < hw / 4; i += kThreads) {
      const float4 v = p4[i];
      const float a = v.x - mean, b = v.y - mean, c = v.z - mean, d = v.w - mean;
      s += (a * a + b * b) + (c * c + d * d);
    }
  } else {
    for (int64_t i = threadIdx.x; i < hw; i += kThreads) {
      const float a = p[i] - mean;
      s += a * a;
    }
  }
  return block_sum(s, sh);
}

// mean, std (= sqrt(var + eps)); var divides by hw - unbiased (torch: 0/0 -> NaN at hw == 1).
__device__ __forceinline__ void plane_stats(const float* p, int64_t hw, int unbiased, float eps, float* sh,
                                            float& mean, float& sd) {
  mean = plane_sum(p, hw, sh) / (float)hw;
  const float ss = plane_sqdev(p, hw, mean, sh);
  sd = sqrtf(ss / (float)(hw - unbiased) + eps);
}

__global__ __launch_bounds__(kThreads) void channel_stats_kernel(const float* __restrict__ x, float* __restrict__ mean,
                                                                 float* __restrict__ sd, int64_t hw, int unbiased,
                                                                 float eps) {
  __shared__ float sh[kWaves];
  const int64_t p = blockIdx.x;
  float m, s;
  plane_stats(x + p * hw, hw, unbiased, eps, sh, m, s);
  if (threadIdx.x == 0) {
    mean[p] = m;
    sd[p] = s;
  }
}

__global__ __launch_bounds__(kThreads) void adain_kernel(const float* __restrict__ content,
                                                         const float* __restrict__ style, float* __restrict__ out,
                                                         int64_t hwc, int64_t hws, float alpha, float beta,
                                                         int swap) {
  __shared__ float sh[kWaves];
  const int64_t p = blockIdx.x;
  const float* c = content + p * hwc;
  float ms, ss, mc, sc;
  plane_stats(style + p * hws, hws, 1, 0.f, sh, ms, ss);
  plane_stats(c, hwc, 1, 0.f, sh, mc, sc);
  const float scale = swap ? ms : ss;
  const float shift = swap ? ss : ms;
  float* o = out + p * hwc;
  if ((hwc & 3) == 0 && ((uintptr_t)c & 15) == 0 && ((uintptr_t)o & 15) == 0) {
    const float4* c4 = reinterpret_cast<const float4*>(c);
    float4* o4 = reinterpret_cast<float4*>(o);
    for (int64_t i = threadIdx.x; i < hwc / 4; i += kThreads) {
      const float4 v = c4[i];
      float4 r;
      r.x = alpha * ((v.x - mc) / sc * scale + shift) + beta * v.x;
      r.y = alpha * ((v.y - mc) / sc * scale + shift) + beta * v.y;
      r.z = alpha * ((v.z - mc) / sc * scale + shift) + beta * v.z;
      r.w = alpha * ((v.w - mc) / sc * scale + shift) + beta * v.w;
      o4[i] = r;
    }
  } else {
    for (int64_t i = threadIdx.x; i < hwc; i += kThreads) {
      const float v = c[i];
      o[i] = alpha * ((v - mc) / sc * scale + shift) + beta * v;
    }
  }
}

// Backward of adain_kernel. With c_hat = (c - mu_c)/sigma_c, (a, b) = (scale, shift) and g = dL/dy:
//   dc = alpha*a*(g - mean(g) - c_hat*sum(g c_hat)/(N-1))/sigma_c + (1-alpha)*g
//   da = alpha*sum(g c_hat), db = alpha*sum(g)  ->  (d mu_s, d sigma_s) by the swap rule
//   ds = d mu_s / Ns + d sigma_s * (s - mu_s) / ((Ns-1) sigma_s)
__global__ __launch_bounds__(kThreads) void adain_backward_kernel(const float* __restrict__ content,
                                                                  const float* __restrict__ style,
                                                                  const float* __restrict__ g, float* __restrict__ dc,
                                                                  float* __restrict__ ds, int64_t hwc, int64_t hws,
                                                                  float alpha, float beta, int swap) {
  __shared__ float sh[kWaves];
  const int64_t p = blockIdx.x;
  const float* c = content + p * hwc;
  const float* s = style + p * hws;
  const float* gp = g + p * hwc;
  float ms, ss, mc, sc;
  plane_stats(s, hws, 1, 0.f, sh, ms, ss);
  plane_stats(c, hwc, 1, 0.f, sh, mc, sc);
  const float a = swap ? ms : ss;
  float sg = 0.f, sgc = 0.f;
  for (int64_t i = threadIdx.x; i < hwc; i += kThreads) {
    const float gi = gp[i];
    sg += gi;
    sgc += gi * (c[i] - mc) / sc;
  }
  const float G = block_sum(sg, sh), GC = block_sum(sgc, sh);
  if (dc) {
    const float gmean = G / (float)hwc, gcz = GC / (float)(hwc - 1);
    float* o = dc + p * hwc;
    for (int64_t i = threadIdx.x; i < hwc; i += kThreads) {
      const float z = (c[i] - mc) / sc;
      o[i] = alpha * a * (gp[i] - gmean - z * gcz) / sc + beta * gp[i];
    }
  }
  if (ds) {
    const float da = alpha * GC, db = alpha * G;
    const float dmu = swap ? da : db, dsd = swap ? db : da;
    float* o = ds + p * hws;
    for (int64_t i = threadIdx.x; i < hws; i += kThreads)
      o[i] = dmu / (float)hws + dsd * (s[i] - ms) / ((float)(hws - 1) * ss);
  }
}

// AdaIN with the style statistics given (one-style-many-contents mode, SURVEY §8e: the style
// owner computes (mean, std) once and broadcasts 2*C floats). Plane p = (n, c) uses
// style_mean[(n * stride_n + c)], stride_n = 0 sharing one style across the batch.
__global__ __launch_bounds__(kThreads) void adain_stats_kernel(const float* __restrict__ content,
                                                               const float* __restrict__ smean,
                                                               const float* __restrict__ sstd,
                                                               float* __restrict__ out, int64_t hwc, int c,
                                                               int stride_n, float alpha, float beta, int swap) {
  __shared__ float sh[kWaves];
  const int64_t p = blockIdx.x;
  const int64_t si = (p / c) * stride_n + p % c;
  const float ms = smean[si], ss = sstd[si];
  const float* x = content + p * hwc;
  float mc, sc;
  plane_stats(x, hwc, 1, 0.f, sh, mc, sc);
  const float scale = swap ? ms : ss, shift = swap ? ss : ms;
  float* o = out + p * hwc;
  for (int64_t i = threadIdx.x; i < hwc; i += kThreads) {
    const float v = x[i];
    o[i] = alpha * ((v - mc) / sc * scale + shift) + beta * v;
  }
}

__global__ void plane_normalize_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                       const float* __restrict__ sd, float* __restrict__ out, int64_t hw,
                                       int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / hw;
    out[i] = (x[i] - mean[p]) / sd[p];
  }
}

}  // namespace

extern "C" {

int ast_channel_stats_f32(const float* x, float* mean, float* std, long long planes, long long hw, int unbiased,
                          float eps, void* stream) {
  if (!x || !mean || !std) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL(channel_stats_kernel, dim3((unsigned)planes), dim3(kThreads), 0, (hipStream_t)stream, x, mean,
                     std, (int64_t)hw, unbiased ? 1 : 0, eps);
  return (int)hipGetLastError();
}

int ast_adain_f32(const float* content, const float* style, float* out, int n, int c, int hc, int wc, int hs, int ws,
                  double alpha, int swap_style_stats, void* stream) {
  if (!content || !style || !out) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hc <= 0 || wc <= 0 || hs <= 0 || ws <= 0) return AST_E_SHAPE;
  // torch: `alpha * t + (1 - alpha) * c` with Python-float scalars applied in fp32
  const float a = (float)alpha, b = (float)(1.0 - alpha);
  hipLaunchKernelGGL(adain_kernel, dim3((unsigned)((int64_t)n * c)), dim3(kThreads), 0, (hipStream_t)stream, content,
                     style, out, (int64_t)hc * wc, (int64_t)hs * ws, a, b, swap_style_stats ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_adain_backward_f32(const float* content, const float* style, const float* grad_out, float* d_content,
                           float* d_style, int n, int c, int hc, int wc, int hs, int ws, double alpha,
                           int swap_style_stats, void* stream) {
  if (!content || !style || !grad_out) return AST_E_NULLPTR;
  if (!d_content && !d_style) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hc <= 0 || wc <= 0 || hs <= 0 || ws <= 0) return AST_E_SHAPE;
  const float a = (float)alpha, b = (float)(1.0 - alpha);
  hipLaunchKernelGGL(adain_backward_kernel, dim3((unsigned)((int64_t)n * c)), dim3(kThreads), 0, (hipStream_t)stream,
                     content, style, grad_out, d_content, d_style, (int64_t)hc * wc, (int64_t)hs * ws, a, b,
                     swap_style_stats ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_adain_stats_f32(const float* content, const float* style_mean, const float* style_std, float* out, int n,
                        int c, int hc, int wc, int style_stride_n, double alpha, int swap_style_stats, void* stream) {
  if (!content || !style_mean || !style_std || !out) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hc <= 0 || wc <= 0 || style_stride_n < 0) return AST_E_SHAPE;
  if (style_stride_n != 0 && style_stride_n < c) return AST_E_SHAPE;
  const float a = (float)alpha, b = (float)(1.0 - alpha);
  hipLaunchKernelGGL(adain_stats_kernel, dim3((unsigned)((int64_t)n * c)), dim3(kThreads), 0, (hipStream_t)stream,
                     content, style_mean, style_std, out, (int64_t)hc * wc, c, style_stride_n, a, b,
                     swap_style_stats ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_plane_normalize_f32(const float* x, const float* mean, const float* std, float* out, long long planes,
                            long long hw, void* stream) {
  if (!x || !mean || !std || !out) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0) return AST_E_SHAPE;
  const int64_t total = (int64_t)planes * hw;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(plane_normalize_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, mean, std, out,
                     (int64_t)hw, total);
  return (int)hipGetLastError();
}

}  // extern "C"
