// The remaining train.py loss terms (SURVEY §8f "next" #2) for gfx950:
//   * compute_hist_loss (losses.py:84-87): SingleDimHistLayer soft histogram (losses.py:40-57,
//     K = 256 bins, L = 1/K, W = L/2.5, one histogram over all C*H*W values of an image, divided by
//     N = C*H -- the reference's x.size(1)*x.size(2)) of both images, then the Earth-Mover distance
//     (losses.py:8-22) of their CDFs, mean over the batch;
//   * out_of_range_loss (train.py:259): huber(x - clip(x.detach(), 0, 1)), mean;
//   * the pixel term of org_img_loss (train.py:268): mean((a - b)^2).
//
// Soft histogram: phi_k(x) = sig((x - mu_k + L/2)/W) - sig((x - mu_k - L/2)/W) with mu_k = L(k+1/2),
// i.e. phi_k = S_k - S_{k+1}, S_j = sig((x - jL)/W): 257 sigmoids per value would give all bins,
// but with L/W = 2.5 a bin d bins away from x gets < e^{-2.5(d-1)}; the kernel evaluates the
// window |j - x/L| <= kHalo (kHalo = 12: the neglected mass is < e^{-27} ~ 2e-12 of each value's
// unit mass, far below fp32 resolution of a bin). The bins are accumulated as exact 32.32
// fixed-point integers (each contribution phi in [0, 1] truncated to a multiple of 2^-32): integer
// addition is associative, so the per-workgroup LDS histograms (ds_add_u64) and their flush into
// the per-image workspace histogram (one 64-bit atomic per bin) give the same bits in any order.
// A NaN anywhere in an image poisons all its bins (a flag), as the reference's dense sum does.
// HBM-bound (one read of x); the window's sigmoids run on the transcendental unit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "det.h"

namespace {

constexpr int kBins = 256;
constexpr int kHalo = 12;
constexpr int kThreads = 256;
constexpr float kL = 1.0f / kBins;
constexpr float kInvW = 2.5f * kBins;  // 1 / W

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + __expf(-z)); }

__device__ __forceinline__ float block_sum(float v, float* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) t += sh[i];
  return t;
}

__device__ __forceinline__ float gs(const float* g) { return g ? *g : 1.0f; }

// window of sigmoid indices j (0..256) around value x: [j0, j1]
__device__ __forceinline__ void window(float x, int& j0, int& j1) {
  const float c = x * (float)kBins;
  const float lo = fmaxf(c - (float)kHalo, -1.0f), hi = fminf(c + (float)kHalo, (float)kBins + 1.0f);
  j0 = max(0, (int)floorf(lo));
  j1 = min(kBins, (int)ceilf(hi));
}

// grid (blocks_per_image, n); acc [n][kBins + 1] int64 (the bins, then the NaN flag), zeroed
constexpr double kFix = 4294967296.0;  // 2^32

__global__ __launch_bounds__(kThreads) void soft_hist_kernel(const float* __restrict__ x, int64_t m,
                                                             unsigned long long* __restrict__ acc) {
  __shared__ unsigned long long hs[kBins];
  __shared__ int nan_seen;
  for (int i = threadIdx.x; i < kBins; i += kThreads) hs[i] = 0ull;
  if (threadIdx.x == 0) nan_seen = 0;
  __syncthreads();
  const float* xb = x + (int64_t)blockIdx.y * m;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < m; i += (int64_t)gridDim.x * kThreads) {
    const float v = xb[i];
    if (!(v == v)) {  // NaN poisons every bin, as in the reference's dense sum
      nan_seen = 1;
      continue;
    }
    int j0, j1;
    window(v, j0, j1);
    if (j0 >= j1) continue;
    float sprev = sigm((v - (float)j0 * kL) * kInvW);
    for (int j = j0 + 1; j <= j1; ++j) {
      const float s = sigm((v - (float)j * kL) * kInvW);
      // bin j-1 = S_{j-1} - S_j >= 0 (S decreases in j); x 2^32 is exact in fp32, the conversion
      // truncates the sub-2^-32 tail
      atomicAdd(&hs[j - 1], (unsigned long long)(fmaxf(sprev - s, 0.f) * 4294967296.0f));
      sprev = s;
    }
  }
  __syncthreads();
  unsigned long long* hb = acc + (int64_t)blockIdx.y * (kBins + 1);
  for (int i = threadIdx.x; i < kBins; i += kThreads)
    if (hs[i]) atomicAdd(&hb[i], hs[i]);
  if (threadIdx.x == 0 && nan_seen) atomicOr(&hb[kBins], 1ull);
}

__global__ void hist_finish_kernel(const unsigned long long* __restrict__ acc, int n, float inv_norm,
                                   float* __restrict__ hist) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * kBins) return;
  const int b = e / kBins, k = e - b * kBins;
  const unsigned long long* hb = acc + (int64_t)b * (kBins + 1);
  hist[e] = hb[kBins] ? __builtin_nanf("") : (float)((double)hb[k] * (1.0 / kFix) * (double)inv_norm);
}

__global__ void zero_u64_kernel(unsigned long long* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0ull;
}

// EMD of the two histograms' CDFs (losses.py:8-22), one workgroup per image:
// loss += weight/n * sum_t (cx_t - cy_t)^2; ghist[s] = gscale*weight/n * 2 * sum_{t>=s} (cx_t - cy_t).
__global__ __launch_bounds__(kBins) void emd_kernel(const float* __restrict__ hx, const float* __restrict__ hy,
                                                    float w_over_n, const float* __restrict__ gscale,
                                                    float* loss, float* __restrict__ ghist) {
  __shared__ float d[kBins];
  __shared__ float sh[kBins / 64];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  d[t] = hx[b * kBins + t] - hy[b * kBins + t];
  __syncthreads();
  // inclusive prefix sum (Hillis-Steele in LDS; 256 entries)
  for (int off = 1; off < kBins; off <<= 1) {
    const float v = t >= off ? d[t - off] : 0.f;
    __syncthreads();
    d[t] += v;
    __syncthreads();
  }
  const float e = d[t];  // cdf_x[t] - cdf_y[t]
  float s = e * e;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((t & 63) == 0) sh[t >> 6] = s;
  __syncthreads();
  if (loss) ast_det::loss_acc_commit(loss, w_over_n * ((sh[0] + sh[1]) + (sh[2] + sh[3])));
  if (!ghist) return;
  // suffix sum of e: sum_{u >= t} e_u
  __syncthreads();
  d[t] = e;
  __syncthreads();
  for (int off = 1; off < kBins; off <<= 1) {
    const float v = t + off < kBins ? d[t + off] : 0.f;
    __syncthreads();
    d[t] += v;
    __syncthreads();
  }
  ghist[b * kBins + t] = 2.0f * w_over_n * gs(gscale) * d[t];
}

// dx = inv_norm * sum_k g_k dphi_k/dx = inv_norm/W * sum_j sig'(a_j) (g_j - g_{j-1}), g_{-1} = g_K = 0.
__global__ __launch_bounds__(kThreads) void soft_hist_backward_kernel(const float* __restrict__ x, int64_t m,
                                                                      float inv_norm, const float* __restrict__ ghist,
                                                                      float* __restrict__ dx, int accumulate) {
  __shared__ float dg[kBins + 1];
  const float* gb = ghist + (int64_t)blockIdx.y * kBins;
  for (int j = threadIdx.x; j <= kBins; j += kThreads) dg[j] = (j < kBins ? gb[j] : 0.f) - (j > 0 ? gb[j - 1] : 0.f);
  __syncthreads();
  const float c = inv_norm * kInvW;
  const float* xb = x + (int64_t)blockIdx.y * m;
  float* db = dx + (int64_t)blockIdx.y * m;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < m; i += (int64_t)gridDim.x * kThreads) {
    const float v = xb[i];
    float acc = 0.f;
    if (v == v) {
      int j0, j1;
      window(v, j0, j1);
      for (int j = j0; j <= j1; ++j) {
        const float s = sigm((v - (float)j * kL) * kInvW);
        acc = fmaf(s * (1.0f - s), dg[j], acc);
      }
    } else {
      acc = v;
    }
    const float g = c * acc;
    db[i] = accumulate ? db[i] + g : g;
  }
}

__device__ __forceinline__ float huber(float d) {
  const float a = fabsf(d);
  return a < 1.f ? 0.5f * d * d : a - 0.5f;
}
__device__ __forceinline__ float huber_grad(float d) { return d < -1.f ? -1.f : (d > 1.f ? 1.f : d); }

// out_of_range_loss: w * mean huber(x - clip(x, 0, 1)); the clipped copy is detached (train.py:259)
__global__ void range_loss_kernel(const float* __restrict__ x, int64_t n, float w_over_n,
                                  const float* __restrict__ gscale, float* loss, float* __restrict__ dx,
                                  int accumulate) {
  __shared__ float sh[kThreads / 64];
  const float c = w_over_n * gs(gscale);
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const float v = x[i];
    const float d = v - fminf(fmaxf(v, 0.f), 1.f);
    s += huber(d);
    if (dx) {
      const float g = c * huber_grad(d);
      dx[i] = accumulate ? dx[i] + g : g;
    }
  }
  const float t = block_sum(s, sh);
  if (loss) ast_det::loss_acc_commit(loss, w_over_n * t);
}

// w * mean((x - y)^2); dx = 2 w (x - y) / n
__global__ void sqdiff_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t n, float w_over_n,
                              const float* __restrict__ gscale, float* loss, float* __restrict__ dx, int accumulate) {
  __shared__ float sh[kThreads / 64];
  const float c = 2.f * w_over_n * gs(gscale);
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const float d = x[i] - y[i];
    s = fmaf(d, d, s);
    if (dx) {
      const float g = c * d;
      dx[i] = accumulate ? dx[i] + g : g;
    }
  }
  const float t = block_sum(s, sh);
  if (loss) ast_det::loss_acc_commit(loss, w_over_n * t);
}

unsigned grid_for(int64_t n, int64_t per_block_min) {
  int64_t b = (n + per_block_min - 1) / per_block_min;
  return (unsigned)(b < 1 ? 1 : (b > AST_LOSS_SLOTS ? AST_LOSS_SLOTS : b));
}

}  // namespace

extern "C" {

long long ast_soft_hist_workspace_floats(int n) { return n > 0 ? 2LL * n * (kBins + 1) : 0; }

int ast_soft_hist_f32(const float* x, int n, long long m, float inv_norm, float* hist, float* workspace,
                      long long workspace_floats, void* stream) {
  if (!x || !hist || !workspace) return AST_E_NULLPTR;
  if (n <= 0 || m <= 0 || n > 65535 || m >= (1LL << 30)) return AST_E_SHAPE;
  if (workspace_floats < ast_soft_hist_workspace_floats(n) || ((uintptr_t)workspace & 7)) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(workspace);
  hipLaunchKernelGGL(zero_u64_kernel, dim3(1), dim3(kThreads), 0, st, acc, (int64_t)n * (kBins + 1));
  const unsigned bpi = grid_for(m, 8 * kThreads) > 512 ? 512 : grid_for(m, 8 * kThreads);
  hipLaunchKernelGGL(soft_hist_kernel, dim3(bpi, n), dim3(kThreads), 0, st, x, (int64_t)m, acc);
  hipLaunchKernelGGL(hist_finish_kernel, dim3((n * kBins + kThreads - 1) / kThreads), dim3(kThreads), 0, st, acc, n,
                     inv_norm, hist);
  return (int)hipGetLastError();
}

int ast_emd_loss_f32(const float* hx, const float* hy, int n, float weight, const float* gscale, float* loss,
                     float* ghist, void* stream) {
  if (!hx || !hy || (!loss && !ghist)) return AST_E_NULLPTR;
  if (n <= 0 || n > AST_LOSS_SLOTS) return AST_E_SHAPE;
  hipLaunchKernelGGL(emd_kernel, dim3(n), dim3(kBins), 0, (hipStream_t)stream, hx, hy, weight / (float)n, gscale,
                     loss, ghist);
  return (int)hipGetLastError();
}

int ast_soft_hist_backward_f32(const float* x, int n, long long m, float inv_norm, const float* ghist, float* dx,
                               int accumulate, void* stream) {
  if (!x || !ghist || !dx) return AST_E_NULLPTR;
  if (n <= 0 || m <= 0 || n > 65535) return AST_E_SHAPE;
  const unsigned bpi = grid_for(m, 4 * kThreads) > 1024 ? 1024 : grid_for(m, 4 * kThreads);
  hipLaunchKernelGGL(soft_hist_backward_kernel, dim3(bpi, n), dim3(kThreads), 0, (hipStream_t)stream, x,
                     (int64_t)m, inv_norm, ghist, dx, accumulate);
  return (int)hipGetLastError();
}

int ast_range_loss_f32(const float* x, long long numel, float weight, const float* gscale, float* loss, float* dx,
                       int accumulate, void* stream) {
  if (!x || (!loss && !dx)) return AST_E_NULLPTR;
  if (numel <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(range_loss_kernel, dim3(std::min(grid_for(numel, 4 * kThreads), 256u)), dim3(kThreads), 0, (hipStream_t)stream,
                     x, (int64_t)numel, weight / (float)numel, gscale, loss, dx, accumulate);
  return (int)hipGetLastError();
}

int ast_sqdiff_mean_f32(const float* x, const float* y, long long numel, float weight, const float* gscale,
                        float* loss, float* dx, int accumulate, void* stream) {
  if (!x || !y || (!loss && !dx)) return AST_E_NULLPTR;
  if (numel <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(sqdiff_kernel, dim3(std::min(grid_for(numel, 4 * kThreads), 256u)), dim3(kThreads), 0, (hipStream_t)stream, x,
                     y, (int64_t)numel, weight / (float)numel, gscale, loss, dx, accumulate);
  return (int)hipGetLastError();
}

}  // extern "C"
