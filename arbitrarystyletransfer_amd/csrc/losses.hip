// Style-transfer losses for gfx950: losses.py gram_matrix (105-109), compute_content_loss
// (124-126), compute_style_loss (128-139), tv_loss (90-103), with mean_variance_norm
// (models.py:64-68) fused into the content term. Each loss kernel produces its value (added into a
// loss accumulator, det.h: per-workgroup partials summed in a fixed order) and, when asked, the
// input gradient, so the training step needs no separate backward pass through PyTorch.
//
//  * gram: batched fp32 MFMA GEMM G[b] = s·F[b]F[b]^T (F = C x HW), split-K over HW (C <= 512, HW
//    up to 512^2: few output tiles, very long K); the splits' partial tiles are summed in split
//    order (det.h), never through atomics.
//  * gram backward: dF[b] (+)= s·(dG+dG^T)[b]·F[b] + ra[b,i]·F[b][i,:] + rb[b,i] — the GEMM
//    epilogue also adds the mean/std-term gradients of compute_style_loss (per-plane affine in F).
//  * Huber: delta = 1, reduction 'mean' (F.huber_loss default).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../include/ast_hip.h"
#include "det.h"
#include "x3.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;

__device__ __forceinline__ float huber(float d) {
  const float a = fabsf(d);
  return a < 1.f ? 0.5f * d * d : a - 0.5f;
}
__device__ __forceinline__ float huber_grad(float d) { return d < -1.f ? -1.f : (d > 1.f ? 1.f : d); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 256-thread block sum; every thread receives the total.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__device__ void plane_mean_std(const float* __restrict__ p, int64_t n, float eps, float* sh, float& mean, float& sd) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) s += p[i];
  mean = block_sum(s, sh) / (float)n;
  float q = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) {
    const float d = p[i] - mean;
    q += d * d;
  }
  sd = sqrtf(block_sum(q, sh) / (float)(n - 1) + eps);
}

__device__ __forceinline__ float gs(const float* g) { return g ? *g : 1.f; }

// One-pass plane moments: every thread keeps shifted sums around its own first element, the
// (count, mean, M2) triples are merged with Chan's parallel formula across lanes and waves.
struct Mom {
  float n, mean, m2;
};

__device__ __forceinline__ Mom mom_merge(Mom a, Mom b) {
  const float n = a.n + b.n;
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float d = b.mean - a.mean, f = b.n / n;
  return {n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}

__device__ __forceinline__ Mom mom_block(Mom m, float* sh) {  // sh: 12 floats
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Mom t{__shfl_xor(m.n, o, 64), __shfl_xor(m.mean, o, 64), __shfl_xor(m.m2, o, 64)};
    m = mom_merge(m, t);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    sh[3 * w] = m.n;
    sh[3 * w + 1] = m.mean;
    sh[3 * w + 2] = m.m2;
  }
  __syncthreads();
  Mom r{sh[0], sh[1], sh[2]};
#pragma unroll
  for (int w = 1; w < 4; ++w) r = mom_merge(r, Mom{sh[3 * w], sh[3 * w + 1], sh[3 * w + 2]});
  return r;
}

// mean and sqrt(M2/(n-1) + eps) of two planes in ONE read of each.
__device__ void plane_mean_std2(const float* __restrict__ p, const float* __restrict__ q, int64_t n, float eps,
                                float* sh, float& mp, float& sp, float& mq, float& sq) {
  float kp = 0.f, kq = 0.f, s1p = 0.f, s2p = 0.f, s1q = 0.f, s2q = 0.f, c = 0.f;
  const int64_t i0 = threadIdx.x;
  if (i0 < n) {
    kp = p[i0];
    kq = q[i0];
  }
  for (int64_t i = i0; i < n; i += kThreads) {
    const float a = p[i] - kp, b = q[i] - kq;
    s1p += a;
    s2p += a * a;
    s1q += b;
    s2q += b * b;
    c += 1.f;
  }
  Mom A{c, c > 0.f ? kp + s1p / c : 0.f, c > 0.f ? fmaxf(s2p - s1p * s1p / c, 0.f) : 0.f};
  Mom B{c, c > 0.f ? kq + s1q / c : 0.f, c > 0.f ? fmaxf(s2q - s1q * s1q / c, 0.f) : 0.f};
  A = mom_block(A, sh);
  B = mom_block(B, sh);
  mp = A.mean;
  sp = sqrtf(A.m2 / (float)(n - 1) + eps);
  mq = B.mean;
  sq = sqrtf(B.m2 / (float)(n - 1) + eps);
}

// ------------------------------------------------------------------------------------------
// Content term: w * huber(mvn(x), mvn(y)) (mean over all elements), dx += d/dx.
// mvn z = (x-mu)/sigma, sigma = sqrt(var_unbiased + 1e-5). With g = dL/dz:
//   dx = (g - mean(g) - z * sum(g z)/(N-1)) / sigma.
// ------------------------------------------------------------------------------------------
// Forward: one read of x and y for both planes' moments, one for the Huber sums. With pstats,
// also keeps per plane (mu_x, sd_x, mu_y, sd_y, mean(g), sum(g z)/(N-1)) for the backward.
__global__ __launch_bounds__(kThreads) void mvn_huber_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                             int64_t planes, int64_t hw, float inv_numel, float w,
                                                             float* loss, float* __restrict__ pstats) {
  __shared__ float sh[12];
  float Hs = 0.f;  // this workgroup's planes, in plane order
  for (int64_t p = blockIdx.x; p < planes; p += gridDim.x) {
    const float* xp = x + p * hw;
    const float* yp = y + p * hw;
    float mx, sx, my, sy;
    plane_mean_std2(xp, yp, hw, 1e-5f, sh, mx, sx, my, sy);
    float sh_ = 0.f, sg = 0.f, sgz = 0.f;
    for (int64_t i = threadIdx.x; i < hw; i += kThreads) {
      const float z = (xp[i] - mx) / sx;
      const float d = z - (yp[i] - my) / sy;
      sh_ += huber(d);
      const float g = huber_grad(d);
      sg += g;
      sgz += g * z;
    }
    Hs += block_sum(sh_, sh);
    if (pstats) {
      const float G = block_sum(sg, sh);
      const float GZ = block_sum(sgz, sh);
      if (threadIdx.x == 0) {
        float* s = pstats + 6 * p;
        s[0] = mx; s[1] = sx; s[2] = my; s[3] = sy;
        s[4] = G / (float)hw;
        s[5] = GZ / (float)(hw - 1);
      }
    }
  }
  if (loss) ast_det::loss_acc_commit(loss, w * Hs * inv_numel);
}

// Backward: dx = c * (huber'(d) - mean(g) - z * sum(g z)/(N-1)) / sd_x, one read of x and y.
// grid (pixel chunks of 4 * kThreads, planes strided by gridDim.y): the plane's statistics are read
// once, 16-byte accesses where the plane is 4-aligned, no per-element index division.
__global__ __launch_bounds__(kThreads) void mvn_huber_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                                 const float* __restrict__ pstats, int64_t hw,
                                                                 int64_t planes, float c,
                                                                 const float* __restrict__ gscale, float* __restrict__ dx,
                                                                 int accumulate) {
  const float cc = c * gs(gscale);
  const bool vec = (hw & 3) == 0 && ((((uintptr_t)x | (uintptr_t)y | (uintptr_t)dx) & 15) == 0);
  for (int64_t p = blockIdx.y; p < planes; p += gridDim.y) {
    const float* s = pstats + 6 * p;
    const float s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3], s4 = s[4], s5 = s[5];
    const float* xp = x + p * hw;
    const float* yp = y + p * hw;
    float* dp = dx + p * hw;
    const float i1 = 1.f / s1, i3 = 1.f / s3, c1 = cc * i1;
    auto one = [&](float xv, float yv) {
      const float z = (xv - s0) * i1;
      const float d = z - (yv - s2) * i3;
      return c1 * (huber_grad(d) - s4 - z * s5);
    };
    for (int64_t i = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 4; i < hw; i += (int64_t)gridDim.x * kThreads * 4) {
      if (vec) {
        const float4 xv = *reinterpret_cast<const float4*>(xp + i), yv = *reinterpret_cast<const float4*>(yp + i);
        float4 v = make_float4(one(xv.x, yv.x), one(xv.y, yv.y), one(xv.z, yv.z), one(xv.w, yv.w));
        if (accumulate) {
          const float4 o = *reinterpret_cast<const float4*>(dp + i);
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        *reinterpret_cast<float4*>(dp + i) = v;
      } else {
        for (int64_t j = i; j < i + 4 && j < hw; ++j) {
          const float v = one(xp[j], yp[j]);
          dp[j] = accumulate ? dp[j] + v : v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Split-plane forms (the *_ws entries): a plane is cut into chunks of kChunk elements, one
// workgroup per (chunk, plane), 16-byte loads where the planes are 4-aligned. The one-workgroup-
// per-plane kernels above leave most of the chip idle on few, large planes (48 image planes of
// 512^2: 0.86 ms for 200 MB) and read with 4-byte loads. Partials go to the workspace and are
// merged in chunk order (det.h), so results do not depend on workgroup timing.
//   part  [planes][nchunks][6]: (count, mean_x, M2_x, mean_y, M2_y, -) of the chunk
//   hpart [planes][nchunks][4]: (sum huber, sum g, sum g z, -) of the chunk
// ------------------------------------------------------------------------------------------
constexpr int kChunk = 8192;

__device__ __forceinline__ bool vec4_ok(const float* x, const float* y, int64_t hw) {
  return (hw & 3) == 0 && ((((uintptr_t)x | (uintptr_t)y) & 15) == 0);
}

__global__ __launch_bounds__(kThreads) void moments_part_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                                int64_t planes, int64_t hw, int nchunks,
                                                                float* __restrict__ part) {
  __shared__ float sh[12];
  const int64_t c0 = (int64_t)blockIdx.x * kChunk, c1 = min(hw, c0 + (int64_t)kChunk);
  const bool vec = vec4_ok(x, y, hw);
  for (int64_t p = blockIdx.y; p < planes; p += gridDim.y) {
    const float* xp = x + p * hw;
    const float* yp = y + p * hw;
    float kp = 0.f, kq = 0.f, s1p = 0.f, s2p = 0.f, s1q = 0.f, s2q = 0.f, c = 0.f;
    auto add = [&](float u, float v) {
      const float a = u - kp, b = v - kq;
      s1p += a;
      s2p += a * a;
      s1q += b;
      s2q += b * b;
    };
    if (vec) {
      const int64_t i0 = c0 + 4 * threadIdx.x;
      if (i0 < c1) {
        kp = xp[i0];
        kq = yp[i0];
      }
#pragma unroll 4
      for (int64_t i = i0; i < c1; i += 4 * kThreads) {
        const float4 a = *reinterpret_cast<const float4*>(xp + i), b = *reinterpret_cast<const float4*>(yp + i);
        add(a.x, b.x);
        add(a.y, b.y);
        add(a.z, b.z);
        add(a.w, b.w);
        c += 4.f;
      }
    } else {
      const int64_t i0 = c0 + threadIdx.x;
      if (i0 < c1) {
        kp = xp[i0];
        kq = yp[i0];
      }
      for (int64_t i = i0; i < c1; i += kThreads) {
        add(xp[i], yp[i]);
        c += 1.f;
      }
    }
    Mom A{c, c > 0.f ? kp + s1p / c : 0.f, c > 0.f ? fmaxf(s2p - s1p * s1p / c, 0.f) : 0.f};
    Mom B{c, c > 0.f ? kq + s1q / c : 0.f, c > 0.f ? fmaxf(s2q - s1q * s1q / c, 0.f) : 0.f};
    A = mom_block(A, sh);
    B = mom_block(B, sh);
    if (threadIdx.x == 0) {
      float* o = part + (p * nchunks + blockIdx.x) * 6;
      o[0] = A.n;
      o[1] = A.mean;
      o[2] = A.m2;
      o[3] = B.mean;
      o[4] = B.m2;
      o[5] = 0.f;
    }
  }
}

// The plane's moments from its chunk partials, merged in chunk order (every caller the same way).
__device__ __forceinline__ void plane_moments(const float* __restrict__ part, int64_t p, int nchunks, int64_t hw,
                                              float eps, float& mx, float& sx, float& my, float& sy) {
  const float* q = part + p * nchunks * 6;
  Mom A{q[0], q[1], q[2]}, B{q[0], q[3], q[4]};
  for (int k = 1; k < nchunks; ++k) {
    const float* r = q + 6 * k;
    A = mom_merge(A, Mom{r[0], r[1], r[2]});
    B = mom_merge(B, Mom{r[0], r[3], r[4]});
  }
  mx = A.mean;
  sx = sqrtf(A.m2 / (float)(hw - 1) + eps);
  my = B.mean;
  sy = sqrtf(B.m2 / (float)(hw - 1) + eps);
}

__global__ __launch_bounds__(kThreads) void mvn_huber_part_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                                  int64_t planes, int64_t hw, int nchunks,
                                                                  const float* __restrict__ part,
                                                                  float* __restrict__ hpart, float* __restrict__ pstats) {
  const int64_t c0 = (int64_t)blockIdx.x * kChunk, c1 = min(hw, c0 + (int64_t)kChunk);
  const bool vec = vec4_ok(x, y, hw);
  for (int64_t p = blockIdx.y; p < planes; p += gridDim.y) {
    float mx, sx, my, sy;
    plane_moments(part, p, nchunks, hw, 1e-5f, mx, sx, my, sy);
    const float* xp = x + p * hw;
    const float* yp = y + p * hw;
    float sh_ = 0.f, sg = 0.f, sgz = 0.f;
    const float isx = 1.f / sx, isy = 1.f / sy;  // two divisions per element made this pass VALU-bound
    auto one = [&](float u, float v) {
      const float z = (u - mx) * isx;
      const float d = z - (v - my) * isy;
      sh_ += huber(d);
      const float g = huber_grad(d);
      sg += g;
      sgz += g * z;
    };
    if (vec) {
#pragma unroll 4
      for (int64_t i = c0 + 4 * threadIdx.x; i < c1; i += 4 * kThreads) {
        const float4 a = *reinterpret_cast<const float4*>(xp + i), b = *reinterpret_cast<const float4*>(yp + i);
        one(a.x, b.x);
        one(a.y, b.y);
        one(a.z, b.z);
        one(a.w, b.w);
      }
    } else {
      for (int64_t i = c0 + threadIdx.x; i < c1; i += kThreads) one(xp[i], yp[i]);
    }
    const float H = ast_det::block_sum_fixed(sh_);
    const float G = ast_det::block_sum_fixed(sg);
    const float GZ = ast_det::block_sum_fixed(sgz);
    if (threadIdx.x == 0) {
      float* o = hpart + (p * nchunks + blockIdx.x) * 4;
      o[0] = H;
      o[1] = G;
      o[2] = GZ;
      o[3] = 0.f;
      if (pstats && blockIdx.x == 0) {
        float* s = pstats + 6 * p;
        s[0] = mx; s[1] = sx; s[2] = my; s[3] = sy;
      }
    }
  }
}

// Per plane (one thread each): the chunk sums in chunk order -> pstats[4..5]; the Huber sums of the
// workgroup's planes, in plane order, into the loss accumulator.
__global__ __launch_bounds__(kThreads) void mvn_huber_fin_kernel(const float* __restrict__ hpart, int64_t planes,
                                                                 int nchunks, int64_t hw, float inv_numel, float w,
                                                                 float* loss, float* __restrict__ pstats) {
  float Hs = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < planes; p += (int64_t)gridDim.x * kThreads) {
    const float* q = hpart + p * nchunks * 4;
    float H = 0.f, G = 0.f, GZ = 0.f;
    for (int k = 0; k < nchunks; ++k) {
      H += q[4 * k];
      G += q[4 * k + 1];
      GZ += q[4 * k + 2];
    }
    Hs += H;
    if (pstats) {
      pstats[6 * p + 4] = G / (float)hw;
      pstats[6 * p + 5] = GZ / (float)(hw - 1);
    }
  }
  const float t = ast_det::block_sum_fixed(Hs);
  if (loss) ast_det::loss_acc_commit(loss, w * t * inv_numel);
}

// style_stats_kernel's (mu_x, sd_x, mu_y, sd_y) from the chunk partials (unbiased, no eps).
__global__ __launch_bounds__(kThreads) void style_stats_fin_kernel(const float* __restrict__ part, int64_t planes,
                                                                   int nchunks, int64_t hw, float* __restrict__ stats) {
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < planes; p += (int64_t)gridDim.x * kThreads) {
    float mx, sx, my, sy;
    plane_moments(part, p, nchunks, hw, 0.f, mx, sx, my, sy);
    stats[4 * p + 0] = mx;
    stats[4 * p + 1] = sx;
    stats[4 * p + 2] = my;
    stats[4 * p + 3] = sy;
  }
}

// Backward of mean_variance_norm alone: dx = (g - mean(g) - z*sum(g z)/(N-1)) / sigma.
__global__ __launch_bounds__(kThreads) void mvn_backward_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                                float* __restrict__ dx, int64_t hw, float eps) {
  __shared__ float sh[4];
  const int64_t p = blockIdx.x;
  const float* xp = x + p * hw;
  const float* gp = g + p * hw;
  float m, sd;
  plane_mean_std(xp, hw, eps, sh, m, sd);
  float sg = 0.f, sgz = 0.f;
  for (int64_t i = threadIdx.x; i < hw; i += kThreads) {
    const float gi = gp[i];
    sg += gi;
    sgz += gi * (xp[i] - m) / sd;
  }
  const float G = block_sum(sg, sh) / (float)hw;
  const float GZ = block_sum(sgz, sh) / (float)(hw - 1);
  float* dp = dx + p * hw;
  for (int64_t i = threadIdx.x; i < hw; i += kThreads) dp[i] = (gp[i] - G - (xp[i] - m) / sd * GZ) / sd;
}

// Backward of channel_stats / calc_mean_std: dx = dmean/N + dstd*(x-mean)/((N-unbiased)*std).
__global__ void stats_backward_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                      const float* __restrict__ sd, const float* __restrict__ dmean,
                                      const float* __restrict__ dsd, float* __restrict__ dx, int64_t hw, int64_t n,
                                      int unbiased, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const int64_t p = i / hw;
    float v = 0.f;
    if (dmean) v += dmean[p] / (float)hw;
    if (dsd) v += dsd[p] * (x[i] - mean[p]) / ((float)(hw - unbiased) * sd[p]);
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

// Plain Huber (compute_content_loss on raw tensors): loss += w*mean(huber(x-y)), dx (+)= grad.
__global__ void huber_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t n, float inv_numel,
                             float w, const float* __restrict__ gscale, float* loss, float* __restrict__ dx,
                             int accumulate) {
  __shared__ float sh[4];
  const float c = w * inv_numel * gs(gscale);
  float s = 0.f;
  if ((n & 3) == 0 && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)(dx ? dx : x)) & 15) == 0) {
    // 16-byte accesses (the grid is capped for the loss commit, so each thread streams many
    // elements: 4x fewer memory instructions); a fixed element-to-thread map, deterministic
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* y4 = reinterpret_cast<const float4*>(y);
    float4* d4 = reinterpret_cast<float4*>(dx);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * kThreads) {
      const float4 a = x4[i], b = y4[i];
      const float d[4] = {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w};
      s += (huber(d[0]) + huber(d[1])) + (huber(d[2]) + huber(d[3]));
      if (dx) {
        float4 v = make_float4(c * huber_grad(d[0]), c * huber_grad(d[1]), c * huber_grad(d[2]), c * huber_grad(d[3]));
        if (accumulate) {
          const float4 o = d4[i];
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        d4[i] = v;
      }
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
      const float d = x[i] - y[i];
      s += huber(d);
      if (dx) {
        const float v = c * huber_grad(d);
        dx[i] = accumulate ? dx[i] + v : v;
      }
    }
  }
  const float t = block_sum(s, sh);
  if (loss) ast_det::loss_acc_commit(loss, w * t * inv_numel);
}

// ------------------------------------------------------------------------------------------
// Style mean/std terms. stats[p] = (mu_x, sd_x, mu_y, sd_y) (unbiased, no eps = channel_stats).
// loss += w*1.25*(mean huber(mu_x-mu_y) + mean huber(sd_x-sd_y)) over the B*C planes;
// per-plane gradient dx = ra*x + rb with ra = dsd/((N-1) sd), rb = dmu/N - ra*mu.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void style_stats_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                               int64_t hw, float* __restrict__ stats) {
  __shared__ float sh[12];
  const int64_t p = blockIdx.x;
  float mx, sx, my, sy;
  plane_mean_std2(x + p * hw, y + p * hw, hw, 0.f, sh, mx, sx, my, sy);
  if (threadIdx.x == 0) {
    stats[4 * p + 0] = mx;
    stats[4 * p + 1] = sx;
    stats[4 * p + 2] = my;
    stats[4 * p + 3] = sy;
  }
}

__global__ void style_moment_loss_kernel(const float* __restrict__ stats, int64_t planes, int64_t hw, float w,
                                         const float* __restrict__ gscale, float* loss, float* __restrict__ ra,
                                         float* __restrict__ rb) {
  __shared__ float sh[4];
  const float inv = 1.f / (float)planes;
  const float c = w * 1.25f * inv * gs(gscale);
  float s = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < planes; p += (int64_t)gridDim.x * kThreads) {
    const float mx = stats[4 * p], sx = stats[4 * p + 1], my = stats[4 * p + 2], sy = stats[4 * p + 3];
    s += huber(mx - my) + huber(sx - sy);
    if (ra) {
      const float dmu = c * huber_grad(mx - my), dsd = c * huber_grad(sx - sy);
      const float a = dsd / ((float)(hw - 1) * sx);
      ra[p] = a;
      rb[p] = dmu / (float)hw - a * mx;
    }
  }
  const float t = block_sum(s, sh);
  if (loss) ast_det::loss_acc_commit(loss, w * 1.25f * t * inv);
}

// Gram huber: loss += w*10*mean(huber(Gx-Gy)); dG = w*10*huber'(Gx-Gy)/numel (gscale'd).
__global__ void gram_huber_kernel(const float* __restrict__ gx, const float* __restrict__ gy, int64_t n, float w,
                                  const float* __restrict__ gscale, float* loss, float* __restrict__ dg) {
  __shared__ float sh[4];
  const float inv = 1.f / (float)n;
  const float c = w * 10.f * inv * gs(gscale);
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const float d = gx[i] - gy[i];
    s += huber(d);
    if (dg) dg[i] = c * huber_grad(d);
  }
  const float t = block_sum(s, sh);
  if (loss) ast_det::loss_acc_commit(loss, w * 10.f * t * inv);
}

// ------------------------------------------------------------------------------------------
// TV: loss += w * (sum (x[.., j]-x[.., j+1])^2 + sum (x[i, ..]-x[i+1, ..])^2); dx (+)= grad.
// ------------------------------------------------------------------------------------------
__global__ void tv_kernel(const float* __restrict__ x, int64_t planes, int H, int W, float w,
                          const float* __restrict__ gscale, float* loss, float* __restrict__ dx, int accumulate) {
  __shared__ float sh[4];
  const int64_t n = planes * H * W;
  const float c = 2.f * w * gs(gscale);
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const int j = (int)(i % W);
    const int r = (int)((i / W) % H);
    const float v = x[i];
    float g = 0.f;
    if (j + 1 < W) {
      const float d = v - x[i + 1];
      s += d * d;
      g += d;
    }
    if (j > 0) g -= x[i - 1] - v;
    if (r + 1 < H) {
      const float d = v - x[i + W];
      s += d * d;
      g += d;
    }
    if (r > 0) g -= x[i - W] - v;
    if (dx) dx[i] = accumulate ? dx[i] + c * g : c * g;
  }
  const float t = block_sum(s, sh);
  if (loss) ast_det::loss_acc_commit(loss, w * t);
}

// ------------------------------------------------------------------------------------------
// Gram forward: G[blockIdx.y][b][i][j] = s * sum_{k in split} F[b][i][k] F[b][j][k], k-range split over
// blockIdx.y (G is the gram itself with one split, else the workspace of partial tiles).
// 64x64 output tile, 4 waves (2x2 of 32x32), BK = 32; F tiles transposed into LDS [k][row].
// G is symmetric: only the tiles ti <= tj are computed (blockIdx.x enumerates
// them row by row), an off-diagonal tile is stored at (ti, tj) and mirrored at (tj, ti), a diagonal
// tile's upper half is stored and mirrored (G is exactly symmetric, whatever the summation order).
// ------------------------------------------------------------------------------------------
constexpr int GT = 64, GBK = 32;

__global__ __launch_bounds__(256) void gram_kernel(const float* __restrict__ F, float* __restrict__ G, int C,
                                                   int64_t K, int64_t kchunk, float s) {
  __shared__ float As[GBK][GT + 4];
  __shared__ float Bs[GBK][GT + 4];
  const int tiles = (C + GT - 1) / GT;
  int ti = 0, tj = blockIdx.x;  // upper-triangle index -> (ti, tj), ti <= tj
  while (tj >= tiles - ti) {
    tj -= tiles - ti;
    ++ti;
  }
  tj += ti;
  const int b = blockIdx.z;
  const int64_t k0 = (int64_t)blockIdx.y * kchunk;
  const int64_t k1 = min(K, k0 + kchunk);
  const float* Fb = F + (int64_t)b * C * K;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wi = wave & 1, wj = wave >> 1;
  // a diagonal tile reads its rows once (both operands from As), and its lower-left 32x32 quadrant,
  // which is never stored (the mirror of the upper-right one), is not computed
  const bool diag = ti == tj, idle = diag && wi > wj;
  const float(*Bp)[GT + 4] = diag ? As : Bs;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const bool vec = ((K & 3) == 0) && ((k0 & 3) == 0);
  // 64 rows x 32 k for each operand: 512 float4 each -> 2 per thread per operand, the next chunk's
  // in registers while the current one's MFMAs run
  float4 va[2], vb[2];
  auto load = [&](int64_t kb) {
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      const int e = tid + rep * 256;  // 0..511
      const int row = e >> 3, kq = (e & 7) * 4;
      const int ri = ti * GT + row, rj = tj * GT + row;
      va[rep] = make_float4(0.f, 0.f, 0.f, 0.f);
      vb[rep] = va[rep];
      const int64_t kk = kb + kq;
      if (vec && kk + 3 < k1) {
        if (ri < C) va[rep] = *reinterpret_cast<const float4*>(Fb + (int64_t)ri * K + kk);
        if (!diag && rj < C) vb[rep] = *reinterpret_cast<const float4*>(Fb + (int64_t)rj * K + kk);
      } else {
        float ta[4] = {0.f, 0.f, 0.f, 0.f}, tb[4] = {0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < 4; ++q) {
          if (kk + q < k1) {
            if (ri < C) ta[q] = Fb[(int64_t)ri * K + kk + q];
            if (!diag && rj < C) tb[q] = Fb[(int64_t)rj * K + kk + q];
          }
        }
        va[rep] = make_float4(ta[0], ta[1], ta[2], ta[3]);
        vb[rep] = make_float4(tb[0], tb[1], tb[2], tb[3]);
      }
    }
  };
  if (k0 < k1) load(k0);
  for (int64_t kb = k0; kb < k1; kb += GBK) {
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      const int e = tid + rep * 256;
      const int row = e >> 3, kq = (e & 7) * 4;
      As[kq + 0][row] = va[rep].x; As[kq + 1][row] = va[rep].y; As[kq + 2][row] = va[rep].z; As[kq + 3][row] = va[rep].w;
      if (!diag) {
        Bs[kq + 0][row] = vb[rep].x; Bs[kq + 1][row] = vb[rep].y; Bs[kq + 2][row] = vb[rep].z; Bs[kq + 3][row] = vb[rep].w;
      }
    }
    __syncthreads();
    if (kb + GBK < k1) load(kb + GBK);
    if (!idle) {
#pragma unroll
      for (int kp = 0; kp < GBK / 2; ++kp) {
        const float a = As[2 * kp + h][wi * 32 + l32];
        const float bv = Bp[2 * kp + h][wj * 32 + l32];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc, 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (idle) return;
  float* Gb = G + ((int64_t)blockIdx.y * gridDim.z + b) * C * C;
  const int j = tj * GT + wj * 32 + l32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = ti * GT + wi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (i < C && j < C && (ti != tj || i <= j)) {  // diagonal tiles: the upper half, mirrored
      Gb[(int64_t)i * C + j] = s * acc[r];
      Gb[(int64_t)j * C + i] = s * acc[r];
    }
  }
}

// Gram forward on the split-bf16 matrix cores (round 6; AST_GRAM_X3=0 selects gram_kernel above).
// Every gram of the style loss is 2 C^2 HW B = 34 GFLOP (C^2 HW is the same at every VGG tap); the
// LDS-staged gram_kernel runs them at 91-147 TF on the fp32 MFMA, bound by its per-chunk staging
// and barriers rather than by the MFMA (an LDS-staged split-bf16 form of it was no faster). Here
// there is no LDS and no barrier in the K loop: the 4 waves of a
// workgroup take interleaved 16-k steps of the workgroup's K range, and each computes the whole
// 64 x 64 tile (2 x 2 blocks of v_mfma_f32_32x32x16_bf16, the six term products). A lane loads its
// 8 consecutive k of 2 (diagonal tile) or 4 rows straight from HBM, one step ahead, and splits them
// in registers (ast_x3::split8). The 4 partial tiles meet in LDS at the end, summed in wave order.
// B = 8: 189 / 202 / 163 / 155 -> 145 / 141 / 140 / 124 us at C = 64 / 128 / 256 / 512
// (profiles/r06gx_gram_ab.txt).
__global__ __launch_bounds__(256, 2) void gram_x3_kernel(const float* __restrict__ F, float* __restrict__ G, int C,
                                                         int64_t K, int64_t kchunk, float s) {
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  __shared__ float red[3][64][65];  // waves 1..3's tiles for wave 0 to add
  const int tiles = (C + GT - 1) / GT;
  int ti = 0, tj = blockIdx.x;  // upper-triangle index -> (ti, tj), ti <= tj
  while (tj >= tiles - ti) {
    tj -= tiles - ti;
    ++ti;
  }
  tj += ti;
  const int b = blockIdx.z;
  const int64_t k0 = (int64_t)blockIdx.y * kchunk;
  const int64_t k1 = min(K, k0 + kchunk);
  const float* Fb = F + (int64_t)b * C * K;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const bool diag = ti == tj;
  const bool vec = ((K & 3) == 0) && ((k0 & 3) == 0);
  f32x16 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][v][r] = 0.f;
  // this lane's rows: A rows ti*64 + 32u + l32, B rows tj*64 + 32v + l32 (= A's on a diagonal tile)
  const float* ra[2];
  const float* rb[2];
  bool oka[2], okb[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = ti * GT + 32 * u + l32, j = tj * GT + 32 * u + l32;
    oka[u] = i < C;
    okb[u] = j < C;
    ra[u] = Fb + (int64_t)(oka[u] ? i : 0) * K;
    rb[u] = Fb + (int64_t)(okb[u] ? j : 0) * K;
  }
  float xa[2][8], xb[2][8];
  auto load = [&](int64_t kk) {  // k = kk + 8h .. +7 of every row
    const int64_t kq = kk + 8 * h;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (vec && kq + 7 < k1) {
        const float4 p0 = oka[u] ? *reinterpret_cast<const float4*>(ra[u] + kq) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 p1 = oka[u] ? *reinterpret_cast<const float4*>(ra[u] + kq + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        xa[u][0] = p0.x; xa[u][1] = p0.y; xa[u][2] = p0.z; xa[u][3] = p0.w;
        xa[u][4] = p1.x; xa[u][5] = p1.y; xa[u][6] = p1.z; xa[u][7] = p1.w;
        if (!diag) {
          const float4 q0 = okb[u] ? *reinterpret_cast<const float4*>(rb[u] + kq) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 q1 = okb[u] ? *reinterpret_cast<const float4*>(rb[u] + kq + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
          xb[u][0] = q0.x; xb[u][1] = q0.y; xb[u][2] = q0.z; xb[u][3] = q0.w;
          xb[u][4] = q1.x; xb[u][5] = q1.y; xb[u][6] = q1.z; xb[u][7] = q1.w;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const bool in = kq + q < k1;
          xa[u][q] = (in && oka[u]) ? ra[u][kq + q] : 0.f;
          if (!diag) xb[u][q] = (in && okb[u]) ? rb[u][kq + q] : 0.f;
        }
      }
    }
  };
  int64_t kk = k0 + 16 * wave;
  if (kk < k1) load(kk);
  for (; kk < k1; kk += 64) {
    bf16x8_t ta[2][3], tb[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      ast_x3::split8(xa[u], ta[u][0], ta[u][1], ta[u][2]);
      if (!diag) ast_x3::split8(xb[u], tb[u][0], tb[u][1], tb[u][2]);
    }
    if (kk + 64 < k1) load(kk + 64);  // the wave's next step, in flight during these MFMAs
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        if (diag && u > v) continue;  // the lower-left block of a diagonal tile is the mirror
        const bf16x8_t* bv = diag ? ta[v] : tb[v];
        f32x16 c = acc[u][v];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta[u][2], bv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta[u][0], bv[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta[u][1], bv[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta[u][1], bv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta[u][0], bv[1], c, 0, 0, 0);
        acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ta[u][0], bv[0], c, 0, 0, 0);
      }
  }
  // C layout: block (u, v), lane (col l32, half h), element r -> row 32u + (r & 3) + 8 (r >> 2) + 4h,
  // column 32v + l32 of the tile
  if (wave > 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          red[wave - 1][32 * u + (r & 3) + 8 * (r >> 2) + 4 * h][32 * v + l32] = acc[u][v][r];
  }
  __syncthreads();
  if (wave > 0) return;
  float* Gb = G + ((int64_t)blockIdx.y * gridDim.z + b) * C * C;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      if (diag && u > v) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int li = 32 * u + (r & 3) + 8 * (r >> 2) + 4 * h, lj = 32 * v + l32;
        const int i = ti * GT + li, j = tj * GT + lj;
        const float t = ((acc[u][v][r] + red[0][li][lj]) + red[1][li][lj]) + red[2][li][lj];
        if (i < C && j < C && (ti != tj || i <= j)) {  // diagonal tiles: the upper half, mirrored
          Gb[(int64_t)i * C + j] = s * t;
          Gb[(int64_t)j * C + i] = s * t;
        }
      }
    }
}

// Gram backward: dF[b][i][n] (+)= s * sum_k (dG[k][i] + dG[i][k]) F[b][k][n] + ra[b,i] F[b][i][n] + rb[b,i].
// Output tile 64 (i) x 128 (n); 4 waves 2x2, each 32 x 64; BK = 16.
#ifndef GRAM_BWD_BK  // K chunk per barrier pair; 32 and 64 were slower (fewer resident workgroups:
#define GRAM_BWD_BK 16  // profiles/r06gbk_gram_bwd_bk.txt)
#endif
constexpr int BI = 64, BNN = 128, BBK = GRAM_BWD_BK;
constexpr int BS_T = BBK * BI / 256, BF_T = BBK * BNN / 4 / 256;  // S entries / F float4 per thread

__global__ __launch_bounds__(256) void gram_bwd_kernel(const float* __restrict__ F, const float* __restrict__ dG,
                                                       float* __restrict__ dF, const float* __restrict__ ra,
                                                       const float* __restrict__ rb, int C, int64_t HW, float s,
                                                       const float* __restrict__ gscale, int accumulate) {
  __shared__ float As[BBK][BI + 4];   // S^T tile: [k][i]
  __shared__ float Bs[BBK][BNN + 4];  // F tile:  [k][n]
  const int b = blockIdx.z;
  const int ti = blockIdx.y;
  const int64_t n0 = (int64_t)blockIdx.x * BNN;
  const float* Fb = F + (int64_t)b * C * HW;
  const float* dGb = dG + (int64_t)b * C * C;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wi = wave & 1, wn = wave >> 1;
  f32x16 acc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  // the next k-chunk's S and F values in registers while the current chunk's MFMAs run
  float sv[BS_T];
  float4 fv[BF_T];
  auto load = [&](int k0) {
    // S tile: BBK k x 64 i, BS_T entries per thread
#pragma unroll
    for (int rep = 0; rep < BS_T; ++rep) {
      const int e = tid + rep * 256;
      const int kk = e >> 6, ii = e & 63;
      const int k = k0 + kk, i = ti * BI + ii;
      sv[rep] = (k < C && i < C) ? dGb[(int64_t)k * C + i] + dGb[(int64_t)i * C + k] : 0.f;
    }
    // F tile: BBK k x 128 n, BF_T float4 per thread
#pragma unroll
    for (int rep = 0; rep < BF_T; ++rep) {
      const int e = tid + rep * 256;
      const int kk = e >> 5, nq = (e & 31) * 4;
      const int k = k0 + kk;
      const int64_t nn = n0 + nq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < C) {
        const float* row = Fb + (int64_t)k * HW;
        if (((HW & 3) == 0) && nn + 3 < HW) {
          v = *reinterpret_cast<const float4*>(row + nn);
        } else {
          float t[4] = {0.f, 0.f, 0.f, 0.f};
          for (int q = 0; q < 4; ++q) if (nn + q < HW) t[q] = row[nn + q];
          v = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
      fv[rep] = v;
    }
  };
  load(0);
  for (int k0 = 0; k0 < C; k0 += BBK) {
#pragma unroll
    for (int rep = 0; rep < BS_T; ++rep) {
      const int e = tid + rep * 256;
      As[e >> 6][e & 63] = sv[rep];
    }
#pragma unroll
    for (int rep = 0; rep < BF_T; ++rep) {
      const int e = tid + rep * 256;
      *reinterpret_cast<float4*>(&Bs[e >> 5][(e & 31) * 4]) = fv[rep];
    }
    __syncthreads();
    if (k0 + BBK < C) load(k0 + BBK);
#pragma unroll
    for (int kp = 0; kp < BBK / 2; ++kp) {
      const float a = As[2 * kp + h][wi * 32 + l32];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float bv = Bs[2 * kp + h][wn * 64 + q * 32 + l32];
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[q], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  float* dFb = dF + (int64_t)b * C * HW;
  const float g = gs(gscale);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int64_t n = n0 + wn * 64 + q * 32 + l32;
    if (n >= HW) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = ti * BI + wi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (i >= C) continue;
      const int64_t off = (int64_t)i * HW + n;
      float v = s * acc[q][r];
      if (ra) v += ra[(int64_t)b * C + i] * Fb[off] + rb[(int64_t)b * C + i];
      v *= g;
      dFb[off] = accumulate ? dFb[off] + v : v;
    }
  }
}

int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, AST_LOSS_SLOTS)); }

// Grid of an elementwise loss kernel that commits to a loss accumulator: every workgroup's commit
// is an agent-scope release (an L2 writeback on the multi-XCD part), measured at ~25 ns per
// workgroup (gram_huber over 4096 workgroups: 104 us for 50 MB) -- so at most 256, looping (1024
// for tv_kernel, whose per-element index math makes long loops slower than the commits).
int loss_grid(int64_t n, int64_t cap = 256) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, cap));
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {
// split-K plan of the gram launch: >= ~1024 workgroups, chunks a multiple of GBK
int64_t gram_splits(int n, int c, int64_t hw, int64_t* kchunk_out) {
  const int tiles = (c + GT - 1) / GT;
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>((hw + 1023) / 1024, 1024 / std::max(1, n * tiles * tiles) + 1));
  int64_t kchunk = (hw + splits - 1) / splits;
  kchunk = (kchunk + GBK - 1) / GBK * GBK;
  splits = (hw + kchunk - 1) / kchunk;
  if (kchunk_out) *kchunk_out = kchunk;
  return splits;
}
}  // namespace

extern "C" {

long long ast_gram_workspace_floats(int n, int c, long long hw) {
  if (n <= 0 || c <= 0 || hw <= 0) return 0;
  const int64_t splits = gram_splits(n, c, hw, nullptr);
  return splits > 1 ? (long long)(splits * n * c * c) : 0;
}

int ast_gram_f32(const float* feat, float* gram, int n, int c, long long hw, float scale, float* workspace,
                 long long workspace_floats, void* stream) {
  if (!feat || !gram) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0 || n > 65535) return AST_E_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (c + GT - 1) / GT;
  int64_t kchunk = 0;
  const int64_t splits = gram_splits(n, c, hw, &kchunk);
  if (splits > 65535) return AST_E_SHAPE;
  if (splits > 1) {
    if (!workspace) return AST_E_NULLPTR;
    if (workspace_floats < ast_gram_workspace_floats(n, c, hw)) return AST_E_SHAPE;
  }
  static const int x3 = [] {  // AST_GRAM_X3=0: the fp32 MFMA gram_kernel (A/B measurements)
    const char* v = getenv("AST_GRAM_X3");
    return v ? atoi(v) : 1;
  }();
  hipLaunchKernelGGL(x3 ? gram_x3_kernel : gram_kernel, dim3(tiles * (tiles + 1) / 2, (unsigned)splits, n), dim3(256),
                     0, s, feat, splits > 1 ? workspace : gram, c, (int64_t)hw, kchunk, scale);
  if (splits > 1) {
    const int64_t cnt = (int64_t)n * c * c;
    const hipError_t e = ast_det::reduce_cols(workspace, splits, cnt, cnt, 1, 0, gram, 0, false, s);
    if (e != hipSuccess) return (int)e;
  }
  return (int)hipGetLastError();
}

int ast_gram_backward_f32(const float* feat, const float* dgram, float* dfeat, const float* row_a, const float* row_b,
                          int n, int c, long long hw, float scale, const float* gscale, int accumulate,
                          void* stream) {
  if (!feat || !dgram || !dfeat) return AST_E_NULLPTR;
  if ((row_a == nullptr) != (row_b == nullptr)) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0 || n > 65535) return AST_E_SHAPE;
  const int64_t nb = (hw + BNN - 1) / BNN;
  if (nb > 0x7fffffff) return AST_E_SHAPE;
  hipLaunchKernelGGL(gram_bwd_kernel, dim3((unsigned)nb, (c + BI - 1) / BI, n), dim3(256), 0, (hipStream_t)stream,
                     feat, dgram, dfeat, row_a, row_b, c, (int64_t)hw, scale, gscale, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_mvn_huber_f32(const float* x, const float* y, long long planes, long long hw, float weight, float* loss,
                      float* pstats, void* stream) {
  if (!x || !y) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 1 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  const unsigned grid = (unsigned)std::min<long long>(planes, AST_LOSS_SLOTS);
  hipLaunchKernelGGL(mvn_huber_kernel, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, x, y, (int64_t)planes,
                     (int64_t)hw, (float)(1.0 / ((double)planes * hw)), weight, loss, pstats);
  return (int)hipGetLastError();
}

long long ast_plane_stats_workspace_floats(long long planes, long long hw) {
  if (planes <= 0 || hw <= 0) return 0;
  return planes * ((hw + kChunk - 1) / kChunk) * 10;
}

// part / hpart of the split-plane kernels inside the caller's workspace
static int plane_split_plan(long long planes, long long hw, float* ws, long long ws_floats, int* nchunks,
                            unsigned* gy) {
  if (!ws) return AST_E_NULLPTR;
  if (ws_floats < ast_plane_stats_workspace_floats(planes, hw)) return AST_E_SHAPE;
  const long long nc = (hw + kChunk - 1) / kChunk;
  if (nc > 0x7fffffffLL) return AST_E_SHAPE;
  *nchunks = (int)nc;
  *gy = (unsigned)std::min<long long>(planes, 65535);
  return AST_OK;
}

int ast_mvn_huber_ws_f32(const float* x, const float* y, long long planes, long long hw, float weight, float* loss,
                         float* pstats, float* workspace, long long workspace_floats, void* stream) {
  if (!x || !y) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 1 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  int nc = 0;
  unsigned gy = 0;
  const int e = plane_split_plan(planes, hw, workspace, workspace_floats, &nc, &gy);
  if (e != AST_OK) return e;
  hipStream_t s = (hipStream_t)stream;
  float* part = workspace;
  float* hpart = workspace + planes * nc * 6;
  hipLaunchKernelGGL(moments_part_kernel, dim3((unsigned)nc, gy), dim3(kThreads), 0, s, x, y, (int64_t)planes,
                     (int64_t)hw, nc, part);
  hipLaunchKernelGGL(mvn_huber_part_kernel, dim3((unsigned)nc, gy), dim3(kThreads), 0, s, x, y, (int64_t)planes,
                     (int64_t)hw, nc, part, hpart, pstats);
  hipLaunchKernelGGL(mvn_huber_fin_kernel, dim3(grid_for(planes)), dim3(kThreads), 0, s, hpart, (int64_t)planes, nc,
                     (int64_t)hw, (float)(1.0 / ((double)planes * hw)), weight, loss, pstats);
  return (int)hipGetLastError();
}

int ast_style_moments_ws_f32(const float* x, const float* y, long long planes, long long hw, float weight,
                             const float* gscale, float* stats, float* loss, float* row_a, float* row_b,
                             float* workspace, long long workspace_floats, void* stream) {
  if (!x || !y || !stats) return AST_E_NULLPTR;
  if ((row_a == nullptr) != (row_b == nullptr)) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  int nc = 0;
  unsigned gy = 0;
  const int e = plane_split_plan(planes, hw, workspace, workspace_floats, &nc, &gy);
  if (e != AST_OK) return e;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(moments_part_kernel, dim3((unsigned)nc, gy), dim3(kThreads), 0, s, x, y, (int64_t)planes,
                     (int64_t)hw, nc, workspace);
  hipLaunchKernelGGL(style_stats_fin_kernel, dim3(grid_for(planes)), dim3(kThreads), 0, s, workspace, (int64_t)planes,
                     nc, (int64_t)hw, stats);
  hipLaunchKernelGGL(style_moment_loss_kernel, dim3(grid_for(planes)), dim3(kThreads), 0, s, stats, (int64_t)planes,
                     (int64_t)hw, weight, gscale, loss, row_a, row_b);
  return (int)hipGetLastError();
}

int ast_mvn_huber_backward_f32(const float* x, const float* y, const float* pstats, long long planes, long long hw,
                               float weight, const float* gscale, float* dx, int accumulate, void* stream) {
  if (!x || !y || !pstats || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 1) return AST_E_SHAPE;
  const int64_t chunks = std::min<int64_t>((hw + 4 * kThreads - 1) / (4 * kThreads), 4096);
  const int64_t py = std::max<int64_t>(1, std::min<int64_t>(planes, 65535));
  hipLaunchKernelGGL(mvn_huber_bwd_kernel, dim3((unsigned)chunks, (unsigned)py), dim3(kThreads), 0, (hipStream_t)stream,
                     x, y, pstats, (int64_t)hw, (int64_t)planes, (float)((double)weight / ((double)planes * hw)), gscale,
                     dx, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_mvn_backward_f32(const float* x, const float* g, float* dx, long long planes, long long hw, float eps,
                         void* stream) {
  if (!x || !g || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 1 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL(mvn_backward_kernel, dim3((unsigned)planes), dim3(kThreads), 0, (hipStream_t)stream, x, g, dx,
                     (int64_t)hw, eps);
  return (int)hipGetLastError();
}

int ast_channel_stats_backward_f32(const float* x, const float* mean, const float* std, const float* dmean,
                                   const float* dstd, float* dx, long long planes, long long hw, int unbiased,
                                   int accumulate, void* stream) {
  if (!x || !mean || !std || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(stats_backward_kernel, dim3(grid_for(planes * hw)), dim3(kThreads), 0, (hipStream_t)stream, x,
                     mean, std, dmean, dstd, dx, (int64_t)hw, (int64_t)planes * hw, unbiased ? 1 : 0,
                     accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_huber_f32(const float* x, const float* y, long long n, float weight, const float* gscale, float* loss,
                  float* dx, int accumulate, void* stream) {
  if (!x || !y) return AST_E_NULLPTR;
  if (n <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(huber_kernel, dim3(loss_grid(n)), dim3(kThreads), 0, (hipStream_t)stream, x, y, (int64_t)n,
                     (float)(1.0 / (double)n), weight, gscale, loss, dx, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_style_moments_f32(const float* x, const float* y, long long planes, long long hw, float weight,
                          const float* gscale, float* stats, float* loss, float* row_a, float* row_b, void* stream) {
  if (!x || !y || !stats) return AST_E_NULLPTR;
  if ((row_a == nullptr) != (row_b == nullptr)) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(style_stats_kernel, dim3((unsigned)planes), dim3(kThreads), 0, s, x, y, (int64_t)hw, stats);
  hipLaunchKernelGGL(style_moment_loss_kernel, dim3(grid_for(planes)), dim3(kThreads), 0, s, stats, (int64_t)planes,
                     (int64_t)hw, weight, gscale, loss, row_a, row_b);
  return (int)hipGetLastError();
}

int ast_gram_huber_f32(const float* gx, const float* gy, long long n, float weight, const float* gscale, float* loss,
                       float* dgram, void* stream) {
  if (!gx || !gy) return AST_E_NULLPTR;
  if (n <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(gram_huber_kernel, dim3(loss_grid(n)), dim3(kThreads), 0, (hipStream_t)stream, gx, gy,
                     (int64_t)n, weight, gscale, loss, dgram);
  return (int)hipGetLastError();
}

int ast_tv_loss_f32(const float* x, long long planes, int h, int w, float weight, const float* gscale, float* loss,
                    float* dx, int accumulate, void* stream) {
  if (!x) return AST_E_NULLPTR;
  if (planes <= 0 || h <= 0 || w <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(tv_kernel, dim3(loss_grid(planes * h * w, 1024)), dim3(kThreads), 0, (hipStream_t)stream, x,
                     (int64_t)planes, h, w, weight, gscale, loss, dx, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

}  // extern "C"
