// MobileNet-variant training kernels (SURVEY §8f "next" #4: AutoEncoder training,
// train_autoencoder.py:88-148) for gfx950, fp32. Unlike the inference kernels (mobilenet.hip: BN
// folded, blocks fused), training needs every intermediate of DepthWiseConv.forward
// (mobilenetv2.py:153-165) and BatchNorm with batch statistics, so the blocks run as a chain of
// composable kernels, each with its backward:
//   gemm_kernel         strided-batched C (+)= A.B on MFMA-fp32 (1x1 convs: forward, input grad,
//                       weight grad with the pixel/batch reduction split across workgroups)
//   dw_fwd / dw_dgrad / dw_wgrad   depthwise kxk, stride 1|2, reflect padding
//   bn_stats / bn_apply / bn_bwd_reduce / bn_bwd_apply   BatchNorm2d in training mode
//   hardswish fwd/bwd, add, nearest upsample x2 fwd/bwd, plane means (SE pool)
//   se_fc_fwd / se_fc_bwd  the SE MLP (Linear-ReLU-Linear-Hardtanh) per image in one workgroup
// Numerics follow torch's CPU kernels' formulas (fp32), not their summation order.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kT = 256;

inline unsigned grid_for(int64_t n, int64_t cap = 1 << 20) {
  int64_t b = (n + kT - 1) / kT;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kT / 64; ++i) t += sh[i];
  return t;
}

// ------------------------------------------------------------------------------------------------
// GEMM: C[b][m][n] (+)= sum_k A[b][m][k] * B[b][k][n], general strides. 64x64 tile per workgroup,
// 4 waves x 32x32 (v_mfma_f32_32x32x2_f32), K in chunks of 16 through LDS. grid.z = batch *
// ksplit; with atomic != 0 partial sums are atomically added (C zeroed by the caller).
// ------------------------------------------------------------------------------------------------
struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  int64_t sAb, sAm, sAk, sBb, sBk, sBn, sCb, sCm, sCn;
  int M, N, K, batch, ksplit, kchunk, accumulate, atomic;
};

constexpr int GT = 64, GK = 16, GP = GT + 4;

__global__ __launch_bounds__(kT) void gemm_kernel(GemmArgs a) {
  __shared__ float As[GK * GP];  // [k][m]
  __shared__ float Bs[GK * GP];  // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  const int b = blockIdx.z / a.ksplit, ks = blockIdx.z % a.ksplit;
  const int kbeg = ks * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const float* A = a.A + b * a.sAb;
  const float* B = a.B + b * a.sBb;
  // staging maps: the contiguous dimension runs along consecutive threads
  const bool a_kfast = a.sAk == 1, b_nfast = a.sBn == 1;
  f32x16 acc = (f32x16){0.f};
  for (int k0 = kbeg; k0 < kend; k0 += GK) {
#pragma unroll
    for (int i = 0; i < GK * GT / kT; ++i) {
      const int e = tid + i * kT;
      const int kk = a_kfast ? (e % GK) : (e / GT), mm = a_kfast ? (e / GK) : (e % GT);
      const int gk = k0 + kk, gm = m0 + mm;
      As[kk * GP + mm] = (gk < kend && gm < a.M) ? A[gm * a.sAm + (int64_t)gk * a.sAk] : 0.f;
      const int kb = b_nfast ? (e / GT) : (e % GK), nb = b_nfast ? (e % GT) : (e / GK);
      const int gkb = k0 + kb, gn = n0 + nb;
      Bs[kb * GP + nb] = (gkb < kend && gn < a.N) ? B[(int64_t)gkb * a.sBk + gn * a.sBn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kp = 0; kp < GK / 2; ++kp)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[(2 * kp + h) * GP + wm * 32 + r], Bs[(2 * kp + h) * GP + wn * 32 + r],
                                                 acc, 0, 0, 0);
    __syncthreads();
  }
  float* C = a.C + b * a.sCb;
  const int n = n0 + wn * 32 + r;
  if (n >= a.N) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (m < a.M) {
      float* c = C + m * a.sCm + n * a.sCn;
      if (a.atomic) atomicAdd(c, acc[i]);
      else *c = a.accumulate ? *c + acc[i] : acc[i];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// depthwise kxk conv with reflect padding p = (k-1)/2 (torch padding_mode="reflect"), stride s
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int refl(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

__global__ void dw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int64_t nc,
                              int c, int h, int wd, int ho, int wo, int k, int s) {
  const int p = (k - 1) / 2;
  const int64_t tot = nc * ho * wo;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < tot; e += (int64_t)gridDim.x * kT) {
    const int ox = (int)(e % wo);
    const int64_t t = e / wo;
    const int oy = (int)(t % ho);
    const int64_t pl = t / ho;
    const int ch = (int)(pl % c);
    const float* xp = x + pl * h * wd;
    const float* wc = w + (int64_t)ch * k * k;
    float acc = 0.f;
    for (int ky = 0; ky < k; ++ky) {
      const int iy = refl(oy * s - p + ky, h);
      for (int kx = 0; kx < k; ++kx) acc = fmaf(wc[ky * k + kx], xp[(int64_t)iy * wd + refl(ox * s - p + kx, wd)], acc);
    }
    y[e] = acc;
  }
}

// dx (zeroed by the caller) += scatter of g * w through the reflect map
__global__ void dw_dgrad_kernel(const float* __restrict__ g, const float* __restrict__ w, float* __restrict__ dx,
                                int64_t nc, int c, int h, int wd, int ho, int wo, int k, int s) {
  const int p = (k - 1) / 2;
  const int64_t tot = nc * ho * wo;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < tot; e += (int64_t)gridDim.x * kT) {
    const int ox = (int)(e % wo);
    const int64_t t = e / wo;
    const int oy = (int)(t % ho);
    const int64_t pl = t / ho;
    const int ch = (int)(pl % c);
    const float gv = g[e];
    float* dp = dx + pl * h * wd;
    const float* wc = w + (int64_t)ch * k * k;
    for (int ky = 0; ky < k; ++ky) {
      const int iy = refl(oy * s - p + ky, h);
      for (int kx = 0; kx < k; ++kx) atomicAdd(dp + (int64_t)iy * wd + refl(ox * s - p + kx, wd), gv * wc[ky * k + kx]);
    }
  }
}

// dw[c][tap] += sum over one image's plane (grid = (c, n)); dw zeroed by the caller
__global__ __launch_bounds__(kT) void dw_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                      float* __restrict__ dw, int c, int h, int wd, int ho, int wo,
                                                      int k, int s) {
  __shared__ float sh[kT / 64];
  const int ch = blockIdx.x, n = blockIdx.y, p = (k - 1) / 2;
  const int64_t pl = (int64_t)n * c + ch;
  const float* xp = x + pl * h * wd;
  const float* gp = g + pl * ho * wo;
  float acc[25];
#pragma unroll
  for (int t = 0; t < 25; ++t) acc[t] = 0.f;
  for (int64_t e = threadIdx.x; e < (int64_t)ho * wo; e += kT) {
    const int ox = (int)(e % wo), oy = (int)(e / wo);
    const float gv = gp[e];
#pragma unroll
    for (int ky = 0; ky < 5; ++ky) {
      if (ky >= k) break;
      const int iy = refl(oy * s - p + ky, h);
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        if (kx >= k) break;
        acc[ky * 5 + kx] = fmaf(gv, xp[(int64_t)iy * wd + refl(ox * s - p + kx, wd)], acc[ky * 5 + kx]);
      }
    }
  }
  for (int ky = 0; ky < k; ++ky)
    for (int kx = 0; kx < k; ++kx) {
      const float t = block_sum(acc[ky * 5 + kx], sh);
      if (threadIdx.x == 0) atomicAdd(dw + (int64_t)ch * k * k + ky * k + kx, t);
    }
}

// ------------------------------------------------------------------------------------------------
// BatchNorm2d, training mode: batch mean and biased variance over (N, H, W) per channel,
// y = (x - mean) * invstd * gamma + beta, invstd = 1/sqrt(var + eps); running statistics with
// momentum and the unbiased variance (torch's batch_norm update).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kT) void bn_stats_kernel(const float* __restrict__ x, int n, int c, int64_t hw, float eps,
                                                      float momentum, float* __restrict__ mean,
                                                      float* __restrict__ invstd, float* __restrict__ run_mean,
                                                      float* __restrict__ run_var) {
  __shared__ float sh[kT / 64];
  const int ch = blockIdx.x;
  const int64_t m = (int64_t)n * hw;
  float s = 0.f;
  for (int b = 0; b < n; ++b) {
    const float* xp = x + ((int64_t)b * c + ch) * hw;
    for (int64_t i = threadIdx.x; i < hw; i += kT) s += xp[i];
  }
  const float mu = block_sum(s, sh) / (float)m;
  float q = 0.f;
  for (int b = 0; b < n; ++b) {
    const float* xp = x + ((int64_t)b * c + ch) * hw;
    for (int64_t i = threadIdx.x; i < hw; i += kT) {
      const float d = xp[i] - mu;
      q = fmaf(d, d, q);
    }
  }
  const float ss = block_sum(q, sh);
  if (threadIdx.x == 0) {
    const float var = ss / (float)m;
    mean[ch] = mu;
    invstd[ch] = 1.0f / sqrtf(var + eps);
    if (run_mean) {
      run_mean[ch] = (1.f - momentum) * run_mean[ch] + momentum * mu;
      run_var[ch] = (1.f - momentum) * run_var[ch] + momentum * (m > 1 ? ss / (float)(m - 1) : var);
    }
  }
}

__global__ void bn_apply_kernel(const float* __restrict__ x, int c, int64_t hw, int64_t total, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, float* __restrict__ y) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const int ch = (int)((e / hw) % c);
    y[e] = (x[e] - mean[ch]) * invstd[ch] * (gamma ? gamma[ch] : 1.f) + (beta ? beta[ch] : 0.f);
  }
}

// per channel: sum(dy) -> dbeta, sum(dy * xhat) -> dgamma
__global__ __launch_bounds__(kT) void bn_bwd_reduce_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                           int n, int c, int64_t hw, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd, float* __restrict__ sdy,
                                                           float* __restrict__ sdyx) {
  __shared__ float sh[kT / 64];
  const int ch = blockIdx.x;
  const float mu = mean[ch], is = invstd[ch];
  float a = 0.f, b2 = 0.f;
  for (int b = 0; b < n; ++b) {
    const int64_t o = ((int64_t)b * c + ch) * hw;
    for (int64_t i = threadIdx.x; i < hw; i += kT) {
      const float g = dy[o + i];
      a += g;
      b2 = fmaf(g, (x[o + i] - mu) * is, b2);
    }
  }
  const float A = block_sum(a, sh);
  const float Bv = block_sum(b2, sh);
  if (threadIdx.x == 0) {
    sdy[ch] = A;
    sdyx[ch] = Bv;
  }
}

__global__ void bn_bwd_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy, int c, int64_t hw,
                                    int64_t total, int64_t m, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                                    const float* __restrict__ sdy, const float* __restrict__ sdyx,
                                    float* __restrict__ dx) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const int ch = (int)((e / hw) % c);
    const float is = invstd[ch], xh = (x[e] - mean[ch]) * is;
    const float gm = gamma ? gamma[ch] : 1.f;
    dx[e] = gm * is * (dy[e] - sdy[ch] / (float)m - xh * sdyx[ch] / (float)m);
  }
}

// ------------------------------------------------------------------------------------------------
// elementwise
// ------------------------------------------------------------------------------------------------
__global__ void hswish_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const float v = x[e];
    y[e] = v * fminf(fmaxf(v + 3.f, 0.f), 6.f) / 6.f;
  }
}

// torch hardswish_backward: x < -3: 0; x <= 3: g * (x / 3 + 0.5); else g
__global__ void hswish_bwd_kernel(const float* __restrict__ x, const float* __restrict__ g, float* __restrict__ dx,
                                  int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) {
    const float v = x[e];
    dx[e] = v < -3.f ? 0.f : (v <= 3.f ? g[e] * (v / 3.f + 0.5f) : g[e]);
  }
}

__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ y, int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < n; e += (int64_t)gridDim.x * kT) y[e] = a[e] + b[e];
}

__global__ void up2_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t planes, int h, int w) {
  const int64_t tot = planes * 4 * h * w;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < tot; e += (int64_t)gridDim.x * kT) {
    const int ox = (int)(e % (2 * w));
    const int64_t t = e / (2 * w);
    const int oy = (int)(t % (2 * h));
    const int64_t pl = t / (2 * h);
    y[e] = x[(pl * h + (oy >> 1)) * w + (ox >> 1)];
  }
}

__global__ void up2_bwd_kernel(const float* __restrict__ g, float* __restrict__ dx, int64_t planes, int h, int w) {
  const int64_t tot = planes * h * w;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < tot; e += (int64_t)gridDim.x * kT) {
    const int x = (int)(e % w);
    const int64_t t = e / w;
    const int y = (int)(t % h);
    const int64_t pl = t / h;
    const float* gp = g + (pl * 2 * h + 2 * y) * 2 * w + 2 * x;
    dx[e] = (gp[0] + gp[1]) + (gp[2 * w] + gp[2 * w + 1]);
  }
}

// per-plane mean (SE AdaptiveAvgPool2d(1)) or, with y, per-plane sum(x * y) (the gate gradient)
__global__ __launch_bounds__(kT) void plane_dot_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       int64_t hw, float scale, float* __restrict__ out) {
  __shared__ float sh[kT / 64];
  const int64_t p = blockIdx.x;
  const float* xp = x + p * hw;
  const float* yp = y ? y + p * hw : nullptr;
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < hw; i += kT) s += yp ? xp[i] * yp[i] : xp[i];
  const float t = block_sum(s, sh);
  if (threadIdx.x == 0) out[p] = t * scale;
}

// y = x * gate[plane] (+ gadd[plane] when given: the SE input gradient dy*g + dpool/hw)
__global__ void plane_scale_kernel(const float* __restrict__ x, const float* __restrict__ gate,
                                   const float* __restrict__ gadd, int64_t hw, int64_t total, float* __restrict__ y) {
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const int64_t p = e / hw;
    y[e] = x[e] * gate[p] + (gadd ? gadd[p] : 0.f);
  }
}

// SE MLP per image (one workgroup): hid = relu(W1 pool + b1); z = W2 hid + b2; gate = clamp(z, 0, 1)
__global__ __launch_bounds__(kT) void se_fc_fwd_kernel(const float* __restrict__ pool, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, int c, int red,
                                                       float* __restrict__ hid, float* __restrict__ z,
                                                       float* __restrict__ gate) {
  extern __shared__ float hs[];
  const int n = blockIdx.x;
  const float* pv = pool + (int64_t)n * c;
  for (int j = threadIdx.x; j < red; j += kT) {
    float a = b1[j];
    for (int i = 0; i < c; ++i) a = fmaf(w1[(int64_t)j * c + i], pv[i], a);
    a = a > 0.f ? a : 0.f;
    hs[j] = a;
    hid[(int64_t)n * red + j] = a;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < c; i += kT) {
    float a = b2[i];
    for (int j = 0; j < red; ++j) a = fmaf(w2[(int64_t)i * red + j], hs[j], a);
    z[(int64_t)n * c + i] = a;
    gate[(int64_t)n * c + i] = fminf(fmaxf(a, 0.f), 1.f);
  }
}

// SE MLP backward per image: dz = dgate * (0 < z < 1); dW2, db2, dh = W2^T dz * (hid > 0), dW1, db1,
// dpool = W1^T dh (scaled by 1/hw for the broadcast back onto the plane). Parameter gradients are
// accumulated with atomics (zeroed by the caller).
__global__ __launch_bounds__(kT) void se_fc_bwd_kernel(const float* __restrict__ dgate, const float* __restrict__ z,
                                                       const float* __restrict__ hid, const float* __restrict__ pool,
                                                       const float* __restrict__ w1, const float* __restrict__ w2,
                                                       int c, int red, float inv_hw, float* __restrict__ dw1,
                                                       float* __restrict__ db1, float* __restrict__ dw2,
                                                       float* __restrict__ db2, float* __restrict__ dpool) {
  extern __shared__ float sm[];
  float* dz = sm;        // [c]
  float* dh = sm + c;    // [red]
  const int n = blockIdx.x;
  for (int i = threadIdx.x; i < c; i += kT) {
    const float zv = z[(int64_t)n * c + i];
    const float d = (zv > 0.f && zv < 1.f) ? dgate[(int64_t)n * c + i] : 0.f;
    dz[i] = d;
    atomicAdd(db2 + i, d);
  }
  __syncthreads();
  const float* hv = hid + (int64_t)n * red;
  for (int e = threadIdx.x; e < c * red; e += kT) {
    const int i = e / red, j = e % red;
    atomicAdd(dw2 + e, dz[i] * hv[j]);
  }
  for (int j = threadIdx.x; j < red; j += kT) {
    float a = 0.f;
    for (int i = 0; i < c; ++i) a = fmaf(w2[(int64_t)i * red + j], dz[i], a);
    a = hv[j] > 0.f ? a : 0.f;
    dh[j] = a;
    atomicAdd(db1 + j, a);
  }
  __syncthreads();
  const float* pv = pool + (int64_t)n * c;
  for (int e = threadIdx.x; e < red * c; e += kT) {
    const int j = e / c, i = e % c;
    atomicAdd(dw1 + e, dh[j] * pv[i]);
  }
  for (int i = threadIdx.x; i < c; i += kT) {
    float a = 0.f;
    for (int j = 0; j < red; ++j) a = fmaf(w1[(int64_t)j * c + i], dh[j], a);
    dpool[(int64_t)n * c + i] = a * inv_hw;
  }
}

}  // namespace

extern "C" {

int ast_mbt_gemm_f32(const float* A, const float* B, float* C, int M, int N, int K, int batch, long long sAb,
                     long long sAm, long long sAk, long long sBb, long long sBk, long long sBn, long long sCb,
                     long long sCm, long long sCn, int ksplit, int accumulate, int atomic, void* stream) {
  if (!A || !B || !C) return AST_E_NULLPTR;
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || ksplit <= 0) return AST_E_SHAPE;
  if (((int64_t)M + GT - 1) / GT > 65535 || (int64_t)batch * ksplit > 65535) return AST_E_SHAPE;
  if (ksplit > 1 || (sCb == 0 && batch > 1)) atomic = 1;  // partial sums meet in C
  GemmArgs a{A, B, C, sAb, sAm, sAk, sBb, sBk, sBn, sCb, sCm, sCn, M, N, K, batch, ksplit, 0, accumulate, atomic};
  a.kchunk = ((K + ksplit - 1) / ksplit + GK - 1) / GK * GK;
  const dim3 grid((unsigned)((N + GT - 1) / GT), (unsigned)((M + GT - 1) / GT), (unsigned)(batch * ksplit));
  hipLaunchKernelGGL(gemm_kernel, grid, dim3(kT), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int ast_mbt_dw_f32(int mode, const float* x, const float* w, const float* g, float* out, int n, int c, int h, int wd,
                   int k, int s, void* stream) {
  if (!w || !out || (mode != 1 && !x) || (mode != 0 && !g)) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || h <= 0 || wd <= 0 || (k != 3 && k != 5) || (s != 1 && s != 2)) return AST_E_SHAPE;
  const int p = (k - 1) / 2;
  if (p >= h || p >= wd) return AST_E_SHAPE;  // reflect padding needs pad < size
  const int ho = (h + 2 * p - k) / s + 1, wo = (wd + 2 * p - k) / s + 1;
  hipStream_t st = (hipStream_t)stream;
  const int64_t nc = (int64_t)n * c;
  if (mode == 0) {
    hipLaunchKernelGGL(dw_fwd_kernel, dim3(grid_for(nc * ho * wo)), dim3(kT), 0, st, x, w, out, nc, c, h, wd, ho, wo, k, s);
  } else if (mode == 1) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * (size_t)(nc * h * wd), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(dw_dgrad_kernel, dim3(grid_for(nc * ho * wo)), dim3(kT), 0, st, g, w, out, nc, c, h, wd, ho, wo,
                       k, s);
  } else {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * (size_t)c * k * k, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(dw_wgrad_kernel, dim3(c, n), dim3(kT), 0, st, x, g, out, c, h, wd, ho, wo, k, s);
  }
  return (int)hipGetLastError();
}

int ast_mbt_bn_fwd_f32(const float* x, int n, int c, long long hw, const float* gamma, const float* beta, float eps,
                       float momentum, float* mean, float* invstd, float* run_mean, float* run_var, float* y,
                       void* stream) {
  if (!x || !mean || !invstd || !y) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(c), dim3(kT), 0, st, x, n, c, (int64_t)hw, eps, momentum, mean, invstd,
                     run_mean, run_var);
  const int64_t total = (int64_t)n * c * hw;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(total)), dim3(kT), 0, st, x, c, (int64_t)hw, total, mean, invstd,
                     gamma, beta, y);
  return (int)hipGetLastError();
}

int ast_mbt_bn_bwd_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                       const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dx, void* stream) {
  if (!x || !dy || !mean || !invstd || !dgamma || !dbeta || !dx) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(c), dim3(kT), 0, st, x, dy, n, c, (int64_t)hw, mean, invstd, dbeta,
                     dgamma);
  const int64_t total = (int64_t)n * c * hw;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(total)), dim3(kT), 0, st, x, dy, c, (int64_t)hw, total,
                     (int64_t)n * hw, mean, invstd, gamma, dbeta, dgamma, dx);
  return (int)hipGetLastError();
}

int ast_mbt_eltwise_f32(int op, const float* a, const float* b, float* y, long long n, int h, int w, void* stream) {
  // op 0: hardswish(a); 1: hardswish backward (x = a, g = b); 2: a + b;
  //    3: nearest upsample x2 of a [n planes][h][w]; 4: its backward (a = grad [n][2h][2w])
  if (!a || !y || ((op == 1 || op == 2) && !b)) return AST_E_NULLPTR;
  if (n <= 0) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  switch (op) {
    case 0: hipLaunchKernelGGL(hswish_kernel, dim3(grid_for(n)), dim3(kT), 0, st, a, y, (int64_t)n); break;
    case 1: hipLaunchKernelGGL(hswish_bwd_kernel, dim3(grid_for(n)), dim3(kT), 0, st, a, b, y, (int64_t)n); break;
    case 2: hipLaunchKernelGGL(add_kernel, dim3(grid_for(n)), dim3(kT), 0, st, a, b, y, (int64_t)n); break;
    case 3:
      if (h <= 0 || w <= 0) return AST_E_SHAPE;
      hipLaunchKernelGGL(up2_kernel, dim3(grid_for(n * 4 * h * w)), dim3(kT), 0, st, a, y, (int64_t)n, h, w);
      break;
    case 4:
      if (h <= 0 || w <= 0) return AST_E_SHAPE;
      hipLaunchKernelGGL(up2_bwd_kernel, dim3(grid_for(n * h * w)), dim3(kT), 0, st, a, y, (int64_t)n, h, w);
      break;
    default: return AST_E_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int ast_mbt_plane_f32(int op, const float* x, const float* y, const float* gate, const float* gadd, float* out,
                      long long planes, long long hw, void* stream) {
  // op 0: out[p] = mean(x[p]); 1: out[p] = sum(x[p] * y[p]); 2: out = x * gate[p] (+ gadd[p])
  if (!x || !out || (op == 1 && !y) || (op == 2 && !gate)) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (op == 0 || op == 1)
    hipLaunchKernelGGL(plane_dot_kernel, dim3((unsigned)planes), dim3(kT), 0, st, x, op == 1 ? y : nullptr,
                       (int64_t)hw, op == 0 ? 1.0f / (float)hw : 1.0f, out);
  else if (op == 2)
    hipLaunchKernelGGL(plane_scale_kernel, dim3(grid_for(planes * hw)), dim3(kT), 0, st, x, gate, gadd, (int64_t)hw,
                       (int64_t)(planes * hw), out);
  else
    return AST_E_UNSUPPORTED;
  return (int)hipGetLastError();
}

int ast_mbt_se_fc_fwd_f32(const float* pool, const float* w1, const float* b1, const float* w2, const float* b2,
                          int n, int c, int red, float* hid, float* z, float* gate, void* stream) {
  if (!pool || !w1 || !b1 || !w2 || !b2 || !hid || !z || !gate) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || red <= 0 || red > 8192) return AST_E_SHAPE;
  hipLaunchKernelGGL(se_fc_fwd_kernel, dim3(n), dim3(kT), sizeof(float) * red, (hipStream_t)stream, pool, w1, b1, w2,
                     b2, c, red, hid, z, gate);
  return (int)hipGetLastError();
}

int ast_mbt_se_fc_bwd_f32(const float* dgate, const float* z, const float* hid, const float* pool, const float* w1,
                          const float* w2, int n, int c, int red, long long hw, float* dw1, float* db1, float* dw2,
                          float* db2, float* dpool, void* stream) {
  if (!dgate || !z || !hid || !pool || !w1 || !w2 || !dw1 || !db1 || !dw2 || !db2 || !dpool) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || red <= 0 || hw <= 0 || c + red > 16384) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  if ((e = hipMemsetAsync(dw1, 0, sizeof(float) * (size_t)red * c, st)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(dw2, 0, sizeof(float) * (size_t)red * c, st)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(db1, 0, sizeof(float) * (size_t)red, st)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(db2, 0, sizeof(float) * (size_t)c, st)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(se_fc_bwd_kernel, dim3(n), dim3(kT), sizeof(float) * (c + red), st, dgate, z, hid, pool, w1, w2, c,
                     red, 1.0f / (float)hw, dw1, db1, dw2, db2, dpool);
  return (int)hipGetLastError();
}

}  // extern "C"
