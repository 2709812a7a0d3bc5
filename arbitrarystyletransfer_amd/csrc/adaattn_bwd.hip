// AdaAttN backward (models.py:81-115) for gfx950: the elementwise / row-reduction stages between
// the batched MFMA GEMMs (ast_mbt_gemm_f32) that the autograd Function in functional.py chains.
//
// Forward (per image, C channels, N content pixels, M style pixels; IN = InstanceNorm2d):
//   Q = Wq IN(c), K = Wk IN(s), V = Wv s,  P = softmax_rows(Q^T K)            [N][M]
//   O = P [V; V^2]^T = [mean | ex2]                                           [N][2C]
//   out = sqrt(relu(ex2 - mean^2)) * IN(c) + mean                              [C][N]
// Backward, given G = dL/dout:
//   dvar = (ex2 - mean^2 > 0) ? G IN(c) / (2 std) : 0       (torch: relu' = 0 at 0, sqrt' never hit)
//   dO = [G - 2 mean dvar | dvar],  D[n] = sum_j dO[n][j] O[n][j]  (= rowsum(P * dP), flash trick)
//   dP = dO [V; V^2],  dS = P * (dP - D),  d[V; V^2] = dO^T P -> dV = dVV[:C] + 2 V * dVV[C:]
//   dQ = K dS^T, dK = Q dS, dWq = sum dQ IN(c)^T, dWk = sum dK IN(s)^T, dWv = sum dV s^T
//   d IN(c) = Wq^T dQ + G std, d IN(s) = Wk^T dK, ds += Wv^T dV; IN backward (biased var + eps).
// All fp32 (the reference trains in fp32).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace {

constexpr int kT = 256;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// one workgroup per row: x = softmax(x) (nn.Softmax(dim=-1): exp(x - max) / sum)
__global__ __launch_bounds__(kT) void softmax_rows_kernel(float* __restrict__ s, int cols) {
  __shared__ float red[kT / 64];
  float* row = s + (int64_t)blockIdx.x * cols;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float m = -INFINITY;
  for (int i = tid; i < cols; i += kT) m = fmaxf(m, row[i]);
  m = wave_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int i = tid; i < cols; i += kT) {
    const float e = expf(row[i] - m);
    row[i] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[w] = sum;
  __syncthreads();
  const float inv = 1.f / ((red[0] + red[1]) + (red[2] + red[3]));
  for (int i = tid; i < cols; i += kT) row[i] *= inv;
}

// per (image, content pixel n): dO[n][0:C] = G - 2 mean dvar, dO[n][C:2C] = dvar, D[n]; optional
// std[c][n] (for d IN(c) = ... + G std)
__global__ __launch_bounds__(kT) void dstats_kernel(const float* __restrict__ o2, const float* __restrict__ g,
                                                    const float* __restrict__ chat, float* __restrict__ do2,
                                                    float* __restrict__ drow, float* __restrict__ stdo, int C,
                                                    int N, int64_t total) {
  // one wave per pixel n, lanes over channels
  const int lane = threadIdx.x & 63;
  const int64_t pix = (int64_t)blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  if (pix >= total) return;  // a ragged last workgroup (wave-uniform)
  const int64_t b = pix / N, n = pix % N;
  const float* o = o2 + pix * 2 * C;
  float* d = do2 + pix * 2 * C;
  const float* gb = g + b * C * N + n;
  const float* cb = chat + b * C * N + n;
  float acc = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float mean = o[c], ex2 = o[C + c];
    const float var = ex2 - mean * mean;
    const float sd = var > 0.f ? sqrtf(var) : 0.f;
    const float gg = gb[(int64_t)c * N];
    const float dvar = var > 0.f ? gg * cb[(int64_t)c * N] / (2.f * sd) : 0.f;
    const float dm = gg - 2.f * mean * dvar;
    d[c] = dm;
    d[C + c] = dvar;
    acc += dm * mean + dvar * ex2;
    if (stdo) stdo[b * C * N + (int64_t)c * N + n] = sd;
  }
  acc = wave_sum(acc);
  if (lane == 0) drow[pix] = acc;
}

// dS = P * (dP - D[row]), in place in dp
__global__ void softmax_bwd_kernel(const float* __restrict__ p, float* __restrict__ dp, const float* __restrict__ drow,
                                   int64_t total, int cols) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    dp[i] = p[i] * (dp[i] - drow[i / cols]);
}

// vv[b][C + c][m] = vv[b][c][m]^2
__global__ void square_half_kernel(float* __restrict__ vv, int64_t cm, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / cm, r = i % cm;
    const float v = vv[b * 2 * cm + r];
    vv[b * 2 * cm + cm + r] = v * v;
  }
}

// dv[b][c][m] = dvv[b][c][m] + 2 v[b][c][m] dvv[b][C + c][m]   (v = vv[:, :C])
__global__ void dv_kernel(const float* __restrict__ dvv, const float* __restrict__ vv, float* __restrict__ dv,
                          int64_t cm, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / cm, r = i % cm;
    dv[i] = dvv[b * 2 * cm + r] + 2.f * vv[b * 2 * cm + r] * dvv[b * 2 * cm + cm + r];
  }
}

// InstanceNorm2d backward (biased variance, eps; no affine), one workgroup per plane:
// dx = (dxh - mean(dxh) - xh * mean(dxh * xh)) / std,  xh = (x - mu) / std, std = sqrt(var + eps)
__global__ __launch_bounds__(kT) void in_backward_kernel(const float* __restrict__ x, const float* __restrict__ mu,
                                                         const float* __restrict__ sd, const float* __restrict__ dxh,
                                                         float* __restrict__ dx, int64_t hw, int accumulate) {
  __shared__ float red[2][kT / 64];
  const int64_t p = blockIdx.x;
  const float* xp = x + p * hw;
  const float* gp = dxh + p * hw;
  float* op = dx + p * hw;
  const float m = mu[p], s = sd[p], inv = 1.f / s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float s1 = 0.f, s2 = 0.f;
  for (int64_t i = tid; i < hw; i += kT) {
    const float g = gp[i], xh = (xp[i] - m) * inv;
    s1 += g;
    s2 += g * xh;
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  const float a = ((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) / (float)hw;
  const float bq = ((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])) / (float)hw;
  for (int64_t i = tid; i < hw; i += kT) {
    const float xh = (xp[i] - m) * inv;
    const float v = (gp[i] - a - xh * bq) * inv;
    op[i] = accumulate ? op[i] + v : v;
  }
}

// dst[i] += a[i] * b[i]
__global__ void fma_inplace_kernel(float* __restrict__ dst, const float* __restrict__ a, const float* __restrict__ b,
                                   int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = fmaf(a[i], b[i], dst[i]);
}

int grid1(int64_t n) { return (int)(n < 1 ? 1 : (n + kT - 1) / kT < 8192 ? (n + kT - 1) / kT : 8192); }

}  // namespace

extern "C" {

int ast_softmax_rows_f32(float* s, long long rows, int cols, void* stream) {
  if (!s) return AST_E_NULLPTR;
  if (rows <= 0 || cols <= 0 || rows > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(kT), 0, (hipStream_t)stream, s, cols);
  return (int)hipGetLastError();
}

int ast_adaattn_dstats_f32(const float* o2, const float* g, const float* chat, float* do2, float* drow, float* std_out,
                           int n, int c, int npix, void* stream) {
  if (!o2 || !g || !chat || !do2 || !drow) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || npix <= 0) return AST_E_SHAPE;
  const int64_t pix = (int64_t)n * npix;
  const int64_t blocks = (pix + kT / 64 - 1) / (kT / 64);
  if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL(dstats_kernel, dim3((unsigned)blocks), dim3(kT), 0, (hipStream_t)stream, o2, g, chat, do2, drow,
                     std_out, c, npix, pix);
  return (int)hipGetLastError();
}

int ast_softmax_backward_f32(const float* p, float* dp, const float* drow, long long rows, int cols, void* stream) {
  if (!p || !dp || !drow) return AST_E_NULLPTR;
  if (rows <= 0 || cols <= 0) return AST_E_SHAPE;
  const int64_t total = (int64_t)rows * cols;
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3(grid1(total)), dim3(kT), 0, (hipStream_t)stream, p, dp, drow, total,
                     cols);
  return (int)hipGetLastError();
}

int ast_adaattn_square_f32(float* vv, int n, long long cm, void* stream) {
  if (!vv) return AST_E_NULLPTR;
  if (n <= 0 || cm <= 0) return AST_E_SHAPE;
  const int64_t total = (int64_t)n * cm;
  hipLaunchKernelGGL(square_half_kernel, dim3(grid1(total)), dim3(kT), 0, (hipStream_t)stream, vv, (int64_t)cm, total);
  return (int)hipGetLastError();
}

int ast_adaattn_dv_f32(const float* dvv, const float* vv, float* dv, int n, long long cm, void* stream) {
  if (!dvv || !vv || !dv) return AST_E_NULLPTR;
  if (n <= 0 || cm <= 0) return AST_E_SHAPE;
  const int64_t total = (int64_t)n * cm;
  hipLaunchKernelGGL(dv_kernel, dim3(grid1(total)), dim3(kT), 0, (hipStream_t)stream, dvv, vv, dv, (int64_t)cm, total);
  return (int)hipGetLastError();
}

int ast_instance_norm_backward_f32(const float* x, const float* mean, const float* std, const float* dxh, float* dx,
                                   long long planes, long long hw, int accumulate, void* stream) {
  if (!x || !mean || !std || !dxh || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL(in_backward_kernel, dim3((unsigned)planes), dim3(kT), 0, (hipStream_t)stream, x, mean, std, dxh,
                     dx, (int64_t)hw, accumulate);
  return (int)hipGetLastError();
}

int ast_fma_inplace_f32(float* dst, const float* a, const float* b, long long n, void* stream) {
  if (!dst || !a || !b) return AST_E_NULLPTR;
  if (n <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(fma_inplace_kernel, dim3(grid1(n)), dim3(kT), 0, (hipStream_t)stream, dst, a, b, (int64_t)n);
  return (int)hipGetLastError();
}

}  // extern "C"
