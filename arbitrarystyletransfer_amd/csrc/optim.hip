// Optimizer step of the training loop (train.py:287-300) for gfx950:
// clip_grad_norm_(params, max_norm, error_if_nonfinite) + torch.optim.Adam, as two multi-tensor
// launches over a device table of (param, grad, exp_avg, exp_avg_sq, numel) entries.
//  1. sq_norm: every workgroup reduces a slice of one tensor; partial sums of squares go to a
//     per-workgroup slot, then the last kernel folds them (deterministic order, no atomics).
//  2. adam: clip coefficient = min(1, max_norm / (sqrt(total) + 1e-6)) read from device memory,
//     then torch's Adam update (non-amsgrad, no weight decay) on each element.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 65536;  // elements per workgroup

struct TensorEntry {
  float* p;
  float* g;
  float* m;
  float* v;
  long long n;
  long long chunk0;  // first global chunk index of this tensor
};

__device__ __forceinline__ float block_sum(float v, float* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__device__ __forceinline__ int find_entry(const TensorEntry* t, int nt, long long chunk) {
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].chunk0 <= chunk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ void sq_norm_kernel(const TensorEntry* __restrict__ t, int nt, float* __restrict__ partial) {
  __shared__ float sh[4];
  const long long chunk = blockIdx.x;
  const TensorEntry e = t[find_entry(t, nt, chunk)];
  const long long b = (chunk - e.chunk0) * kChunk;
  const long long end = b + kChunk < e.n ? b + kChunk : e.n;
  float s = 0.f;
  for (long long i = b + threadIdx.x; i < end; i += kThreads) {
    const float g = e.g[i];
    s += g * g;
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[chunk] = s;
}

// state[0] = total norm, state[1] = clip coefficient
__global__ void norm_finish_kernel(const float* __restrict__ partial, long long nchunks, float max_norm,
                                   float* __restrict__ state) {
  __shared__ float sh[4];
  float s = 0.f;
  for (long long i = threadIdx.x; i < nchunks; i += kThreads) s += partial[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    state[0] = norm;
    // torch: clamp(max_norm / (norm + 1e-6), max=1) -- a NaN norm gives a NaN coefficient
    const float c = max_norm / (norm + 1e-6f);
    state[1] = (c < 1.f || c != c) ? c : 1.f;
  }
}

// torch foreach Adam: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
// denom = sqrt(exp_avg_sq) / sqrt(bc2) + eps; p.addcdiv_(exp_avg, denom, -lr/bc1).
// sched != null (graph-capturable form): the step count and the bias-correction scalars come from
// device memory (sched[1] != 0: skip the step), written by adam_sched_kernel just before.
__global__ void adam_kernel(const TensorEntry* __restrict__ t, int nt, const float* __restrict__ state, float lr,
                            float w1, float beta2, float w2, float eps, float step_size, float bc2_sqrt,
                            const float* __restrict__ sched) {
  if (sched) {
    if (sched[1] != 0.f) return;  // non-finite gradient norm: nothing changes (torch raises first)
    step_size = sched[2];
    bc2_sqrt = sched[3];
  }
  const long long chunk = blockIdx.x;
  const TensorEntry e = t[find_entry(t, nt, chunk)];
  const long long b = (chunk - e.chunk0) * kChunk;
  const long long end = b + kChunk < e.n ? b + kChunk : e.n;
  const float clip = state ? state[1] : 1.f;
  for (long long i = b + threadIdx.x; i < end; i += kThreads) {
    float g = e.g[i];
    if (state) {
      g = g * clip;
      e.g[i] = g;  // clip_grad_norm_ scales the gradients in place
    }
    const float m0 = e.m[i];
    const float m = w1 < 0.5f ? m0 + w1 * (g - m0) : g - (g - m0) * (1.f - w1);  // at::lerp
    const float v = e.v[i] * beta2 + w2 * g * g;
    e.m[i] = m;
    e.v[i] = v;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    e.p[i] = e.p[i] + (-step_size) * (m / denom);
  }
}

// sched = [step, skip, lr / bc1, sqrt(bc2)]: one thread advances the device step count and computes
// the bias corrections in double, as torch's Python scalars (skip, step unchanged, when check_finite
// and the gradient norm state[0] is not finite)
__global__ void adam_sched_kernel(const float* __restrict__ state, double lr, double beta1, double beta2,
                                  int check_finite, float* __restrict__ sched) {
  if (threadIdx.x != 0) return;
  if (check_finite && state) {
    const float nrm = state[0];
    if (!(fabsf(nrm) <= 3.402823466e38f)) {
      sched[1] = 1.f;
      return;
    }
  }
  const float step = sched[0] + 1.f;
  sched[0] = step;
  sched[1] = 0.f;
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  sched[2] = (float)(lr / bc1);
  sched[3] = (float)sqrt(bc2);
}

__global__ void grad_scale_kernel(const TensorEntry* __restrict__ t, int nt, const float* __restrict__ state) {
  const long long chunk = blockIdx.x;
  const TensorEntry e = t[find_entry(t, nt, chunk)];
  const long long b = (chunk - e.chunk0) * kChunk;
  const long long end = b + kChunk < e.n ? b + kChunk : e.n;
  const float c = state[1];
  for (long long i = b + threadIdx.x; i < end; i += kThreads) e.g[i] = e.g[i] * c;
}

}  // namespace

extern "C" {

int ast_grad_scale_f32(const void* dev_table, int ntensors, long long nchunks, const float* state, void* stream) {
  if (!dev_table || !state) return AST_E_NULLPTR;
  if (ntensors <= 0 || nchunks <= 0 || nchunks > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL(grad_scale_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, (hipStream_t)stream,
                     (const TensorEntry*)dev_table, ntensors, state);
  return (int)hipGetLastError();
}

size_t ast_optim_table_bytes(int ntensors) { return (size_t)ntensors * sizeof(TensorEntry); }

long long ast_optim_build_table(void* host_table, int ntensors, float* const* params, float* const* grads,
                                float* const* exp_avg, float* const* exp_avg_sq, const long long* numel) {
  if (!host_table || ntensors <= 0) return AST_E_NULLPTR;
  TensorEntry* t = (TensorEntry*)host_table;
  long long chunks = 0;
  for (int i = 0; i < ntensors; ++i) {
    if (!params[i] || !grads[i] || numel[i] <= 0) return AST_E_NULLPTR;
    t[i].p = params[i];
    t[i].g = grads[i];
    t[i].m = exp_avg ? exp_avg[i] : nullptr;
    t[i].v = exp_avg_sq ? exp_avg_sq[i] : nullptr;
    t[i].n = numel[i];
    t[i].chunk0 = chunks;
    chunks += (numel[i] + kChunk - 1) / kChunk;
  }
  return chunks;
}

int ast_grad_norm_f32(const void* dev_table, int ntensors, long long nchunks, float* partial, float max_norm,
                      float* state, void* stream) {
  if (!dev_table || !partial || !state) return AST_E_NULLPTR;
  if (ntensors <= 0 || nchunks <= 0 || nchunks > 0x7fffffffLL) return AST_E_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sq_norm_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, (const TensorEntry*)dev_table,
                     ntensors, partial);
  hipLaunchKernelGGL(norm_finish_kernel, dim3(1), dim3(kThreads), 0, s, partial, nchunks, max_norm, state);
  return (int)hipGetLastError();
}

int ast_adam_step_f32(const void* dev_table, int ntensors, long long nchunks, const float* state, double lr,
                      double beta1, double beta2, double eps, int step, void* stream) {
  if (!dev_table) return AST_E_NULLPTR;
  if (ntensors <= 0 || nchunks <= 0 || nchunks > 0x7fffffffLL || step <= 0) return AST_E_SHAPE;
  // torch.optim.Adam (foreach): scalars are Python floats (double) until they reach the fp32
  // kernel; bias corrections as Python computes them.
  const double bc1 = 1.0 - pow(beta1, step);
  const double bc2 = 1.0 - pow(beta2, step);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, (hipStream_t)stream,
                     (const TensorEntry*)dev_table, ntensors, state, (float)lr, (float)(1.0 - beta1), (float)beta2,
                     (float)(1.0 - beta2), (float)eps, (float)(lr / bc1), (float)sqrt(bc2), nullptr);
  return (int)hipGetLastError();
}

int ast_adam_step_sched_f32(const void* dev_table, int ntensors, long long nchunks, const float* state, double lr,
                            double beta1, double beta2, double eps, float* sched, int check_finite, void* stream) {
  if (!dev_table || !sched) return AST_E_NULLPTR;
  if (ntensors <= 0 || nchunks <= 0 || nchunks > 0x7fffffffLL) return AST_E_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_sched_kernel, dim3(1), dim3(64), 0, s, state, lr, beta1, beta2, check_finite ? 1 : 0, sched);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, (const TensorEntry*)dev_table,
                     ntensors, state, (float)lr, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     0.f, 1.f, (const float*)sched);
  return (int)hipGetLastError();
}

}  // extern "C"
