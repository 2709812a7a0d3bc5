// Deterministic reductions shared by the kernels (SURVEY.md §5 race detection / determinism): no
// result may depend on the order in which workgroups finish, so partial sums never meet in floating
// -point atomics. Two patterns:
//  * partials + ordered reduce: every workgroup writes its partial tile into a caller-provided
//    workspace with plain stores; an extra launch then sums the partials of each output element in
//    a fixed order (reduce_cols: [slot][element] layouts such as split-K GEMM tiles; reduce_rows:
//    [element][slot] layouts such as the SE-pool sums, slots contiguous);
//  * loss accumulators (scalar losses): a device buffer of AST_LOSS_ACC_FLOATS floats —
//    [0] the value, [1] an arrival counter (uint32, kept at 0 between launches), [2..] one partial
//    per workgroup. Each workgroup stores its partial and takes a ticket; the workgroup that
//    arrives last sums all partials in workgroup order and adds the total to [0]. Orders of
//    arrival differ run to run, the summation order does not.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace ast_det {
namespace {

// Sum of v over the workgroup in a fixed order (wave butterflies, then waves in index order).
// blockDim.x a multiple of 64, at most 1024; every thread receives the total.
__device__ __forceinline__ float block_sum_fixed(float v) {
  __shared__ float sh_[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh_[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
  const int nw = (int)(blockDim.x >> 6);
  for (int i = 0; i < nw; ++i) t += sh_[i];
  __syncthreads();
  return t;
}

// Add this workgroup's contribution v (valid in thread 0) to the loss accumulator acc (see above).
// Every thread of the workgroup must call it (it synchronises the workgroup); the grid may have at
// most AST_LOSS_SLOTS workgroups (host-checked).
__device__ __forceinline__ void loss_acc_commit(float* acc, float v) {
  __shared__ int last_;
  const unsigned nb = gridDim.x * gridDim.y * gridDim.z;
  const unsigned bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  unsigned* counter = reinterpret_cast<unsigned*>(acc + 1);
  if (threadIdx.x == 0) {
    __hip_atomic_store(acc + 2 + bid, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last_ = prev == nb - 1;
  }
  __syncthreads();
  if (!last_) return;
  // Every reading thread acquires at agent scope, not only thread 0 (whose fetch_add did): the
  // partials come from workgroups on other XCDs, whose L2s are not coherent with this one's, and the
  // workgroup barrier alone orders nothing beyond the workgroup.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  float s = 0.f;
  for (unsigned i = threadIdx.x; i < nb; i += blockDim.x)
    s += __hip_atomic_load(acc + 2 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s = block_sum_fixed(s);
  if (threadIdx.x == 0) {
    acc[0] += s;
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// [slot][element] partials: out[b * ob + j] (+)= sum_s part[b * pb + s * stride + j], j < count.
// A workgroup of 64 * G threads owns 64 consecutive elements; thread group g sums the slots
// s = g, g + G, ... in order (16 loads in flight), and the G group sums are added in group order.
template <int G>
__global__ __launch_bounds__(64 * G) void reduce_cols_kernel(const float* __restrict__ part, int64_t slots,
                                                             int64_t stride, int64_t count, int64_t pb,
                                                             float* __restrict__ out, int64_t ob, int accumulate) {
  __shared__ float sh[G][64];
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + l;
  const float* p = part + (int64_t)blockIdx.y * pb + j;
  float s = 0.f;
  if (j < count) {
    int64_t sl = g;
    for (; sl + 15 * G < slots; sl += 16 * G) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(sl + u * G) * stride];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; sl < slots; sl += G) s += p[sl * stride];
  }
  sh[g][l] = s;
  __syncthreads();
  if (g == 0 && j < count) {
    float t = sh[0][l];
#pragma unroll
    for (int i = 1; i < G; ++i) t += sh[i][l];
    float* o = out + (int64_t)blockIdx.y * ob + j;
    *o = accumulate ? *o + t : t;
  }
}

// [row][slot] partials (slots contiguous): out[r] = sum_s part[r * slots + s], one wave per row,
// lane l summing s = l, l + 64, ... in order, then a fixed butterfly.
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ part, int64_t rows, int slots,
                                                          float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (r >= rows) return;
  const float* p = part + r * slots;
  float s = 0.f;
  int i = l;
  for (; i + 192 < slots; i += 256) {
    const float a = p[i], b = p[i + 64], c = p[i + 128], d = p[i + 192];
    s += a;
    s += b;
    s += c;
    s += d;
  }
  for (; i < slots; i += 64) s += p[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (l == 0) out[r] = s;
}

inline hipError_t reduce_cols(const float* part, int64_t slots, int64_t stride, int64_t count, int64_t batch,
                              int64_t pb, float* out, int64_t ob, bool accumulate, hipStream_t st) {
  if (count <= 0 || batch <= 0) return hipSuccess;
  const int64_t bx = (count + 63) / 64;
  if (bx > 0x7fffffffLL || batch > 65535) return hipErrorInvalidValue;
  if (slots >= 64)
    hipLaunchKernelGGL(reduce_cols_kernel<8>, dim3((unsigned)bx, (unsigned)batch), dim3(512), 0, st, part, slots,
                       stride, count, pb, out, ob, accumulate ? 1 : 0);
  else
    hipLaunchKernelGGL(reduce_cols_kernel<1>, dim3((unsigned)bx, (unsigned)batch), dim3(64), 0, st, part, slots,
                       stride, count, pb, out, ob, accumulate ? 1 : 0);
  return hipGetLastError();
}

inline hipError_t reduce_rows(const float* part, int64_t rows, int slots, float* out, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  const int64_t bx = (rows + 3) / 4;
  if (bx > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((unsigned)bx), dim3(256), 0, st, part, rows, slots, out);
  return hipGetLastError();
}

}  // namespace
}  // namespace ast_det
