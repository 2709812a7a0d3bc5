// VALU issue-rate microbenchmark for the depthwise-conv design: v_fma_f32, v_pk_fma_f32,
// v_dot2_f32_bf16 at 1..8 waves per SIMD. Prints GFLOP-equivalent rates (2 per FMA lane-op).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 4096;

__global__ void k_fma(float* out, float s) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(s), "v"(a[(i + 1) & 7]));
  }
  float r = 0; for (int i = 0; i < 8; ++i) r += a[i];
  if (r == 1234.5f) out[threadIdx.x] = r;
}
__global__ void k_pkfma(float* out, float s) {
  f2 a[8];
  f2 sv = {s, s};
  for (int i = 0; i < 8; ++i) a[i] = f2{threadIdx.x * 0.001f + i, 1.f};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(sv), "v"(a[(i + 1) & 7]));
  }
  float r = 0; for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y;
  if (r == 1234.5f) out[threadIdx.x] = r;
}
__global__ void k_dot2(float* out, float s) {
  float a[8];
  unsigned b[8];
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 0.001f + i; b[i] = 0x3f803f80u + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_dot2_f32_bf16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b[i]), "v"(b[(i + 3) & 7]));
  }
  float r = 0; for (int i = 0; i < 8; ++i) r += a[i];
  if (r == 1234.5f) out[threadIdx.x] = r;
}

int main() {
  float* d; hipMalloc(&d, 4096 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[3] = {"v_fma_f32", "v_pk_fma_f32", "v_dot2_f32_bf16"};
  const double lane_ops[3] = {1, 2, 2};  // MACs per lane per instruction
  for (int kind = 0; kind < 3; ++kind) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      const int blocks = 256 * wps;  // 256-thread blocks = 1 wave per SIMD per block
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
        if (kind == 1) hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
        if (kind == 2) hipLaunchKernelGGL(k_dot2, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
      };
      launch(); hipDeviceSynchronize();
      hipEventRecord(e0); for (int r = 0; r < 5; ++r) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
      const double instr = (double)blocks * 4 * ITERS * 8;  // wave-instructions
      const double tflops = instr * 64 * lane_ops[kind] * 2 / (ms * 1e-3) / 1e12;
      const double cyc_per_instr_simd = (ms * 1e-3 * 2.4e9) / (instr / 1024);
      printf("%-16s waves/SIMD %d: %.3f ms  %.1f TFLOP/s  %.2f cyc/wave-instr/SIMD\n", names[kind], wps, ms, tflops, cyc_per_instr_simd);
    }
  }
  return 0;
}
