// 3x3 convolution of a 1..3-channel input on v_mfma_f32_32x32x16_bf16 in split-bf16 (fp32-accurate)
// arithmetic, for gfx950 (round 6; configurations 42, 43 of conv3x3_igemm.hip).
//
// Replaces the reference's first VGG conv, nn.Conv2d(3, 64, 3, padding=1) behind Normalization
// (models.py:120-131, :199-216), and serves every other conv whose input has <= 3 channels: the
// input gradient of the decoder's last conv (64 -> 3, models.py:598-628) is a zero-padded same conv
// of the 3-channel output gradient (ast_conv3x3_dgrad_f32).
//
// The implicit GEMM of conv3x3_x3_kernel stages K in 16-channel chunks, so a 3-channel input fills
// 27 of 144 K rows; the direct VALU kernel (conv3x3_cin4_kernel) spends 27 fp32 FMAs per output and
// ran at 1.6-3.4 TB/s of its output bytes (profiles/r06y_kernel_stats_*.txt). Here the whole K = 27
// (channel-major taps k = 9c + 3ky + kx; k 27..31 read a zero channel) is two K-16 parts of
// v_mfma_f32_32x32x16_bf16:
//  * A = 32 output channels x K: the lane's three weight terms (ast_x3::split8) in registers for the
//    workgroup's life;
//  * B = K x 32 output pixels of a row, gathered from the workgroup's source tile, staged once in LDS
//    as the three bf16 term planes (hi, mid, lo; ast_x3::split3) of the normalised image;
//  * the six largest term products of the split-bf16 kernels, smallest first;
//  * C: lane (pixel lane & 31, half lane >> 5) holds 16 output channels of one pixel, so each store
//    instruction writes two whole 128-byte lines (32 consecutive pixels of 2 channels). The
//    16x16x32 form of this kernel (pixels on the M side: 4 pixels of 16 channels per lane, one 16-byte
//    store each) wrote 64-byte pieces of 16 planes per instruction and ran at 2.4 TB/s against the
//    VALU kernel's 4.2 TB/s on the config-3 conv_1 (pre + act; profiles/r06c3_ab.txt).
// MFMA work: ~50 us per 16 x 64 x 512^2 launch at one wave per SIMD; the launch is bound by its stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "x3.h"
#include "cin3.h"

namespace {

using ast_x3::bf16;
using ast_x3::bf16x8;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256;   // 4 waves
constexpr int TWC = 64;   // output columns per tile: 2 N-blocks of 32 pixels

template <int TH>
struct C3 {
  static constexpr int SR = TH + 2;             // source rows incl. halo
  static constexpr int RS = TWC + 2;            // source columns incl. halo (LDS row stride, elements)
  static constexpr int CS = SR * RS;            // one channel of one term plane
  static constexpr int PL = 4 * CS;             // one term plane: channels 0..2 and the zero channel 3
  static constexpr int ST_T = (PL + NT - 1) / NT;  // staged elements per thread
  static constexpr int RPW = TH / 4;            // output rows per wave
};

// source index of padded coordinate v (may be -1 or n): zero padding -1 outside, ReflectionPad2d(1)
__device__ __forceinline__ int src_index1(int v, int n, int reflect) {
  if (v >= 0 && v < n) return v;
  if (!reflect) return -1;
  const int r = v < 0 ? -v : 2 * (n - 1) - v;
  return r < 0 ? 0 : (r >= n ? n - 1 : r);
}

__device__ __forceinline__ float relu_f(float v) { return v < 0.f ? 0.f : v; }  // relu(NaN) = NaN

__device__ __forceinline__ unsigned short bits(bf16 v) { return __builtin_bit_cast(unsigned short, v); }

// DG: the input-gradient epilogue of conv3x3_igemm.hip dgrad_epi_one (same arithmetic; y_pre only, no
// bias), its mask loaded before the block's MFMAs; otherwise bias + y_pre / y_act. The epilogue
// modes are template / wave-uniform branches around whole store loops: a per-element choice between
// the store-only and the load-using paths made the compiler wait on vmcnt -- which on gfx9 also
// counts stores -- once per element (0.51 ms for the config-2 conv_1 against 0.31 ms unified).
template <int TH, bool NORM, bool DG>
__global__ __launch_bounds__(NT, DG ? 2 : 3) void conv3x3_cin3_x3_kernel(Cin3Args a) {
  using C = C3<TH>;
  __shared__ unsigned short Xs[3 * C::PL];  // [term hi|mid|lo][channel 0..3][SR][RS] bf16 bits
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, l32 = lane & 31, kh = lane >> 5;
  const int H = a.H, W = a.W;
  const int ngr = (a.Cout + 63) >> 6, tiles_x = (W + TWC - 1) / TWC, tiles_y = (H + TH - 1) / TH;
  int t = blockIdx.x;
  const int grp = t % ngr;
  t /= ngr;
  const int bx = t % tiles_x;
  t /= tiles_x;
  const int by = t % tiles_y;
  const int n = t / tiles_y;
  const int x0 = bx * TWC, y0 = by * TH, co0 = grp * 64;
  const int64_t plane = (int64_t)H * W;
  const float* __restrict__ xin =
      n < a.nsplit ? a.x + (int64_t)n * a.Cin * plane : a.x2 + (int64_t)(n - a.nsplit) * a.Cin * plane;

  // source tile [channel][row][col] (channel 3 and channels past Cin are zero), loads issued first
  float sv[C::ST_T];
#pragma unroll
  for (int i = 0; i < C::ST_T; ++i) {
    const int e = min(tid + i * NT, C::PL - 1);
    const int col = e % C::RS, cr = e / C::RS, r = cr % C::SR, c = cr / C::SR;
    const int sy = src_index1(y0 - 1 + r, H, a.reflect), sx = src_index1(x0 - 1 + col, W, a.reflect);
    const bool ok = c < a.Cin && sy >= 0 && sx >= 0;
    sv[i] = ok ? xin[c * plane + (int64_t)sy * W + sx] : 0.f;
    if (NORM && ok) sv[i] = (sv[i] - a.in_mean[c]) / a.in_std[c];  // padding stays 0 after normalisation
  }

  // A terms: lane (channel co0 + 32q + l32, k-half kh) holds k = 16r + 8kh + j, j = 0..7; k >= 27
  // (the zero channel) is a zero weight. The bias of the workgroup's 64 channels sits in LDS (in
  // registers it held the kernel at two waves per SIMD).
  bf16x8 wa[2][2][3];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int co = co0 + 32 * q + l32;  // < cout_pad: the packed slab is in bounds
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * r + 8 * kh + j;
        w[j] = k < 27 ? a.wp[(int64_t)k * a.cout_pad + co] : 0.f;
      }
      ast_x3::split8(w, wa[q][r][0], wa[q][r][1], wa[q][r][2]);
    }
  }
  __shared__ __attribute__((aligned(16))) float Bias[64];
  if (tid < 64) Bias[tid] = (!DG && a.bias && co0 + tid < a.Cout) ? a.bias[co0 + tid] : 0.f;

#pragma unroll
  for (int i = 0; i < C::ST_T; ++i) {
    const int e = tid + i * NT;
    if (e < C::PL) {
      bf16 h, md, lo;
      ast_x3::split3(sv[i], h, md, lo);
      Xs[e] = bits(h);
      Xs[C::PL + e] = bits(md);
      Xs[2 * C::PL + e] = bits(lo);
    }
  }
  __syncthreads();

  // the lane's gather addresses (hi plane) at the wave's first output row, pixel l32 of the tile
  int ad[2][8];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * r + 8 * kh + j, c = k / 9, tp = k - 9 * c;
      ad[r][j] = c * C::CS + (wv * C::RPW + tp / 3) * C::RS + tp % 3 + l32;
    }

#pragma unroll 1
  for (int i = 0; i < C::RPW; ++i) {
    const int yy = y0 + wv * C::RPW + i;
#pragma unroll
    for (int pb = 0; pb < TWC / 32; ++pb) {
      const int off = i * C::RS + 32 * pb;
      u32x4 xb[2][3];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            xb[r][tt][jj] = (unsigned)Xs[tt * C::PL + ad[r][2 * jj] + off] |
                            ((unsigned)Xs[tt * C::PL + ad[r][2 * jj + 1] + off] << 16);
      // the input-gradient mask of the block's outputs, in flight under the MFMAs
      const int xx = x0 + 32 * pb + l32;
      const bool out = yy < H && xx < W;
      const bool full = co0 + 64 <= a.Cout;  // every accumulator element is an output channel
      const int64_t o0 = (((int64_t)n * a.Cout + co0 + 4 * kh) * H + yy) * W + xx;
      // element v of accumulator q: channel co0 + 32q + 8(v >> 2) + 4kh + (v & 3)
      auto at = [&](int q, int v) { return o0 + (int64_t)(32 * q + 8 * (v >> 2) + (v & 3)) * plane; };
      auto live = [&](int q, int v) { return full || co0 + 32 * q + 8 * (v >> 2) + 4 * kh + (v & 3) < a.Cout; };
      // (branch-free: a load under a per-element branch was followed by its own vmcnt(0) wait, which
      // also waits for every store in flight)
      float em[2][16];
      if constexpr (DG) {
        if (const float* const mp = a.e_mask) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v) em[q][v] = mp[(out && live(q, v)) ? at(q, v) : 0];
        } else {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v) em[q][v] = 1.f;
        }
      }
      f32x16 acc[2];
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[q][v] = 0.f;
      // the six largest term products (w_t . x_u, t + u <= 2), smallest first
      constexpr int TW_[6] = {2, 0, 1, 1, 0, 0}, TX_[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
      for (int p = 0; p < 6; ++p)
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[q][r][TW_[p]], __builtin_bit_cast(bf16x8, xb[r][TX_[p]]),
                                                             acc[q], 0, 0, 0);

      if constexpr (DG) {  // the mask is first read here (else its compares are hoisted above the MFMAs)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(em[q][v]));
      }
      if (!out) continue;
      if constexpr (DG) {
        float* const yp = a.y_pre;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int v = 0; v < 16; ++v)
            if (live(q, v)) {
              const int64_t o = at(q, v);
              float g = acc[q][v];
              if (a.e_add_pre) g = g + a.e_add_pre[o];
              const bool keep = em[q][v] > 0.f;  // no mask reads as > 0
              yp[o] = a.e_add_post ? (keep ? a.e_add_post[o] + g : a.e_add_post[o]) : (keep ? g : 0.f);
            }
      } else {
        float bq[2][16];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float4 b4 = *reinterpret_cast<const float4*>(Bias + 32 * q + 8 * j + 4 * kh);
            bq[q][4 * j] = b4.x;
            bq[q][4 * j + 1] = b4.y;
            bq[q][4 * j + 2] = b4.z;
            bq[q][4 * j + 3] = b4.w;
          }
        if (float* const yp = a.y_pre) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v)
              if (live(q, v)) yp[at(q, v)] = acc[q][v] + bq[q][v];
        }
        if (float* const ya = a.y_act) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v)
              if (live(q, v)) ya[at(q, v)] = relu_f(acc[q][v] + bq[q][v]);
        }
      }
    }
  }
}

template <int TH>
int launch_th(const Cin3Args& a, hipStream_t s) {
  const int64_t nblk = (int64_t)a.N * ((a.H + TH - 1) / TH) * ((a.W + TWC - 1) / TWC) * ((a.Cout + 63) / 64);
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  const dim3 g((unsigned)nblk), b(NT);
  if (a.y_pre && (a.e_mask || a.e_add_pre || a.e_add_post)) {
    if (a.in_mean || a.bias || a.y_act) return AST_E_UNSUPPORTED;  // the input gradient has none of them
    hipLaunchKernelGGL((conv3x3_cin3_x3_kernel<TH, false, true>), g, b, 0, s, a);
  } else if (a.in_mean) {
    hipLaunchKernelGGL((conv3x3_cin3_x3_kernel<TH, true, false>), g, b, 0, s, a);
  } else {
    hipLaunchKernelGGL((conv3x3_cin3_x3_kernel<TH, false, false>), g, b, 0, s, a);
  }
  return (int)hipGetLastError();
}

}  // namespace

int launch_conv_cin3_x3(const Cin3Args& a, int th, hipStream_t s) {
  if (a.Cin < 1 || a.Cin > 3) return AST_E_UNSUPPORTED;
  if (a.cout_pad < (a.Cout + 63) / 64 * 64) return AST_E_UNSUPPORTED;  // the B slab reads stay in bounds
  if ((int64_t)a.Cin * a.H * a.W >= ((int64_t)1 << 31)) return AST_E_SHAPE;
  return th == 8 ? launch_th<8>(a, s) : launch_th<16>(a, s);
}
