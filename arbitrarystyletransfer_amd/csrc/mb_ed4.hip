// MobileNet expand + depthwise, v4: see the comment below.
// Its own translation unit because it is built with -fno-slp-vectorize (Makefile): the depthwise taps
// are scalar v_fma_f32 by design -- on gfx950 v_pk_fma_f32 issues at half rate, so SLP packing the
// independent taps bought no throughput and cost ~120 register shuffles per input row.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../include/ast_hip.h"
#include "mb_common.h"

namespace ast_mb {
namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Reflection-pad source index for i in [-(n-1), 2n-2]; clamped for out-of-tile garbage lanes.
__device__ __forceinline__ int refl(int i, int n) {
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * n - 2 - i : i;
  return min(max(i, 0), n - 1);
}

__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, (bf16)v);
}

// ------------------------------------------------------------------------------------------------
// expand + depthwise, v4 (bf16, stride 1, expand blocks): the hidden rows never leave registers
// ------------------------------------------------------------------------------------------------
// v3 reads ~32 B of LDS per depthwise output (Toeplitz operands) and is LDS/latency-bound. Here one
// wave owns 32 hidden channels of a strip of 32 input columns and slides down a band of rows:
//   expand:    C[pixel][channel] = X[pixel][cin] . W1^T on v_mfma_f32_32x32x16_bf16. In its C layout
//              (col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)) a lane holds ONE
//              channel and 16 pixels; the A rows are assigned so that these are 16 consecutive
//              columns in register order (lane half 0: columns 0..15, half 1: 16..31).
//   depthwise: per input row Hardswish in registers; the two columns across the half boundary come
//              from the partner lane (l ^ 32). Each input row is added into the K output rows it
//              touches (K rotating register accumulators: static indices by unrolling the row loop
//              by K); an output row is finished after its last input row (+bias, Hardswish, SE pool
//              sum, bf16).
//   store:     per output row the wave's 32 channels x 28 columns pass through a small LDS image so
//              the D writes are 8-byte pieces, 7 consecutive lanes per channel row.
// A strip of 32 input columns yields 28 outputs (x0 = 28 s - 2, outputs at local columns 2..29 for
// both kernel sizes, which keeps the D pieces 8-byte aligned); a band of TH output rows reads
// TH + K - 1 input rows. x is read straight from global memory (8 channels of one pixel per lane and
// k-step; the other channel blocks of the strip read the same bytes from L2). The hidden activation
// stays fp32 (v3 rounds it to bf16 in LDS). One wave per workgroup: no barrier but the wave's own.
__device__ __forceinline__ float hswish_fast(float v) {  // x * clamp(x/6 + 1/2, 0, 1): within 2 ulp of hswish
  return v * __builtin_amdgcn_fmed3f(fmaf(v, 1.f / 6.f, 0.5f), 0.f, 1.f);
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

#ifndef ED4_PD3
#define ED4_PD3 0  // x rows in flight beyond the next one, k = 3
#endif
#ifndef ED4_PD5
#define ED4_PD5 0  // and k = 5
#endif
#ifndef ED4_WG4
#define ED4_WG4 1  // multi-strip workgroups with 16-byte D stores where wo % 8 == 0
#endif
#ifndef ED4_WGN
#define ED4_WGN 4  // strips (waves) per such workgroup (even)
#endif
#ifndef ED4_TH
#define ED4_TH 31  // output rows per band (TH + K - 1 a multiple of K for K = 3, 5)
#endif
#ifndef ED4_DOT2
#define ED4_DOT2 0  // k5 stride-1 depthwise taps 0-3 on bf16 v_dot2 (A/B builds)
#endif
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

// WG4 (wo % 8 == 0): a workgroup is 4 waves on 4 adjacent strips (same channel block and band). Their
// 4 x 28 output columns are contiguous, so each output row goes through one shared LDS image and
// leaves as 16-byte stores covering 224-byte runs at 16-byte alignment. (Per wave, 56-byte runs of
// 8-byte stores were store-issue-bound: a build without the D stores ran the k3 blocks 2x faster.)
// R1 (the ratio-1 blocks: DecoderBlock's upsample block, mobilenetv2.py:103-116, and the depthwise
// pass of the split ada_out): no expand conv -- the MFMA multiplies the block's own 32 channels by
// an identity B (exact: bf16 x 1.0 accumulated once in fp32), which is the transposition into the
// lane-per-channel layout; no Hardswish before the depthwise. UP = 2 resolves the nearest upsample
// in the gather (reflect on the upsampled grid, then halve).
// NOD (pool-only pass of the fused block pair, see expand_dw_pw4_kernel): the same row pipeline and SE
// pool sums, no D stores.
#ifndef ED4_K5_WPE
#define ED4_K5_WPE 2  // minimum waves per SIMD of the k5 kernels with cin_pad <= 48 (A/B builds)
#endif
template <int K, int KS, int TH, int PD, bool VEC, bool WG4, bool R1 = false, int UP = 1, bool NOD = false>
__global__ __launch_bounds__(WG4 ? 64 * ED4_WGN : 64, (K == 5 && KS >= 6) ? 1 : (K == 5 && KS <= 3) ? ED4_K5_WPE : 2) void expand_dw4_kernel(EdArgs a, int strips, int bands, int ncb, int total) {
  constexpr int P = (K - 1) / 2, NJ = TH + K - 1, OW = 28, SP = 40;  // SP: staging row pitch (bf16)
  constexpr int NW = ED4_WGN, CPR = NW * OW / 8;  // WG4: strips per workgroup, 16-byte chunks per row
  constexpr int GP = NW * OW + 8;  // WG4 staging row pitch (bf16): 16-byte aligned rows
  __shared__ __align__(16) bf16 stage[WG4 ? 2 * 32 * GP : 32 * SP];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, wv = WG4 ? threadIdx.x >> 6 : 0;
  // XCD-aware order (workgroup b runs on XCD b % 8): consecutive logical ids -- the channel blocks
  // of one strip, which read the same x -- share an XCD and its L2
  const int per = (total + 7) >> 3;
  const int L = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (L >= total) return;
  const int cb = L % ncb;
  int rest = L / ncb;
  const int sg = WG4 ? (strips + NW - 1) / NW : strips;  // strip groups of the grid
  const int s = WG4 ? NW * (rest % sg) + wv : rest % sg;
  rest /= sg;
  const int band = rest % bands;
  const int n = rest / bands;
  const int x0 = s * OW - 2, y0 = band * TH;
  const int ch = cb * 32 + r;
  const bool chv = ch < a.hid;

  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = chv ? a.wdw[ch * K * K + i] : 0.f;
  const float bd = chv ? a.bdw[ch] : 0.f, b1 = (chv && !R1) ? a.b1[ch] : 0.f;
#if ED4_DOT2
  constexpr bool DOT2 = K == 5 && !R1;
  bf2 wp[DOT2 ? K : 1][3];  // taps (0, 1), (2, 3), (4, 0) of each kernel row as bf16 pairs
  if constexpr (DOT2) {
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      wp[ky][0] = bf2{(bf16)wk[ky * K], (bf16)wk[ky * K + 1]};
      wp[ky][1] = bf2{(bf16)wk[ky * K + 2], (bf16)wk[ky * K + 3]};
      wp[ky][2] = bf2{(bf16)wk[ky * K + 4], (bf16)0.f};
    }
  }
#endif
  const int hid16 = (a.hid + 15) / 16 * 16;
  bf16x8 bw[KS];  // B[k = 8h + j][col r] = W1[ch][16 s + 8h + j]; R1: identity on the block's channels
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    if constexpr (R1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) bw[q][j] = (bf16)(16 * q + 8 * h + j == r ? 1.f : 0.f);
    } else {
      bw[q] = ch < hid16 ? *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.w1) +
                                                            (int64_t)ch * a.cin_pad + 16 * q + 8 * h)
                         : bf16x8{};
    }
  }

  // A[row r][k = 8h + j] = x[channel 16 s + 8h + j (+ 32 cb for R1)][pixel pc(r)]
  const int pc = 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3);
  const int gx = refl(x0 + pc, a.wd) / UP;
  const int hw2 = 2 * a.h * a.w;  // bytes per channel plane (host-checked: cin * hw2 < 2^31)
  // one buffer descriptor per image: channels >= cin (the zero-weight padding of the last k-step)
  // fall outside its range and load as 0; x2 is not used (the host takes v4 only for c1 == cin)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(reinterpret_cast<const bf16*>(a.x1) + (int64_t)n * a.cin * (hw2 / 2)), 0, a.cin * hw2,
      0x00020000);
  // raw 16-bit x values of the rows in flight, packed into MFMA fragments only when their row starts:
  // packing right after the loads (what the compiler does with a bf16x8 built from the loads) makes
  // the wave wait for them at once, so no load would overlap the VALU work
  unsigned xraw[PD + 1][KS][8];
  auto load_row = [&](int j, unsigned (*raw)[8]) {
    const int vrow = (8 * h + (R1 ? 32 * cb : 0)) * hw2 + 2 * (refl(y0 - P + j, a.hd) / UP * a.w + gx);
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) raw[q][e] = __builtin_amdgcn_raw_buffer_load_b16(xr, vrow + (16 * q + e) * hw2, 0, 0);
  };

  const int64_t plane_o = (int64_t)a.ho * a.wo;
  // D through a per-image buffer descriptor: a piece that must not be written (past the right or
  // bottom border, a padding channel, the unused lanes of the last pass) gets an offset outside the
  // range and is dropped by the hardware, so every row issues the same stores on every path -- with
  // a data-dependent store count the compiler's vmcnt bookkeeping degrades to waiting for all stores
  // before the next row's x fragments can be used
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<bf16*>(a.d) + (int64_t)n * a.hid * plane_o, 0, (int)(2 * a.hid * plane_o), 0x00020000);
  constexpr unsigned kDrop = 0x80000000u;
  const bool edge = x0 + 2 + OW > a.wo;  // last strip: outputs past the right border
  float psum = 0.f;
  int rb = 0;  // WG4 staging image of the next output row
  auto finish = [&](int orow, const float* v, bool live) {
    const int oy = y0 + orow;
    const bool rowv = live && oy < a.ho;  // uniform
    float y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = hswish_fast(v[i]);
    // SE pool: valid local columns are 2..15 (half 0) and 16..29 (half 1)
    float t = 0.f;
    if (!edge) {
      t = h ? y[0] + y[1] : y[14] + y[15];
#pragma unroll
      for (int i = 2; i < 14; ++i) t += y[i];
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int lc = 16 * h + i;
        t += (lc >= 2 && lc < 30 && x0 + lc < a.wo) ? y[i] : 0.f;
      }
    }
    psum += rowv ? t : 0.f;
    if constexpr (NOD) return;
    unsigned pk[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      pk[i] = (unsigned)bf16_bits(y[2 * i]) | ((unsigned)bf16_bits(y[2 * i + 1]) << 16);
    if constexpr (WG4) {
      // this wave's 14 valid columns per half: local 2..15 (half 0) / 16..29 (half 1) -> image columns
      // 28 wv + 0..13 / 28 wv + 14..27 of channel row r, in buffer `rb` (a row alternates the two)
      unsigned* gw = reinterpret_cast<unsigned*>(stage + rb * 32 * GP + r * GP + OW * wv + 14 * h);
#pragma unroll
      for (int i = 0; i < 7; ++i) gw[i] = pk[i + 1 - h];
      lds_barrier();
      // 32 channel rows x 14 chunks of 8 columns (16 bytes) over the workgroup's 256 threads
      const int sb = (s - wv) * OW;  // first output column of the workgroup (strip group start)
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const int q = threadIdx.x + 64 * NW * t2;
        const int cl = min(q / CPR, 31), k8 = q - CPR * (q / CPR);
        const uint4 v = *reinterpret_cast<const uint4*>(stage + rb * 32 * GP + cl * GP + 8 * k8);
        const int xg = sb + 8 * k8;
        const bool ok = rowv && q < 32 * CPR && cb * 32 + cl < a.hid && xg < a.wo;
        const unsigned off = ok ? (unsigned)(2 * ((cb * 32 + cl) * plane_o + (int64_t)oy * a.wo + xg)) : kDrop;
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, dr, (int)off, 0, 0);
      }
      rb ^= 1;  // the other image next row: one barrier per row orders the reuse two rows later
      return;
    }
    uint4* sw = reinterpret_cast<uint4*>(stage + r * SP + 16 * h);
    sw[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    sw[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    lds_barrier();
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      const int q = lane + 64 * t4;  // 32 channel rows x 7 pieces of local columns 2+4i .. 5+4i
      const int cl = min(q / 7, 31), i4 = q - 7 * (q / 7);
      const unsigned* sp = reinterpret_cast<const unsigned*>(stage + cl * SP + 2 + 4 * i4);
      const unsigned v0 = sp[0], v1 = sp[1];
      const int xg = x0 + 2 + 4 * i4;
      const bool ok = rowv && q < 224 && cb * 32 + cl < a.hid;
      const unsigned base = (unsigned)(2 * ((cb * 32 + cl) * plane_o + (int64_t)oy * a.wo + xg));
      if constexpr (VEC) {
        const unsigned off = ok && xg + 4 <= a.wo ? base : kDrop;
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v0, v1}, dr, (int)off, 0, 0);
      } else {
        const unsigned short e4[4] = {(unsigned short)v0, (unsigned short)(v0 >> 16), (unsigned short)v1,
                                      (unsigned short)(v1 >> 16)};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          __builtin_amdgcn_raw_buffer_store_b16(e4[e], dr, (int)(ok && xg + e < a.wo ? base + 2 * e : kDrop), 0, 0);
      }
    }
    // the next row's staging writes follow these reads in this wave's program order
  };

  // Every row issues the same loads and stores on every path (NJ % K == 0, the next row is loaded
  // even past the band -- refl keeps it in bounds -- and finish runs for every row, its stores dropped
  // when the row is not an output row): the compiler then waits at each row start only for the x
  // loads, not for the D stores issued after them.
  static_assert(NJ % K == 0, "TH + K - 1 must be a multiple of K");
  float acc[K][16];
#pragma unroll
  for (int d = 0; d <= PD; ++d) load_row(d, xraw[d]);
  for (int jb = 0; jb < NJ; jb += K) {
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const int j = jb + u;
      f32x16 c;
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = b1;
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        u32x4 f;
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = (xraw[0][q][2 * e] & 0xffffu) | (xraw[0][q][2 * e + 1] << 16);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f), bw[q], c, 0, 0, 0);
      }
#pragma unroll
      for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int q = 0; q < KS; ++q)
#pragma unroll
          for (int e = 0; e < 8; ++e) xraw[d][q][e] = xraw[d + 1][q][e];
      load_row(j + PD + 1, xraw[PD]);  // in flight during this row's VALU work
      float e[20];
#pragma unroll
      for (int i = 0; i < 16; ++i) e[2 + i] = R1 ? c[i] : hswish_fast(c[i]);
      const float r0 = __shfl_xor(h ? e[2] : e[16], 32, 64), r1 = __shfl_xor(h ? e[3] : e[17], 32, 64);
      e[0] = r0;   // half 1: columns 14, 15 (half 0's are never used: its outputs 0, 1 are halo)
      e[1] = r1;
      e[18] = r0;  // half 0: columns 16, 17 (likewise unused by half 1)
      e[19] = r1;
#if ED4_DOT2
      // k5 taps as bf16 pairs on v_dot2c_f32_bf16 (fp32 accumulate): (0, 1), (2, 3), (4, zero)
      bf2 E[DOT2 ? 20 : 1];
      if constexpr (DOT2) {
#pragma unroll
        for (int m = 0; m < 20; ++m) E[m] = bf2{(bf16)e[m], m + 1 < 20 ? (bf16)e[m + 1] : (bf16)0.f};
      }
#endif
#pragma unroll
      for (int ky = K - 1; ky >= 0; --ky) {
        const int orow = j - ky;
        const int slot = ((u - ky) % K + K) % K;
        const bool live = orow >= 0 && orow < TH;  // uniform
        if (live) {
#if ED4_DOT2
          if constexpr (DOT2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              float v = ky == 0 ? bd : acc[slot][i];
              v = __builtin_amdgcn_fdot2_f32_bf16(wp[ky][0], E[i], v, false);
              v = __builtin_amdgcn_fdot2_f32_bf16(wp[ky][1], E[i + 2], v, false);
              acc[slot][i] = __builtin_amdgcn_fdot2_f32_bf16(wp[ky][2], E[i + 4], v, false);
            }
          } else
#endif
          {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              float v = ky == 0 ? bd : acc[slot][i];
#pragma unroll
              for (int kx = 0; kx < K; ++kx) v = fmaf(wk[ky * K + kx], e[i + 2 - P + kx], v);
              acc[slot][i] = v;
            }
          }
        }
        if (ky == K - 1) finish(orow, acc[slot], live);
      }
    }
  }
  psum += __shfl_xor(psum, 32, 64);
  // one slot per (band, strip) of the image; strips past the right border (WG4 padding waves) store 0
  if (h == 0 && chv) a.pool[((int64_t)n * a.hid + ch) * a.slots + band * (a.slots / bands) + s] = psum;
}


template <int K, int KS, bool R1 = false, int UP = 1>
int launch_ks(EdArgs a, hipStream_t st) {
  constexpr int TH = ED4_TH, PD = K == 3 ? ED4_PD3 : ED4_PD5;
  const int strips = (a.wo + 27) / 28, bands = (a.ho + TH - 1) / TH, ncb = (a.hid + 31) / 32;
  const int64_t total = (int64_t)ncb * strips * bands * a.n;
  if (total > 0x7ffffff0LL) return AST_E_SHAPE;
  const int64_t grid = (total + 7) / 8 * 8;
  if constexpr (!R1 && UP == 1 && K == 3) {
    if (a.nod) {  // pool-only pass of the fused pair: per-wave strips, no D stores
      if (ed_plan(a, (int64_t)bands * strips)) return 0;
      hipLaunchKernelGGL((expand_dw4_kernel<K, KS, TH, PD, true, false, false, 1, true>), dim3((unsigned)grid), dim3(64), 0,
                         st, a, strips, bands, ncb, (int)total);
      return (int)hipGetLastError();
    }
  }
  if (a.nod) return AST_E_UNSUPPORTED;
  // WG4 for k = 3 only: measured 3.3 -> 2.9 ms on the 16->96 block at 1024^2, while the k5 blocks
  // lose 10-50% to the per-row workgroup barrier (their rows are longer and less uniform)
  if (ED4_WG4 && K == 3 && a.wo % 8 == 0) {  // WG4: 4 strips per workgroup, 16-byte D stores
    const int64_t total4 = (int64_t)ncb * ((strips + ED4_WGN - 1) / ED4_WGN) * bands * a.n, grid4 = (total4 + 7) / 8 * 8;
    if (ed_plan(a, (int64_t)bands * ((strips + ED4_WGN - 1) / ED4_WGN) * ED4_WGN)) return 0;
    hipLaunchKernelGGL((expand_dw4_kernel<K, KS, TH, PD, true, true, R1, UP>), dim3((unsigned)grid4), dim3(64 * ED4_WGN), 0, st, a,
                       strips, bands, ncb, (int)total4);
  } else if (ed_plan(a, (int64_t)bands * strips)) {
    return 0;
  } else if (a.wo % 4 == 0) {
    // VEC: wo % 4 == 0, so a 4-column D piece is 8-byte aligned and wholly inside or outside the row
    hipLaunchKernelGGL((expand_dw4_kernel<K, KS, TH, PD, true, false, R1, UP>), dim3((unsigned)grid), dim3(64), 0, st, a,
                       strips, bands, ncb, (int)total);
  } else {
    hipLaunchKernelGGL((expand_dw4_kernel<K, KS, TH, PD, false, false, R1, UP>), dim3((unsigned)grid), dim3(64), 0, st, a,
                       strips, bands, ncb, (int)total);
  }
  return (int)hipGetLastError();
}

template <int K>
int launch_k(EdArgs a, hipStream_t st) {
  switch (a.cin_pad / 16) {
    case 1: return launch_ks<K, 1>(a, st);
    case 2: return launch_ks<K, 2>(a, st);
    case 3: return launch_ks<K, 3>(a, st);
    case 4: return launch_ks<K, 4>(a, st);
    case 5: return launch_ks<K, 5>(a, st);
    case 6: return launch_ks<K, 6>(a, st);
    case 8: return launch_ks<K, 8>(a, st);
    default: return AST_E_UNSUPPORTED;
  }
}


// Stride 2 (the encoder's down-sampling blocks): the same wave layout -- 32 channels x a strip of 32
// input columns, expand on the 32x32x16 MFMA, one channel per lane with 16 columns in registers --
// but a lane makes the outputs at its 8 even local columns, and an input row j feeds the output rows
// r with j = 2r + ky: S = (K + 1) / 2 rotating accumulators of 8 (static slots by unrolling the row
// loop by 2S). A strip yields 14 outputs (input local columns 2, 4, .., 28 for k = 3 and 5), a band
// TH output rows from 2 TH + K - 2 input rows (padded to a multiple of 2S; the extra rows' outputs
// are dropped). D leaves per output row through LDS as 4-byte pieces (14 columns = 7 dwords per
// channel row, 4-byte aligned when wo is even).
template <int K, int KS, int TH>
__global__ __launch_bounds__(64, 2) void expand_dw4s2_kernel(EdArgs a, int strips, int bands, int ncb, int total) {
  constexpr int P = (K - 1) / 2, S = (K + 1) / 2, U = 2 * S, NJ0 = 2 * TH + K - 2;
  constexpr int NJ = (NJ0 + U - 1) / U * U, OW = 14, SP = 16;  // SP: staging row pitch (bf16)
  __shared__ __align__(16) bf16 stage[32 * SP];
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int per = (total + 7) >> 3;
  const int L = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (L >= total) return;
  const int cb = L % ncb;
  int rest = L / ncb;
  const int s = rest % strips;
  rest /= strips;
  const int band = rest % bands;
  const int n = rest / bands;
  const int x0 = 2 * s * OW - 2, y0 = band * TH;  // x0: input column of local 0; y0: first output row
  const int ch = cb * 32 + r;
  const bool chv = ch < a.hid;

  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = chv ? a.wdw[ch * K * K + i] : 0.f;
  const float bd = chv ? a.bdw[ch] : 0.f, b1 = chv ? a.b1[ch] : 0.f;
  const int hid16 = (a.hid + 15) / 16 * 16;
  bf16x8 bw[KS];
#pragma unroll
  for (int q = 0; q < KS; ++q)
    bw[q] = ch < hid16 ? *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.w1) +
                                                          (int64_t)ch * a.cin_pad + 16 * q + 8 * h)
                       : bf16x8{};
  const int pc = 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3);
  const int gx = refl(x0 + pc, a.wd);
  const int hw2 = 2 * a.h * a.w;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(reinterpret_cast<const bf16*>(a.x1) + (int64_t)n * a.cin * (hw2 / 2)), 0, a.cin * hw2,
      0x00020000);
  unsigned xraw[KS][8];
  auto load_row = [&](int j) {
    const int vrow = 8 * h * hw2 + 2 * (refl(2 * y0 - P + j, a.hd) * a.w + gx);
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) xraw[q][e] = __builtin_amdgcn_raw_buffer_load_b16(xr, vrow + (16 * q + e) * hw2, 0, 0);
  };

  const int64_t plane_o = (int64_t)a.ho * a.wo;
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<bf16*>(a.d) + (int64_t)n * a.hid * plane_o, 0, (int)(2 * a.hid * plane_o), 0x00020000);
  constexpr unsigned kDrop = 0x80000000u;
  const int oc0 = s * OW;                // first output column of the strip
  const bool edge = oc0 + OW > a.wo;
  float psum = 0.f;
  // this lane's outputs: local input columns 16h + 2i, i = 0..7; valid i = 1..7 (half 0) / 0..6 (half 1),
  // output columns oc0 + 7h + i - (1 - h)
  auto finish = [&](int orow, const float* v, bool live) {
    const int oy = y0 + orow;
    const bool rowv = live && oy < a.ho;  // uniform
    float y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = hswish_fast(v[i]);
    float t = 0.f;
    if (!edge) {
      t = h ? y[0] : y[7];
#pragma unroll
      for (int i = 1; i < 7; ++i) t += y[i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int j = 7 * h + i - (1 - h);  // output index within the strip
        t += (j >= 7 * h && j < 7 * h + 7 && oc0 + j < a.wo) ? y[i] : 0.f;
      }
    }
    psum += rowv ? t : 0.f;
    unsigned short* sw = reinterpret_cast<unsigned short*>(stage + r * SP + 7 * h);
#pragma unroll
    for (int i = 0; i < 7; ++i) sw[i] = bf16_bits(y[i + 1 - h]);
    lds_barrier();
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      const int q = lane + 64 * t4;  // 32 channel rows x 7 dword pieces
      const int cl = min(q / 7, 31), k2 = q - 7 * (q / 7);
      const unsigned v0 = *reinterpret_cast<const unsigned*>(stage + cl * SP + 2 * k2);
      const int xg = oc0 + 2 * k2;
      const bool ok = rowv && q < 224 && cb * 32 + cl < a.hid && xg < a.wo;
      const unsigned off = ok ? (unsigned)(2 * ((cb * 32 + cl) * plane_o + (int64_t)oy * a.wo + xg)) : kDrop;
      __builtin_amdgcn_raw_buffer_store_b32(v0, dr, (int)off, 0, 0);
    }
  };

  float acc[S][8];
  load_row(0);
  for (int jb = 0; jb < NJ; jb += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = jb + u;
      f32x16 c;
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = b1;
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        u32x4 f;
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = (xraw[q][2 * e] & 0xffffu) | (xraw[q][2 * e + 1] << 16);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f), bw[q], c, 0, 0, 0);
      }
      load_row(j + 1);
      float e[20];
#pragma unroll
      for (int i = 0; i < 16; ++i) e[2 + i] = hswish_fast(c[i]);
      const float r0 = __shfl_xor(h ? e[2] : e[16], 32, 64), r1 = __shfl_xor(h ? e[3] : e[17], 32, 64);
      e[0] = r0;
      e[1] = r1;
      e[18] = r0;
      e[19] = r1;
#pragma unroll
      for (int ky = K - 1; ky >= 0; --ky) {
        if ((u - ky) % 2 != 0) continue;  // static: the rows this input row feeds
        const int orow = (j - ky) / 2;     // j - ky is even
        const int slot = (((u - ky) / 2) % S + S) % S;
        const bool live = j - ky >= 0 && orow < TH;
        if (live) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            float v = ky == 0 ? bd : acc[slot][i];
#pragma unroll
            for (int kx = 0; kx < K; ++kx) v = fmaf(wk[ky * K + kx], e[2 * i + 2 - P + kx], v);
            acc[slot][i] = v;
          }
        }
        if (ky == K - 1) finish(orow, acc[slot], live);
      }
    }
  }
  psum += __shfl_xor(psum, 32, 64);
  if (h == 0 && chv) a.pool[((int64_t)n * a.hid + ch) * a.slots + band * strips + s] = psum;
}

template <int K, int KS>
int launch_s2_ks(EdArgs a, hipStream_t st) {
  constexpr int TH = 32;
  const int strips = (a.wo + 13) / 14, bands = (a.ho + TH - 1) / TH, ncb = (a.hid + 31) / 32;
  const int64_t total = (int64_t)ncb * strips * bands * a.n;
  if (total > 0x7ffffff0LL) return AST_E_SHAPE;
  const int64_t grid = (total + 7) / 8 * 8;
  if (ed_plan(a, (int64_t)bands * strips)) return 0;
  hipLaunchKernelGGL((expand_dw4s2_kernel<K, KS, TH>), dim3((unsigned)grid), dim3(64), 0, st, a, strips, bands, ncb,
                     (int)total);
  return (int)hipGetLastError();
}

template <int K>
int launch_s2(EdArgs a, hipStream_t st) {
  switch (a.cin_pad / 16) {
    case 1: return launch_s2_ks<K, 1>(a, st);
    case 2: return launch_s2_ks<K, 2>(a, st);
    case 3: return launch_s2_ks<K, 3>(a, st);
    case 4: return launch_s2_ks<K, 4>(a, st);
    default: return AST_E_UNSUPPORTED;
  }
}


// ------------------------------------------------------------------------------------------------
// Fused block pair, pass 2: expand + depthwise recomputed, SE-gated pw-linear conv in the kernel
// ------------------------------------------------------------------------------------------------
// Materialising the depthwise output D costs a hidden-width write and read per block (the pw kernel
// re-reads it), yet the SE gate needs the whole image pooled before the pw-linear conv can run. The
// pair: pass 1 is expand_dw4_kernel<.., NOD> (pool sums only, no D), ast_mb_se_fold folds the gate
// into wg[n], and this pass recomputes expand + depthwise and applies wg directly. A workgroup is one
// strip x band of one image:
//  * NCB compute waves: wave cb computes hidden channels 32 cb .. 32 cb + 31 exactly as
//    expand_dw4_kernel (same instructions, same rounding) and writes each finished output row to LDS
//    as bf16 [channel][32 columns] -- the values D would hold;
//  * one GEMM wave (wave NCB) consumes row r while the compute waves produce row r + 1 (two row
//    images; one workgroup barrier per row orders both the hand-over and the reuse): the pw GEMM
//    out[co][px] = sum_c wg[n][co][c] D[c][px] as 16 x 16 tiles on v_mfma_f32_16x16x32_bf16 with
//    pw_kernel's operand layout and chunk order (A = wg[n] from LDS, B through ds_read_b64_tr_b16),
//    then + b2 (+ residual) as pw_kernel does: the output is bit-identical to expand_dw4 + se_fold +
//    pw. 28 of the 32 columns are stored.
// HBM traffic per block: x twice (both passes) and out once, against x, D written, D read and out.
// Timing-only builds (scripts/build_variants.sh; wrong results): EDPW_T_NOSTORE drops the GEMM wave's
// residual loads and output stores, EDPW_T_NOGEMM its MFMAs too, EDPW_T_NODW the compute waves'
// depthwise FMAs.
#ifndef EDPW_T_NOSTORE
#define EDPW_T_NOSTORE 0
#endif
#ifndef EDPW_T_NOGEMM
#define EDPW_T_NOGEMM 0
#endif
#ifndef EDPW_T_NODW
#define EDPW_T_NODW 0
#endif
#ifndef EDPW_T_GEMM1
#define EDPW_T_GEMM1 0  // the GEMM wave sums one 32-channel block instead of NCB
#endif
template <int KS, int NCB, int NCO>
__global__ __launch_bounds__(64 * (NCB + 1)) __attribute__((amdgpu_waves_per_eu(3))) void expand_dw_pw4_kernel(
    EdpwArgs pa, int strips, int bands, int total) {
  constexpr int K = 3, P = 1, TH = ED4_TH, NJ = TH + K - 1, OW = 28, DP = 48;  // DP: D image row pitch (bf16)
  constexpr int NT = 2 * NCO;  // 16 x 16 output tiles per row: (output-channel block, pixel half)
  // wg[n] in LDS, row pitch = 8 (mod 128) elements: the A fragments' 8-byte reads (16 rows x 2
  // k-groups per half-wave) hit distinct banks
  constexpr int WP = (NCB * 32 + 127) / 128 * 128 + 8;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  __shared__ __align__(16) bf16 dimg[2][NCB * 32 * DP];
  __shared__ __align__(16) bf16 wsm[NCO * 16 * WP];
  __shared__ __align__(16) float ostg[NCO * 16 * 32];  // GEMM wave: a row's outputs [co][28 px] (+ b2)
  const EdArgs& a = pa.e;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, cb = threadIdx.x >> 6;
  const int per = (total + 7) >> 3;
  const int L = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (L >= total) return;
  const int s = L % strips;
  const int rest = L / strips;
  const int band = rest % bands;
  const int n = rest / bands;
  const int x0 = s * OW - 2, y0 = band * TH;
  {
    const bf16* wn = reinterpret_cast<const bf16*>(pa.wg) + (int64_t)n * pa.cout_pad * pa.hid_pad;
    for (int e = threadIdx.x; e < NCO * 16 * NCB * 4; e += 64 * (NCB + 1)) {  // 8-element pieces
      const int row = e / (NCB * 4), c8 = e - row * (NCB * 4);
      *reinterpret_cast<u32x4*>(wsm + row * WP + 8 * c8) =
          *reinterpret_cast<const u32x4*>(wn + (int64_t)row * pa.hid_pad + 8 * c8);
    }
  }  // (ordered before the first GEMM by the first row barrier)

  if (cb == NCB) {  // ---- GEMM wave ----
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int64_t plane_o = (int64_t)a.ho * a.wo;
    const int orange = (int)(2 * pa.cout * plane_o);
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<bf16*>(pa.out) + (int64_t)n * pa.cout * plane_o, 0, orange, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(reinterpret_cast<const bf16*>(pa.res ? pa.res : pa.out)) + (int64_t)n * pa.cout * plane_o,
        0, pa.res ? orange : 0, 0x00020000);
    constexpr unsigned kDrop = 0x80000000u;
    float bco[NCO][4];
#pragma unroll
    for (int m = 0; m < NCO; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = 16 * m + 4 * g + j;
        bco[m][j] = (pa.b2 && co < pa.cout) ? pa.b2[co] : 0.f;
      }
    // wo % 4 == 0 (every config-5 map): the row's outputs leave through ostg as 8-byte pieces of 4
    // pixels (7 per channel row; the strip starts at a multiple of 28 columns) and the residual
    // arrives the same way -- 2-byte scattered accesses made the stores the pass's largest cost
    // (a timing build without them: 28.7 -> 20.1 ms per config-5 step). Same arithmetic and
    // rounding as below: bit-identical.
    if ((a.wo & 3) == 0) {
      constexpr int NP = NCO * 16 * 7, PPL = (NP + 63) / 64;  // pieces per row, per lane
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      // the A fragments (wg[n], the same for every row) stay in registers: read once, after the first
      // row barrier (which also orders wsm's staging), instead of per row. (Every wave of the
      // workgroup must pass the same number of barriers: no extra one here.)
      s16x4 afr[NCO][NCB][2];
      for (int orow = 0; orow < TH; ++orow) {
        const int oy = y0 + orow;
        const bool rowv = oy < a.ho;
        unsigned poff[PPL];
        u32x2 prv[PPL];
#pragma unroll
        for (int i = 0; i < PPL; ++i) {
          const int p = lane + 64 * i, co = p / 7, seg = p - 7 * co, ox = x0 + 2 + 4 * seg;
          poff[i] = (rowv && p < NP && co < pa.cout && ox < a.wo)
                        ? (unsigned)(2 * (co * plane_o + (int64_t)oy * a.wo + ox)) : kDrop;
          prv[i] = (pa.res && !EDPW_T_NOSTORE) ? __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rr, (int)poff[i], 0, 0))
                                               : u32x2{0u, 0u};
        }
        lds_barrier();  // row orow's image is complete
        if (orow == 0) {
#pragma unroll
          for (int m = 0; m < NCO; ++m) {
            const bf16* wr = wsm + (m * 16 + (lane & 15)) * WP + 4 * g;
#pragma unroll
            for (int kc = 0; kc < NCB; ++kc) {
              afr[m][kc][0] = *reinterpret_cast<const s16x4*>(wr + 32 * kc);
              afr[m][kc][1] = *reinterpret_cast<const s16x4*>(wr + 32 * kc + 16);
            }
          }
        }
        const bf16* img = dimg[orow & 1];
        // k-major over the NT tiles: each tile's k-steps in the same order (bit-identical), NT - 1
        // independent MFMAs between consecutive ones on one accumulator, and each image fragment
        // read once per k-step for both output-channel tiles
        f32x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < (EDPW_T_NOGEMM ? 0 : EDPW_T_GEMM1 ? 1 : NCB); ++kc) {
          bf16x8 bfr[2];
#pragma unroll
          for (int ph = 0; ph < 2; ++ph) {
            const int col = ph * 16 + 4 * p4;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (32 * kc + 4 * g + q4) * DP + col));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (32 * kc + 16 + 4 * g + q4) * DP + col));
            bfr[ph] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, __builtin_shufflevector(afr[t / 2][kc][0], afr[t / 2][kc][1], 0, 1, 2, 3, 4, 5,
                                                                   6, 7)),
                bfr[t & 1], acc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int px = (t & 1) * 16 + (lane & 15);
          if (px >= 2 && px < 2 + OW) {
#pragma unroll
            for (int j = 0; j < 4; ++j) ostg[(t / 2 * 16 + 4 * g + j) * 32 + px - 2] = acc[t][j] + bco[t / 2][j];
          }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes are done
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < PPL; ++i) {
          const int p = min(lane + 64 * i, NP - 1), co = p / 7, seg = p - 7 * co;
          const f32x4 v = *reinterpret_cast<const f32x4*>(ostg + co * 32 + 4 * seg);
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = v[e];
            if (pa.res) {
              const unsigned w = prv[i][e >> 1];
              o[e] = o[e] + (float)__builtin_bit_cast(bf16, (unsigned short)(e & 1 ? w >> 16 : w & 0xffffu));
            }
          }
          const u32x2 pk = {(unsigned)bf16_bits(o[0]) | ((unsigned)bf16_bits(o[1]) << 16),
                            (unsigned)bf16_bits(o[2]) | ((unsigned)bf16_bits(o[3]) << 16)};
          if (!EDPW_T_NOSTORE || o[0] == 1.2345e-30f)
            __builtin_amdgcn_raw_buffer_store_b64(pk, orr, (int)poff[i], 0, 0);
        }
      }
      return;
    }
    for (int orow = 0; orow < TH; ++orow) {
      const int oy = y0 + orow;
      const bool rowv = oy < a.ho;
      unsigned off[NT][4];
      unsigned short rv[NT][4];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int px = (t & 1) * 16 + (lane & 15), ox = x0 + px;
        const bool ok = rowv && px >= 2 && px < 2 + OW && ox < a.wo;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = t / 2 * 16 + 4 * g + j;
          off[t][j] = (ok && co < pa.cout) ? (unsigned)(2 * (co * plane_o + (int64_t)oy * a.wo + ox)) : kDrop;
          rv[t][j] = (pa.res && !EDPW_T_NOSTORE) ? __builtin_amdgcn_raw_buffer_load_b16(rr, (int)off[t][j], 0, 0)
                                                 : (unsigned short)0;
        }
      }
      lds_barrier();  // row orow's image is complete
      const bf16* img = dimg[orow & 1];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = (t & 1) * 16 + 4 * p4;
        const bf16* wr = wsm + (t / 2 * 16 + (lane & 15)) * WP + 4 * g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < (EDPW_T_NOGEMM ? 0 : NCB); ++kc) {
          const s16x4 alo = *reinterpret_cast<const s16x4*>(wr + 32 * kc);
          const s16x4 ahi = *reinterpret_cast<const s16x4*>(wr + 32 * kc + 16);
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (32 * kc + 4 * g + q4) * DP + col));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (32 * kc + 16 + 4 * g + q4) * DP + col));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7)),
              __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7)), acc, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float o = acc[j] + bco[t / 2][j];
          if (pa.res) o = o + (float)__builtin_bit_cast(bf16, rv[t][j]);
          if (!EDPW_T_NOSTORE || o == 1.2345e-30f)
            __builtin_amdgcn_raw_buffer_store_b16(bf16_bits(o), orr, (int)off[t][j], 0, 0);
        }
      }
    }
    return;
  }

  // ---- compute waves: expand_dw4_kernel's row pipeline for channels 32 cb .. 32 cb + 31 ----
  const int ch = cb * 32 + r;
  const bool chv = ch < a.hid;
  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = chv ? a.wdw[ch * K * K + i] : 0.f;
  const float bd = chv ? a.bdw[ch] : 0.f, b1 = chv ? a.b1[ch] : 0.f;
  const int hid16 = (a.hid + 15) / 16 * 16;
  bf16x8 bw[KS];
#pragma unroll
  for (int q = 0; q < KS; ++q)
    bw[q] = ch < hid16 ? *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.w1) +
                                                          (int64_t)ch * a.cin_pad + 16 * q + 8 * h)
                       : bf16x8{};
  const int pc = 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3);
  const int gx = refl(x0 + pc, a.wd);
  const int hw2 = 2 * a.h * a.w;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(reinterpret_cast<const bf16*>(a.x1) + (int64_t)n * a.cin * (hw2 / 2)), 0, a.cin * hw2,
      0x00020000);
  unsigned xraw[KS][8];
  auto load_row = [&](int j) {
    const int vrow = 8 * h * hw2 + 2 * (refl(y0 - P + j, a.hd) * a.w + gx);
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) xraw[q][e] = __builtin_amdgcn_raw_buffer_load_b16(xr, vrow + (16 * q + e) * hw2, 0, 0);
  };
  auto finish = [&](int orow, const float* v, bool live) {
    if (!live) return;  // uniform over the workgroup
    float y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = hswish_fast(v[i]);
    unsigned pk[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      pk[i] = (unsigned)bf16_bits(y[2 * i]) | ((unsigned)bf16_bits(y[2 * i + 1]) << 16);
    u32x4* dw = reinterpret_cast<u32x4*>(dimg[orow & 1] + ch * DP + 16 * h);
    dw[0] = u32x4{pk[0], pk[1], pk[2], pk[3]};
    dw[1] = u32x4{pk[4], pk[5], pk[6], pk[7]};
    lds_barrier();  // hand the row to the GEMM wave (which has finished the row two back)
  };

  static_assert(NJ % K == 0, "TH + K - 1 must be a multiple of K");
  float acc[K][16];
  load_row(0);
  for (int jb = 0; jb < NJ; jb += K) {
#pragma unroll
    for (int u = 0; u < K; ++u) {
      const int j = jb + u;
      f32x16 c;
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = b1;
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        u32x4 f;
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = (xraw[q][2 * e] & 0xffffu) | (xraw[q][2 * e + 1] << 16);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f), bw[q], c, 0, 0, 0);
      }
      load_row(j + 1);
      float e[20];
#pragma unroll
      for (int i = 0; i < 16; ++i) e[2 + i] = hswish_fast(c[i]);
      const float r0 = __shfl_xor(h ? e[2] : e[16], 32, 64), r1 = __shfl_xor(h ? e[3] : e[17], 32, 64);
      e[0] = r0;
      e[1] = r1;
      e[18] = r0;
      e[19] = r1;
#pragma unroll
      for (int ky = K - 1; ky >= 0; --ky) {
        const int orow = j - ky;
        const int slot = ((u - ky) % K + K) % K;
        const bool live = orow >= 0 && orow < TH;
        if (live) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = ky == 0 ? bd : acc[slot][i];
#pragma unroll
            for (int kx = 0; kx < (EDPW_T_NODW ? (ky == 0 && kx == 0 ? 1 : 0) : K); ++kx)
              v = fmaf(wk[ky * K + kx], e[i + 2 - P + kx], v);
            acc[slot][i] = v;
          }
        }
        if (ky == K - 1) finish(orow, acc[slot], live);
      }
    }
  }
}

}  // namespace

int launch_ed4(EdArgs a, int k, int stride, hipStream_t st) {
  if (a.nod && (!a.w1 || stride != 1 || k != 3)) return AST_E_UNSUPPORTED;
  if (a.c1 != a.cin || (a.w1 && a.cin_pad % 16 != 0) || (int64_t)a.cin_pad * 2 * a.h * a.w >= 0x7fffffffLL ||
      (int64_t)a.hid * 2 * a.ho * a.wo >= 0x7fffffffLL)
    return AST_E_UNSUPPORTED;
  if (!a.w1) {  // ratio-1 block: k3, stride 1, hid == cin, optional x2 upsample
    if (k != 3 || stride != 1 || a.hid != a.cin || (int64_t)a.cin * 2 * a.h * a.w >= 0x7fffffffLL) return AST_E_UNSUPPORTED;
    if (a.hd == 2 * a.h && a.wd == 2 * a.w) return launch_ks<3, 2, true, 2>(a, st);
    if (a.hd == a.h && a.wd == a.w) return launch_ks<3, 2, true, 1>(a, st);
    return AST_E_UNSUPPORTED;
  }
  if (a.hd != a.h || a.wd != a.w) return AST_E_UNSUPPORTED;  // no upsample
  // k3 with wide inputs on small maps (128^2 and below: 128->384, 96->288, 80->320 in config 5)
  // measured faster on v3 (0.48 vs 0.59 ms for 128->384): the 28-column strips waste 9% of a
  // 128-column map and the grid is a few waves deep
  if (k == 3 && stride == 1 && a.cin_pad >= 80 && (int64_t)a.ho * a.wo <= 128 * 128) return AST_E_UNSUPPORTED;
  if (stride == 2) {
    if (a.wo % 2 != 0) return AST_E_UNSUPPORTED;  // 4-byte D pieces
    if (k == 3) return launch_s2<3>(a, st);
    if (k == 5) return launch_s2<5>(a, st);
    return AST_E_UNSUPPORTED;
  }
  if (k == 3) return launch_k<3>(a, st);
  if (k == 5) {
    static const int v5 = [] {  // AST_MB_ED5=0: the v4 k5 kernels (A/B measurements)
      const char* v = getenv("AST_MB_ED5");
      return v ? atoi(v) : 1;
    }();
    if (v5) {
      const int r = launch_ed5(a, k, stride, st);
      if (r != AST_E_UNSUPPORTED) return r;
    }
    return launch_k<5>(a, st);
  }
  return AST_E_UNSUPPORTED;
}


// (cin_pad / 16, hidden channel blocks of 32, output channel blocks of 16) instantiated for the
// fused pair: the stride-1 k3 expand blocks of config 5 with narrow inputs (16 -> 96 -> 16,
// 24 -> 144 -> 24 | 16)
#define EDPW_SHAPES(X) X(1, 3, 1) X(2, 5, 2) X(2, 5, 1)

int edpw4_supported(int cin_pad, int hid, int cout, int k, int stride, int up, int ho, int wo) {
  if (k != 3 || stride != 1 || up != 1 || ho < 2 || wo < 2) return 0;
  const int ks = cin_pad / 16, ncb = (hid + 31) / 32, nco = (cout + 15) / 16;
#define EDPW_CASE(KS_, NCB_, NCO_) if (ks == KS_ && ncb == NCB_ && nco == NCO_) return 1;
  EDPW_SHAPES(EDPW_CASE)
#undef EDPW_CASE
  return 0;
}

int launch_edpw4(const EdpwArgs& pa, hipStream_t st) {
  const EdArgs& a = pa.e;
  if (!a.w1 || a.c1 != a.cin || a.hd != a.h || a.wd != a.w || a.ho != a.h || a.wo != a.w || a.cin_pad % 16 != 0)
    return AST_E_UNSUPPORTED;
  if (!edpw4_supported(a.cin_pad, a.hid, pa.cout, 3, 1, 1, a.ho, a.wo)) return AST_E_UNSUPPORTED;
  if (pa.hid_pad != (a.hid + 31) / 32 * 32 || pa.cout_pad != (pa.cout + 15) / 16 * 16) return AST_E_SHAPE;
  if ((int64_t)a.cin_pad * 2 * a.h * a.w >= 0x7fffffffLL || (int64_t)pa.cout * 2 * a.ho * a.wo >= 0x7fffffffLL)
    return AST_E_UNSUPPORTED;
  constexpr int TH = ED4_TH;
  const int strips = (a.wo + 27) / 28, bands = (a.ho + TH - 1) / TH;
  const int64_t total = (int64_t)strips * bands * a.n;
  if (total > 0x7ffffff0LL) return AST_E_SHAPE;
  const unsigned grid = (unsigned)((total + 7) / 8 * 8);
  const int ks = a.cin_pad / 16, ncb = (a.hid + 31) / 32, nco = (pa.cout + 15) / 16;
#define EDPW_CASE(KS_, NCB_, NCO_)                                                                       \
  if (ks == KS_ && ncb == NCB_ && nco == NCO_) {                                                         \
    hipLaunchKernelGGL((expand_dw_pw4_kernel<KS_, NCB_, NCO_>), dim3(grid), dim3(64 * (NCB_ + 1)), 0, st, pa, strips, \
                       bands, (int)total);                                                               \
    return (int)hipGetLastError();                                                                       \
  }
  EDPW_SHAPES(EDPW_CASE)
#undef EDPW_CASE
  return AST_E_UNSUPPORTED;
}

}  // namespace ast_mb
