// MobileNet-style inverted-residual path for gfx950.
//
// The reference block (DepthWiseConv, mobilenetv2.py:95-165) is
//     pw 1x1 (+BN) -> Hardswish -> dw kxk reflect, stride s (+BN) -> Hardswish -> SELayer -> pw 1x1 (+BN) (+x)
// with the ratio-1 form (decoder upsample blocks, models.py:248-271) skipping the expand conv.
// Eval-mode BatchNorm is folded into the conv weights/biases on the host. Each block runs as:
//
//   expand_dw_kernel   x tile (+halo, reflect) -> LDS; expand GEMM on MFMA (bf16 16x16x32 or fp32
//                      16x16x4) into a 16-channel LDS chunk of the hidden tensor, Hardswish; depthwise
//                      kxk on VALU from LDS, +bias, Hardswish; writes the dw output D once and adds the
//                      per-(n, channel) sums that SELayer's AdaptiveAvgPool needs (atomics).
//                      The expanded hidden tensor never reaches HBM. Three generations: v1 (any dtype,
//                      stride 1/2), v2 (bf16, one barrier per chunk), v3 (bf16, stride 1, expand
//                      blocks: the depthwise on MFMA in Toeplitz form, parameters resident in LDS).
//   se_fold_kernel     SE MLP per image (mobilenetv2.py:63-81) and folds the gate into the pw-linear
//                      weights: Wg[n][co][c] = W2[co][c] * gate[n][c]   (x*gate then conv == conv with Wg).
//   pw_kernel          per-image GEMM out = Wg[n] . D + b (+ residual, optionally nearest-upsampled),
//                      D staged through LDS transposed so both MFMA operands are k-contiguous.
//
// Storage type T is float or __bf16; all arithmetic and accumulation is fp32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../include/ast_hip.h"
#include "mb_common.h"
#include "det.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16 v) { return (float)v; }
template <typename T>
__device__ __forceinline__ T from_f(float v) { return (T)v; }

// torch Hardswish: x * min(max(x + 3, 0), 6) / 6 (here * (1/6): within 1 ulp, no IEEE divide sequence)
__device__ __forceinline__ float hswish(float v) { return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f); }

// Workgroup barrier for LDS hand-offs only. __syncthreads() also fences global memory, i.e. waits
// for every outstanding global load and store of the wave (vmcnt(0)): that would drain the dw
// kernel's output stores and the pw kernel's in-flight prefetch at every chunk.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Reflection-pad source index for i in [-(n-1), 2n-2]; clamped for out-of-tile garbage lanes.
__device__ __forceinline__ int refl(int i, int n) {
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * n - 2 - i : i;
  return min(max(i, 0), n - 1);
}

// One 16x16 MFMA k-step from two row-major [row][k] LDS images (A: 16 rows from `a`, B: 16 rows from `b`).
template <typename T>
struct Mma;
template <>
struct Mma<bf16> {
  static constexpr int KS = 32;   // k per instruction
  static constexpr int PAD = 8;   // row padding (elements): rows stay 16-byte aligned
  __device__ static f32x4 step(const bf16* a, const bf16* b, int lda, int ldb, int k0, f32x4 acc, int lane) {
    const int r = lane & 15, kk = k0 + 8 * (lane >> 4);
    const bf16x8 fa = *reinterpret_cast<const bf16x8*>(a + r * lda + kk);
    const bf16x8 fb = *reinterpret_cast<const bf16x8*>(b + r * ldb + kk);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc, 0, 0, 0);
  }
  // k = 16 tail (lane l: A[l&15][4(l>>4)+j], B[4(l>>4)+j][l&15]), so K pads to 16, not 32
  __device__ static f32x4 step16(const bf16* a, const bf16* b, int lda, int ldb, int k0, f32x4 acc, int lane) {
    typedef short s4 __attribute__((ext_vector_type(4)));
    const int r = lane & 15, kk = k0 + 4 * (lane >> 4);
    const s4 fa = *reinterpret_cast<const s4*>(a + r * lda + kk);
    const s4 fb = *reinterpret_cast<const s4*>(b + r * ldb + kk);
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fa, fb, acc, 0, 0, 0);
  }
  // acc += A . B over k in [0, kpad), kpad a multiple of 16
  __device__ static f32x4 gemm(const bf16* a, const bf16* b, int lda, int ldb, int kpad, f32x4 acc, int lane) {
    int k0 = 0;
    for (; k0 + KS <= kpad; k0 += KS) acc = step(a, b, lda, ldb, k0, acc, lane);
    if (k0 < kpad) acc = step16(a, b, lda, ldb, k0, acc, lane);
    return acc;
  }
};
template <>
struct Mma<float> {
  static constexpr int KS = 4;
  static constexpr int PAD = 4;   // keeps rows 16-byte aligned for the staging writes
  __device__ static f32x4 step(const float* a, const float* b, int lda, int ldb, int k0, f32x4 acc, int lane) {
    const int r = lane & 15, kk = k0 + (lane >> 4);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a[r * lda + kk], b[r * ldb + kk], acc, 0, 0, 0);
  }
  __device__ static f32x4 gemm(const float* a, const float* b, int lda, int ldb, int kpad, f32x4 acc, int lane) {
    for (int k0 = 0; k0 < kpad; k0 += KS) acc = step(a, b, lda, ldb, k0, acc, lane);
    return acc;
  }
};

// 8 consecutive 16-byte-aligned elements -> fp32
__device__ __forceinline__ void load8(const float* s, float* v) {
  const float4 a = reinterpret_cast<const float4*>(s)[0], b = reinterpret_cast<const float4*>(s)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const bf16* s, float* v) {
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(s);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
}

// ------------------------------------------------------------------------------------------------
// expand + depthwise (+ SE pool sums)
// ------------------------------------------------------------------------------------------------
using ast_mb::EdArgs;  // mb_common.h (shared with mb_ed4.hip)
using ast_mb::EdpwArgs;

constexpr int kChunk = 16;  // hidden channels per LDS chunk

template <int K, int S, int TH, int TW_>
struct EdGeom {
  static constexpr int TW = TW_;
  static constexpr int IH = (TH - 1) * S + K;
  static constexpr int IW = (TW - 1) * S + K;
  static constexpr int NP = IH * IW;
  static constexpr int HP = (NP + 15) / 16 * 16;  // halo pixels as MFMA N tiles
  static constexpr int RP = TH / 2;         // output row pairs
  static constexpr int CG = 16 / RP;        // column groups per row pair
  static constexpr int CW = TW / CG;        // output columns per thread
  static_assert(RP * CG == 16 && CW * CG == TW && CW >= 1, "tile");
  // Hidden-chunk LDS image hs[channel][row][col]: row pitch = 1 (mod 4), channel pitch = 1 (mod 8),
  // so a half-wave's depthwise reads (2 channels x RP row pairs x CG column groups) fall in 32
  // distinct banks for stride 1.
  static constexpr int IWP = IW + ((1 - IW) % 4 + 4) % 4;
  static constexpr int HPS = (IH * IWP + 7) / 8 * 8 + 1;
};

template <typename T, int K, int S, int TH, int TW>
__host__ __device__ constexpr size_t ed_lds_bytes(int cin_pad, bool expand) {
  using G = EdGeom<K, S, TH, TW>;
  const size_t xs = expand ? (size_t)G::HP * (cin_pad + Mma<T>::PAD) * sizeof(T) : 0;
  const size_t ws = expand ? (size_t)kChunk * (cin_pad + Mma<T>::PAD) * sizeof(T) : 0;
  const size_t hs = (size_t)kChunk * G::HPS * sizeof(float);
  return xs + ws + hs;
}

template <typename T, int N>
struct VecOf {
  typedef T type __attribute__((ext_vector_type(N)));
};

// Store N consecutive outputs: one vector store when the run is whole and aligned.
template <typename T, int N>
__device__ __forceinline__ void store_run(T* o, const float* y, int count) {
  if (count == N && ((uintptr_t)o % (sizeof(T) * N)) == 0) {
    typename VecOf<T, N>::type v;
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = from_f<T>(y[c]);
    *reinterpret_cast<typename VecOf<T, N>::type*>(o) = v;
  } else {
#pragma unroll
    for (int c = 0; c < N; ++c)
      if (c < count) o[c] = from_f<T>(y[c]);
  }
}

#ifndef ED_SKIP
#define ED_SKIP 0  // experiment builds of the v1 kernel: 1 = no D store, 2 = no depthwise FMAs, 4 = no expand
#endif
template <typename T, int K, int S, int UP, bool EXPAND, int TH, int TW>
__global__ __launch_bounds__(kThreads, 2) void expand_dw_kernel(EdArgs a) {
  using G = EdGeom<K, S, TH, TW>;
  constexpr int P = (K - 1) / 2;
  extern __shared__ __align__(16) unsigned char smem[];
  const int ldx = a.cin_pad + Mma<T>::PAD;
  T* xs = reinterpret_cast<T*>(smem);
  T* ws = xs + (EXPAND ? G::HP * ldx : 0);
  float* hs = reinterpret_cast<float*>(smem + (EXPAND ? (size_t)(G::HP + kChunk) * ldx * sizeof(T) : 0));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int b = blockIdx.x;
  const int tx = b % a.tiles_x;
  b /= a.tiles_x;
  const int ty = b % a.tiles_y;
  const int n = b / a.tiles_y;
  const int oy0 = ty * TH, ox0 = tx * G::TW;
  const int iy0 = oy0 * S - P, ix0 = ox0 * S - P;
  const T* x1 = reinterpret_cast<const T*>(a.x1);
  const T* x2 = reinterpret_cast<const T*>(a.x2);
  const int64_t hw = (int64_t)a.h * a.w;

  // source offset (within a plane) of halo pixel p: reflect pad in the dw grid, then the upsample
  auto src_off = [&](int p) -> int {
    int gy = refl(iy0 + p / G::IW, a.hd), gx = refl(ix0 + p % G::IW, a.wd);
    if (UP == 2) { gy >>= 1; gx >>= 1; }
    return gy * a.w + gx;
  };
  auto plane = [&](int c) -> const T* {
    return c < a.c1 ? x1 + ((int64_t)n * a.c1 + c) * hw : x2 + ((int64_t)n * (a.cin - a.c1) + (c - a.c1)) * hw;
  };

  if (EXPAND) {  // stage the x halo tile once, channel-minor: xs[p][c], one 16-byte write per channel group
    constexpr int CV = 16 / sizeof(T);
    const int groups = a.cin_pad / CV;
    // channel c lives at xb1 + c*hw (c < c1) or xb2 + c*hw (c >= c1): wave-uniform selection
    const T* xb1 = x1 + (int64_t)n * a.c1 * hw;
    const T* xb2 = x2 + (int64_t)n * (a.cin - a.c1) * hw - (int64_t)a.c1 * hw;
    for (int p = tid; p < G::HP; p += kThreads) {  // lanes run along pixels: coalesced global loads
      const bool valid = p < G::NP;
      const int off = valid ? src_off(p) : 0;
      for (int g = 0; g < groups; ++g) {
        typename VecOf<T, CV>::type v;
#pragma unroll
        for (int j = 0; j < CV; ++j) {
          const int c = g * CV + j;
          T x = from_f<T>(0.f);
          if (c < a.cin && valid) x = (c < a.c1 ? xb1 : xb2)[(int64_t)c * hw + off];
          v[j] = x;
        }
        *reinterpret_cast<typename VecOf<T, CV>::type*>(xs + p * ldx + g * CV) = v;
      }
    }
  }

  // depthwise thread mapping: hidden channel hl of the chunk, output rows 2*rp, 2*rp+1, columns cg*CW..
  const int hl = tid >> 4, rp = (tid & 15) / G::CG, cg = (tid & 15) % G::CG;
  const int r0 = rp * 2, c0 = cg * G::CW;
  constexpr int NT = G::HP / 16;              // MFMA N tiles (halo pixels / 16)
  constexpr int TPW = (NT + 3) / 4;           // per wave
  int hoff[TPW];                              // this lane's hs offset in each of its tiles (-1: padding)
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int p = (wave + 4 * i) * 16 + (lane & 15);
    hoff[i] = p < G::NP ? (p / G::IW) * G::IWP + p % G::IW : -1;
  }
  // tiles wholly inside the output: no bounds checks, and every CW run is a vector-aligned store
  const bool interior = oy0 + TH <= a.ho && ox0 + G::TW <= a.wo && (a.wo % G::CW) == 0;
  const int64_t plane_o = (int64_t)a.ho * a.wo;
  T* dbase = reinterpret_cast<T*>(a.d) + (int64_t)n * a.hid * plane_o + (int64_t)(oy0 + r0) * a.wo + ox0 + c0;
  constexpr int CV = 16 / sizeof(T);

  __shared__ float wdc[kChunk * K * K], bdc[kChunk], b1c[kChunk];  // this chunk's dw weights/biases

  // The next chunk's weights are fetched into registers while this chunk computes.
  constexpr int WSV = 4;                      // expand-weight vectors per thread (cin_pad <= 512)
  constexpr int WDV = (kChunk * K * K + kThreads - 1) / kThreads;
  const int nv = EXPAND ? a.cin_pad / CV : 0;
  uint4 pw1[WSV];
  float pwd[WDV], pb = 0.f;
  // (a macro, not a lambda: a by-reference closure over these arrays sent them to scratch memory)
#define ED_FETCH(H0)                                                                                       \
  {                                                                                                        \
    const int hh = (H0);                                                                                   \
    if (EXPAND) {                                                                                          \
      const T* w1 = reinterpret_cast<const T*>(a.w1) + (int64_t)hh * a.cin_pad;                            \
      _Pragma("unroll") for (int i = 0; i < WSV; ++i) {                                                    \
        const int e = tid + i * kThreads, r = e / max(nv, 1), v = e - r * nv;                              \
        uint4 val = make_uint4(0, 0, 0, 0);                                                                \
        if (e < kChunk * nv) val = *reinterpret_cast<const uint4*>(w1 + r * a.cin_pad + v * CV);           \
        pw1[i] = val;                                                                                      \
      }                                                                                                    \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < WDV; ++i) {                                                      \
      const int e = tid + i * kThreads;                                                                    \
      float val = 0.f;                                                                                     \
      if (e < kChunk * K * K && hh * K * K + e < a.hid * K * K) val = a.wdw[hh * K * K + e];               \
      pwd[i] = val;                                                                                        \
    }                                                                                                      \
    float bv = 0.f;                                                                                        \
    if (tid < kChunk) {                                                                                    \
      if (hh + tid < a.hid) bv = a.bdw[hh + tid];                                                          \
    } else if (EXPAND && tid < 2 * kChunk) {                                                               \
      if (hh + tid - kChunk < a.hid) bv = a.b1[hh + tid - kChunk];                                         \
    }                                                                                                      \
    pb = bv;                                                                                               \
  }
  ED_FETCH(0);

  for (int h0 = 0; h0 < a.hid; h0 += kChunk) {
#pragma unroll
    for (int i = 0; i < WDV; ++i)
      if (tid + i * kThreads < kChunk * K * K) wdc[tid + i * kThreads] = pwd[i];
    if (tid < kChunk) bdc[tid] = pb;
    else if (tid < 2 * kChunk) b1c[tid - kChunk] = pb;
    if (EXPAND) {
#pragma unroll
      for (int i = 0; i < WSV; ++i) {
        const int e = tid + i * kThreads, r = e / max(nv, 1), v = e - r * nv;
        if (e < kChunk * nv) *reinterpret_cast<uint4*>(ws + r * ldx + v * CV) = pw1[i];
      }
    }
    lds_barrier();  // xs (first chunk), ws and the chunk's weights/biases ready
    if (h0 + kChunk < a.hid) ED_FETCH(h0 + kChunk);
    if (EXPAND && !(ED_SKIP & 4)) {
      float bias[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[r] = b1c[4 * (lane >> 4) + r];
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int t = wave + 4 * i;
        if (t < NT) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
          acc = Mma<T>::gemm(ws, xs + t * 16 * ldx, ldx, ldx, a.cin_pad, acc, lane);
          if (hoff[i] >= 0) {
            float* hp = hs + hoff[i] + 4 * (lane >> 4) * G::HPS;
#pragma unroll
            for (int r = 0; r < 4; ++r) hp[r * G::HPS] = hswish(acc[r] + bias[r]);
          }
        }
      }
    } else if (!EXPAND) {
      for (int p = tid; p < G::NP; p += kThreads) {
        const int off = src_off(p);
        float* hp = hs + (p / G::IW) * G::IWP + p % G::IW;
#pragma unroll 4
        for (int r = 0; r < kChunk; ++r) hp[r * G::HPS] = h0 + r < a.hid ? to_f(plane(h0 + r)[off]) : 0.f;
      }
    }
    lds_barrier();

    // depthwise kxk on the chunk
    const int hc = h0 + hl;
    if (hc < a.hid) {
      float wk[K * K];
#pragma unroll
      for (int i = 0; i < K * K; ++i) wk[i] = wdc[hl * K * K + i];
      float acc[2][G::CW];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < G::CW; ++c) acc[r][c] = 0.f;
      constexpr int NCOL = (G::CW - 1) * S + K;
      const float* hrow = hs + hl * G::HPS + (r0 * S) * G::IWP + c0 * S;
#pragma unroll
      for (int j = 0; j < S + K; ++j) {
        float v[NCOL];
#pragma unroll
        for (int m = 0; m < NCOL; ++m) v[m] = hrow[j * G::IWP + m];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int ky = j - r * S;
          if (ky >= 0 && ky < K && !(ED_SKIP & 2)) {
#pragma unroll
            for (int kx = 0; kx < K; ++kx)
#pragma unroll
              for (int c = 0; c < G::CW; ++c) acc[r][c] = fmaf(wk[ky * K + kx], v[c * S + kx], acc[r][c]);
          }
        }
      }
      const float bd = bdc[hl];
      float psum = 0.f;
      T* drow = dbase + (int64_t)hc * plane_o;
      if (interior) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          typename VecOf<T, G::CW>::type v;
#pragma unroll
          for (int c = 0; c < G::CW; ++c) {
            const float y = hswish(acc[r][c] + bd);
            psum += y;
            v[c] = from_f<T>(y);
          }
          if (!(ED_SKIP & 1)) *reinterpret_cast<typename VecOf<T, G::CW>::type*>(drow + r * a.wo) = v;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          if (oy0 + r0 + r >= a.ho) continue;
          const int ncol = min(G::CW, a.wo - (ox0 + c0));
          float y[G::CW];
#pragma unroll
          for (int c = 0; c < G::CW; ++c) {
            y[c] = hswish(acc[r][c] + bd);
            if (c < ncol) psum += y[c];
          }
          if (ncol > 0) store_run<T, G::CW>(drow + r * a.wo, y, ncol);
        }
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) psum += __shfl_xor(psum, o, 64);
      if ((tid & 15) == 0) a.pool[((int64_t)n * a.hid + hc) * a.slots + ty * a.tiles_x + tx] = psum;
    }
    lds_barrier();  // hs / ws reused by the next chunk
  }
#undef ED_FETCH
}

// ------------------------------------------------------------------------------------------------
// expand + depthwise, v2 (bf16 storage, stride 1): one barrier per hidden chunk
// ------------------------------------------------------------------------------------------------
// 512 threads, a TH x TW output tile of one image, hidden channels in chunks of 16. Per iteration c:
//   (1) issue the global loads of chunk c+2's parameters (expand weights, dw weights, biases);
//   (2) expand chunk c+1 on MFMA (operands swapped so each lane holds 4 consecutive halo pixels of
//       one hidden channel), + bias, Hardswish, one 8-byte bf16 write into hidden image hs[(c+1)&1];
//       ratio-1 blocks instead load chunk c+1's (upsampled, reflect-padded) input tile;
//   (3) depthwise chunk c from hs[c&1]: each thread owns R output rows x 4 columns of one channel,
//       reads its (R+K-1) x 8 input window with 8-byte LDS reads, fp32 FMAs, + bias, Hardswish,
//       the SE pool partial sum (half-wave shuffle, one atomic per channel) and the bf16 D store;
//   (4) write chunk c+2's parameters into the 3-slot LDS ring; one LDS-only barrier.
// The hidden image holds bf16 (a bf16 model stores the expanded tensor in bf16); all arithmetic fp32.
template <int K, int TH, int TW, int R, int NT_ = 512>
struct Ed2Geom {
  static constexpr int NT = NT_;
  static constexpr int IH = TH + K - 1, IW = TW + K - 1;
  static constexpr int IWE = (IW + 3) / 4 * 4;     // halo row length of the expand enumeration
  static constexpr int NPE = IH * IWE;
  static constexpr int HP = (NPE + 15) / 16 * 16;  // expand pixels, MFMA tiles of 16
  static constexpr int NTILE = HP / 16;
  static constexpr int TPC = (TH / R) * (TW / 4);  // threads per channel
  static_assert(NT / TPC == 16, "16 hidden channels per chunk (the MFMA N)");
  static_assert(TPC == 32 || TPC == 64, "a channel's threads are one half-wave or wave (pool shuffle)");
  // image pitch: the next row group's rows land 16 banks away (conflict-free 8-byte reads)
  static constexpr int pitch() {
    for (int p = IWE; p <= IWE + 16; p += 4)
      if ((R * p) % 64 == 32) return p;
    return IWE;
  }
  static constexpr int IWP = pitch();
  static constexpr int CHP = (IH * IWP + 63) / 64 * 64 + 4;  // channel pitch (bf16), = 4 mod 64
  static constexpr int NR = R + K - 1;                      // input rows per thread
  static constexpr int KKP = (K * K + 3) / 4 * 4;           // dw weight row pitch (floats)
  static constexpr int WIN = 16 * IH * IWE;                 // ratio-1 input elements per chunk
};

struct Ed2Slot {  // byte offsets inside one parameter slot
  int w1, wd, b1, bd, bytes;
};
template <int K>
__host__ __device__ constexpr Ed2Slot ed2_slot(int ldx, bool expand) {
  const int w1b = expand ? 16 * ldx * 2 : 0;
  const int wdb = 16 * ((K * K + 3) / 4 * 4) * 4;
  return Ed2Slot{0, w1b, w1b + wdb, w1b + wdb + 64, w1b + wdb + 128};
}

template <int K, int TH, int TW, int R, int NT = 512>
__host__ __device__ constexpr size_t ed2_lds_bytes(int cin_pad, bool expand, int hid) {
  using G = Ed2Geom<K, TH, TW, R, NT>;
  const int ldx = cin_pad + 8;
  const size_t xs = expand ? (size_t)G::HP * ldx * 2 : 0;
  const size_t hs = (size_t)2 * 16 * G::CHP * 2;
  return xs + hs + 4 * (size_t)ed2_slot<K>(ldx, expand).bytes + (size_t)(hid + 3) / 4 * 16;
}

#ifndef ED2_PHASE_FENCE
#define ED2_PHASE_FENCE 1
#endif
#ifndef ED2_SKIP
#define ED2_SKIP 0  // experiment builds: 1 = no D store, 2 = no depthwise FMAs, 4 = no expand
#endif
template <int K, int UP, bool EXPAND, int TH, int TW, int R, int NT_>
__global__ __launch_bounds__(NT_, 4) void expand_dw2_kernel(EdArgs a) {  // 4 waves per SIMD: <= 128 VGPRs
  using G = Ed2Geom<K, TH, TW, R, NT_>;
  constexpr int NT = G::NT, IH = G::IH, IW = G::IW, IWE = G::IWE, IWP = G::IWP, CHP = G::CHP, NR = G::NR;
  constexpr int P = (K - 1) / 2;
  extern __shared__ __align__(16) unsigned char smem[];
  const int ldx = a.cin_pad + 8;
  const Ed2Slot sl = ed2_slot<K>(ldx, EXPAND);
  bf16* xs = reinterpret_cast<bf16*>(smem);
  bf16* hs = xs + (EXPAND ? G::HP * ldx : 0);                               // [2][16][CHP]
  unsigned char* ring = reinterpret_cast<unsigned char*>(hs + 2 * 16 * CHP);  // [4][slot]
  float* pool_s = reinterpret_cast<float*>(ring + 4 * sl.bytes);              // [hid] this tile's SE sums

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // image index fastest: co-resident workgroups belong to different images
  const int n = blockIdx.x % a.n;
  int b = blockIdx.x / a.n;
  const int tx = b % a.tiles_x;
  const int ty = b / a.tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 - P, ix0 = ox0 - P;
  const int64_t hw = (int64_t)a.h * a.w;
  const bf16* x1 = reinterpret_cast<const bf16*>(a.x1);
  const bf16* x2 = reinterpret_cast<const bf16*>(a.x2);
  const int nch = (a.hid + 15) / 16;

  // source offset (within a plane) of halo position (row, col) of the dw input grid
  auto src_off = [&](int row, int col) -> int {
    int gy = refl(iy0 + row, a.hd), gx = refl(ix0 + min(col, IW - 1), a.wd);
    if (UP == 2) { gy >>= 1; gx >>= 1; }
    return gy * a.w + gx;
  };

  if (EXPAND) {  // x halo tile, channel-minor: xs[p][c]; p = row * IWE + col (cols >= IW duplicate IW-1)
    const bf16* xb1 = x1 + (int64_t)n * a.c1 * hw;
    const bf16* xb2 = x2 + (int64_t)n * (a.cin - a.c1) * hw - (int64_t)a.c1 * hw;
    for (int p = tid; p < G::HP; p += NT) {
      const int pp = min(p, G::NPE - 1);
      const int off = src_off(pp / IWE, pp % IWE);
      for (int g0 = 0; g0 < a.cin_pad; g0 += 32) {  // 32 loads in flight, then four 16-byte writes
        bf16x8 v[4];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const int c = g0 + j;
          bf16 xv = (bf16)0.f;
          if (c < a.cin) xv = (c < a.c1 ? xb1 : xb2)[(int64_t)c * hw + off];
          v[j >> 3][j & 7] = xv;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (g0 + 8 * q < a.cin_pad) *reinterpret_cast<bf16x8*>(xs + p * ldx + g0 + 8 * q) = v[q];
      }
    }
  }

  // ---- parameter ring: global -> registers (set B) -> registers (set A, one iteration later, so
  // the loads' latency is a whole iteration) -> LDS slot cc % 4 ----
  constexpr int NSLOT = 4;
  const int nw1 = EXPAND ? 16 * a.cin_pad / 8 : 0;  // uint4 vectors of expand weights per chunk
  uint4 pw1B = make_uint4(0, 0, 0, 0), pw1A = pw1B;
  float pwdB = 0.f, pbB = 0.f, pwdA = 0.f, pbA = 0.f;
#define ED2_FETCH(CC)                                                                                      \
  {                                                                                                        \
    const int h0 = (CC) * 16;                                                                              \
    if (EXPAND && tid < nw1) {                                                                             \
      const int r = tid / (a.cin_pad / 8), v = tid % (a.cin_pad / 8);                                      \
      pw1B = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.w1) + (int64_t)(h0 + r) * a.cin_pad + v * 8); \
    }                                                                                                      \
    pwdB = 0.f;                                                                                            \
    if (tid < 16 * K * K && h0 + tid / (K * K) < a.hid) pwdB = a.wdw[(int64_t)h0 * K * K + tid];           \
    pbB = 0.f;                                                                                             \
    if (tid < 16) {                                                                                        \
      if (h0 + tid < a.hid) pbB = a.bdw[h0 + tid];                                                         \
    } else if (EXPAND && tid < 32) {                                                                       \
      if (h0 + tid - 16 < a.hid) pbB = a.b1[h0 + tid - 16];                                                \
    }                                                                                                      \
  }
#define ED2_STASH(CC)                                                                                      \
  {                                                                                                        \
    unsigned char* s_ = ring + ((CC) % NSLOT) * sl.bytes;                                                  \
    if (EXPAND && tid < nw1) {                                                                             \
      const int r = tid / (a.cin_pad / 8), v = tid % (a.cin_pad / 8);                                      \
      *reinterpret_cast<uint4*>(s_ + sl.w1 + (r * ldx + v * 8) * 2) = pw1A;                                \
    }                                                                                                      \
    if (tid < 16 * K * K) reinterpret_cast<float*>(s_ + sl.wd)[(tid / (K * K)) * G::KKP + tid % (K * K)] = pwdA; \
    if (tid < 16) reinterpret_cast<float*>(s_ + sl.bd)[tid] = pbA;                                         \
    else if (EXPAND && tid < 32) reinterpret_cast<float*>(s_ + sl.b1)[tid - 16] = pbA;                     \
  }
#define ED2_ROTATE() { pw1A = pw1B; pwdA = pwdB; pbA = pbB; }

  // ratio-1 blocks: the chunk's input tile straight from x (upsample + reflect), two register sets
  // like the parameters (loads consumed one iteration after they are issued)
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  constexpr int WP = EXPAND ? 1 : (G::WIN / 2 + NT - 1) / NT;  // bf16 pairs per thread
  bf16x2 rinB[WP], rinA[WP];
#define ED2_LOAD_IN(CC)                                                                                    \
  if constexpr (!EXPAND) {                                                                                 \
    _Pragma("unroll") for (int i = 0; i < WP; ++i) {                                                       \
      const int e = 2 * (tid + i * NT);                                                                    \
      bf16x2 v = {(bf16)0.f, (bf16)0.f};                                                                   \
      if (e < G::WIN) {                                                                                    \
        const int ch_ = e / (IH * IWE), rem = e % (IH * IWE), row = rem / IWE, col = rem % IWE;            \
        const int c_ = (CC) * 16 + ch_;                                                                    \
        if (c_ < a.hid) {                                                                                  \
          const bf16* xp = x1 + ((int64_t)n * a.cin + c_) * hw;                                            \
          v[0] = xp[src_off(row, col)];                                                                    \
          v[1] = xp[src_off(row, col + 1)];                                                                \
        }                                                                                                  \
      }                                                                                                    \
      rinB[i] = v;                                                                                         \
    }                                                                                                      \
  }
#define ED2_STORE_IN(BUF)                                                                                  \
  if constexpr (!EXPAND) {                                                                                 \
    _Pragma("unroll") for (int i = 0; i < WP; ++i) {                                                       \
      const int e = 2 * (tid + i * NT);                                                                    \
      if (e < G::WIN) {                                                                                    \
        const int ch_ = e / (IH * IWE), rem = e % (IH * IWE);                                              \
        *reinterpret_cast<bf16x2*>(hs + (BUF) * 16 * CHP + ch_ * CHP + (rem / IWE) * IWP + rem % IWE) = rinA[i]; \
      }                                                                                                    \
    }                                                                                                      \
  }
#define ED2_ROTATE_IN() if constexpr (!EXPAND) { _Pragma("unroll") for (int i = 0; i < WP; ++i) rinA[i] = rinB[i]; }

  // expand chunk cc into hs[buf]: this wave's tiles t = wave, wave + 8, ... (K outer, tiles inner,
  // so every tile's LDS operand reads of one K step are in flight together)
  constexpr int TPW = (G::NTILE + NT / 64 - 1) / (NT / 64);
  auto expand = [&](int cc, int buf) {
    if constexpr (EXPAND && !(ED2_SKIP & 4)) {
      const unsigned char* s_ = ring + (cc % NSLOT) * sl.bytes;
      const bf16* ws = reinterpret_cast<const bf16*>(s_ + sl.w1);
      const float bias = reinterpret_cast<const float*>(s_ + sl.b1)[lane & 15];
      f32x4 acc[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int r = lane & 15;
      int k0 = 0;
      for (; k0 + 32 <= a.cin_pad; k0 += 32) {
        const int kk = k0 + 8 * (lane >> 4);
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(ws + r * ldx + kk);
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
          const int t = wave + (NT / 64) * i;
          if (t < G::NTILE) {
            const bf16x8 fa = *reinterpret_cast<const bf16x8*>(xs + (t * 16 + r) * ldx + kk);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[i], 0, 0, 0);
          }
        }
      }
      if (k0 < a.cin_pad) {  // k = 16 tail
        typedef short s4 __attribute__((ext_vector_type(4)));
        const int kk = k0 + 4 * (lane >> 4);
        const s4 fb = *reinterpret_cast<const s4*>(ws + r * ldx + kk);
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
          const int t = wave + (NT / 64) * i;
          if (t < G::NTILE) {
            const s4 fa = *reinterpret_cast<const s4*>(xs + (t * 16 + r) * ldx + kk);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fa, fb, acc[i], 0, 0, 0);
          }
        }
      }
      bf16* hb = hs + buf * 16 * CHP + (lane & 15) * CHP;
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int t = wave + (NT / 64) * i;
        const int p0 = t * 16 + 4 * (lane >> 4);
        if (t < G::NTILE && p0 < G::NPE) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = (bf16)hswish(acc[i][j] + bias);
          *reinterpret_cast<bf16x4*>(hb + (p0 / IWE) * IWP + p0 % IWE) = o;
        }
      }
    }
  };

  // depthwise mapping: channel ch of the chunk, output rows rg*R.., columns sg*4..
  constexpr int TPC = G::TPC;
  const int ch = tid / TPC, rg = (tid % TPC) >> 3, sg = tid & 7;
  const int r0 = rg * R, c0 = sg * 4;
  const int64_t plane_o = (int64_t)a.ho * a.wo;
  const bool interior = oy0 + TH <= a.ho && ox0 + TW <= a.wo && (a.wo % 4) == 0;
  bf16* dbase = reinterpret_cast<bf16*>(a.d) + (int64_t)n * a.hid * plane_o + (int64_t)(oy0 + r0) * a.wo + ox0 + c0;

  auto depthwise = [&](int cc, int buf) {
    const int hc = cc * 16 + ch;
    if (hc >= a.hid) return;  // uniform per half-wave
    const unsigned char* s = ring + (cc % NSLOT) * sl.bytes;
    const float* wd = reinterpret_cast<const float*>(s + sl.wd) + ch * G::KKP;  // LDS broadcast reads
    const float bd = reinterpret_cast<const float*>(s + sl.bd)[ch];
    const bf16* hrow = hs + buf * 16 * CHP + ch * CHP + r0 * IWP + c0;
    typedef short s16x4v __attribute__((ext_vector_type(4)));
    float acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const s16x4v lo = *reinterpret_cast<const s16x4v*>(hrow + j * IWP);
      const s16x4v hi = *reinterpret_cast<const s16x4v*>(hrow + j * IWP + 4);
      float v[8];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        v[m] = __builtin_bit_cast(float, (unsigned)(unsigned short)lo[m] << 16);
        v[m + 4] = __builtin_bit_cast(float, (unsigned)(unsigned short)hi[m] << 16);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ky = j - r;
        if (ky >= 0 && ky < K && !(ED2_SKIP & 2)) {
          float wr[K];
#pragma unroll
          for (int kx = 0; kx < K; ++kx) wr[kx] = wd[ky * K + kx];
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(wr[kx], v[c + kx], acc[r][c]);
        }
      }
    }
    float psum = 0.f;
    bf16* drow = dbase + (int64_t)hc * plane_o;
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bf16x4 o;
      float y[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        y[c] = hswish(acc[r][c] + bd);
        o[c] = (bf16)y[c];
      }
      if (interior) {
        psum += (y[0] + y[1]) + (y[2] + y[3]);
        if (!(ED2_SKIP & 1)) *reinterpret_cast<bf16x4*>(drow + r * a.wo) = o;
      } else if (oy0 + r0 + r < a.ho) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (ox0 + c0 + c < a.wo) {
            psum += y[c];
            drow[r * a.wo + c] = o[c];
          }
      }
    }
#pragma unroll
    for (int o = TPC / 2; o > 0; o >>= 1) psum += __shfl_xor(psum, o, 64);
    if ((tid % TPC) == 0) pool_s[hc] = psum;  // each channel once per tile: stored at the end
  };

  // ---- prologue: parameters of chunks 0 and 1 in slots, chunk 2's in flight, chunk 0's image ----
  ED2_FETCH(0);
  ED2_ROTATE();
  ED2_STASH(0);
  if (nch > 1) { ED2_FETCH(1); ED2_ROTATE(); ED2_STASH(1); }
  if (nch > 2) ED2_FETCH(2);
  ED2_LOAD_IN(0);
  ED2_ROTATE_IN();
  ED2_STORE_IN(0);
  if (nch > 1) ED2_LOAD_IN(1);
  lds_barrier();  // xs, slots 0/1, (ratio-1) hs[0]
  expand(0, 0);
  lds_barrier();
  for (int c = 0; c < nch; ++c) {
    ED2_ROTATE();                       // chunk c+2's parameters (issued one iteration ago)
    ED2_ROTATE_IN();                    // ratio-1: chunk c+1's input tile
    if (c + 3 < nch) ED2_FETCH(c + 3);
    if (!EXPAND && c + 2 < nch) ED2_LOAD_IN(c + 2);
    if (c + 1 < nch) expand(c + 1, (c + 1) & 1);
    if constexpr (ED2_PHASE_FENCE) __builtin_amdgcn_sched_barrier(0);  // keeps the phases' live ranges apart
    depthwise(c, c & 1);
    if (c + 2 < nch) ED2_STASH(c + 2);
    if (c + 1 < nch) ED2_STORE_IN((c + 1) & 1);
    lds_barrier();
  }
  if (!(ED2_SKIP & 8))
    for (int c = tid; c < a.hid; c += NT) a.pool[((int64_t)n * a.hid + c) * a.slots + b] = pool_s[c];
#undef ED2_FETCH
#undef ED2_STASH
#undef ED2_ROTATE
#undef ED2_LOAD_IN
#undef ED2_STORE_IN
#undef ED2_ROTATE_IN
}

// ------------------------------------------------------------------------------------------------
// expand + depthwise, v3 (bf16, stride 1, expand blocks): the depthwise on MFMA
// ------------------------------------------------------------------------------------------------
// The v1/v2 kernels are VALU-issue-bound (PMC, k5 40->240 at 1024^2: 9.7k VALU instructions per
// wave for 1.9k depthwise FMAs per thread; two waves per SIMD at ~2 cycles each fill the wave
// lifetime). Here the kxk depthwise of one hidden channel over the 8 x 32 output tile is one set of
// 16x16x32 bf16 MFMAs (Toeplitz form):
//   M = output column xout within a 16-column half, N = (output row r, half ct) (16 pairs),
//   K = (ky, input column xin), 24 columns per ky (k*24 padded to 32-steps: 3 steps k3, 4 steps k5)
//   D[xout][(r, ct)] = sum_{ky, xin} T[xout][(ky, xin)] * H[r + ky][16 ct + xin]
//   T[xout][(ky, xin)] = w[ky][xin - xout] if 0 <= xin - xout < k, else 0.
// The B operand is two 8-byte LDS reads of the hidden image per step. The A operand (Toeplitz, per
// channel) comes from a small LDS table Z per chunk: for each (channel, ky) the weight row zero-padded
// (index 15 + kx holds w[ky][kx]) in two copies shifted by one element, so a lane's 8 consecutive
// entries start on a 4-byte boundary in one of them; windows that hold no weight read a zero block.
// Layout constants were chosen with a bank model of the gfx950 LDS (b64: 2 x 32-lane groups over 64
// banks; b32: 32 banks): the Z reads are conflict-free, the H reads within 1.5-2x of ideal.
// The expand bias is the MFMA accumulator's initial value, as is the depthwise bias. The hidden image
// is bf16 (v2's convention); all accumulation fp32.
template <int K, int NT_ = 512>
struct Ed3Geom {
  static constexpr int TH = 8, TW = 32, NT = NT_;
  static constexpr int CPW = 16 / (NT / 64);       // depthwise channels per wave per chunk
  static constexpr int IH = TH + K - 1, IW = TW + K - 1;
  static constexpr int IWE = (IW + 3) / 4 * 4;     // halo row length of the expand enumeration (36)
  static constexpr int NPE = IH * IWE;
  static constexpr int HP = (NPE + 15) / 16 * 16;  // expand pixels, MFMA tiles of 16
  static constexpr int NTILE = HP / 16;
  static constexpr int TPW = (NTILE + NT / 64 - 1) / (NT / 64);  // expand tiles per wave
  static constexpr int IWP = 44;                   // hidden row pitch (bf16); columns [IWE, 40) stay zero
  // hidden channel pitch (bf16): room for the last expand tile's overhang past the halo (HP - NPE
  // elements after row IH-1), and pitch/4 odd so the expand's 8-byte writes (16 lanes = 16 channels)
  // hit 16 distinct bank pairs
  static constexpr int CHP0 = IH * IWP + (HP - NPE);
  static constexpr int CHP = CHP0 + ((CHP0 / 4) % 2 == 0 ? 4 : 8);
  static constexpr int KSEG = 24;                  // K columns per ky
  static constexpr int KSTEPS = (K * KSEG + 31) / 32;
  static constexpr int ZWC = K == 5 ? 9 : 8;       // words per shifted copy
  static constexpr int ZROW = K == 5 ? 21 : 17;    // words per (channel, ky)
  static constexpr int ZZERO = K == 5 ? 112 : 51;  // offset of a channel's 4 zero words
  static constexpr int ZCH = ZZERO + 4;            // words per channel
  static constexpr int ZSLOT = 16 * ZCH;           // words per chunk
  static_assert(IWE + 4 <= 40 && 40 <= IWP, "B reads reach column 16 + 16 + 7");
  static_assert((14 + K - 8) / 2 + 4 <= ZWC && 2 * ZWC <= ZROW && K * ZROW <= ZZERO, "Z table");
};

struct Ed3Lds {  // byte offsets; every block parameter is resident for the whole tile
  size_t xs, hs, w1, b1, bd, wd, z, pool, total;
};
template <int K>
__host__ __device__ constexpr Ed3Lds ed3_lds(int cin_pad, int hid) {
  using G = Ed3Geom<K>;  // (the LDS layout does not depend on the workgroup size)
  const size_t ldx = cin_pad + 8, hp = (size_t)(hid + 15) / 16 * 16;
  Ed3Lds l{};
  l.xs = 0;
  l.hs = (size_t)G::HP * ldx * 2;
  l.w1 = l.hs + (size_t)2 * 16 * G::CHP * 2;
  l.b1 = l.w1 + hp * ldx * 2;
  l.bd = l.b1 + hp * 4;
  l.wd = l.bd + hp * 4;
  l.z = l.wd + (hp * K * K * 2 + 15) / 16 * 16;
  l.pool = l.z + (size_t)2 * G::ZSLOT * 4;
  l.total = l.pool + hp * 4;
  return l;
}

__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, (bf16)v);
}

// Sum over each 16-lane row by DPP (no LDS round trips): every lane ends with its row's sum.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum_dpp(float v) {
  v += dpp_f<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  return v;
}

template <int K, int NT_, int OCC>
__global__ __launch_bounds__(NT_, OCC) void expand_dw3_kernel(EdArgs a) {
  using G = Ed3Geom<K, NT_>;
  constexpr int CPW = G::CPW;
  constexpr int NT = G::NT, IWE = G::IWE, IWP = G::IWP, CHP = G::CHP, KSTEPS = G::KSTEPS, TPW = G::TPW;
  constexpr int P = (K - 1) / 2;
  extern __shared__ __align__(16) unsigned char smem[];
  const int ldx = a.cin_pad + 8;
  const int hp = (a.hid + 15) / 16 * 16;
  const Ed3Lds L = ed3_lds<K>(a.cin_pad, a.hid);
  bf16* xs = reinterpret_cast<bf16*>(smem + L.xs);
  bf16* hs = reinterpret_cast<bf16*>(smem + L.hs);  // [2][16][CHP]
  bf16* w1s = reinterpret_cast<bf16*>(smem + L.w1);  // [hp][ldx]
  float* b1s = reinterpret_cast<float*>(smem + L.b1);
  float* bds = reinterpret_cast<float*>(smem + L.bd);
  unsigned short* wds = reinterpret_cast<unsigned short*>(smem + L.wd);  // bf16 [hp][K*K]
  unsigned* zt = reinterpret_cast<unsigned*>(smem + L.z);               // [2][16][ZCH]
  float* pool_s = reinterpret_cast<float*>(smem + L.pool);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.x % a.n;  // image fastest
  const int b = blockIdx.x / a.n;
  const int tx = b % a.tiles_x, ty = b / a.tiles_x;
  const int oy0 = ty * G::TH, ox0 = tx * G::TW;
  const int iy0 = oy0 - P, ix0 = ox0 - P;
  const int64_t hw = (int64_t)a.h * a.w;
  const bf16* x1 = reinterpret_cast<const bf16*>(a.x1);
  const bf16* x2 = reinterpret_cast<const bf16*>(a.x2);
  const int nch = hp / 16;

  // ---- prologue: all parameters and the x halo tile into LDS; zero Z and hs columns [IWE, 40) ----
  {
    const int vpr = a.cin_pad / 8;  // 16-byte vectors per expand-weight row
    const uint4* w1g = reinterpret_cast<const uint4*>(a.w1);
    for (int i = tid; i < hp * vpr; i += NT) {
      const int r = i / vpr, v = i - r * vpr;
      *reinterpret_cast<uint4*>(w1s + r * ldx + v * 8) = w1g[i];
    }
    for (int i = tid; i < hp; i += NT) {
      b1s[i] = i < a.hid ? a.b1[i] : 0.f;
      bds[i] = i < a.hid ? a.bdw[i] : 0.f;
      pool_s[i] = 0.f;
    }
    for (int i = tid; i < hp * K * K; i += NT) wds[i] = i < a.hid * K * K ? bf16_bits(a.wdw[i]) : (unsigned short)0;
    for (int i = tid; i < 2 * G::ZSLOT; i += NT) zt[i] = 0u;
    for (int i = tid; i < 2 * 16 * G::IH; i += NT) {
      unsigned* p = reinterpret_cast<unsigned*>(hs + (i / G::IH) * CHP + (i % G::IH) * IWP + IWE);
#pragma unroll
      for (int q = 0; q < (40 - IWE) / 2; ++q) p[q] = 0u;
    }
    // x halo tile, channel-minor: xs[p][c]; p = row * IWE + col (cols >= IW duplicate IW-1)
    const bf16* xb1 = x1 + (int64_t)n * a.c1 * hw;
    const bf16* xb2 = x2 + (int64_t)n * (a.cin - a.c1) * hw - (int64_t)a.c1 * hw;
    for (int p = tid; p < G::HP; p += NT) {
      const int pp = min(p, G::NPE - 1);
      const int gy = refl(iy0 + pp / IWE, a.hd), gx = refl(ix0 + min(pp % IWE, G::IW - 1), a.wd);
      const int off = gy * a.w + gx;
      for (int g0 = 0; g0 < a.cin_pad; g0 += 32) {
        bf16x8 v[4];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const int c = g0 + j;
          bf16 xv = (bf16)0.f;
          if (c < a.cin) xv = (c < a.c1 ? xb1 : xb2)[(int64_t)c * hw + off];
          v[j >> 3][j & 7] = xv;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (g0 + 8 * q < a.cin_pad) *reinterpret_cast<bf16x8*>(xs + p * ldx + g0 + 8 * q) = v[q];
      }
    }
  }

  // Toeplitz weights of chunk cc into Z slot cc & 1 (only the weight positions; the rest stays zero)
  const int zch = tid / (K * K), zky = (tid % (K * K)) / K, zkx = tid % K;
  unsigned short* zw = reinterpret_cast<unsigned short*>(zt + zch * G::ZCH + zky * G::ZROW) + 7 + zkx;
  auto build_z = [&](int cc) {
    if (tid < 16 * K * K) {
      const unsigned short wb = wds[cc * 16 * K * K + tid];
      unsigned short* z_ = zw + (cc & 1) * G::ZSLOT * 2;
      z_[0] = wb;                   // copy 0: element 15 + kx - 8
      z_[2 * G::ZWC - 1] = wb;      // copy 1: element 15 + kx - 9
    }
  };

  // expand: per-lane LDS offsets, fixed over chunks. A wave past the last halo tile recomputes it
  // and rewrites the same values (no branch); pixel groups past the halo land in the channel pitch's
  // overhang.
  const int r16 = lane & 15, q4 = lane >> 4;
  int xoff[TPW], hoff[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = min(wave + (NT / 64) * i, G::NTILE - 1);
    xoff[i] = (t * 16 + r16) * ldx;
    const int p0 = t * 16 + 4 * q4;
    hoff[i] = r16 * CHP + (p0 / IWE) * IWP + p0 % IWE;
  }
  typedef short s4 __attribute__((ext_vector_type(4)));
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  auto expand = [&](int cc, bf16* hbuf) {
    const bf16* ws = w1s + cc * 16 * ldx + r16 * ldx;
    const float bias = b1s[cc * 16 + r16];
    f32x4 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x4{bias, bias, bias, bias};
    int k0 = 0;
    for (; k0 + 32 <= a.cin_pad; k0 += 32) {
      const int kk = k0 + 8 * q4;
      const bf16x8 fb = *reinterpret_cast<const bf16x8*>(ws + kk);
      bf16x8 fa[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(xs + xoff[i] + kk);
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i], 0, 0, 0);
    }
    if (k0 < a.cin_pad) {  // k = 16 tail
      const int kk = k0 + 4 * q4;
      const s4 fb = *reinterpret_cast<const s4*>(ws + kk);
      s4 fa[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) fa[i] = *reinterpret_cast<const s4*>(xs + xoff[i] + kk);
#pragma unroll
      for (int i = 0; i < TPW; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fa[i], fb, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)hswish(acc[i][j]);
      *reinterpret_cast<bf16x4*>(hbuf + hoff[i]) = o;
    }
  };

  // depthwise: per-lane operand offsets of the MFMA steps (constant over channels and chunks)
  const int r_ = r16 >> 1, ct_ = r16 & 1;  // this lane's N index (as a B column) -> (row, half)
  int zoff[KSTEPS], boff[KSTEPS];
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) {
    const int k0 = 32 * s + 8 * q4, ky = k0 / G::KSEG, x0 = k0 % G::KSEG;
    const int o = x0 - r16 + 15;  // window start in the zero-padded weight row
    const int c = o & 1;
    zoff[s] = (ky < K && o >= 8 && o <= 14 + K) ? ky * G::ZROW + c * G::ZWC + (o - 8 - c) / 2 : G::ZZERO;
    boff[s] = (r_ + min(ky, K - 1)) * IWP + 16 * ct_ + x0;
  }
  const int64_t plane_o = (int64_t)a.ho * a.wo;
  const int orow = oy0 + r_, ocol = ox0 + 16 * ct_ + 4 * q4;  // this lane's 4 outputs (C[m][n] layout)
  const bool interior = oy0 + G::TH <= a.ho && ox0 + G::TW <= a.wo && (a.wo % 4) == 0;
  bf16* dbase = reinterpret_cast<bf16*>(a.d) + (int64_t)n * a.hid * plane_o + (int64_t)orow * a.wo + ocol;

  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  auto depthwise = [&](int cc, const bf16* hbuf) {
    // CPW channels per wave; every operand read issued before the MFMA chains
    u32x4 av[CPW][KSTEPS], bv[CPW][KSTEPS];
#pragma unroll
    for (int cw = 0; cw < CPW; ++cw) {
      const int ch = wave * CPW + cw;
      const unsigned* zc = zt + (cc & 1) * G::ZSLOT + ch * G::ZCH;
      const bf16* himg = hbuf + ch * CHP;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const unsigned* zp = zc + zoff[s];
        av[cw][s] = u32x4{zp[0], zp[1], zp[2], zp[3]};
        const u32x2 b0 = *reinterpret_cast<const u32x2*>(himg + boff[s]);
        const u32x2 b1 = *reinterpret_cast<const u32x2*>(himg + boff[s] + 4);
        bv[cw][s] = u32x4{b0[0], b0[1], b1[0], b1[1]};
      }
    }
    f32x4 acc[CPW];
#pragma unroll
    for (int cw = 0; cw < CPW; ++cw) {
      const float bd = bds[cc * 16 + wave * CPW + cw];
      acc[cw] = f32x4{bd, bd, bd, bd};
    }
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
      for (int cw = 0; cw < CPW; ++cw)
        acc[cw] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[cw][s]),
                                                          __builtin_bit_cast(bf16x8, bv[cw][s]), acc[cw], 0, 0, 0);
#pragma unroll
    for (int cw = 0; cw < CPW; ++cw) {
      const int hc = cc * 16 + wave * CPW + cw;
      if (hc >= a.hid) break;  // wave-uniform (the padded tail of the last chunk)
      float y[4], psum;
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = hswish(acc[cw][j]);
      bf16* drow = dbase + (int64_t)hc * plane_o;
      if (interior) {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)y[j];
        psum = (y[0] + y[1]) + (y[2] + y[3]);
        *reinterpret_cast<bf16x4*>(drow) = o;
      } else {
        psum = 0.f;
        if (orow < a.ho) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (ocol + j < a.wo) {
              psum += y[j];
              drow[j] = (bf16)y[j];
            }
        }
      }
      psum = row_sum_dpp(psum);  // every lane: its 16-lane row's sum
      // the wave's four rows in a fixed order (this wave alone owns channel hc of the tile)
      psum = (__shfl(psum, 0, 64) + __shfl(psum, 16, 64)) + (__shfl(psum, 32, 64) + __shfl(psum, 48, 64));
      if (lane == 0) pool_s[hc] = psum;
    }
  };

  bf16* const hs0 = hs;
  bf16* const hs1 = hs + 16 * CHP;
  lds_barrier();  // parameters, xs, zeroed Z and pool
  build_z(0);
  expand(0, hs0);
  lds_barrier();
  // two chunks per trip so the hidden-image buffers are fixed addresses
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) {
      build_z(c + 1);
      expand(c + 1, hs1);
    }
    __builtin_amdgcn_sched_barrier(0);
    depthwise(c, hs0);
    lds_barrier();
    if (c + 1 >= nch) break;
    if (c + 2 < nch) {
      build_z(c + 2);
      expand(c + 2, hs0);
    }
    __builtin_amdgcn_sched_barrier(0);
    depthwise(c + 1, hs1);
    lds_barrier();
  }
  for (int c = tid; c < a.hid; c += NT) a.pool[((int64_t)n * a.hid + c) * a.slots + b] = pool_s[c];
}

// ------------------------------------------------------------------------------------------------
// SE MLP + gate folding into the pw-linear weights
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads) void se_fold_kernel(const float* __restrict__ pool, int hid, float hw,
                                                           const float* __restrict__ fc1w,
                                                           const float* __restrict__ fc1b, int red,
                                                           const float* __restrict__ fc2w,
                                                           const float* __restrict__ fc2b,
                                                           const float* __restrict__ w2, int cout, int cout_pad,
                                                           int hid_pad, T* __restrict__ wg) {
  extern __shared__ float sm[];
  float* mean = sm;          // [hid]
  float* hmid = sm + hid;    // [red]
  float* gate = hmid + red;  // [hid]
  const int n = blockIdx.x;
  for (int c = threadIdx.x; c < hid; c += kThreads) mean[c] = pool[(int64_t)n * hid + c] / hw;
  __syncthreads();
  // FC1 / FC2: one thread per output, the sum in channel order; unrolled so that 8 weight loads are in
  // flight at a time (a load-use chain per channel left each launch ~50 us of L2 latency)
  for (int j = threadIdx.x; j < red; j += kThreads) {
    float s = fc1b[j];
#pragma unroll 8
    for (int c = 0; c < hid; ++c) s = fmaf(fc1w[(int64_t)j * hid + c], mean[c], s);
    hmid[j] = fmaxf(s, 0.f);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < hid; c += kThreads) {
    float s = fc2b[c];
#pragma unroll 8
    for (int j = 0; j < red; ++j) s = fmaf(fc2w[(int64_t)c * red + j], hmid[j], s);
    gate[c] = fminf(fmaxf(s, 0.f), 1.f);
  }
  __syncthreads();
  // the gated weights row by row: a wave per output channel, lanes along the hidden channels (the
  // flat form paid an integer division per element: ~75 us per launch, 46 launches per config-5 step)
  T* o = wg + (int64_t)n * cout_pad * hid_pad;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int co = wv; co < cout_pad; co += kThreads / 64) {
    const float* wr = w2 + (int64_t)co * hid;
    T* orow = o + (int64_t)co * hid_pad;
    for (int c = lane; c < hid_pad; c += 64) orow[c] = from_f<T>(co < cout && c < hid ? wr[c] * gate[c] : 0.f);
  }
}

// ------------------------------------------------------------------------------------------------
// pointwise GEMM: out[n][co][p] = sum_c Wg[n][co][c] * D[n][c][p] + b[co] (+ res)
// ------------------------------------------------------------------------------------------------
struct PwArgs {
  const void* d;
  int n, hid, hid_pad, h, w;
  const void* wg;
  int64_t wg_stride;  // elements between images' weight sets (0: shared)
  const float* bias;
  int cout, cout_pad;
  const void* res;  // [n][cout][h][w], or [n][cout][h/2][w/2] with res_up
  int res_up;
  void* out;
  int tiles;
  // expand-as-GEMM use (ast_mb_expand_gemm): K channels [c1, hid) come from d2 (the un-materialised
  // torch.cat), act = 1 applies Hardswish; output channels in slices of MT*16 over gridDim.y
  const void* d2;
  int c1;
  int act;
};

constexpr int kPwPx = 256;  // pixels per workgroup (4 waves x 64)
#ifndef PW_PX_BF16
#define PW_PX_BF16 256  // bf16 pw with <= 48 output channels: pixels per workgroup (256 | 512)
#endif
constexpr int kPwK = 32;    // hidden channels per LDS stage

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// D is staged in its natural [channel][pixel] layout (16-byte writes, global loads coalesced along
// pixels). bf16: the 16x16x32 B operand wants 8 channels of one pixel per lane, which the gfx950
// transposed read ds_read_b64_tr_b16 delivers from that layout; the MFMA k order is permuted to
// (4g..4g+3, 16+4g..16+4g+3) for lane group g (A uses the same order), so each half-wave's read
// touches 8 consecutive rows, conflict-free with a row pitch of 16 (mod 128) elements.
template <typename T, int MT, int PX = kPwPx>
__global__ __launch_bounds__(kThreads, 2) void pw_kernel(PwArgs a) {
  constexpr int TT = PX / 64;  // 16-pixel MFMA tiles per wave
  constexpr bool BF = sizeof(T) == 2;
  constexpr int LDP = PX + (BF ? 16 : 4);     // D image row pitch (elements)
  constexpr int LDW = kPwK + Mma<T>::PAD;        // weight image row pitch
  constexpr int VEC = 16 / sizeof(T);            // elements per 16-byte vector
  constexpr int NV = kPwK * PX / VEC / kThreads;
  constexpr int VPR = PX / VEC;               // vectors per channel row
  __shared__ __align__(16) T ds[kPwK * LDP];
  __shared__ __align__(16) T ws[MT * 16 * LDW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.x / a.tiles;
  const int64_t p0 = (int64_t)(blockIdx.x % a.tiles) * PX;
  const int64_t hw = (int64_t)a.h * a.w;
  const int co0 = blockIdx.y * MT * 16;  // output-channel slice (0 for the pw-linear launches)
  const int cout_l = min(a.cout - co0, MT * 16);
  // K channel kc of image n: d[n][kc] for kc < c1, else d2[n][kc - c1]
  const T* dn = reinterpret_cast<const T*>(a.d) + (int64_t)n * a.c1 * hw;
  const T* dn2 = reinterpret_cast<const T*>(a.d2) + (int64_t)n * (a.hid - a.c1) * hw - (int64_t)a.c1 * hw;
  const T* wn = reinterpret_cast<const T*>(a.wg) + (int64_t)n * a.wg_stride + (int64_t)co0 * a.hid_pad;
  const bool vec = (hw % VEC) == 0 && p0 + PX <= hw;

  constexpr int WV = (MT * 16 * kPwK / VEC + kThreads - 1) / kThreads;
  uint4 pre[NV];  // next chunk of D, prefetched into registers
  uint4 prw[WV];  // and of the weights
  // (a macro, not a lambda, and no address-taken temporaries: both sent these arrays to scratch)
#define PW_FETCH(K0)                                                                                       \
  {                                                                                                        \
    const int kb = (K0);                                                                                   \
    _Pragma("unroll") for (int i = 0; i < NV; ++i) {                                                       \
      const int e = tid + i * kThreads, c = e / VPR, q = (e % VPR) * VEC;                                  \
      uint4 val = make_uint4(0, 0, 0, 0);                                                                  \
      if (vec) {                                                                                           \
        if (kb + c < a.hid) val = *reinterpret_cast<const uint4*>((kb + c < a.c1 ? dn : dn2) + (int64_t)(kb + c) * hw + p0 + q); \
      } else {                                                                                             \
        typename VecOf<T, VEC>::type tv;                                                                   \
        _Pragma("unroll") for (int j = 0; j < VEC; ++j) {                                                  \
          T x = from_f<T>(0.f);                                                                            \
          if (kb + c < a.hid && p0 + q + j < hw) x = (kb + c < a.c1 ? dn : dn2)[(int64_t)(kb + c) * hw + p0 + q + j]; \
          tv[j] = x;                                                                                       \
        }                                                                                                  \
        val = __builtin_bit_cast(uint4, tv);                                                               \
      }                                                                                                    \
      pre[i] = val;                                                                                        \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < WV; ++i) {                                                       \
      const int e = tid + i * kThreads, r = e / (kPwK / VEC), v = e % (kPwK / VEC);                        \
      uint4 val = make_uint4(0, 0, 0, 0);                                                                  \
      if (e < MT * 16 * kPwK / VEC) val = *reinterpret_cast<const uint4*>(wn + (int64_t)r * a.hid_pad + kb + v * VEC); \
      prw[i] = val;                                                                                        \
    }                                                                                                      \
  }

  f32x4 acc[MT][TT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < TT; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  PW_FETCH(0);
  for (int k0 = 0; k0 < a.hid_pad; k0 += kPwK) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + i * kThreads, c = e / VPR, q = (e % VPR) * VEC;
      *reinterpret_cast<uint4*>(ds + c * LDP + q) = pre[i];
    }
#pragma unroll
    for (int i = 0; i < WV; ++i) {
      const int e = tid + i * kThreads, r = e / (kPwK / VEC), v = e % (kPwK / VEC);
      if (e < MT * 16 * kPwK / VEC) *reinterpret_cast<uint4*>(ws + r * LDW + v * VEC) = prw[i];
    }
    lds_barrier();
    if (k0 + kPwK < a.hid_pad) PW_FETCH(k0 + kPwK);  // in flight during the MFMAs and across the barrier
    if constexpr (BF) {
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
      bf16x8 bfr[TT];
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const int col = wave * (PX / 4) + t * 16 + 4 * p;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ds + (4 * g + q) * LDP + col));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ds + (16 + 4 * g + q) * LDP + col));
        bfr[t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const T* wr = ws + (m * 16 + (lane & 15)) * LDW + 4 * g;
        const s16x4 lo = *reinterpret_cast<const s16x4*>(wr);
        const s16x4 hi = *reinterpret_cast<const s16x4*>(wr + 16);
        const bf16x8 afr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[t], acc[m][t], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < kPwK; ks += 4) {
        const int kr = ks + (lane >> 4);
        float bfr[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) bfr[t] = ds[kr * LDP + wave * (PX / 4) + t * 16 + (lane & 15)];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const float afr = ws[(m * 16 + (lane & 15)) * LDW + kr];
#pragma unroll
          for (int t = 0; t < TT; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(afr, bfr[t], acc[m][t], 0, 0, 0);
        }
      }
    }
    lds_barrier();
  }

  T* out = reinterpret_cast<T*>(a.out) + ((int64_t)n * a.cout + co0) * hw;
  const T* res = reinterpret_cast<const T*>(a.res);
  const float* bias = a.bias ? a.bias + co0 : nullptr;
  if constexpr (BF) {
    // Whole tile, no upsampled residual: the accumulators go through LDS (16 output channels at a
    // time, fp32, row pitch 260 floats: conflict-free) so every lane stores 8 consecutive pixels
    // with one 16-byte write (the direct epilogue's 2-byte stores cover 32-byte runs only).
    constexpr int EP = PX + 4;
    static_assert(16 * EP * sizeof(float) <= sizeof(ds), "epilogue staging fits the D image");
    if (vec && (hw % 8) == 0 && (!a.res_up || (a.w % 8) == 0)) {
      float* st = reinterpret_cast<float*>(ds);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (m * 16 >= cout_l) break;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int t = 0; t < TT; ++t) st[(4 * (lane >> 4) + r) * EP + wave * (PX / 4) + t * 16 + (lane & 15)] = acc[m][t][r];
        lds_barrier();
#pragma unroll
        for (int i = 0; i < 2 * PX / 256; ++i) {
          const int e = tid + i * kThreads, row = e / (PX / 8), q = (e % (PX / 8)) * 8;  // 16 rows x PX/8 vectors
          const int co = m * 16 + row;
          if (co < cout_l) {
            const f32x4 v0 = *reinterpret_cast<const f32x4*>(st + row * EP + q);
            const f32x4 v1 = *reinterpret_cast<const f32x4*>(st + row * EP + q + 4);
            const float bco = bias ? bias[co] : 0.f;
            float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
            const int64_t off = (int64_t)co * hw + p0 + q;
            if (res && a.res_up) {  // nearest x2 residual: 4 source pixels, each used twice
              const int pix = (int)(p0 + q), y = pix / a.w, x = pix - y * a.w;
              const int hr = a.h / 2, wr = a.w / 2;
              const uint2 rv = *reinterpret_cast<const uint2*>(
                  res + (((int64_t)n * a.cout + co0 + co) * hr + (y >> 1)) * wr + (x >> 1));
              typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
              const bf16x4v rb = __builtin_bit_cast(bf16x4v, rv);
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = v[j] + bco + to_f(rb[j >> 1]);
            } else if (res) {
              const uint4 rv = *reinterpret_cast<const uint4*>(res + ((int64_t)n * a.cout + co0) * hw + off);
              const bf16x8 rb = __builtin_bit_cast(bf16x8, rv);
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = v[j] + bco + to_f(rb[j]);
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += bco;
            }
            if (a.act) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = hswish(v[j]);
            }
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = from_f<T>(v[j]);
            *reinterpret_cast<uint4*>(out + off) = __builtin_bit_cast(uint4, o);
          }
        }
        lds_barrier();
      }
      return;
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m * 16 + 4 * (lane >> 4) + r;
      if (co >= cout_l) continue;
      const float bco = bias ? bias[co] : 0.f;
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const int64_t p = p0 + wave * (PX / 4) + t * 16 + (lane & 15);
        if (p >= hw) continue;
        float v = acc[m][t][r] + bco;
        if (res) {
          if (a.res_up) {
            const int pi = (int)p, y = pi / a.w, x = pi - y * a.w;  // p < h*w < 2^31 (host-checked)
            const int hr = a.h / 2, wr = a.w / 2;
            v += to_f(res[(((int64_t)n * a.cout + co0 + co) * hr + (y >> 1)) * wr + (x >> 1)]);
          } else {
            v += to_f(res[((int64_t)n * a.cout + co0 + co) * hw + p]);
          }
        }
        if (a.act) v = hswish(v);
        out[(int64_t)co * hw + p] = from_f<T>(v);
      }
    }
}

#undef PW_FETCH

// ------------------------------------------------------------------------------------------------
// dense 3x3 reflect conv with few channels (block 0: 3->16 + Hardswish; decoder out: 16->3 + bias)
// ------------------------------------------------------------------------------------------------
template <typename TI, typename TO, int CIN, int COUT, int ACT>
__global__ __launch_bounds__(kThreads) void dense3x3_kernel(const TI* __restrict__ x, const float* __restrict__ wt,
                                                            const float* __restrict__ bias, TO* __restrict__ y,
                                                            int h, int w, int64_t groups_per_image,
                                                            int64_t total) {
  __shared__ float wsm[COUT * CIN * 9];
  for (int i = threadIdx.x; i < COUT * CIN * 9; i += kThreads) wsm[i] = wt[i];
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;  // 4-pixel group
  if (g >= total) return;
  const int64_t n = g / groups_per_image;
  const int64_t gi = g - n * groups_per_image;
  const int gpr = (w + 3) / 4;
  const int oy = (int)(gi / gpr), ox0 = (int)(gi % gpr) * 4;
  if (oy >= h) return;
  const int64_t hw = (int64_t)h * w;
  float acc[COUT][4];
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[co][q] = bias ? bias[co] : 0.f;
  int xs[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) xs[m] = refl(ox0 - 1 + m, w);
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
    const TI* xp = x + (n * CIN + ci) * hw;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const TI* row = xp + (int64_t)refl(oy - 1 + ky, h) * w;
      float v[6];
#pragma unroll
      for (int m = 0; m < 6; ++m) v[m] = to_f(row[xs[m]]);
#pragma unroll
      for (int co = 0; co < COUT; ++co)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float wv = wsm[((co * CIN + ci) * 3 + ky) * 3 + kx];
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[co][q] = fmaf(wv, v[q + kx], acc[co][q]);
        }
    }
  }
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    TO* o = y + (n * COUT + co) * hw + (int64_t)oy * w + ox0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (ox0 + q < w) {
        float v = acc[co][q];
        if (ACT == 1) v = hswish(v);
        if (ACT == 2) v = fminf(fmaxf(v, 0.f), 1.f);
        o[q] = from_f<TO>(v);
      }
    }
  }
}

// 8 output pixels per thread for rows whose width is a multiple of 8: the 8 centre inputs of a tap
// row are one 16-byte (bf16) or two 16-byte (fp32) loads, the two neighbours scalar loads (with the
// reflection at the image borders), and each output channel leaves as 16-byte stores -- the 4-pixel
// kernel above issues ~8x more memory instructions per pixel (config 5: 1.1-1.6 TB/s).
template <typename T>
__device__ __forceinline__ void load8f(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
  } else {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

template <typename TI, typename TO, int CIN, int COUT_ALL, int ACT, int CB = COUT_ALL>
__global__ __launch_bounds__(kThreads) void dense3x3v8_kernel(const TI* __restrict__ x, const float* __restrict__ wt,
                                                              const float* __restrict__ bias, TO* __restrict__ y,
                                                              int h, int w, int64_t groups_per_image, int64_t total) {
  // CB output channels per thread: blockIdx.y selects the block of channels (block 0's 16 channels
  // as two blocks of 8 keep the accumulators at 64 registers)
  constexpr int COUT = CB;
  __shared__ float wsm[COUT * CIN * 9];
  const int cb0 = blockIdx.y * CB;
  for (int i = threadIdx.x; i < COUT * CIN * 9; i += kThreads) wsm[i] = wt[cb0 * CIN * 9 + i];
  __syncthreads();
  if (bias) bias += cb0;
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;  // 8-pixel group
  if (g >= total) return;
  const int64_t n = g / groups_per_image;
  const int64_t gi = g - n * groups_per_image;
  const int gpr = w / 8;
  const int oy = (int)(gi / gpr), ox0 = (int)(gi % gpr) * 8;
  const int64_t hw = (int64_t)h * w;
  float acc[COUT][8];
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[co][q] = bias ? bias[co] : 0.f;
  const int xl = refl(ox0 - 1, w), xr = refl(ox0 + 8, w);
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
    const TI* xp = x + (n * CIN + ci) * hw;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const TI* row = xp + (int64_t)refl(oy - 1 + ky, h) * w;
      float v[10];
      load8f(row + ox0, v + 1);
      v[0] = to_f(row[xl]);
      v[9] = to_f(row[xr]);
#pragma unroll
      for (int co = 0; co < COUT; ++co)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float wv = wsm[((co * CIN + ci) * 3 + ky) * 3 + kx];
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[co][q] = fmaf(wv, v[q + kx], acc[co][q]);
        }
    }
  }
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    TO* o = y + (n * COUT_ALL + cb0 + co) * hw + (int64_t)oy * w + ox0;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[q] = acc[co][q];
      if (ACT == 1) v[q] = hswish(v[q]);
      if (ACT == 2) v[q] = fminf(fmaxf(v[q], 0.f), 1.f);
    }
    if constexpr (sizeof(TO) == 2) {
      bf16x8 ob;
#pragma unroll
      for (int q = 0; q < 8; ++q) ob[q] = (bf16)v[q];
      *reinterpret_cast<bf16x8*>(o) = ob;
    } else {
      reinterpret_cast<float4*>(o)[0] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(o)[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// AdaIN on bf16 maps (fp32 statistics), models.py:43-51 (+ alpha blend, models.py:471)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float block_sum256(float v, float* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

__device__ __forceinline__ void plane_stats_bf16(const bf16* p, int64_t n, float* sh, float& mean, float& sd) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) s += (float)p[i];
  mean = block_sum256(s, sh) / (float)n;
  float q = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) {
    const float d = (float)p[i] - mean;
    q += d * d;
  }
  sd = sqrtf(block_sum256(q, sh) / (float)(n - 1));
}

__global__ __launch_bounds__(kThreads) void adain_bf16_kernel(const bf16* __restrict__ content,
                                                              const bf16* __restrict__ style, bf16* __restrict__ out,
                                                              int64_t hwc, int64_t hws, float alpha, float beta,
                                                              int swap) {
  __shared__ float sh[4];
  const int64_t p = blockIdx.x;
  const bf16* c = content + p * hwc;
  float ms, ss, mc, sc;
  plane_stats_bf16(style + p * hws, hws, sh, ms, ss);
  plane_stats_bf16(c, hwc, sh, mc, sc);
  const float scale = swap ? ms : ss, shift = swap ? ss : ms;
  bf16* o = out + p * hwc;
  for (int64_t i = threadIdx.x; i < hwc; i += kThreads) {
    const float v = (float)c[i];
    o[i] = (bf16)(alpha * ((v - mc) / sc * scale + shift) + beta * v);
  }
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
constexpr size_t kLdsBudget = 80 * 1024;      // two workgroups per CU
constexpr size_t kLdsBudgetMax = 150 * 1024;  // one workgroup per CU

template <typename T, int K, int S, int UP, bool EXPAND, int TH, int TW>
int launch_ed_th(EdArgs a, hipStream_t st) {
  using G = EdGeom<K, S, TH, TW>;
  a.tiles_x = (a.wo + G::TW - 1) / G::TW;
  a.tiles_y = (a.ho + TH - 1) / TH;
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.n;
  if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
  if (ed_plan(a, (int64_t)a.tiles_x * a.tiles_y)) return 0;
  const size_t lds = ed_lds_bytes<T, K, S, TH, TW>(a.cin_pad, EXPAND);
  auto kern = expand_dw_kernel<T, K, S, UP, EXPAND, TH, TW>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), lds, st, a);
  return (int)hipGetLastError();
}

int g_ed_th = 0;  // AST_MB_ED_TH=16|4|2 sets the v1 tile height (A/B measurements)

template <typename T, int K, int S, int UP, bool EXPAND>
int launch_ed(EdArgs a, hipStream_t st) {
  constexpr int TW = S == 1 ? 32 : 16;  // output tile width; 8/4/2 rows as LDS allows
  if (g_ed_th == 16 && ed_lds_bytes<T, K, S, 16, TW>(a.cin_pad, EXPAND) <= kLdsBudgetMax)
    return launch_ed_th<T, K, S, UP, EXPAND, 16, TW>(a, st);
  if (g_ed_th == 4 && ed_lds_bytes<T, K, S, 4, TW>(a.cin_pad, EXPAND) <= kLdsBudget)
    return launch_ed_th<T, K, S, UP, EXPAND, 4, TW>(a, st);
  if (g_ed_th == 2 && ed_lds_bytes<T, K, S, 2, TW>(a.cin_pad, EXPAND) <= kLdsBudget)
    return launch_ed_th<T, K, S, UP, EXPAND, 2, TW>(a, st);
  if (ed_lds_bytes<T, K, S, 8, TW>(a.cin_pad, EXPAND) <= kLdsBudget)
    return launch_ed_th<T, K, S, UP, EXPAND, 8, TW>(a, st);
  if (ed_lds_bytes<T, K, S, 4, TW>(a.cin_pad, EXPAND) <= kLdsBudget)
    return launch_ed_th<T, K, S, UP, EXPAND, 4, TW>(a, st);
  if (ed_lds_bytes<T, K, S, 2, TW>(a.cin_pad, EXPAND) <= kLdsBudgetMax)
    return launch_ed_th<T, K, S, UP, EXPAND, 2, TW>(a, st);
  if (S == 1 && ed_lds_bytes<T, K, S, 2, 16>(a.cin_pad, EXPAND) <= kLdsBudgetMax)  // wide fp32 inputs (ada_out)
    return launch_ed_th<T, K, S, UP, EXPAND, 2, 16>(a, st);
  return AST_E_UNSUPPORTED;
}

int g_ed_big = 1;  // AST_MB_ED_BIG=0 disables the 16-wave tile (A/B measurements)

template <int K, int UP, bool EXPAND, int TH, int TW, int R, int NT = 512>
int launch_ed2(EdArgs a, hipStream_t st) {
  a.tiles_x = (a.wo + TW - 1) / TW;
  a.tiles_y = (a.ho + TH - 1) / TH;
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.n;
  if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
  if (ed_plan(a, (int64_t)a.tiles_x * a.tiles_y)) return 0;
  const size_t lds = ed2_lds_bytes<K, TH, TW, R, NT>(a.cin_pad, EXPAND, a.hid);
  auto kern = expand_dw2_kernel<K, UP, EXPAND, TH, TW, R, NT>;
  const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NT), lds, st, a);
  return (int)hipGetLastError();
}

// bf16, stride 1: the v2 kernel (two workgroups per CU when the tile's LDS fits 80 KB)
template <int K, int UP, bool EXPAND>
int launch_ed2_auto(EdArgs a, hipStream_t st) {
  if (EXPAND && a.cin_pad > 256) return AST_E_UNSUPPORTED;
  const int h = a.hid;
  if (ed2_lds_bytes<K, 8, 32, 2>(a.cin_pad, EXPAND, h) <= kLdsBudget) return launch_ed2<K, UP, EXPAND, 8, 32, 2>(a, st);
  if (g_ed_big && ed2_lds_bytes<K, 8, 32, 1, 1024>(a.cin_pad, EXPAND, h) <= kLdsBudgetMax)  // 16 waves, 1 WG/CU
    return launch_ed2<K, UP, EXPAND, 8, 32, 1, 1024>(a, st);
  if (ed2_lds_bytes<K, 4, 32, 1>(a.cin_pad, EXPAND, h) <= kLdsBudget) return launch_ed2<K, UP, EXPAND, 4, 32, 1>(a, st);
  if (ed2_lds_bytes<K, 4, 32, 1>(a.cin_pad, EXPAND, h) <= kLdsBudgetMax) return launch_ed2<K, UP, EXPAND, 4, 32, 1>(a, st);
  return AST_E_UNSUPPORTED;
}

int g_ed_version = 4;  // AST_MB_ED=1|2|3 select the v1|v2|v3 kernels (A/B measurements); 4: v4 where it applies

int g_ed3_nt = 0;  // AST_MB_ED3_NT=512|1024 forces the v3 workgroup size (A/B measurements)

template <int K>
int launch_ed3(EdArgs a, hipStream_t st) {
  using G = Ed3Geom<K>;
  if (a.cin_pad > 256) return AST_E_UNSUPPORTED;
  const size_t lds = ed3_lds<K>(a.cin_pad, a.hid).total;
  if (lds > kLdsBudgetMax) return AST_E_UNSUPPORTED;
  a.tiles_x = (a.wo + G::TW - 1) / G::TW;
  a.tiles_y = (a.ho + G::TH - 1) / G::TH;
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.n;
  if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
  if (ed_plan(a, (int64_t)a.tiles_x * a.tiles_y)) return 0;
  // two 8-wave workgroups per CU when the LDS allows, else one 16-wave workgroup (latency hiding)
  const bool two = lds <= kLdsBudget;
  const int nt = g_ed3_nt ? g_ed3_nt : two ? 512 : 1024;
  auto kern = nt == 512 ? (two ? expand_dw3_kernel<K, 512, 2> : expand_dw3_kernel<K, 512, 1>)
                        : expand_dw3_kernel<K, 1024, 1>;
  const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(nt), lds, st, a);
  return (int)hipGetLastError();
}

template <typename T>
int dispatch_ed(EdArgs a, int k, int s, int up, bool expand, hipStream_t st) {
  if (sizeof(T) == 2 && (up == 1 || !expand) && g_ed_version >= 4 && a.c1 == a.cin &&
      (int64_t)a.cin_pad * 2 * a.h * a.w < 0x7fffffffLL) {
    const int r = ast_mb::launch_ed4(a, k, s, st);
    if (r != AST_E_UNSUPPORTED || a.nod) return r;
  }
  if (a.nod) return AST_E_UNSUPPORTED;  // pool-only: the v4 kernels only
  if (sizeof(T) == 2 && s == 1 && up == 1 && expand && g_ed_version >= 3) {
    const int r = k == 3 ? launch_ed3<3>(a, st) : k == 5 ? launch_ed3<5>(a, st) : AST_E_UNSUPPORTED;
    if (r != AST_E_UNSUPPORTED) return r;
  }
  if (sizeof(T) == 2 && s == 1 && g_ed_version >= 2) {
    int r = AST_E_UNSUPPORTED;
    if (expand && up == 1 && k == 3) r = launch_ed2_auto<3, 1, true>(a, st);
    // k5 with narrow inputs: v2 only has the 4-row tile here (the 8-row one exceeds 80 KB of LDS),
    // whose halo recompute makes it slower than v1 (measured, scripts/bench_mb_blocks.py)
    else if (expand && up == 1 && k == 5 && a.cin_pad > 48) r = launch_ed2_auto<5, 1, true>(a, st);
    else if (!expand && k == 3 && up == 1) r = launch_ed2_auto<3, 1, false>(a, st);
    else if (!expand && k == 3 && up == 2) r = launch_ed2_auto<3, 2, false>(a, st);
    if (r != AST_E_UNSUPPORTED) return r;
  }
  if (expand && up == 1) {
    if (k == 3 && s == 1) return launch_ed<T, 3, 1, 1, true>(a, st);
    if (k == 3 && s == 2) return launch_ed<T, 3, 2, 1, true>(a, st);
    if (k == 5 && s == 1) return launch_ed<T, 5, 1, 1, true>(a, st);
    if (k == 5 && s == 2) return launch_ed<T, 5, 2, 1, true>(a, st);
  }
  if (!expand && k == 3 && s == 1) {
    if (up == 2) return launch_ed<T, 3, 1, 2, false>(a, st);
    if (up == 1) return launch_ed<T, 3, 1, 1, false>(a, st);
  }
  return AST_E_UNSUPPORTED;
}

template <typename T>
int dispatch_pw(PwArgs a, hipStream_t st) {
  const int mt = a.cout_pad / 16;
  constexpr int PXB = sizeof(T) == 2 ? PW_PX_BF16 : kPwPx;  // pixels per workgroup, MT <= 3
  const int px = mt <= 3 ? PXB : kPwPx;
  const int64_t tiles = ((int64_t)a.h * a.w + px - 1) / px;
  if ((int64_t)a.n * tiles > 0x7fffffffLL) return AST_E_SHAPE;
  a.tiles = (int)tiles;
  const int slices = (a.cout + a.cout_pad - 1) / a.cout_pad;  // 1 for pw-linear
  const dim3 grid((unsigned)(a.n * tiles), (unsigned)slices);
  switch (mt) {
    case 1: hipLaunchKernelGGL((pw_kernel<T, 1, PXB>), grid, dim3(kThreads), 0, st, a); break;
    case 2: hipLaunchKernelGGL((pw_kernel<T, 2, PXB>), grid, dim3(kThreads), 0, st, a); break;
    case 3: hipLaunchKernelGGL((pw_kernel<T, 3, PXB>), grid, dim3(kThreads), 0, st, a); break;
    case 4: hipLaunchKernelGGL((pw_kernel<T, 4>), grid, dim3(kThreads), 0, st, a); break;
    case 5: hipLaunchKernelGGL((pw_kernel<T, 5>), grid, dim3(kThreads), 0, st, a); break;
    case 6: hipLaunchKernelGGL((pw_kernel<T, 6>), grid, dim3(kThreads), 0, st, a); break;
    case 8: hipLaunchKernelGGL((pw_kernel<T, 8>), grid, dim3(kThreads), 0, st, a); break;
    default: return AST_E_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

template <typename TI, typename TO, int CIN, int COUT, int ACT>
int launch_dense(const void* x, const float* w, const float* b, void* y, int n, int h, int wd, hipStream_t st) {
  // whole 8-pixel groups, 16-byte aligned rows; at most 8 output channels per thread (16 x 8 pixels of
  // accumulators would leave one wave per SIMD)
  if (wd % 8 == 0 && wd >= 16) {
    constexpr int CB = COUT <= 8 ? COUT : 8;
    static_assert(COUT % CB == 0, "whole channel blocks");
    const int64_t gpi = (int64_t)h * (wd / 8);
    const int64_t blocks = (n * gpi + kThreads - 1) / kThreads;
    if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
    hipLaunchKernelGGL((dense3x3v8_kernel<TI, TO, CIN, COUT, ACT, CB>), dim3((unsigned)blocks, COUT / CB), dim3(kThreads),
                       0, st, reinterpret_cast<const TI*>(x), w, b, reinterpret_cast<TO*>(y), h, wd, gpi, n * gpi);
    return (int)hipGetLastError();
  }
  const int64_t gpi = (int64_t)h * ((wd + 3) / 4);
  const int64_t blocks = (n * gpi + kThreads - 1) / kThreads;
  if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL((dense3x3_kernel<TI, TO, CIN, COUT, ACT>), dim3((unsigned)blocks), dim3(kThreads), 0, st,
                     reinterpret_cast<const TI*>(x), w, b, reinterpret_cast<TO*>(y), h, wd, gpi, n * gpi);
  return (int)hipGetLastError();
}

}  // namespace

namespace {
// Argument checks and EdArgs of ast_mb_expand_dw (shared with its workspace query).
int ed_setup(int dtype, const void* x1, const void* x2, int c1, int n, int cin, int h, int w, int up, const void* w1p,
             int hid, int cin_pad, int k, int stride, int ho, int wo, EdArgs* out) {
  if (n <= 0 || cin <= 0 || h <= 1 || w <= 1 || hid <= 0 || ho <= 0 || wo <= 0) return AST_E_SHAPE;
  if (up != 1 && up != 2) return AST_E_SHAPE;
  if (!x2) { x2 = x1; c1 = cin; }
  if (c1 <= 0 || c1 > cin) return AST_E_SHAPE;
  if (k != 3 && k != 5) return AST_E_UNSUPPORTED;
  if (stride != 1 && stride != 2) return AST_E_UNSUPPORTED;
  const int p = (k - 1) / 2;
  if ((h * up + 2 * p - k) / stride + 1 != ho || (w * up + 2 * p - k) / stride + 1 != wo) return AST_E_SHAPE;
  if (h * up <= p || w * up <= p) return AST_E_SHAPE;  // reflection pad needs pad < size
  const bool expand = w1p != nullptr;
  if (expand) {
    const int ks = dtype == 1 ? 16 : 4;
    if (cin_pad < cin || cin_pad % ks != 0) return AST_E_SHAPE;
  } else if (hid != cin) {
    return AST_E_SHAPE;
  }
  if (dtype != 0 && dtype != 1) return AST_E_UNSUPPORTED;
  static const int ver = [] {
    const char* v = getenv("AST_MB_ED");
    return v ? atoi(v) : 4;
  }();
  g_ed_version = ver;
  static const int big = [] {
    const char* v = getenv("AST_MB_ED_BIG");
    return v ? atoi(v) : 1;
  }();
  g_ed_big = big;
  static const int th = [] {
    const char* v = getenv("AST_MB_ED_TH");
    return v ? atoi(v) : 0;
  }();
  g_ed_th = th;
  static const int ed3_nt = [] {
    const char* v = getenv("AST_MB_ED3_NT");
    return v ? atoi(v) : 0;
  }();
  g_ed3_nt = ed3_nt;
  *out = EdArgs{x1, x2, c1, n, cin, h, w, h * up, w * up, ho, wo, w1p, nullptr, hid, expand ? cin_pad : 0,
                nullptr, nullptr, nullptr, nullptr, 0, 0, 0, nullptr};
  return 0;
}

int ed_dispatch(int dtype, EdArgs a, int k, int stride, int up, hipStream_t st) {
  const bool expand = a.w1 != nullptr;
  if (dtype == 0) return dispatch_ed<float>(a, k, stride, up, expand, st);
  return dispatch_ed<bf16>(a, k, stride, up, expand, st);
}
}  // namespace

// Eval-mode BatchNorm folded into the preceding conv (mobilenetv2.py DepthWiseConv, the planned
// inference path): s = gamma / sqrt(var + eps), w' = w * s per output row, b' = beta - mean * s --
// the same operations and roundings as the torch expression it replaces (add, sqrt, div, mul; mean * s
// rounded before the subtraction), one launch instead of six elementwise ones per conv, written
// straight into the padded [rows_out][ld] layout the kernels read (padding zero).
__global__ void fold_bn_kernel(const float* __restrict__ w, int cout, int k, const float* __restrict__ gamma,
                               const float* __restrict__ beta, const float* __restrict__ mean,
                               const float* __restrict__ var, float eps, int has_bn, float* __restrict__ w_out,
                               int ld, int rows_out, float* __restrict__ b_out) {
#pragma clang fp contract(off)  // mean * s rounded before the subtraction, as torch's two kernels
  const int64_t total = (int64_t)rows_out * ld;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / ld), c = (int)(e - (int64_t)r * ld);
    float v = 0.f;
    if (r < cout && c < k) {
      v = w[(int64_t)r * k + c];
      if (has_bn) v = v * (gamma[r] / __builtin_sqrtf(var[r] + eps));
    }
    w_out[e] = v;
    if (c == 0 && b_out && r < cout) {
      float b = 0.f;
      if (has_bn) {
        const float sc = gamma[r] / __builtin_sqrtf(var[r] + eps);
        const float ms = mean[r] * sc;
        b = beta[r] - ms;
      }
      b_out[r] = b;
    }
  }
}

extern "C" {

long long ast_mb_expand_dw_workspace_floats(int dtype, int has_x2, int c1, int n, int cin, int h, int w, int up,
                                            int expand, int hid, int cin_pad, int k, int stride, int ho, int wo) {
  // (the pool-only form, d == NULL, never needs more slots than the D-writing form planned here)
  static const char dummy = 0;  // stand-in pointers: the plan only looks at their presence
  EdArgs a;
  if (ed_setup(dtype, &dummy, has_x2 ? &dummy : nullptr, c1, n, cin, h, w, up, expand ? &dummy : nullptr, hid,
               cin_pad, k, stride, ho, wo, &a))
    return 0;
  long long slots = 0;
  a.plan = &slots;
  if (ed_dispatch(dtype, a, k, stride, up, nullptr) != 0 || slots <= 0) return 0;
  return (long long)n * hid * slots;
}

int ast_mb_expand_dw(int dtype, const void* x1, const void* x2, int c1, int n, int cin, int h, int w, int up,
                     const void* w1p, const float* b1, int hid, int cin_pad, const float* wdw, const float* bdw,
                     int k, int stride, void* d, float* pool, int ho, int wo, float* workspace,
                     long long workspace_floats, void* stream) {
  if (!x1 || !wdw || !bdw || !pool || !workspace) return AST_E_NULLPTR;
  if (w1p && !b1) return AST_E_NULLPTR;
  EdArgs a;
  if (const int e = ed_setup(dtype, x1, x2, c1, n, cin, h, w, up, w1p, hid, cin_pad, k, stride, ho, wo, &a)) return e;
  a.nod = d == nullptr;  // pool-only pass of the fused pair
  hipStream_t st = (hipStream_t)stream;
  long long slots = 0;
  a.plan = &slots;
  if (const int e = ed_dispatch(dtype, a, k, stride, up, st)) return e;
  if (slots <= 0 || slots > 0x7fffffff) return AST_E_UNSUPPORTED;
  if (workspace_floats < (long long)n * hid * slots) return AST_E_SHAPE;  // workspace too small
  a.plan = nullptr;
  a.b1 = b1;
  a.wdw = wdw;
  a.bdw = bdw;
  a.d = d;
  a.pool = workspace;  // [n][hid][slots] tile sums
  if (const int e = ed_dispatch(dtype, a, k, stride, up, st)) return e;
  // pool[n][c] = the channel's tile sums in tile order
  return (int)ast_det::reduce_rows(workspace, (int64_t)n * hid, (int)slots, pool, st);
}

int ast_mb_expand_dw_pw_supported(int dtype, int has_x2, int cin, int cin_pad, int hid, int cout, int k, int stride,
                                  int up, int ho, int wo) {
  if (dtype != 1 || has_x2 || cin <= 0 || cin_pad < cin || cin_pad % 16) return 0;
  return ast_mb::edpw4_supported(cin_pad, hid, cout, k, stride, up, ho, wo);
}

int ast_mb_expand_dw_pw(int dtype, const void* x, int n, int cin, int h, int w, const void* w1p, const float* b1,
                        int hid, int cin_pad, const float* wdw, const float* bdw, int k, const void* wg, int cout,
                        int cout_pad, int hid_pad, const float* b2, const void* res, void* out, void* stream) {
  if (!x || !w1p || !b1 || !wdw || !bdw || !wg || !out) return AST_E_NULLPTR;
  if (n <= 0 || cout <= 0) return AST_E_SHAPE;
  if (!ast_mb_expand_dw_pw_supported(dtype, 0, cin, cin_pad, hid, cout, k, 1, 1, h, w)) return AST_E_UNSUPPORTED;
  EdpwArgs pa{};
  if (const int e = ed_setup(dtype, x, nullptr, cin, n, cin, h, w, 1, w1p, hid, cin_pad, k, 1, h, w, &pa.e)) return e;
  pa.e.b1 = b1;
  pa.e.wdw = wdw;
  pa.e.bdw = bdw;
  pa.wg = wg;
  pa.b2 = b2;
  pa.res = res;
  pa.out = out;
  pa.cout = cout;
  pa.cout_pad = cout_pad;
  pa.hid_pad = hid_pad;
  return ast_mb::launch_edpw4(pa, (hipStream_t)stream);
}

int ast_mb_se_fold(int dtype, const float* pool, int n, int hid, long long hw, const float* fc1w,
                   const float* fc1b, int red, const float* fc2w, const float* fc2b, const float* w2, int cout,
                   int cout_pad, int hid_pad, void* wg, void* stream) {
  if (!pool || !fc1w || !fc1b || !fc2w || !fc2b || !w2 || !wg) return AST_E_NULLPTR;
  if (n <= 0 || hid <= 0 || hw <= 0 || red <= 0 || cout <= 0 || cout_pad < cout || hid_pad < hid) return AST_E_SHAPE;
  const size_t sm = sizeof(float) * (size_t)(2 * hid + red);
  if (sm > 64 * 1024) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(se_fold_kernel<float>, dim3(n), dim3(kThreads), sm, st, pool, hid, (float)hw, fc1w, fc1b, red,
                       fc2w, fc2b, w2, cout, cout_pad, hid_pad, reinterpret_cast<float*>(wg));
  else if (dtype == 1)
    hipLaunchKernelGGL(se_fold_kernel<bf16>, dim3(n), dim3(kThreads), sm, st, pool, hid, (float)hw, fc1w, fc1b, red,
                       fc2w, fc2b, w2, cout, cout_pad, hid_pad, reinterpret_cast<bf16*>(wg));
  else
    return AST_E_UNSUPPORTED;
  return (int)hipGetLastError();
}

int ast_mb_pw(int dtype, const void* d, int n, int hid, int hid_pad, int h, int w, const void* wg,
              long long wg_stride, const float* bias, int cout, int cout_pad, const void* res, int res_up, void* out,
              void* stream) {
  if (!d || !wg || !out) return AST_E_NULLPTR;
  if (n <= 0 || hid <= 0 || h <= 0 || w <= 0 || cout <= 0) return AST_E_SHAPE;
  if (hid_pad < hid || hid_pad % kPwK != 0 || cout_pad < cout || cout_pad % 16 != 0) return AST_E_SHAPE;
  if (res_up && (h % 2 || w % 2)) return AST_E_SHAPE;
  if ((int64_t)h * w >= ((int64_t)1 << 31)) return AST_E_SHAPE;  // 32-bit pixel index in the epilogue
  if (cout_pad > 128 || cout > cout_pad) return AST_E_UNSUPPORTED;
  PwArgs a{d, n, hid, hid_pad, h, w, wg, (int64_t)wg_stride, bias, cout, cout_pad, res, res_up ? 1 : 0, out, 0,
           d, hid, 0};
  if (dtype == 0) return dispatch_pw<float>(a, (hipStream_t)stream);
  if (dtype == 1) return dispatch_pw<bf16>(a, (hipStream_t)stream);
  return AST_E_UNSUPPORTED;
}

int ast_mb_expand_gemm(int dtype, const void* x1, const void* x2, int c1, int n, int cin, int h, int w,
                       const void* w1p, const float* b1, int hid, int cin_pad, void* out, void* stream) {
  if (!x1 || !w1p || !b1 || !out) return AST_E_NULLPTR;
  if (n <= 0 || cin <= 0 || h <= 0 || w <= 0 || hid <= 0) return AST_E_SHAPE;
  if (!x2) { x2 = x1; c1 = cin; }
  if (c1 <= 0 || c1 > cin) return AST_E_SHAPE;
  if (cin_pad < cin || cin_pad % kPwK != 0) return AST_E_SHAPE;
  if (hid % 128 != 0) return AST_E_UNSUPPORTED;  // whole 128-channel slices: no w1p row past hid is read
  if ((int64_t)h * w >= ((int64_t)1 << 31)) return AST_E_SHAPE;
  PwArgs a{x1, n, cin, cin_pad, h, w, w1p, 0, b1, hid, 128, nullptr, 0, out, 0, x2, c1, 1};
  const hipStream_t st = (hipStream_t)stream;
  if (dtype == 1) {
    const int64_t tiles = ((int64_t)h * w + kPwPx - 1) / kPwPx;
    if ((int64_t)n * tiles > 0x7fffffffLL) return AST_E_SHAPE;
    a.tiles = (int)tiles;
    hipLaunchKernelGGL((pw_kernel<bf16, 8>), dim3((unsigned)(n * tiles), (unsigned)((hid + 127) / 128)), dim3(kThreads),
                       0, st, a);
    return (int)hipGetLastError();
  }
  return AST_E_UNSUPPORTED;
}

int ast_mb_conv3x3_dense(int dtype_in, int dtype_out, const void* x, const float* wt, const float* bias, void* y,
                         int n, int cin, int cout, int h, int w, int act, void* stream) {
  if (!x || !wt || !y) return AST_E_NULLPTR;
  if (n <= 0 || h <= 1 || w <= 1) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  // block 0 (mobilenetv2.py:38-43): fp32 image -> Hardswish
  if (cin == 3 && cout == 16 && act == 1) {
    if (dtype_in == 0 && dtype_out == 0) return launch_dense<float, float, 3, 16, 1>(x, wt, bias, y, n, h, w, st);
    if (dtype_in == 0 && dtype_out == 1) return launch_dense<float, bf16, 3, 16, 1>(x, wt, bias, y, n, h, w, st);
    if (dtype_in == 1 && dtype_out == 1) return launch_dense<bf16, bf16, 3, 16, 1>(x, wt, bias, y, n, h, w, st);
  }
  // decoder output conv (models.py:300-316): optional Hardtanh(0, 1)
  if (cin == 16 && cout == 3 && (act == 0 || act == 2)) {
    if (dtype_in == 0 && dtype_out == 0)
      return act ? launch_dense<float, float, 16, 3, 2>(x, wt, bias, y, n, h, w, st)
                 : launch_dense<float, float, 16, 3, 0>(x, wt, bias, y, n, h, w, st);
    if (dtype_in == 1 && dtype_out == 0)
      return act ? launch_dense<bf16, float, 16, 3, 2>(x, wt, bias, y, n, h, w, st)
                 : launch_dense<bf16, float, 16, 3, 0>(x, wt, bias, y, n, h, w, st);
    if (dtype_in == 1 && dtype_out == 1)
      return act ? launch_dense<bf16, bf16, 16, 3, 2>(x, wt, bias, y, n, h, w, st)
                 : launch_dense<bf16, bf16, 16, 3, 0>(x, wt, bias, y, n, h, w, st);
  }
  return AST_E_UNSUPPORTED;
}

int ast_adain_bf16(const void* content, const void* style, void* out, int n, int c, int hc, int wc, int hs, int ws,
                   double alpha, int swap_style_stats, void* stream) {
  if (!content || !style || !out) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hc <= 0 || wc <= 0 || hs <= 0 || ws <= 0) return AST_E_SHAPE;
  const float a = (float)alpha, b = (float)(1.0 - alpha);
  hipLaunchKernelGGL(adain_bf16_kernel, dim3((unsigned)((int64_t)n * c)), dim3(kThreads), 0, (hipStream_t)stream,
                     reinterpret_cast<const bf16*>(content), reinterpret_cast<const bf16*>(style),
                     reinterpret_cast<bf16*>(out), (int64_t)hc * wc, (int64_t)hs * ws, a, b, swap_style_stats ? 1 : 0);
  return (int)hipGetLastError();
}

int ast_mb_fold_bn_f32(const float* w, int cout, int k, const float* gamma, const float* beta, const float* mean,
                       const float* var, float eps, int has_bn, float* w_out, int ld, int rows_out, float* b_out,
                       void* stream) {
  if (!w || !w_out || (has_bn && (!gamma || !beta || !mean || !var))) return AST_E_NULLPTR;
  if (cout <= 0 || k <= 0 || ld < k || rows_out < cout) return AST_E_SHAPE;
  const int64_t total = (int64_t)rows_out * ld;
  const int blocks = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
  hipLaunchKernelGGL(fold_bn_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, cout, k, gamma, beta, mean,
                     var, eps, has_bn, w_out, ld, rows_out, b_out);
  return (int)hipGetLastError();
}

}  // extern "C"
