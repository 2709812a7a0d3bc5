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
//                      The expanded hidden tensor never reaches HBM.
//   se_fold_kernel     SE MLP per image (mobilenetv2.py:63-81) and folds the gate into the pw-linear
//                      weights: Wg[n][co][c] = W2[co][c] * gate[n][c]   (x*gate then conv == conv with Wg).
//   pw_kernel          per-image GEMM out = Wg[n] . D + b (+ residual, optionally nearest-upsampled),
//                      D staged through LDS transposed so both MFMA operands are k-contiguous.
//
// Storage type T is float or __bf16; all arithmetic and accumulation is fp32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

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
struct EdArgs {
  const void* x1;
  const void* x2;   // channels [c1, cin) come from x2 (torch.cat fused away), may equal x1
  int c1;
  int n, cin, h, w;  // x geometry (pre-upsample)
  int hd, wd;        // depthwise input grid (= h*up, w*up)
  int ho, wo;        // depthwise output
  const void* w1;    // expand weights T [hid_pad16][cin_pad] (BN folded); null -> ratio-1 block
  const float* b1;   // [hid]
  int hid, cin_pad;
  const float* wdw;  // depthwise weights [hid][k*k] (BN folded)
  const float* bdw;  // [hid]
  void* d;           // [n][hid][ho][wo]
  float* pool;       // [n][hid], accumulated
  int tiles_x, tiles_y;
};

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
    if (EXPAND) {
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
    } else {
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
          if (ky >= 0 && ky < K) {
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
          *reinterpret_cast<typename VecOf<T, G::CW>::type*>(drow + r * a.wo) = v;
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
      if ((tid & 15) == 0) atomicAdd(a.pool + (int64_t)n * a.hid + hc, psum);
    }
    lds_barrier();  // hs / ws reused by the next chunk
  }
#undef ED_FETCH
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
  for (int j = threadIdx.x; j < red; j += kThreads) {
    float s = fc1b[j];
    for (int c = 0; c < hid; ++c) s = fmaf(fc1w[(int64_t)j * hid + c], mean[c], s);
    hmid[j] = fmaxf(s, 0.f);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < hid; c += kThreads) {
    float s = fc2b[c];
    for (int j = 0; j < red; ++j) s = fmaf(fc2w[(int64_t)c * red + j], hmid[j], s);
    gate[c] = fminf(fmaxf(s, 0.f), 1.f);
  }
  __syncthreads();
  T* o = wg + (int64_t)n * cout_pad * hid_pad;
  for (int e = threadIdx.x; e < cout_pad * hid_pad; e += kThreads) {
    const int co = e / hid_pad, c = e - co * hid_pad;
    o[e] = from_f<T>(co < cout && c < hid ? w2[(int64_t)co * hid + c] * gate[c] : 0.f);
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
};

constexpr int kPwPx = 256;  // pixels per workgroup (4 waves x 64)
constexpr int kPwK = 32;    // hidden channels per LDS stage

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// D is staged in its natural [channel][pixel] layout (16-byte writes, global loads coalesced along
// pixels). bf16: the 16x16x32 B operand wants 8 channels of one pixel per lane, which the gfx950
// transposed read ds_read_b64_tr_b16 delivers from that layout; the MFMA k order is permuted to
// (4g..4g+3, 16+4g..16+4g+3) for lane group g (A uses the same order), so each half-wave's read
// touches 8 consecutive rows, conflict-free with a row pitch of 16 (mod 128) elements.
template <typename T, int MT>
__global__ __launch_bounds__(kThreads, 2) void pw_kernel(PwArgs a) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int LDP = kPwPx + (BF ? 16 : 4);     // D image row pitch (elements)
  constexpr int LDW = kPwK + Mma<T>::PAD;        // weight image row pitch
  constexpr int VEC = 16 / sizeof(T);            // elements per 16-byte vector
  constexpr int NV = kPwK * kPwPx / VEC / kThreads;
  constexpr int VPR = kPwPx / VEC;               // vectors per channel row
  __shared__ __align__(16) T ds[kPwK * LDP];
  __shared__ __align__(16) T ws[MT * 16 * LDW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.x / a.tiles;
  const int64_t p0 = (int64_t)(blockIdx.x % a.tiles) * kPwPx;
  const int64_t hw = (int64_t)a.h * a.w;
  const T* dn = reinterpret_cast<const T*>(a.d) + (int64_t)n * a.hid * hw;
  const T* wn = reinterpret_cast<const T*>(a.wg) + (int64_t)n * a.wg_stride;
  const bool vec = (hw % VEC) == 0 && p0 + kPwPx <= hw;

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
        if (kb + c < a.hid) val = *reinterpret_cast<const uint4*>(dn + (int64_t)(kb + c) * hw + p0 + q);   \
      } else {                                                                                             \
        typename VecOf<T, VEC>::type tv;                                                                   \
        _Pragma("unroll") for (int j = 0; j < VEC; ++j) {                                                  \
          T x = from_f<T>(0.f);                                                                            \
          if (kb + c < a.hid && p0 + q + j < hw) x = dn[(int64_t)(kb + c) * hw + p0 + q + j];              \
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

  f32x4 acc[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

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
      bf16x8 bfr[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = wave * 64 + t * 16 + 4 * p;
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
        for (int t = 0; t < 4; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[t], acc[m][t], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < kPwK; ks += 4) {
        const int kr = ks + (lane >> 4);
        float bfr[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) bfr[t] = ds[kr * LDP + wave * 64 + t * 16 + (lane & 15)];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const float afr = ws[(m * 16 + (lane & 15)) * LDW + kr];
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(afr, bfr[t], acc[m][t], 0, 0, 0);
        }
      }
    }
    lds_barrier();
  }

  T* out = reinterpret_cast<T*>(a.out) + (int64_t)n * a.cout * hw;
  const T* res = reinterpret_cast<const T*>(a.res);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m * 16 + 4 * (lane >> 4) + r;
      if (co >= a.cout) continue;
      const float bco = a.bias ? a.bias[co] : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int64_t p = p0 + wave * 64 + t * 16 + (lane & 15);
        if (p >= hw) continue;
        float v = acc[m][t][r] + bco;
        if (res) {
          if (a.res_up) {
            const int y = (int)(p / a.w), x = (int)(p % a.w);
            const int hr = a.h / 2, wr = a.w / 2;
            v += to_f(res[(((int64_t)n * a.cout + co) * hr + (y >> 1)) * wr + (x >> 1)]);
          } else {
            v += to_f(res[((int64_t)n * a.cout + co) * hw + p]);
          }
        }
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
  const size_t lds = ed_lds_bytes<T, K, S, TH, TW>(a.cin_pad, EXPAND);
  auto kern = expand_dw_kernel<T, K, S, UP, EXPAND, TH, TW>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), lds, st, a);
  return (int)hipGetLastError();
}

template <typename T, int K, int S, int UP, bool EXPAND>
int launch_ed(EdArgs a, hipStream_t st) {
  constexpr int TW = S == 1 ? 32 : 16;  // output tile width; 8/4/2 rows as LDS allows
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

template <typename T>
int dispatch_ed(EdArgs a, int k, int s, int up, bool expand, hipStream_t st) {
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
  const int64_t tiles = ((int64_t)a.h * a.w + kPwPx - 1) / kPwPx;
  if ((int64_t)a.n * tiles > 0x7fffffffLL) return AST_E_SHAPE;
  a.tiles = (int)tiles;
  const dim3 grid((unsigned)(a.n * tiles));
  switch (mt) {
    case 1: hipLaunchKernelGGL((pw_kernel<T, 1>), grid, dim3(kThreads), 0, st, a); break;
    case 2: hipLaunchKernelGGL((pw_kernel<T, 2>), grid, dim3(kThreads), 0, st, a); break;
    case 3: hipLaunchKernelGGL((pw_kernel<T, 3>), grid, dim3(kThreads), 0, st, a); break;
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
  const int64_t gpi = (int64_t)h * ((wd + 3) / 4);
  const int64_t blocks = (n * gpi + kThreads - 1) / kThreads;
  if (blocks > 0x7fffffffLL) return AST_E_SHAPE;
  hipLaunchKernelGGL((dense3x3_kernel<TI, TO, CIN, COUT, ACT>), dim3((unsigned)blocks), dim3(kThreads), 0, st,
                     reinterpret_cast<const TI*>(x), w, b, reinterpret_cast<TO*>(y), h, wd, gpi, n * gpi);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int ast_mb_expand_dw(int dtype, const void* x1, const void* x2, int c1, int n, int cin, int h, int w, int up,
                     const void* w1p, const float* b1, int hid, int cin_pad, const float* wdw, const float* bdw,
                     int k, int stride, void* d, float* pool, int ho, int wo, void* stream) {
  if (!x1 || !wdw || !bdw || !d || !pool) return AST_E_NULLPTR;
  if (w1p && !b1) return AST_E_NULLPTR;
  if (n <= 0 || cin <= 0 || h <= 1 || w <= 1 || hid <= 0 || ho <= 0 || wo <= 0) return AST_E_SHAPE;
  if (up != 1 && up != 2) return AST_E_SHAPE;
  if (!x2) { x2 = x1; c1 = cin; }
  if (c1 <= 0 || c1 > cin) return AST_E_SHAPE;
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
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(pool, 0, sizeof(float) * (size_t)n * hid, st);
  if (e != hipSuccess) return (int)e;
  EdArgs a{x1, x2, c1, n, cin, h, w, h * up, w * up, ho, wo, w1p, b1, hid, expand ? cin_pad : 0, wdw, bdw, d, pool, 0, 0};
  if (dtype == 0) return dispatch_ed<float>(a, k, stride, up, expand, st);
  if (dtype == 1) return dispatch_ed<bf16>(a, k, stride, up, expand, st);
  return AST_E_UNSUPPORTED;
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
  PwArgs a{d, n, hid, hid_pad, h, w, wg, (int64_t)wg_stride, bias, cout, cout_pad, res, res_up ? 1 : 0, out, 0};
  if (dtype == 0) return dispatch_pw<float>(a, (hipStream_t)stream);
  if (dtype == 1) return dispatch_pw<bf16>(a, (hipStream_t)stream);
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

}  // extern "C"
