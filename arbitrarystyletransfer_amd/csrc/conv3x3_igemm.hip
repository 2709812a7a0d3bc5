// 3x3 stride-1 convolution as an MFMA-fp32 implicit GEMM for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's nn.Conv2d(k3,p1)+ReLU(+MaxPool) chain of PretrainedEncoder
// (models.py:199-240) and the [Upsample]+ReflectionPad+Conv+ReLU chain of the mirrored decoder
// (models.py:598-628). GEMM view: out[pixel][cout] = sum_{cin,tap} in[pixel+tap][cin] * w[cin,tap][cout].
//
// Design:
//  * v_mfma_f32_32x32x2_f32: exact fp32 products (an fmaf chain), 64 FLOP/clk/SIMD = the
//    157.3 TF fp32 matrix peak. Lane l feeds A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31].
//  * M = one 32-pixel output row segment per MFMA tile (lanes -> consecutive x: conflict-free
//    LDS reads and float4 NCHW stores), N = 32 output channels, K pair = two input channels at
//    the same tap.
//  * A workgroup owns a TH x 32 output tile x BN channels. Per K-chunk of CK input channels it
//    stages the SOURCE tile (before the x2 nearest upsample) with a 1-pixel halo in LDS: float4
//    row loads for the interior, scalar loads for the two halo columns, rows remapped for
//    zero / reflect padding. Upsample + reflect padding of the upsampled grid equals
//    replicate-padding of the source grid, so both are resolved by the per-lane LDS read
//    address. The conv_1 ImageNet normalisation is applied to loaded values (padding stays 0,
//    as the reference pads the normalised image). The CK x 9 x BN weight slab is staged beside
//    it; both double-buffered, next chunk's global loads in flight while the MFMAs run.
//  * Epilogue: bias, optional pre-ReLU store (the conv_i taps of the loss network), ReLU store,
//    and a fused 2x2 max-pool done in registers (a lane holds both rows of a window).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "x3.h"
#include "cin3.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));  // register staging (HIP float4 arrays defeat SROA)

constexpr int TW = 32;  // output tile width = one MFMA M-tile

struct ConvArgs {
  const float* x;
  const float* x2;  // optional second input batch: images [nsplit, N) read from x2 (content|style pair)
  int nsplit;
  const float* wp;  // packed [cin_pad][9][cout_pad]
  const float* bias;
  float* y_pre;
  float* y_act;
  float* y_pool;
  const float* in_mean;
  const float* in_std;
  int N, Cin, Hin, Win, Cout, H, W;
  int cin_pad, cout_pad;
  int reflect;  // 0: zero pad, 1: reflect pad (of the upsampled grid)
  int tiles_x, tiles_y;
  // input-gradient epilogue (x3 kernels only; ast_conv3x3_dgrad_f32): with v the conv output at an
  // output position (of y_pre, or of y_pool when e_sum2), v = v + e_add_pre; then
  // v = e_mask > 0 ? e_add_post + v : e_add_post (the ReLU backward of the layer below, with its
  // pre-ReLU tap gradient; a missing add_post reads as 0, a missing mask as > 0)
  const float* e_mask;
  const float* e_add_pre;
  const float* e_add_post;
  int e_sum2;  // y_pool holds the 2x2 SUM of the output (nearest-upsample adjoint), no ReLU / max
};

__device__ __forceinline__ bool dgrad_epi(const ConvArgs& a) { return a.e_mask || a.e_add_pre || a.e_add_post; }

// the input-gradient epilogue of one output value at flat offset off (see ConvArgs)
__device__ __forceinline__ float dgrad_epi_one(const ConvArgs& a, float v, int64_t off) {
  if (a.e_add_pre) v = v + a.e_add_pre[off];
  const bool keep = !a.e_mask || a.e_mask[off] > 0.f;
  if (a.e_add_post) return keep ? a.e_add_post[off] + v : a.e_add_post[off];
  return keep ? v : 0.f;
}

__device__ __forceinline__ float4 dgrad_epi4(const ConvArgs& a, float4 v, int64_t off) {
  if (a.e_add_pre) {
    const float4 u = *reinterpret_cast<const float4*>(a.e_add_pre + off);
    v = make_float4(v.x + u.x, v.y + u.y, v.z + u.z, v.w + u.w);
  }
  float4 m = make_float4(1.f, 1.f, 1.f, 1.f), p = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.e_mask) m = *reinterpret_cast<const float4*>(a.e_mask + off);
  if (a.e_add_post) {
    p = *reinterpret_cast<const float4*>(a.e_add_post + off);
    return make_float4(m.x > 0.f ? p.x + v.x : p.x, m.y > 0.f ? p.y + v.y : p.y, m.z > 0.f ? p.z + v.z : p.z,
                       m.w > 0.f ? p.w + v.w : p.w);
  }
  return make_float4(m.x > 0.f ? v.x : 0.f, m.y > 0.f ? v.y : 0.f, m.z > 0.f ? v.z : 0.f, m.w > 0.f ? v.w : 0.f);
}

constexpr int kCinAlign = 8;    // packed cin padding (>= every CK)
constexpr int kCoutAlign = 64;  // packed cout padding

// Source-grid index of padded coordinate g (may be -1 or n) for the pad mode; -1 = zero.
//  reflect, no upsample: ReflectionPad2d(1)        -> reflect
//  reflect, upsample x2: reflect on 2n grid        -> replicate on the n grid
//  zeros:                                          -> -1 outside
template <int UP>
__device__ __forceinline__ int src_index(int g, int n, int reflect) {
  if (g >= 0 && g < n) return g;
  if (!reflect) return -1;
  if (UP == 2) return g < 0 ? 0 : n - 1;
  int r = g < 0 ? -g : 2 * (n - 1) - g;
  return r < 0 ? 0 : (r >= n ? n - 1 : r);
}

// torch semantics: relu(NaN) = NaN, max_pool propagates NaN.
__device__ __forceinline__ float relu_f(float v) { return v < 0.f ? 0.f : v; }
__device__ __forceinline__ float max_nan(float a, float b) { return (b > a || b != b) ? b : a; }

template <int WM, int WN, int RM, int RN, int CK, int UP>
struct Cfg {
  static constexpr int NT = WM * WN * 64;
  static constexpr int TH = WM * RM;             // output rows per tile
  static constexpr int BN = WN * RN * 32;        // output channels per tile
  static constexpr int SW = TW / UP;             // source columns per tile (interior)
  static constexpr int SR = TH / UP + 2;         // source rows per tile incl. halo
  static constexpr int RS = SW + 8;              // LDS row stride: [pad3|halo|interior(16B aligned)|halo|pad]
  static constexpr int C0 = 4;                   // LDS column of source column sx0
  static constexpr int A_ELEMS = CK * SR * RS;
  static constexpr int B_ELEMS = CK * 9 * BN;
  static constexpr int QV = SW / 4;              // float4 per interior row
  static constexpr int A_ITEMS = CK * SR * (QV + 2);     // fast path: QV vectors + 2 halo scalars per row
  static constexpr int A_PER_T = (A_ITEMS + NT - 1) / NT;
  static constexpr int S_ITEMS = CK * SR * (SW + 2);     // slow path: scalar per column
  static constexpr int B_VEC = B_ELEMS / 4;
  static constexpr int B_PER_T = (B_VEC + NT - 1) / NT;
  static constexpr int LDS_BYTES = 2 * (A_ELEMS + B_ELEMS) * 4;
};

// Workgroup -> (spatial tile, output-channel group). The G channel groups of one spatial tile
// read the same input tile, so they get ids b, b+8, ..., b+8(G-1): dispatched together, and onto
// one XCD under the observed round-robin placement (speed only, never correctness).
__device__ __forceinline__ bool decode_block(int id, int ntiles, int groups, int& tile, int& group) {
  const int xcd = id & 7, rest = id >> 3;
  group = rest % groups;
  tile = (rest / groups) * 8 + xcd;
  return tile < ntiles;
}

// Epilogue of a wave's RM x RN tiles of 32x32 accumulators (A = pixels, B = channels: lane l32 =
// output channel n0c + 32j + l32, register 4g + r = pixel x0 + 8g + 4h + r of row y0 + row0 + i):
// +bias, pre-ReLU / ReLU float4 stores, fused 2x2 max-pool (a lane holds both rows of a window).
template <int RM, int RN>
__device__ __forceinline__ void store_tiles(const ConvArgs& a, const f32x16 (&acc)[RM][RN], int n, int x0, int y0,
                                            int row0, int n0c, int h, int l32) {
  const int H = a.H, W = a.W;
  const int64_t plane = (int64_t)H * W;
  const bool vec4 = (W & 3) == 0;
  const int Ho = H >> 1, Wo = W >> 1;
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int co = n0c + j * 32 + l32;
    const bool cok = co < a.Cout;
    const float bv = (cok && a.bias) ? a.bias[co] : 0.f;
    const int64_t obase = ((int64_t)n * a.Cout + co) * plane;
    if (a.y_pre || a.y_act) {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int yy = y0 + row0 + i;
        if (!cok || yy >= H) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int xx = x0 + 8 * g + 4 * h;
          if (xx >= W) continue;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][j][4 * g + r] + bv;
          const int64_t off = obase + (int64_t)yy * W + xx;
          const bool full = vec4 && xx + 3 < W;
          if (a.y_pre) {
            if (full) *reinterpret_cast<float4*>(a.y_pre + off) = make_float4(v[0], v[1], v[2], v[3]);
            else for (int r = 0; r < 4; ++r) if (xx + r < W) a.y_pre[off + r] = v[r];
          }
          if (a.y_act) {
            float u[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) u[r] = relu_f(v[r]);
            if (full) *reinterpret_cast<float4*>(a.y_act + off) = make_float4(u[0], u[1], u[2], u[3]);
            else for (int r = 0; r < 4; ++r) if (xx + r < W) a.y_act[off + r] = u[r];
          }
        }
      }
    }
    if (a.y_pool && cok) {
      const int64_t pbase = ((int64_t)n * a.Cout + co) * Ho * Wo;
#pragma unroll
      for (int i = 0; i + 1 < RM; i += 2) {
        const int py = (y0 + row0 + i) >> 1;
        if (py >= Ho) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int px = (x0 + 8 * g + 4 * h) >> 1;
          if (px >= Wo) continue;
          float m[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            m[r] = max_nan(relu_f(acc[i][j][4 * g + r] + bv), relu_f(acc[i + 1][j][4 * g + r] + bv));
          const float p0 = max_nan(m[0], m[1]), p1 = max_nan(m[2], m[3]);
          const int64_t off = pbase + (int64_t)py * Wo + px;
          if (px + 1 < Wo && (Wo & 1) == 0) {
            *reinterpret_cast<float2*>(a.y_pool + off) = make_float2(p0, p1);
          } else {
            a.y_pool[off] = p0;
            if (px + 1 < Wo) a.y_pool[off + 1] = p1;
          }
        }
      }
    }
  }
}

template <int WM, int WN, int RM, int RN, int CK, int UP, bool SWAP, bool NORM>
__global__ __launch_bounds__(WM * WN * 64, WM * WN >= 16 ? 1 : 2) void conv3x3_f32_kernel(ConvArgs a) {
  using C = Cfg<WM, WN, RM, RN, CK, UP>;
  constexpr int NT = C::NT, TH = C::TH, BN = C::BN, SW = C::SW, SR = C::SR, RS = C::RS, QV = C::QV;
  constexpr int A_ELEMS = C::A_ELEMS, B_ELEMS = C::B_ELEMS;
  static_assert(CK % 2 == 0, "two channels per MFMA k-pair");
  static_assert(TH % 2 == 0, "even tile height (pool windows, upsample row pairs)");
  static_assert(UP == 1 || UP == 2, "");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                // [2][CK][SR][RS]
  float* Bs = smem + 2 * A_ELEMS;  // [2][CK*9][BN]

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, l32 = lane & 31;
  const int wm = wave % WM, wn = wave / WM;

  int t, grp;
  if (!decode_block(blockIdx.x, a.tiles_x * a.tiles_y * a.N, (a.Cout + BN - 1) / BN, t, grp)) return;
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  const int n = t / a.tiles_y;
  const int x0 = tx * TW, y0 = ty * TH;
  const int sx0 = x0 / UP, sy0 = y0 / UP - 1;  // source tile origin (row includes the halo)
  const int n0 = grp * BN;
  const int Hin = a.Hin, Win = a.Win;
  const bool fast = (sx0 + SW <= Win) && ((Win & 3) == 0);  // block-uniform

  const float* __restrict__ xin =
      n < a.nsplit ? a.x + (int64_t)n * a.Cin * Hin * Win : a.x2 + (int64_t)(n - a.nsplit) * a.Cin * Hin * Win;
  const int plane_in = Hin * Win;
  const int nchunks = (a.Cin + CK - 1) / CK;

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Per-lane LDS column of the A operand for each kx: source column of output x0+l32+kx-1.
  int acol[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) acol[kx] = C::C0 + (((x0 + l32 + kx - 1) >> (UP - 1)) - sx0);
  const int abase = h * SR * RS;                       // lane half h reads channel 2kp+h
  const int bbase = h * 9 * BN + wn * RN * 32 + l32;

  // One K-chunk of MFMAs from LDS buffer `buf` (CK input channels x 9 taps).
#define CONV_CHUNK_MFMA(buf)                                                                                 \
  {                                                                                                         \
    const float* as = As + (buf) * A_ELEMS + abase;                                                         \
    const float* bs = Bs + (buf) * B_ELEMS + bbase;                                                         \
    _Pragma("unroll") for (int ky = 0; ky < 3; ++ky) {                                                      \
      _Pragma("unroll") for (int kx = 0; kx < 3; ++kx) {                                                    \
        const int tap = ky * 3 + kx;                                                                        \
        _Pragma("unroll") for (int kp = 0; kp < CK / 2; ++kp) {                                             \
          float av[RM], bv[RN];                                                                             \
          _Pragma("unroll") for (int i = 0; i < RM; ++i) {                                                  \
            const int orow = wm * RM + i + ky - 1; /* -1 .. TH */                                           \
            const int srow = (UP == 1) ? orow + 1 : (orow >> 1) + 1;                                        \
            av[i] = as[(2 * kp * SR + srow) * RS + acol[kx]];                                               \
          }                                                                                                 \
          _Pragma("unroll") for (int j = 0; j < RN; ++j) bv[j] = bs[(2 * kp * 9 + tap) * BN + j * 32];      \
          _Pragma("unroll") for (int i = 0; i < RM; ++i)                                                    \
            _Pragma("unroll") for (int j = 0; j < RN; ++j)                                                  \
              acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_32x32x2f32(bv[j], av[i], acc[i][j], 0, 0, 0)     \
                               : __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);    \
        }                                                                                                   \
      }                                                                                                     \
    }                                                                                                       \
  }

  // Weight slab staging: B_VEC float4 per chunk; indices past the slab are clamped onto its last
  // vector (duplicate loads and identical LDS writes, no branch).
  constexpr int B_VEC = C::B_VEC, B_T = C::B_PER_T;
  int boff[B_T];
#pragma unroll
  for (int i = 0; i < B_T; ++i) {
    const int vi = min(tid + i * NT, B_VEC - 1), f = vi * 4, row = f / BN;
    boff[i] = row * a.cout_pad + (f - row * BN);
  }
  const float* __restrict__ wbase = a.wp + n0;

  if (fast) {
    // Source-tile staging, branch-free: per-lane offsets computed once per tile; per chunk the
    // channel base is a wave-uniform pointer. Interior items are float4 row pieces; each halo item
    // is the aligned float4 that holds the (zero / reflect / replicate) halo column, one component kept.
    constexpr int AI = CK * SR * QV, AI_T = (AI + NT - 1) / NT;
    constexpr int AH = CK * SR * 2, AH_T = (AH + NT - 1) / NT;
    int ai_g[AI_T], ai_l[AI_T], ai_c[AI_T];
    bool ai_ok[AI_T];
#pragma unroll
    for (int i = 0; i < AI_T; ++i) {
      const int e = min(tid + i * NT, AI - 1), q = e % QV, cr = e / QV, r = cr % SR, c = cr / SR;
      const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
      ai_ok[i] = sy >= 0;
      ai_c[i] = c;
      ai_g[i] = c * plane_in + max(sy, 0) * Win + sx0 + 4 * q;
      ai_l[i] = cr * RS + C::C0 + 4 * q;
    }
    int ah_g[AH_T], ah_l[AH_T], ah_c[AH_T], ah_k[AH_T];  // ah_k: component 0..3, or -1 = zero
#pragma unroll
    for (int i = 0; i < AH_T; ++i) {
      const int e = min(tid + i * NT, AH - 1), side = e & 1, cr = e >> 1, r = cr % SR, c = cr / SR;
      const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
      const int sx = src_index<UP>(side ? sx0 + SW : sx0 - 1, Win, a.reflect);
      const bool ok = sy >= 0 && sx >= 0;
      ah_k[i] = ok ? (sx & 3) : -1;
      ah_c[i] = c;
      ah_g[i] = c * plane_in + max(sy, 0) * Win + (ok ? (sx & ~3) : 0);
      ah_l[i] = cr * RS + (side ? C::C0 + SW : C::C0 - 1);
    }
    f32x4 ra[AI_T], rh[AH_T], rb[B_T];
    float nm[NORM ? AI_T : 1], ns[NORM ? AI_T : 1], hm[NORM ? AH_T : 1], hs[NORM ? AH_T : 1];

    // issue every global load of chunk KC (no waits: the values are consumed by CONV_WRITE_CHUNK).
    // (macros, not lambdas: a by-reference closure over the register arrays sends them to scratch)
#define CONV_LOAD_CHUNK(KC)                                                                               \
    {                                                                                                     \
      const int cin0 = (KC) * CK;                                                                         \
      const int cmax = a.Cin - 1 - cin0; /* chunk channels > cmax are zero */                             \
      const float* __restrict__ xb = xin + (int64_t)cin0 * plane_in;                                      \
      _Pragma("unroll") for (int i = 0; i < AI_T; ++i) {                                                  \
        ra[i] = *reinterpret_cast<const f32x4*>(xb + (ai_c[i] <= cmax ? ai_g[i] : 0));                   \
        if (NORM) {                                                                                       \
          const int ch = cin0 + min(ai_c[i], cmax);                                                       \
          nm[i] = a.in_mean[ch];                                                                          \
          ns[i] = a.in_std[ch];                                                                           \
        }                                                                                                 \
      }                                                                                                   \
      _Pragma("unroll") for (int i = 0; i < AH_T; ++i) {                                                  \
        rh[i] = *reinterpret_cast<const f32x4*>(xb + (ah_c[i] <= cmax ? ah_g[i] : 0));                   \
        if (NORM) {                                                                                       \
          const int ch = cin0 + min(ah_c[i], cmax);                                                       \
          hm[i] = a.in_mean[ch];                                                                          \
          hs[i] = a.in_std[ch];                                                                           \
        }                                                                                                 \
      }                                                                                                   \
      const float* __restrict__ wb = wbase + (int64_t)cin0 * 9 * a.cout_pad;                              \
      _Pragma("unroll") for (int i = 0; i < B_T; ++i) rb[i] = *reinterpret_cast<const f32x4*>(wb + boff[i]); \
    }
#define CONV_WRITE_CHUNK(KC, BUF)                                                                         \
    {                                                                                                     \
      const int cmax = a.Cin - 1 - (KC) * CK;                                                             \
      float* as = As + (BUF) * A_ELEMS;                                                                   \
      _Pragma("unroll") for (int i = 0; i < AI_T; ++i) {                                                  \
        f32x4 v = ra[i];                                                                                  \
        if (NORM) v = (v - nm[i]) / ns[i];                                                                \
        if (!(ai_ok[i] && ai_c[i] <= cmax)) v = f32x4{0.f, 0.f, 0.f, 0.f};                                \
        *reinterpret_cast<f32x4*>(as + ai_l[i]) = v;                                                      \
      }                                                                                                   \
      _Pragma("unroll") for (int i = 0; i < AH_T; ++i) {                                                  \
        const int k = ah_k[i];                                                                            \
        const f32x4 q4 = rh[i];                                                                           \
        float v = k == 0 ? q4.x : (k == 1 ? q4.y : (k == 2 ? q4.z : q4.w));                               \
        if (NORM) v = (v - hm[i]) / hs[i];                                                                \
        as[ah_l[i]] = (k >= 0 && ah_c[i] <= cmax) ? v : 0.f;                                              \
      }                                                                                                   \
      float* bs = Bs + (BUF) * B_ELEMS;                                                                   \
      _Pragma("unroll") for (int i = 0; i < B_T; ++i)                                                     \
        *reinterpret_cast<f32x4*>(bs + min(tid + i * NT, B_VEC - 1) * 4) = rb[i];                         \
    }

    CONV_LOAD_CHUNK(0);
    CONV_WRITE_CHUNK(0, 0);
    __syncthreads();
    for (int kc = 0; kc < nchunks; ++kc) {
      const int buf = kc & 1;
      const int kn = min(kc + 1, nchunks - 1);  // the last iteration re-loads into the idle buffer
      CONV_LOAD_CHUNK(kn);
      __builtin_amdgcn_sched_barrier(0);         // keep the loads ahead of the MFMAs
      CONV_CHUNK_MFMA(buf);
      __builtin_amdgcn_sched_barrier(0);
      CONV_WRITE_CHUNK(kn, buf ^ 1);
      __syncthreads();
    }
  } else {
    // Irregular tiles (right edge narrower than the tile, or W % 4 != 0): scalar gather, no prefetch.
    auto fill_a_slow = [&](int cin0, float* as) {
      for (int e = tid; e < C::S_ITEMS; e += NT) {
        const int col = e % (SW + 2);
        const int cr = e / (SW + 2);
        const int r = cr % SR, c = cr / SR;
        const int cin = cin0 + c;
        const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
        const int sx = src_index<UP>(sx0 - 1 + col, Win, a.reflect);
        float v = 0.f;
        if (cin < a.Cin && sy >= 0 && sx >= 0) {
          v = xin[cin * plane_in + sy * Win + sx];
          if (NORM) v = (v - a.in_mean[cin]) / a.in_std[cin];
        }
        as[cr * RS + C::C0 - 1 + col] = v;
      }
    };
    for (int kc = 0; kc < nchunks; ++kc) {
      const int cin0 = kc * CK;
      fill_a_slow(cin0, As);
      const float* __restrict__ wb = wbase + (int64_t)cin0 * 9 * a.cout_pad;
#pragma unroll
      for (int i = 0; i < B_T; ++i)
        *reinterpret_cast<float4*>(Bs + min(tid + i * NT, B_VEC - 1) * 4) = *reinterpret_cast<const float4*>(wb + boff[i]);
      __syncthreads();
      CONV_CHUNK_MFMA(0);
      __syncthreads();
    }
  }
#undef CONV_CHUNK_MFMA
#undef CONV_LOAD_CHUNK
#undef CONV_WRITE_CHUNK

  // ---------------- epilogue ----------------
  const int H = a.H, W = a.W;
  const int64_t plane = (int64_t)H * W;
  const int Ho = H >> 1, Wo = W >> 1;
  if constexpr (SWAP) {
    // C^T: lane l32 = output column x0+l32, register r = channel (r&3)+8(r>>2)+4h of the
    // 32-channel tile. One dword store per register writes two whole 128-B row segments.
    const int xx = x0 + l32;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int cbase = n0 + (wn * RN + j) * 32 + 4 * h;
      float bvr[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = cbase + (r & 3) + 8 * (r >> 2);
        bvr[r] = (co < a.Cout && a.bias) ? a.bias[co] : 0.f;
      }
      if (a.y_pre || a.y_act) {
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const int yy = y0 + wm * RM + i;
          if (yy >= H || xx >= W) continue;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = cbase + (r & 3) + 8 * (r >> 2);
            if (co >= a.Cout) continue;
            const float v = acc[i][j][r] + bvr[r];
            const int64_t off = ((int64_t)n * a.Cout + co) * plane + (int64_t)yy * W + xx;
            if (a.y_pre) a.y_pre[off] = v;
            if (a.y_act) a.y_act[off] = relu_f(v);
          }
        }
      }
      if (a.y_pool) {
        const int px = xx >> 1;
#pragma unroll
        for (int i = 0; i + 1 < RM; i += 2) {
          const int py = (y0 + wm * RM + i) >> 1;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = cbase + (r & 3) + 8 * (r >> 2);
            float m = max_nan(relu_f(acc[i][j][r] + bvr[r]), relu_f(acc[i + 1][j][r] + bvr[r]));
            m = max_nan(m, __shfl_xor(m, 1, 64));  // horizontal neighbour = adjacent lane
            if ((l32 & 1) == 0 && co < a.Cout && py < Ho && px < Wo)
              a.y_pool[((int64_t)n * a.Cout + co) * Ho * Wo + (int64_t)py * Wo + px] = m;
          }
        }
      }
    }
    return;
  }
  store_tiles<RM, RN>(a, acc, n, x0, y0, wm * RM, n0 + wn * RN * 32, h, l32);
}

// ------------------------------------------------------------------------------------------------
// Split-bf16 ("bf16x3") implicit GEMM: fp32 accuracy on the bf16 matrix cores.
//
// Every fp32 operand is split exactly into three bf16 terms, x = hi + mid + lo (hi = bf16(x),
// mid = bf16(x - hi), lo = x - hi - mid, which has <= 8 significant bits and so is exact in bf16).
// The product x*w is the sum of the 9 cross products; the 3 dropped ones (mid*lo, lo*mid, lo*lo) are
// below 2^-24 |x w|, i.e. under fp32's own rounding of the product. Six v_mfma_f32_32x32x16_bf16
// (products exact in fp32, fp32 accumulation) therefore give an fp32-accurate conv at 6 x 16 cycles
// per 32x32x16 block against 8 x 64 cycles (32x32x2 f32) for the same block on the fp32 MFMA:
// 2.67x the fp32 matrix peak (2.5 PF / 6 = 419 TF of fp32-equivalent work).
//
// Layout (16-byte units = 8 bf16 channels):
//  * LDS activations [plane][h][src row][src col]: h = which 8 of the chunk's 16 input channels.
//    The A operand of lane l (pixel l&31, channels 8(l>>5)..+7) is one ds_read_b128; 32 lanes read
//    32 consecutive 16-B units per half -> conflict-free under the b128 lane grouping.
//  * LDS weights [plane][tap][h][co]: the B operand of lane l (channel l&31) likewise.
//  * global weight pack (after the fp32 pack, see ast_conv3x3_packed_numel):
//    [chunk of 16 ci][plane][tap][h][cout_pad][8] bf16, so a chunk's slab rows are contiguous.
// The source tile (with halo, zero / reflect padding and the x2 nearest upsample resolved per
// pixel, as in the fp32 kernel) is gathered with dword loads coalesced along x, split on the VALU
// and written once per chunk; the next chunk's loads are in flight during the MFMAs.
// ------------------------------------------------------------------------------------------------
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 struct defeats SROA: scratch)

constexpr int kX3K = 16;  // input channels per chunk (= the MFMA K)
#ifndef X3_STAGED_EPI
#define X3_STAGED_EPI 1  // epilogue through LDS (store_tiles_staged); 0 = direct stores (A/B)
#endif

__host__ __device__ constexpr int64_t x3_split_offset(int cin, int cout) {  // floats before the split part
  return (int64_t)((cin + 7) / 8 * 8) * 9 * ((cout + 63) / 64 * 64);
}

// x = hi + mid + lo exactly for finite x. A finite |x| above bf16's largest value (3.3895e38) would
// round hi to inf: hi is clamped to that largest value instead, and the remainder stays exact.
// Non-finite x: hi = x, mid = lo = 0. The MFMA also multiplies hi by the weight's mid and lo terms,
// which are often exactly 0, so an output reached by an inf input is +-inf (as torch's inf * w) or
// NaN; NaN inputs give NaN, as in torch. tests/test_gpu_parity.py pins both behaviours.
__device__ __forceinline__ void split3(float x, bf16& hi, bf16& mid, bf16& lo) {
  const bool finite = fabsf(x) <= 3.402823466e38f;
  hi = (bf16)x;
  if (finite && !(fabsf((float)hi) <= 3.402823466e38f)) hi = (bf16)copysignf(3.38953139e38f, x);
  float r = finite ? x - (float)hi : 0.f;
  mid = (bf16)r;
  lo = (bf16)(r - (float)mid);
}

// fp32 pack [ci_pad8][9][cout_pad] -> split pack [ci16 chunk][plane][tap][h][cout_pad][8]
__global__ void pack_x3_kernel(const float* __restrict__ wp, bf16* __restrict__ ws, int cin_pad8, int cin16,
                               int cout_pad) {
  const int64_t total = (int64_t)cin16 * 9 * cout_pad;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(idx % cout_pad);
    const int64_t rt = idx / cout_pad;
    const int tap = (int)(rt % 9);
    const int ci = (int)(rt / 9);
    const float v = ci < cin_pad8 ? wp[((int64_t)ci * 9 + tap) * cout_pad + co] : 0.f;
    bf16 t[3];
    split3(v, t[0], t[1], t[2]);
    const int kc = ci / kX3K, hh = (ci >> 3) & 1, e = ci & 7;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      ws[((((int64_t)(kc * 3 + p) * 9 + tap) * 2 + hh) * cout_pad + co) * 8 + e] = t[p];
  }
}

#ifndef X3_HS_PAD
#define X3_HS_PAD 1
#endif

template <int WM, int RM, int RN, int UP>
struct X3Cfg {
  static constexpr int NT = WM * 64;
  static constexpr int TH = WM * RM;                 // output rows per tile
  static constexpr int BN = RN * 32;                 // output channels per tile
  static constexpr int SR = TH / UP + 2;             // source rows incl. halo
  static constexpr int SC = TW / UP + 2;             // source columns incl. halo
  static constexpr int A_ITEMS = 2 * SR * SC;        // gather items: 16-B units of 8 channels, both halves
  // 16-B units per 8-channel half, padded to a multiple of 16 units (64 banks): the M16 A operand
  // reads both halves (and two planes) in one ds_read_b128, whose lane groups {0-3,12-15,20-27} /
  // {4-11,16-19,28-31} mix the halves -- unpadded (612 units = 16 banks apart) they collide on 16
  // banks per group (2-way, profiles/r04p: 22% of the LDS cycles were conflicts)
  static constexpr int HS = X3_HS_PAD ? (SR * SC + 15) / 16 * 16 : SR * SC;
  static constexpr int A_PLANE = 2 * HS;             // 16-B units per plane
  static constexpr int A_UNITS = 3 * A_PLANE;
  static constexpr int B_ROWS = 3 * 9 * 2;           // (plane, tap, h)
  static constexpr int B_UNITS = B_ROWS * BN;
  static constexpr int A_T = (A_ITEMS + NT - 1) / NT;  // gather items per thread (one item = 8 channels)
  static constexpr int B_T = (B_UNITS + NT - 1) / NT;
  static constexpr int NS = UP == 1 ? RM + 2 : RM / 2 + 2;  // source rows a wave's RM output rows read
  static constexpr int LDS_TILES = (A_UNITS + B_UNITS) * 16;
  // staged epilogue regions: the M16 and persistent kernels always stage through LDS, whatever
  // X3_STAGED_EPI (which only selects the 32x32 kernel's direct-store A/B form) says
  static constexpr int LDS_EPI = WM * 32 * RM * 36 * 4;
  static constexpr int LDS_BYTES = LDS_TILES > LDS_EPI ? LDS_TILES : LDS_EPI;
  // M16 kernel: A tile, the weight slab's lo plane, and its hi + mid planes twice (the next chunk's
  // arrive by LDS-DMA during the current chunk's MFMAs)
  static constexpr int LDS_TILES_M16 = (A_UNITS + 18 * BN + 2 * 36 * BN) * 16;
  static constexpr int LDS_BYTES_M16 = LDS_TILES_M16 > LDS_EPI ? LDS_TILES_M16 : LDS_EPI;
};

// source row (relative to the wave's first) of output row i at tap row ky
template <int UP>
__host__ __device__ constexpr int x3_srel(int i, int ky) { return UP == 1 ? i + ky : ((i + ky - 1) >> 1) + 1; }

// Epilogue through LDS (x3 kernel): in the MFMA layout a lane holds one output channel, so a
// direct float4 store scatters over 64 rows/planes per instruction (store-issue-bound). Each wave
// writes its accumulators (+bias) to its own LDS region [32 channels][RM rows][32 px + 4], then
// stores rows: 8 lanes per 128-byte run, pre-ReLU / ReLU / 2x2 max-pool as store_tiles. The
// caller's barrier must precede it (the region overlaps the operand tiles).
// Row stores of one 32-channel group from a wave's staged region [32 channels][RM rows][36 floats]
// (channel ch = output channel cbase + ch): pre-ReLU / ReLU float4 rows, 8 lanes per 128-byte run,
// and the fused 2x2 max-pool.
template <int RM>
__device__ __forceinline__ void store_region(const ConvArgs& a, const float* __restrict__ region, int n, int x0,
                                             int y0, int row0, int cbase, int lane) {
  constexpr int RP = 36;  // row pitch (floats): 32 px + 4
  const int H = a.H, W = a.W;
  const int64_t plane = (int64_t)H * W;
  const bool vec4 = (W & 3) == 0;
  const int Ho = H >> 1, Wo = W >> 1;
  if (a.y_pre || a.y_act) {
#pragma unroll
    for (int it = 0; it < 32 * RM * 8 / 64; ++it) {
      const int item = it * 64 + lane;
      const int q = item & 7, row = (item >> 3) % RM, ch = item / (8 * RM);
      const int co = cbase + ch, yy = y0 + row0 + row, xx = x0 + 4 * q;
      if (co >= a.Cout || yy >= H || xx >= W) continue;
      const float4 v = *reinterpret_cast<const float4*>(region + (ch * RM + row) * RP + 4 * q);
      const int64_t off = ((int64_t)n * a.Cout + co) * plane + (int64_t)yy * W + xx;
      const bool full = vec4 && xx + 3 < W;
      const float vv[4] = {v.x, v.y, v.z, v.w};
      if (dgrad_epi(a)) {  // input gradient: y_pre only
        if (full) *reinterpret_cast<float4*>(a.y_pre + off) = dgrad_epi4(a, v, off);
        else for (int r = 0; r < 4; ++r) if (xx + r < W) a.y_pre[off + r] = dgrad_epi_one(a, vv[r], off + r);
        continue;
      }
      if (a.y_pre) {
        if (full) *reinterpret_cast<float4*>(a.y_pre + off) = v;
        else for (int r = 0; r < 4; ++r) if (xx + r < W) a.y_pre[off + r] = vv[r];
      }
      if (a.y_act) {
        const float4 u = make_float4(relu_f(v.x), relu_f(v.y), relu_f(v.z), relu_f(v.w));
        if (full) *reinterpret_cast<float4*>(a.y_act + off) = u;
        else for (int r = 0; r < 4; ++r) if (xx + r < W) a.y_act[off + r] = relu_f(vv[r]);
      }
    }
  }
  if (a.y_pool) {
#pragma unroll
    for (int it = 0; it < 32 * (RM / 2) * 8 / 64; ++it) {
      const int item = it * 64 + lane;
      const int q = item & 7, prow = (item >> 3) % (RM / 2), ch = item / (8 * (RM / 2));
      const int co = cbase + ch, py = (y0 + row0) / 2 + prow, px = (x0 + 4 * q) >> 1;
      if (co >= a.Cout || py >= Ho || px >= Wo) continue;
      const float4 r0 = *reinterpret_cast<const float4*>(region + (ch * RM + 2 * prow) * RP + 4 * q);
      const float4 r1 = *reinterpret_cast<const float4*>(region + (ch * RM + 2 * prow + 1) * RP + 4 * q);
      const int64_t off = ((int64_t)n * a.Cout + co) * Ho * Wo + (int64_t)py * Wo + px;
      float p0, p1;
      if (a.e_sum2) {  // nearest-upsample adjoint: the window's sum, row by row (pad_up_adjoint's order)
        p0 = dgrad_epi_one(a, ((r0.x + r0.y) + r1.x) + r1.y, off);
        p1 = px + 1 < Wo ? dgrad_epi_one(a, ((r0.z + r0.w) + r1.z) + r1.w, off + 1) : 0.f;
      } else {
        const float m0 = max_nan(relu_f(r0.x), relu_f(r1.x)), m1 = max_nan(relu_f(r0.y), relu_f(r1.y));
        const float m2 = max_nan(relu_f(r0.z), relu_f(r1.z)), m3 = max_nan(relu_f(r0.w), relu_f(r1.w));
        p0 = max_nan(m0, m1);
        p1 = max_nan(m2, m3);
      }
      if (px + 1 < Wo && (Wo & 1) == 0) {
        *reinterpret_cast<float2*>(a.y_pool + off) = make_float2(p0, p1);
      } else {
        a.y_pool[off] = p0;
        if (px + 1 < Wo) a.y_pool[off + 1] = p1;
      }
    }
  }
}

template <int RM, int RN>
__device__ __forceinline__ void store_tiles_staged(const ConvArgs& a, const f32x16 (&acc)[RM][RN], int n, int x0,
                                                   int y0, int row0, int n0c, int h, int l32, int lane,
                                                   float* __restrict__ region) {
  constexpr int RP = 36;  // row pitch (floats): 32 px + 4
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    {
      const int co = n0c + j * 32 + l32;
      const float bv = (co < a.Cout && a.bias) ? a.bias[co] : 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(region + (l32 * RM + i) * RP + 8 * g + 4 * h) =
              make_float4(acc[i][j][4 * g] + bv, acc[i][j][4 * g + 1] + bv, acc[i][j][4 * g + 2] + bv,
                          acc[i][j][4 * g + 3] + bv);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    store_region<RM>(a, region, n, x0, y0, row0, n0c + j * 32, lane);
    if (j + 1 < RN) {
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();  // reads of this j done before the next j's writes
    }
  }
}

// Diagnostic build only (X3_STAMP=1, scripts/build_variants.sh; never the product library): every
// wave of the first X3_STAMP_WGS workgroups records the shader-clock counter at its phase boundaries
// (entry, prologue done, and per K chunk: loads issued / MFMAs done / first barrier / store + second
// barrier; epilogue start / end) in three VGPRs (lane k holds stamp k), stored once at the end to
// x3_stamp_buf, which no other code reads; scripts/x3_stamps.py reads it back.
#ifndef X3_STAMP
#define X3_STAMP 0
#endif
#if X3_STAMP
constexpr int kX3StampWgs = 2048, kX3StampRec = 200;
__device__ unsigned x3_stamp_buf[kX3StampWgs * 16 * kX3StampRec];
#define X3_ST(IDX)                                                                  \
  {                                                                                 \
    const unsigned t_ = (unsigned)__builtin_readcyclecounter();                     \
    const int i_ = (IDX);                                                           \
    st0 = lane == i_ ? t_ : st0;                                                    \
    st1 = lane == i_ - 64 ? t_ : st1;                                               \
    st2 = lane == i_ - 128 ? t_ : st2;                                              \
  }
#define X3_ST_STEP(KC, NCH, ST)                                                        \
  if ((KC) == 5) X3_ST(4 + 4 * (NCH) + (ST))  /* per-step stamps of chunk 5 */
#else
#define X3_ST(IDX)
#define X3_ST_STEP(KC, NCH, ST)
#endif

// M16: the same kernel on v_mfma_f32_16x16x32_bf16 (16 pixels x 16 output channels x K 32). The six
// split products fold into three K-32 MFMAs -- K = (16 channels of one term | 16 of another):
//   [x_hi | x_mid] . [w_hi ; w_hi]  = x_hi w_hi  + x_mid w_hi
//   [x_hi | x_lo ] . [w_mid; w_hi]  = x_hi w_mid + x_lo w_hi
//   [x_hi | x_mid] . [w_lo ; w_mid] = x_hi w_lo  + x_mid w_mid
// -- the same products and cycles per FLOP as the 32x32x16 form; on random data the chip holds a
// higher clock with the 16x16 shape (MI355X_MICROARCH.md, DVFS give-back item 7). A lane's k-group
// g = lane >> 4 selects the term plane (g < 2: the first, else the second) and the 8-channel half
// (g & 1), so every operand is still one ds_read_b128 from the same LDS images.
// PER (M16 only): persistent form -- gridDim.x workgroups walk the blocks b = blockIdx.x + k gridDim.x
// (gridDim.x a multiple of 8, so b % 8 and the XCD stay fixed), the same code per block; between
// blocks an LDS-only barrier (the epilogue regions are read before the next prologue writes the
// tiles), so the epilogue's global stores drain under the next block's prologue instead of
// holding the CU until the workgroup retires.
template <int WM, int RM, int RN, int UP, int OCC, bool M16 = false, bool PER = false>
__global__ __launch_bounds__(WM * 64, OCC) void conv3x3_x3_kernel(ConvArgs a) {
  using C = X3Cfg<WM, RM, RN, UP>;
  constexpr int NT = C::NT, TH = C::TH, BN = C::BN, SR = C::SR, SC = C::SC, A_PLANE = C::A_PLANE;
  constexpr int HS = C::HS, A_ITEMS = C::A_ITEMS;
  constexpr int A_T = C::A_T, B_T = C::B_T, NS = C::NS;
  static_assert(RM % 2 == 0, "even rows per wave (pool windows, upsample row pairs)");
  extern __shared__ __attribute__((aligned(16))) u32x4 x3_smem[];
  u32x4* As = x3_smem;
  u32x4* Bs = x3_smem + C::A_UNITS;
  // M16: [lo plane][hi + mid planes, buffer 0][hi + mid planes, buffer 1] after the A tile
  u32x4* Blo = x3_smem + C::A_UNITS;
  u32x4* Bhm0 = Blo + 18 * BN;

#if X3_STAMP
  unsigned st0 = 0, st1 = 0, st2 = 0;
  X3_ST(0);
#endif
  static_assert(!PER || M16, "persistent form of the M16 kernel only");
  const int ntl = a.tiles_x * a.tiles_y * a.N, ngr = (a.Cout + BN - 1) / BN;
  const int nblk = (ntl + 7) / 8 * 8 * ngr;
  for (int bid = blockIdx.x;; bid += gridDim.x) {
  if constexpr (PER) {
    if (bid >= nblk) break;
    if (bid != (int)blockIdx.x) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // PER: the thread index laundered per block, so nothing derived from it is hoisted out of the
  // block loop and held live through it (that spilled 60-80 VGPRs); recomputing is a few VALU ops
  int tid_ = threadIdx.x;
  if constexpr (PER) asm volatile("" : "+v"(tid_));
  const int tid = tid_, wm = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  int t, grp;
  if (!decode_block(bid, ntl, ngr, t, grp)) {
    if constexpr (PER) continue;
    return;
  }
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  const int n = t / a.tiles_y;
  const int x0 = tx * TW, y0 = ty * TH;
  const int sx0 = x0 / UP, sy0 = y0 / UP - 1;
  const int n0 = grp * BN;
  const int Hin = a.Hin, Win = a.Win, plane_in = Hin * Win;
  const float* __restrict__ xin =
      n < a.nsplit ? a.x + (int64_t)n * a.Cin * plane_in : a.x2 + (int64_t)(n - a.nsplit) * a.Cin * plane_in;
  const u32x4* __restrict__ wsplit =
      reinterpret_cast<const u32x4*>(a.wp + x3_split_offset(a.Cin, a.Cout));
  const int nch = (a.Cin + kX3K - 1) / kX3K;
  const int64_t chunk_units = (int64_t)C::B_ROWS * a.cout_pad;

  // gather items: (h, source row, source column), fixed per thread for every chunk. Loads are
  // raw buffer loads: per-chunk descriptor (wave-uniform), per-item 32-bit voffset (pixel + 8h
  // channels), channel j in soffset: no per-load address arithmetic. A zero-padding pixel gets an
  // out-of-range voffset, which the buffer range check turns into 0.
  unsigned g_off[A_T], g_pix[A_T];
  int g_lds[A_T], g_h[A_T];
  bool g_ok[A_T];
#pragma unroll
  for (int i = 0; i < A_T; ++i) {
    const int e = min(tid + i * NT, A_ITEMS - 1);
    const int c = e % SC, rest = e / SC, r = rest % SR, hh = rest / SR;
    const int sy = src_index<UP>(sy0 + r, Hin, a.reflect), sx = src_index<UP>(sx0 - 1 + c, Win, a.reflect);
    g_ok[i] = sy >= 0 && sx >= 0;
    g_pix[i] = (unsigned)(max(sy, 0) * Win + max(sx, 0));
    g_off[i] = g_ok[i] ? 4u * (unsigned)(8 * hh * plane_in) + 4u * g_pix[i] : 0x7ffffff0u;
    g_lds[i] = hh * HS + r * SC + c;
    g_h[i] = hh;
  }
  const int plane_b = 4 * plane_in;
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<u32x4*>(wsplit), 0, (int)min<int64_t>(0x7fffffff, (int64_t)nch * chunk_units * 16), 0x00020000);
  int b_src[B_T], b_dst[B_T];
#pragma unroll
  for (int i = 0; i < B_T; ++i) {
    const int u = min(tid + i * NT, C::B_UNITS - 1), row = u / BN, j = u - row * BN;
    b_src[i] = 16 * (row * a.cout_pad + n0 + j);
    b_dst[i] = u;
  }
  float ra[A_T][8];
  u32x4 rb[M16 ? 1 : B_T];
  bf16x8 pv[M16 ? A_T : 1][3];
  // channel ci0 + 8h + j of item i; a partial last chunk clamps the channel (values masked at store)
#define X3_LOAD_A(KC, I0, I1)                                                                           \
  {                                                                                                     \
    const int ci0 = (KC) * kX3K;                                                                        \
    if (ci0 + kX3K <= a.Cin) {                                                                          \
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(                              \
          const_cast<float*>(xin + (int64_t)ci0 * plane_in), 0, kX3K * plane_b, 0x00020000);           \
      _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                     \
        _Pragma("unroll") for (int i = (I0); i < (I1); ++i)                                             \
          ra[i][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)g_off[i], j * plane_b, 0)); \
    } else {                                                                                            \
      _Pragma("unroll") for (int i = (I0); i < (I1); ++i)                                               \
        _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                   \
          ra[i][j] = xin[(int64_t)min(ci0 + 8 * g_h[i] + j, a.Cin - 1) * plane_in + g_pix[i]];          \
    }                                                                                                   \
  }
#define X3_LOAD_B(KC)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < (M16 ? 0 : B_T); ++i)                                           \
    rb[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, b_src[i], (int)((KC) * chunk_units * 16), 0));
  // M16: the weight slab goes global -> LDS by LDS-DMA (global_load_lds_dwordx4, one lane-linear
  // 1-KiB piece of the slab per wave-instruction, no VGPRs and no ds_write), issued right after the
  // barrier that frees Bs; the barrier after the A tile's writes waits for it (vmcnt(0))
  // slab rows (plane, tap, half): hi + mid planes = rows 0-35, lo plane = rows 36-53
  static_assert((36 * BN) % 64 == 0 && (18 * BN) % 64 == 0, "whole 1-KiB pieces");
  constexpr int HM_PIECES = 36 * BN / 64, LO_PIECES = 18 * BN / 64;
#define X3_DMA_ROWS(KC, ROW0, NPIECES, DST)                                                             \
  _Pragma("unroll") for (int i = 0; i < ((NPIECES) + WM - 1) / WM; ++i) {                               \
    const int piece = wm + i * WM;                                                                      \
    if (piece < (NPIECES)) {                                                                            \
      const int u = piece * 64 + lane, row = u / BN, j = u - row * BN;                                  \
      const u32x4* src = wsplit + (int64_t)(KC) * chunk_units + (int64_t)((ROW0) + row) * a.cout_pad + n0 + j; \
      __builtin_amdgcn_global_load_lds((const void*)src,                                                \
                                       (__attribute__((address_space(3))) void*)((DST) + piece * 64), 16, 0, 0); \
    }                                                                                                   \
  }
#define X3_DMA_HM(KC) X3_DMA_ROWS(KC, 0, HM_PIECES, Bhm0 + ((KC) & 1) * 36 * BN)
#define X3_DMA_LO(KC) X3_DMA_ROWS(KC, 36, LO_PIECES, Blo)
  // M16: the gathered x split into its term planes in registers (before the barrier, in the slack of
  // a wave that finished its MFMAs early), written after it
#define X3_SPLIT_A(KC)                                                                                  \
  _Pragma("unroll") for (int i = 0; i < A_T; ++i) {                                                     \
    if ((KC) * kX3K + kX3K > a.Cin) { /* partial last chunk: padding and channels past Cin */            \
      const int cn = a.Cin - (KC) * kX3K - 8 * g_h[i];                                                  \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) ra[i][j] = (g_ok[i] && j < cn) ? ra[i][j] : 0.f;     \
    }                                                                                                   \
    ast_x3::split8(ra[i], pv[i][0], pv[i][1], pv[i][2]);                                                \
  }
#define X3_WRITE_A                                                                                      \
  _Pragma("unroll") for (int i = 0; i < A_T; ++i)                                                       \
    if (tid + i * NT < A_ITEMS)                                                                         \
      _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                     \
        As[p * A_PLANE + g_lds[i]] = __builtin_bit_cast(u32x4, pv[i][p]);
#define X3_LOAD(KC)         \
  {                         \
    X3_LOAD_A(KC, 0, A_T);  \
    X3_LOAD_B(KC);          \
  }
  // split into the three term planes (ast_x3::split8: paired conversions, bit-identical to split3)
#define X3_STORE(KC)                                                                                    \
  {                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < A_T; ++i) {                                                   \
      if (tid + i * NT < A_ITEMS) {                                                                     \
        if ((KC) * kX3K + kX3K > a.Cin) { /* partial last chunk: padding and channels past Cin */        \
          const int cn = a.Cin - (KC) * kX3K - 8 * g_h[i];                                              \
          _Pragma("unroll") for (int j = 0; j < 8; ++j) ra[i][j] = (g_ok[i] && j < cn) ? ra[i][j] : 0.f; \
        }                                                                                               \
        bf16x8 pv[3];                                                                                   \
        ast_x3::split8(ra[i], pv[0], pv[1], pv[2]);                                                     \
        _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                   \
          As[p * A_PLANE + g_lds[i]] = __builtin_bit_cast(u32x4, pv[p]);                                \
      }                                                                                                 \
    }                                                                                                   \
    _Pragma("unroll") for (int i = 0; i < B_T; ++i)                                                     \
      if (tid + i * NT < C::B_UNITS) Bs[b_dst[i]] = rb[i];                                              \
  }

  constexpr int Q = 2 * RN;  // M16: 16-channel column tiles per wave
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  f32x16 acc[M16 ? 1 : RM][M16 ? 1 : RN];
  f32x4v acc16[M16 ? RM : 1][M16 ? 2 : 1][M16 ? Q : 1];
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int q = 0; q < Q; ++q) acc16[i][pt][q] = f32x4v{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }

  int acol[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) acol[kx] = ((x0 + l32 + kx - 1) >> (UP - 1)) - sx0 + 1;
  const int srow0 = wm * RM / UP;
  // M16 lane roles: pixel / channel l16 of a 16-tile, k-group g16 -> (term plane, 8-channel half)
  const int l16 = lane & 15, g16 = lane >> 4, hh16 = g16 & 1;
  int acol16[2][3];
#pragma unroll
  for (int pt = 0; pt < 2; ++pt)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) acol16[pt][kx] = ((x0 + 16 * pt + l16 + kx - 1) >> (UP - 1)) - sx0 + 1;
  const int apl1 = (g16 < 2 ? 0 : 1) * A_PLANE, apl2 = (g16 < 2 ? 0 : 2) * A_PLANE;  // [hi|mid], [hi|lo]

  if constexpr (M16) {
    X3_DMA_HM(0);
    X3_DMA_LO(0);
    X3_LOAD_A(0, 0, A_T);
    X3_SPLIT_A(0);
    X3_WRITE_A;
  } else {
    X3_LOAD(0);
    X3_STORE(0);
  }
  __syncthreads();
  X3_ST(1);
  static_assert(A_T < 9, "one gather item per tap of the MFMA phase");
  for (int kc = 0; kc < nch; ++kc) {
    if (!M16 && kc + 1 < nch) X3_LOAD(kc + 1);
    __builtin_amdgcn_sched_barrier(0);
    X3_ST(2 + 4 * kc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (M16) {
      // Software-pipelined MFMA phase (round 5): steps s = (kx, ky, row i), kx outermost; the LDS operands of step s + 1 (its A fragments and, when it opens a
      // tap, the tap's B fragments) are read while step s's MFMAs run. The stamps showed the wave
      // that finishes a chunk last, alone on its SIMD, issuing MFMAs at ~70% of the pipe rate: each
      // step waited on reads issued just before it (profiles/r05_x3_stamps.txt). Same products in
      // the same order per accumulator as the round-4 loop: bit-identical.
      constexpr int NSTEP = 9 * RM;
      bf16x8 gb[2][3][Q];  // B fragments (g1, g2, g3) of a tap, by tap parity
      bf16x8 fa[2][2][2];  // A fragments (f1, f2) x pixel tile of a step, by step parity
      // this chunk's B planes: g1 = [hi; hi], g2 = [mid | hi; hi], g3 = [lo; mid] by k-group
      const u32x4* __restrict__ bhm = Bhm0 + (kc & 1) * 36 * BN;
      const u32x4* __restrict__ bp1 = bhm;                                         // hi
      const u32x4* __restrict__ bp2 = bhm + (g16 < 2 ? 18 * BN : 0);               // mid | hi
      const u32x4* __restrict__ bp3 = g16 < 2 ? Blo : bhm + 18 * BN;               // lo | mid
#define X3P_READ_B(BUF, T)                                                                              \
      {                                                                                                 \
        const int tap_ = ((T) % 3) * 3 + (T) / 3;                                                       \
        _Pragma("unroll") for (int q = 0; q < Q; ++q) {                                                 \
          const int col = q * 16 + l16;                                                                 \
          gb[BUF][0][q] = __builtin_bit_cast(bf16x8, bp1[(tap_ * 2 + hh16) * BN + col]);               \
          gb[BUF][1][q] = __builtin_bit_cast(bf16x8, bp2[(tap_ * 2 + hh16) * BN + col]);               \
          gb[BUF][2][q] = __builtin_bit_cast(bf16x8, bp3[(tap_ * 2 + hh16) * BN + col]);               \
        }                                                                                               \
      }
#define X3P_READ_A(BUF, S)                                                                              \
      {                                                                                                 \
        const int t_ = (S) / RM, i_ = (S) % RM, kx_ = t_ / 3, ky_ = t_ % 3;                             \
        const int srow = hh16 * HS + (srow0 + x3_srel<UP>(i_, ky_)) * SC;                               \
        _Pragma("unroll") for (int pt = 0; pt < 2; ++pt) {                                              \
          fa[BUF][0][pt] = __builtin_bit_cast(bf16x8, As[apl1 + srow + acol16[pt][kx_]]);               \
          fa[BUF][1][pt] = __builtin_bit_cast(bf16x8, As[apl2 + srow + acol16[pt][kx_]]);               \
        }                                                                                               \
      }
      X3P_READ_B(0, 0);
      X3P_READ_A(0, 0);
#pragma unroll
      for (int st = 0; st < NSTEP; ++st) {
        const int t = st / RM, i = st % RM, sb = st & 1, tb = t & 1;
        X3_ST_STEP(kc, nch, st);
        // the next chunk's global loads, spread over the first taps (one gather item per tap):
        // issued all at once they queued behind the CU's memory pipeline for ~3k cycles per chunk
        // with no MFMA issued (scripts/x3_stamps.py, profiles/r05_x3_stamps.txt)
        if (i == 0 && t < A_T && kc + 1 < nch) {
          __builtin_amdgcn_sched_barrier(0);
          X3_LOAD_A(kc + 1, t, t + 1)
          __builtin_amdgcn_sched_barrier(0);
        }
        // the next chunk's hi + mid weight planes into the other buffer (LDS-DMA, no VGPRs)
        if (i == 0 && t == A_T && kc + 1 < nch) {
          __builtin_amdgcn_sched_barrier(0);
          X3_DMA_HM(kc + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        int nrd = 0;
        if (st + 1 < NSTEP) {
          X3P_READ_A(sb ^ 1, st + 1);
          nrd = 4;
          if ((st + 1) % RM == 0) {
            X3P_READ_B(tb ^ 1, (st + 1) / RM);
            nrd += 3 * Q;
          }
        }
        // the three products of an accumulator in the same order, but product-major: 2Q
        // independent MFMAs separate each from the next one on the same accumulator
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int q = 0; q < Q; ++q)
            acc16[i][pt][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[sb][0][pt], gb[tb][2][q], acc16[i][pt][q], 0, 0, 0);
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int q = 0; q < Q; ++q)
            acc16[i][pt][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[sb][1][pt], gb[tb][1][q], acc16[i][pt][q], 0, 0, 0);
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int q = 0; q < Q; ++q)
            acc16[i][pt][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[sb][0][pt], gb[tb][0][q], acc16[i][pt][q], 0, 0, 0);
        // one LDS read per MFMA while the next step's reads last, then the rest of the MFMAs
#pragma unroll
        for (int r = 0; r < nrd; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        if (nrd == 4) __builtin_amdgcn_sched_group_barrier(0x008, 6 * Q - 4, 0);
        else if (nrd == 4 + 3 * Q) __builtin_amdgcn_sched_group_barrier(0x008, 3 * Q - 4, 0);
        else __builtin_amdgcn_sched_group_barrier(0x008, 6 * Q, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
#undef X3P_READ_A
#undef X3P_READ_B
    } else {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        bf16x8 bfr[3][RN][3];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p)
              bfr[ky][j][p] = __builtin_bit_cast(bf16x8, Bs[((p * 9 + ky * 3 + kx) * 2 + h) * BN + j * 32 + l32]);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          bf16x8 af[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            af[p] = __builtin_bit_cast(bf16x8, As[p * A_PLANE + h * HS + (srow0 + s) * SC + acol[kx]]);
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
              if (x3_srel<UP>(i, ky) != s) continue;
#pragma unroll
              for (int j = 0; j < RN; ++j) {
                f32x16 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], bfr[ky][j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[ky][j][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bfr[ky][j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bfr[ky][j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[ky][j][1], c, 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[ky][j][0], c, 0, 0, 0);
              }
            }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    X3_ST(3 + 4 * kc);
    if (kc + 1 < nch) {
      if constexpr (M16) {
        X3_SPLIT_A(kc + 1);
        __syncthreads();  // every wave is done reading this chunk
        X3_ST(4 + 4 * kc);
        X3_DMA_LO(kc + 1);
        X3_WRITE_A;
      } else {
        __syncthreads();  // every wave is done reading this chunk
        X3_ST(4 + 4 * kc);
        X3_STORE(kc + 1);
      }
      __syncthreads();
      X3_ST(5 + 4 * kc);
    }
  }
#undef X3_LOAD
#undef X3_LOAD_A
#undef X3_LOAD_B
#undef X3_STORE
#undef X3_DMA_ROWS
#undef X3_DMA_HM
#undef X3_DMA_LO
#undef X3_SPLIT_A
#undef X3_WRITE_A
  if constexpr (M16) {
    // staged epilogue, 32 channels (two 16-tiles) per pass: lane (l16, g16) holds pixels 16 pt + 4 g16
    // + r of channel 16 q + l16 -> one float4 per (row, pixel tile) into the region
    __syncthreads();  // every wave is done reading the last chunk's tiles
    X3_ST(2 + 4 * nch);
    float* region = reinterpret_cast<float*>(x3_smem) + wm * 32 * RM * 36;
    // ReLU + 2x2 max-pool as the only output (the encoder's pool layers in config 2): pooled in
    // registers -- a lane holds both rows of its windows (acc16[2pr], acc16[2pr + 1]) and 4
    // consecutive pixels -- with no LDS round trip. One exchange with lane ^ 16 gives every lane 4
    // consecutive pooled pixels: even g16 its own pair and the partner's of tile pt = 0, odd g16 the
    // partner's and its own of pt = 1, so the 4 lanes of a channel store its 16 pooled pixels as one
    // 64-byte run (store_region's granularity). Same max_nan order as store_region: bit-identical.
    if (a.y_pool && !a.y_pre && !a.y_act && !a.e_sum2 && !dgrad_epi(a)) {
      const int Ho = a.H >> 1, Wo = a.W >> 1;
      const bool odd = g16 & 1;
      const int pc = (x0 >> 1) + (odd ? 8 + 2 * (g16 - 1) : 2 * g16);
      const bool vec = (Wo & 3) == 0 && pc + 3 < Wo;
#pragma unroll
      for (int q = 0; q < 2 * RN; ++q) {
        const int co = n0 + 16 * q + l16;
        const float bv = (co < a.Cout && a.bias) ? a.bias[co] : 0.f;
#pragma unroll
        for (int pr = 0; pr < RM / 2; ++pr) {
          float pv[2][2];
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) {
            const f32x4v r0 = acc16[2 * pr][pt][q], r1 = acc16[2 * pr + 1][pt][q];
            const float m0 = max_nan(relu_f(r0[0] + bv), relu_f(r1[0] + bv));
            const float m1 = max_nan(relu_f(r0[1] + bv), relu_f(r1[1] + bv));
            const float m2 = max_nan(relu_f(r0[2] + bv), relu_f(r1[2] + bv));
            const float m3 = max_nan(relu_f(r0[3] + bv), relu_f(r1[3] + bv));
            pv[pt][0] = max_nan(m0, m1);
            pv[pt][1] = max_nan(m2, m3);
          }
          const float e0 = __shfl_xor(odd ? pv[0][0] : pv[1][0], 16, 64);
          const float e1 = __shfl_xor(odd ? pv[0][1] : pv[1][1], 16, 64);
          const float o[4] = {odd ? e0 : pv[0][0], odd ? e1 : pv[0][1], odd ? pv[1][0] : e0, odd ? pv[1][1] : e1};
          const int py = ((y0 + wm * RM) >> 1) + pr;
          if (co >= a.Cout || py >= Ho) continue;
          float* dst = a.y_pool + ((int64_t)n * a.Cout + co) * Ho * Wo + (int64_t)py * Wo + pc;
          if (vec) {
            *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (pc + k < Wo) dst[k] = o[k];
          }
        }
      }
    } else
#pragma unroll
    for (int j = 0; j < RN; ++j) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int q = 2 * j + qq, co = n0 + 16 * q + l16;
        const float bv = (co < a.Cout && a.bias) ? a.bias[co] : 0.f;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) {
            const f32x4v v = acc16[i][pt][q];
            *reinterpret_cast<float4*>(region + ((16 * qq + l16) * RM + i) * 36 + 16 * pt + 4 * g16) =
                make_float4(v[0] + bv, v[1] + bv, v[2] + bv, v[3] + bv);
          }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      store_region<RM>(a, region, n, x0, y0, wm * RM, n0 + 32 * j, lane);
      if (j + 1 < RN) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    }
#if X3_STAMP
    __builtin_amdgcn_s_waitcnt(0);  // the epilogue's stores have left (vmcnt 0)
    X3_ST(3 + 4 * nch);
    if (blockIdx.x < kX3StampWgs) {
      unsigned* rec = x3_stamp_buf + ((size_t)blockIdx.x * 16 + wm) * kX3StampRec;
      rec[lane] = st0;
      rec[64 + lane] = st1;
      rec[128 + lane] = st2;
      if (lane == 0) {
        rec[192] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID: wave, SIMD, CU, SE
        rec[193] = __builtin_amdgcn_s_getreg(20 | (3 << 11));   // HW_REG_XCC_ID
        rec[194] = blockIdx.x;
        rec[195] = nch;
        rec[196] = 0x57a3u;
      }
    }
#endif
  } else {
#if X3_STAGED_EPI
    __syncthreads();  // every wave is done reading the last chunk's tiles
    store_tiles_staged<RM, RN>(a, acc, n, x0, y0, wm * RM, n0, h, l32, lane,
                               reinterpret_cast<float*>(x3_smem) + wm * 32 * RM * 36);
#else
    store_tiles<RM, RN>(a, acc, n, x0, y0, wm * RM, n0, h, l32);
#endif
  }
  if constexpr (!PER) break;
  }  // block loop
}

// Persistent form of the M16 split-bf16 kernel (round 4). One workgroup per CU
// slot walks the blocks b = blockIdx.x + k * gridDim.x (same XCD for all of them: b % 8 is fixed,
// and decode_block keeps the output-channel groups of a pixel tile on one XCD), and per block:
//   * the NEXT block's first K-chunk (its gather and weight slab) is loaded during the current
//     block's last chunk of MFMAs, so no block starts with an unoverlapped gather;
//   * the epilogue's global stores are left in flight (LDS-only barriers after it), so the store
//     tail of one block runs under the next block's first MFMAs instead of holding the CU.
// Per block the arithmetic, k order and rounding are conv3x3_x3_kernel<M16>'s: bit-identical.
// Measured on config 2 (profiles/r04_conv_persistent.txt): 1-2 % SLOWER per dispatch than the
// one-block-per-workgroup form, also on grids of one block per slot, so the loss is per-block code
// (argument re-reads, per-block address recomputation), not the static block walk; opt-in only
// (AST_CONV_PERSIST=1 maps 28-31 to 32-35).
__device__ __forceinline__ void x3_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// The kernel's ConvArgs re-read from the kernarg segment at the point of use: the empty asm hides the
// pointer's provenance, so the compiler cannot hoist the argument loads out of the block loop and keep
// every field in SGPRs across it (the persistent loop otherwise runs out of SGPRs and spills).
// A wave-uniform pointer the divergence analysis cannot see as one (it is assigned under the block
// loop's control flow): pinned to SGPRs, so the buffer descriptors built from it need no
// readfirstlane loop per load.
__device__ __forceinline__ const float* x3p_uniform(const float* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ const ConvArgs& x3p_args() {
  auto p = __builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const ConvArgs*)p;
}

template <int WM, int RM, int RN, int UP, int OCC>
__global__ __launch_bounds__(WM * 64, OCC) void conv3x3_x3p_kernel(ConvArgs, int nblk) {
#define A_ x3p_args()
  using C = X3Cfg<WM, RM, RN, UP>;
  constexpr int NT = C::NT, TH = C::TH, BN = C::BN, SR = C::SR, SC = C::SC, A_PLANE = C::A_PLANE;
  constexpr int HS = C::HS, A_ITEMS = C::A_ITEMS;
  constexpr int A_T = C::A_T, B_T = C::B_T;
  constexpr int Q = 2 * RN;
  static_assert(RM % 2 == 0, "even rows per wave (pool windows, upsample row pairs)");
  extern __shared__ __attribute__((aligned(16))) u32x4 x3_smem[];
  u32x4* As = x3_smem;
  u32x4* Bs = x3_smem + C::A_UNITS;
  typedef float f32x4v __attribute__((ext_vector_type(4)));

  const int tid = threadIdx.x, wm = tid >> 6, lane = tid & 63;
  const int nch = (A_.Cin + kX3K - 1) / kX3K;

  // the blocks of this workgroup: b = blockIdx.x + k * gridDim.x; a padding block (tile >= ntiles)
  // is only ever followed by padding blocks, so the walk ends at the first one
#define X3P_DECODE(B, OK, X0, Y0, IMG, N0)                                                            \
  {                                                                                                 \
    int t_, grp_;                                                                                   \
    OK = (B) < nblk && decode_block((B), A_.tiles_x * A_.tiles_y * A_.N, (A_.Cout + BN - 1) / BN, t_, grp_);                                 \
    if (OK) {                                                                                       \
      X0 = (t_ % A_.tiles_x) * TW;                                                                   \
      t_ /= A_.tiles_x;                                                                              \
      Y0 = (t_ % A_.tiles_y) * TH;                                                                   \
      IMG = t_ / A_.tiles_y;                                                                           \
      N0 = grp_ * BN;                                                                               \
    }                                                                                               \
  }
  // gather state of the block whose chunks are being loaded
  unsigned g_off[A_T], g_pix[A_T];
  int g_lds[A_T], g_h[A_T];
  bool g_ok[A_T];
  int b_src[B_T];
  const float* __restrict__ xin = A_.x;
#define X3P_SETUP(X0, Y0, IMG, N0)                                                                   \
  {                                                                                                 \
    const int plane_in = (A_.Hin * A_.Win), Hin = A_.Hin, Win = A_.Win;                                \
    xin = x3p_uniform((IMG) < A_.nsplit ? A_.x + (int64_t)(IMG) * A_.Cin * plane_in                      \
                                     : A_.x2 + (int64_t)((IMG) - A_.nsplit) * A_.Cin * plane_in);        \
    const int sx0_ = (X0) / UP, sy0_ = (Y0) / UP - 1;                                               \
    int tv_ = tid; /* laundered: the per-thread item decode is redone here, not hoisted and spilled */ \
    asm volatile("" : "+v"(tv_));                                                                   \
    _Pragma("unroll") for (int i = 0; i < A_T; ++i) {                                               \
      const int e = min(tv_ + i * NT, A_ITEMS - 1);                                                 \
      const int c = e % SC, rest = e / SC, r = rest % SR, hh = rest / SR;                           \
      const int sy = src_index<UP>(sy0_ + r, Hin, A_.reflect), sx = src_index<UP>(sx0_ - 1 + c, Win, A_.reflect); \
      g_ok[i] = sy >= 0 && sx >= 0;                                                                 \
      g_pix[i] = (unsigned)(max(sy, 0) * Win + max(sx, 0));                                         \
      g_off[i] = g_ok[i] ? 4u * (unsigned)(8 * hh * plane_in) + 4u * g_pix[i] : 0x7ffffff0u;        \
      g_lds[i] = hh * HS + r * SC + c;                                                              \
      g_h[i] = hh;                                                                                  \
    }                                                                                               \
    _Pragma("unroll") for (int i = 0; i < B_T; ++i) {                                               \
      const int u = min(tv_ + i * NT, C::B_UNITS - 1), row = u / BN, j = u - row * BN;              \
      b_src[i] = 16 * (row * A_.cout_pad + (N0) + j);                                                \
    }                                                                                               \
  }
  float ra[A_T][8];
  u32x4 rb[B_T];
#define X3P_LOAD(KC)                                                                                    \
  {                                                                                                     \
    const int ci0 = (KC) * kX3K, plane_in = (A_.Hin * A_.Win), plane_b = 4 * plane_in;                       \
    const int64_t chunk_units = ((int64_t)C::B_ROWS * A_.cout_pad);                                                        \
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(                             \
        const_cast<float*>(A_.wp + x3_split_offset(A_.Cin, A_.Cout)), 0,                               \
        (int)min<int64_t>(0x7fffffff, (int64_t)nch * chunk_units * 16), 0x00020000);                   \
    if (ci0 + kX3K <= A_.Cin) {                                                                          \
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(                              \
          const_cast<float*>(xin + (int64_t)ci0 * plane_in), 0, kX3K * plane_b, 0x00020000);           \
      _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                     \
        _Pragma("unroll") for (int i = 0; i < A_T; ++i)                                                 \
          ra[i][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)g_off[i], j * plane_b, 0)); \
    } else {                                                                                            \
      _Pragma("unroll") for (int i = 0; i < A_T; ++i)                                                   \
        _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                   \
          ra[i][j] = xin[(int64_t)min(ci0 + 8 * g_h[i] + j, A_.Cin - 1) * plane_in + g_pix[i]];          \
    }                                                                                                   \
    _Pragma("unroll") for (int i = 0; i < B_T; ++i)                                                     \
      rb[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, b_src[i], (int)((KC) * chunk_units * 16), 0)); \
  }
#define X3P_STORE(KC)                                                                                   \
  {                                                                                                     \
    const ConvArgs& ka_ = x3p_args(); /* one laundered argument pointer per expansion */                \
    _Pragma("unroll") for (int i = 0; i < A_T; ++i) {                                                   \
      if (tid + i * NT < A_ITEMS) {                                                                     \
        if ((KC) * kX3K + kX3K > ka_.Cin) {                                                               \
          const int cn = ka_.Cin - (KC) * kX3K - 8 * g_h[i];                                              \
          _Pragma("unroll") for (int j = 0; j < 8; ++j) ra[i][j] = (g_ok[i] && j < cn) ? ra[i][j] : 0.f; \
        }                                                                                               \
        bf16x8 pv[3];                                                                                   \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                 \
          bf16 t0, t1, t2;                                                                              \
          split3(ra[i][j], t0, t1, t2);                                                                 \
          pv[0][j] = t0;                                                                                \
          pv[1][j] = t1;                                                                                \
          pv[2][j] = t2;                                                                                \
        }                                                                                               \
        _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                   \
          As[p * A_PLANE + g_lds[i]] = __builtin_bit_cast(u32x4, pv[p]);                                \
      }                                                                                                 \
    }                                                                                                   \
    _Pragma("unroll") for (int i = 0; i < B_T; ++i)                                                     \
      if (tid + i * NT < C::B_UNITS) Bs[tid + i * NT] = rb[i];                                          \
  }

  int b = blockIdx.x, x0 = 0, y0 = 0, n = 0, n0 = 0;
  bool ok;
  X3P_DECODE(b, ok, x0, y0, n, n0);
  if (!ok) return;  // uniform: the whole workgroup
  X3P_SETUP(x0, y0, n, n0);
  X3P_LOAD(0);
  X3P_STORE(0);
  x3_lds_barrier();
  while (true) {
    const int b2 = b + gridDim.x;
    int nx0 = 0, ny0 = 0, nn = 0, nn0 = 0;
    bool has_next;
    X3P_DECODE(b2, has_next, nx0, ny0, nn, nn0);
    // the MFMA loop's LDS addresses derive from lane values laundered per block, so they are
    // recomputed here rather than hoisted out of the block loop and held live through the epilogue
    int lv = lane, wv = wm;
    asm volatile("" : "+v"(lv), "+v"(wv));
    const int ml16 = lv & 15, mg16 = lv >> 4, mhh16 = mg16 & 1;
    const int apl1 = (mg16 < 2 ? 0 : 1) * A_PLANE, apl2 = (mg16 < 2 ? 0 : 2) * A_PLANE;  // [hi|mid], [hi|lo]
    const int bpl1 = 0, bpl2 = mg16 < 2 ? 1 : 0, bpl3 = mg16 < 2 ? 2 : 1;              // [hi;hi], [mid;hi], [lo;mid]
    const int srow0 = wv * RM / UP;
    int acol16[2][3];
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) acol16[pt][kx] = ((x0 + 16 * pt + ml16 + kx - 1) >> (UP - 1)) - x0 / UP + 1;
    f32x4v acc16[RM][2][Q];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int q = 0; q < Q; ++q) acc16[i][pt][q] = f32x4v{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < nch; ++kc) {
      if (kc + 1 < nch) X3P_LOAD(kc + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int tap = ky * 3 + kx;
          bf16x8 g1[Q], g2[Q], g3[Q];
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int col = q * 16 + ml16;
            g1[q] = __builtin_bit_cast(bf16x8, Bs[((bpl1 * 9 + tap) * 2 + mhh16) * BN + col]);
            g2[q] = __builtin_bit_cast(bf16x8, Bs[((bpl2 * 9 + tap) * 2 + mhh16) * BN + col]);
            g3[q] = __builtin_bit_cast(bf16x8, Bs[((bpl3 * 9 + tap) * 2 + mhh16) * BN + col]);
          }
#pragma unroll
          for (int i = 0; i < RM; ++i) {
            const int srow = mhh16 * HS + (srow0 + x3_srel<UP>(i, ky)) * SC;
            bf16x8 f1[2], f2[2];
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
              f1[pt] = __builtin_bit_cast(bf16x8, As[apl1 + srow + acol16[pt][kx]]);
              f2[pt] = __builtin_bit_cast(bf16x8, As[apl2 + srow + acol16[pt][kx]]);
            }
            // the three products of an accumulator in the same order, but product-major: 2Q
            // independent MFMAs separate each from the next one on the same accumulator
#pragma unroll
            for (int pt = 0; pt < 2; ++pt)
#pragma unroll
              for (int q = 0; q < Q; ++q)
                acc16[i][pt][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[pt], g3[q], acc16[i][pt][q], 0, 0, 0);
#pragma unroll
            for (int pt = 0; pt < 2; ++pt)
#pragma unroll
              for (int q = 0; q < Q; ++q)
                acc16[i][pt][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f2[pt], g2[q], acc16[i][pt][q], 0, 0, 0);
#pragma unroll
            for (int pt = 0; pt < 2; ++pt)
#pragma unroll
              for (int q = 0; q < Q; ++q)
                acc16[i][pt][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[pt], g1[q], acc16[i][pt][q], 0, 0, 0);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kc + 1 < nch) {  // LDS-only barriers: the previous block's epilogue stores keep draining
        x3_lds_barrier();  // every wave is done reading this chunk
        X3P_STORE(kc + 1);
        x3_lds_barrier();
      }
    }
    // epilogue: as conv3x3_x3_kernel<M16>, but every accumulator goes to the wave's LDS region first
    // (RN x 32 channels: the accumulators are dead before the stores, while the next block's first
    // chunk is held in registers), and the global stores are left in flight
    if (has_next) {  // the next block's first chunk, in flight during this block's epilogue
      X3P_SETUP(nx0, ny0, nn, nn0);
      X3P_LOAD(0);
    }
    x3_lds_barrier();  // every wave is done reading the last chunk's tiles
    int el = lane, ew = wm;  // laundered as in the MFMA loop
    asm volatile("" : "+v"(el), "+v"(ew));
    const int el16 = el & 15, eg16 = el >> 4;
    float* region = reinterpret_cast<float*>(x3_smem) + ew * 32 * RM * 36;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int q = 2 * j + qq, co = n0 + 16 * q + el16;
        const float bv = (co < A_.Cout && A_.bias) ? A_.bias[co] : 0.f;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) {
            const f32x4v v = acc16[i][pt][q];
            *reinterpret_cast<float4*>(region + ((16 * qq + el16) * RM + i) * 36 + 16 * pt + 4 * eg16) =
                make_float4(v[0] + bv, v[1] + bv, v[2] + bv, v[3] + bv);
          }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      store_region<RM>(A_, region, n, x0, y0, ew * RM, n0 + 32 * j, el);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    if (!has_next) break;
    x3_lds_barrier();  // every wave is done with its epilogue region (the stores stay in flight)
    X3P_STORE(0);      // the next block's first chunk (loaded during the last MFMAs)
    x3_lds_barrier();
    b = b2;
    x0 = nx0;
    y0 = ny0;
    n = nn;
    n0 = nn0;
  }
#undef X3P_DECODE
#undef X3P_SETUP
#undef X3P_LOAD
#undef X3P_STORE
#undef A_
}

// Direct (VALU) 3x3 conv for cout <= 4 — the decoder's final 64->3 conv (models.py:627). As a
// GEMM its N = 3 would leave >90% of every MFMA tile idle; as a direct conv each thread makes
// 4 adjacent output pixels x COUT channels, weights are wave-uniform scalar loads, and the kernel
// is bound by reading its input once from HBM. Same source-tile staging as the MFMA kernel.
template <int COUT, int UP>
__global__ __launch_bounds__(256, 3) void conv3x3_smallc_kernel(ConvArgs a) {
  constexpr int NT = 256, TH = 8, TWS = 128, CK = 4;
  constexpr int SW = TWS / UP, SR = TH / UP + 2, RS = SW + 8, C0 = 4, QV = SW / 4;
  constexpr int A_ITEMS = CK * SR * (QV + 2);
  __shared__ __attribute__((aligned(16))) float As[CK * SR * RS];

  const int tid = threadIdx.x;
  const int tx = tid & 31, ty = tid >> 5;
  int t = blockIdx.x;
  const int bx = t % a.tiles_x;
  t /= a.tiles_x;
  const int by = t % a.tiles_y;
  const int n = t / a.tiles_y;
  const int x0 = bx * TWS, y0 = by * TH;
  const int sx0 = x0 / UP, sy0 = y0 / UP - 1;
  const int Hin = a.Hin, Win = a.Win;
  const bool fast = (sx0 + SW <= Win) && ((Win & 3) == 0);
  const float* __restrict__ xin =
      n < a.nsplit ? a.x + (int64_t)n * a.Cin * Hin * Win : a.x2 + (int64_t)(n - a.nsplit) * a.Cin * Hin * Win;
  const float* __restrict__ wp = a.wp;
  const int plane_in = Hin * Win;

  float acc[COUT][4];
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[co][j] = 0.f;

  __shared__ __attribute__((aligned(16))) float Ws[CK * 9 * 4];  // [c][tap][co(4)] of this chunk
  constexpr int A_PER_T = (A_ITEMS + NT - 1) / NT;
  for (int cin0 = 0; cin0 < a.Cin; cin0 += CK) {
    float4 ra[A_PER_T];
    if (fast) {  // issue every global load of the chunk before the barrier, store after it
#pragma unroll
      for (int i = 0; i < A_PER_T; ++i) {
        const int e = tid + i * NT;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < A_ITEMS) {
          const int q = e % (QV + 2);
          const int cr = e / (QV + 2);
          const int r = cr % SR, c = cr / SR;
          const int cin = cin0 + c;
          const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
          if (cin < a.Cin && sy >= 0) {
            const float* row = xin + cin * plane_in + sy * Win;
            if (q < QV) {
              v = *reinterpret_cast<const float4*>(row + sx0 + 4 * q);
            } else {
              const int sx = src_index<UP>(q == QV ? sx0 - 1 : sx0 + SW, Win, a.reflect);
              if (sx >= 0) v.x = row[sx];
            }
          }
        }
        ra[i] = v;
      }
    }
    float wv = 0.f;
    if (tid < CK * 9 * 4) {
      const int c = tid / 36, rem = tid % 36, tap = rem / 4, co = rem % 4;
      if (cin0 + c < a.Cin && co < COUT) wv = wp[((cin0 + c) * 9 + tap) * a.cout_pad + co];
    }
    __syncthreads();  // previous chunk's reads are done
    if (tid < CK * 9 * 4) Ws[tid] = wv;
    if (fast) {
#pragma unroll
      for (int i = 0; i < A_PER_T; ++i) {
        const int e = tid + i * NT;
        if (e < A_ITEMS) {
          const int q = e % (QV + 2);
          float* row = As + (e / (QV + 2)) * RS;
          if (q < QV) *reinterpret_cast<float4*>(row + C0 + 4 * q) = ra[i];
          else row[q == QV ? C0 - 1 : C0 + SW] = ra[i].x;
        }
      }
    } else {
      for (int e = tid; e < CK * SR * (SW + 2); e += NT) {
        const int col = e % (SW + 2);
        const int cr = e / (SW + 2);
        const int r = cr % SR, c = cr / SR;
        const int cin = cin0 + c;
        const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
        const int sx = src_index<UP>(sx0 - 1 + col, Win, a.reflect);
        As[cr * RS + C0 - 1 + col] = (cin < a.Cin && sy >= 0 && sx >= 0) ? xin[cin * plane_in + sy * Win + sx] : 0.f;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int c = 0; c < CK; ++c) {  // channels past Cin hold zero inputs and zero weights
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int orow = ty + ky - 1;
        const int srow = (UP == 1) ? orow + 1 : (orow >> 1) + 1;
        const float* rowp = As + (c * SR + srow) * RS + C0;
        constexpr int NV = UP == 1 ? 6 : 4;
        float v[NV];
        if constexpr (UP == 1) {
          // columns 4tx-1 .. 4tx+4: one aligned 16-byte read (consecutive lanes, conflict-free) and
          // the two neighbours from the adjacent lanes (lane shuffles); the scalar reads at a
          // 4-word lane stride were 4-way bank conflicts. Each half-wave is one output row, so its
          // first and last lanes read their outer neighbour themselves.
          const float4 mid = *reinterpret_cast<const float4*>(rowp + 4 * tx);
          // (lane shuffles; the DPP wave_shr / wave_shl forms these replaced are GFX8/9-era controls)
          float left = __shfl_up(mid.w, 1, 64);
          float right = __shfl_down(mid.x, 1, 64);
          if (tx == 0) left = rowp[-1];
          if (tx == 31) right = rowp[128];
          v[0] = left;
          v[1] = mid.x;
          v[2] = mid.y;
          v[3] = mid.z;
          v[4] = mid.w;
          v[5] = right;
        } else {
#pragma unroll
          for (int m = 0; m < NV; ++m) v[m] = rowp[2 * tx - 1 + m];
        }
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float4 w4 = *reinterpret_cast<const float4*>(Ws + (c * 9 + ky * 3 + kx) * 4);  // LDS broadcast
          const float wco[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int co = 0; co < COUT; ++co) {
            const float w = wco[co];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int m = UP == 1 ? j + kx : ((j + kx - 1) >> 1) + 1;
              acc[co][j] = fmaf(v[m], w, acc[co][j]);
            }
          }
        }
      }
    }
  }

  const int H = a.H, W = a.W;
  const int yy = y0 + ty, xx = x0 + 4 * tx;
  if (yy >= H || xx >= W) return;
  const bool full = ((W & 3) == 0) && xx + 3 < W;
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    if (co >= a.Cout) break;
    const float bv = a.bias ? a.bias[co] : 0.f;
    float v[4], u[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = acc[co][j] + bv;
      u[j] = relu_f(v[j]);
    }
    const int64_t off = (((int64_t)n * a.Cout + co) * H + yy) * W + xx;
    if (a.y_pre) {
      if (full) *reinterpret_cast<float4*>(a.y_pre + off) = make_float4(v[0], v[1], v[2], v[3]);
      else for (int j = 0; j < 4; ++j) if (xx + j < W) a.y_pre[off + j] = v[j];
    }
    if (a.y_act) {
      if (full) *reinterpret_cast<float4*>(a.y_act + off) = make_float4(u[0], u[1], u[2], u[3]);
      else for (int j = 0; j < 4; ++j) if (xx + j < W) a.y_act[off + j] = u[j];
    }
  }
}

// Direct (VALU) 3x3 conv for cout <= 4, register-streaming form (round 5; configs 36, 37): no LDS
// tile and no barrier per input channel. A wave owns 2 output rows x 256 columns (4 per lane); per
// input channel each lane loads its 4 source rows as one 16-byte piece each, takes the columns left
// and right of its piece from the neighbouring lanes (the wave's edge lanes and the image borders
// load theirs), and accumulates 2 rows x 4 pixels x COUT outputs over the 9 taps (weights: one LDS
// broadcast float4 per tap). The next two channels' rows are in flight during the current channel's
// FMAs. Same tap-major, channel-minor FMA order per output as conv3x3_smallc_kernel: bit-identical.
// The smallc form stages 4-channel chunks in LDS behind two barriers each and ran at ~2 TB/s of its
// input (latency-bound, 8x64x512^2 -> 3: 0.27 ms); this one streams.
template <int COUT>
__global__ __launch_bounds__(256) void conv3x3_smallc2_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float Wsm[];  // [cin][9 taps][4 co]
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  int t = blockIdx.x;
  const int bx = t % a.tiles_x;
  t /= a.tiles_x;
  const int by = t % a.tiles_y;
  const int n = t / a.tiles_y;
  const int H = a.H, W = a.W, Cin = a.Cin;
  const int x = bx * 256 + 4 * lane, y0 = by * 8 + 2 * wv;
  for (int e = tid; e < Cin * 36; e += 256) {
    const int ci = e / 36, rem = e - ci * 36, tap = rem >> 2, co = rem & 3;
    Wsm[e] = co < COUT ? a.wp[((int64_t)ci * 9 + tap) * a.cout_pad + co] : 0.f;
  }
  __syncthreads();
  const float* __restrict__ xin =
      n < a.nsplit ? a.x + (int64_t)n * Cin * H * W : a.x2 + (int64_t)(n - a.nsplit) * Cin * H * W;
  const int64_t plane = (int64_t)H * W;
  // source rows y0 - 1 .. y0 + 2 (zero pad: -1 = none; reflect: mirrored)
  int srow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) srow[r] = src_index<1>(y0 - 1 + r, H, a.reflect);
  const bool inx = x < W;                                      // W % 4 == 0 (host)
  const int xl = src_index<1>(x - 1, W, a.reflect), xr = src_index<1>(x + 4, W, a.reflect);
  const bool own_l = lane == 0 || x == 0, own_r = lane == 63 || x + 4 >= W;  // load the neighbour itself
  float acc[2][COUT][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int co = 0; co < COUT; ++co)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][co][j] = 0.f;
  // three channel buffers: channels c + 1 and c + 2 are in flight while channel c is computed
  float4 cen[3][4];
  float el[3][4], er[3][4];
  auto load = [&](int c, float4 (&cv)[4], float (&l)[4], float (&r)[4]) {
    const float* xc = xin + (int64_t)c * plane;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = srow[k] >= 0;
      const float* row = xc + (int64_t)(ok ? srow[k] : 0) * W;
      cv[k] = (ok && inx) ? *reinterpret_cast<const float4*>(row + x) : make_float4(0.f, 0.f, 0.f, 0.f);
      l[k] = (ok && own_l && xl >= 0) ? row[xl] : 0.f;
      r[k] = (ok && own_r && xr >= 0) ? row[xr] : 0.f;
    }
  };
  auto compute = [&](int c, const float4 (&cv)[4], const float (&l)[4], const float (&r)[4]) {
    float v[4][6];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float left = __shfl_up(cv[k].w, 1, 64), right = __shfl_down(cv[k].x, 1, 64);
      v[k][0] = own_l ? l[k] : left;
      v[k][1] = cv[k].x;
      v[k][2] = cv[k].y;
      v[k][3] = cv[k].z;
      v[k][4] = cv[k].w;
      v[k][5] = own_r ? r[k] : right;
    }
    const float4* wc = reinterpret_cast<const float4*>(Wsm + c * 36);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float4 w4 = wc[ky * 3 + kx];
        const float wco[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int co = 0; co < COUT; ++co)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][co][j] = fmaf(v[i + ky][j + kx], wco[co], acc[i][co][j]);
      }
  };
  load(0, cen[0], el[0], er[0]);
  if (Cin > 1) load(1, cen[1], el[1], er[1]);
  for (int c0 = 0; c0 < Cin; c0 += 3) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {  // buffer u holds channel c0 + u
      const int c = c0 + u;
      if (c < Cin) {
        if (c + 2 < Cin) load(c + 2, cen[(u + 2) % 3], el[(u + 2) % 3], er[(u + 2) % 3]);
        compute(c, cen[u], el[u], er[u]);
      }
    }
  }
  if (!inx) return;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int yy = y0 + i;
    if (yy >= H) continue;
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      if (co >= a.Cout) break;
      const float bv = a.bias ? a.bias[co] : 0.f;
      const float4 o = make_float4(acc[i][co][0] + bv, acc[i][co][1] + bv, acc[i][co][2] + bv, acc[i][co][3] + bv);
      const int64_t off = (((int64_t)n * a.Cout + co) * H + yy) * W + x;
      if (a.y_pre) *reinterpret_cast<float4*>(a.y_pre + off) = o;
      if (a.y_act) *reinterpret_cast<float4*>(a.y_act + off) = make_float4(relu_f(o.x), relu_f(o.y), relu_f(o.z), relu_f(o.w));
    }
  }
}

// Direct (VALU) 3x3 conv for cin <= 4 — VGG conv_1 (3->64, models.py:199-216, with the
// Normalization of models.py:120-131 applied in the gather). As an implicit GEMM its K = 27 runs
// in 4-channel K-chunks behind 64-channel MFMA tiles and the launch is bound by writing 21x its
// input bytes; here a workgroup stages its 8x128-pixel source tile (+halo) once, each thread keeps
// its 3x6 input window per channel in registers and loops over the output channels 4 at a time:
// the workgroup's weights sit in LDS and each tap's 4 output channels are one broadcast 16-byte
// read (as wave-uniform scalar loads, 108 weights per trip spilled 150 SGPRs: 2 SGPR reloads per
// FMA pair); every store is a 512-B row run.
// NTS (configs 20, 22, 23) used to store through nontemporal stores; it is kept only as a
// configuration index and stores normally: the nontemporal form was the first suspect for the
// run-to-run differences seen under a second process's GPU load (DESIGN.md §4 open item), and the
// plain form costs nothing measurable (config 2: 568.6 img/s, profiles/r03_race_fix_trials.txt) --
// but the differences persist without it, so it was not their cause.
template <int CIN, bool NORM, int TH, bool NTS, int OCC>
__global__ __launch_bounds__(TH * 32, OCC) void conv3x3_cin4_kernel(ConvArgs a, const float* __restrict__ wp) {
  constexpr int NT = TH * 32, TWS = 128, COG = 4;
  constexpr int SR = TH + 2, RS = TWS + 8, C0 = 4;
  __shared__ __attribute__((aligned(16))) float As[CIN * SR * RS];
  extern __shared__ __attribute__((aligned(16))) float cin4_w[];  // [CIN * 9][cout_pad]

  const int tid = threadIdx.x;
  const int tx = tid & 31, ty = tid >> 5;
  int t = blockIdx.x;
  const int bx = t % a.tiles_x;
  t /= a.tiles_x;
  const int by = t % a.tiles_y;
  const int n = t / a.tiles_y;
  const int x0 = bx * TWS, y0 = by * TH;
  const int H = a.H, W = a.W;
  const float* __restrict__ xin =
      n < a.nsplit ? a.x + (int64_t)n * a.Cin * H * W : a.x2 + (int64_t)(n - a.nsplit) * a.Cin * H * W;
  const int plane = H * W;

  // Source tile, normalised; zero for zero padding and for channels past Cin (padding is
  // applied to the normalised image, as the reference pads after Normalization).
  // (all loads issued before any LDS store: one memory latency per tile, not one per element)
  constexpr int ST = CIN * SR * (TWS + 2), ST_T = (ST + NT - 1) / NT;
  float sv[ST_T];
#pragma unroll
  for (int i = 0; i < ST_T; ++i) {
    const int e = min(tid + i * NT, ST - 1);
    const int col = e % (TWS + 2);
    const int cr = e / (TWS + 2);
    const int r = cr % SR, c = cr / SR;
    const int sy = src_index<1>(y0 - 1 + r, H, a.reflect);
    const int sx = src_index<1>(x0 - 1 + col, W, a.reflect);
    const bool ok = c < a.Cin && sy >= 0 && sx >= 0;
    sv[i] = ok ? xin[c * plane + max(sy, 0) * W + max(sx, 0)] : 0.f;
  }
  for (int i = tid; i < CIN * 9 * a.cout_pad / 4; i += NT)
    reinterpret_cast<float4*>(cin4_w)[i] = reinterpret_cast<const float4*>(wp)[i];
#pragma unroll
  for (int i = 0; i < ST_T; ++i) {
    const int e = tid + i * NT;
    if (e < ST) {
      const int col = e % (TWS + 2);
      const int cr = e / (TWS + 2);
      const int c = cr / SR;
      float v = sv[i];
      if (NORM) {
        const int r = cr % SR;
        const bool ok = c < a.Cin && src_index<1>(y0 - 1 + r, H, a.reflect) >= 0 &&
                        src_index<1>(x0 - 1 + col, W, a.reflect) >= 0;
        v = ok ? (v - a.in_mean[c]) / a.in_std[c] : 0.f;  // padding stays 0 after normalisation
      }
      As[cr * RS + C0 - 1 + col] = v;
    }
  }
  __syncthreads();

  float v[CIN][3][6];
#pragma unroll
  for (int c = 0; c < CIN; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int m = 0; m < 6; ++m) v[c][ky][m] = As[(c * SR + ty + ky) * RS + C0 - 1 + 4 * tx + m];

  const int yy = y0 + ty, xx = x0 + 4 * tx;
  const bool ok = yy < H && xx < W;
  const bool full = ((W & 3) == 0) && xx + 3 < W;
  const int64_t obase = (int64_t)n * a.Cout * plane + (int64_t)yy * W + xx;
  const int cout_pad = a.cout_pad;
  for (int co0 = 0; co0 < a.Cout; co0 += COG) {  // cout_pad is a multiple of COG: slab reads in bounds
    float acc[COG][4];
#pragma unroll
    for (int k = 0; k < COG; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[k][j] = 0.f;
    // tap-major, channel-minor: the MFMA kernel's accumulation order (bit-identical results)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int c = 0; c < CIN; ++c) {
          const float4 w4 = *reinterpret_cast<const float4*>(cin4_w + (c * 9 + ky * 3 + kx) * cout_pad + co0);
          const float wk[COG] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int k = 0; k < COG; ++k) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[k][j] = fmaf(v[c][ky][j + kx], wk[k], acc[k][j]);
          }
        }
    if (!ok) continue;
#pragma unroll
    for (int k = 0; k < COG; ++k) {
      const int co = co0 + k;
      if (co >= a.Cout) break;
      const float bv = a.bias ? a.bias[co] : 0.f;
      float o[4], u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = acc[k][j] + bv;
        u[j] = relu_f(o[j]);
      }
      const int64_t off = obase + (int64_t)co * plane;
      if (a.y_pre && dgrad_epi(a)) {  // input gradient (ast_conv3x3_dgrad_f32): y_pre only
        if (full) {
          *reinterpret_cast<float4*>(a.y_pre + off) = dgrad_epi4(a, make_float4(o[0], o[1], o[2], o[3]), off);
        } else {
          for (int j = 0; j < 4; ++j) if (xx + j < W) a.y_pre[off + j] = dgrad_epi_one(a, o[j], off + j);
        }
        continue;
      }
      if (a.y_pre) {
        if (full) {
          *reinterpret_cast<float4*>(a.y_pre + off) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
          for (int j = 0; j < 4; ++j) if (xx + j < W) a.y_pre[off + j] = o[j];
        }
      }
      if (a.y_act) {
        if (full) {
          *reinterpret_cast<float4*>(a.y_act + off) = make_float4(u[0], u[1], u[2], u[3]);
        } else {
          for (int j = 0; j < 4; ++j) if (xx + j < W) a.y_act[off + j] = u[j];
        }
      }
    }
  }
}

__global__ void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ wp, int cout, int cin,
                                    int cout_pad, int cin_pad) {
  const int64_t total = (int64_t)cin_pad * 9 * cout_pad;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(idx % cout_pad);
    const int64_t rt = idx / cout_pad;
    const int tap = (int)(rt % 9);
    const int ci = (int)(rt / 9);
    wp[idx] = (ci < cin && co < cout) ? w[((int64_t)co * cin + ci) * 9 + tap] : 0.f;
  }
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline int round_up(int a, int b) { return cdiv(a, b) * b; }

template <int WM, int WN, int RM, int RN, int CK, int UP, bool SWAP, bool NORM>
int launch_one(const ConvArgs& a0, hipStream_t s) {
  using C = Cfg<WM, WN, RM, RN, CK, UP>;
  ConvArgs a = a0;
  a.tiles_x = cdiv(a.W, TW);
  a.tiles_y = cdiv(a.H, C::TH);
  if (cdiv(a.Cout, C::BN) * C::BN > a.cout_pad) return AST_E_UNSUPPORTED;  // weight-slab reads stay in bounds
  const int64_t ntiles = (int64_t)a.tiles_x * a.tiles_y * a.N;
  const int64_t nblk = (ntiles + 7) / 8 * 8 * cdiv(a.Cout, C::BN);
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  auto kern = conv3x3_f32_kernel<WM, WN, RM, RN, CK, UP, SWAP, NORM>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS_BYTES);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(C::NT), C::LDS_BYTES, s, a);
  return (int)hipGetLastError();
}

template <int WM, int WN, int RM, int RN, int CK, bool SWAP = false>
int launch_cfg(const ConvArgs& a, hipStream_t s, int up) {
  if (a.in_mean)  // ImageNet normalisation in the gather: conv_1 only (never upsampled)
    return up == 2 ? launch_one<WM, WN, RM, RN, CK, 2, SWAP, true>(a, s) : launch_one<WM, WN, RM, RN, CK, 1, SWAP, true>(a, s);
  return up == 2 ? launch_one<WM, WN, RM, RN, CK, 2, SWAP, false>(a, s) : launch_one<WM, WN, RM, RN, CK, 1, SWAP, false>(a, s);
}

template <int COUT>
int launch_smallc(const ConvArgs& a0, hipStream_t s, int up) {
  ConvArgs a = a0;
  if (a.Cout > COUT || a.y_pool) return AST_E_UNSUPPORTED;
  a.tiles_x = cdiv(a.W, 128);
  a.tiles_y = cdiv(a.H, 8);
  const int64_t nblk = (int64_t)a.tiles_x * a.tiles_y * a.N;
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  if (up == 2)
    hipLaunchKernelGGL((conv3x3_smallc_kernel<COUT, 2>), dim3((unsigned)nblk), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3_smallc_kernel<COUT, 1>), dim3((unsigned)nblk), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

template <int COUT>
int launch_smallc2(const ConvArgs& a0, hipStream_t s, int up) {
  ConvArgs a = a0;
  if (a.Cout > COUT || a.y_pool || up != 1 || (a.W & 3) || a.in_mean || a.Cin > 1024) return AST_E_UNSUPPORTED;
  a.tiles_x = cdiv(a.W, 256);
  a.tiles_y = cdiv(a.H, 8);
  const int64_t nblk = (int64_t)a.tiles_x * a.tiles_y * a.N;
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  const int lds = a.Cin * 36 * 4;
  auto kern = conv3x3_smallc2_kernel<COUT>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 1024 * 36 * 4);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(256), lds, s, a);
  return (int)hipGetLastError();
}

template <int TH, bool NTS, int OCC = 1>
int launch_cin4(const ConvArgs& a0, hipStream_t s, int up) {
  ConvArgs a = a0;
  if (a.Cin > 4 || a.y_pool || up != 1) return AST_E_UNSUPPORTED;
  a.tiles_x = cdiv(a.W, 128);
  a.tiles_y = cdiv(a.H, TH);
  const int64_t nblk = (int64_t)a.tiles_x * a.tiles_y * a.N;
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  const dim3 g((unsigned)nblk), b(TH * 32);
  const bool norm = a.in_mean != nullptr;
  // weights in LDS: the instantiation's CIN (3, else 4: Cin 1 and 2 run the CIN = 4 kernel, which
  // copies and reads 4 channels' slabs -- the packed fp32 part holds cin_pad8 >= 4 of them, zero past
  // Cin), not a.Cin, or channels Cin..3 are read past the allocation
  const int cin_k = a.Cin == 3 ? 3 : 4;
  const size_t wl = (size_t)cin_k * 9 * a.cout_pad * sizeof(float);
  if (a.cout_pad % 4 || wl > 32 * 1024) return AST_E_UNSUPPORTED;
  if (a.Cin == 3) {
    if (norm) hipLaunchKernelGGL((conv3x3_cin4_kernel<3, true, TH, NTS, OCC>), g, b, wl, s, a, a.wp);
    else hipLaunchKernelGGL((conv3x3_cin4_kernel<3, false, TH, NTS, OCC>), g, b, wl, s, a, a.wp);
  } else {
    if (norm) hipLaunchKernelGGL((conv3x3_cin4_kernel<4, true, TH, NTS, OCC>), g, b, wl, s, a, a.wp);
    else hipLaunchKernelGGL((conv3x3_cin4_kernel<4, false, TH, NTS, OCC>), g, b, wl, s, a, a.wp);
  }
  return (int)hipGetLastError();
}

// split-bf16 MFMA conv of a 1..3-channel input (conv_cin3.hip): no pool / upsample
template <int TH>
int launch_cin3x3(const ConvArgs& a, hipStream_t s, int up) {
  if (a.Cin > 3 || a.y_pool || up != 1) return AST_E_UNSUPPORTED;
  Cin3Args c{};
  c.x = a.x; c.x2 = a.x2; c.nsplit = a.nsplit; c.wp = a.wp; c.bias = a.bias;
  c.y_pre = a.y_pre; c.y_act = a.y_act; c.in_mean = a.in_mean; c.in_std = a.in_std;
  c.e_mask = a.e_mask; c.e_add_pre = a.e_add_pre; c.e_add_post = a.e_add_post;
  c.N = a.N; c.Cin = a.Cin; c.H = a.H; c.W = a.W; c.Cout = a.Cout; c.cout_pad = a.cout_pad; c.reflect = a.reflect;
  return launch_conv_cin3_x3(c, TH, s);
}

int cu_count() {  // CUs of the current device (looked up on a device's first call)
  static int cus_of[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  int cus = dev >= 0 && dev < 64 ? cus_of[dev] : 0;
  if (!cus) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (dev >= 0 && dev < 64) cus_of[dev] = cus;
  }
  return cus;
}

template <int WM, int RM, int RN, int UP, int OCC, bool M16, bool PER = false>
int launch_x3_one(const ConvArgs& a0, hipStream_t s) {
  using C = X3Cfg<WM, RM, RN, UP>;
  ConvArgs a = a0;
  a.tiles_x = cdiv(a.W, TW);
  a.tiles_y = cdiv(a.H, C::TH);
  if (cdiv(a.Cout, C::BN) * C::BN > a.cout_pad) return AST_E_UNSUPPORTED;
  const int64_t ntiles = (int64_t)a.tiles_x * a.tiles_y * a.N;
  int64_t nblk = (ntiles + 7) / 8 * 8 * cdiv(a.Cout, C::BN);
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  if (PER) {  // one workgroup per CU slot, a multiple of 8 (the XCD of a block stays fixed)
    const int64_t slots = (int64_t)(cu_count() + 7) / 8 * 8 * OCC;
    nblk = nblk < slots ? nblk : slots;
  }
  auto kern = conv3x3_x3_kernel<WM, RM, RN, UP, OCC, M16, PER>;
  constexpr int lds = M16 ? C::LDS_BYTES_M16 : C::LDS_BYTES;
  static_assert(lds * OCC <= 160 * 1024, "LDS per CU");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(C::NT), lds, s, a);
  return (int)hipGetLastError();
}

// persistent form: one workgroup per CU slot (OCC per CU), a multiple of 8 (XCD-consistent stride)
template <int WM, int RM, int RN, int UP, int OCC>
int launch_x3p_one(const ConvArgs& a0, hipStream_t s) {
  using C = X3Cfg<WM, RM, RN, UP>;
  ConvArgs a = a0;
  a.tiles_x = cdiv(a.W, TW);
  a.tiles_y = cdiv(a.H, C::TH);
  if (cdiv(a.Cout, C::BN) * C::BN > a.cout_pad) return AST_E_UNSUPPORTED;
  const int64_t ntiles = (int64_t)a.tiles_x * a.tiles_y * a.N;
  const int64_t nblk = (ntiles + 7) / 8 * 8 * cdiv(a.Cout, C::BN);
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  static int cus_of[64] = {};  // CU count per device (looked up on a device's first call)
  int dev = 0;
  (void)hipGetDevice(&dev);
  int cus = dev >= 0 && dev < 64 ? cus_of[dev] : 0;
  if (!cus) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (dev >= 0 && dev < 64) cus_of[dev] = cus;
  }
  const int64_t slots = (int64_t)(cus + 7) / 8 * 8 * OCC;
  const unsigned grid = (unsigned)(nblk < slots ? nblk : slots);
  auto kern = conv3x3_x3p_kernel<WM, RM, RN, UP, OCC>;
  constexpr int lds = C::LDS_BYTES;
  static_assert(lds * OCC <= 160 * 1024, "LDS per CU");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(C::NT), lds, s, a, (int)nblk);
  return (int)hipGetLastError();
}

template <int WM, int RM, int RN, int OCC = 1>
int launch_x3p(const ConvArgs& a, hipStream_t s, int up) {
  if (a.in_mean) return AST_E_UNSUPPORTED;
  if ((int64_t)a.Cin * a.Hin * a.Win * 4 >= ((int64_t)1 << 31)) return AST_E_UNSUPPORTED;  // 32-bit buffer offsets
  return up == 2 ? launch_x3p_one<WM, RM, RN, 2, OCC>(a, s) : launch_x3p_one<WM, RM, RN, 1, OCC>(a, s);
}

// split-bf16 MFMA kernel: no fused input normalisation (conv_1 runs the direct cin<=4 kernel)
template <int WM, int RM, int RN, int OCC = 1, bool M16 = false, bool PER = false>
int launch_x3(const ConvArgs& a, hipStream_t s, int up) {
  if (a.in_mean) return AST_E_UNSUPPORTED;
  if ((int64_t)a.Cin * a.Hin * a.Win * 4 >= ((int64_t)1 << 31)) return AST_E_UNSUPPORTED;  // 32-bit buffer offsets
  return up == 2 ? launch_x3_one<WM, RM, RN, 2, OCC, M16, PER>(a, s) : launch_x3_one<WM, RM, RN, 1, OCC, M16, PER>(a, s);
}

struct CfgEntry {
  int (*fn)(const ConvArgs&, hipStream_t, int);
  int bn;        // output channels per workgroup (weight-slab width)
  int th;        // output rows per workgroup
  int rm;        // output rows per wave (pool needs an even count)
  int max_cout;  // 0 = any
};

// Index -> configuration. Keep the table stable (tests/tuner address entries by index).
const CfgEntry kConfigs[] = {
    {launch_cfg<4, 1, 2, 2, 8>, 64, 8, 2, 0},    // 0: 8x32 px x 64 ch, CK 8, 4 waves
    {launch_cfg<4, 1, 2, 2, 4>, 64, 8, 2, 0},    // 1: 8x32 px x 64 ch, CK 4, 4 waves
    {launch_cfg<2, 2, 4, 2, 4>, 128, 8, 4, 0},   // 2: 8x32 px x 128 ch, CK 4, 4 waves
    {launch_cfg<2, 2, 2, 2, 8>, 128, 4, 2, 0},   // 3: 4x32 px x 128 ch, CK 8, 4 waves
    {launch_cfg<4, 1, 4, 2, 4>, 64, 16, 4, 0},   // 4: 16x32 px x 64 ch, CK 4, 4 waves
    {launch_cfg<2, 2, 2, 2, 4>, 128, 4, 2, 0},   // 5: 4x32 px x 128 ch, CK 4, 4 waves
    {launch_cfg<4, 2, 2, 2, 4>, 128, 8, 2, 0},   // 6: 8x32 px x 128 ch, CK 4, 8 waves
    {launch_cfg<8, 1, 2, 2, 4>, 64, 16, 2, 0},   // 7: 16x32 px x 64 ch, CK 4, 8 waves
    {launch_cfg<4, 2, 4, 2, 4>, 128, 16, 4, 0},  // 8: 16x32 px x 128 ch, CK 4, 8 waves
    {launch_cfg<2, 1, 2, 2, 4>, 64, 4, 2, 0},    // 9: 4x32 px x 64 ch, CK 4, 2 waves
    {launch_smallc<3>, 4, 8, 2, 3},              // 10: direct VALU conv, cout <= 3
    {launch_smallc<4>, 4, 8, 2, 4},              // 11: direct VALU conv, cout <= 4
    // swapped operands (C^T: pixels on lanes -> whole-line dword stores)
    {launch_cfg<8, 1, 2, 2, 4, true>, 64, 16, 2, 0},   // 12: as 7
    {launch_cfg<4, 2, 2, 2, 4, true>, 128, 8, 2, 0},   // 13: as 6
    {launch_cfg<4, 2, 4, 2, 4, true>, 128, 16, 4, 0},  // 14: as 8
    {launch_cfg<4, 1, 2, 2, 4, true>, 64, 8, 2, 0},    // 15: as 1
    {launch_cfg<8, 2, 2, 2, 4>, 128, 16, 2, 0},        // 16: 16x32 px x 128 ch, CK 4, 16 waves (1 WG/CU)
    {launch_cfg<8, 2, 2, 2, 4, true>, 128, 16, 2, 0},  // 17: as 16, swapped
    {launch_cin4<8, false>, 64, 8, 1, 0},               // 18: direct VALU conv, cin <= 4, no pool/upsample
    {launch_cin4<16, false>, 64, 16, 1, 0},             // 19: as 18, 16-row tiles
    {launch_cin4<8, true>, 64, 8, 1, 0},                // 20: as 18, nontemporal stores
    {launch_cin4<4, false>, 64, 4, 1, 0},               // 21: as 18, 4-row tiles
    {launch_cin4<16, true>, 64, 16, 1, 0},              // 22: 16-row tiles, nontemporal stores
    {launch_cin4<32, true>, 64, 32, 1, 0},              // 23: 32-row tiles, nontemporal stores
    // split-bf16 (fp32-accurate) MFMA implicit GEMM
    {launch_x3<8, 2, 2>, 64, 16, 2, 0},                 // 24: 16x32 px x 64 ch, 8 waves
    {launch_x3<4, 2, 2>, 64, 8, 2, 0},                  // 25: 8x32 px x 64 ch, 4 waves
    {launch_x3<4, 2, 1, 2>, 32, 8, 2, 0},               // 26: 8x32 px x 32 ch, 4 waves, 2 workgroups/CU
    {launch_x3<8, 2, 1, 1>, 32, 16, 2, 0},              // 27: 16x32 px x 32 ch, 8 waves
    // the same tiles on the 16x16x32 bf16 MFMA (three K-32 products per block)
    {launch_x3<8, 2, 2, 1, true>, 64, 16, 2, 0},        // 28: as 24
    {launch_x3<4, 2, 2, 1, true>, 64, 8, 2, 0},         // 29: as 25
    {launch_x3<4, 2, 1, 2, true>, 32, 8, 2, 0},         // 30: as 26
    {launch_x3<8, 2, 1, 1, true>, 32, 16, 2, 0},        // 31: as 27
    // persistent forms of 28-31 (next block's first chunk under the last MFMAs, store tail overlapped)
    {launch_x3p<8, 2, 2>, 64, 16, 2, 0},                // 32: as 28
    {launch_x3p<4, 2, 2>, 64, 8, 2, 0},                 // 33: as 29
    {launch_x3p<4, 2, 1, 2>, 32, 8, 2, 0},              // 34: as 30
    {launch_x3p<8, 2, 1, 1>, 32, 16, 2, 0},             // 35: as 31
    // register-streaming direct VALU conv for cout <= 4 (no LDS tile, no per-channel barrier)
    {launch_smallc2<3>, 4, 8, 2, 3},                    // 36: cout <= 3
    {launch_smallc2<4>, 4, 8, 2, 4},                    // 37: cout <= 4
    // persistent forms of 28-31 (round 5): the same kernel looping over blocks
    {launch_x3<8, 2, 2, 1, true, true>, 64, 16, 2, 0},  // 38: as 28
    {launch_x3<4, 2, 2, 1, true, true>, 64, 8, 2, 0},   // 39: as 29
    {launch_x3<4, 2, 1, 2, true, true>, 32, 8, 2, 0},   // 40: as 30
    {launch_x3<8, 2, 1, 1, true, true>, 32, 16, 2, 0},  // 41: as 31
    // split-bf16 MFMA conv of a 1..3-channel input, K = 27 in one K-32 block (round 6, conv_cin3.hip)
    {launch_cin3x3<16>, 64, 16, 1, 0},                  // 42: 16x64 px x 64 ch, 4 waves
    {launch_cin3x3<8>, 64, 8, 1, 0},                    // 43: 8x64 px x 64 ch, 4 waves
};
constexpr int kNumConfigs = sizeof(kConfigs) / sizeof(kConfigs[0]);

int auto_config(int cin, int cout, int n, int h, int w, int up, bool pool, bool norm) {
  // cout <= 4: the register-streaming direct conv where it applies (W % 4 == 0, no upsample / pool /
  // normalisation), else the LDS-staged one (profiles/r05_smallc.txt: 8x64x512^2 -> 3, 0.294 -> 0.226 ms)
  if (cout <= 4 && up == 1 && !pool && !norm && (w & 3) == 0) return cout <= 3 ? 36 : 37;
  if (cout <= 3) return 10;
  if (cout <= 4) return 11;
  // image-input convs (conv_1) and the decoder's last input gradient: the split-bf16 MFMA kernel for
  // cin <= 3 (profiles/r06c3_ab5.txt: 16 x 64 x 512^2 conv_1 0.41 -> 0.31 ms), else the direct conv
  if (cin <= 3 && up == 1 && !pool) return 42;
  if (cin <= 4 && up == 1 && !pool) return 20;
  if (cin >= kX3K && !norm && (long)cin * (h / up) * (w / up) * 4 < (1L << 31)) {
    // split-bf16 MFMA (fp32-accurate, 2.67x the fp32 matrix rate): 8x32 px x 32 ch tiles, two
    // workgroups per CU; upsampled convs the 16-row tile (profiles/r02_conv_cfgs.log)
    const long t16 = (long)n * cdiv(h, 16) * cdiv(w, 32) * cdiv(cout, 32);
    return (up == 2 && t16 >= 512) ? 27 : 26;
  }
  // 16x32 px x 64 ch, 8 waves: fastest on every VGG shape measured (profiles/, conv_tuning.json);
  // the 4-wave 8x32 tile when that leaves too few workgroups to fill 256 CUs.
  const long tiles = (long)n * cdiv(h, 16) * cdiv(w, 32) * cdiv(cout, 64);
  return tiles >= 256 ? 7 : 1;
}

}  // namespace

extern "C" {

const char* ast_version(void) { return "ast_hip 0.3 gfx950"; }

int ast_loss_acc_floats(void) { return AST_LOSS_ACC_FLOATS; }

size_t ast_conv3x3_packed_numel(int cout, int cin) {
  if (cout <= 0 || cin <= 0) return 0;
  const size_t cout_pad = (size_t)round_up(cout, kCoutAlign);
  // fp32 pack [cin_pad8][9][cout_pad], then the split-bf16 pack [cin_pad16][9][cout_pad] x 3 bf16
  return (size_t)round_up(cin, kCinAlign) * 9 * cout_pad + (size_t)round_up(cin, kX3K) * 9 * cout_pad * 3 / 2;
}

int ast_conv3x3_pack_split_f32(float* w_packed, int cout, int cin, void* stream) {
  if (!w_packed) return AST_E_NULLPTR;
  if (cout <= 0 || cin <= 0) return AST_E_SHAPE;
  const int cout_pad = round_up(cout, kCoutAlign);
  const int64_t total = (int64_t)round_up(cin, kX3K) * 9 * cout_pad;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_x3_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w_packed,
                     reinterpret_cast<bf16*>(w_packed + x3_split_offset(cin, cout)), round_up(cin, kCinAlign),
                     round_up(cin, kX3K), cout_pad);
  return (int)hipGetLastError();
}

int ast_conv3x3_pack_weights_f32(const float* w, float* w_packed, int cout, int cin, void* stream) {
  if (!w || !w_packed) return AST_E_NULLPTR;
  if (cout <= 0 || cin <= 0) return AST_E_SHAPE;
  const int cout_pad = round_up(cout, kCoutAlign), cin_pad = round_up(cin, kCinAlign);
  const int64_t total = (int64_t)cin_pad * 9 * cout_pad;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_weights_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, w_packed, cout, cin,
                     cout_pad, cin_pad);
  const int e = (int)hipGetLastError();
  return e ? e : ast_conv3x3_pack_split_f32(w_packed, cout, cin, stream);
}

int ast_conv3x3_num_configs(void) { return kNumConfigs; }

#if X3_STAMP
// diagnostic build only: copy / clear the stamp records of conv3x3_x3_kernel<M16>
int ast_dbg_x3_stamps(void* host, size_t bytes, int clear) {
  const size_t n = std::min(bytes, sizeof(x3_stamp_buf));
  if (clear) {
    void* d = nullptr;
    const hipError_t e = hipGetSymbolAddress(&d, HIP_SYMBOL(x3_stamp_buf));
    return e ? (int)e : (int)hipMemset(d, 0, sizeof(x3_stamp_buf));
  }
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(x3_stamp_buf), n, 0, hipMemcpyDeviceToHost);
}
#endif

int ast_conv3x3_fwd_f32_cfg(int cfg, const float* x, const float* x2, int n2, const float* w_packed,
                            const float* bias, float* y_pre, float* y_act, float* y_pool, const float* in_mean,
                            const float* in_std, int n, int cin, int h_in, int w_in, int cout, int upsample,
                            int pad_mode, void* stream) {
  if (!x || !w_packed) return AST_E_NULLPTR;
  if (n2 < 0 || (n2 > 0 && !x2)) return AST_E_NULLPTR;
  if (!y_pre && !y_act && !y_pool) return AST_E_NULLPTR;
  if ((in_mean == nullptr) != (in_std == nullptr)) return AST_E_NULLPTR;
  if (n <= 0 || cin <= 0 || h_in <= 0 || w_in <= 0 || cout <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (pad_mode != 0 && pad_mode != 1) return AST_E_UNSUPPORTED;
  const int H = h_in * upsample, W = w_in * upsample;
  if (pad_mode == 1 && (H < 2 || W < 2)) return AST_E_SHAPE;  // ReflectionPad2d(1) needs size >= 2
  if ((int64_t)cin * h_in * w_in >= ((int64_t)1 << 31)) return AST_E_SHAPE;         // per-image offsets are 32-bit
  if ((int64_t)round_up(cin, kCinAlign) * 9 * round_up(cout, kCoutAlign) >= ((int64_t)1 << 31)) return AST_E_SHAPE;
  if (cfg < 0) cfg = auto_config(cin, cout, n + n2, H, W, upsample, y_pool != nullptr, in_mean != nullptr);
  if (cfg >= kNumConfigs) return AST_E_UNSUPPORTED;
  static const int m16 = [] {  // AST_CONV_M16=0|1: the split-bf16 tiles (24-27) on the 32x32x16 | 16x16x32 MFMA
    const char* v = getenv("AST_CONV_M16");
    return v ? atoi(v) : 1;
  }();
  if (cfg >= 24 && cfg <= 27 && m16 == 1) cfg += 4;
  if (cfg >= 28 && cfg <= 31 && m16 == 0) cfg -= 4;
  static const int persist = [] {  // AST_CONV_PERSIST=1: the M16 tiles 28-31 in their persistent form 32-35
    const char* v = getenv("AST_CONV_PERSIST");
    return v ? atoi(v) : 0;
  }();
  if (cfg >= 28 && cfg <= 31 && persist == 1) cfg += 4;
  if (cfg >= 28 && cfg <= 31 && persist == 2) cfg += 10;  // AST_CONV_PERSIST=2: 38-41
  const CfgEntry& e = kConfigs[cfg];
  if (y_pool && (e.rm % 2 != 0 || e.max_cout)) return AST_E_UNSUPPORTED;
  if (e.max_cout && cout > e.max_cout) return AST_E_UNSUPPORTED;
  if (e.bn > kCoutAlign && (cout % e.bn) != 0) return AST_E_UNSUPPORTED;
  ConvArgs a{};
  a.x = x; a.x2 = x2; a.nsplit = n; a.wp = w_packed; a.bias = bias;
  a.y_pre = y_pre; a.y_act = y_act; a.y_pool = y_pool;
  a.in_mean = in_mean; a.in_std = in_std;
  a.N = n + n2; a.Cin = cin; a.Hin = h_in; a.Win = w_in; a.Cout = cout; a.H = H; a.W = W;
  a.cin_pad = round_up(cin, kCinAlign);
  a.cout_pad = round_up(cout, kCoutAlign);
  a.reflect = pad_mode;
  return e.fn(a, (hipStream_t)stream, upsample);
}

int ast_conv3x3_dgrad_f32(int cfg, const float* dy, const float* w_tf_packed, float* dx, const float* mask,
                          const float* add_pre, const float* add_post, int n, int cout, int h, int w, int cin,
                          int upsample, void* stream) {
  if (!dy || !w_tf_packed || !dx) return AST_E_NULLPTR;
  if (n <= 0 || cout <= 0 || h <= 0 || w <= 0 || cin <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (upsample == 2 && ((h | w) & 1)) return AST_E_SHAPE;  // the upsampled grid has even sides
  if ((int64_t)cout * h * w >= ((int64_t)1 << 31)) return AST_E_SHAPE;
  if ((int64_t)round_up(cout, kCinAlign) * 9 * round_up(cin, kCoutAlign) >= ((int64_t)1 << 31)) return AST_E_SHAPE;
  const bool sum2 = upsample == 2;
  if (cfg < 0) cfg = auto_config(cout, cin, n, h, w, 1, sum2, false);
  // the epilogue is in the split-bf16 kernels (24-35) and, without the 2x2 sum, the cin <= 4 kernels
  // (18-23) and the cin <= 3 MFMA kernels (42, 43)
  if (!((cfg >= 24 && cfg <= 35) || (((cfg >= 18 && cfg <= 23) || cfg == 42 || cfg == 43) && !sum2)) ||
      cfg >= kNumConfigs)
    return AST_E_UNSUPPORTED;
  static const int m16 = [] {
    const char* v = getenv("AST_CONV_M16");
    return v ? atoi(v) : 1;
  }();
  if (cfg >= 24 && cfg <= 27 && m16 == 1) cfg += 4;
  if (cfg >= 28 && cfg <= 31 && m16 == 0) cfg -= 4;
#if !X3_STAGED_EPI
  // the 32x32 kernels' direct-store epilogue (store_tiles) has no input-gradient epilogue: the
  // caller then runs the plain conv and ast_dgrad_finish_f32
  if (cfg >= 24 && cfg <= 27) return AST_E_UNSUPPORTED;
#endif
  const CfgEntry& e = kConfigs[cfg];
  if (sum2 && e.rm % 2 != 0) return AST_E_UNSUPPORTED;
  if (e.bn > kCoutAlign && (cin % e.bn) != 0) return AST_E_UNSUPPORTED;
  ConvArgs a{};
  a.x = dy; a.nsplit = n; a.wp = w_tf_packed;
  (sum2 ? a.y_pool : a.y_pre) = dx;
  a.e_mask = mask; a.e_add_pre = add_pre; a.e_add_post = add_post; a.e_sum2 = sum2 ? 1 : 0;
  a.N = n; a.Cin = cout; a.Hin = h; a.Win = w; a.Cout = cin; a.H = h; a.W = w;
  a.cin_pad = round_up(cout, kCinAlign);
  a.cout_pad = round_up(cin, kCoutAlign);
  a.reflect = 0;  // the interior of the padded-input gradient: a zero-padded same conv of dy
  return e.fn(a, (hipStream_t)stream, 1);
}

int ast_conv3x3_fwd_f32(const float* x, const float* w_packed, const float* bias, float* y_pre, float* y_act,
                        float* y_pool, const float* in_mean, const float* in_std, int n, int cin, int h_in, int w_in,
                        int cout, int upsample, int pad_mode, void* stream) {
  return ast_conv3x3_fwd_f32_cfg(-1, x, nullptr, 0, w_packed, bias, y_pre, y_act, y_pool, in_mean, in_std, n, cin, h_in, w_in,
                                 cout, upsample, pad_mode, stream);
}

}  // extern "C"
