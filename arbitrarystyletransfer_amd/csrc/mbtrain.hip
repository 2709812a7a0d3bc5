// MobileNet-variant training kernels (SURVEY §8f "next" #4: AutoEncoder training,
// train_autoencoder.py:88-148) for gfx950, fp32. Unlike the inference kernels (mobilenet.hip: BN
// folded, blocks fused), training needs every intermediate of DepthWiseConv.forward
// (mobilenetv2.py:153-165) and BatchNorm with batch statistics, so the blocks run as a chain of
// composable kernels, each with its backward:
//   gemm_kernel         strided-batched C (+)= A.B on MFMA-fp32 (1x1 convs: forward, input grad,
//                       weight grad with the pixel/batch reduction split across workgroups)
//   (the depthwise kxk conv and its gradients are in mbt_dw.hip)
//   bn_stats / bn_apply / bn_bwd_reduce / bn_bwd_apply   BatchNorm2d in training mode
//   hardswish fwd/bwd, add, nearest upsample x2 fwd/bwd, plane means (SE pool)
//   se_fc_fwd / se_fc_bwd  the SE MLP (Linear-ReLU-Linear-Hardtanh) per image in one workgroup
// Numerics follow torch's CPU kernels' formulas (fp32), not their summation order.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "det.h"
#include "x3.h"

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
// 4 waves x 32x32 (v_mfma_f32_32x32x2_f32), K in chunks of 32 through LDS; the next chunk's global
// loads are issued before the current chunk's MFMAs (register prefetch). grid.z = batch * ksplit;
// with part != null every (image, K-split) tile is stored dense into part[z][m][n] (z = blockIdx.z)
// and gemm_reduce_kernel sums them in z order into C (no atomics: deterministic).
// Folding (NCHW 1x1 convs): foldN = P folds the image index into N (column n -> image n / P, pixel
// n % P through the batch strides of B and C), so small planes still fill 64-wide tiles; foldK = P
// folds it into K (the weight gradient's reduction over images x pixels). Both need batch == 1.
// ------------------------------------------------------------------------------------------------
struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  float* part;  // partial tiles [batch * ksplit][M][N], or null: C written directly
  int64_t sAb, sAm, sAk, sBb, sBk, sBn, sCb, sCm, sCn;
  int M, N, K, batch, ksplit, kchunk, accumulate, foldK, foldN;
  int vecA, vecB;  // k-contiguous A / B read as float4 runs of 4 k (host-checked alignment, below)
};

typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4g __attribute__((ext_vector_type(4)));
constexpr int GT = 64, GK = 32, GP = GT + 1, GL = GK * GT / kT;

__global__ __launch_bounds__(kT) void gemm_kernel(GemmArgs a) {
  __shared__ float As[GK * GP];  // [k][m]
  __shared__ float Bs[GK * GP];  // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  const int b = blockIdx.z / a.ksplit, ks = blockIdx.z % a.ksplit;
  const int kbeg = ks * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  // staging maps: the contiguous dimension runs along consecutive threads
  const bool akf = a.sAk == 1, bnf = a.sBn == 1;
  const float* A = a.A + b * a.sAb;
  const float* B = a.B + b * a.sBb;
  // fixed per-thread coordinates of the staged elements
  const int a_k = tid & 31, a_m = tid >> 5;   // k-fast A: k = a_k, m = a_m + 8i
  const int a_m2 = tid & 63, a_k2 = tid >> 6;  // m-fast A: m = a_m2, k = a_k2 + 4i
  const int b_n = tid & 63, b_k = tid >> 6;    // n-fast B: n = b_n, k = b_k + 4i
  const int b_k2 = tid & 31, b_n2 = tid >> 5;  // k-fast B: k = b_k2, n = b_n2 + 8i
  int64_t bcol = 0;                             // n-fast B column offset (with the folded image)
  if (bnf) {
    const int gn = n0 + b_n;
    if (a.foldN) {
      const int bb = gn / a.foldN;
      bcol = bb * a.sBb + (int64_t)(gn - bb * a.foldN);
    } else {
      bcol = gn;
    }
  }
  f32x8 ra, rb;
  // float4 staging of a k-contiguous operand: thread t loads k = 4 (t & 7) .. + 3 of rows t >> 3 and
  // (t >> 3) + 32 -- two 16-byte loads where the scalar map makes eight 4-byte ones; a run of 4 k
  // never straddles an image or the chunk end (K, kchunk, foldK multiples of 4: host-checked)
  const int v_k = 4 * (tid & 7), v_r = tid >> 3;
  auto vload = [&](const float* base, int64_t sRow, int64_t sImg, int r0, int rmax, int k0, int kend_) {
    const int gk = k0 + v_k;
    int64_t kb = gk;
    if (a.foldK) {
      const int bb = gk / a.foldK;
      kb = bb * sImg + (int64_t)(gk - bb * a.foldK);
    }
    f32x8 v;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int gr = r0 + v_r + 32 * p;
      const f32x4g q = (gk < kend_ && gr < rmax) ? *reinterpret_cast<const f32x4g*>(base + (int64_t)gr * sRow + kb)
                                                 : f32x4g{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * p + j] = q[j];
    }
    return v;
  };
  auto load = [&](int k0) {
    if (akf && a.vecA) {
      ra = vload(A, a.sAm, a.sAb, m0, a.M, k0, kend);
    } else if (akf) {
      const int gk = k0 + a_k;
      int64_t kb = gk;
      if (a.foldK) {
        const int bb = gk / a.foldK;
        kb = bb * a.sAb + (int64_t)(gk - bb * a.foldK);
      }
#pragma unroll
      for (int i = 0; i < GL; ++i) {
        const int gm = m0 + a_m + 8 * i;
        ra[i] = (gk < kend && gm < a.M) ? A[gm * a.sAm + kb] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < GL; ++i) {
        const int gk = k0 + a_k2 + 4 * i, gm = m0 + a_m2;
        ra[i] = (gk < kend && gm < a.M) ? A[gm * a.sAm + (int64_t)gk * a.sAk] : 0.f;
      }
    }
    if (bnf) {
#pragma unroll
      for (int i = 0; i < GL; ++i) {
        const int gk = k0 + b_k + 4 * i;
        rb[i] = (gk < kend && n0 + b_n < a.N) ? B[(int64_t)gk * a.sBk + bcol] : 0.f;
      }
    } else if (a.vecB) {
      rb = vload(B, a.sBn, a.sBb, n0, a.N, k0, kend);
    } else {
      const int gk = k0 + b_k2;
      int64_t kb = (int64_t)gk * a.sBk;
      if (a.foldK) {
        const int bb = gk / a.foldK;
        kb = bb * a.sBb + (int64_t)(gk - bb * a.foldK) * a.sBk;
      }
#pragma unroll
      for (int i = 0; i < GL; ++i) {
        const int gn = n0 + b_n2 + 8 * i;
        rb[i] = (gk < kend && gn < a.N) ? B[kb + gn * a.sBn] : 0.f;
      }
    }
  };
  f32x16 acc = (f32x16){0.f};
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += GK) {
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      if (akf && a.vecA) As[(v_k + (i & 3)) * GP + v_r + 32 * (i >> 2)] = ra[i];
      else if (akf) As[a_k * GP + a_m + 8 * i] = ra[i];
      else As[(a_k2 + 4 * i) * GP + a_m2] = ra[i];
      if (bnf) Bs[(b_k + 4 * i) * GP + b_n] = rb[i];
      else if (a.vecB) Bs[(v_k + (i & 3)) * GP + v_r + 32 * (i >> 2)] = rb[i];
      else Bs[b_k2 * GP + b_n2 + 8 * i] = rb[i];
    }
    __syncthreads();
    if (k0 + GK < kend) load(k0 + GK);
#pragma unroll
    for (int kp = 0; kp < GK / 2; ++kp)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[(2 * kp + h) * GP + wm * 32 + r], Bs[(2 * kp + h) * GP + wn * 32 + r],
                                                 acc, 0, 0, 0);
    __syncthreads();
  }
  const int n = n0 + wn * 32 + r;
  if (n >= a.N) return;
  if (a.part) {
    float* P = a.part + (int64_t)blockIdx.z * a.M * a.N + n;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (m < a.M) P[(int64_t)m * a.N] = acc[i];
    }
    return;
  }
  int64_t ccol;
  if (a.foldN) {
    const int bb = n / a.foldN;
    ccol = bb * a.sCb + (int64_t)(n - bb * a.foldN) * a.sCn;
  } else {
    ccol = b * a.sCb + (int64_t)n * a.sCn;
  }
  float* C = a.C + ccol;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (m < a.M) {
      float* c = C + m * a.sCm;
      *c = a.accumulate ? *c + acc[i] : acc[i];
    }
  }
}

// Wide-N form for the forward / input-gradient 1x1 convs (batch 1, B and C pixel-contiguous, no K
// split, pixels per image a multiple of 4): 64 (m) x 256 (n) per workgroup, so each B row is read
// as one 1 KB run per wave instruction (16-byte loads) -- gemm_kernel's 64-column tiles read
// 256-byte runs of 16-240 rows that lie 100 KB apart and streamed at 2.3-2.7 TB/s
// (profiles/r03_gemm_probe.txt). Wave w owns columns 64w .. 64w + 63 and all 64 rows (2 x 2
// accumulators of 32 x 32; the second row block is skipped when M <= 32); K in chunks of 16 with
// the next chunk's loads in flight during the MFMAs. Same products and k order as gemm_kernel.
#ifndef WGW_K
#define WGW_K 16  // k rows per chunk (32 and 64 measured slower: profiles/r04_gemm_wide_variants.txt)
#endif
constexpr int WGN = 256, WGK = WGW_K;
#ifndef WGW_T_NOSTORE
#define WGW_T_NOSTORE 0  // timing builds: gemm_wide_kernel without its C stores (wrong results)
#endif

__global__ __launch_bounds__(kT) void gemm_wide_kernel(GemmArgs a, int P) {
  __shared__ float As[WGK][GT + 4];   // [k][m]
  __shared__ float Bs[WGK][WGN + 4];  // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * GT;
  const int n0 = blockIdx.x * WGN;
  const bool two = m0 + 32 < a.M;  // second 32-row block live (uniform)
  // B staging: quad qn = tid & 63 of row kr = (tid >> 6) + 4 i; A staging: row m = tid >> 2, k 4 (tid & 3) + j
  const int qn = tid & 63, kr0 = tid >> 6;
  const int nq = n0 + 4 * qn;
  const bool nv = nq < a.N;  // a quad never straddles images (P % 4 == 0, N % 4 == 0)
  const int img = nv ? nq / P : 0;
  const float* bbase = a.B + (int64_t)img * a.sBb + (nq - img * P);
  const int am = tid >> 2, ak = (WGK / 4) * (tid & 3);
  const bool amv = m0 + am < a.M;
  const float* abase = a.A + (int64_t)(m0 + am) * a.sAm;
  float4 rb[WGK / 4];
  float ra[WGK / 4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < WGK / 4; ++i) {
      const int k = k0 + kr0 + 4 * i;
      rb[i] = (nv && k < a.K) ? *reinterpret_cast<const float4*>(bbase + (int64_t)k * a.sBk) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < WGK / 4; ++j) {
      const int k = k0 + ak + j;
      ra[j] = (amv && k < a.K) ? abase[(int64_t)k * a.sAk] : 0.f;
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0.f};
  load(0);
  for (int k0 = 0; k0 < a.K; k0 += WGK) {
#pragma unroll
    for (int i = 0; i < WGK / 4; ++i) *reinterpret_cast<float4*>(&Bs[kr0 + 4 * i][4 * qn]) = rb[i];
#pragma unroll
    for (int j = 0; j < WGK / 4; ++j) As[ak + j][am] = ra[j];
    __syncthreads();
    if (k0 + WGK < a.K) load(k0 + WGK);
#pragma unroll
    for (int kp = 0; kp < WGK / 2; ++kp) {
      const float a0 = As[2 * kp + h][r], a1 = As[2 * kp + h][32 + r];
      const float b0 = Bs[2 * kp + h][64 * wave + r], b1 = Bs[2 * kp + h][64 * wave + 32 + r];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      if (two) {
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int n = n0 + 64 * wave + 32 * ni + r;
    if (n >= a.N) continue;
    const int im = n / P;
    float* cc = a.C + (int64_t)im * a.sCb + (n - im * P);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      if (mi == 1 && !two) break;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = m0 + 32 * mi + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < a.M && (!WGW_T_NOSTORE || acc[mi][ni][i] == 1.2345e-30f)) {
          float* c = cc + (int64_t)m * a.sCm;
          *c = a.accumulate ? *c + acc[mi][ni][i] : acc[mi][ni][i];
        }
      }
    }
  }
}

// C[b][m][n] (+)= sum over the tiles z of C's image (z = b * ksplit + ks; all z when C is shared
// across the batch, sCb == 0) of part[z][m][n], in z order.
__global__ __launch_bounds__(kT) void gemm_reduce_kernel(GemmArgs a, int zper) {
  const int64_t mn = (int64_t)a.M * a.N;
  const int cb = blockIdx.y;  // C image (0 when shared)
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < mn; e += (int64_t)gridDim.x * kT) {
    const float* p = a.part + (int64_t)cb * zper * mn + e;
    float s = 0.f;
    int z = 0;
    // 16 loads in flight per thread, added in z order (the grid is small: mn is a weight's size)
    for (; z + 16 <= zper; z += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(int64_t)(z + u) * mn];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; z + 4 <= zper; z += 4) {
      const float v0 = p[(int64_t)z * mn], v1 = p[(int64_t)(z + 1) * mn];
      const float v2 = p[(int64_t)(z + 2) * mn], v3 = p[(int64_t)(z + 3) * mn];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; z < zper; ++z) s += p[(int64_t)z * mn];
    const int m = (int)(e / a.N), n = (int)(e - (int64_t)m * a.N);
    int64_t ccol;
    if (a.foldN) {
      const int bb = n / a.foldN;
      ccol = bb * a.sCb + (int64_t)(n - bb * a.foldN) * a.sCn;
    } else {
      ccol = (int64_t)cb * a.sCb + (int64_t)n * a.sCn;
    }
    float* c = a.C + ccol + (int64_t)m * a.sCm;
    *c = a.accumulate ? *c + s : s;
  }
}

// ------------------------------------------------------------------------------------------------
// Split-bf16 GEMM (the default for the 1x1 convs): C = A.B with fp32 inputs carried as three bf16
// terms (x3.h) and the six largest term products, folded into three v_mfma_f32_16x16x32_bf16 per 16
// channels of K (conv3x3_igemm.hip's M16 scheme) -- fp32-level accuracy at 2.7x the fp32 MFMA rate,
// so the skinny-K / skinny-MN shapes of a MobileNet block stay HBM-bound.
// Tile BM (m) x BN (n), 4 waves of (BM/2) x (BN/2), K in chunks of 32. The MFMA's A operand is the
// N side (B^T rows), its B operand the M side, so a lane's accumulator holds 4 consecutive n of one
// m: the epilogue writes 16-byte vectors along n (C rows are n-contiguous in every caller).
// LDS: per side [3 terms][rows][32 + 8] bf16 (80-byte rows: the b128 fragment reads of 16 rows hit
// distinct banks). Staging: a thread owns (row, 8 consecutive k) items -- two 16-byte loads when k
// is contiguous, else eight loads coalesced across the lanes' consecutive rows -- splits them and
// writes one 16-byte vector per term; the next chunk's loads are in flight during the MFMAs.
// Folded K (foldK = P) needs P % 8 == 0 so that 8 consecutive k stay in one image (host-checked).
// ------------------------------------------------------------------------------------------------
constexpr int X3KC = 32, X3KP = X3KC + 8;

struct X3Flags {
  int vecA, vecB, vecC, vecP;  // 16-byte paths legal: A / B k-runs, C / partial-tile n-runs
  int ntn;                     // n-tiles; a workgroup walks n-tiles blockIdx.x, + gridDim.x, ...
};

// Staging map of one operand side with R rows: item it -> (row, 8-k group). When k is the
// contiguous dimension, 4 consecutive lanes take the 4 groups of one row (128-byte runs per row);
// otherwise consecutive lanes take consecutive rows (every k load coalesced across the lanes).
template <int R>
__device__ __forceinline__ void x3_item(int it, bool kfast, int& row, int& kg) {
  if (kfast) {
    row = it >> 2;
    kg = it & 3;
  } else {
    row = it % R;
    kg = it / R;
  }
}

template <int BM, int BN>
__global__ __launch_bounds__(kT, 2) void gemm_x3_kernel(GemmArgs a, X3Flags f) {
  using ast_x3::bf16;
  using ast_x3::bf16x8;
  using ast_x3::f32x4;
  __shared__ __attribute__((aligned(16))) bf16 Ns[3][BN][X3KP];
  __shared__ __attribute__((aligned(16))) bf16 Ms[3][BM][X3KP];
  constexpr int WN = BN / 2, WM = BM / 2, TN = WN / 16, TM = WM / 16;
  constexpr int NI = BN * 4 / kT, MI = BM * 4 / kT;  // staging items per thread
  static_assert(NI >= 1 && MI >= 1 && BN * 4 % kT == 0 && BM * 4 % kT == 0, "tile");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int m0 = blockIdx.y * BM;
  const int b = blockIdx.z / a.ksplit, ks = blockIdx.z % a.ksplit;
  const int kbeg = ks * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  if ((int)blockIdx.x >= f.ntn) return;  // (an empty K split still stores its zero tiles)
  const bool kfA = a.sAk == 1, kfB = a.sBk == 1;
  const float* A = a.A + b * a.sAb;
  const float* B = a.B + b * a.sBb;
  // k offsets: folded K walks images through the batch stride (batch == 1 then)
  auto koffA = [&](int k) -> int64_t {
    if (a.foldK) {
      const int bb = k / a.foldK;
      return bb * a.sAb + (int64_t)(k - bb * a.foldK) * a.sAk;
    }
    return (int64_t)k * a.sAk;
  };
  auto koffB = [&](int k) -> int64_t {
    if (a.foldK) {
      const int bb = k / a.foldK;
      return bb * a.sBb + (int64_t)(k - bb * a.foldK) * a.sBk;
    }
    return (int64_t)k * a.sBk;
  };
  int64_t noff[NI], moff[MI];
  bool nok[NI], mok[MI];
  auto set_ntile = [&](int t) {  // per-item column offsets of n-tile t
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      int row, kg;
      x3_item<BN>(tid + i * kT, kfB, row, kg);
      const int n = t * BN + row;
      nok[i] = n < a.N;
      if (a.foldN) {
        const int bb = n / a.foldN;
        noff[i] = bb * a.sBb + (int64_t)(n - bb * a.foldN) * a.sBn;
      } else {
        noff[i] = (int64_t)n * a.sBn;
      }
    }
  };
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    int row, kg;
    x3_item<BM>(tid + i * kT, kfA, row, kg);
    const int m = m0 + row;
    mok[i] = m < a.M;
    moff[i] = (int64_t)m * a.sAm;
  }
  float rn[NI][8], rm[MI][8];
  auto load8 = [&](const float* base, bool ok, int kf, int64_t sK, bool vec, float* v) {
    if (ok && vec && kf + 8 <= kend) {
      const f32x4 u0 = *(const f32x4*)base, u1 = *(const f32x4*)(base + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = u0[j];
        v[4 + j] = u1[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (ok && kf + j < kend) ? base[j * sK] : 0.f;
    }
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      int row, kg;
      x3_item<BN>(tid + i * kT, kfB, row, kg);
      const int kf = k0 + 8 * kg;
      const float* p = B + noff[i] + (kf < kend ? koffB(kf) : 0);
      load8(p, nok[i], kf, a.sBk, f.vecB, rn[i]);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      int row, kg;
      x3_item<BM>(tid + i * kT, kfA, row, kg);
      const int kf = k0 + 8 * kg;
      const float* p = A + moff[i] + (kf < kend ? koffA(kf) : 0);
      load8(p, mok[i], kf, a.sAk, f.vecA, rm[i]);
    }
  };
  auto split_store = [&](const float* v, bf16* d0, bf16* d1, bf16* d2) {
    bf16x8 t0, t1, t2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16 h, md, l;
      ast_x3::split3(v[j], h, md, l);
      t0[j] = h;
      t1[j] = md;
      t2[j] = l;
    }
    *(bf16x8*)d0 = t0;
    *(bf16x8*)d1 = t1;
    *(bf16x8*)d2 = t2;
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      int row, kg;
      x3_item<BN>(tid + i * kT, kfB, row, kg);
      split_store(rn[i], &Ns[0][row][8 * kg], &Ns[1][row][8 * kg], &Ns[2][row][8 * kg]);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      int row, kg;
      x3_item<BM>(tid + i * kT, kfA, row, kg);
      split_store(rm[i], &Ms[0][row][8 * kg], &Ms[1][row][8 * kg], &Ms[2][row][8 * kg]);
    }
  };
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r16 = lane & 15;
  const bool first = g < 2;
  // epilogue of n-tile t: lane holds D[n = 4 (lane >> 4) + r][m = lane & 15] of each 16 x 16 tile
  auto epilogue = [&](int t) {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = t * BN + wn * WN + i * 16 + 4 * g;
      if (n >= a.N) continue;
      const bool full = n + 3 < a.N;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * WM + j * 16 + r16;
        if (m >= a.M) continue;
        const f32x4 v = acc[i][j];
        if (a.part) {
          float* P = a.part + ((int64_t)blockIdx.z * a.M + m) * a.N + n;
          if (full && f.vecP) {
            *(f32x4*)P = v;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < a.N) P[r] = v[r];
          }
          continue;
        }
        if (full && f.vecC) {  // 4 consecutive n in one image, n-contiguous and aligned (host-checked)
          int64_t ccol;
          if (a.foldN) {
            const int bb = n / a.foldN;
            ccol = bb * a.sCb + (int64_t)(n - bb * a.foldN);
          } else {
            ccol = b * a.sCb + n;
          }
          f32x4* c = (f32x4*)(a.C + ccol + (int64_t)m * a.sCm);
          *c = a.accumulate ? *c + v : v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nn = n + r;
            if (nn >= a.N) break;
            int64_t ccol;
            if (a.foldN) {
              const int bb = nn / a.foldN;
              ccol = bb * a.sCb + (int64_t)(nn - bb * a.foldN) * a.sCn;
            } else {
              ccol = b * a.sCb + (int64_t)nn * a.sCn;
            }
            float* c = a.C + ccol + (int64_t)m * a.sCm;
            *c = a.accumulate ? *c + v[r] : v[r];
          }
        }
      }
    }
  };
  // (n-tile, K chunk) pairs in one pipelined walk: the next pair's loads (the next tile's first
  // chunk after a tile's last) are in flight during this pair's MFMAs and the tile's epilogue
  int t = blockIdx.x, k0 = kbeg;
  set_ntile(t);
  load(k0);
  for (;;) {
    __syncthreads();  // the previous chunk's fragments are read
    stage();
    __syncthreads();
    int nt = t, nk = k0 + X3KC;
    if (nk >= kend) {
      nt = t + gridDim.x;
      nk = kbeg;
    }
    const bool more = nt < f.ntn;
    if (more) {
      if (nt != t) set_ntile(nt);
      load(nk);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ko = s * 16 + 8 * (g & 1);
      bf16x8 f1[TN], f2[TN], g1[TM], g2[TM], g3[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int row = wn * WN + i * 16 + r16;
        f1[i] = *(const bf16x8*)&Ns[first ? 0 : 1][row][ko];
        f2[i] = *(const bf16x8*)&Ns[first ? 0 : 2][row][ko];
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int row = wm * WM + j * 16 + r16;
        g1[j] = *(const bf16x8*)&Ms[0][row][ko];
        g2[j] = *(const bf16x8*)&Ms[first ? 1 : 0][row][ko];
        g3[j] = *(const bf16x8*)&Ms[first ? 2 : 1][row][ko];
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          f32x4 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[i], g3[j], c, 0, 0, 0);  // n_hi m_lo + n_mid m_mid
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f2[i], g2[j], c, 0, 0, 0);  // n_hi m_mid + n_lo m_hi
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[i], g1[j], c, 0, 0, 0);  // n_hi m_hi + n_mid m_hi
        }
    }
    if (k0 + X3KC >= kend) {  // the tile's last chunk: store and restart the accumulators
      epilogue(t);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    if (!more) break;
    t = nt;
    k0 = nk;
  }
}

// ------------------------------------------------------------------------------------------------
// BatchNorm2d, training mode: batch mean and biased variance over (N, H, W) per channel,
// y = (x - mean) * invstd * gamma + beta, invstd = 1/sqrt(var + eps); running statistics with
// momentum and the unbiased variance (torch's batch_norm update).
// Statistics in two steps: every (segment, image, channel) workgroup writes its count, mean and
// M2 (sums shifted by the segment's first element against cancellation), then one thread per
// channel merges them in double (Chan et al.'s pairwise update).
// ------------------------------------------------------------------------------------------------
constexpr int BN_SEG = 16 * kT;

__global__ __launch_bounds__(kT) void bn_part_stats_kernel(const float* __restrict__ x, int c, int64_t hw,
                                                           float* __restrict__ part) {
  __shared__ float sh[kT / 64];
  const int sx = blockIdx.x, b = blockIdx.y, ch = blockIdx.z;
  const float* xp = x + ((int64_t)b * c + ch) * hw + (int64_t)sx * BN_SEG;
  const int len = (int)min((int64_t)BN_SEG, hw - (int64_t)sx * BN_SEG);
  const float k0 = xp[0];
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < len; i += kT) {
    const float d = xp[i] - k0;
    s1 += d;
    s2 = fmaf(d, d, s2);
  }
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    const int S = gridDim.x * gridDim.y;
    float* o = part + ((int64_t)ch * S + (int64_t)b * gridDim.x + sx) * 3;
    const float inv = 1.0f / (float)len;
    o[0] = (float)len;
    o[1] = k0 + s1 * inv;
    o[2] = fmaxf(s2 - s1 * s1 * inv, 0.f);
  }
}

// per channel: Chan merge of the S segment partials into this process's (count, mean, M2), double
__global__ void bn_local_stats_kernel(const float* __restrict__ part, int S, int c, double* __restrict__ stats) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float* p = part + (int64_t)ch * S * 3;
  double na = p[0], mu = p[1], m2 = p[2];
  for (int i = 1; i < S; ++i) {
    const double nb = p[3 * i], mb = p[3 * i + 1], m2b = p[3 * i + 2];
    const double nt = na + nb, d = mb - mu;
    mu += d * nb / nt;
    m2 += m2b + d * d * na * nb / nt;
    na = nt;
  }
  stats[3 * ch] = na;
  stats[3 * ch + 1] = mu;
  stats[3 * ch + 2] = m2;
}

// merge `parts` processes' [parts][c][3] statistics (SyncBatchNorm: gathered over ranks; 1 part
// on one GPU) into mean / invstd, the running statistics and 1 / total count
__global__ void bn_merge_stats_kernel(const double* __restrict__ stats, int parts, int c, float eps, float momentum,
                                      float* __restrict__ mean, float* __restrict__ invstd,
                                      float* __restrict__ run_mean, float* __restrict__ run_var,
                                      float* __restrict__ inv_count) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  double na = 0.0, mu = 0.0, m2 = 0.0;
  for (int r = 0; r < parts; ++r) {
    const double* p = stats + ((int64_t)r * c + ch) * 3;
    const double nb = p[0];
    if (nb <= 0.0) continue;
    const double nt = na + nb, d = p[1] - mu;
    mu += d * nb / nt;
    m2 += p[2] + d * d * na * nb / nt;
    na = nt;
  }
  const double var = na > 0.0 ? m2 / na : 0.0;
  mean[ch] = (float)mu;
  invstd[ch] = 1.0f / sqrtf((float)var + eps);
  if (run_mean) {
    run_mean[ch] = (1.f - momentum) * run_mean[ch] + momentum * (float)mu;
    run_var[ch] = (1.f - momentum) * run_var[ch] + momentum * (float)(na > 1 ? m2 / (na - 1) : var);
  }
  if (inv_count && ch == 0) inv_count[0] = (float)(1.0 / na);
}

// op 0 hardswish(a), 1 hardswish backward (x = a, g = b; torch: x < -3: 0; x <= 3: g (x/3 + 1/2);
// else g), 2 a + b
template <int OP>
__device__ __forceinline__ float elt(float a, float b) {
  if (OP == 0) return a * fminf(fmaxf(a + 3.f, 0.f), 6.f) / 6.f;
  if (OP == 1) return a < -3.f ? 0.f : (a <= 3.f ? b * (a / 3.f + 0.5f) : b);
  return a + b;
}

// the BatchNorm affine, one expression for the forward and the backward's recomputation (so a
// fused Hardswish sees bit-identical inputs in both)
__device__ __forceinline__ float bn_aff(float x, float mu, float sc, float bt) { return (x - mu) * sc + bt; }

// grid (chunks of 4*kT pixels, planes (strided by gridDim.y)); ACT 1: Hardswish of the output
// (DepthWiseConv's BatchNorm2d -> Hardswish pair, mobilenetv2.py:122-126, in one pass)
template <int ACT>
__global__ __launch_bounds__(kT) void bn_apply_kernel(const float* __restrict__ x, int c, int64_t hw, int planes,
                                                      const float* __restrict__ mean, const float* __restrict__ invstd,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float* __restrict__ y) {
  for (int pl = blockIdx.y; pl < planes; pl += gridDim.y) {
    const int ch = pl % c;
    const float sc = invstd[ch] * (gamma ? gamma[ch] : 1.f), mu = mean[ch], bt = beta ? beta[ch] : 0.f;
    const float* xp = x + (int64_t)pl * hw;
    float* yp = y + (int64_t)pl * hw;
    if ((hw & 3) == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {  // one 16-byte access per thread
      const int64_t i4 = (int64_t)blockIdx.x * kT + threadIdx.x;
      if (4 * i4 < hw) {
        const float4 xv = reinterpret_cast<const float4*>(xp)[i4];
        float v[4] = {bn_aff(xv.x, mu, sc, bt), bn_aff(xv.y, mu, sc, bt), bn_aff(xv.z, mu, sc, bt),
                      bn_aff(xv.w, mu, sc, bt)};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ACT ? elt<0>(v[e], 0.f) : v[e];
        reinterpret_cast<float4*>(yp)[i4] = make_float4(v[0], v[1], v[2], v[3]);
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = (int64_t)blockIdx.x * 4 * kT + j * kT + threadIdx.x;
      if (i < hw) {
        const float v = bn_aff(xp[i], mu, sc, bt);
        yp[i] = ACT ? elt<0>(v, 0.f) : v;
      }
    }
  }
}

// per (segment, image, channel): sum(dy), sum(dy * xhat); ACT 1: dy is the gradient of
// Hardswish(BN(x)), taken through the Hardswish at the recomputed BN output
template <int ACT>
__global__ __launch_bounds__(kT) void bn_part_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                         int c, int64_t hw, const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ part) {
  __shared__ float sh[kT / 64];
  const int sx = blockIdx.x, b = blockIdx.y, ch = blockIdx.z;
  const int64_t o = ((int64_t)b * c + ch) * hw + (int64_t)sx * BN_SEG;
  const int len = (int)min((int64_t)BN_SEG, hw - (int64_t)sx * BN_SEG);
  const float mu = mean[ch], is = invstd[ch];
  const float sc = ACT ? is * (gamma ? gamma[ch] : 1.f) : 0.f, bt = ACT && beta ? beta[ch] : 0.f;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < len; i += kT) {
    const float xv = x[o + i];
    const float gv = ACT ? elt<1>(bn_aff(xv, mu, sc, bt), dy[o + i]) : dy[o + i];
    s1 += gv;
    s2 = fmaf(gv, (xv - mu) * is, s2);
  }
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    const int S = gridDim.x * gridDim.y;
    float* p = part + ((int64_t)ch * S + (int64_t)b * gridDim.x + sx) * 2;
    p[0] = s1;
    p[1] = s2;
  }
}

__global__ void bn_finalize_bwd_kernel(const float* __restrict__ part, int S, int c, float* __restrict__ sdy,
                                       float* __restrict__ sdyx, float* __restrict__ inv_count, float inv_value) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float* p = part + (int64_t)ch * S * 2;
  double a = 0.0, b = 0.0;
  for (int i = 0; i < S; ++i) {
    a += p[2 * i];
    b += p[2 * i + 1];
  }
  sdy[ch] = (float)a;    // sum dy      (= dbeta)
  sdyx[ch] = (float)b;   // sum dy xhat (= dgamma)
  if (inv_count && ch == 0) inv_count[0] = inv_value;
}

template <int ACT>
__global__ __launch_bounds__(kT) void bn_bwd_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          int c, int64_t hw, int planes,
                                                          const float* __restrict__ inv_count,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ sdy,
                                                          const float* __restrict__ sdyx, float* __restrict__ dx) {
  for (int pl = blockIdx.y; pl < planes; pl += gridDim.y) {
    const int ch = pl % c;
    const float is = invstd[ch], mu = mean[ch], gm = (gamma ? gamma[ch] : 1.f) * is;
    const float bt = ACT && beta ? beta[ch] : 0.f;
    const float inv_m = inv_count[0], a = sdy[ch] * inv_m, bq = sdyx[ch] * inv_m;
    const int64_t base = (int64_t)pl * hw;
    if ((hw & 3) == 0 && (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) == 0) {  // 16-byte accesses
      const int64_t i4 = (int64_t)blockIdx.x * kT + threadIdx.x;
      if (4 * i4 < hw) {
        const float4 x4 = reinterpret_cast<const float4*>(x + base)[i4];
        const float4 g4 = reinterpret_cast<const float4*>(dy + base)[i4];
        const float xs[4] = {x4.x, x4.y, x4.z, x4.w}, gs[4] = {g4.x, g4.y, g4.z, g4.w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = ACT ? elt<1>(bn_aff(xs[e], mu, gm, bt), gs[e]) : gs[e];
          const float xh = (xs[e] - mu) * is;
          o[e] = gm * (gv - a - xh * bq);
        }
        reinterpret_cast<float4*>(dx + base)[i4] = make_float4(o[0], o[1], o[2], o[3]);
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = (int64_t)blockIdx.x * 4 * kT + j * kT + threadIdx.x;
      if (i < hw) {
        const float xv = x[base + i];
        const float gv = ACT ? elt<1>(bn_aff(xv, mu, gm, bt), dy[base + i]) : dy[base + i];
        const float xh = (xv - mu) * is;
        dx[base + i] = gm * (gv - a - xh * bq);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// elementwise
// ------------------------------------------------------------------------------------------------
// eltwise_kernel: elt<OP> over four elements per thread, as one 16-byte access when the host saw
// n % 4 == 0 and 16-byte aligned pointers.
typedef float f32x4 __attribute__((ext_vector_type(4)));


template <int OP, bool V4>
__global__ __launch_bounds__(kT) void eltwise_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     float* __restrict__ y, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * kT + threadIdx.x) * 4;
  if (V4) {
    if (i0 >= n) return;
    const f32x4 va = *(const f32x4*)(a + i0);
    const f32x4 vb = OP == 0 ? va : *(const f32x4*)(b + i0);
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = elt<OP>(va[j], vb[j]);
    *(f32x4*)(y + i0) = r;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = i0 + j;
      if (i < n) y[i] = elt<OP>(a[i], OP == 0 ? 0.f : b[i]);
    }
  }
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

// per-plane mean (SE AdaptiveAvgPool2d(1)) or, with y, per-plane sum(x * y) (the gate gradient).
// ACT 1: the SE input is hardswish of the stored tensor (DepthWiseConv's Hardswish -> SELayer,
// mobilenetv2.py:151-156, without materialising the activation): mean(hardswish(x)), or
// sum(x * hardswish(y)).
template <int ACT>
__global__ __launch_bounds__(kT) void plane_dot_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       int64_t hw, float scale, float* __restrict__ out) {
  __shared__ float sh[kT / 64];
  const int64_t p = blockIdx.x;
  const float* xp = x + p * hw;
  const float* yp = y ? y + p * hw : nullptr;
  float s = 0.f;
  if ((hw & 3) == 0 && ((uintptr_t)xp & 15) == 0 && (!yp || ((uintptr_t)yp & 15) == 0)) {
    // 16-byte loads, four independent partial sums per thread (a fixed order: deterministic); the
    // scalar loop below issued 4x the loads, each sum one dependent chain
    const float4* x4 = reinterpret_cast<const float4*>(xp);
    const float4* y4 = reinterpret_cast<const float4*>(yp);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    for (int64_t i = threadIdx.x; i < hw / 4; i += kT) {
      const float4 a = x4[i];
      if (yp) {
        const float4 b = y4[i];
        s0 += a.x * (ACT ? elt<0>(b.x, 0.f) : b.x);
        s1 += a.y * (ACT ? elt<0>(b.y, 0.f) : b.y);
        s2 += a.z * (ACT ? elt<0>(b.z, 0.f) : b.z);
        s3 += a.w * (ACT ? elt<0>(b.w, 0.f) : b.w);
      } else {
        s0 += ACT ? elt<0>(a.x, 0.f) : a.x;
        s1 += ACT ? elt<0>(a.y, 0.f) : a.y;
        s2 += ACT ? elt<0>(a.z, 0.f) : a.z;
        s3 += ACT ? elt<0>(a.w, 0.f) : a.w;
      }
    }
    s = (s0 + s1) + (s2 + s3);
  } else {
    for (int64_t i = threadIdx.x; i < hw; i += kT) {
      if (yp) s += xp[i] * (ACT ? elt<0>(yp[i], 0.f) : yp[i]);
      else s += ACT ? elt<0>(xp[i], 0.f) : xp[i];
    }
  }
  const float t = block_sum(s, sh);
  if (threadIdx.x == 0) out[p] = t * scale;
}

// OP 0: y = x * gate[plane] (+ gadd[plane] when given: the SE input gradient dy*g + dpool/hw);
// OP 1: y = hardswish(x) * gate[plane] (the SE output over the un-materialised activation);
// OP 2: y = hardswish'(a) * (x * gate[plane] + gadd[plane]) (the SE input gradient taken on
// through the Hardswish at its input a). grid (chunks of 4*kT pixels, planes strided by gridDim.y)
template <int OP>
__global__ __launch_bounds__(kT) void plane_scale_kernel(const float* __restrict__ x, const float* __restrict__ gate,
                                                         const float* __restrict__ gadd, const float* __restrict__ a,
                                                         int64_t hw, int64_t planes, float* __restrict__ y) {
  const bool v4 = (hw & 3) == 0 && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)(OP == 2 ? a : x)) & 15) == 0;
  for (int64_t p = blockIdx.y; p < planes; p += gridDim.y) {
    const float gv = gate[p], av = gadd ? gadd[p] : 0.f;
    const float* xp = x + p * hw;
    const float* ap = OP == 2 ? a + p * hw : nullptr;
    float* yp = y + p * hw;
    if (v4) {  // the block's 4 kT elements as one 16-byte access per thread (same values)
      const int64_t i4 = (int64_t)blockIdx.x * kT + threadIdx.x;
      if (4 * i4 < hw) {
        const float4 xv = reinterpret_cast<const float4*>(xp)[i4];
        float4 o;
        if (OP == 0) {
          o = make_float4(fmaf(xv.x, gv, av), fmaf(xv.y, gv, av), fmaf(xv.z, gv, av), fmaf(xv.w, gv, av));
        } else if (OP == 1) {
          o = make_float4(elt<0>(xv.x, 0.f) * gv, elt<0>(xv.y, 0.f) * gv, elt<0>(xv.z, 0.f) * gv,
                          elt<0>(xv.w, 0.f) * gv);
        } else {
          const float4 av4 = reinterpret_cast<const float4*>(ap)[i4];
          o = make_float4(elt<1>(av4.x, fmaf(xv.x, gv, av)), elt<1>(av4.y, fmaf(xv.y, gv, av)),
                          elt<1>(av4.z, fmaf(xv.z, gv, av)), elt<1>(av4.w, fmaf(xv.w, gv, av)));
        }
        reinterpret_cast<float4*>(yp)[i4] = o;
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = (int64_t)blockIdx.x * 4 * kT + j * kT + threadIdx.x;
      if (i < hw) {
        if (OP == 0) yp[i] = fmaf(xp[i], gv, av);
        else if (OP == 1) yp[i] = elt<0>(xp[i], 0.f) * gv;
        else yp[i] = elt<1>(ap[i], fmaf(xp[i], gv, av));
      }
    }
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
#pragma unroll 16
    for (int i = 0; i < c; ++i) a = fmaf(w1[(int64_t)j * c + i], pv[i], a);
    a = a > 0.f ? a : 0.f;
    hs[j] = a;
    hid[(int64_t)n * red + j] = a;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < c; i += kT) {
    float a = b2[i];
#pragma unroll 16
    for (int j = 0; j < red; ++j) a = fmaf(w2[(int64_t)i * red + j], hs[j], a);
    z[(int64_t)n * c + i] = a;
    gate[(int64_t)n * c + i] = fminf(fmaxf(a, 0.f), 1.f);
  }
}

// SE MLP backward, per image (one workgroup): dz = dgate * (0 < z < 1), dh = W2^T dz * (hid > 0),
// dpool = W1^T dh (scaled by 1/hw for the broadcast back onto the plane); dz and dh go to the
// workspace ([n][c] then [n][red]) for se_fc_param_grad_kernel.
__global__ __launch_bounds__(kT) void se_fc_bwd_kernel(const float* __restrict__ dgate, const float* __restrict__ z,
                                                       const float* __restrict__ hid, const float* __restrict__ w1,
                                                       const float* __restrict__ w2, int n_img, int c, int red,
                                                       float inv_hw, float* __restrict__ ws,
                                                       float* __restrict__ dpool) {
  extern __shared__ float sm[];
  float* dz = sm;        // [c]
  float* dh = sm + c;    // [red]
  const int n = blockIdx.x;
  float* dzg = ws + (int64_t)n * c;
  float* dhg = ws + (int64_t)n_img * c + (int64_t)n * red;
  for (int i = threadIdx.x; i < c; i += kT) {
    const float zv = z[(int64_t)n * c + i];
    const float d = (zv > 0.f && zv < 1.f) ? dgate[(int64_t)n * c + i] : 0.f;
    dz[i] = d;
    dzg[i] = d;
  }
  __syncthreads();
  const float* hv = hid + (int64_t)n * red;
  for (int j = threadIdx.x; j < red; j += kT) {
    float a = 0.f;
#pragma unroll 16
    for (int i = 0; i < c; ++i) a = fmaf(w2[(int64_t)i * red + j], dz[i], a);
    a = hv[j] > 0.f ? a : 0.f;
    dh[j] = a;
    dhg[j] = a;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < c; i += kT) {
    float a = 0.f;
#pragma unroll 16
    for (int j = 0; j < red; ++j) a = fmaf(w1[(int64_t)j * c + i], dh[j], a);
    dpool[(int64_t)n * c + i] = a * inv_hw;
  }
}

// SE parameter gradients, one thread per parameter, summed over the images in image order:
// dW2[i][j] = sum_n dz[n][i] hid[n][j], db2[i] = sum_n dz[n][i], dW1[j][i] = sum_n dh[n][j] pool[n][i],
// db1[j] = sum_n dh[n][j].
__global__ __launch_bounds__(kT) void se_fc_param_grad_kernel(const float* __restrict__ ws,
                                                              const float* __restrict__ hid,
                                                              const float* __restrict__ pool, int n_img, int c,
                                                              int red, float* __restrict__ dw1,
                                                              float* __restrict__ db1, float* __restrict__ dw2,
                                                              float* __restrict__ db2) {
  const float* dz = ws;
  const float* dh = ws + (int64_t)n_img * c;
  const int64_t cr = (int64_t)c * red, total = 2 * cr + c + red;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    float s = 0.f;
    if (e < cr) {  // dW2[i][j]
      const int i = (int)(e / red), j = (int)(e - (int64_t)i * red);
      for (int n = 0; n < n_img; ++n) s = fmaf(dz[(int64_t)n * c + i], hid[(int64_t)n * red + j], s);
      dw2[e] = s;
    } else if (e < 2 * cr) {  // dW1[j][i]
      const int64_t f = e - cr;
      const int j = (int)(f / c), i = (int)(f - (int64_t)j * c);
      for (int n = 0; n < n_img; ++n) s = fmaf(dh[(int64_t)n * red + j], pool[(int64_t)n * c + i], s);
      dw1[f] = s;
    } else if (e < 2 * cr + c) {
      const int i = (int)(e - 2 * cr);
      for (int n = 0; n < n_img; ++n) s += dz[(int64_t)n * c + i];
      db2[i] = s;
    } else {
      const int j = (int)(e - 2 * cr - c);
      for (int n = 0; n < n_img; ++n) s += dh[(int64_t)n * red + j];
      db1[j] = s;
    }
  }
}

dim3 plane_grid(int64_t hw, int64_t planes) {
  return dim3((unsigned)((hw + 4 * kT - 1) / (4 * kT)), (unsigned)(planes < 65535 ? planes : 65535));
}

template <int OP>
void launch_eltwise(const float* a, const float* b, float* y, int64_t n, hipStream_t st) {
  const bool v4 = (n & 3) == 0 && (((uintptr_t)a | (uintptr_t)(b ? b : a) | (uintptr_t)y) & 15) == 0;
  const dim3 grid((unsigned)((n + 4 * kT - 1) / (4 * kT)));
  if (v4) hipLaunchKernelGGL((eltwise_kernel<OP, true>), grid, dim3(kT), 0, st, a, b, y, n);
  else hipLaunchKernelGGL((eltwise_kernel<OP, false>), grid, dim3(kT), 0, st, a, b, y, n);
}

}  // namespace

extern "C" {

long long ast_mbt_gemm_workspace_floats(int M, int N, int batch, int ksplit, long long sCb) {
  if (M <= 0 || N <= 0 || batch <= 0 || ksplit <= 0) return 0;
  const bool part = ksplit > 1 || (sCb == 0 && batch > 1);
  return part ? (long long)batch * ksplit * M * N : 0;
}

int ast_mbt_gemm_f32(const float* A, const float* B, float* C, int M, int N, int K, int batch, long long sAb,
                     long long sAm, long long sAk, long long sBb, long long sBk, long long sBn, long long sCb,
                     long long sCm, long long sCn, int ksplit, int accumulate, int foldK, int foldN,
                     float* workspace, long long workspace_floats, void* stream) {
  if (!A || !B || !C) return AST_E_NULLPTR;
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || ksplit <= 0 || foldK < 0 || foldN < 0) return AST_E_SHAPE;
  if (((int64_t)M + GT - 1) / GT > 65535 || (int64_t)batch * ksplit > 65535) return AST_E_SHAPE;
  if ((foldK || foldN) && (batch != 1 || (foldK && foldN))) return AST_E_SHAPE;
  if (foldK && (sAk != 1 || sBk != 1 || K % foldK)) return AST_E_UNSUPPORTED;  // both operands k-contiguous
  if (foldN && (sBn != 1 || N % foldN)) return AST_E_UNSUPPORTED;
  const long long need = ast_mbt_gemm_workspace_floats(M, N, batch, ksplit, sCb);
  if (need > 0 && !workspace) return AST_E_NULLPTR;
  if (workspace_floats < need) return AST_E_SHAPE;
  GemmArgs a{A, B, C, need > 0 ? workspace : nullptr, sAb, sAm, sAk, sBb, sBk, sBn, sCb, sCm, sCn, M, N, K, batch,
             ksplit, 0, accumulate, foldK, foldN, 0, 0};
  a.kchunk = ((K + ksplit - 1) / ksplit + GK - 1) / GK * GK;
  {  // float4 k-runs: K, the chunk and the folded image stride multiples of 4, 16-byte aligned rows
    static const int vec = [] {  // AST_MBGEMM_VEC=0: scalar staging (A/B runs)
      const char* v = getenv("AST_MBGEMM_VEC");
      return v ? atoi(v) : 1;
    }();
    const bool kok = vec && K % 4 == 0 && a.kchunk % 4 == 0 && (foldK == 0 || foldK % 4 == 0);
    a.vecA = kok && sAk == 1 && sAm % 4 == 0 && sAb % 4 == 0 && ((uintptr_t)A & 15) == 0;
    a.vecB = kok && sBk == 1 && sBn != 1 && sBn % 4 == 0 && sBb % 4 == 0 && ((uintptr_t)B & 15) == 0;
  }
  hipStream_t st = (hipStream_t)stream;
  // AST_MBGEMM_X3=1: the split-bf16 kernel (fp32-level accuracy, repeatable; measured 3% slower
  // on the AST step than the fp32-MFMA kernel, whose skinny-K shapes are latency-, not MFMA-bound)
  static const int x3 = [] {
    const char* v = getenv("AST_MBGEMM_X3");
    return v ? atoi(v) : 0;
  }();
  const dim3 grid((unsigned)((N + GT - 1) / GT), (unsigned)((M + GT - 1) / GT), (unsigned)(batch * ksplit));
  static const int wide = [] {  // AST_MBGEMM_WIDE=0: gemm_kernel for these shapes too (A/B measurements)
    const char* v = getenv("AST_MBGEMM_WIDE");
    return v ? atoi(v) : 1;
  }();
  {
    const int P = foldN ? foldN : N;
    if (wide && !x3 && batch == 1 && ksplit == 1 && !foldK && sBn == 1 && sCn == 1 && need == 0 && P % 4 == 0 &&
        N % 4 == 0 && sBk % 4 == 0 && (foldN == 0 || sBb % 4 == 0) && ((uintptr_t)B & 15) == 0) {
      const dim3 g((unsigned)((N + WGN - 1) / WGN), (unsigned)((M + GT - 1) / GT));
      hipLaunchKernelGGL(gemm_wide_kernel, g, dim3(kT), 0, st, a, P);
      return (int)hipGetLastError();
    }
  }
  if (x3 && (foldK == 0 || foldK % 8 == 0)) {  // split-bf16 path (8 consecutive k stay in one image)
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    X3Flags fl{};
    fl.vecA = sAk == 1 && al(A) && sAm % 4 == 0 && (sAb % 4 == 0 || (batch == 1 && !foldK));
    fl.vecB = sBk == 1 && al(B) && sBn % 4 == 0 && (sBb % 4 == 0 || (batch == 1 && !foldK && !foldN));
    fl.vecC = sCn == 1 && al(C) && sCm % 4 == 0 && (sCb % 4 == 0 || (batch == 1 && !foldN)) &&
              (foldN ? foldN % 4 == 0 : true);
    fl.vecP = N % 4 == 0 && (need == 0 || al(workspace));
    // n-tiles walked by a grid of ~2 resident workgroups per CU (pipelined across tiles)
    fl.ntn = (N + 127) / 128;
    const int mt = (M + 63) / 64, zb = batch * ksplit;
    const int want = (int)((512 + (int64_t)mt * zb - 1) / ((int64_t)mt * zb));
    const dim3 gx((unsigned)(want < fl.ntn ? want : fl.ntn), (unsigned)mt, (unsigned)zb);
    hipLaunchKernelGGL((gemm_x3_kernel<64, 128>), gx, dim3(kT), 0, st, a, fl);
  } else {
    hipLaunchKernelGGL(gemm_kernel, grid, dim3(kT), 0, st, a);
  }
  if (need > 0) {  // the partial tiles, summed in (image, split) order
    const bool shared = sCb == 0 && batch > 1;
    const int cimgs = shared ? 1 : batch;
    const int zper = shared ? batch * ksplit : ksplit;
    const int64_t mn = (int64_t)M * N;
    hipLaunchKernelGGL(gemm_reduce_kernel, dim3(grid_for(mn, 8192), (unsigned)cimgs), dim3(kT), 0, st, a, zper);
  }
  return (int)hipGetLastError();
}

// workspace: segment partials (3 floats per (segment, image, channel)), then 8-byte aligned the
// composite's own [c][3] double statistics and its 1 / count slot
long long ast_mbt_bn_workspace_floats(int n, int c, long long hw) {
  if (n <= 0 || c <= 0 || hw <= 0) return 0;
  const long long parts = 3LL * c * n * ((hw + BN_SEG - 1) / BN_SEG);
  return (parts + 1) / 2 * 2 + 6LL * c + 2;
}

static int bn_check(int n, int c, long long hw, const float* workspace, long long workspace_floats) {
  if (!workspace) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0 || n > 65535 || c > 65535) return AST_E_SHAPE;
  if (workspace_floats < ast_mbt_bn_workspace_floats(n, c, hw)) return AST_E_SHAPE;  // workspace too small
  return 0;
}

int ast_mbt_bn_stats_f32(const float* x, int n, int c, long long hw, float* workspace, long long workspace_floats,
                         double* stats, void* stream) {
  if (!x || !stats) return AST_E_NULLPTR;
  if (int e = bn_check(n, c, hw, workspace, workspace_floats)) return e;
  hipStream_t st = (hipStream_t)stream;
  const int segs = (int)((hw + BN_SEG - 1) / BN_SEG);
  hipLaunchKernelGGL(bn_part_stats_kernel, dim3(segs, n, c), dim3(kT), 0, st, x, c, (int64_t)hw, workspace);
  hipLaunchKernelGGL(bn_local_stats_kernel, dim3((c + 63) / 64), dim3(64), 0, st, workspace, segs * n, c, stats);
  return (int)hipGetLastError();
}

int ast_mbt_bn_merge_f32(const double* stats, int parts, int c, float eps, float momentum, float* mean, float* invstd,
                         float* run_mean, float* run_var, float* inv_count, void* stream) {
  if (!stats || !mean || !invstd || ((run_mean == nullptr) != (run_var == nullptr))) return AST_E_NULLPTR;
  if (parts <= 0 || c <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(bn_merge_stats_kernel, dim3((c + 63) / 64), dim3(64), 0, (hipStream_t)stream, stats, parts, c,
                     eps, momentum, mean, invstd, run_mean, run_var, inv_count);
  return (int)hipGetLastError();
}

int ast_mbt_bn_act_apply_f32(const float* x, int n, int c, long long hw, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int act, float* y, void* stream) {
  if (!x || !mean || !invstd || !y) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0 || (int64_t)n * c > 0x7fffffffLL) return AST_E_SHAPE;
  if (act != 0 && act != 1) return AST_E_UNSUPPORTED;
  const dim3 grid = plane_grid(hw, (int64_t)n * c);
  if (act)
    hipLaunchKernelGGL(bn_apply_kernel<1>, grid, dim3(kT), 0, (hipStream_t)stream, x, c, (int64_t)hw, n * c, mean,
                       invstd, gamma, beta, y);
  else
    hipLaunchKernelGGL(bn_apply_kernel<0>, grid, dim3(kT), 0, (hipStream_t)stream, x, c, (int64_t)hw, n * c, mean,
                       invstd, gamma, beta, y);
  return (int)hipGetLastError();
}

int ast_mbt_bn_apply_f32(const float* x, int n, int c, long long hw, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, float* y, void* stream) {
  return ast_mbt_bn_act_apply_f32(x, n, c, hw, mean, invstd, gamma, beta, 0, y, stream);
}

int ast_mbt_bn_act_fwd_f32(const float* x, int n, int c, long long hw, const float* gamma, const float* beta,
                           float eps, float momentum, float* mean, float* invstd, float* run_mean, float* run_var,
                           int act, float* y, float* workspace, long long workspace_floats, void* stream) {
  if (!x || !mean || !invstd || !y) return AST_E_NULLPTR;
  if (int e = bn_check(n, c, hw, workspace, workspace_floats)) return e;
  const long long off = ast_mbt_bn_workspace_floats(n, c, hw) - 6LL * c - 2;
  double* stats = (double*)(workspace + off);
  int e = ast_mbt_bn_stats_f32(x, n, c, hw, workspace, workspace_floats, stats, stream);
  if (!e) e = ast_mbt_bn_merge_f32(stats, 1, c, eps, momentum, mean, invstd, run_mean, run_var, nullptr, stream);
  if (!e) e = ast_mbt_bn_act_apply_f32(x, n, c, hw, mean, invstd, gamma, beta, act, y, stream);
  return e;
}

int ast_mbt_bn_fwd_f32(const float* x, int n, int c, long long hw, const float* gamma, const float* beta, float eps,
                       float momentum, float* mean, float* invstd, float* run_mean, float* run_var, float* y,
                       float* workspace, long long workspace_floats, void* stream) {
  return ast_mbt_bn_act_fwd_f32(x, n, c, hw, gamma, beta, eps, momentum, mean, invstd, run_mean, run_var, 0, y,
                                workspace, workspace_floats, stream);
}

static void bn_part_bwd(int act, int segs, int n, int c, const float* x, const float* dy, long long hw,
                        const float* mean, const float* invstd, const float* gamma, const float* beta, float* part,
                        hipStream_t st) {
  if (act)
    hipLaunchKernelGGL(bn_part_bwd_kernel<1>, dim3(segs, n, c), dim3(kT), 0, st, x, dy, c, (int64_t)hw, mean, invstd,
                       gamma, beta, part);
  else
    hipLaunchKernelGGL(bn_part_bwd_kernel<0>, dim3(segs, n, c), dim3(kT), 0, st, x, dy, c, (int64_t)hw, mean, invstd,
                       gamma, beta, part);
}

static void bn_bwd_apply(int act, int n, int c, const float* x, const float* dy, long long hw,
                         const float* inv_count, const float* mean, const float* invstd, const float* gamma,
                         const float* beta, const float* sdy, const float* sdyx, float* dx, hipStream_t st) {
  const dim3 grid = plane_grid(hw, (int64_t)n * c);
  if (act)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, grid, dim3(kT), 0, st, x, dy, c, (int64_t)hw, n * c, inv_count, mean,
                       invstd, gamma, beta, sdy, sdyx, dx);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<0>, grid, dim3(kT), 0, st, x, dy, c, (int64_t)hw, n * c, inv_count, mean,
                       invstd, gamma, beta, sdy, sdyx, dx);
}

int ast_mbt_bn_act_bwd_sums_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                                const float* invstd, const float* gamma, const float* beta, int act,
                                float* workspace, long long workspace_floats, float* sums, void* stream) {
  if (!x || !dy || !mean || !invstd || !sums) return AST_E_NULLPTR;
  if (act != 0 && act != 1) return AST_E_UNSUPPORTED;
  if (int e = bn_check(n, c, hw, workspace, workspace_floats)) return e;
  hipStream_t st = (hipStream_t)stream;
  const int segs = (int)((hw + BN_SEG - 1) / BN_SEG);
  bn_part_bwd(act, segs, n, c, x, dy, hw, mean, invstd, gamma, beta, workspace, st);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((c + 63) / 64), dim3(64), 0, st, workspace, segs * n, c, sums,
                     sums + c, nullptr, 0.f);
  return (int)hipGetLastError();
}

int ast_mbt_bn_bwd_sums_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                            const float* invstd, float* workspace, long long workspace_floats, float* sums,
                            void* stream) {
  return ast_mbt_bn_act_bwd_sums_f32(x, dy, n, c, hw, mean, invstd, nullptr, nullptr, 0, workspace,
                                     workspace_floats, sums, stream);
}

int ast_mbt_bn_act_bwd_apply_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                                 const float* invstd, const float* gamma, const float* beta, int act,
                                 const float* sums, const float* inv_count, float* dx, void* stream) {
  if (!x || !dy || !mean || !invstd || !sums || !inv_count || !dx) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hw <= 0 || (int64_t)n * c > 0x7fffffffLL) return AST_E_SHAPE;
  if (act != 0 && act != 1) return AST_E_UNSUPPORTED;
  bn_bwd_apply(act, n, c, x, dy, hw, inv_count, mean, invstd, gamma, beta, sums, sums + c, dx, (hipStream_t)stream);
  return (int)hipGetLastError();
}

int ast_mbt_bn_bwd_apply_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                             const float* invstd, const float* gamma, const float* sums, const float* inv_count,
                             float* dx, void* stream) {
  return ast_mbt_bn_act_bwd_apply_f32(x, dy, n, c, hw, mean, invstd, gamma, nullptr, 0, sums, inv_count, dx, stream);
}

int ast_mbt_bn_act_bwd_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                           const float* invstd, const float* gamma, const float* beta, int act, float* dgamma,
                           float* dbeta, float* dx, float* workspace, long long workspace_floats, void* stream) {
  if (!dgamma || !dbeta) return AST_E_NULLPTR;
  if (act != 0 && act != 1) return AST_E_UNSUPPORTED;
  if (int e = bn_check(n, c, hw, workspace, workspace_floats)) return e;
  if (!x || !dy || !mean || !invstd || !dx) return AST_E_NULLPTR;
  const long long off = ast_mbt_bn_workspace_floats(n, c, hw) - 6LL * c - 2;
  float* inv_count = workspace + off;
  hipStream_t st = (hipStream_t)stream;
  const int segs = (int)((hw + BN_SEG - 1) / BN_SEG);
  bn_part_bwd(act, segs, n, c, x, dy, hw, mean, invstd, gamma, beta, workspace, st);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((c + 63) / 64), dim3(64), 0, st, workspace, segs * n, c, dbeta,
                     dgamma, inv_count, (float)(1.0 / ((double)n * (double)hw)));
  bn_bwd_apply(act, n, c, x, dy, hw, inv_count, mean, invstd, gamma, beta, dbeta, dgamma, dx, st);
  return (int)hipGetLastError();
}

int ast_mbt_bn_bwd_f32(const float* x, const float* dy, int n, int c, long long hw, const float* mean,
                       const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dx,
                       float* workspace, long long workspace_floats, void* stream) {
  return ast_mbt_bn_act_bwd_f32(x, dy, n, c, hw, mean, invstd, gamma, nullptr, 0, dgamma, dbeta, dx, workspace,
                                workspace_floats, stream);
}

int ast_mbt_eltwise_f32(int op, const float* a, const float* b, float* y, long long n, int h, int w, void* stream) {
  // op 0: hardswish(a); 1: hardswish backward (x = a, g = b); 2: a + b;
  //    3: nearest upsample x2 of a [n planes][h][w]; 4: its backward (a = grad [n][2h][2w])
  if (!a || !y || ((op == 1 || op == 2) && !b)) return AST_E_NULLPTR;
  if (n <= 0) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  switch (op) {
    case 0:
    case 1:
    case 2:
      if (n >= (1LL << 40)) return AST_E_SHAPE;
      if (op == 0) launch_eltwise<0>(a, nullptr, y, (int64_t)n, st);
      else if (op == 1) launch_eltwise<1>(a, b, y, (int64_t)n, st);
      else launch_eltwise<2>(a, b, y, (int64_t)n, st);
      break;
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

int ast_mbt_plane_act_f32(int op, const float* x, const float* y, const float* gate, const float* gadd,
                          const float* a, float* out, long long planes, long long hw, void* stream) {
  // op 0: out[p] = mean(x[p]); 1: out[p] = sum(x[p] * y[p]); 2: out = x * gate[p] (+ gadd[p]);
  //    3: out[p] = mean(hardswish(x[p])); 4: out[p] = sum(x[p] * hardswish(y[p]));
  //    5: out = hardswish(x) * gate[p]; 6: out = hardswish'(a) * (x * gate[p] + gadd[p])
  if (!x || !out || ((op == 1 || op == 4) && !y) || ((op == 2 || op == 5 || op == 6) && !gate) || (op == 6 && !a))
    return AST_E_NULLPTR;
  if (planes <= 0 || hw <= 0 || planes > 0x7fffffffLL) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const dim3 pg((unsigned)planes);
  switch (op) {
    case 0:
    case 1:
      hipLaunchKernelGGL(plane_dot_kernel<0>, pg, dim3(kT), 0, st, x, op == 1 ? y : nullptr, (int64_t)hw,
                         op == 0 ? 1.0f / (float)hw : 1.0f, out);
      break;
    case 3:
    case 4:
      hipLaunchKernelGGL(plane_dot_kernel<1>, pg, dim3(kT), 0, st, x, op == 4 ? y : nullptr, (int64_t)hw,
                         op == 3 ? 1.0f / (float)hw : 1.0f, out);
      break;
    case 2:
      hipLaunchKernelGGL(plane_scale_kernel<0>, plane_grid(hw, planes), dim3(kT), 0, st, x, gate, gadd, nullptr,
                         (int64_t)hw, (int64_t)planes, out);
      break;
    case 5:
      hipLaunchKernelGGL(plane_scale_kernel<1>, plane_grid(hw, planes), dim3(kT), 0, st, x, gate, nullptr, nullptr,
                         (int64_t)hw, (int64_t)planes, out);
      break;
    case 6:
      hipLaunchKernelGGL(plane_scale_kernel<2>, plane_grid(hw, planes), dim3(kT), 0, st, x, gate, gadd, a,
                         (int64_t)hw, (int64_t)planes, out);
      break;
    default:
      return AST_E_UNSUPPORTED;
  }
  return (int)hipGetLastError();
}

int ast_mbt_plane_f32(int op, const float* x, const float* y, const float* gate, const float* gadd, float* out,
                      long long planes, long long hw, void* stream) {
  if (op < 0 || op > 2) return AST_E_UNSUPPORTED;
  return ast_mbt_plane_act_f32(op, x, y, gate, gadd, nullptr, out, planes, hw, stream);
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
                          float* db2, float* dpool, float* workspace, long long workspace_floats, void* stream) {
  if (!dgate || !z || !hid || !pool || !w1 || !w2 || !dw1 || !db1 || !dw2 || !db2 || !dpool || !workspace)
    return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || red <= 0 || hw <= 0 || c + red > 16384) return AST_E_SHAPE;
  if (workspace_floats < (long long)n * (c + red)) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(se_fc_bwd_kernel, dim3(n), dim3(kT), sizeof(float) * (c + red), st, dgate, z, hid, w1, w2, n, c,
                     red, 1.0f / (float)hw, workspace, dpool);
  const int64_t total = 2LL * c * red + c + red;
  hipLaunchKernelGGL(se_fc_param_grad_kernel, dim3(grid_for(total, 4096)), dim3(kT), 0, st, workspace, hid, pool, n,
                     c, red, dw1, db1, dw2, db2);
  return (int)hipGetLastError();
}

}  // extern "C"
