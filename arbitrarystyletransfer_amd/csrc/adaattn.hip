// AdaAttN (models.py:70-115) for gfx950: attention-weighted style statistics.
//
//   q = W_q(IN(c)), k = W_k(IN(s)), v = W_v(s)                       (1x1 convs, no bias)
//   A = softmax_keys(q^T k)                                           [Nq x Nk] per image
//   mean = A v,  std = sqrt(relu(A v^2 - mean^2)),  out = std * IN(c) + mean
// with IN = InstanceNorm2d (biased variance, eps 1e-5, no affine).
//
// Three launches per call:
//   in_stats_kernel    per-(n,c) mean / rstd of content and style (two-pass, one WG per plane)
//   project_kernel     Q, K, V as [n][Cp][Npad] (Cp = C rounded to 32, Npad = N rounded to 32;
//                      padding is written as zeros) -- an MFMA-fp32 channel GEMM with the
//                      instance norm applied while the input is read
//   attend_f32_kernel  flash-style fused Q K^T -> online softmax -> P [V, V^2] -> epilogue. The
//                      Nq x Nk score matrix never leaves registers. 4 waves x 32 queries per
//                      workgroup; K/V blocks of 32 keys are double-buffered in LDS.
//
// MFMA orientation (v_mfma_f32_32x32x2_f32, exact fp32): the scores are computed transposed,
// S^T = K Q^T, so the accumulator has the QUERY on the lane and 16 keys in registers. That tile is
// directly the B operand of O^T = [V, V^2]^T P^T (summing over keys = S^T's row index), so P
// never moves between lanes, and O^T again has the query on the lane: the epilogue's stores are
// 128-byte rows of the NCHW output. The softmax row max / sum need one lane^32 exchange.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include "../../include/ast_hip.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kStatThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float ld(const float* p) { return *p; }
__device__ __forceinline__ float ld(const __bf16* p) { return (float)*p; }

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kStatThreads / 64; ++i) t += sh[i];
  return t;
}

// InstanceNorm2d statistics: mean and 1/sqrt(biased var + eps) per (n, c) plane; blockIdx.y picks
// the tensor (0 = content, 1 = style).
template <typename T>
__global__ __launch_bounds__(kStatThreads) void in_stats_kernel(const T* __restrict__ c, const T* __restrict__ s,
                                                                float* __restrict__ stats, int planes, int64_t hwc,
                                                                int64_t hws, float eps) {
  __shared__ float sh[kStatThreads / 64];
  const int p = blockIdx.x;
  const bool style = blockIdx.y == 1;
  const int64_t hw = style ? hws : hwc;
  const T* __restrict__ x = (style ? s : c) + (int64_t)p * hw;
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < hw; i += kStatThreads) acc += ld(x + i);
  const float mean = block_sum(acc, sh) / (float)hw;
  acc = 0.f;
  for (int64_t i = threadIdx.x; i < hw; i += kStatThreads) {
    const float d = ld(x + i) - mean;
    acc += d * d;
  }
  const float var = block_sum(acc, sh) / (float)hw;
  if (threadIdx.x == 0) {
    float* o = stats + (style ? 2 : 0) * (int64_t)planes;
    o[p] = mean;
    o[planes + p] = 1.0f / sqrtf(var + eps);
  }
}

// ------------------------------------------------------------------------------------------------
// Projections: Y[b][o][p] = sum_c W[o][c] * xn[b][c][p], xn = (x - mean) * rstd (Q, K) or x (V).
// Workgroup = 4 waves x 32 pixels; each wave holds all Cp output channels (Cp/32 accumulators).
// W is staged transposed in LDS as Wt[c][o] (row pitch Cp + 32 floats: the two half-waves read
// rows c and c+1, which then fall in disjoint bank halves).
// ------------------------------------------------------------------------------------------------
struct ProjArgs {
  const void* c;
  const void* s;
  const float* wq;
  const float* wk;
  const float* wv;
  const float* stats;  // [4][n*C]: content mean, content rstd, style mean, style rstd
  float* q;            // [n][Cp][Nqp]
  float* k;            // [n][Cp][Nkp]
  float* v;            // [n][Cp][Nkp]
  int n, C, Cp, nq, nk, nqp, nkp;
};

template <typename T, int CT>  // CT = Cp / 32 output-channel tiles
__global__ __launch_bounds__(256) void project_kernel(ProjArgs a) {
  extern __shared__ float wt[];  // [C_even][Cp + 32]
  const int which = blockIdx.z;  // 0 = q, 1 = k, 2 = v
  const int b = blockIdx.y;
  const int N = which == 0 ? a.nq : a.nk;
  const int Np = which == 0 ? a.nqp : a.nkp;
  const int p0 = blockIdx.x * 128;
  if (p0 >= Np) return;  // whole workgroup: no barrier is skipped by part of it
  const int C = a.C, Cp = a.Cp, ce = (C + 1) & ~1, pitch = Cp + 32;
  const float* __restrict__ w = which == 0 ? a.wq : (which == 1 ? a.wk : a.wv);
  for (int i = threadIdx.x; i < ce * Cp; i += 256) {
    const int c = i / Cp, o = i - c * Cp;
    wt[c * pitch + o] = (c < C && o < C) ? w[(int64_t)o * C + c] : 0.f;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int px = p0 + wv * 32 + r;
  const T* __restrict__ x = (const T*)(which == 0 ? a.c : a.s) + (int64_t)b * C * N;
  const float* mean = which == 0 ? a.stats : a.stats + 2 * (int64_t)a.n * C;
  const float* rstd = mean + (int64_t)a.n * C;
  mean += (int64_t)b * C;
  rstd += (int64_t)b * C;
  const bool norm = which != 2, pin = px < N;

  f32x16 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) acc[t] = (f32x16){0.f};

  for (int m = 0; m < ce / 2; ++m) {
    const int c = 2 * m + h;
    float xv = 0.f;
    if (pin && c < C) {
      xv = ld(x + (int64_t)c * N + px);
      if (norm) xv = (xv - mean[c]) * rstd[c];
    }
    const float* wr = wt + c * pitch + r;
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[t * 32], xv, acc[t], 0, 0, 0);
  }
  float* __restrict__ y = (which == 0 ? a.q : (which == 1 ? a.k : a.v)) + (int64_t)b * Cp * Np;
  const int pw = p0 + wv * 32 + r;
  if (pw < Np) {
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        y[(int64_t)o * Np + pw] = acc[t][i];
      }
  }
}

// ------------------------------------------------------------------------------------------------
// Fused attention, fp32.
// ------------------------------------------------------------------------------------------------
struct AttnArgs {
  const float* q;  // [n][Cp][Nqp]
  const float* k;  // [n][Cp][Nkp]
  const float* v;  // [n][Cp][Nkp]
  const void* c;   // content [n][C][Nq] (for IN(c) in the epilogue)
  const float* stats;
  void* out;  // [n][C][Nq]
  int n, C, Cp, nq, nk, nqp, nkp, qtiles;
  int ksplit, kchunk;  // split-K over the keys, as AttnB16Args
  float* part;
};

constexpr int BK = 32;        // keys per block
constexpr int KP = BK;        // K block row pitch (floats): rows c, c+1 -> disjoint bank halves
constexpr int VP = BK + 4;    // V block row pitch: 16 lanes x f32x4 over 16 distinct bank quads

__device__ __forceinline__ void map_tile(int id, int total, int tiles_per_image, int& b, int& tile) {
  // XCD-aware order: the hardware places workgroup id on XCD (id % 8). Give each XCD a contiguous
  // range of (image, tile) so the workgroups of one image share K/V through one L2.
  int lin = id;
  if ((total & 7) == 0) lin = (id & 7) * (total >> 3) + (id >> 3);
  b = lin / tiles_per_image;
  tile = lin - b * tiles_per_image;
}

// K/V staging registers as named members. Native ext_vector f32x4, not HIP's float4 struct: its
// copies lower to memcpy through a private-memory temporary (scratch) that SROA does not remove.
template <int CT>
struct KVRegs {
  f32x4 k0, k1, k2, k3, v0, v1, v2, v3;
  __device__ __forceinline__ void load(const float* __restrict__ kb, const float* __restrict__ vb, int tid, int nkp,
                                       int kbase) {
    const int off = (tid >> 3) * nkp + (tid & 7) * 4 + kbase, step = 32 * nkp;  // +256 threads = +32 rows
    k0 = *reinterpret_cast<const f32x4*>(kb + off);
    v0 = *reinterpret_cast<const f32x4*>(vb + off);
    if constexpr (CT > 1) {
      k1 = *reinterpret_cast<const f32x4*>(kb + off + step);
      v1 = *reinterpret_cast<const f32x4*>(vb + off + step);
    }
    if constexpr (CT > 2) {
      k2 = *reinterpret_cast<const f32x4*>(kb + off + 2 * step);
      v2 = *reinterpret_cast<const f32x4*>(vb + off + 2 * step);
    }
    if constexpr (CT > 3) {
      k3 = *reinterpret_cast<const f32x4*>(kb + off + 3 * step);
      v3 = *reinterpret_cast<const f32x4*>(vb + off + 3 * step);
    }
  }
  template <int KPITCH, int VPITCH>
  __device__ __forceinline__ void store(float* ks, float* vs, int tid) const {
    const int row = tid >> 3, col = (tid & 7) * 4;
    float* kp = ks + row * KPITCH + col;
    float* vp = vs + row * VPITCH + col;
    *reinterpret_cast<f32x4*>(kp) = k0;
    *reinterpret_cast<f32x4*>(vp) = v0;
    if constexpr (CT > 1) {
      *reinterpret_cast<f32x4*>(kp + 32 * KPITCH) = k1;
      *reinterpret_cast<f32x4*>(vp + 32 * VPITCH) = v1;
    }
    if constexpr (CT > 2) {
      *reinterpret_cast<f32x4*>(kp + 64 * KPITCH) = k2;
      *reinterpret_cast<f32x4*>(vp + 64 * VPITCH) = v2;
    }
    if constexpr (CT > 3) {
      *reinterpret_cast<f32x4*>(kp + 96 * KPITCH) = k3;
      *reinterpret_cast<f32x4*>(vp + 96 * VPITCH) = v3;
    }
  }
};

// Lazy rescaling: the running row max is only raised when a block's max exceeds it by more than
// 2^kRescaleLog2 (log2 units), so exp2 arguments stay <= kRescaleLog2 (no fp32 overflow) and the
// accumulators are rescaled a handful of times per row instead of whenever the max moves. The
// final division by the row sum (accumulated against the same stale max) makes this exact.
constexpr float kRescaleLog2 = 8.0f;

template <typename TO, int CT>
__global__ __launch_bounds__(256, 1) void attend_f32_kernel(AttnArgs a) {
  constexpr int CP = CT * 32;
  // Q tile [CP][128 queries], column XOR-swizzled by (c & 1) << 5 so a wave's two half-waves
  // (rows c, c+1) read disjoint bank halves; K/V blocks double-buffered.
  __shared__ float qs[CP * 128];
  __shared__ float ks[2][CP * KP];
  __shared__ float vs[2][CP * VP];
  int b, tile;
  const int ntq = a.n * a.qtiles, sp = (int)blockIdx.x / ntq;  // split index (0 without a split)
  map_tile((int)blockIdx.x - sp * ntq, ntq, a.qtiles, b, tile);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const int q0 = tile * 128;
  const int qi = q0 + wv * 32 + r;  // this lane's query (column of every accumulator tile)

  {
    const float* __restrict__ qb = a.q + (int64_t)b * CP * a.nqp + q0;  // nqp is a multiple of 128
#pragma unroll
    for (int i = 0; i < CP / 8; ++i) {
      const int e = tid + i * 256, row = e >> 5, col = (e & 31) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(qb + (int64_t)row * a.nqp + col);
      *reinterpret_cast<f32x4*>(&qs[row * 128 + (col ^ ((row & 1) << 5))]) = v;
    }
  }

  const float* __restrict__ kb = a.k + (int64_t)b * CP * a.nkp;
  const float* __restrict__ vb = a.v + (int64_t)b * CP * a.nkp;
  // K/V block staging: CT f32x4 of K and CT of V per thread and block (row = channel, 8 f32x4
  // per 32-key row), prefetched into registers one block ahead.
  KVRegs<CT> kv;
  f32x16 om[CT], osq[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    om[t] = (f32x16){0.f};
    osq[t] = (f32x16){0.f};
  }
  float mrow = -INFINITY, lsum = 0.f;  // mrow in log2 units

  const int j0 = sp * a.kchunk, nblk = min(a.nkp / BK, j0 + a.kchunk);
  kv.load(kb, vb, tid, a.nkp, j0 * BK);
  kv.template store<KP, VP>(ks[0], vs[0], tid);
  const float* qq = &qs[h * 128 + ((wv * 32 + r) ^ (h << 5))];
  for (int j = j0; j < nblk; ++j) {
    const int buf = (j - j0) & 1;
    if (j + 1 < nblk) kv.load(kb, vb, tid, a.nkp, (j + 1) * BK);
    __syncthreads();

    // S^T[key][query] for 32 keys (rows) x this wave's 32 queries (lanes); two independent
    // accumulation chains (alternate channel pairs).
    f32x16 s0 = (f32x16){0.f}, s1 = (f32x16){0.f};
    const float* kk = &ks[buf][h * KP + r];
#pragma unroll
    for (int m = 0; m < CP / 2; m += 2) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x2f32(kk[2 * m * KP], qq[2 * m * 128], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x2f32(kk[(2 * m + 2) * KP], qq[(2 * m + 2) * 128], s1, 0, 0, 0);
    }
    f32x16 s = (s0 + s1) * kLog2e;

    // Online softmax over keys (registers + the lane^32 partner).
    const int kbase = j * BK;
    {
      const int lim = a.nk - kbase - 4 * h;  // keys >= nk are masked (only in the last block)
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = ((i & 3) + 8 * (i >> 2) < lim) ? s[i] : -INFINITY;
    }
    float mb = s[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mb = fmaxf(mb, s[i]);
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    if (__builtin_expect(__ballot(mb > mrow + kRescaleLog2) != 0, 0)) {
      const float mnew = fmaxf(mrow, mb);
      const float alpha = __builtin_amdgcn_exp2f(mrow - mnew);  // 0 on the first block
      lsum *= alpha;
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        om[t] *= alpha;
        osq[t] *= alpha;
        __builtin_amdgcn_sched_barrier(0);  // one tile at a time: bounded register pressure
      }
      mrow = mnew;
    }
    float p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      p[i] = __builtin_amdgcn_exp2f(s[i] - mrow);
      lsum += p[i];
    }

    // O^T[ch][query] += V^T P^T and (V^2)^T P^T. MFMA (g, e) pairs k = h with key 4h + 8g + e,
    // which is exactly register 4g + e of this lane's P; V is read as f32x4 over e. The channel
    // tiles are innermost: 2*CT independent accumulation chains.
    const float* vv = &vs[buf][r * VP + 4 * h];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v4[CT];
#pragma unroll
      for (int t = 0; t < CT; ++t) v4[t] = *reinterpret_cast<const f32x4*>(vv + t * 32 * VP + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int t = 0; t < CT; ++t) {
          const float ve = e == 0 ? v4[t].x : e == 1 ? v4[t].y : e == 2 ? v4[t].z : v4[t].w;
          om[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(ve, p[4 * g + e], om[t], 0, 0, 0);
          osq[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(ve * ve, p[4 * g + e], osq[t], 0, 0, 0);
        }
      }
    }
    if (j + 1 < nblk) kv.template store<KP, VP>(ks[buf ^ 1], vs[buf ^ 1], tid);
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  if (a.part) {  // this split's partials (layout of AttnB16Args::part)
    const int64_t mq = (int64_t)a.ksplit * a.n * a.nqp;
    float* pm = a.part + ((int64_t)sp * a.n + b) * a.nqp;
    float* po = a.part + 2 * mq + ((int64_t)sp * a.n + b) * 2 * CP * a.nqp;
    if (h == 0) {
      pm[qi] = mrow;
      pm[mq + qi] = ltot;
    }
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ch = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        po[(int64_t)ch * a.nqp + qi] = om[t][i];
        po[(int64_t)(CP + ch) * a.nqp + qi] = osq[t][i];
      }
    return;
  }
  // Epilogue: out[b][ch][qi] = std * (c - mean_c) * rstd_c + mean.
  if (qi >= a.nq) return;
  const float inv = 1.0f / ltot;
  const float* cmean = a.stats + (int64_t)b * a.C;
  const float* crstd = a.stats + (int64_t)a.n * a.C + (int64_t)b * a.C;
  const TO* __restrict__ cb = (const TO*)a.c + (int64_t)b * a.C * a.nq;
  TO* __restrict__ ob = (TO*)a.out + (int64_t)b * a.C * a.nq;
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ch = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (ch < a.C) {
        const float mean = om[t][i] * inv;
        float var = fmaf(-mean, mean, osq[t][i] * inv);
        var = var < 0.f ? 0.f : var;  // ReLU (NaN passes, as torch.relu)
        const int64_t o = (int64_t)ch * a.nq + qi;
        const float xn = (ld(cb + o) - cmean[ch]) * crstd[ch];
        const float y = fmaf(sqrtf(var), xn, mean);
        ob[o] = (TO)y;
      }
    }
}


// ================================================================================================
// bf16 path (bf16 storage, fp32 accumulation): the MobileNet-variant AST runs in bf16.
//   Q, K  [n][Np][Cp]  pixel-major (an MFMA-bf16 A/B fragment is 8 consecutive channels)
//   V, V2 [n][Cp][Nkp] channel-major; V is centred by the style's channel mean before the 1x1 conv
//         (V' = W_v (s - mean_s); the epilogue adds W_v mean_s back, which the softmax weights
//         summing to 1 makes exact) and V2 = bf16(V'^2) is squared from the fp32 projection, so
//         E[v^2] - mean^2 is formed from small, accurately rounded terms.
// ================================================================================================
struct ProjB16Args {
  const bf16* c;
  const bf16* s;
  const float* wq;
  const float* wk;
  const float* wv;
  const float* stats;  // [4][n*C]
  bf16* q;             // [n][Nqp][Cp]
  bf16* k;             // [n][Nkp][Cp]
  bf16* v;             // [n][Cp][Nkp]
  bf16* v2;            // [n][Cp][Nkp]
  int n, C, Cp, nq, nk, nqp, nkp;
};

// bf16 projections on v_mfma_f32_32x32x16_bf16. Workgroup = 4 waves x 32 pixels. The input tile
// [C][128 px] is read with 16-byte loads, normalised in fp32 ((x - mean) * rstd for Q/K, x - mean
// for V) and written to LDS pixel-major as bf16 (xs[px][CK + 8]); W is staged as bf16
// ws[o][CK + 8] (CK = C rounded to 16, zero padded). A fragment = 8 consecutive channels of one
// row of either image (16-byte, conflict-free reads). Q/K: D[pixel][o] (lane = o: 64-byte rows
// of the pixel-major output); V: D[o][pixel] (lane = pixel) plus V^2 from the fp32 accumulator.
template <int CT>
__global__ __launch_bounds__(256) void project_bf16_kernel(ProjB16Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  const int which = blockIdx.z;  // 0 = q, 1 = k, 2 = v (+ v2)
  const int b = blockIdx.y;
  const int N = which == 0 ? a.nq : a.nk;
  const int Np = which == 0 ? a.nqp : a.nkp;
  const int p0 = blockIdx.x * 128;
  if (p0 >= Np) return;
  constexpr int CP = CT * 32;
  const int C = a.C, CK = (C + 15) & ~15, RP = CK + 8;
  bf16* xs = reinterpret_cast<bf16*>(psm);  // [128][RP]
  bf16* ws = xs + 128 * RP;                 // [CP][RP]
  const float* __restrict__ w = which == 0 ? a.wq : (which == 1 ? a.wk : a.wv);
  const int tid = threadIdx.x;
  for (int i = tid; i < CP * CK; i += 256) {
    const int o = i / CK, c = i - o * CK;
    ws[o * RP + c] = (bf16)((o < C && c < C) ? w[(int64_t)o * C + c] : 0.f);
  }
  const bf16* __restrict__ x = (which == 0 ? a.c : a.s) + (int64_t)b * C * N;
  const float* mean = (which == 0 ? a.stats : a.stats + 2 * (int64_t)a.n * C) + (int64_t)b * C;
  const float* rstd = mean + (int64_t)a.n * C;
  const bool scale = which != 2;
  // Q carries the softmax's log2(e) (scores come out in log2 units: exp2 without a multiply)
  const float qs = which == 0 ? kLog2e : 1.f;
  // 16 pieces of 8 pixels per channel row; vector loads when the row is 16-byte aligned
  const bool vec = (N % 8) == 0;
  for (int i = tid; i < CK * 16; i += 256) {
    const int c = i >> 4, q = (i & 15) * 8, px = p0 + q;
    float v[8];
    if (c < C) {
      const float m = mean[c], rs = (scale ? rstd[c] : 1.f) * qs;
      const bf16* xr = x + (int64_t)c * N;
      if (vec && px + 8 <= N) {
        const bf16x8 t = *reinterpret_cast<const bf16x8*>(xr + px);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ((float)t[j] - m) * rs;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = px + j < N ? ((float)xr[px + j] - m) * rs : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) xs[(q + j) * RP + c] = (bf16)v[j];
  }
  __syncthreads();

  const int lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  f32x16 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) acc[t] = (f32x16){0.f};
  const bf16* xrow = xs + (wv * 32 + r) * RP + 8 * h;
  for (int k0 = 0; k0 < CK; k0 += 16) {
    const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xrow + k0);
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const bf16x8 wf = *reinterpret_cast<const bf16x8*>(ws + (t * 32 + r) * RP + 8 * h + k0);
      acc[t] = which == 2 ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc[t], 0, 0, 0)
                          : __builtin_amdgcn_mfma_f32_32x32x16_bf16(xf, wf, acc[t], 0, 0, 0);
    }
  }
  const int pw0 = p0 + wv * 32;
  if (which == 2) {
    bf16* __restrict__ y = a.v + (int64_t)b * CP * Np;
    bf16* __restrict__ y2 = a.v2 + (int64_t)b * CP * Np;
    const int pw = pw0 + r;
    if (pw < Np) {
#pragma unroll
      for (int t = 0; t < CT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int o = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          const float vv = acc[t][i];
          y[(int64_t)o * Np + pw] = (bf16)vv;
          y2[(int64_t)o * Np + pw] = (bf16)(vv * vv);
        }
    }
  } else {
    bf16* __restrict__ y = (which == 0 ? a.q : a.k) + (int64_t)b * Np * CP;
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int p = pw0 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (p < Np) y[(int64_t)p * CP + t * 32 + r] = (bf16)acc[t][i];
      }
  }
}

// mean of V over the style pixels, per (n, o): W_v mean_s (added back in the epilogue).
__global__ __launch_bounds__(128) void vmean_kernel(const float* __restrict__ wv, const float* __restrict__ stats,
                                                    float* __restrict__ vmean, int n, int C) {
  const int b = blockIdx.x;
  const float* ms = stats + 2 * (int64_t)n * C + (int64_t)b * C;
  for (int o = threadIdx.x; o < C; o += 128) {
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(wv[(int64_t)o * C + c], ms[c], acc);
    vmean[(int64_t)b * C + o] = acc;
  }
}

struct AttnB16Args {
  const bf16* q;   // [n][Nqp][Cp]
  const bf16* k;   // [n][Nkp][Cp]
  const bf16* v;   // [n][Cp][Nkp]
  const bf16* v2;  // [n][Cp][Nkp]
  const bf16* c;   // content [n][C][Nq]
  const float* stats;
  const float* vmean;  // [n][C]
  bf16* out;
  int n, C, Cp, nq, nk, nqp, nkp, qtiles;
  // split-K over the keys (flash-decoding; small batches): split s of ksplit takes key blocks
  // [s kchunk, (s + 1) kchunk) and writes its running max, sum and unnormalised [V, V^2] sums to
  // part ([ksplit][n][nqp] m, then l, then [ksplit][n][2 Cp][nqp]); attn_merge_kernel combines them
  int ksplit, kchunk;
  float* part;
};

// 8 waves x 32 queries per workgroup, 32-key blocks, v_mfma_f32_32x32x16_bf16.
//   S^T = K Q^T: A = K from LDS ([key][Cp + 8] bf16 rows: 16-byte reads, conflict-free), B = this
//   lane's Q fragment (registers, loaded once).
//   P = bf16(exp2(S - m)) straight from the accumulator: registers 8s..8s+7 are the B fragment of
//   k-step s with key order 16s + 8(j>>2) + 4h + (j&3). V and V^2 rows ([ch][40] bf16, 80-byte
//   pitch) store each 16-key group in exactly that order (keys 0-3, 8-11, 4-7, 12-15), so the A
//   operand (V^T) is one conflict-free 16-byte read (ds_read_b128: 256 B/clk, vs 128 for the
//   ds_read2_b64 pair a natural key order needs).
constexpr int KPB = 8;   // K row padding (bf16)
constexpr int VPB = 40;  // V row pitch (bf16): 20 dwords, distinct bank quads per b128 lane group

template <int CT, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attend_bf16_kernel(AttnB16Args a) {
  constexpr int CP = CT * 32, KROW = CP + KPB;
  __shared__ __attribute__((aligned(16))) bf16 ks[2][BK * KROW];
  __shared__ __attribute__((aligned(16))) bf16 vs[2][CP * VPB];
  __shared__ __attribute__((aligned(16))) bf16 v2s[2][CP * VPB];
  int b, tile;
  const int ntq = a.n * a.qtiles, sp = (int)blockIdx.x / ntq;  // split index (0 without a split)
  map_tile((int)blockIdx.x - sp * ntq, ntq, a.qtiles, b, tile);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const int qi = tile * (NW * 32) + wv * 32 + r;

  bf16x8 qf[CP / 16];
  {
    const bf16* qp = a.q + ((int64_t)b * a.nqp + qi) * CP + 8 * h;
#pragma unroll
    for (int s = 0; s < CP / 16; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s);
  }
  // Retire the Q loads here: otherwise the compiler's wait-count placement waits for them inside
  // the loop, where the same waits then also drain every block's K/V prefetch.
  __builtin_amdgcn_s_waitcnt(0);

  // staging: K block = 32 rows x CP bf16 (CP/8 16-byte pieces per row); V, V2 blocks = CP rows x
  // 32 keys (4 pieces per row). One piece of each per thread (CP = 128), fewer threads otherwise.
  const bf16* __restrict__ kb = a.k + (int64_t)b * a.nkp * CP;
  const bf16* __restrict__ vb = a.v + (int64_t)b * CP * a.nkp;
  const bf16* __restrict__ v2b = a.v2 + (int64_t)b * CP * a.nkp;
  constexpr int NT = NW * 64, NPIECE = CP * 4;  // 16-byte pieces per block of each of K, V, V2
  constexpr int PPT = (NPIECE + NT - 1) / NT;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x4 kr[PPT], vr[PPT], v2r[PPT];
  auto gload = [&](int kbase) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      if (NPIECE % NT == 0 || e < NPIECE) {
        const int krow = e / (CP / 8), kcol = (e % (CP / 8)) * 8, vrow = e >> 2, vcol = (e & 3) * 8;
        kr[i] = *reinterpret_cast<const u32x4*>(kb + (int64_t)(kbase + krow) * CP + kcol);
        vr[i] = *reinterpret_cast<const u32x4*>(vb + (int64_t)vrow * a.nkp + kbase + vcol);
        v2r[i] = *reinterpret_cast<const u32x4*>(v2b + (int64_t)vrow * a.nkp + kbase + vcol);
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      if (NPIECE % NT == 0 || e < NPIECE) {
        const int krow = e / (CP / 8), kcol = (e % (CP / 8)) * 8, vrow = e >> 2, vcol = (e & 3) * 8;
        *reinterpret_cast<u32x4*>(&ks[buf][krow * KROW + kcol]) = kr[i];
        // keys vcol..vcol+7 (vcol = 8u): first 4 to slot 16(u>>1) + 4(u&1), last 4 eight slots later
        const int u = vcol >> 3, slot = 16 * (u >> 1) + 4 * (u & 1);
        bf16* pv = &vs[buf][vrow * VPB + slot];
        *reinterpret_cast<u32x2*>(pv) = (u32x2){vr[i][0], vr[i][1]};
        *reinterpret_cast<u32x2*>(pv + 8) = (u32x2){vr[i][2], vr[i][3]};
        bf16* pv2 = &v2s[buf][vrow * VPB + slot];
        *reinterpret_cast<u32x2*>(pv2) = (u32x2){v2r[i][0], v2r[i][1]};
        *reinterpret_cast<u32x2*>(pv2 + 8) = (u32x2){v2r[i][2], v2r[i][3]};
      }
    }
  };

  f32x16 om[CT], osq[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    om[t] = (f32x16){0.f};
    osq[t] = (f32x16){0.f};
  }
  float mrow = -INFINITY;
  f32x2 lsum2 = {0.f, 0.f};
  const int j0 = sp * a.kchunk, nblk = min(a.nkp / BK, j0 + a.kchunk);
  gload(j0 * BK);
  lstore(0);
  for (int j = j0; j < nblk; ++j) {
    const int buf = (j - j0) & 1;
    if (j + 1 < nblk) gload((j + 1) * BK);
    __syncthreads();

    // S^T in log2 units (Q carries log2 e); two independent accumulation chains (a 32x32x16
    // MFMA's dependent latency is twice its issue interval)
    f32x16 s0 = (f32x16){0.f}, s1 = (f32x16){0.f};
    const bf16* kk = &ks[buf][r * KROW + 8 * h];
#pragma unroll
    for (int st = 0; st < CP / 16; st += 2) {
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(kk + 16 * st), qf[st], s0, 0, 0, 0);
      if (st + 1 < CP / 16)
        s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(kk + 16 * st + 16), qf[st + 1],
                                                     s1, 0, 0, 0);
    }
    f32x16 s = s0 + s1;
    if (j * BK + BK > a.nk) {  // last block only (wave-uniform)
      const int lim = a.nk - j * BK - 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = ((i & 3) + 8 * (i >> 2) < lim) ? s[i] : -INFINITY;
    }
    float mb = s[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mb = fmaxf(mb, s[i]);
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    if (__builtin_expect(__ballot(mb > mrow + kRescaleLog2) != 0, 0)) {
      const float mnew = fmaxf(mrow, mb);
      const float alpha = __builtin_amdgcn_exp2f(mrow - mnew);
      lsum2 *= alpha;
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        om[t] *= alpha;
        osq[t] *= alpha;
        __builtin_amdgcn_sched_barrier(0);
      }
      mrow = mnew;
    }
    bf16x8 pb[2];
    {
      const f32x2 m2 = {mrow, mrow};
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        f32x2 d = (f32x2){s[i], s[i + 1]} - m2;
        d[0] = __builtin_amdgcn_exp2f(d[0]);
        d[1] = __builtin_amdgcn_exp2f(d[1]);
        lsum2 += d;
        pb[i >> 3][i & 7] = (bf16)d[0];
        pb[i >> 3][(i & 7) + 1] = (bf16)d[1];
      }
    }

#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int off = (t * 32 + r) * VPB + 16 * st + 8 * h;
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(&vs[buf][off]);
        const bf16x8 va2 = *reinterpret_cast<const bf16x8*>(&v2s[buf][off]);
        om[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb[st], om[t], 0, 0, 0);
        osq[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va2, pb[st], osq[t], 0, 0, 0);
      }
    }
    if (j + 1 < nblk) lstore(buf ^ 1);
  }

  const float lsum = lsum2[0] + lsum2[1];
  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  if (a.part) {  // this split's partials (all nqp queries; the merge reads the first nq)
    const int64_t mq = (int64_t)a.ksplit * a.n * a.nqp;
    float* pm = a.part + ((int64_t)sp * a.n + b) * a.nqp;
    float* po = a.part + 2 * mq + ((int64_t)sp * a.n + b) * 2 * CP * a.nqp;
    if (h == 0) {
      pm[qi] = mrow;
      pm[mq + qi] = ltot;
    }
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ch = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        po[(int64_t)ch * a.nqp + qi] = om[t][i];
        po[(int64_t)(CP + ch) * a.nqp + qi] = osq[t][i];
      }
    return;
  }
  if (qi >= a.nq) return;
  const float inv = 1.0f / ltot;
  const float* cmean = a.stats + (int64_t)b * a.C;
  const float* crstd = a.stats + (int64_t)a.n * a.C + (int64_t)b * a.C;
  const float* vm = a.vmean + (int64_t)b * a.C;
  const bf16* __restrict__ cb = a.c + (int64_t)b * a.C * a.nq;
  bf16* __restrict__ ob = a.out + (int64_t)b * a.C * a.nq;
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ch = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (ch < a.C) {
        const float mean = om[t][i] * inv;  // of the centred V
        float var = fmaf(-mean, mean, osq[t][i] * inv);
        var = var < 0.f ? 0.f : var;
        const int64_t o = (int64_t)ch * a.nq + qi;
        const float xn = ((float)cb[o] - cmean[ch]) * crstd[ch];
        ob[o] = (bf16)fmaf(sqrtf(var), xn, mean + vm[ch]);
      }
    }
}

// The splits of attend_*_kernel combined, in split order, then the epilogue: with M = max_s m_s,
// w_s = 2^(m_s - M): mean = sum w_s O_s / sum w_s l_s, E[v^2] likewise (bf16: + the V mean).
struct MergeArgs {
  const void* c;
  const float* stats;
  const float* vmean;  // null on the fp32 path (V not centred)
  void* out;
  const float* part;
  int n, C, Cp, nq, nqp, ksplit;
};

template <typename TO>
__global__ __launch_bounds__(256) void attn_merge_kernel(MergeArgs a) {
  const int64_t total = (int64_t)a.n * a.C * a.nq;
  const int64_t mq = (int64_t)a.ksplit * a.n * a.nqp;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int q = (int)(idx % a.nq);
    const int64_t bc = idx / a.nq;
    const int ch = (int)(bc % a.C), b = (int)(bc / a.C);
    float M = -INFINITY;
    for (int s = 0; s < a.ksplit; ++s) M = fmaxf(M, a.part[((int64_t)s * a.n + b) * a.nqp + q]);
    float L = 0.f, O = 0.f, O2 = 0.f;
    for (int s = 0; s < a.ksplit; ++s) {
      const int64_t mi = ((int64_t)s * a.n + b) * a.nqp + q;
      const float w = __builtin_amdgcn_exp2f(a.part[mi] - M);
      const float* po = a.part + 2 * mq + ((int64_t)s * a.n + b) * 2 * a.Cp * a.nqp;
      L = fmaf(w, a.part[mq + mi], L);
      O = fmaf(w, po[(int64_t)ch * a.nqp + q], O);
      O2 = fmaf(w, po[(int64_t)(a.Cp + ch) * a.nqp + q], O2);
    }
    const float inv = 1.0f / L;
    const float mean = O * inv;
    float var = fmaf(-mean, mean, O2 * inv);
    var = var < 0.f ? 0.f : var;
    const int64_t o = ((int64_t)b * a.C + ch) * a.nq + q;
    const float xn = ((float)((const TO*)a.c)[o] - a.stats[(int64_t)b * a.C + ch]) *
                     a.stats[(int64_t)a.n * a.C + (int64_t)b * a.C + ch];
    ((TO*)a.out)[o] = (TO)fmaf(sqrtf(var), xn, a.vmean ? mean + a.vmean[(int64_t)b * a.C + ch] : mean);
  }
}

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace


namespace {

struct AttnLayout {  // workspace carve-up (bytes), shared by the size query and the launcher
  int cp, nqp, nkp, ksplit, kchunk;
  size_t stats, vmean, q, k, v, v2, part, total;
};

// bf16 path: split the keys when the query tiles leave the chip underfilled (< 256 workgroups):
// ~512 workgroups, >= 2 key blocks per split (AST_ATTN_KSPLIT=0: never, for A/B runs)
void attn_split(int dtype, int n, int nqp, int nkp, int& ksplit, int& kchunk) {
  static const int on = [] {
    const char* v = getenv("AST_ATTN_KSPLIT");
    return v ? atoi(v) : 1;
  }();
  const int nblk = nkp / BK;
  const bool big = dtype != 0 && (int64_t)n * (nqp / 256) >= 512;  // fp32: 128 queries per workgroup
  const int64_t wgs = (int64_t)n * (nqp / (big ? 256 : 128));
  int ks = 1;
  if (on && wgs < 256 && nblk >= 4) ks = (int)std::min<int64_t>((512 + wgs - 1) / wgs, nblk / 2);
  kchunk = (nblk + ks - 1) / ks;
  ksplit = (nblk + kchunk - 1) / kchunk;  // every split non-empty
}

AttnLayout attn_layout(int dtype, int n, int c, int nq, int nk) {
  AttnLayout L;
  L.cp = round_up(c, 32);
  L.nqp = round_up(nq, dtype == 0 ? 128 : 256);
  L.nkp = round_up(nk, BK);
  const size_t es = dtype == 0 ? 4 : 2;
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  L.stats = 0;
  L.vmean = al(4 * sizeof(float) * (size_t)n * c);
  L.q = L.vmean + al(sizeof(float) * (size_t)n * c);
  L.k = L.q + al(es * (size_t)n * L.cp * L.nqp);
  L.v = L.k + al(es * (size_t)n * L.cp * L.nkp);
  L.v2 = L.v + al(es * (size_t)n * L.cp * L.nkp);
  L.part = dtype == 0 ? L.v2 : L.v2 + al(es * (size_t)n * L.cp * L.nkp);
  attn_split(dtype, n, L.nqp, L.nkp, L.ksplit, L.kchunk);
  L.total = L.part + (L.ksplit > 1 ? al(sizeof(float) * (size_t)L.ksplit * n * L.nqp * (2 + 2 * (size_t)L.cp)) : 0);
  return L;
}

template <typename K>
hipError_t set_lds(K kern, size_t bytes) {
  return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" {

size_t ast_adaattn_workspace_bytes(int dtype, int n, int c, int hc, int wc, int hs, int ws) {
  if (n <= 0 || c <= 0 || hc <= 0 || wc <= 0 || hs <= 0 || ws <= 0 || (dtype != 0 && dtype != 1)) return 0;
  return attn_layout(dtype, n, c, hc * wc, hs * ws).total;
}

int ast_adaattn_fwd(int dtype, const void* content, const void* style, const float* wq, const float* wk,
                    const float* wv, void* out, void* workspace, size_t workspace_bytes, int n, int c, int hc,
                    int wc, int hs, int ws, void* stream) {
  if (!content || !style || !wq || !wk || !wv || !out || !workspace) return AST_E_NULLPTR;
  if (n <= 0 || c <= 0 || hc <= 0 || wc <= 0 || hs <= 0 || ws <= 0) return AST_E_SHAPE;
  if (dtype != 0 && dtype != 1) return AST_E_UNSUPPORTED;
  if (c > 128) return AST_E_UNSUPPORTED;
  if ((int64_t)hc * wc > (1 << 28) || (int64_t)hs * ws > (1 << 28) || (int64_t)n * c > (1 << 28)) return AST_E_SHAPE;
  if (workspace_bytes < ast_adaattn_workspace_bytes(dtype, n, c, hc, wc, hs, ws)) return AST_E_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int nq = hc * wc, nk = hs * ws;
  const AttnLayout L = attn_layout(dtype, n, c, nq, nk);
  const int cp = L.cp, nqp = L.nqp, nkp = L.nkp, ct = cp / 32;
  unsigned char* wsb = (unsigned char*)workspace;
  float* stats = (float*)(wsb + L.stats);
  const dim3 pgrid((unsigned)(round_up(nqp > nkp ? nqp : nkp, 128) / 128), (unsigned)n, 3);
  const size_t plds = sizeof(float) * (size_t)((c + 1) & ~1) * (cp + 32);
  hipError_t e;

  if (dtype == 0) {
    float* q = (float*)(wsb + L.q);
    float* k = (float*)(wsb + L.k);
    float* v = (float*)(wsb + L.v);
    hipLaunchKernelGGL(in_stats_kernel<float>, dim3(n * c, 2), dim3(kStatThreads), 0, st, (const float*)content,
                       (const float*)style, stats, n * c, (int64_t)nq, (int64_t)nk, 1e-5f);
    ProjArgs pa{content, style, wq, wk, wv, stats, q, k, v, n, c, cp, nq, nk, nqp, nkp};
    void (*proj)(ProjArgs) = ct == 1 ? project_kernel<float, 1> : ct == 2 ? project_kernel<float, 2>
                           : ct == 3 ? project_kernel<float, 3> : project_kernel<float, 4>;
    if ((e = set_lds(proj, plds)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(proj, pgrid, dim3(256), plds, st, pa);
    const int qtiles = nqp / 128;
    float* part = L.ksplit > 1 ? (float*)(wsb + L.part) : nullptr;
    AttnArgs aa{q, k, v, content, stats, out, n, c, cp, nq, nk, nqp, nkp, qtiles, L.ksplit, L.kchunk, part};
    void (*att)(AttnArgs) = ct == 1 ? attend_f32_kernel<float, 1> : ct == 2 ? attend_f32_kernel<float, 2>
                          : ct == 3 ? attend_f32_kernel<float, 3> : attend_f32_kernel<float, 4>;
    hipLaunchKernelGGL(att, dim3((unsigned)(n * qtiles * L.ksplit)), dim3(256), 0, st, aa);
    if (L.ksplit > 1) {
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
      const int64_t tot = (int64_t)n * c * nq;
      MergeArgs ma{content, stats, nullptr, out, part, n, c, cp, nq, nqp, L.ksplit};
      hipLaunchKernelGGL(attn_merge_kernel<float>, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 8192)), dim3(256),
                         0, st, ma);
    }
    return (int)hipGetLastError();
  }

  bf16* q = (bf16*)(wsb + L.q);
  bf16* k = (bf16*)(wsb + L.k);
  bf16* v = (bf16*)(wsb + L.v);
  bf16* v2 = (bf16*)(wsb + L.v2);
  float* vmean = (float*)(wsb + L.vmean);
  hipLaunchKernelGGL(in_stats_kernel<bf16>, dim3(n * c, 2), dim3(kStatThreads), 0, st, (const bf16*)content,
                     (const bf16*)style, stats, n * c, (int64_t)nq, (int64_t)nk, 1e-5f);
  hipLaunchKernelGGL(vmean_kernel, dim3(n), dim3(128), 0, st, wv, stats, vmean, n, c);
  ProjB16Args pa{(const bf16*)content, (const bf16*)style, wq, wk, wv, stats, q, k, v, v2, n, c, cp, nq, nk, nqp, nkp};
  void (*proj)(ProjB16Args) = ct == 1 ? project_bf16_kernel<1> : ct == 2 ? project_bf16_kernel<2>
                            : ct == 3 ? project_bf16_kernel<3> : project_bf16_kernel<4>;
  const size_t plds16 = 2 * (size_t)(128 + cp) * (((c + 15) & ~15) + 8);
  if ((e = set_lds(proj, plds16)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(proj, pgrid, dim3(256), plds16, st, pa);
  // 8 waves (256 queries) per workgroup: each K/V block staged in LDS serves 256 queries. Small
  // problems (< 512 such workgroups) use 4-wave workgroups instead, to spread over more CUs.
  const bool big = (int64_t)n * (nqp / 256) >= 512;
  const int nw = big ? 8 : 4, qtiles = nqp / (nw * 32);
  float* part = L.ksplit > 1 ? (float*)(wsb + L.part) : nullptr;
  AttnB16Args aa{q, k, v, v2, (const bf16*)content, stats, vmean, (bf16*)out, n, c, cp, nq, nk, nqp, nkp, qtiles,
                 L.ksplit, L.kchunk, part};
  void (*att)(AttnB16Args);
  if (big)
    att = ct == 1 ? attend_bf16_kernel<1, 8> : ct == 2 ? attend_bf16_kernel<2, 8> : ct == 3 ? attend_bf16_kernel<3, 8>
                                                                                    : attend_bf16_kernel<4, 8>;
  else
    att = ct == 1 ? attend_bf16_kernel<1, 4> : ct == 2 ? attend_bf16_kernel<2, 4> : ct == 3 ? attend_bf16_kernel<3, 4>
                                                                                    : attend_bf16_kernel<4, 4>;
  hipLaunchKernelGGL(att, dim3((unsigned)(n * qtiles * L.ksplit)), dim3(nw * 64), 0, st, aa);
  if (L.ksplit > 1) {
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    const int64_t tot = (int64_t)n * c * nq;
    MergeArgs ma{content, stats, vmean, out, part, n, c, cp, nq, nqp, L.ksplit};
    hipLaunchKernelGGL(attn_merge_kernel<bf16>, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 8192)), dim3(256),
                       0, st, ma);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
