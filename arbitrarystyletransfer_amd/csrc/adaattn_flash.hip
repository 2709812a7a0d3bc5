// AdaAttN backward without the attention matrix (models.py:81-115): flash-style
// passes that recompute the scores per 16 x 16 (query, key) block in registers, so neither P nor dS
// ([n][Nq][Nk], 1 GB per image at 128^2 maps) is ever stored. The math is adaattn_bwd.hip's:
//   S = Q^T K,  P = softmax_keys(S),  O = P [V; V^2]^T = [mean | ex2]                  [Nq][2C]
//   dO and D[q] = sum_j dO[q][j] O[q][j]  (adaattn_bwd.hip dstats_kernel, unchanged)
//   dP = dO [V; V^2],  dS = P * (dP - D),  d[V; V^2] = dO^T P,  dK = Q dS,  dQ = K dS^T
// Three passes, each one launch over (64-row tile, image):
//   stats  (lane = query): O and the row log-sum-exp (log2 units) by an online softmax over key blocks
//   kv     (lane = key):   per query block: S, P = exp2(S log2e - lse), dP, dS; accumulates d[V; V^2] and
//                          dK for the lane's key over every query (no cross-lane or cross-block sums)
//   q      (lane = query): per key block: S^T, P^T, dP^T, dS^T; accumulates dQ for the lane's query
// Every output element is summed by one lane in a fixed order: deterministic, no atomics.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation, as the reference trains in
// fp32). Lane l feeds A[i = l & 15][k = l >> 4] and B[k = l >> 4][j = l & 15] and holds D[4 (l >> 4) + r]
// [l & 15], r = 0..3. A product summed over the lane's own register index (queries or keys 4g + r of
// the block, g = l >> 4) takes that operand straight from the accumulator registers of the previous
// product: instruction r pairs k = g with index 4g + r. Operands that vary along the tile's rows come
// from LDS tiles [rows][16] at pitch 17 (two access patterns, both at most 2-way bank conflicts);
// the block's other operand (the lane's own query or key over all channels) sits in registers.
// Channels C: a multiple of 16, at most 128 (the host keeps the materialised path otherwise).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TP = 17;  // LDS pitch (floats) of a [rows][16] tile
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kRescaleLog2 = 8.0f;  // lazy online-softmax rescale, as attend_f32_kernel

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// A [rows][cols] matrix's columns col0..col0+15 as a [rows][16] tile (columns >= ncols read as 0),
// prefetched into registers (E per thread) and stored into LDS at pitch TP.
template <int ROWS>
struct ColTile {
  static constexpr int E = ROWS * 16 / 256;
  float r[E];
  __device__ __forceinline__ void load(const float* __restrict__ src, int64_t ld, int col0, int ncols, int tid) {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = tid + i * 256, row = e >> 4, col = e & 15;
      r[i] = col0 + col < ncols ? src[(int64_t)row * ld + col0 + col] : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ t, int tid) const {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = tid + i * 256;
      t[(e >> 4) * TP + (e & 15)] = r[i];
    }
  }
};

// rows row0..row0+15 of a [nrows][ROWS] matrix (row-major, rows >= nrows read as 0) TRANSPOSED into
// a [ROWS][16] tile: global reads run along the contiguous dimension
template <int ROWS>
struct RowTileT {
  static constexpr int E = ROWS * 16 / 256;
  float r[E];
  __device__ __forceinline__ void load(const float* __restrict__ src, int row0, int nrows, int tid) {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = tid + i * 256, c = e % ROWS, q = e / ROWS;
      r[i] = row0 + q < nrows ? src[(int64_t)(row0 + q) * ROWS + c] : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ t, int tid) const {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = tid + i * 256, c = e % ROWS, q = e / ROWS;
      t[c * TP + q] = r[i];
    }
  }
};

// ---- stats: O = softmax(S) [V; V^2]^T and lse2 per query ---------------------------------------
template <int CT>
__global__ __launch_bounds__(256) void flash_stats_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                          const float* __restrict__ vv, float* __restrict__ o2,
                                                          float* __restrict__ lse2, int nq, int nk) {
  constexpr int C = CT * 16;
  __shared__ float kt[2][C * TP];
  __shared__ float vt[2][2 * C * TP];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 15, g = lane >> 4;
  const int qi = blockIdx.x * 64 + w * 16 + j;
  const float* __restrict__ qb = q + (int64_t)b * C * nq;
  const float* __restrict__ kb = k + (int64_t)b * C * nk;
  const float* __restrict__ vb = vv + (int64_t)b * 2 * C * nk;
  float qr[C / 4];
#pragma unroll
  for (int m = 0; m < C / 4; ++m) qr[m] = qi < nq ? qb[(int64_t)(4 * m + g) * nq + qi] : 0.f;
  f32x4 acc[2 * CT];
#pragma unroll
  for (int t = 0; t < 2 * CT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow = -INFINITY, lsum = 0.f;
  ColTile<C> kp;
  ColTile<2 * C> vp;
  const int nblk = (nk + 15) / 16;
  kp.load(kb, nk, 0, nk, tid);
  vp.load(vb, nk, 0, nk, tid);
  kp.store(kt[0], tid);
  vp.store(vt[0], tid);
  for (int jb = 0; jb < nblk; ++jb) {
    const int buf = jb & 1;
    if (jb + 1 < nblk) {
      kp.load(kb, nk, (jb + 1) * 16, nk, tid);
      vp.load(vb, nk, (jb + 1) * 16, nk, tid);
    }
    __syncthreads();
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};  // S^T[key 4g + r][query j]
    const float* ka = kt[buf] + g * TP + j;
#pragma unroll
    for (int m = 0; m < C / 4; ++m) s = mma(ka[4 * m * TP], qr[m], s);
    float p[4];
    float mb = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = jb * 16 + 4 * g + r < nk ? s[r] * kLog2e : -INFINITY;
      mb = fmaxf(mb, p[r]);
    }
    mb = fmaxf(mb, __shfl_xor(mb, 16, 64));
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    if (__builtin_expect(__ballot(mb > mrow + kRescaleLog2) != 0, 0)) {
      const float mnew = fmaxf(mrow, mb);
      const float alpha = exp2f(mrow - mnew);  // 0 on the first block
      lsum *= alpha;
#pragma unroll
      for (int t = 0; t < 2 * CT; ++t) acc[t] *= alpha;
      mrow = mnew;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = exp2f(p[r] - mrow);
      lsum += p[r];
    }
    const float* va = vt[buf] + j * TP + 4 * g;  // VV[16 t + j][key 4g + r]
#pragma unroll
    for (int t = 0; t < 2 * CT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t] = mma(va[16 * t * TP + r], p[r], acc[t]);
    if (jb + 1 < nblk) {
      kp.store(kt[buf ^ 1], tid);
      vp.store(vt[buf ^ 1], tid);
    }
  }
  float lt = lsum + __shfl_xor(lsum, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  if (qi >= nq) return;
  const float inv = 1.f / lt;
  float* __restrict__ ob = o2 + ((int64_t)b * nq + qi) * 2 * C + 4 * g;
#pragma unroll
  for (int t = 0; t < 2 * CT; ++t) *reinterpret_cast<f32x4*>(ob + 16 * t) = acc[t] * inv;
  if (g == 0) lse2[(int64_t)b * nq + qi] = mrow + log2f(lt);
}

// ---- kv: dK and d[V; V^2] (lane = key) ---------------------------------------------------------
template <int CT>
__global__ __launch_bounds__(256) void flash_bwd_kv_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ vv, const float* __restrict__ do2,
                                                           const float* __restrict__ lse2, const float* __restrict__ drow,
                                                           float* __restrict__ dk, float* __restrict__ dvv, int nq,
                                                           int nk) {
  constexpr int C = CT * 16;
  __shared__ float qt[2][C * TP];       // Q[c][query]
  __shared__ float dt[2][2 * C * TP];   // dO^T[c2][query]
  __shared__ float ls[2][16], dd[2][16];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 15, g = lane >> 4;
  const int kj = blockIdx.x * 64 + w * 16 + j;
  const float* __restrict__ qb = q + (int64_t)b * C * nq;
  const float* __restrict__ kb = k + (int64_t)b * C * nk;
  const float* __restrict__ vb = vv + (int64_t)b * 2 * C * nk;
  const float* __restrict__ gb = do2 + (int64_t)b * nq * 2 * C;
  const float* __restrict__ lb = lse2 + (int64_t)b * nq;
  const float* __restrict__ db = drow + (int64_t)b * nq;
  float kr[C / 4], vr[C / 2];
#pragma unroll
  for (int m = 0; m < C / 4; ++m) kr[m] = kj < nk ? kb[(int64_t)(4 * m + g) * nk + kj] : 0.f;
#pragma unroll
  for (int m = 0; m < C / 2; ++m) vr[m] = kj < nk ? vb[(int64_t)(4 * m + g) * nk + kj] : 0.f;
  f32x4 dka[CT], dva[2 * CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) dka[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2 * CT; ++t) dva[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  ColTile<C> qp;
  RowTileT<2 * C> gp;
  float lv = 0.f, dv = 0.f;
  const int nblk = (nq + 15) / 16;
  auto load = [&](int blk) {
    qp.load(qb, nq, blk * 16, nq, tid);
    gp.load(gb, blk * 16, nq, tid);
    if (tid < 16) {
      const int qq = blk * 16 + tid;
      lv = qq < nq ? lb[qq] : INFINITY;  // padded queries: P = exp2(-inf) = 0
      dv = qq < nq ? db[qq] : 0.f;
    }
  };
  auto store = [&](int bf) {
    qp.store(qt[bf], tid);
    gp.store(dt[bf], tid);
    if (tid < 16) {
      ls[bf][tid] = lv;
      dd[bf][tid] = dv;
    }
  };
  load(0);
  store(0);
  for (int qblk = 0; qblk < nblk; ++qblk) {
    const int buf = qblk & 1;
    if (qblk + 1 < nblk) load(qblk + 1);
    __syncthreads();
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};  // [query 4g + r][key j]
    const float* qa = qt[buf] + g * TP + j;
#pragma unroll
    for (int m = 0; m < C / 4; ++m) s = mma(qa[4 * m * TP], kr[m], s);
    const float* ga = dt[buf] + g * TP + j;
#pragma unroll
    for (int m = 0; m < C / 2; ++m) dp = mma(ga[4 * m * TP], vr[m], dp);
    float p[4], ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = exp2f(fmaf(s[r], kLog2e, -ls[buf][4 * g + r]));
      ds[r] = p[r] * (dp[r] - dd[buf][4 * g + r]);
    }
    const float* gt = dt[buf] + j * TP + 4 * g;  // dO[query 4g + r][c2 = 16 t + j]
#pragma unroll
    for (int t = 0; t < 2 * CT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) dva[t] = mma(gt[16 * t * TP + r], p[r], dva[t]);
    const float* qtt = qt[buf] + j * TP + 4 * g;  // Q[c = 16 t + j][query 4g + r]
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) dka[t] = mma(qtt[16 * t * TP + r], ds[r], dka[t]);
    if (qblk + 1 < nblk) store(buf ^ 1);
  }
  if (kj >= nk) return;
  float* __restrict__ dkb = dk + (int64_t)b * C * nk + kj;
  float* __restrict__ dvb = dvv + (int64_t)b * 2 * C * nk + kj;
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dkb[(int64_t)(16 * t + 4 * g + r) * nk] = dka[t][r];
#pragma unroll
  for (int t = 0; t < 2 * CT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dvb[(int64_t)(16 * t + 4 * g + r) * nk] = dva[t][r];
}

// ---- q: dQ (lane = query) ----------------------------------------------------------------------
template <int CT>
__global__ __launch_bounds__(256) void flash_bwd_q_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                          const float* __restrict__ vv, const float* __restrict__ do2,
                                                          const float* __restrict__ lse2, const float* __restrict__ drow,
                                                          float* __restrict__ dq, int nq, int nk) {
  constexpr int C = CT * 16;
  __shared__ float kt[2][C * TP];       // K[c][key]
  __shared__ float vt[2][2 * C * TP];   // VV[c2][key]
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 15, g = lane >> 4;
  const int qi = blockIdx.x * 64 + w * 16 + j;
  const bool qin = qi < nq;
  const float* __restrict__ qb = q + (int64_t)b * C * nq;
  const float* __restrict__ kb = k + (int64_t)b * C * nk;
  const float* __restrict__ vb = vv + (int64_t)b * 2 * C * nk;
  const float* __restrict__ gq = do2 + ((int64_t)b * nq + (qin ? qi : 0)) * 2 * C;
  float qr[C / 4], gr[C / 2];
#pragma unroll
  for (int m = 0; m < C / 4; ++m) qr[m] = qin ? qb[(int64_t)(4 * m + g) * nq + qi] : 0.f;
#pragma unroll
  for (int m = 0; m < C / 2; ++m) gr[m] = qin ? gq[4 * m + g] : 0.f;
  const float lq = qin ? lse2[(int64_t)b * nq + qi] : 0.f;
  const float dq_row = qin ? drow[(int64_t)b * nq + qi] : 0.f;
  f32x4 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  ColTile<C> kp;
  ColTile<2 * C> vp;
  const int nblk = (nk + 15) / 16;
  kp.load(kb, nk, 0, nk, tid);
  vp.load(vb, nk, 0, nk, tid);
  kp.store(kt[0], tid);
  vp.store(vt[0], tid);
  for (int jb = 0; jb < nblk; ++jb) {
    const int buf = jb & 1;
    if (jb + 1 < nblk) {
      kp.load(kb, nk, (jb + 1) * 16, nk, tid);
      vp.load(vb, nk, (jb + 1) * 16, nk, tid);
    }
    __syncthreads();
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};  // [key 4g + r][query j]
    const float* ka = kt[buf] + g * TP + j;
#pragma unroll
    for (int m = 0; m < C / 4; ++m) s = mma(ka[4 * m * TP], qr[m], s);
    const float* va = vt[buf] + g * TP + j;
#pragma unroll
    for (int m = 0; m < C / 2; ++m) dp = mma(va[4 * m * TP], gr[m], dp);
    float ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = jb * 16 + 4 * g + r < nk ? exp2f(fmaf(s[r], kLog2e, -lq)) : 0.f;
      ds[r] = p * (dp[r] - dq_row);
    }
    const float* kt2 = kt[buf] + j * TP + 4 * g;  // K[c = 16 t + j][key 4g + r]
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t] = mma(kt2[16 * t * TP + r], ds[r], acc[t]);
    if (jb + 1 < nblk) {
      kp.store(kt[buf ^ 1], tid);
      vp.store(vt[buf ^ 1], tid);
    }
  }
  if (!qin) return;
  float* __restrict__ dqb = dq + (int64_t)b * C * nq + qi;
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dqb[(int64_t)(16 * t + 4 * g + r) * nq] = acc[t][r];
}

int check_shape(int n, int c, int nq, int nk) {
  if (n <= 0 || nq <= 0 || nk <= 0) return AST_E_SHAPE;
  if (c % 16 || c < 16 || c > 128 || c == 80 || c == 112) return AST_E_UNSUPPORTED;
  if (n > 65535 || (nq + 63) / 64 > 0x7fffffff || (nk + 63) / 64 > 0x7fffffff) return AST_E_SHAPE;
  return 0;
}

#define AST_FLASH_DISPATCH(KERNEL, GRIDX, ...)                                                       \
  switch (c / 16) {                                                                                 \
    case 1: hipLaunchKernelGGL(KERNEL<1>, dim3(GRIDX, n), dim3(256), 0, st, __VA_ARGS__); break;    \
    case 2: hipLaunchKernelGGL(KERNEL<2>, dim3(GRIDX, n), dim3(256), 0, st, __VA_ARGS__); break;    \
    case 3: hipLaunchKernelGGL(KERNEL<3>, dim3(GRIDX, n), dim3(256), 0, st, __VA_ARGS__); break;    \
    case 4: hipLaunchKernelGGL(KERNEL<4>, dim3(GRIDX, n), dim3(256), 0, st, __VA_ARGS__); break;    \
    case 6: hipLaunchKernelGGL(KERNEL<6>, dim3(GRIDX, n), dim3(256), 0, st, __VA_ARGS__); break;    \
    default: hipLaunchKernelGGL(KERNEL<8>, dim3(GRIDX, n), dim3(256), 0, st, __VA_ARGS__); break;   \
  }

}  // namespace

extern "C" {

int ast_adaattn_flash_supported(int c) { return check_shape(1, c, 1, 1) == 0 ? 1 : 0; }

int ast_adaattn_flash_stats_f32(const float* q, const float* k, const float* vv, float* o2, float* lse2, int n, int c,
                                int nq, int nk, void* stream) {
  if (!q || !k || !vv || !o2 || !lse2) return AST_E_NULLPTR;
  if (const int e = check_shape(n, c, nq, nk)) return e;
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = (unsigned)((nq + 63) / 64);
  AST_FLASH_DISPATCH(flash_stats_kernel, gx, q, k, vv, o2, lse2, nq, nk)
  return (int)hipGetLastError();
}

int ast_adaattn_flash_bwd_kv_f32(const float* q, const float* k, const float* vv, const float* do2, const float* lse2,
                                 const float* drow, float* dk, float* dvv, int n, int c, int nq, int nk, void* stream) {
  if (!q || !k || !vv || !do2 || !lse2 || !drow || !dk || !dvv) return AST_E_NULLPTR;
  if (const int e = check_shape(n, c, nq, nk)) return e;
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = (unsigned)((nk + 63) / 64);
  AST_FLASH_DISPATCH(flash_bwd_kv_kernel, gx, q, k, vv, do2, lse2, drow, dk, dvv, nq, nk)
  return (int)hipGetLastError();
}

int ast_adaattn_flash_bwd_q_f32(const float* q, const float* k, const float* vv, const float* do2, const float* lse2,
                                const float* drow, float* dq, int n, int c, int nq, int nk, void* stream) {
  if (!q || !k || !vv || !do2 || !lse2 || !drow || !dq) return AST_E_NULLPTR;
  if (const int e = check_shape(n, c, nq, nk)) return e;
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = (unsigned)((nq + 63) / 64);
  AST_FLASH_DISPATCH(flash_bwd_q_kernel, gx, q, k, vv, do2, lse2, drow, dq, nq, nk)
  return (int)hipGetLastError();
}

}  // extern "C"
