// MobileNet expand + depthwise, v5: the 5x5 depthwise of the
// stride-1 expand blocks on the matrix cores.
//
// v4 (mb_ed4.hip) keeps the hidden rows in registers and runs the depthwise as 25 scalar v_fma_f32
// per output; on the k5 blocks that is ~0.6 VALU wave-instructions per output at ~4 cycles each, and
// the SIMD's VALU issue, not HBM, sets the time (profiles/r02_pmc_ed4.txt: 19.2k VALU per wave, 14k
// of them depthwise FMAs). Here the depthwise of one hidden channel over a 32-row x 28-column output
// tile is a Toeplitz product on v_mfma_f32_32x32x16_bf16:
//
//   D[m][n] = sum_ky sum_w  T_ky,w[m][k] . H[n + ky][16 w + k]      (m = output column 0..31 of which
//                                                                    28 are kept, n = output row)
//   T_ky,w[m][k] = wdw[ky][16 w + k - m]  where 0 <= 16 w + k - m <= 4, else 0
//
// i.e. 5 kernel rows x 2 sixteen-column windows = 10 MFMAs per channel and tile (1024 MACs for every
// 25 useful ones is cheap: the matrix pipe has ~40x the VALU's MAC rate). The operands:
//   B (hidden image, K = input column, N = output row): lane (n, g) reads 8 consecutive bf16 of
//     hidden row n + ky -- one ds_read_b128 from the [channel][row][col] LDS image, row pitch 80 B
//     (conflict-free for the b128 lane groups);
//   A (Toeplitz weights, M = output column): lane (m, g) needs the 8 entries s..s+7 of the channel's
//     zero-padded kernel row R_ky (R[t] = w[ky][t - 31]), s = 16 w + 8 g - m + 31; eight copies of
//     the row's nonzero neighbourhood, each shifted by one element, make every window one aligned
//     ds_read_b128 (4 x ds_read_b32 from two copies ran LDS-bound at two waves per SIMD).
// The hidden values are rounded to bf16 (the MFMA operand) and so are the folded depthwise weights:
// a bf16 model's own tensors (the reference in bf16 stores the expand output as bf16); accumulation
// is fp32. The tests bound the block against the fp32 oracle at the bf16 bar.
//
// A workgroup is 8 waves on one output tile (32 rows x 28 columns of one image) and loops over the
// hidden channels in chunks of 32:
//   expand:    the 36 input rows x 32 columns on v_mfma_f32_32x32x16_bf16 (C[pixel][channel], a lane
//              holds one channel and 16 consecutive columns of a row, as in v4), bias, Hardswish, bf16,
//              two ds_write_b128 per lane into the hidden image (channel pitch 2896 B: conflict-free);
//              the x fragments of a wave's rows stay in registers across the chunks;
//   depthwise: each wave 4 channels: 10 MFMAs, +bias, Hardswish, the SE-pool partial sum, bf16; D
//              staged through the channel's own (consumed) hidden image and stored as 8-byte pieces,
//              7 lanes per 56-byte row run (buffer stores: pieces past the image get an out-of-range
//              offset and drop).
// Two barriers per chunk; 136 KB of LDS, one workgroup (two waves per SIMD) per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "mb_common.h"

namespace ast_mb {
namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int refl5(int i, int n) {  // reflection pad, clamped for garbage rows / columns
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * n - 2 - i : i;
  return min(max(i, 0), n - 1);
}

__device__ __forceinline__ unsigned short bits16(float v) { return __builtin_bit_cast(unsigned short, (bf16)v); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2(float lo, float hi) {  // one v_cvt_pk_bf16_f32 (RNE) per pair
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}

__device__ __forceinline__ float hswish5(float v) {  // x * clamp(x/6 + 1/2, 0, 1), as v4's hswish_fast
  return v * __builtin_amdgcn_fmed3f(fmaf(v, 1.f / 6.f, 0.5f), 0.f, 1.f);
}

#ifndef ED5_SKIP
#define ED5_SKIP 0  // timing-only builds (wrong results): 1 no D stores, 2 no depthwise MFMAs / operand reads,
                    // 4 no expand MFMAs, 8 no Toeplitz A reads (constant A), 16 no hidden-image writes
#endif

constexpr int K5 = 5, P5 = 2;
constexpr int TH = 32;             // output rows per tile (N of the depthwise MFMA)
constexpr int OW = 28;             // output columns per tile (M = 32, the last 4 dropped)
constexpr int IR = TH + K5 - 1;    // 36 input rows
constexpr int RP = 80;             // hidden row pitch (bytes): 16 * odd -> conflict-free B reads
constexpr int CP = IR * RP + 16;   // channel pitch 2896 B: CP / 4 = 4 * odd mod 32 -> conflict-free writes
constexpr int TP = 5 * 8 * 32;     // Toeplitz table bytes per channel: [ky][copy 0..7][16 bf16]
constexpr int NCH = 32;            // hidden channels per chunk
constexpr int NW = 8;              // waves per workgroup
constexpr int LDS_H = NCH * CP;    // 92,672
constexpr int LDS_T = NCH * TP;    // 40,960
constexpr int NT = (IR + NW - 1) / NW;  // input-row slots per wave (5)

template <int KS>
__global__ __launch_bounds__(64 * NW, 2) void expand_dw5_kernel(EdArgs a, int strips, int bands, int ncb, int total) {
  __shared__ __align__(16) unsigned char lds[LDS_H + LDS_T];
  unsigned char* const Hs = lds;
  unsigned char* const Ts = lds + LDS_H;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  // XCD-aware order (workgroup b runs on XCD b % 8): consecutive tiles of an image row band share an L2
  const int per = (total + 7) >> 3;
  const int L = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (L >= total) return;  // uniform over the workgroup
  const int s = L % strips;
  const int rest = L / strips;
  const int band = rest % bands, n = rest / bands;
  const int x0 = s * OW - P5, y0 = band * TH;

  // zero the Toeplitz tables once: only the 25 x 2 weight entries per channel change per chunk
  for (int i = tid; i < LDS_T / 16; i += 64 * NW) reinterpret_cast<uint4*>(Ts)[i] = make_uint4(0u, 0u, 0u, 0u);

  // x fragments of this wave's input rows j = wv + 8 t (A of the expand: lane (pixel r, k-group h))
  const int pc = 16 * ((r >> 2) & 1) + (r & 3) + 4 * (r >> 3);  // C rows of a lane half = 16 consecutive columns
  const int gx = refl5(x0 + pc, a.w);
  const int hw2 = 2 * a.h * a.w;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(reinterpret_cast<const bf16*>(a.x1) + (int64_t)n * a.cin * (hw2 / 2)), 0, a.cin * hw2,
      0x00020000);
  bf16x8 xa[NT][KS];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = wv + NW * t;
    if (j < IR) {
      const int vrow = 8 * h * hw2 + 2 * (refl5(y0 - P5 + j, a.h) * a.w + gx);
      unsigned raw[KS][8];
#pragma unroll
      for (int q = 0; q < KS; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          raw[q][e] = (ED5_SKIP & 32) ? (unsigned)(vrow + q + e) & 0x3f3fu
                                      : __builtin_amdgcn_raw_buffer_load_b16(xr, vrow + (16 * q + e) * hw2, 0, 0);
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        u32x4 f;
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = (raw[q][2 * e] & 0xffffu) | (raw[q][2 * e + 1] << 16);
        xa[t][q] = __builtin_bit_cast(bf16x8, f);
      }
    }
  }

  // depthwise operand offsets: A (Toeplitz) start s = 16 w + 8 h - r + 31, from the copy that makes it
  // 4-byte aligned; B lane (row r, k-group h) at r * RP + 16 h
  // The 8 entries s..s+7 are all zero unless s is in [24, 35]; the other windows read entries 36..43
  // (zeros), so every window lies in R[24..43]. Copy k of a kernel row holds R[24 + k .. 39 + k]: the
  // window starting at s comes from copy s & 7 at entry s - (s & 7) - 24 (0 or 8), a 16-byte-aligned
  // ds_read_b128; the 16 distinct (copy, half) slots of a row are 256 B, so a lane group reads
  // conflict-free (identical windows broadcast).
  int aoff[2];
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    int st = 16 * w + 8 * h - r + 31;
    st = (st < 24 || st > 35) ? 36 : st;
    aoff[w] = 32 * (st & 7) + 2 * (st - (st & 7) - 24);
  }
  const int boff = r * RP + 16 * h;

  const int64_t plane_o = (int64_t)a.ho * a.wo;
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<bf16*>(a.d) + (int64_t)n * a.hid * plane_o, 0, (int)(2 * a.hid * plane_o), 0x00020000);
  constexpr unsigned kDrop = 0x80000000u;
  // output geometry of this lane in the depthwise C layout: row y0 + r, columns 28 s + 8 q + 4 h + 0..3
  const int oy = y0 + r;
  const bool rowv = oy < a.ho;
  const bool edge = s * OW + OW > a.wo;  // last strip: columns past the right border
  const int hid16 = (a.hid + 15) / 16 * 16;
  // the chunk parameters through buffer descriptors: channels past hid (hid16 for the expand rows) read
  // as 0 without a branch, so every chunk issues the same loads
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w1), 0,
                                                                       2 * hid16 * a.cin_pad, 0x00020000);
  const __amdgpu_buffer_rsrc_t b1r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.b1), 0, 4 * a.hid, 0x00020000);
  const __amdgpu_buffer_rsrc_t wdr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.wdw), 0, 100 * a.hid, 0x00020000);
  const __amdgpu_buffer_rsrc_t bdr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.bdw), 0, 4 * a.hid, 0x00020000);
  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
      a.pool + (int64_t)n * a.hid * a.slots, 0, 4 * a.hid * a.slots, 0x00020000);
  const int it1 = min(tid + 64 * NW, NCH * 25 - 1);  // second Toeplitz item of this thread (if < 800)
  // Parameters of chunk cb, loaded one chunk ahead: issued before the current chunk's D stores, so
  // waiting for them never waits for those stores (vmcnt counts loads and stores in issue order)
  struct ChunkW {
    bf16x8 bw[KS];
    float b1, wt0, wt1, bd[4];
  };
  auto load_chunk = [&](int cb, ChunkW& cw) {
    const int ch = cb * NCH + r;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
      const u32x4v v = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(w1r, 2 * (ch * a.cin_pad + 16 * q + 8 * h), 0, 0));
      cw.bw[q] = __builtin_bit_cast(bf16x8, v);
    }
    cw.b1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b1r, 4 * ch, 0, 0));
    cw.wt0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           wdr, 4 * (cb * NCH * 25 + tid), 0, 0));
    cw.wt1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           wdr, 4 * (cb * NCH * 25 + it1), 0, 0));
#pragma unroll
    for (int u = 0; u < 4; ++u)
      cw.bd[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bdr, 4 * (cb * NCH + wv * 4 + u), 0, 0));
  };
  auto write_t = [&](int it, float v) {  // weight (ky, kx) of a channel into its 8 copies: copy k entry 7 + kx - k
    const int c = it / 25, t = it - 25 * c, ky = t / 5, kx = t - 5 * ky;
    const unsigned short b = bits16(v);
    unsigned short* row = reinterpret_cast<unsigned short*>(Ts + c * TP + ky * 256) + 7 + kx;
#pragma unroll
    for (int k = 0; k < 8; ++k) row[16 * k - k] = b;
  };
  ChunkW cur;
  load_chunk(0, cur);
  // wait for every load before the loop: otherwise the wait-count analysis merges the loop entry (loads
  // pending) with the back edge (only the previous chunk's stores pending) and makes the first use of a
  // parameter in every chunk wait for all of those stores
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  lds_barrier();
  for (int cb = 0; cb < ncb; ++cb) {
    // ---- this chunk's depthwise weights into the Toeplitz rows (items = channel * 25 + tap)
    write_t(tid, cur.wt0);
    if (tid + 64 * NW < NCH * 25) write_t(tid + 64 * NW, cur.wt1);
    // ---- expand: rows j = wv + 8 t, 32 channels, C[pixel][channel]; every row's MFMAs first, then
    // the activations (a row's three MFMAs are a dependent chain: done row by row, the wave waited on
    // each chain before the row's VALU work)
    f32x16 ce[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (wv + NW * t < IR) {
#pragma unroll
        for (int i = 0; i < 16; ++i) ce[t][i] = cur.b1;
#pragma unroll
        for (int q = 0; q < KS; ++q)
          if (!(ED5_SKIP & 4)) ce[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[t][q], cur.bw[q], ce[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int j = wv + NW * t;
      if (j < IR) {
        unsigned pk[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) pk[i] = pack2(hswish5(ce[t][2 * i]), hswish5(ce[t][2 * i + 1]));
        uint4* dst = reinterpret_cast<uint4*>(Hs + r * CP + j * RP + 32 * h);
        if (!(ED5_SKIP & 16)) {
          dst[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          dst[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        } else if (pk[0] == 0x12345678u) {
          dst[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
      }
    }
    lds_barrier();
    ChunkW nxt;
    load_chunk(cb + 1, nxt);  // past the last chunk every read is out of range (0), never used
    // ---- depthwise: channels wv * 4 + u of the chunk
    float psum[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = wv * 4 + u, ch = cb * NCH + c;
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = cur.bd[u];
      const unsigned char* tb = Ts + c * TP;
      const unsigned char* hb = Hs + c * CP + boff;
#pragma unroll
      for (int ky = 0; ky < K5; ++ky) {
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          if (ED5_SKIP & 2) continue;
          const u32x4 af = (ED5_SKIP & 8) ? u32x4{(unsigned)aoff[w], 0u, 1u, 2u}
                                          : *reinterpret_cast<const u32x4*>(tb + ky * 256 + aoff[w]);
          const u32x4 bf = *reinterpret_cast<const u32x4*>(hb + ky * RP + 32 * w);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af), __builtin_bit_cast(bf16x8, bf),
                                                        acc, 0, 0, 0);
        }
      }
      // epilogue: lane (row r, half h), registers 4 q + e = column 8 q + 4 h + e
      float y[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) y[i] = hswish5(acc[i]);
      float t = 0.f;
      if (!edge) {
#pragma unroll
        for (int i = 0; i < 12; ++i) t += y[i];
        if (h == 0) t += (y[12] + y[13]) + (y[14] + y[15]);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = 8 * (i >> 2) + 4 * h + (i & 3);
          t += (m < OW && s * OW + m < a.wo) ? y[i] : 0.f;
        }
      }
      psum[u] = rowv ? t : 0.f;
      // D through this channel's own hidden image (only this wave reads it, and its reads of it are
      // done: LDS operations of a wave complete in order): staged as [row][28 columns] bf16 (56-byte
      // rows, conflict-free 8-byte writes), read back so that 7 consecutive lanes cover one row, so an
      // 8-byte store instruction writes ~9 whole 56-byte row runs instead of 16 bytes in each of 32 rows
      // (the direct form was bound by the store path: ~32 cycles per instruction)
      unsigned char* stg = Hs + c * CP;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q < 3 || h == 0)
          *reinterpret_cast<u32x2*>(stg + r * 56 + (2 * q + h) * 8) =
              u32x2{pack2(y[4 * q], y[4 * q + 1]), pack2(y[4 * q + 2], y[4 * q + 3])};
      }
      const bool chv = ch < a.hid;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = lane + 64 * k, row = i / 7, pc7 = i - 7 * row, col = s * OW + 4 * pc7;
        const u32x2 v = *reinterpret_cast<const u32x2*>(stg + 8 * min(i, 223));
        const bool ok = chv && i < 224 && y0 + row < a.ho && col + 4 <= a.wo;
        const unsigned off = ok ? (unsigned)(2 * ((int64_t)ch * plane_o + (int64_t)(y0 + row) * a.wo + col)) : kDrop;
        if (!(ED5_SKIP & 1)) __builtin_amdgcn_raw_buffer_store_b64(v, dr, (int)off, 0, 0);
        else if (v[0] == 0x12345678u) __builtin_amdgcn_raw_buffer_store_b64(v, dr, (int)off, 0, 0);
      }
    }
    // SE-pool partial sums of the wave's 4 channels over the tile (one slot per tile, plain stores;
    // lanes other than 0 and padding channels store out of range)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v = psum[u];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      const int ch = cb * NCH + wv * 4 + u;
      const unsigned off = lane == 0 && ch < a.hid ? (unsigned)(4 * (ch * a.slots + band * strips + s)) : kDrop;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), pr, (int)off, 0, 0);
    }
    lds_barrier();  // the next chunk rewrites the hidden image and the Toeplitz weights
    cur = nxt;
  }
}

template <int KS>
int launch_ks5(EdArgs a, hipStream_t st) {
  const int strips = (a.wo + OW - 1) / OW, bands = (a.ho + TH - 1) / TH, ncb = (a.hid + NCH - 1) / NCH;
  const int64_t total = (int64_t)strips * bands * a.n;
  if (total > 0x7ffffff0LL) return AST_E_SHAPE;
  if (ed_plan(a, (int64_t)bands * strips)) return 0;
  const int64_t grid = (total + 7) / 8 * 8;
  hipLaunchKernelGGL((expand_dw5_kernel<KS>), dim3((unsigned)grid), dim3(64 * NW), 0, st, a, strips, bands, ncb,
                     (int)total);
  return (int)hipGetLastError();
}

}  // namespace

int launch_ed5(EdArgs a, int k, int stride, hipStream_t st) {
  // bf16 expand blocks, k 5, stride 1, no upsample, cin <= 48, 8-byte D pieces (wo % 4 == 0), and
  // at least one whole tile of rows / columns (the reflection of the tile's halo stays in the image)
  if (!a.w1 || k != 5 || stride != 1 || a.nod || a.c1 != a.cin || a.hd != a.h || a.wd != a.w) return AST_E_UNSUPPORTED;
  if (a.cin_pad % 16 != 0 || a.cin_pad > 48 || a.wo % 4 != 0 || a.ho < 3 || a.wo < 3) return AST_E_UNSUPPORTED;
  if ((int64_t)a.cin_pad * 2 * a.h * a.w >= 0x7fffffffLL || (int64_t)a.hid * 2 * a.ho * a.wo >= 0x7fffffffLL)
    return AST_E_UNSUPPORTED;
  switch (a.cin_pad / 16) {
    case 1: return launch_ks5<1>(a, st);
    case 2: return launch_ks5<2>(a, st);
    case 3: return launch_ks5<3>(a, st);
    default: return AST_E_UNSUPPORTED;
  }
}

}  // namespace ast_mb
