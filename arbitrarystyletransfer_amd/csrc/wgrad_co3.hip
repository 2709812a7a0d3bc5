// Weight gradient of a 3x3 conv with Cout <= 3 on v_mfma_f32_32x32x16_bf16 in split-bf16
// (fp32-accurate) arithmetic, for gfx950 (round 6) -- the decoder's image conv (64 -> 3,
// models.py:598-628, trained by train.py:191-300) and the other image-output convs.
//
// dW[co][ci][ky][kx] = sum_p dy[co][p] xpad[ci][p + (ky-1, kx-1)]. As a GEMM over output pixels the
// N side would be Cout = 3 of a 32-wide tile; substituting q = p + tap puts the taps there instead:
//   dW[ci][(co, ky, kx)] = sum_q xpad[ci][q] * dy[co][q - (ky-1, kx-1)],
// M = input channels (2 x 32 per workgroup), N = 27 of 32, K = positions q of the padded grid.
//  * A = xpad rows, loaded straight from HBM (8 consecutive q per lane: two 16-byte loads; the
//    padded rows -1 and H are the reflect / replicate source rows), split into three bf16 terms in
//    registers (ast_x3::split8);
//  * B = dy, staged per q tile (4 padded rows x 64 columns) in LDS as three term planes, one copy
//    per (co, kx) shifted by kx so that every lane's 8 consecutive q are one aligned ds_read_b128;
//  * the six largest term products, smallest first; a workgroup walks a contiguous range of q tiles
//    with its accumulators in registers and writes one partial dW (and db) slot, summed in slot
//    order by the caller (det.h reduce_cols): bitwise reproducible.
// The two padded border COLUMNS (q x = -1, W; non-zero under reflect / upsample padding) touch only
// taps kx = 0 and 2 and are a small VALU pass (wgrad_co3_border_kernel) into WGCO3_BORDER_SLOTS more slots.
// The VALU kernel this replaces (wgrad_smallco_kernel, 27 fp32 FMAs per input value) took 0.83 ms
// on the config-3 decoder's 8 x 64 x 512^2 -> 3 conv (profiles/r06y_kernel_stats_train.txt).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "x3.h"
#include "wgco3.h"

namespace {

using ast_x3::bf16;
using ast_x3::bf16x8;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;                      // 4 waves: wave w takes padded row y0 + w of a q tile
constexpr int TQH = WGCO3_TQH, TQW = WGCO3_TQW;
constexpr int DR = TQH + 2;                  // dy rows of a q tile
constexpr int DC = TQW + 8;                  // LDS row stride (bf16)
constexpr int NCP = 9;                       // shifted copies: (co, kx)
constexpr int ZROW = NCP * DR;               // a zero row (lanes n >= 27 or co >= Cout)
constexpr int TPL = (ZROW + 1) * DC;         // one term plane
constexpr int DEL = NCP * DR * TQW;          // staged elements per q tile
constexpr int D_T = (DEL + NT - 1) / NT;

// source index (upsampled grid) of padded coordinate g in [-1, n]; -1 = zero padding
template <int UP>
__device__ __forceinline__ int src_pad(int g, int n, int reflect) {
  if (g >= 0 && g < n) return g;
  if (!reflect) return -1;
  if (UP == 2) return g < 0 ? 0 : n - 1;  // reflect of the upsampled grid = replicate of the source
  const int r = g < 0 ? -g : 2 * (n - 1) - g;
  return r < 0 ? 0 : (r >= n ? n - 1 : r);
}

__device__ __forceinline__ unsigned short bits(bf16 v) { return __builtin_bit_cast(unsigned short, v); }

template <int UP>
__global__ __launch_bounds__(NT, 2) void wgrad_co3_kernel(WgCo3Args a) {
  __shared__ __attribute__((aligned(16))) unsigned short Ds[2][3][TPL];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, l32 = lane & 31, kh = lane >> 5;
  const int H = a.Hin * UP, W = a.Win * UP;
  const int cgi = blockIdx.x % a.cgroups;
  const int64_t split = blockIdx.x / a.cgroups;
  const int ci0 = cgi * 64;
  const int64_t t0 = split * a.tiles_per_block, t1 = min(a.ntiles, t0 + a.tiles_per_block);
  for (int c = tid; c < DC; c += NT)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int t = 0; t < 3; ++t) Ds[b][t][ZROW * DC + c] = 0;

  // the lane's N column: (co, ky, kx) = n / 9, n % 9 / 3, n % 3; its B row for this wave's q row is
  // r = w - ky + 2 of copy (co, kx)
  const int co_n = l32 / 9, ky_n = l32 % 9 / 3, kx_n = l32 % 3;
  const bool nv = l32 < 27 && co_n < a.Cout;
  const int boff = (nv ? ((co_n * 3 + kx_n) * DR + wv - ky_n + 2) * DC : ZROW * DC) + 8 * kh;

  f32x16 acc[2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[mb][v] = 0.f;
  float dbs[3] = {0.f, 0.f, 0.f};

  int buf = 0;
  for (int64_t tile = t0; tile < t1; ++tile) {
    int64_t tt = tile;
    const int tx = (int)(tt % a.tiles_x);
    tt /= a.tiles_x;
    const int ty = (int)(tt % a.tiles_y);
    const int n = (int)(tt / a.tiles_y);
    const int y0 = ty * TQH - 1, x0 = tx * TQW;  // q tile: padded rows y0.., interior columns x0..
    const float* __restrict__ dyn = a.dy + (int64_t)n * a.Cout * a.dy_plane + a.dy_off;

    // dy tile: element (copy (co, kx), r, c) = dy[co][y0 - 1 + r][x0 + c - kx + 1], 0 outside
    float dv[D_T];
#pragma unroll
    for (int i = 0; i < D_T; ++i) {
      const int e = min(tid + i * NT, DEL - 1);
      const int c = e % TQW, rest = e / TQW, r = rest % DR, cp = rest / DR, co = cp / 3, kx = cp % 3;
      const int yy = y0 - 1 + r, xx = x0 + c - kx + 1;
      const bool ok = co < a.Cout && yy >= 0 && yy < H && xx >= 0 && xx < W;
      dv[i] = ok ? dyn[(int64_t)co * a.dy_plane + (int64_t)yy * a.dy_pitch + xx] : 0.f;
    }
    // A: this wave's padded row, 4 K-steps of 16 q, 2 x 32 input channels
    const int qy = y0 + wv;
    const int sr = qy <= H ? src_pad<UP>(qy, H, a.reflect) : -1;
    float xa[4][2][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qx = x0 + 16 * j + 8 * kh;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        const int ci = ci0 + 32 * mb + l32;
        const bool ok = sr >= 0 && ci < a.Cin && x0 + 16 * j < W;  // W % 16 == 0: a K-step is all in or out
        const float* row = a.x + (((int64_t)n * a.Cin + (ok ? ci : 0)) * a.Hin + (ok ? sr / UP : 0)) * a.Win;
        if (UP == 1) {
          const float4 u = ok ? *reinterpret_cast<const float4*>(row + qx) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 w = ok ? *reinterpret_cast<const float4*>(row + qx + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
          xa[j][mb][0] = u.x; xa[j][mb][1] = u.y; xa[j][mb][2] = u.z; xa[j][mb][3] = u.w;
          xa[j][mb][4] = w.x; xa[j][mb][5] = w.y; xa[j][mb][6] = w.z; xa[j][mb][7] = w.w;
        } else {  // nearest x2: source columns qx/2 .. qx/2 + 3, each twice
          const float4 u = ok ? *reinterpret_cast<const float4*>(row + qx / 2) : make_float4(0.f, 0.f, 0.f, 0.f);
          xa[j][mb][0] = xa[j][mb][1] = u.x; xa[j][mb][2] = xa[j][mb][3] = u.y;
          xa[j][mb][4] = xa[j][mb][5] = u.z; xa[j][mb][6] = xa[j][mb][7] = u.w;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < D_T; ++i) {
      const int e = tid + i * NT;
      if (e < DEL) {
        const int c = e % TQW, rest = e / TQW, r = rest % DR, cp = rest / DR;
        bf16 h, md, lo;
        ast_x3::split3(dv[i], h, md, lo);
        const int o = (cp * DR + r) * DC + c;
        Ds[buf][0][o] = bits(h);
        Ds[buf][1][o] = bits(md);
        Ds[buf][2][o] = bits(lo);
        // db: the dy pixels this q tile owns (rows y0..y0+TQH-1, columns x0..x0+TQW-1), once each
        const int co = cp / 3;
        if (cp % 3 == 1 && r >= 1 && r <= TQH) {
          if (co == 0) dbs[0] += dv[i];
          else if (co == 1) dbs[1] += dv[i];
          else dbs[2] += dv[i];
        }
      }
    }
    __syncthreads();  // Ds[buf] complete; Ds[buf ^ 1] was last read before this barrier
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (x0 + 16 * j >= W) break;
      bf16x8 at[2][3];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) ast_x3::split8(xa[j][mb], at[mb][0], at[mb][1], at[mb][2]);
      bf16x8 bt[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) bt[t] = *reinterpret_cast<const bf16x8*>(&Ds[buf][t][boff + 16 * j]);
      // the six largest term products (x_t . dy_u, t + u <= 2), smallest first
      constexpr int TA[6] = {2, 0, 1, 1, 0, 0}, TB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
      for (int p = 0; p < 6; ++p)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          acc[mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(at[mb][TA[p]], bt[TB[p]], acc[mb], 0, 0, 0);
    }
    buf ^= 1;
  }

  // the four waves' accumulators through LDS (the dy planes are no longer read), summed in wave order
  __syncthreads();
  float* red = reinterpret_cast<float*>(&Ds[0][0][0]);  // [wave][mb * 16 + v][lane]: 32 KB
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int v = 0; v < 16; ++v) red[(wv * 32 + mb * 16 + v) * 64 + lane] = acc[mb][v];
  // db over the workgroup: wave shuffles, then the waves in order (after the dW entries)
  float* redb = red + 4 * 32 * 64;
#pragma unroll
  for (int co = 0; co < 3; ++co) {
    float s = dbs[co];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
    if (lane == 0) redb[wv * 3 + co] = s;
  }
  __syncthreads();
  const int64_t wcount = (int64_t)a.Cout * a.Cin * 9;
  for (int i = tid; i < 32 * 64; i += NT) {
    const int ln = i % 64, mv = i / 64, mb = mv / 16, v = mv % 16;
    const int n_ = ln & 31;
    const int ci = ci0 + 32 * mb + 8 * (v >> 2) + 4 * (ln >> 5) + (v & 3);
    const int co = n_ / 9, tap = n_ % 9;
    if (n_ < 27 && co < a.Cout && ci < a.Cin) {
      const float s = (red[(0 * 32 + mv) * 64 + ln] + red[(1 * 32 + mv) * 64 + ln]) +
                      (red[(2 * 32 + mv) * 64 + ln] + red[(3 * 32 + mv) * 64 + ln]);
      a.dw[split * wcount + ((int64_t)co * a.Cin + ci) * 9 + tap] = s;
    }
  }
  if (a.db && cgi == 0 && tid < a.Cout)
    a.db[split * a.Cout + tid] = (redb[0 * 3 + tid] + redb[1 * 3 + tid]) + (redb[2 * 3 + tid] + redb[3 * 3 + tid]);
}

// The padded border columns q x = -1 and W (reflect / upsample padding): only taps kx = 0 (dy
// column 0) and kx = 2 (dy column W-1) see them. A workgroup sums its channel over its range of
// (image, padded row) and writes its slot's entries for that channel (kx = 1 entries zero).
// Grid (Cin, WGCO3_BORDER_SLOTS): workgroup (ci, b) sums the b-th range of (image, padded row) pairs
// into slot splits + b. (One workgroup per channel left 192 CUs idle and took 76 us against the main
// kernel's 185 on 8 x 64 x 512^2: the dy reads, repeated per channel, are scattered dwords.)
constexpr int NTB = 256;

template <int UP>
__global__ __launch_bounds__(NTB) void wgrad_co3_border_kernel(WgCo3Args a) {
  __shared__ float red[NTB / 64][18];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int ci = blockIdx.x, b = blockIdx.y;
  const int H = a.Hin * UP, W = a.Win * UP;
  const int cl = src_pad<UP>(-1, W, a.reflect) / UP, cr = src_pad<UP>(W, W, a.reflect) / UP;
  float s[2][3][3];  // [side][co][ky]
#pragma unroll
  for (int sd = 0; sd < 2; ++sd)
#pragma unroll
    for (int co = 0; co < 3; ++co)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) s[sd][co][ky] = 0.f;
  const int64_t rows = (int64_t)a.N * (H + 2);
  const int64_t per = (rows + WGCO3_BORDER_SLOTS - 1) / WGCO3_BORDER_SLOTS;
  const int64_t r1 = min(rows, (b + 1) * per);
#pragma unroll 2
  for (int64_t i = b * per + tid; i < r1; i += NTB) {
    const int n = (int)(i / (H + 2)), qy = (int)(i % (H + 2)) - 1;
    const int sr = src_pad<UP>(qy, H, a.reflect);
    if (sr < 0) continue;
    const float* row = a.x + (((int64_t)n * a.Cin + ci) * a.Hin + sr / UP) * a.Win;
    const float xl = row[cl], xr = row[cr];
    const float* dyn = a.dy + (int64_t)n * a.Cout * a.dy_plane + a.dy_off;
#pragma unroll
    for (int co = 0; co < 3; ++co) {
      if (co >= a.Cout) break;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int yy = qy - ky + 1;
        if (yy < 0 || yy >= H) continue;
        const float* d = dyn + (int64_t)co * a.dy_plane + (int64_t)yy * a.dy_pitch;
        s[0][co][ky] = fmaf(xl, d[0], s[0][co][ky]);
        s[1][co][ky] = fmaf(xr, d[W - 1], s[1][co][ky]);
      }
    }
  }
#pragma unroll
  for (int sd = 0; sd < 2; ++sd)
#pragma unroll
    for (int co = 0; co < 3; ++co)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        float v = s[sd][co][ky];
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) red[wv][(sd * 3 + co) * 3 + ky] = v;
      }
  __syncthreads();
  const int64_t wcount = (int64_t)a.Cout * a.Cin * 9;
  if (tid < a.Cout * 9) {
    const int co = tid / 9, tap = tid % 9, ky = tap / 3, kx = tap % 3;
    float v = 0.f;
    if (kx != 1) {
      const int k = ((kx == 0 ? 0 : 1) * 3 + co) * 3 + ky;
#pragma unroll
      for (int w = 0; w < NTB / 64; ++w) v += red[w][k];
    }
    a.dw[(a.splits + b) * wcount + ((int64_t)co * a.Cin + ci) * 9 + tap] = v;
  }
  if (a.db && ci == 0 && tid < a.Cout) a.db[(a.splits + b) * a.Cout + tid] = 0.f;
}

}  // namespace

bool wgrad_co3_supported(int cin, int h_in, int w_in, int cout, int up) {
  const int W = w_in * up;
  return cout >= 1 && cout <= 3 && cin >= 1 && (W % 16) == 0 && h_in >= 1 && (up == 1 || up == 2);
}

int launch_wgrad_co3(const WgCo3Args& a, hipStream_t s) {
  const int64_t nblk = a.splits * a.cgroups;
  if (nblk <= 0 || nblk >= 0x7fffffff) return AST_E_SHAPE;
  if (a.up == 2) hipLaunchKernelGGL(wgrad_co3_kernel<2>, dim3((unsigned)nblk), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(wgrad_co3_kernel<1>, dim3((unsigned)nblk), dim3(NT), 0, s, a);
  if (a.reflect) {  // zero padding: the border columns are zero and the slot does not exist
    if (a.up == 2) hipLaunchKernelGGL(wgrad_co3_border_kernel<2>, dim3((unsigned)a.Cin, WGCO3_BORDER_SLOTS), dim3(NTB), 0, s, a);
    else hipLaunchKernelGGL(wgrad_co3_border_kernel<1>, dim3((unsigned)a.Cin, WGCO3_BORDER_SLOTS), dim3(NTB), 0, s, a);
  }
  return (int)hipGetLastError();
}
