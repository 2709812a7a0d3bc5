// Backward of the 3x3 conv blocks for gfx950 (training step).
//
// Input gradient ("dgrad"): the forward MFMA kernel run on a transposed+flipped weight pack
// (ast_conv3x3_pack_weights_ex_f32).
//  * Zero-padded convs (VGG encoder / loss network): dX = conv3x3_same(dY, W') directly.
//  * Decoder [Upsample] + ReflectionPad + Conv: the ReLU-masked output gradient is written into a
//    zero-padded buffer (pad_grad_kernel), so one "same" conv over it yields the FULL gradient of
//    the reflect-padded input, borders included; the reflect-pad / nearest-upsample adjoint then
//    folds it onto the source grid (pad_up_adjoint_full_kernel).
//
// Weight gradient ("wgrad"): dW[co][ci][tap] = sum_pix dY[co][pix] * P[ci][pix+tap] as an MFMA
// fp32 GEMM with K = pixels. A workgroup (4 waves) owns 64 output x 64 input channels x 9 taps;
// each wave 32 x 32 x 9 taps in 9 accumulators. Per 2x32-pixel tile it stages the input halo tile
// (same source-tile staging as the forward kernel: zero/reflect pad and upsample resolved by the
// LDS read address, so the 9 taps are constant offsets) and the dY tile; a workgroup sweeps a
// range of tiles and adds its partial dW with fp32 atomics (the pixel range is split across
// workgroups). dY may be read from the padded gradient buffer (pitch/plane/offset).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../include/ast_hip.h"
#include "x3.h"
#include "wgco3.h"
#include "det.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float relu_f(float v) { return v < 0.f ? 0.f : v; }

template <int UP>
__device__ __forceinline__ int src_index(int g, int n, int reflect) {
  if (g >= 0 && g < n) return g;
  if (!reflect) return -1;
  if (UP == 2) return g < 0 ? 0 : n - 1;
  int r = g < 0 ? -g : 2 * (n - 1) - g;
  return r < 0 ? 0 : (r >= n ? n - 1 : r);
}

// wp[ci_pad][9][co_pad] layout of the forward pack, but for the transposed+flipped filter:
// W'[o=ci][i=co][ky][kx] = W[co][ci][2-ky][2-kx] / (scale ? scale[ci] : 1)
__global__ void pack_tf_kernel(const float* __restrict__ w, float* __restrict__ wp, int cout, int cin, int pad_out,
                               int pad_in, const float* __restrict__ scale) {
  const int64_t total = (int64_t)pad_in * 9 * pad_out;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(idx % pad_out);  // ci of the original
    const int64_t rt = idx / pad_out;
    const int tap = (int)(rt % 9);
    const int i = (int)(rt / 9);         // co of the original
    float v = 0.f;
    if (o < cin && i < cout) {
      v = w[((int64_t)i * cin + o) * 9 + (8 - tap)];
      if (scale) v = v / scale[o];
    }
    wp[idx] = v;
  }
}

// dy = g_pre + (pre > 0) * (g_act + unpool(g_pool)): backward of y_pre -> ReLU -> MaxPool2x2.
// unpool routes each pooled gradient to the first maximal element of its 2x2 window (row-major),
// as PyTorch's max_pool2d does; the last NaN of a window wins it.
__global__ void act_backward_kernel(const float* __restrict__ pre, const float* __restrict__ g_pre,
                                    const float* __restrict__ g_act, const float* __restrict__ g_pool,
                                    float* __restrict__ dy, int64_t planes, int H, int W) {
  const int Ho = H >> 1, Wo = W >> 1;
  const int64_t n = planes * H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    const int y = (int)((i / W) % H);
    const int64_t p = i / ((int64_t)H * W);
    const float v = pre[i];
    float g = g_pre ? g_pre[i] : 0.f;
    if (v > 0.f) {
      float a = g_act ? g_act[i] : 0.f;
      if (g_pool) {
        const int py = y >> 1, px = x >> 1;
        if (py < Ho && px < Wo) {
          const float* base = pre + p * H * W + (int64_t)(2 * py) * W + 2 * px;
          const float c[4] = {relu_f(base[0]), relu_f(base[1]), relu_f(base[W]), relu_f(base[W + 1])};
          int best = 0;
#pragma unroll
          for (int q = 1; q < 4; ++q)
            if (c[q] > c[best] || c[q] != c[q]) best = q;  // torch: val > max || isnan(val)
          const int mine = (y & 1) * 2 + (x & 1);
          if (best == mine) a += g_pool[p * Ho * Wo + (int64_t)py * Wo + px];
        }
      }
      g += a;
    }
    dy[i] = g;
  }
}

// out_pad [planes, H+2, Wp] = zero-padded (mask > 0 ? g : 0) (mask optional): the output gradient
// laid out so that a zero-padded "same" conv with the transposed+flipped filter produces the
// FULL gradient of the reflect-padded input, borders included.
__global__ void pad_grad_kernel(const float* __restrict__ g, const float* __restrict__ mask, float* __restrict__ out,
                                int64_t planes, int H, int W, int Wp) {
  const int64_t n = planes * (H + 2) * Wp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Wp);
    const int r = (int)((i / Wp) % (H + 2));
    const int64_t p = i / ((int64_t)(H + 2) * Wp);
    float v = 0.f;
    if (r >= 1 && r <= H && c >= 1 && c <= W) {
      const int64_t s = (p * H + (r - 1)) * W + (c - 1);
      v = g[s];
      if (mask && !(mask[s] > 0.f)) v = 0.f;
    }
    out[i] = v;
  }
}

// dx[v] = sum of the full padded-input gradient dP [planes, H+2, Wp] over the padded positions
// that the reflect pad (and nearest upsample) map onto source pixel v:
//   up == 1: p -> refl(p-1) = v;   up == 2: p -> refl(p-1) -> v = u >> 1 (refl on the 2x grid).
__global__ void pad_up_adjoint_full_kernel(const float* __restrict__ dp, float* __restrict__ dx, int64_t planes,
                                           int h_in, int w_in, int up, int Wp) {
  const int H = h_in * up, W = w_in * up;
  const int64_t total = planes * h_in * w_in;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int vx = (int)(idx % w_in);
    const int vy = (int)((idx / w_in) % h_in);
    const int64_t p = idx / ((int64_t)h_in * w_in);
    int rows[4], nr = 0, cols[4], nc = 0;
    for (int k = 0; k < up; ++k) {
      rows[nr++] = up * vy + k + 1;
      cols[nc++] = up * vx + k + 1;
    }
    if (up == 1) {
      if (vy == 1) rows[nr++] = 0;
      if (vy == H - 2) rows[nr++] = H + 1;
      if (vx == 1) cols[nc++] = 0;
      if (vx == W - 2) cols[nc++] = W + 1;
    } else {
      if (vy == 0) rows[nr++] = 0;
      if (vy == h_in - 1) rows[nr++] = H + 1;
      if (vx == 0) cols[nc++] = 0;
      if (vx == w_in - 1) cols[nc++] = W + 1;
    }
    const float* d = dp + p * (int64_t)(H + 2) * Wp;
    float s = 0.f;
    for (int a = 0; a < nr; ++a)
      for (int b = 0; b < nc; ++b) s += d[(int64_t)rows[a] * Wp + cols[b]];
    dx[idx] = s;
  }
}

// Row-parallel forms of the three kernels above (the defaults where the row width allows): a thread
// owns 4 consecutive columns of one (plane, row) with 16-byte loads/stores where aligned, and the
// index math is one 32-bit division per 4 outputs -- the flat forms spent their time in 64-bit
// div/mod per element (config 3: ~10 ms per step over 32 launches, HBM-bound work of ~5).
__global__ __launch_bounds__(256) void act_backward_v4_kernel(const float* __restrict__ pre,
                                                              const float* __restrict__ g_pre,
                                                              const float* __restrict__ g_act,
                                                              const float* __restrict__ g_pool,
                                                              float* __restrict__ dy, unsigned nq, int H, int W) {
  const unsigned q = (unsigned)W >> 2;  // quads per row (W % 4 == 0)
  const int Ho = H >> 1, Wo = W >> 1;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < nq; t += gridDim.x * blockDim.x) {
    const unsigned row = t / q, x0 = 4 * (t - row * q);
    const unsigned p = row / (unsigned)H;
    const int y = (int)(row - p * (unsigned)H);
    const int64_t off = (int64_t)row * W + x0;
    const float4 v4 = *reinterpret_cast<const float4*>(pre + off);
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    float g[4] = {0.f, 0.f, 0.f, 0.f}, a[4] = {0.f, 0.f, 0.f, 0.f};
    if (g_pre) {
      const float4 u = *reinterpret_cast<const float4*>(g_pre + off);
      g[0] = u.x; g[1] = u.y; g[2] = u.z; g[3] = u.w;
    }
    if (g_act) {
      const float4 u = *reinterpret_cast<const float4*>(g_act + off);
      a[0] = u.x; a[1] = u.y; a[2] = u.z; a[3] = u.w;
    }
    const int py = y >> 1;
    if (g_pool && py < Ho) {
      // the 2x2 windows (py, x0/2) and (py, x0/2 + 1): this row and its partner row
      const int64_t top = ((int64_t)p * H + 2 * py) * W + x0;
      const float4 r0 = *reinterpret_cast<const float4*>(pre + top);
      const float4 r1 = *reinterpret_cast<const float4*>(pre + top + W);
      const float c0[4] = {r0.x, r0.y, r0.z, r0.w}, c1[4] = {r1.x, r1.y, r1.z, r1.w};
      const float2 gp = *reinterpret_cast<const float2*>(g_pool + ((int64_t)p * Ho + py) * Wo + (x0 >> 1));
      const float gpw[2] = {gp.x, gp.y};
#pragma unroll
      for (int w2 = 0; w2 < 2; ++w2) {
        const int px = (int)(x0 >> 1) + w2;
        if (px >= Wo) continue;
        const float c[4] = {relu_f(c0[2 * w2]), relu_f(c0[2 * w2 + 1]), relu_f(c1[2 * w2]), relu_f(c1[2 * w2 + 1])};
        int best = 0;
#pragma unroll
        for (int qq = 1; qq < 4; ++qq)
          if (c[qq] > c[best] || c[qq] != c[qq]) best = qq;  // torch: val > max || isnan(val)
        if ((best >> 1) == (y & 1)) a[2 * w2 + (best & 1)] += gpw[w2];
      }
    }
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j] > 0.f ? g[j] + a[j] : g[j];
    *reinterpret_cast<float4*>(dy + off) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// out[r][c] = g[r-1][c-1]: output quad q holds input columns 4q-1 .. 4q+2 = (quad q-1).w, (quad
// q).xyz -- two aligned 16-byte loads (the neighbour thread's quad comes from L1/L2), W % 4 == 0
__global__ __launch_bounds__(256) void pad_grad_v4_kernel(const float* __restrict__ g, const float* __restrict__ mask,
                                                          float* __restrict__ out, unsigned nq, int H, int W, int Wp) {
  const unsigned q = (unsigned)Wp >> 2;  // Wp % 4 == 0
  const int wq = W >> 2;                 // input quads per row
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < nq; t += gridDim.x * blockDim.x) {
    const unsigned orow = t / q;
    const int oq = (int)(t - orow * q), c0 = 4 * oq;
    const unsigned p = orow / (unsigned)(H + 2);
    const int r = (int)(orow - p * (unsigned)(H + 2));
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    if (r >= 1 && r <= H) {
      const float* grow = g + ((int64_t)p * H + (r - 1)) * W;
      const float* mrow = mask ? mask + ((int64_t)p * H + (r - 1)) * W : nullptr;
      float in[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // input columns c0 - 4 + 3 .. c0 + 3: in[j] = column c0 - 1 + j
      float mk[5] = {1.f, 1.f, 1.f, 1.f, 1.f};
      if (oq >= 1 && oq - 1 < wq) {
        in[0] = grow[c0 - 1];
        if (mrow) mk[0] = mrow[c0 - 1];
      }
      if (oq < wq) {
        const float4 v = *reinterpret_cast<const float4*>(grow + c0);
        in[1] = v.x; in[2] = v.y; in[3] = v.z; in[4] = v.w;
        if (mrow) {
          const float4 m = *reinterpret_cast<const float4*>(mrow + c0);
          mk[1] = m.x; mk[2] = m.y; mk[3] = m.z; mk[4] = m.w;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c >= 1 && c <= W) o[j] = (mrow && !(mk[j] > 0.f)) ? 0.f : in[j];
      }
    }
    *reinterpret_cast<float4*>(out + (int64_t)orow * Wp + c0) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// (same sums and summation order as pad_up_adjoint_full_kernel). A row's main columns come from
// aligned 16-byte loads: UP = 1, columns vx0 + 1 .. vx0 + 4 from the two quads at vx0; UP = 2,
// columns 2 vx0 + 1 .. 2 vx0 + 8 from the three quads at 2 vx0 (host: Wp % 4 == 0, Wp >= W + 4).
template <int UP>
__global__ __launch_bounds__(256) void pad_up_adjoint_v4_kernel(const float* __restrict__ dp, float* __restrict__ dx,
                                                                unsigned nq, int h_in, int w_in, int Wp) {
  constexpr int NW = UP == 1 ? 8 : 12;  // window of loaded columns
  const int H = h_in * UP, W = w_in * UP;
  const unsigned q = (unsigned)w_in >> 2;  // w_in % 4 == 0
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < nq; t += gridDim.x * blockDim.x) {
    const unsigned row = t / q;
    const int vx0 = 4 * (int)(t - row * q);
    const unsigned p = row / (unsigned)h_in;
    const int vy = (int)(row - p * (unsigned)h_in);
    int rows[4], nr = 0;
#pragma unroll
    for (int k = 0; k < UP; ++k) rows[nr++] = UP * vy + k + 1;
    if (UP == 1) {
      if (vy == 1) rows[nr++] = 0;
      if (vy == H - 2) rows[nr++] = H + 1;
    } else {
      if (vy == 0) rows[nr++] = 0;
      if (vy == h_in - 1) rows[nr++] = H + 1;
    }
    const float* d = dp + (int64_t)p * (H + 2) * Wp;
    const int cb = UP * vx0;  // first loaded column
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < nr; ++a) {
      const float* dr = d + (int64_t)rows[a] * Wp;
      float win[NW];
#pragma unroll
      for (int k = 0; k < NW / 4; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(dr + cb + 4 * k);
        win[4 * k] = v.x; win[4 * k + 1] = v.y; win[4 * k + 2] = v.z; win[4 * k + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int vx = vx0 + j;
        // the columns of pad_up_adjoint_full_kernel, in its order
#pragma unroll
        for (int k = 0; k < UP; ++k) s[j] += win[UP * j + k + 1];
        if (UP == 1) {
          if (vx == 1) s[j] += dr[0];
          if (vx == W - 2) s[j] += dr[W + 1];
        } else {
          if (vx == 0) s[j] += dr[0];
          if (vx == w_in - 1) s[j] += dr[W + 1];
        }
      }
    }
    *reinterpret_cast<float4*>(dx + (int64_t)row * w_in + vx0) = make_float4(s[0], s[1], s[2], s[3]);
  }
}

// dx = g * (mask > 0) (ReLU backward given the ReLU output).
__global__ void relu_mask_kernel(const float* __restrict__ g, const float* __restrict__ mask, float* __restrict__ out,
                                 int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mask[i] > 0.f ? g[i] : 0.f;
}

// Input-gradient epilogue outside the conv (configurations without it: ops.conv3x3_dgrad's fallback):
// dx[p][r][c] = epi(up == 2 ? the 2x2 window sum of raw (row by row) : raw[p][r][c]) with
// epi(v) = mask > 0 ? add_post + (v + add_pre) : add_post -- conv3x3_igemm.hip's dgrad_epi_one.
__global__ void dgrad_finish_kernel(const float* __restrict__ raw, float* __restrict__ dx, const float* __restrict__ mask,
                                    const float* __restrict__ add_pre, const float* __restrict__ add_post,
                                    int64_t planes, int h, int w, int up) {
  const int64_t total = planes * h * w;
  const int W = w * up;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % w);
    const int64_t pr = i / w;  // plane * h + r
    float v;
    if (up == 2) {
      const float* r0 = raw + (2 * pr) * W + 2 * c;
      v = ((r0[0] + r0[1]) + r0[W]) + r0[W + 1];
    } else {
      v = raw[i];
    }
    if (add_pre) v = v + add_pre[i];
    const bool keep = !mask || mask[i] > 0.f;
    dx[i] = add_post ? (keep ? add_post[i] + v : add_post[i]) : (keep ? v : 0.f);
  }
}

// Reflect-pad border of the input gradient (DecoderConvFn, ReflectionPad2d(1) after an optional x2
// nearest upsample, models.py:598-628). The input-gradient conv computes the interior of the
// padded-input gradient dP (a zero-padded same conv of dy); the reflect pad's adjoint also folds
// dP's four border lines onto the source. With U = upsample(x) [H = h up, W = w up], dy [cout, H, W]:
//   line 0  dP[ci][0][q]   = sum_{co, kx} w[co][ci][0][kx] dy[co][0][q - kx]      (-> U row 1)
//   line 1  dP[ci][H+1][q] = sum_{co, kx} w[co][ci][2][kx] dy[co][H-1][q - kx]    (-> U row H - 2)
//   line 2  dP[ci][p][0]   = sum_{co, ky} w[co][ci][ky][0] dy[co][p - ky][0]      (-> U col 1)
//   line 3  dP[ci][p][W+1] = sum_{co, ky} w[co][ci][ky][2] dy[co][p - ky][W - 1]  (-> U col W - 2)
// -- each a 1-D 3-tap correlation of a dy line (length L = W or H) over all cout, output length L + 2.
// Pass 1 (border_lines_kernel) computes the four lines into a workspace [n][4][cin][Lmax + 2] as small
// LDS-tiled GEMMs (workgroup: 32 ci x 64 positions, cout in chunks of 32); pass 2
// (border_fold_kernel) gives each x element any line lands on one thread, which sums its
// contributions in a fixed order and adds them, ReLU-masked like the interior, to dx: one writer
// per element, no atomics.
constexpr int BL_CI = 32, BL_Q = 64, BL_CO = 32;

// dy's first and last columns made contiguous, cols[n][cout][2][H] (one strided pass; the line
// kernel's column lines then read them like its row lines, instead of re-reading one 4-byte word
// per 64-byte line from every ci block)
__global__ __launch_bounds__(256) void border_cols_kernel(const float* __restrict__ dy, float* __restrict__ cols,
                                                          int64_t rows, int H, int W) {
  // rows = n * cout * 2 * H: (plane, side, y)
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < rows; i += (int64_t)gridDim.x * 256) {
    const int y = (int)(i % H);
    const int64_t ps = i / H;
    const int side = (int)(ps & 1);
    const int64_t pl = ps >> 1;
    cols[i] = dy[(pl * H + y) * W + (side ? W - 1 : 0)];
  }
}

__global__ __launch_bounds__(256) void border_lines_kernel(const float* __restrict__ dy, const float* __restrict__ cols,
                                                           const float* __restrict__ wt, float* __restrict__ lines,
                                                           int cout, int cin, int H, int W, int Lp) {
  __shared__ float Ds[BL_CO][BL_Q + 2];
  __shared__ float Ws[BL_CO][BL_CI][3];
  const int line = blockIdx.z & 3, n = blockIdx.z >> 2;
  const int q0 = blockIdx.x * BL_Q, ci0 = blockIdx.y * BL_CI;
  const bool row = line < 2;
  const int L = row ? W : H;
  if (q0 >= L + 2) return;
  // a line's source per output channel: a dy row (rows), or a contiguous column of cols
  const int64_t plane = row ? (int64_t)H * W : 2 * (int64_t)H;
  const int fixed = (line & 1) ? 2 : 0;
  const float* dyn = row ? dy + (int64_t)n * cout * plane + (line == 0 ? 0 : (int64_t)(H - 1) * W)
                         : cols + (int64_t)n * cout * plane + (line == 2 ? 0 : H);
  const int t = threadIdx.x, ci = t >> 3, qg = t & 7;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  // the next cout chunk's line values and weights are loaded into registers while this chunk's FMAs
  // run (per-thread staging coordinates fixed across chunks)
  constexpr int ND = (BL_CO * (BL_Q + 2) + 255) / 256, NWT = BL_CO * BL_CI * 3 / 256;
  static_assert(BL_CO * BL_CI * 3 % 256 == 0, "whole weight items per thread");
  float dreg[ND], wreg[NWT];
  auto gload = [&](int c0) {
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int e = t + 256 * i;
      const int co = e / (BL_Q + 2), j = e - co * (BL_Q + 2), src = q0 - 2 + j;
      dreg[i] = (e < BL_CO * (BL_Q + 2) && c0 + co < cout && src >= 0 && src < L)
                    ? dyn[(int64_t)(c0 + co) * plane + src] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NWT; ++i) {
      const int e = t + 256 * i;
      const int co = e / (BL_CI * 3), r = e - co * (BL_CI * 3), cc = r / 3, k = r - 3 * cc;
      // w[co][ci][ky][kx]: rows vary kx at ky = fixed, columns vary ky at kx = fixed
      const int tap = row ? 3 * fixed + k : 3 * k + fixed;
      wreg[i] = (c0 + co < cout && ci0 + cc < cin) ? wt[((int64_t)(c0 + co) * cin + ci0 + cc) * 9 + tap] : 0.f;
    }
  };
  gload(0);
  for (int c0 = 0; c0 < cout; c0 += BL_CO) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ND; ++i)
      if (t + 256 * i < BL_CO * (BL_Q + 2)) (&Ds[0][0])[t + 256 * i] = dreg[i];
#pragma unroll
    for (int i = 0; i < NWT; ++i) (&Ws[0][0][0])[t + 256 * i] = wreg[i];
    __syncthreads();
    if (c0 + BL_CO < cout) gload(c0 + BL_CO);
    const int cn = min(BL_CO, cout - c0);
    for (int co = 0; co < cn; ++co) {
      const float w0 = Ws[co][ci][0], w1 = Ws[co][ci][1], w2 = Ws[co][ci][2];
      float dv[10];
#pragma unroll
      for (int j = 0; j < 10; ++j) dv[j] = Ds[co][8 * qg + j];
      // dP[q] = sum_k w[k] D[q - k]; Ds[j] = D[q0 - 2 + j], q = q0 + 8 qg + i -> j = 8 qg + i + 2 - k
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(w2, dv[i], fmaf(w1, dv[i + 1], fmaf(w0, dv[i + 2], acc[i])));
    }
  }
  if (ci0 + ci >= cin) return;
  float* out = lines + (((int64_t)n * 4 + line) * cin + ci0 + ci) * Lp;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = q0 + 8 * qg + i;
    if (q < L + 2) out[q] = acc[i];
  }
}

__global__ __launch_bounds__(256) void border_fold_kernel(const float* __restrict__ lines, float* __restrict__ dx,
                                                          const float* __restrict__ mask, int cin, int h, int w, int up,
                                                          int Lp, int targets) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= targets) return;
  const int pl = blockIdx.y;  // n * cin + ci
  const int n = pl / cin, ci = pl - n * cin;
  const int H = h * up, W = w * up;
  // x rows / cols the four border lines land on
  const int rt = 1 / up, rb = (H - 2) / up, ct = 1 / up, cr = (W - 2) / up;
  const int nrow = rb != rt ? 2 : 1;
  int r, c;
  if (t < nrow * w) {
    r = t < w ? rt : rb;
    c = t < w ? t : t - w;
  } else {
    const int hr = h - nrow, t2 = t - nrow * w, side = t2 / hr;
    r = t2 - side * hr;  // the r-th row that is neither rt nor rb
    const int lo = min(rt, rb), hi = max(rt, rb);
    if (r >= lo) ++r;
    if (nrow == 2 && r >= hi) ++r;
    c = side == 0 ? ct : cr;
  }
  const float* ln = lines + ((int64_t)n * 4 * cin + ci) * Lp;
  const int64_t ls = (int64_t)cin * Lp;  // line stride
  // padded columns q whose source column lands on x column c: U columns up c .. up c + up - 1
  // (q = u + 1), plus the border columns
  int qs[4], nq = 0;
  for (int k = 0; k < up; ++k) qs[nq++] = up * c + k + 1;
  if (c == ct) qs[nq++] = 0;
  if (c == cr) qs[nq++] = W + 1;
  float s = 0.f;
  if (r == rt)
    for (int k = 0; k < nq; ++k) s += ln[qs[k]];
  if (r == rb)
    for (int k = 0; k < nq; ++k) s += ln[ls + qs[k]];
  if (c == ct)
    for (int k = 0; k < up; ++k) s += ln[2 * ls + up * r + k + 1];
  if (c == cr)
    for (int k = 0; k < up; ++k) s += ln[3 * ls + up * r + k + 1];
  const int64_t off = (int64_t)pl * h * w + (int64_t)r * w + c;
  if (!mask || mask[off] > 0.f) dx[off] = dx[off] + s;
}

// ------------------------------------------------------------------------------------------
// Weight gradient.
// ------------------------------------------------------------------------------------------
constexpr int WG_CO = 64, WG_CI = 64, WG_TH = 2, WG_TW = 32, WG_PIX = WG_TH * WG_TW;
constexpr int WG_DS = WG_CO + 1;  // dY tile [pix][co] row stride (odd: transposed stores conflict-free)

template <int UP>
struct WgCfg {
  static constexpr int SW = WG_TW / UP;
  static constexpr int SR = WG_TH / UP + 2;
  static constexpr int RS = SW + 8;
  static constexpr int C0 = 4;
  static constexpr int PS = SR * RS + 1;  // per-channel plane stride (odd: ci on lanes is conflict-free)
  static constexpr int QV = SW / 4;
  static constexpr int LDS = (WG_CI * PS + WG_PIX * WG_DS) * 4;
};

struct WgArgs {
  const float* x;
  const float* dy;
  float* dw;  // partials: split s writes its dW tile into dw + s * Cout * Cin * 9 (the workspace)
  float* db;  // and its db into db + s * Cout (workspace; null: no bias)
  int N, Cin, Hin, Win, Cout, reflect;
  int dy_pitch;        // row stride of dy
  int64_t dy_plane;    // plane stride of dy
  int64_t dy_off;      // offset of element (0, 0) inside a plane
  int tiles_x, tiles_y;
  int64_t tiles_per_block, ntiles;
};

template <int UP>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgArgs a) {
  using C = WgCfg<UP>;
  constexpr int SW = C::SW, SR = C::SR, RS = C::RS, PS = C::PS, QV = C::QV, C0 = C::C0;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ps = smem;                   // [WG_CI][PS]
  float* Ds = smem + WG_CI * PS;      // [WG_PIX][WG_DS]
  const int Hin = a.Hin, Win = a.Win;
  const int H = Hin * UP, W = Win * UP;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wco = wave & 1, wci = wave >> 1;
  const int co_groups = (a.Cout + WG_CO - 1) / WG_CO;
  const int ci_groups = (a.Cin + WG_CI - 1) / WG_CI;
  int b = blockIdx.x;
  const int cog = b % co_groups;
  b /= co_groups;
  const int cig = b % ci_groups;
  const int64_t split = b / ci_groups;
  const int co0 = cog * WG_CO, ci0 = cig * WG_CI;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bacc = 0.f;  // bias partial: co = tid & 63, pixels of quarter tid >> 6

  // per-lane LDS column offsets of the B operand for kx = 0..2 (pixel column parity = h)
  int bcol[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) bcol[kx] = (UP == 1) ? (C0 - 1 + h + kx) : (C0 + ((h + kx - 1) >> 1));
  const float* prow_base = Ps + (wci * 32 + l32) * PS;
  const int arow = wco * 32 + l32;

  const int64_t t0 = a.tiles_per_block * split;
  const int64_t t1 = min(a.ntiles, t0 + a.tiles_per_block);
  for (int64_t tile = t0; tile < t1; ++tile) {
    int64_t tt = tile;
    const int tx = (int)(tt % a.tiles_x);
    tt /= a.tiles_x;
    const int ty = (int)(tt % a.tiles_y);
    const int n = (int)(tt / a.tiles_y);
    const int x0 = tx * WG_TW, y0 = ty * WG_TH;
    const int sx0 = x0 / UP, sy0 = y0 / UP - 1;
    const float* xin = a.x + (int64_t)n * a.Cin * Hin * Win;
    const int plane_in = Hin * Win;
    __syncthreads();
    // ---- input halo tile [ci][SR][RS] ----
    if ((sx0 + SW <= Win) && ((Win & 3) == 0)) {
      for (int e = tid; e < WG_CI * SR * (QV + 2); e += 256) {
        const int q = e % (QV + 2);
        const int cr = e / (QV + 2);
        const int r = cr % SR, c = cr / SR;
        const int ci = ci0 + c;
        const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
        float* row = Ps + c * PS + r * RS;
        if (q < QV) {
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ci < a.Cin && sy >= 0) v = *reinterpret_cast<const float4*>(xin + (int64_t)ci * plane_in + sy * Win + sx0 + 4 * q);
          row[C0 + 4 * q] = v.x; row[C0 + 4 * q + 1] = v.y; row[C0 + 4 * q + 2] = v.z; row[C0 + 4 * q + 3] = v.w;
        } else {
          const int sx = src_index<UP>(q == QV ? sx0 - 1 : sx0 + SW, Win, a.reflect);
          row[q == QV ? C0 - 1 : C0 + SW] =
              (ci < a.Cin && sy >= 0 && sx >= 0) ? xin[(int64_t)ci * plane_in + sy * Win + sx] : 0.f;
        }
      }
    } else {
      for (int e = tid; e < WG_CI * SR * (SW + 2); e += 256) {
        const int col = e % (SW + 2);
        const int cr = e / (SW + 2);
        const int r = cr % SR, c = cr / SR;
        const int ci = ci0 + c;
        const int sy = src_index<UP>(sy0 + r, Hin, a.reflect);
        const int sx = src_index<UP>(sx0 - 1 + col, Win, a.reflect);
        Ps[c * PS + r * RS + C0 - 1 + col] =
            (ci < a.Cin && sy >= 0 && sx >= 0) ? xin[(int64_t)ci * plane_in + sy * Win + sx] : 0.f;
      }
    }
    // ---- dY tile [pix][co] (pix = row*32 + col), zero outside ----
    const float* dyn = a.dy + (int64_t)n * a.Cout * a.dy_plane + a.dy_off;
    for (int e = tid; e < WG_CO * WG_PIX; e += 256) {
      const int pix = e % WG_PIX, c = e / WG_PIX;
      const int co = co0 + c, yy = y0 + pix / WG_TW, xx = x0 + pix % WG_TW;
      float v = 0.f;
      if (co < a.Cout && yy < H && xx < W) v = dyn[(int64_t)co * a.dy_plane + (int64_t)yy * a.dy_pitch + xx];
      Ds[pix * WG_DS + c] = v;
    }
    __syncthreads();
    if (a.db && cig == 0) {
      const int c = tid & 63, q = tid >> 6;
#pragma unroll
      for (int k = 0; k < WG_PIX / 4; ++k) bacc += Ds[(q * (WG_PIX / 4) + k) * WG_DS + c];
    }
#pragma unroll 2
    for (int kp = 0; kp < WG_PIX / 2; ++kp) {
      const int prow = (2 * kp) / WG_TW;   // wave-uniform
      const int pc0 = (2 * kp) % WG_TW;    // even; the lane's pixel column is pc0 + h
      const float av = Ds[(2 * kp + h) * WG_DS + arow];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int srow = (UP == 1) ? prow + ky : ((prow + ky - 1) >> 1) + 1;
        const float* rp = prow_base + srow * RS + ((UP == 1) ? pc0 : (pc0 >> 1));
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float bv = rp[bcol[kx]];
          acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[ky * 3 + kx], 0, 0, 0);
        }
      }
    }
  }
  // C[i = co][j = ci]: col j = l32, rows i = (r&3)+8(r>>2)+4h
  const int ci = ci0 + wci * 32 + l32;
  float* const dwp = a.dw + (int64_t)split * a.Cout * a.Cin * 9;
  if (ci < a.Cin) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wco * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co < a.Cout) dwp[((int64_t)co * a.Cin + ci) * 9 + t] = acc[t][r];
      }
    }
  }
  if (a.db && cig == 0) {  // the 4 quarter-partials of each co, added in quarter order
    __shared__ float bq[4][64];
    __syncthreads();
    bq[tid >> 6][tid & 63] = bacc;
    __syncthreads();
    if (tid < 64 && co0 + tid < a.Cout) a.db[split * a.Cout + co0 + tid] = (bq[0][tid] + bq[1][tid]) + (bq[2][tid] + bq[3][tid]);
  }
}

// Weight gradient for Cout <= 4 (the decoders' image convs, models.py:627), or Cout <= 16 with
// Cin <= 16 (the MobileNet image convs 3->16 / 16->3): as an MFMA GEMM with 64x64 tiles these
// leave >93% of every tile idle, so this is a VALU reduction instead. A workgroup
// owns SC_CG input channels and sweeps a range of 8x32-pixel tiles (one output pixel per thread):
// the tile's input halo (padded/upsampled grid coordinates resolved at staging) sits in LDS, each
// thread accumulates COUT x SC_CG x 9 products of its pixel's dY with the 9 shifted inputs, and
// the partial dW is reduced over the workgroup (wave shuffles + LDS) into one atomic per weight.
constexpr int SC_TH = 8, SC_TW = 32, SC_RS = SC_TW + 2, SC_PS = (SC_TH + 2) * SC_RS;

template <int COUT, int SC_CG, int UP>
__global__ __launch_bounds__(256) void wgrad_smallco_kernel(WgArgs a) {
  __shared__ float xs[SC_CG * SC_PS];
  __shared__ float red[4][COUT * SC_CG * 9 + COUT];
  const int Hin = a.Hin, Win = a.Win, H = Hin * UP, W = Win * UP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ty = tid / SC_TW, tx = tid % SC_TW;
  const int ci_groups = (a.Cin + SC_CG - 1) / SC_CG;
  const int cig = blockIdx.x % ci_groups;
  const int64_t split = blockIdx.x / ci_groups;
  const int ci0 = cig * SC_CG;
  float acc[COUT][SC_CG * 9];
  float bacc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
    bacc[o] = 0.f;
#pragma unroll
    for (int t = 0; t < SC_CG * 9; ++t) acc[o][t] = 0.f;
  }
  const int64_t t0 = a.tiles_per_block * split;
  const int64_t t1 = min(a.ntiles, t0 + a.tiles_per_block);
  // register prefetch (round 5): the next tile's input halo and dY are loaded while this tile's
  // FMAs run (the staging was latency-bound: loads -> barrier -> dY loads -> FMAs per tile).
  // Per-thread staging coordinates are fixed across tiles; same products in the same order.
  constexpr int NX = (SC_CG * SC_PS + 255) / 256;
  int xc[NX], xr[NX], xcol[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int e = tid + 256 * i, rc = e % SC_PS;
    xc[i] = e / SC_PS;
    xr[i] = rc / SC_RS;
    xcol[i] = rc % SC_RS;
  }
  float xv[NX], dv[COUT];
  bool dok = false;
  auto load = [&](int64_t tile) {
    int64_t tt = tile;
    const int bx = (int)(tt % a.tiles_x);
    tt /= a.tiles_x;
    const int by = (int)(tt % a.tiles_y);
    const int n = (int)(tt / a.tiles_y);
    const int x0 = bx * SC_TW, y0 = by * SC_TH;
    const float* xin = a.x + ((int64_t)n * a.Cin + ci0) * Hin * Win;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      float v = 0.f;
      if (tid + 256 * i < SC_CG * SC_PS && ci0 + xc[i] < a.Cin) {
        int gy = y0 - 1 + xr[i], gx = x0 - 1 + xcol[i];   // padded, upsampled grid
        bool ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
        if (!ok && a.reflect && gy >= -1 && gy <= H && gx >= -1 && gx <= W) {
          gy = gy < 0 ? -gy : (gy >= H ? 2 * (H - 1) - gy : gy);
          gx = gx < 0 ? -gx : (gx >= W ? 2 * (W - 1) - gx : gx);
          ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
        }
        if (ok) v = xin[((int64_t)xc[i] * Hin + gy / UP) * Win + gx / UP];
      }
      xv[i] = v;
    }
    const int yy = y0 + ty, xx = x0 + tx;
    dok = yy < H && xx < W;
    const float* dyn = a.dy + (int64_t)n * a.Cout * a.dy_plane + a.dy_off + (int64_t)yy * a.dy_pitch + xx;
#pragma unroll
    for (int o = 0; o < COUT; ++o) dv[o] = (dok && o < a.Cout) ? dyn[(int64_t)o * a.dy_plane] : 0.f;
  };
  if (t0 < t1) load(t0);
  for (int64_t tile = t0; tile < t1; ++tile) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NX; ++i)
      if (tid + 256 * i < SC_CG * SC_PS) xs[tid + 256 * i] = xv[i];
    __syncthreads();
    const bool cur_ok = dok;
    float d[COUT];
#pragma unroll
    for (int o = 0; o < COUT; ++o) d[o] = dv[o];
    if (tile + 1 < t1) load(tile + 1);
    if (cur_ok) {
#pragma unroll
      for (int o = 0; o < COUT; ++o) bacc[o] += d[o];
#pragma unroll
      for (int c = 0; c < SC_CG; ++c)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const float v = xs[c * SC_PS + (ty + ky) * SC_RS + tx + kx];
#pragma unroll
            for (int o = 0; o < COUT; ++o) acc[o][c * 9 + ky * 3 + kx] = fmaf(d[o], v, acc[o][c * 9 + ky * 3 + kx]);
          }
    }
  }
  // reduce over the workgroup: 64-lane shuffles, then the 4 waves through LDS
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
#pragma unroll
    for (int t = 0; t < SC_CG * 9; ++t) {
      float v = acc[o][t];
#pragma unroll
      for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
      if (lane == 0) red[wave][o * SC_CG * 9 + t] = v;
    }
    float b = bacc[o];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) b += __shfl_xor(b, m, 64);
    if (lane == 0) red[wave][COUT * SC_CG * 9 + o] = b;
  }
  __syncthreads();
  for (int e = tid; e < COUT * SC_CG * 9 + COUT; e += 256) {
    const float v = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
    if (e < COUT * SC_CG * 9) {
      const int o = e / (SC_CG * 9), t = e % (SC_CG * 9), c = t / 9, tap = t % 9;
      if (o < a.Cout && ci0 + c < a.Cin) a.dw[split * a.Cout * a.Cin * 9 + ((int64_t)o * a.Cin + ci0 + c) * 9 + tap] = v;
    } else if (a.db && cig == 0 && e - COUT * SC_CG * 9 < a.Cout) {
      a.db[split * a.Cout + (e - COUT * SC_CG * 9)] = v;
    }
  }
}

// Aligned-shape weight gradient (Cin, Cout multiples of 64; output W a multiple of 32, H even):
// the same tile, LDS images and MFMA loop as wgrad_kernel, with the staging rebuilt around a
// register prefetch -- the next tile's input halo (float4 pieces, halo columns as single floats)
// and dY are loaded while the current tile's MFMAs run, from per-thread offsets computed once.
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int UP>
__global__ __launch_bounds__(256, 2) void wgrad2_kernel(WgArgs a) {
  using C = WgCfg<UP>;
  constexpr int SW = C::SW, SR = C::SR, RS = C::RS, PS = C::PS, QV = C::QV, C0 = C::C0;
  constexpr int NI = WG_CI * SR * QV;        // float4 input pieces per tile
  constexpr int KI = (NI + 255) / 256;
  constexpr int NH = WG_CI * SR * 2;         // halo columns per tile
  constexpr int KH = (NH + 255) / 256;
  constexpr int KD = WG_CO * WG_PIX / 256;   // dY values per thread (16)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ps = smem;                   // [WG_CI][PS]
  float* Ds = smem + WG_CI * PS;      // [WG_PIX][WG_DS]
  const int Hin = a.Hin, Win = a.Win;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wco = wave & 1, wci = wave >> 1;
  const int co_groups = a.Cout / WG_CO, ci_groups = a.Cin / WG_CI;
  int b = blockIdx.x;
  const int cog = b % co_groups;
  b /= co_groups;
  const int cig = b % ci_groups;
  const int split = b / ci_groups;
  const int co0 = cog * WG_CO, ci0 = cig * WG_CI;
  const int plane_in = Hin * Win;

  // staging items (recomputed where used, constant divisors): float4 piece e = tid + 256k ->
  // (channel, halo row, column q); halo item -> (channel, row, left/right)
#define WG2_ITEM(k)                                                      \
  const int e_ = min(tid + 256 * (k), NI - 1);                           \
  const int q_ = e_ % QV, cr_ = e_ / QV, r_ = cr_ % SR, c_ = cr_ / SR;
#define WG2_HALO(k)                                                      \
  const int e_ = min(tid + 256 * (k), NH - 1);                           \
  const int s_ = e_ & 1, cr_ = e_ >> 1, r_ = cr_ % SR, c_ = cr_ / SR;
  const int d_pix = tid & 63, d_c = tid >> 6;
  const int d_off = (d_pix / WG_TW) * a.dy_pitch + d_pix % WG_TW;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = (f32x16){0.f};
  float bacc = 0.f;
  int bcol[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) bcol[kx] = (UP == 1) ? (C0 - 1 + h + kx) : (C0 + ((h + kx - 1) >> 1));
  const float* prow_base = Ps + (wci * 32 + l32) * PS;
  const int arow = wco * 32 + l32;

  f32x4 xr[KI];
  float hr[KH];
  float dr[KD];
  auto load_tile = [&](int tile) {
    int tt = tile;
    const int tx = tt % a.tiles_x;
    tt /= a.tiles_x;
    const int ty = tt % a.tiles_y;
    const int n = tt / a.tiles_y;
    const int x0 = tx * WG_TW, y0 = ty * WG_TH;
    const int sx0 = x0 / UP, sy0 = y0 / UP - 1;
    const float* xin = a.x + (int64_t)n * a.Cin * plane_in;
    const int sxl = src_index<UP>(sx0 - 1, Win, a.reflect), sxr = src_index<UP>(sx0 + SW, Win, a.reflect);
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      WG2_ITEM(k)
      const int sy = src_index<UP>(sy0 + r_, Hin, a.reflect);
      xr[k] = sy >= 0 ? *reinterpret_cast<const f32x4*>(xin + (ci0 + c_) * plane_in + sy * Win + sx0 + 4 * q_)
                      : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      WG2_HALO(k)
      const int sy = src_index<UP>(sy0 + r_, Hin, a.reflect), sx = s_ ? sxr : sxl;
      hr[k] = (sy >= 0 && sx >= 0) ? xin[(ci0 + c_) * plane_in + sy * Win + sx] : 0.f;
    }
    const float* dyn = a.dy + (int64_t)n * a.Cout * a.dy_plane + a.dy_off + (int64_t)y0 * a.dy_pitch + x0 + d_off +
                       (int64_t)(co0 + d_c) * a.dy_plane;
#pragma unroll
    for (int k = 0; k < KD; ++k) dr[k] = dyn[(int64_t)(4 * k) * a.dy_plane];
  };

  const int t0 = (int)(a.tiles_per_block * split);
  const int t1 = (int)min(a.ntiles, (int64_t)t0 + a.tiles_per_block);
  if (t0 < t1) load_tile(t0);
  for (int tile = t0; tile < t1; ++tile) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      WG2_ITEM(k)
      float* d = Ps + c_ * PS + r_ * RS + C0 + 4 * q_;
      d[0] = xr[k][0]; d[1] = xr[k][1]; d[2] = xr[k][2]; d[3] = xr[k][3];
    }
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      WG2_HALO(k)
      Ps[c_ * PS + r_ * RS + (s_ ? C0 + SW : C0 - 1)] = hr[k];
    }
#pragma unroll
    for (int k = 0; k < KD; ++k) Ds[d_pix * WG_DS + d_c + 4 * k] = dr[k];
    __syncthreads();
    if (tile + 1 < t1) load_tile(tile + 1);
    if (a.db && cig == 0) {
      const int c = tid & 63, q = tid >> 6;
#pragma unroll
      for (int k = 0; k < WG_PIX / 4; ++k) bacc += Ds[(q * (WG_PIX / 4) + k) * WG_DS + c];
    }
#pragma unroll 2
    for (int kp = 0; kp < WG_PIX / 2; ++kp) {
      const int prow = (2 * kp) / WG_TW;
      const int pc0 = (2 * kp) % WG_TW;
      const float av = Ds[(2 * kp + h) * WG_DS + arow];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int srow = (UP == 1) ? prow + ky : ((prow + ky - 1) >> 1) + 1;
        const float* rp = prow_base + srow * RS + ((UP == 1) ? pc0 : (pc0 >> 1));
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
          acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, rp[bcol[kx]], acc[ky * 3 + kx], 0, 0, 0);
      }
    }
  }
  const int ci = ci0 + wci * 32 + l32;
  float* const dwp = a.dw + (int64_t)split * a.Cout * a.Cin * 9;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wco * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      dwp[((int64_t)co * a.Cin + ci) * 9 + t] = acc[t][r];
    }
  if (a.db && cig == 0) {  // the 4 quarter-partials of each co, added in quarter order
    __shared__ float bq[4][64];
    __syncthreads();
    bq[tid >> 6][tid & 63] = bacc;
    __syncthreads();
    if (tid < 64) a.db[(int64_t)split * a.Cout + co0 + tid] = (bq[0][tid] + bq[1][tid]) + (bq[2][tid] + bq[3][tid]);
  }
#undef WG2_ITEM
#undef WG2_HALO
}

// Split-bf16 weight gradient (fp32-accurate on the bf16 matrix cores; the x = hi + mid + lo split and
// the 6-product sum of conv3x3_igemm.hip's x3 kernel). dW[co][ci][tap] = sum_pix dY[co][pix] *
// X[ci][pix + tap] as a GEMM with K = pixels, v_mfma_f32_32x32x16_bf16:
//  * A = dY (rows co): LDS [plane][co][pixel] (row pitch 144 B: conflict-free ds_read_b128 of 8
//    consecutive pixels per lane);
//  * B = X shifted by the tap (cols ci): LDS [plane][ci half][halo pixel][32 ci] (64-B rows), read
//    with ds_read_b64_tr_b16 -- a lane supplies the address of ITS pixel row, so the tap shift, the
//    zero/reflect padding and the nearest x2 upsample are all just row addresses, at any alignment.
// A workgroup (4 waves, 2 x 2 over co x ci) owns 64 co x 64 ci x 9 taps (each wave 32 x 32 x 9 in 9
// accumulators) and sweeps a range of 2 x 32-pixel tiles; ~80 KB LDS: two workgroups per CU, so
// one's staging (global loads, split, LDS writes) overlaps the other's MFMAs. Partial dW and db meet
// through fp32 atomics, as in wgrad2_kernel.
typedef __bf16 bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// as split3 in conv3x3_igemm.hip (finite overflow of hi clamped; non-finite x carried by hi alone)
__device__ __forceinline__ void wg_split3(float x, bf16_t& hi, bf16_t& mid, bf16_t& lo) {
  const bool finite = fabsf(x) <= 3.402823466e38f;
  hi = (bf16_t)x;
  if (finite && !(fabsf((float)hi) <= 3.402823466e38f)) hi = (bf16_t)copysignf(3.38953139e38f, x);
  float r = finite ? x - (float)hi : 0.f;
  mid = (bf16_t)r;
  lo = (bf16_t)(r - (float)mid);
}

template <int UP>
struct Wg3Cfg {
  static constexpr int SR = WG_TH / UP + 2, SC = WG_TW / UP + 2;
  static constexpr int NPIX = SR * SC;                       // halo pixels
  static constexpr int XROW = 64;                            // bytes per halo pixel row (32 ci)
  static constexpr int XHALF = NPIX * XROW;                  // bytes per ci half
  static constexpr int XPLANE = 2 * XHALF;
  static constexpr int DP = 144;                             // dY row pitch (bytes): 64 px + 8 pad
  static constexpr int DPLANE = WG_CO * DP;
  static constexpr int DOFF = 3 * XPLANE;                    // dY image after the X image
  static constexpr int LDS = 3 * XPLANE + 3 * DPLANE;
  static constexpr int XI = NPIX * 4;                        // X items per ci half: (pixel, 8-channel group)
  static constexpr int XT = (XI + 255) / 256;
};

template <int UP>
__global__ __launch_bounds__(256, 2) void wgrad3_kernel(WgArgs a) {
  using C = Wg3Cfg<UP>;
  constexpr int SC = C::SC, NPIX = C::NPIX, XT = C::XT;
  extern __shared__ __attribute__((aligned(16))) unsigned char wg3_smem[];
  const int Hin = a.Hin, Win = a.Win, plane_in = Hin * Win;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wco = wave & 1, wci = wave >> 1;
  const int co_groups = a.Cout / WG_CO, ci_groups = a.Cin / WG_CI;
  int b = blockIdx.x;
  const int cog = b % co_groups;
  b /= co_groups;
  const int cig = b % ci_groups;
  const int split = b / ci_groups;
  const int co0 = cog * WG_CO, ci0 = cig * WG_CI;

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = (f32x16){0.f};
  float bacc[2] = {0.f, 0.f};

  // X staging items: e = tid + 256k -> pixel p = e % NPIX (lanes run along pixels: coalesced
  // loads), channel group g = e / NPIX (8 channels)
  // dY staging items: e = tid + 256k (k = 0, 1) -> co = e / 8, pixel octet o = e % 8
  // B operand (tr read) lane roles: q = (lane >> 2) & 3 (row), p = lane & 3 (column quad), cb =
  // (lane >> 4) & 1 (16-column block)
  const int trq = (lane >> 2) & 3, trp = lane & 3, trcb = (lane >> 4) & 1;
  const int xcol_b = wci * C::XHALF + (16 * trcb + 4 * trp) * 2;  // byte offset of this lane's 4 ci
  const int arow_b = C::DOFF + (wco * 32 + l32) * C::DP + 16 * h;  // A: co row, pixel octet h of the k-step

  const int t0 = (int)(a.tiles_per_block * split);
  const int t1 = (int)min(a.ntiles, (int64_t)t0 + a.tiles_per_block);
  for (int tile = t0; tile < t1; ++tile) {
    int tt = tile;
    const int tx = tt % a.tiles_x;
    tt /= a.tiles_x;
    const int ty = tt % a.tiles_y;
    const int n = tt / a.tiles_y;
    const int x0 = tx * WG_TW, y0 = ty * WG_TH;
    const int sx0 = x0 / UP, sy0 = y0 / UP - 1;
    const float* __restrict__ xin = a.x + ((int64_t)n * a.Cin + ci0) * plane_in;
    // ---- staging. X is loaded one ci half at a time (registers): half 0 and dY before the barrier
    // (in flight during the other waves' last MFMAs of the previous tile), half 1 right after it,
    // in flight while half 0 and dY are split and written ----
    float xv[XT][8];
#define WG3_LOAD_X(HALF)                                                                                  \
    _Pragma("unroll") for (int k = 0; k < XT; ++k) {                                                      \
      const int e = min(tid + 256 * k, C::XI - 1), p = e % NPIX, g = (HALF) * 4 + e / NPIX;               \
      const int r = p / SC, c = p % SC;                                                                   \
      const int sy = src_index<UP>(sy0 + r, Hin, a.reflect), sx = src_index<UP>(sx0 - 1 + c, Win, a.reflect); \
      const bool ok = sy >= 0 && sx >= 0;                                                                 \
      const float* src = xin + (int64_t)(8 * g) * plane_in + max(sy, 0) * Win + max(sx, 0);              \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                     \
        const float v = src[(int64_t)j * plane_in];                                                       \
        xv[k][j] = ok ? v : 0.f;                                                                          \
      }                                                                                                   \
    }
#define WG3_STORE_X(HALF)                                                                                 \
    _Pragma("unroll") for (int k = 0; k < XT; ++k) {                                                      \
      const int e = tid + 256 * k;                                                                        \
      if (e < C::XI) {                                                                                    \
        const int p = e % NPIX, g = (HALF) * 4 + e / NPIX;                                                \
        bf16x8_t pv[3];                                                                                   \
        ast_x3::split8(xv[k], pv[0], pv[1], pv[2]);  /* = wg_split3 per value, paired conversions */    \
        const int off = (g >> 2) * C::XHALF + p * C::XROW + (g & 3) * 16;                                 \
        _Pragma("unroll") for (int pl = 0; pl < 3; ++pl)                                                  \
          *reinterpret_cast<u32x4_t*>(wg3_smem + pl * C::XPLANE + off) = __builtin_bit_cast(u32x4_t, pv[pl]); \
      }                                                                                                   \
    }
    WG3_LOAD_X(0)
    float dv[2][8];
    const float* __restrict__ dyn = a.dy + (int64_t)n * a.Cout * a.dy_plane + a.dy_off;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + 256 * k, co = e >> 3, o = e & 7;
      const float* src = dyn + (int64_t)(co0 + co) * a.dy_plane + (int64_t)(y0 + (o >> 2)) * a.dy_pitch + x0 + 8 * (o & 3);
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[k][j] = src[j];
    }
    __syncthreads();  // the previous tile's operand reads are done
    WG3_STORE_X(0)
    WG3_LOAD_X(1)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + 256 * k, co = e >> 3, o = e & 7;
      bf16x8_t pv[3];
#pragma unroll
      for (int j = 0; j < 8; ++j) bacc[k] += dv[k][j];
      ast_x3::split8(dv[k], pv[0], pv[1], pv[2]);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        *reinterpret_cast<u32x4_t*>(wg3_smem + C::DOFF + pl * C::DPLANE + co * C::DP + 16 * o) =
            __builtin_bit_cast(u32x4_t, pv[pl]);
    }
    WG3_STORE_X(1)
#undef WG3_LOAD_X
#undef WG3_STORE_X
    __syncthreads();
    // ---- 4 k-steps of 16 pixels: output row pr = ks >> 1, columns 16 (ks & 1) + 0..15 ----
#pragma unroll 1
    for (int ks = 0; ks < 4; ++ks) {
      const int pr = ks >> 1, cj = 16 * (ks & 1);
      bf16x8_t af[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        af[pl] = *reinterpret_cast<const bf16x8_t*>(wg3_smem + arow_b + pl * C::DPLANE + 32 * ks);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int srow = (UP == 1) ? pr + ky : ((pr + ky - 1) >> 1) + 1;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          // this lane's rows: k = 8h + 4rr + q of the k-step -> output column cj + k
          int pix[2];
#pragma unroll
          for (int rr = 0; rr < 2; ++rr) {
            const int xo = cj + 8 * h + 4 * rr + trq;  // output column within the tile
            const int scol = (UP == 1) ? xo + kx : ((xo + kx - 1) >> 1) + 1;
            pix[rr] = srow * SC + scol;
          }
          bf16x8_t bfr[3];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const unsigned char* base = wg3_smem + pl * C::XPLANE + xcol_b;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + pix[0] * C::XROW));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + pix[1] * C::XROW));
            bfr[pl] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
          f32x16 c = acc[ky * 3 + kx];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], bfr[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bfr[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bfr[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[1], c, 0, 0, 0);
          acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[0], c, 0, 0, 0);
        }
      }
    }
  }
  const int ci = ci0 + wci * 32 + l32;
  float* const dwp = a.dw + (int64_t)split * a.Cout * a.Cin * 9;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wco * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      dwp[((int64_t)co * a.Cin + ci) * 9 + t] = acc[t][r];
    }
  if (a.db && cig == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // the 8 threads of one co are 8 consecutive lanes
      float v = bacc[k];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if ((tid & 7) == 0) a.db[(int64_t)split * a.Cout + co0 + ((tid + 256 * k) >> 3)] = v;
    }
  }
}

int g_wgrad_v1 = 0;  // AST_WGRAD_V1=1: always the general kernel (A/B measurements)
// AST_BWD_ROWPAR=0: the flat elementwise backward kernels (A/B measurements)
const int g_rowpar = [] {
  const char* v = getenv("AST_BWD_ROWPAR");
  return v ? atoi(v) : 1;
}();

int grid1(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline int round_up(int a, int b) { return cdiv(a, b) * b; }

}  // namespace

extern "C" {

int ast_conv3x3_pack_weights_ex_f32(const float* w, float* w_packed, int cout, int cin, int transpose_flip,
                                    const float* in_scale, void* stream) {
  if (!w || !w_packed) return AST_E_NULLPTR;
  if (cout <= 0 || cin <= 0) return AST_E_SHAPE;
  if (!transpose_flip) {
    if (in_scale) return AST_E_UNSUPPORTED;
    return ast_conv3x3_pack_weights_f32(w, w_packed, cout, cin, stream);
  }
  // packed as a conv with cin' = cout, cout' = cin
  const int pad_out = round_up(cin, 64), pad_in = round_up(cout, 8);
  hipLaunchKernelGGL(pack_tf_kernel, dim3(grid1((int64_t)pad_in * 9 * pad_out)), dim3(256), 0, (hipStream_t)stream,
                     w, w_packed, cout, cin, pad_out, pad_in, in_scale);
  const int e = (int)hipGetLastError();
  return e ? e : ast_conv3x3_pack_split_f32(w_packed, cin, cout, stream);   // conv with cin' = cout, cout' = cin
}

int ast_conv_act_backward_f32(const float* pre, const float* g_pre, const float* g_act, const float* g_pool,
                              float* dy, long long planes, int h, int w, void* stream) {
  if (!pre || !dy) return AST_E_NULLPTR;
  if (planes <= 0 || h <= 0 || w <= 0) return AST_E_SHAPE;
  const bool al = ((((uintptr_t)pre | (uintptr_t)g_pre | (uintptr_t)g_act | (uintptr_t)dy) & 15) == 0) &&
                  (((uintptr_t)g_pool & 7) == 0);
  if (g_rowpar && w % 4 == 0 && al && planes * h * (w / 4) < 0x7fffffffLL) {
    const unsigned nq = (unsigned)(planes * h * (w / 4));
    hipLaunchKernelGGL(act_backward_v4_kernel, dim3(grid1(nq)), dim3(256), 0, (hipStream_t)stream, pre, g_pre, g_act,
                       g_pool, dy, nq, h, w);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(act_backward_kernel, dim3(grid1(planes * h * w)), dim3(256), 0, (hipStream_t)stream, pre, g_pre,
                     g_act, g_pool, dy, (int64_t)planes, h, w);
  return (int)hipGetLastError();
}

int ast_relu_mask_f32(const float* g, const float* mask, float* out, long long n, void* stream) {
  if (!g || !mask || !out) return AST_E_NULLPTR;
  if (n <= 0) return AST_E_SHAPE;
  hipLaunchKernelGGL(relu_mask_kernel, dim3(grid1(n)), dim3(256), 0, (hipStream_t)stream, g, mask, out, (int64_t)n);
  return (int)hipGetLastError();
}

int ast_grad_pad_f32(const float* g, const float* mask, float* out_pad, long long planes, int h, int w, int pitch,
                     void* stream) {
  if (!g || !out_pad) return AST_E_NULLPTR;
  if (planes <= 0 || h <= 0 || w <= 0 || pitch < w + 2) return AST_E_SHAPE;
  if (g_rowpar && pitch % 4 == 0 && w % 4 == 0 && ((((uintptr_t)out_pad | (uintptr_t)g | (uintptr_t)mask) & 15) == 0) &&
      planes * (h + 2) * (pitch / 4) < 0x7fffffffLL) {
    const unsigned nq = (unsigned)(planes * (h + 2) * (pitch / 4));
    hipLaunchKernelGGL(pad_grad_v4_kernel, dim3(grid1(nq)), dim3(256), 0, (hipStream_t)stream, g, mask, out_pad, nq, h,
                       w, pitch);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(pad_grad_kernel, dim3(grid1(planes * (h + 2) * pitch)), dim3(256), 0, (hipStream_t)stream, g,
                     mask, out_pad, (int64_t)planes, h, w, pitch);
  return (int)hipGetLastError();
}

int ast_dgrad_finish_f32(const float* raw, float* dx, const float* mask, const float* add_pre, const float* add_post,
                         long long planes, int h, int w, int upsample, void* stream) {
  if (!raw || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || h <= 0 || w <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  hipLaunchKernelGGL(dgrad_finish_kernel, dim3(grid1(planes * h * w)), dim3(256), 0, (hipStream_t)stream, raw, dx, mask,
                     add_pre, add_post, (int64_t)planes, h, w, upsample);
  return (int)hipGetLastError();
}

long long ast_dgrad_reflect_border_workspace_floats(int n, int cout, int cin, int h, int w_in, int upsample) {
  if (n <= 0 || cout <= 0 || cin <= 0 || h <= 0 || w_in <= 0 || (upsample != 1 && upsample != 2)) return 0;
  // the four lines [n][4][cin][max(H, W) + 2], then dy's edge columns [n][cout][2][H]
  return (long long)n * 4 * cin * (std::max(h, w_in) * upsample + 2) + (long long)n * cout * 2 * h * upsample;
}

int ast_dgrad_reflect_border_f32(const float* dy, const float* w, float* dx, const float* mask, float* workspace,
                                 long long workspace_floats, int n, int cout, int cin, int h, int w_in, int upsample,
                                 void* stream) {
  if (!dy || !w || !dx || !workspace) return AST_E_NULLPTR;
  if (n <= 0 || cout <= 0 || cin <= 0 || h <= 0 || w_in <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (h * upsample < 2 || w_in * upsample < 2) return AST_E_SHAPE;  // ReflectionPad2d(1) needs size >= 2
  if ((int64_t)n * cin >= 65536 || (int64_t)n * 4 >= 65536 || (int64_t)cout * h * w_in * upsample * upsample >= ((int64_t)1 << 31))
    return AST_E_SHAPE;
  if (workspace_floats < ast_dgrad_reflect_border_workspace_floats(n, cout, cin, h, w_in, upsample)) return AST_E_SHAPE;
  const int H = h * upsample, W = w_in * upsample, Lp = std::max(H, W) + 2;
  float* cols = workspace + (int64_t)n * 4 * cin * Lp;
  const int64_t crows = (int64_t)n * cout * 2 * H;
  hipLaunchKernelGGL(border_cols_kernel, dim3((unsigned)std::min<int64_t>((crows + 255) / 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, dy, cols, crows, H, W);
  int e = (int)hipGetLastError();
  if (e) return e;
  hipLaunchKernelGGL(border_lines_kernel, dim3((Lp + BL_Q - 1) / BL_Q, (cin + BL_CI - 1) / BL_CI, n * 4), dim3(256), 0,
                     (hipStream_t)stream, dy, cols, w, workspace, cout, cin, H, W, Lp);
  e = (int)hipGetLastError();
  if (e) return e;
  const int rt = 1 / upsample, rb = (H - 2) / upsample, ct = 1 / upsample, cr = (W - 2) / upsample;
  const int nrow = rb != rt ? 2 : 1, ncol = cr != ct ? 2 : 1;
  const int targets = nrow * w_in + (h - nrow) * ncol;
  hipLaunchKernelGGL(border_fold_kernel, dim3((targets + 255) / 256, n * cin), dim3(256), 0, (hipStream_t)stream,
                     workspace, dx, mask, cin, h, w_in, upsample, Lp, targets);
  return (int)hipGetLastError();
}

int ast_pad_up_adjoint_f32(const float* dp_full, float* dx, long long planes, int h_in, int w_in, int upsample,
                           int pitch, void* stream) {
  if (!dp_full || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || h_in <= 0 || w_in <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (h_in * upsample < 2 || w_in * upsample < 2 || pitch < w_in * upsample + 2) return AST_E_SHAPE;
  if (g_rowpar && w_in % 4 == 0 && pitch % 4 == 0 && pitch >= w_in * upsample + 4 &&
      ((((uintptr_t)dx | (uintptr_t)dp_full) & 15) == 0) && planes * h_in * (w_in / 4) < 0x7fffffffLL) {
    const unsigned nq = (unsigned)(planes * h_in * (w_in / 4));
    if (upsample == 1)
      hipLaunchKernelGGL(pad_up_adjoint_v4_kernel<1>, dim3(grid1(nq)), dim3(256), 0, (hipStream_t)stream, dp_full, dx,
                         nq, h_in, w_in, pitch);
    else
      hipLaunchKernelGGL(pad_up_adjoint_v4_kernel<2>, dim3(grid1(nq)), dim3(256), 0, (hipStream_t)stream, dp_full, dx,
                         nq, h_in, w_in, pitch);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(pad_up_adjoint_full_kernel, dim3(grid1(planes * h_in * w_in)), dim3(256), 0, (hipStream_t)stream,
                     dp_full, dx, (int64_t)planes, h_in, w_in, upsample, pitch);
  return (int)hipGetLastError();
}

}  // extern "C"

namespace {
// Launch plan shared by the wgrad entry point and its workspace query: the kernel family, its
// tile grid and the number of pixel-range splits (each split's partial dW/db is one workspace slot).
struct WgPlan {
  bool small;  // wgrad_smallco_kernel
  bool co3;    // wgrad_co3_kernel (split-bf16 MFMA, Cout <= 3; wgrad_co3.hip)
  int tiles_x, tiles_y, groups;
  int64_t ntiles, tiles_per_block, splits;
};

int g_wgrad_co3 = 1;  // AST_WGRAD_CO3=0: Cout <= 3 on the VALU kernel (A/B measurements)

WgPlan wgrad_plan(int n, int cin, int h_in, int w_in, int cout, int upsample, bool allow_co3 = true) {
  WgPlan p{};
  const int H = h_in * upsample, W = w_in * upsample;
  p.co3 = allow_co3 && g_wgrad_co3 && !g_wgrad_v1 && wgrad_co3_supported(cin, h_in, w_in, cout, upsample);
  p.small = !p.co3 && (cout <= 4 || (cout <= 16 && cin <= 16)) && !g_wgrad_v1;
  int64_t target;
  if (p.co3) {  // q tiles: the padded rows x the interior columns; 64 input channels per workgroup
    p.tiles_x = cdiv(W, WGCO3_TQW);
    p.tiles_y = cdiv(H + 2, WGCO3_TQH);
    p.groups = cdiv(cin, 64);
    target = 1024;
  } else if (p.small) {  // VALU reduction (wgrad_smallco_kernel)
    const int cg = cout <= 4 ? 4 : 1;  // input channels per workgroup (accumulators: cout x cg x 9)
    p.tiles_x = cdiv(W, SC_TW);
    p.tiles_y = cdiv(H, SC_TH);
    p.groups = cdiv(cin, cg);
    target = 2048;
  } else {
    p.tiles_x = cdiv(W, WG_TW);
    p.tiles_y = cdiv(H, WG_TH);
    p.groups = cdiv(cout, WG_CO) * cdiv(cin, WG_CI);
    target = 1024;  // ~1024 workgroups (4 per CU); each sweeps a contiguous range of pixel tiles
  }
  p.ntiles = (int64_t)p.tiles_x * p.tiles_y * n;
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(p.ntiles, (target + p.groups - 1) / p.groups));
  p.tiles_per_block = (p.ntiles + splits - 1) / splits;
  p.splits = (p.ntiles + p.tiles_per_block - 1) / p.tiles_per_block;
  return p;
}

void wgrad_env() {
  static const int v1 = [] {
    const char* v = getenv("AST_WGRAD_V1");
    return v ? atoi(v) : 0;
  }();
  g_wgrad_v1 = v1;
  static const int co3 = [] {
    const char* v = getenv("AST_WGRAD_CO3");
    return v ? atoi(v) : 1;
  }();
  g_wgrad_co3 = co3;
}

// partial slots a plan needs: its splits, plus the border-column slots of the Cout <= 3 MFMA form
int64_t wgrad_slots(const WgPlan& p) { return p.splits + (p.co3 ? WGCO3_BORDER_SLOTS : 0); }
}  // namespace

extern "C" {

long long ast_conv3x3_wgrad_workspace_floats(int n, int cin, int h_in, int w_in, int cout, int upsample) {
  if (n <= 0 || cin <= 0 || h_in <= 0 || w_in <= 0 || cout <= 0 || (upsample != 1 && upsample != 2)) return 0;
  wgrad_env();
  const WgPlan p = wgrad_plan(n, cin, h_in, w_in, cout, upsample);
  int64_t slots = wgrad_slots(p);
  if (p.co3)  // an unaligned x falls back to the VALU plan (ast_conv3x3_wgrad_ex_f32)
    slots = std::max<int64_t>(slots, wgrad_slots(wgrad_plan(n, cin, h_in, w_in, cout, upsample, false)));
  return (long long)(slots * ((int64_t)cout * cin * 9 + cout));
}

int ast_conv3x3_wgrad_ex_f32(const float* x, const float* dy, float* dw, float* db, int n, int cin, int h_in,
                             int w_in, int cout, int upsample, int pad_mode, int dy_pitch, long long dy_plane,
                             long long dy_offset, float* workspace, long long workspace_floats, void* stream) {
  if (!x || !dy || !dw || !workspace) return AST_E_NULLPTR;
  if (n <= 0 || cin <= 0 || h_in <= 0 || w_in <= 0 || cout <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (pad_mode != 0 && pad_mode != 1) return AST_E_UNSUPPORTED;
  const int H = h_in * upsample, W = w_in * upsample;
  if (pad_mode == 1 && (H < 2 || W < 2)) return AST_E_SHAPE;
  if (dy_pitch == 0) {
    dy_pitch = W;
    dy_plane = (long long)H * W;
    dy_offset = 0;
  }
  if (dy_pitch < W || dy_plane < (long long)H * dy_pitch || dy_offset < 0) return AST_E_SHAPE;
  if (workspace_floats < ast_conv3x3_wgrad_workspace_floats(n, cin, h_in, w_in, cout, upsample)) return AST_E_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  wgrad_env();
  // the MFMA form's 16-byte row loads need a 16-byte aligned x
  const WgPlan p = wgrad_plan(n, cin, h_in, w_in, cout, upsample, ((uintptr_t)x & 15) == 0);
  const int64_t wcount = (int64_t)cout * cin * 9;
  if (p.co3) {
    WgCo3Args c{};
    c.x = x; c.dy = dy;
    const int64_t nslot = wgrad_slots(p);
    c.dw = workspace;                                     // [slots][cout][cin][9]
    c.db = db ? workspace + nslot * wcount : nullptr;     // [slots][cout]
    c.N = n; c.Cin = cin; c.Hin = h_in; c.Win = w_in; c.Cout = cout; c.reflect = pad_mode; c.up = upsample;
    c.dy_pitch = dy_pitch; c.dy_plane = dy_plane; c.dy_off = dy_offset;
    c.tiles_x = p.tiles_x; c.tiles_y = p.tiles_y; c.cgroups = p.groups;
    c.ntiles = p.ntiles; c.tiles_per_block = p.tiles_per_block; c.splits = p.splits;
    int e = launch_wgrad_co3(c, s);
    if (e) return e;
    // the slots summed in slot order (the border-column slots last, present with reflect padding)
    const int64_t slots = pad_mode ? nslot : p.splits;
    hipError_t he = ast_det::reduce_cols(workspace, slots, wcount, wcount, 1, 0, dw, 0, false, s);
    if (he == hipSuccess && db) he = ast_det::reduce_cols(c.db, slots, cout, cout, 1, 0, db, 0, false, s);
    return (int)he;
  }
  WgArgs a{};
  a.x = x; a.dy = dy;
  a.dw = workspace;                                      // [splits][cout][cin][9]
  a.db = db ? workspace + p.splits * wcount : nullptr;  // [splits][cout]
  a.N = n; a.Cin = cin; a.Hin = h_in; a.Win = w_in; a.Cout = cout; a.reflect = pad_mode;
  a.dy_pitch = dy_pitch; a.dy_plane = dy_plane; a.dy_off = dy_offset;
  a.tiles_x = p.tiles_x;
  a.tiles_y = p.tiles_y;
  a.ntiles = p.ntiles;
  a.tiles_per_block = p.tiles_per_block;
  const int64_t nblk = p.splits * p.groups;
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  if (p.small) {
    const dim3 grid((unsigned)nblk);
    if (cout <= 3) {
      if (upsample == 2) hipLaunchKernelGGL((wgrad_smallco_kernel<3, 4, 2>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad_smallco_kernel<3, 4, 1>), grid, dim3(256), 0, s, a);
    } else if (cout == 4) {
      if (upsample == 2) hipLaunchKernelGGL((wgrad_smallco_kernel<4, 4, 2>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad_smallco_kernel<4, 4, 1>), grid, dim3(256), 0, s, a);
    } else {
      if (upsample == 2) hipLaunchKernelGGL((wgrad_smallco_kernel<16, 1, 2>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((wgrad_smallco_kernel<16, 1, 1>), grid, dim3(256), 0, s, a);
    }
  } else {
    const bool aligned = cin % WG_CI == 0 && cout % WG_CO == 0 && W % WG_TW == 0 && H % WG_TH == 0 && w_in % 4 == 0 &&
                         a.ntiles < 0x7fffffff && (int64_t)n * cin * h_in * w_in < 0x7fffffffLL &&
                         (int64_t)cout * dy_plane < 0x7fffffffLL && !g_wgrad_v1;
    static const int wver = [] {
      const char* v = getenv("AST_WGRAD_VERSION");   // 2 = the fp32 MFMA wgrad2 kernel (A/B measurements)
      return v ? atoi(v) : 3;
    }();
    if (aligned && wver >= 3) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)wgrad3_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  Wg3Cfg<1>::LDS);
        (void)hipFuncSetAttribute((const void*)wgrad3_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  Wg3Cfg<2>::LDS);
        attr = true;
      }
      if (upsample == 2)
        hipLaunchKernelGGL(wgrad3_kernel<2>, dim3((unsigned)nblk), dim3(256), Wg3Cfg<2>::LDS, s, a);
      else
        hipLaunchKernelGGL(wgrad3_kernel<1>, dim3((unsigned)nblk), dim3(256), Wg3Cfg<1>::LDS, s, a);
    } else if (aligned && upsample == 2)
      hipLaunchKernelGGL(wgrad2_kernel<2>, dim3((unsigned)nblk), dim3(256), WgCfg<2>::LDS, s, a);
    else if (aligned)
      hipLaunchKernelGGL(wgrad2_kernel<1>, dim3((unsigned)nblk), dim3(256), WgCfg<1>::LDS, s, a);
    else if (upsample == 2)
      hipLaunchKernelGGL(wgrad_kernel<2>, dim3((unsigned)nblk), dim3(256), WgCfg<2>::LDS, s, a);
    else
      hipLaunchKernelGGL(wgrad_kernel<1>, dim3((unsigned)nblk), dim3(256), WgCfg<1>::LDS, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  // the splits' partials, summed in split order
  e = ast_det::reduce_cols(workspace, p.splits, wcount, wcount, 1, 0, dw, 0, false, s);
  if (e == hipSuccess && db) e = ast_det::reduce_cols(a.db, p.splits, cout, cout, 1, 0, db, 0, false, s);
  return (int)e;
}

int ast_conv3x3_wgrad_f32(const float* x, const float* dy, float* dw, float* db, int n, int cin, int h_in, int w_in,
                          int cout, int upsample, int pad_mode, float* workspace, long long workspace_floats,
                          void* stream) {
  return ast_conv3x3_wgrad_ex_f32(x, dy, dw, db, n, cin, h_in, w_in, cout, upsample, pad_mode, 0, 0, 0, workspace,
                                  workspace_floats, stream);
}

}  // extern "C"
