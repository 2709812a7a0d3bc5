// Backward of the 3x3 conv blocks for gfx950 (training step).
//
// Input gradient ("dgrad"): dX = conv3x3_same(dY, W^T flipped) with zero padding — the forward
// MFMA kernel run on a transposed+flipped weight pack (ast_conv3x3_pack_weights_ex_f32). For the
// decoder's [Upsample] + ReflectionPad + Conv that gives the gradient of the *padded* input at
// its interior; the 4 border lines are computed here (dgrad_border_kernel) and the reflect-pad /
// nearest-upsample adjoint folds everything back onto the source grid (pad_up_adjoint_kernel).
//
// Weight gradient ("wgrad"): dW[co][ci][tap] = sum_pix dY[co][pix] * P[ci][pix+tap] as an MFMA
// fp32 GEMM with K = pixels: per workgroup 64 output x 32 input channels x 9 taps, looping over a
// range of 4x32-pixel tiles, fp32 atomics into dW at the end (the pixel range is split across
// workgroups). P is staged exactly like the forward kernel's source tile (zero/reflect pad and
// upsample resolved by the LDS read address).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"

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
// W'[o=ci][i=co][ky][kx] = W[co][ci][2-ky][2-kx] * (row_scale ? row_scale[ci] : 1)
__global__ void pack_tf_kernel(const float* __restrict__ w, float* __restrict__ wp, int cout, int cin, int pad_out,
                               int pad_in, const float* __restrict__ scale) {
  // forward-pack view of W': "cout" = cin, "cin" = cout
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

// Border lines of dP = full correlation of dY (N, Cout, H, W) with W (the gradient of the
// reflect-padded input at padded rows 0 and H+1 and padded columns 0 and W+1).
// border layout per (n, ci): [top (W+2)][bottom (W+2)][left (H)][right (H)].
__global__ void dgrad_border_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                    float* __restrict__ border, int N, int Cout, int Cin, int H, int W) {
  const int L = 2 * (W + 2) + 2 * H;
  const int64_t total = (int64_t)N * Cin * L;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx % L);
    const int64_t nc = idx / L;
    const int ci = (int)(nc % Cin);
    const int n = (int)(nc / Cin);
    int py, px;
    if (e < W + 2) { py = 0; px = e; }
    else if (e < 2 * (W + 2)) { py = H + 1; px = e - (W + 2); }
    else if (e < 2 * (W + 2) + H) { py = 1 + e - 2 * (W + 2); px = 0; }
    else { py = 1 + e - 2 * (W + 2) - H; px = W + 1; }
    // dP[py][px] = sum_{co,ky,kx} dY[co][py-ky][px-kx] * W[co][ci][ky][kx]
    float s = 0.f;
    for (int co = 0; co < Cout; ++co) {
      const float* d = dy + ((int64_t)n * Cout + co) * H * W;
      const float* wk = w + ((int64_t)co * Cin + ci) * 9;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int oy = py - ky;
        if (oy < 0 || oy >= H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int ox = px - kx;
          if (ox < 0 || ox >= W) continue;
          s = fmaf(d[(int64_t)oy * W + ox], wk[ky * 3 + kx], s);
        }
      }
    }
    border[idx] = s;
  }
}

// dx[v] (source grid, h_in x w_in) = sum over padded positions p mapping onto v of dP[p]:
//   interior dP[p] = dpin[p-1] (p in [1, H]); border dP from dgrad_border_kernel.
//   up == 1: p -> u = refl(p-1) = v;   up == 2: p -> u = refl(p-1) -> v = u >> 1.
// mask (optional, same shape as dx): dx = mask > 0 ? dx : 0 (ReLU of the layer that made x).
__global__ void pad_up_adjoint_kernel(const float* __restrict__ dpin, const float* __restrict__ border,
                                      const float* __restrict__ mask, float* __restrict__ dx, int64_t planes,
                                      int h_in, int w_in, int up) {
  const int H = h_in * up, W = w_in * up;
  const int L = 2 * (W + 2) + 2 * H;
  const int64_t total = planes * h_in * w_in;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int vx = (int)(idx % w_in);
    const int vy = (int)((idx / w_in) % h_in);
    const int64_t p = idx / ((int64_t)h_in * w_in);
    // padded rows/cols (as dP indices) that land on vy / vx
    int rows[4], nr = 0, cols[4], nc = 0;
    for (int k = 0; k < up; ++k) { rows[nr++] = up * vy + k + 1; cols[nc++] = up * vx + k + 1; }
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
    const float* dp = dpin + p * H * W;
    const float* bd = border + p * L;
    float s = 0.f;
    for (int a = 0; a < nr; ++a) {
      const int r = rows[a];
      for (int b = 0; b < nc; ++b) {
        const int c = cols[b];
        float v;
        if (r == 0) v = bd[c];
        else if (r == H + 1) v = bd[(W + 2) + c];
        else if (c == 0) v = bd[2 * (W + 2) + (r - 1)];
        else if (c == W + 1) v = bd[2 * (W + 2) + H + (r - 1)];
        else v = dp[(int64_t)(r - 1) * W + (c - 1)];
        s += v;
      }
    }
    if (mask && !(mask[idx] > 0.f)) s = 0.f;
    dx[idx] = s;
  }
}

// dx = g * (mask > 0) (ReLU backward for an input gradient with no pad/upsample adjoint).
__global__ void relu_mask_kernel(const float* __restrict__ g, const float* __restrict__ mask, float* __restrict__ out,
                                 int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mask[i] > 0.f ? g[i] : 0.f;
}

// ------------------------------------------------------------------------------------------
// Weight gradient.
// ------------------------------------------------------------------------------------------
constexpr int WG_CO = 64, WG_CI = 32, WG_TH = 4, WG_TW = 32, WG_PIX = WG_TH * WG_TW;

template <int UP>
struct WgCfg {
  static constexpr int SW = WG_TW / UP;
  static constexpr int SR = WG_TH / UP + 2;
  static constexpr int RS = SW + 8;
  static constexpr int PS = SR * RS + 1;     // per-channel plane stride (odd: ci on lanes is conflict-free)
  static constexpr int DS = WG_PIX + 1;      // per-co stride of the dY tile
  static constexpr int LDS = (WG_CI * PS + WG_CO * DS) * 4;
};

template <int UP>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                       float* __restrict__ dw, float* __restrict__ db, int N, int Cin,
                                                       int Hin, int Win, int Cout, int reflect, int tiles_x,
                                                       int tiles_y, int64_t tiles_per_block, int64_t ntiles) {
  using C = WgCfg<UP>;
  constexpr int SW = C::SW, SR = C::SR, RS = C::RS, PS = C::PS, DS = C::DS;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ps = smem;                  // [WG_CI][PS]
  float* Ds = smem + WG_CI * PS;     // [WG_CO][DS]
  const int H = Hin * UP, W = Win * UP;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wco = wave & 1, wtap = wave >> 1;      // co half, tap group {0..4} / {5..8}
  const int co_groups = (Cout + WG_CO - 1) / WG_CO;
  const int ci_groups = (Cin + WG_CI - 1) / WG_CI;
  int b = blockIdx.x;
  const int cog = b % co_groups;
  b /= co_groups;
  const int cig = b % ci_groups;
  const int64_t split = b / ci_groups;
  const int co0 = cog * WG_CO, ci0 = cig * WG_CI;

  f32x16 acc[5];
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bacc = 0.f;  // bias gradient partial (tid < 64 -> co0 + tid), only for cig == 0

  const int64_t t0 = split * tiles_per_block;
  const int64_t t1 = min(ntiles, t0 + tiles_per_block);
  for (int64_t tile = t0; tile < t1; ++tile) {
    int64_t tt = tile;
    const int tx = (int)(tt % tiles_x);
    tt /= tiles_x;
    const int ty = (int)(tt % tiles_y);
    const int n = (int)(tt / tiles_y);
    const int x0 = tx * WG_TW, y0 = ty * WG_TH;
    const int sx0 = x0 / UP, sy0 = y0 / UP - 1;
    __syncthreads();
    // stage P (source tile with halo, scalar gather: simple and general)
    const float* xin = x + (int64_t)n * Cin * Hin * Win;
    for (int e = tid; e < WG_CI * SR * (SW + 2); e += 256) {
      const int col = e % (SW + 2);
      const int cr = e / (SW + 2);
      const int r = cr % SR, c = cr / SR;
      const int ci = ci0 + c;
      const int sy = src_index<UP>(sy0 + r, Hin, reflect);
      const int sx = src_index<UP>(sx0 - 1 + col, Win, reflect);
      float v = 0.f;
      if (ci < Cin && sy >= 0 && sx >= 0) v = xin[(int64_t)ci * Hin * Win + (int64_t)sy * Win + sx];
      Ps[c * PS + r * RS + 3 + col] = v;
    }
    // stage dY tile [co][pix] (pix = row*32 + col), zero outside
    const float* dyn = dy + (int64_t)n * Cout * H * W;
    for (int e = tid; e < WG_CO * WG_PIX; e += 256) {
      const int pix = e % WG_PIX, c = e / WG_PIX;
      const int co = co0 + c, yy = y0 + pix / WG_TW, xx = x0 + pix % WG_TW;
      float v = 0.f;
      if (co < Cout && yy < H && xx < W) v = dyn[(int64_t)co * H * W + (int64_t)yy * W + xx];
      Ds[c * DS + pix] = v;
    }
    __syncthreads();
    if (cig == 0 && tid < WG_CO) {
      float s = 0.f;
      for (int pix = 0; pix < WG_PIX; ++pix) s += Ds[tid * DS + pix];
      bacc += s;
    }
    // K loop over pixel pairs
#pragma unroll 2
    for (int kp = 0; kp < WG_PIX / 2; ++kp) {
      const int pix = 2 * kp + h;
      const int prow = pix / WG_TW, pcol = pix % WG_TW;
      const float a = Ds[(wco * 32 + l32) * DS + pix];
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int tap = wtap * 5 + t;
        if (tap < 9) {
          const int ky = tap / 3, kx = tap % 3;
          const int orow = prow + ky - 1;
          const int srow = (UP == 1) ? orow + 1 : (orow >> 1) + 1;
          const int scol = 3 + (((x0 + pcol + kx - 1) >> (UP - 1)) - sx0 + 1);
          const float bv = Ps[l32 * PS + srow * RS + scol];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[t], 0, 0, 0);
        }
      }
    }
  }
  // C[i = co][j = ci]: col j = l32, rows i = (r&3)+8(r>>2)+4h
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int tap = wtap * 5 + t;
    if (tap >= 9) continue;
    const int ci = ci0 + l32;
    if (ci >= Cin) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wco * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co < Cout) atomicAdd(dw + ((int64_t)co * Cin + ci) * 9 + tap, acc[t][r]);
    }
  }
  if (db && cig == 0 && tid < WG_CO && co0 + tid < Cout) atomicAdd(db + co0 + tid, bacc);
}

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
  return (int)hipGetLastError();
}

int ast_conv_act_backward_f32(const float* pre, const float* g_pre, const float* g_act, const float* g_pool,
                              float* dy, long long planes, int h, int w, void* stream) {
  if (!pre || !dy) return AST_E_NULLPTR;
  if (planes <= 0 || h <= 0 || w <= 0) return AST_E_SHAPE;
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

int ast_conv3x3_dgrad_border_f32(const float* dy, const float* w, float* border, int n, int cout, int cin, int h,
                                 int w_, void* stream) {
  if (!dy || !w || !border) return AST_E_NULLPTR;
  if (n <= 0 || cout <= 0 || cin <= 0 || h <= 0 || w_ <= 0) return AST_E_SHAPE;
  const int64_t total = (int64_t)n * cin * (2 * (w_ + 2) + 2 * h);
  hipLaunchKernelGGL(dgrad_border_kernel, dim3(grid1(total)), dim3(256), 0, (hipStream_t)stream, dy, w, border, n,
                     cout, cin, h, w_);
  return (int)hipGetLastError();
}

int ast_pad_up_adjoint_f32(const float* dp_interior, const float* border, const float* mask, float* dx,
                           long long planes, int h_in, int w_in, int upsample, void* stream) {
  if (!dp_interior || !border || !dx) return AST_E_NULLPTR;
  if (planes <= 0 || h_in <= 0 || w_in <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (h_in * upsample < 2 || w_in * upsample < 2) return AST_E_SHAPE;
  hipLaunchKernelGGL(pad_up_adjoint_kernel, dim3(grid1(planes * h_in * w_in)), dim3(256), 0, (hipStream_t)stream,
                     dp_interior, border, mask, dx, (int64_t)planes, h_in, w_in, upsample);
  return (int)hipGetLastError();
}

int ast_conv3x3_wgrad_f32(const float* x, const float* dy, float* dw, float* db, int n, int cin, int h_in, int w_in,
                          int cout, int upsample, int pad_mode, void* stream) {
  if (!x || !dy || !dw) return AST_E_NULLPTR;
  if (n <= 0 || cin <= 0 || h_in <= 0 || w_in <= 0 || cout <= 0) return AST_E_SHAPE;
  if (upsample != 1 && upsample != 2) return AST_E_UNSUPPORTED;
  if (pad_mode != 0 && pad_mode != 1) return AST_E_UNSUPPORTED;
  const int H = h_in * upsample, W = w_in * upsample;
  if (pad_mode == 1 && (H < 2 || W < 2)) return AST_E_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * (size_t)cout * cin * 9, s);
  if (e != hipSuccess) return (int)e;
  if (db) {
    e = hipMemsetAsync(db, 0, sizeof(float) * (size_t)cout, s);
    if (e != hipSuccess) return (int)e;
  }
  const int tiles_x = cdiv(W, WG_TW), tiles_y = cdiv(H, WG_TH);
  const int64_t ntiles = (int64_t)tiles_x * tiles_y * n;
  const int groups = cdiv(cout, WG_CO) * cdiv(cin, WG_CI);
  // ~2048 workgroups; each sweeps a contiguous range of pixel tiles
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(ntiles, (2048 + groups - 1) / groups));
  const int64_t per = (ntiles + splits - 1) / splits;
  splits = (ntiles + per - 1) / per;
  const int64_t nblk = splits * groups;
  if (nblk >= 0x7fffffff) return AST_E_SHAPE;
  if (upsample == 2) {
    hipLaunchKernelGGL(wgrad_kernel<2>, dim3((unsigned)nblk), dim3(256), WgCfg<2>::LDS, s, x, dy, dw, db, n, cin,
                       h_in, w_in, cout, pad_mode, tiles_x, tiles_y, per, ntiles);
  } else {
    hipLaunchKernelGGL(wgrad_kernel<1>, dim3((unsigned)nblk), dim3(256), WgCfg<1>::LDS, s, x, dy, dw, db, n, cin,
                       h_in, w_in, cout, pad_mode, tiles_x, tiles_y, per, ntiles);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
