// Depthwise k x k conv (k 3|5, stride 1|2, reflect padding (k-1)/2) for the MobileNet-variant
// training path (DepthWiseConv's depthwise layer, mobilenetv2.py:148-149, :116-117) with its input
// and weight gradients, fp32. At the AST's 160^2 training size these planes are the step's largest
// tensors (decoder blocks: 8 x 240 x 160 x 160), so all three kernels are HBM-bound and LDS-tiled:
//   tile   TH x TW outputs of one plane (TW 16|32|64 lanes along a row, R rows per thread,
//          TH = R * 256 / TW), chosen per plane size by dw_plan to waste the fewest lanes;
//   fwd    stage the tile's reflect-padded input window in LDS (each element read from HBM once),
//          every thread slides down its column keeping R accumulators (K LDS reads per input row);
//          taps are summed in (ky, kx) order, as the reference's conv2d loop nest reads them;
//   dgrad  one pass: dpad (the gradient w.r.t. the padded input) for the tile plus a 2P halo is
//          built in LDS from the staged output gradient, then folded through the reflection
//          (border pixels add the padded positions that reflect onto them);
//   wgrad  stage the input window, keep the K*K partial sums of R outputs in registers over up to
//          `tpb` tiles of one plane, reduce across the workgroup, store one partial row per
//          (image, tile group); ast_det::reduce_cols sums a channel's rows in order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ast_hip.h"
#include "det.h"

namespace {

constexpr int kT = 256;

// reflect once (pad < n), then clamp: window positions past what any output reads are loaded
// from a valid address and never used
__device__ __forceinline__ int reflc(int i, int n) {
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * (n - 1) - i : i;
  return min(max(i, 0), n - 1);
}

template <int K, int S, int TW, int R>
struct Geo {
  static constexpr int P = (K - 1) / 2, KK = K * K;
  static constexpr int NS = kT / TW, TH = NS * R;           // strips (one per R rows) per tile
  static constexpr int IH = (TH - 1) * S + K, IW = (TW - 1) * S + K;  // input window of a tile
  static constexpr int IWP = IW + 1;
  static constexpr int SR = (R - 1) * S + K;                 // input rows one strip reads
};

// Hardswish and its derivative (torch's formulas; the expressions of mbtrain.hip's elt<0> / elt<1>,
// so a fused activation is bit-identical to the materialised one)
__device__ __forceinline__ float hswish(float a) { return a * fminf(fmaxf(a + 3.f, 0.f), 6.f) / 6.f; }
__device__ __forceinline__ float hswish_bwd(float a, float g) {
  return a < -3.f ? 0.f : (a <= 3.f ? g * (a / 3.f + 0.5f) : g);
}

// stage x[plane] rows iy0.., cols ix0.. (reflected) into xs[IH][IWP]; act: the conv's input is
// hardswish(x) (DepthWiseConv's Hardswish -> depthwise conv, mobilenetv2.py:144-149, fused)
template <class G>
__device__ __forceinline__ void stage_input(float* xs, const float* __restrict__ xp, int iy0, int ix0, int h, int wd,
                                            bool act) {
  for (int e = threadIdx.x; e < G::IH * G::IW; e += kT) {
    const int r = e / G::IW, c = e - r * G::IW;
    const float v = xp[reflc(iy0 + r, h) * wd + reflc(ix0 + c, wd)];
    xs[r * G::IWP + c] = act ? hswish(v) : v;
  }
}

template <int K, int S, int TW, int R>
__global__ __launch_bounds__(kT) void dwt_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     float* __restrict__ y, int planes, int c, int h, int wd, int ho,
                                                     int wo, int tiles_x, int act) {
  using G = Geo<K, S, TW, R>;
  __shared__ float xs[G::IH * G::IWP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lx = lane % TW, strip = wave * (64 / TW) + lane / TW;
  const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
  const int oy0 = ty * G::TH, ox0 = tx * TW;
  for (int pl = blockIdx.y; pl < planes; pl += gridDim.y) {
    const float* wc = w + (pl % c) * G::KK;
    float wr[G::KK];
#pragma unroll
    for (int t = 0; t < G::KK; ++t) wr[t] = wc[t];
    __syncthreads();  // the previous plane's window is consumed
    stage_input<G>(xs, x + (int64_t)pl * h * wd, oy0 * S - G::P, ox0 * S - G::P, h, wd, act != 0);
    __syncthreads();
    float acc[R];
#pragma unroll
    for (int j = 0; j < R; ++j) acc[j] = 0.f;
    const float* base = xs + strip * R * S * G::IWP + lx * S;
#pragma unroll
    for (int rr = 0; rr < G::SR; ++rr) {
      float v[K];
#pragma unroll
      for (int kx = 0; kx < K; ++kx) v[kx] = base[rr * G::IWP + kx];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int ky = rr - j * S;
        if (ky >= 0 && ky < K) {
#pragma unroll
          for (int kx = 0; kx < K; ++kx) acc[j] = fmaf(wr[ky * K + kx], v[kx], acc[j]);
        }
      }
    }
    const int ox = ox0 + lx;
    float* yp = y + (int64_t)pl * ho * wo;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int oy = oy0 + strip * R + j;
      if (oy < ho && ox < wo) yp[oy * wo + ox] = acc[j];
    }
  }
}

// dgrad: tile = TH x TW pixels of the INPUT plane (h x wd)
template <int K, int S, int TW, int R>
struct DGeo {
  using G = Geo<K, S, TW, R>;
  static constexpr int P = G::P;
  static constexpr int QH = G::TH + 4 * P, QW = TW + 4 * P;       // dpad window (padded coords)
  static constexpr int QWP = QW + 1;
  static constexpr int GH = (QH + K - 2) / S + 2, GW = (QW + K - 2) / S + 2;  // output-gradient window
  static constexpr int GWP = GW + 1;
  static constexpr int RR = 4;                                    // dpad rows per item (stride 1)
};

__device__ __forceinline__ int floor_div2(int a) { return a >> 1; }  // arithmetic shift: floor

template <int K, int S, int TW, int R>
__global__ __launch_bounds__(kT) void dwt_dgrad_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                       const float* __restrict__ xa, float* __restrict__ dx,
                                                       int planes, int c, int h, int wd, int ho, int wo,
                                                       int tiles_x) {
  using G = Geo<K, S, TW, R>;
  using D = DGeo<K, S, TW, R>;
  constexpr int P = G::P;
  __shared__ float gs[D::GH * D::GWP];
  __shared__ float ds[D::QH * D::QWP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lx = lane % TW, strip = wave * (64 / TW) + lane / TW;
  const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
  const int iy0 = ty * G::TH, ix0 = tx * TW;
  const int qy0 = iy0 - P, qx0 = ix0 - P;  // dpad window origin (padded coordinates)
  // output-gradient window origin: the lowest o with o * S + t = q for q >= q0, t < K
  const int gy0 = S == 1 ? qy0 - (K - 1) : floor_div2(qy0 - (K - 1));
  const int gx0 = S == 1 ? qx0 - (K - 1) : floor_div2(qx0 - (K - 1));
  // the pad positions reflecting onto this thread's column (-1 = none), in window coordinates
  const int ix = ix0 + lx;
  const int cx1 = (ix >= 1 && ix <= P) ? P - ix - qx0 : -1;
  const int cx2 = (ix >= wd - 1 - P && ix <= wd - 2) ? 2 * (wd - 1) - ix + P - qx0 : -1;
  for (int pl = blockIdx.y; pl < planes; pl += gridDim.y) {
    const float* wc = w + (pl % c) * G::KK;
    float wr[G::KK];
#pragma unroll
    for (int t = 0; t < G::KK; ++t) wr[t] = wc[t];
    const float* gp = g + (int64_t)pl * ho * wo;
    __syncthreads();
    for (int e = threadIdx.x; e < D::GH * D::GW; e += kT) {
      const int r = e / D::GW, cc = e - r * D::GW;
      const int oy = gy0 + r, ox = gx0 + cc;
      gs[r * D::GWP + cc] = (oy >= 0 && oy < ho && ox >= 0 && ox < wo) ? gp[oy * wo + ox] : 0.f;
    }
    __syncthreads();
    // dpad[q] = sum over taps t with q - t = S * o of g[o] * w[t]
    if (S == 1) {
      constexpr int NSTR = (D::QH + D::RR - 1) / D::RR;
      for (int it = threadIdx.x; it < D::QW * NSTR; it += kT) {
        const int qc = it % D::QW, q0 = (it / D::QW) * D::RR;
        float acc[D::RR];
#pragma unroll
        for (int j = 0; j < D::RR; ++j) acc[j] = 0.f;
        // window row of g for dpad row q and tap ty: q - ty + K - 1 (column likewise)
#pragma unroll
        for (int a = 0; a < D::RR + K - 1; ++a) {
          float v[K];
          const int gr = min(q0 + a, D::GH - 1);
#pragma unroll
          for (int b = 0; b < K; ++b) v[b] = gs[gr * D::GWP + qc + b];
#pragma unroll
          for (int j = 0; j < D::RR; ++j) {
            const int tyy = j + K - 1 - a;
            if (tyy >= 0 && tyy < K) {
#pragma unroll
              for (int b = 0; b < K; ++b) acc[j] = fmaf(v[b], wr[tyy * K + (K - 1 - b)], acc[j]);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < D::RR; ++j)
          if (q0 + j < D::QH) ds[(q0 + j) * D::QWP + qc] = acc[j];
      }
    } else {
      for (int it = threadIdx.x; it < D::QH * D::QW; it += kT) {
        const int qr = it / D::QW, qc = it - qr * D::QW;
        const int q = qy0 + qr, qx = qx0 + qc;
        float acc = 0.f;
#pragma unroll
        for (int tyy = 0; tyy < K; ++tyy) {
          if (((q - tyy) & 1) != 0) continue;
          const int gr = floor_div2(q - tyy) - gy0;
#pragma unroll
          for (int txx = 0; txx < K; ++txx) {
            if (((qx - txx) & 1) != 0) continue;
            acc = fmaf(gs[gr * D::GWP + floor_div2(qx - txx) - gx0], wr[tyy * K + txx], acc);
          }
        }
        ds[qr * D::QWP + qc] = acc;
      }
    }
    __syncthreads();
    // fold the reflection: dx[i] = dpad[i + P] + the pad positions that reflect onto i
    float* dxp = dx + (int64_t)pl * h * wd;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int iy = iy0 + strip * R + j;
      if (iy >= h || ix >= wd) continue;
      const int ry0 = iy + P - qy0, rx0 = ix + P - qx0;
      const int ry1 = (iy >= 1 && iy <= P) ? P - iy - qy0 : -1;
      const int ry2 = (iy >= h - 1 - P && iy <= h - 2) ? 2 * (h - 1) - iy + P - qy0 : -1;
      float acc = ds[ry0 * D::QWP + rx0];
      if (cx1 >= 0) acc += ds[ry0 * D::QWP + cx1];
      if (cx2 >= 0) acc += ds[ry0 * D::QWP + cx2];
      if (ry1 >= 0) {
        acc += ds[ry1 * D::QWP + rx0];
        if (cx1 >= 0) acc += ds[ry1 * D::QWP + cx1];
        if (cx2 >= 0) acc += ds[ry1 * D::QWP + cx2];
      }
      if (ry2 >= 0) {
        acc += ds[ry2 * D::QWP + rx0];
        if (cx1 >= 0) acc += ds[ry2 * D::QWP + cx1];
        if (cx2 >= 0) acc += ds[ry2 * D::QWP + cx2];
      }
      // xa: the conv input was hardswish(xa): the gradient continues through it
      dxp[iy * wd + ix] = xa ? hswish_bwd(xa[(int64_t)pl * h * wd + iy * wd + ix], acc) : acc;
    }
  }
}

// wgrad: part[(ch * n + img) * groups + group][tap]; grid (groups, n, c)
template <int K, int S, int TW, int R>
__global__ __launch_bounds__(kT) void dwt_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                       float* __restrict__ part, int c, int h, int wd, int ho, int wo,
                                                       int tiles_x, int ntiles, int tpb, int act) {
  using G = Geo<K, S, TW, R>;
  constexpr int KK = G::KK;
  __shared__ float xs[G::IH * G::IWP];
  __shared__ float sh[kT / 64][KK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lx = lane % TW, strip = wave * (64 / TW) + lane / TW;
  const int ch = blockIdx.z, img = blockIdx.y;
  const int64_t pl = (int64_t)img * c + ch;
  const float* xp = x + pl * h * wd;
  const float* gp = g + pl * ho * wo;
  float acc[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) acc[t] = 0.f;
  const int t_end = min(ntiles, (int)(blockIdx.x + 1) * tpb);
  for (int tile = blockIdx.x * tpb; tile < t_end; ++tile) {
    const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const int oy0 = ty * G::TH, ox0 = tx * TW, ox = ox0 + lx;
    __syncthreads();
    stage_input<G>(xs, xp, oy0 * S - G::P, ox0 * S - G::P, h, wd, act != 0);
    float gv[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int oy = oy0 + strip * R + j;
      gv[j] = (oy < ho && ox < wo) ? gp[oy * wo + ox] : 0.f;
    }
    __syncthreads();
    const float* base = xs + strip * R * S * G::IWP + lx * S;
#pragma unroll
    for (int rr = 0; rr < G::SR; ++rr) {
      float v[K];
#pragma unroll
      for (int kx = 0; kx < K; ++kx) v[kx] = base[rr * G::IWP + kx];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int ky = rr - j * S;
        if (ky >= 0 && ky < K) {
#pragma unroll
          for (int kx = 0; kx < K; ++kx) acc[ky * K + kx] = fmaf(gv[j], v[kx], acc[ky * K + kx]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    float v = acc[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    acc[t] = v;
  }
  if (lane == 0) {
#pragma unroll
    for (int t = 0; t < KK; ++t) sh[wave][t] = acc[t];
  }
  __syncthreads();
  if (threadIdx.x < KK) {
    const int t = threadIdx.x;
    const int64_t row = ((int64_t)ch * gridDim.y + img) * gridDim.x + blockIdx.x;
    part[row * KK + t] = (sh[0][t] + sh[1][t]) + (sh[2][t] + sh[3][t]);
  }
}

// ------------------------------------------------------------------------------------------------
// host: tile plan and dispatch
// ------------------------------------------------------------------------------------------------
struct DwPlan {
  int tw, r, th, tiles_x, tiles_y;
};

// the (TW, R) among {16, 32, 64} x {2, 4, 8} that wastes the fewest lanes on an H x W plane;
// ties go to the larger tile (fewer halo re-reads)
DwPlan dw_plan(int H, int W) {
  DwPlan best{64, 8, 32, 1, 1};
  double best_u = -1.0;
  const int tws[3] = {64, 32, 16}, rs[3] = {8, 4, 2};
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) {
      const int tw = tws[a], r = rs[b], th = r * kT / tw;
      const int tx = (W + tw - 1) / tw, ty = (H + th - 1) / th;
      const double u = (double)H * W / ((double)tx * tw * ty * th);
      if (u > best_u * 1.0001) {
        best_u = u;
        best = DwPlan{tw, r, th, tx, ty};
      }
    }
  return best;
}

constexpr int kTpb = 8;  // wgrad: tiles of one plane per workgroup

int wgrad_groups(const DwPlan& p) {
  const int nt = p.tiles_x * p.tiles_y;
  return (nt + kTpb - 1) / kTpb;
}

template <template <int, int, int, int> class F, typename... A>
void dw_launch(int k, int s, const DwPlan& p, A... args) {
#define AST_DWT_R(KK, SS, TW)                       \
  if (p.r == 2) F<KK, SS, TW, 2>::run(args...);      \
  else if (p.r == 4) F<KK, SS, TW, 4>::run(args...); \
  else F<KK, SS, TW, 8>::run(args...);
#define AST_DWT_TW(KK, SS)                 \
  if (p.tw == 16) { AST_DWT_R(KK, SS, 16) } \
  else if (p.tw == 32) { AST_DWT_R(KK, SS, 32) } \
  else { AST_DWT_R(KK, SS, 64) }
  if (k == 3 && s == 1) { AST_DWT_TW(3, 1) }
  else if (k == 3) { AST_DWT_TW(3, 2) }
  else if (s == 1) { AST_DWT_TW(5, 1) }
  else { AST_DWT_TW(5, 2) }
#undef AST_DWT_TW
#undef AST_DWT_R
}

struct DwArgs {
  const float *x, *w, *g;
  float *out, *part;
  int n, c, h, wd, ho, wo, groups, act;
  DwPlan p;
  hipStream_t st;
};

template <int K, int S, int TW, int R>
struct FwdL {
  static void run(const DwArgs& a) {
    const int64_t nc = (int64_t)a.n * a.c;
    const dim3 grid((unsigned)(a.p.tiles_x * a.p.tiles_y), (unsigned)(nc < 65535 ? nc : 65535));
    hipLaunchKernelGGL((dwt_fwd_kernel<K, S, TW, R>), grid, dim3(kT), 0, a.st, a.x, a.w, a.out, (int)nc, a.c, a.h, a.wd,
                       a.ho, a.wo, a.p.tiles_x, a.act);
  }
};

template <int K, int S, int TW, int R>
struct DgradL {
  static void run(const DwArgs& a) {
    const int64_t nc = (int64_t)a.n * a.c;
    const dim3 grid((unsigned)(a.p.tiles_x * a.p.tiles_y), (unsigned)(nc < 65535 ? nc : 65535));
    hipLaunchKernelGGL((dwt_dgrad_kernel<K, S, TW, R>), grid, dim3(kT), 0, a.st, a.g, a.w, a.act ? a.x : nullptr, a.out,
                       (int)nc, a.c, a.h, a.wd, a.ho, a.wo, a.p.tiles_x);
  }
};

template <int K, int S, int TW, int R>
struct WgradL {
  static void run(const DwArgs& a) {
    const dim3 grid((unsigned)a.groups, (unsigned)a.n, (unsigned)a.c);
    hipLaunchKernelGGL((dwt_wgrad_kernel<K, S, TW, R>), grid, dim3(kT), 0, a.st, a.x, a.g, a.part, a.c, a.h, a.wd,
                       a.ho, a.wo, a.p.tiles_x, a.p.tiles_x * a.p.tiles_y, kTpb, a.act);
  }
};

}  // namespace

extern "C" {

long long ast_mbt_dw_workspace_floats(int n, int c, int h, int wd, int k) {
  if (n <= 0 || c <= 0 || h <= 0 || wd <= 0 || (k != 3 && k != 5)) return 0;
  const int p = (k - 1) / 2;
  long long groups = 0;
  for (int s = 1; s <= 2; ++s) {  // mode 2's partial rows, for either stride
    const int ho = (h + 2 * p - k) / s + 1, wo = (wd + 2 * p - k) / s + 1;
    if (ho <= 0 || wo <= 0) continue;
    const long long gr = wgrad_groups(dw_plan(ho, wo));
    groups = gr > groups ? gr : groups;
  }
  return (long long)c * n * groups * k * k;
}

int ast_mbt_dw_act_f32(int mode, const float* x, const float* w, const float* g, float* out, int n, int c, int h,
                       int wd, int k, int s, int act, float* workspace, long long workspace_floats, void* stream) {
  if (!w || !out || ((mode != 1 || act) && !x) || (mode != 0 && !g) || (mode == 2 && !workspace))
    return AST_E_NULLPTR;
  if (act != 0 && act != 1) return AST_E_UNSUPPORTED;
  if (mode < 0 || mode > 2) return AST_E_UNSUPPORTED;
  if (n <= 0 || c <= 0 || h <= 0 || wd <= 0 || (k != 3 && k != 5) || (s != 1 && s != 2)) return AST_E_SHAPE;
  const int p = (k - 1) / 2;
  if (p >= h || p >= wd) return AST_E_SHAPE;  // reflect padding needs pad < size
  const int ho = (h + 2 * p - k) / s + 1, wo = (wd + 2 * p - k) / s + 1;
  const int64_t nc = (int64_t)n * c;
  if (nc * (h + 2 * p) * (wd + 2 * p) >= (1LL << 31) || n > 65535 || c > 65535) return AST_E_SHAPE;  // 32-bit indices
  DwArgs a{x, w, g, out, workspace, n, c, h, wd, ho, wo, 0, act, {}, (hipStream_t)stream};
  if (mode == 0) {
    a.p = dw_plan(ho, wo);
    dw_launch<FwdL>(k, s, a.p, a);
  } else if (mode == 1) {
    a.p = dw_plan(h, wd);  // tiles of the input plane
    dw_launch<DgradL>(k, s, a.p, a);
  } else {
    a.p = dw_plan(ho, wo);
    a.groups = wgrad_groups(a.p);
    const int64_t rows = (int64_t)n * a.groups;  // partial rows per channel, (image, group) order
    if (workspace_floats < (long long)c * rows * k * k) return AST_E_SHAPE;  // workspace too small
    dw_launch<WgradL>(k, s, a.p, a);
    const hipError_t e = ast_det::reduce_cols(workspace, rows, k * k, k * k, c, rows * k * k, out, k * k, false,
                                              (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
  }
  return (int)hipGetLastError();
}

int ast_mbt_dw_f32(int mode, const float* x, const float* w, const float* g, float* out, int n, int c, int h, int wd,
                   int k, int s, float* workspace, long long workspace_floats, void* stream) {
  return ast_mbt_dw_act_f32(mode, x, w, g, out, n, c, h, wd, k, s, 0, workspace, workspace_floats, stream);
}

}  // extern "C"
