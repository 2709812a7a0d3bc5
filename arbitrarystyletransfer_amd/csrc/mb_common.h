// Shared between mobilenet.hip (v1-v3 expand+depthwise kernels, SE, pw, launch dispatch) and
// mb_ed4.hip (the v4 expand+depthwise kernel, compiled separately without SLP vectorisation).
#pragma once
#include <hip/hip_runtime.h>

namespace ast_mb {

// Arguments of one expand (+BN, Hardswish) -> depthwise kxk (+BN, Hardswish) -> SE-pool launch
// (DepthWiseConv, mobilenetv2.py:95-165, up to the SE gate).
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
  float* pool;       // SE-pool partial sums [n][hid][slots]: one slot per output tile of an image,
                     // plain stores (the host sums the slots in order: deterministic)
  int tiles_x, tiles_y;
  int slots;         // output tiles per image (set by the launcher)
  long long* plan;   // non-null: the launcher only stores its slot count here and launches nothing
  int nod;           // pool-only pass of the fused block pair: SE-pool sums, no D (v4 k3 stride 1 only)
};

// The recompute-and-project pass of the fused block pair (expand_dw_pw4_kernel, mb_ed4.hip): the
// expand + depthwise of EdArgs recomputed per output row, the SE-gated pw-linear conv applied from
// registers/LDS, out = wg[n] . D + b2 (+ res); D never reaches HBM.
struct EdpwArgs {
  EdArgs e;           // x1, n, cin, h, w, ho, wo, w1, b1, hid, cin_pad, wdw, bdw (d, pool unused)
  const void* wg;     // [n][cout_pad][hid_pad] bf16 (ast_mb_se_fold)
  const float* b2;    // [cout] or null
  const void* res;    // [n][cout][ho][wo] or null (identity blocks)
  void* out;          // [n][cout][ho][wo]
  int cout, cout_pad, hid_pad;
};

// The launchers' plan-mode exit: the slot count of the launch that would run.
inline bool ed_plan(EdArgs& a, long long slots) {
  a.slots = (int)slots;
  if (a.plan) {
    *a.plan = slots;
    return true;
  }
  return false;
}

// v4 (bf16, no upsample, expand blocks with c1 == cin, k in {3, 5}; stride 1 with cin_pad in
// {16..96, 128}, stride 2 with cin_pad <= 64 and even wo): returns AST_E_UNSUPPORTED when the shape
// is outside that set (the caller falls back to v3 / v1).
int launch_ed4(EdArgs a, int k, int stride, hipStream_t st);

// v5 (mb_ed5.hip: bf16 expand blocks, k 5, stride 1, cin_pad <= 48, wo % 4 == 0): the depthwise on
// the matrix cores (Toeplitz form); AST_E_UNSUPPORTED outside that set (the caller runs v4).
int launch_ed5(EdArgs a, int k, int stride, hipStream_t st);

// 1 if launch_edpw4 runs this block shape (bf16, k 3, stride 1, no upsample, c1 == cin), else 0.
int edpw4_supported(int cin_pad, int hid, int cout, int k, int stride, int up, int ho, int wo);
int launch_edpw4(const EdpwArgs& a, hipStream_t st);

}  // namespace ast_mb
