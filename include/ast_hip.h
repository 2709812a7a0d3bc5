/* ast_hip.h — C ABI of the MI355X (gfx950) AdaIN style-transfer hot path.
 *
 * The reference (rwickman/ArbitraryStyleTransfer) is pure Python: its "plugin" surface is the
 * nn.Module / function API of models.py, model_util.py and losses.py. Each entry point below is
 * the native kernel that replaces one reference operator; arbitrarystyletransfer_amd/ binds them
 * with ctypes behind that same module API (see INTEGRATION.md for the binding).
 *
 * Conventions: every tensor is a dense device pointer (HBM), fp32, NCHW unless stated;
 * `stream` is a hipStream_t passed as void*; no call allocates, copies to host or synchronises,
 * so every call is legal inside hipGraph capture. Return value: 0 on success, a negative
 * AST_E* code for an argument error (nothing launched), or a positive hipError_t.
 */
#ifndef AST_HIP_H
#define AST_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AST_OK 0
#define AST_E_NULLPTR (-1)
#define AST_E_SHAPE (-2)
#define AST_E_UNSUPPORTED (-3)

/* Library version / capability string (e.g. "ast_hip 0.1 gfx950"). */
const char* ast_version(void);

/* ---------------------------------------------------------------------------------------------
 * 3x3 convolution, stride 1, "same" size, as an MFMA-fp32 implicit GEMM.
 * Replaces nn.Conv2d(k=3, padding=1) + ReLU (+ MaxPool2d(2,2)) of PretrainedEncoder
 * (models.py:199-224, forward :230-240) and ReflectionPad2d(1) + Conv2d + ReLU (+ the preceding
 * nn.Upsample(x2, nearest)) of the mirrored decoder (models.py:598-628).
 * ------------------------------------------------------------------------------------------ */

/* Number of floats of the packed weight buffer for a [cout, cin, 3, 3] filter bank. */
size_t ast_conv3x3_packed_numel(int cout, int cin);

/* Repack w[cout][cin][3][3] into the kernel layout (zero padded). */
int ast_conv3x3_pack_weights_f32(const float* w, float* w_packed, int cout, int cin, void* stream);

/* y = conv3x3(pad(upsample(x))) + bias, with fused epilogue stores.
 *   x        [n, cin, h_in, w_in]; output spatial size h = h_in*upsample, w = w_in*upsample
 *   upsample 1 or 2 (nearest, applied before padding, as Upsample -> ReflectionPad -> Conv)
 *   pad_mode 0 = zeros (VGG encoder, Conv2d(padding=1)), 1 = reflect (ReflectionPad2d(1))
 *   in_mean/in_std  optional [cin]: input normalised as (x - mean)/std before padding
 *                   (Normalization, models.py:120-131, fused into conv_1; may be NULL)
 *   y_pre    optional [n, cout, h, w]      conv output before ReLU (the conv_i taps)
 *   y_act    optional [n, cout, h, w]      ReLU(conv) (relu_i)
 *   y_pool   optional [n, cout, h/2, w/2]  MaxPool2d(2,2)(ReLU(conv)) (pool_i)
 *   bias     optional [cout]
 */
int ast_conv3x3_fwd_f32(const float* x, const float* w_packed, const float* bias,
                        float* y_pre, float* y_act, float* y_pool,
                        const float* in_mean, const float* in_std,
                        int n, int cin, int h_in, int w_in, int cout,
                        int upsample, int pad_mode, void* stream);

/* General form. cfg selects a kernel configuration (0..ast_conv3x3_num_configs()-1, tuner /
 * tests), cfg < 0 = automatic. x2/n2: optional second input batch of n2 images appended after
 * the n images of x (one launch encodes a content batch and a style batch; outputs hold n + n2
 * images). x2 = NULL and n2 = 0 for a single batch. */
int ast_conv3x3_num_configs(void);
int ast_conv3x3_fwd_f32_cfg(int cfg, const float* x, const float* x2, int n2,
                            const float* w_packed, const float* bias,
                            float* y_pre, float* y_act, float* y_pool,
                            const float* in_mean, const float* in_std,
                            int n, int cin, int h_in, int w_in, int cout,
                            int upsample, int pad_mode, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Per-channel statistics and AdaIN.
 * ------------------------------------------------------------------------------------------ */

/* mean[p], std[p] over each of `planes` contiguous planes of `hw` elements.
 * std = sqrt(sum((x-mean)^2) / (hw - unbiased) + eps).
 *   channel_stats (model_util.py:3-8):  unbiased=1, eps=0
 *   calc_mean_std (models.py:54-62):    unbiased=1, eps=1e-5 */
int ast_channel_stats_f32(const float* x, float* mean, float* std, long long planes, long long hw,
                          int unbiased, float eps, void* stream);

/* AdaIN.forward (models.py:43-51) + alpha blend (models.py:471), one launch:
 *   t   = (c - mu_c) / sigma_c * scale + shift,   stats = channel_stats (unbiased, no eps)
 *   out = alpha * t + (1 - alpha) * c
 * swap_style_stats=1 reproduces the reference literally (scale = mu_s, shift = sigma_s,
 * SURVEY.md F1); 0 is canonical AdaIN (scale = sigma_s, shift = mu_s).
 * content [n, c, hc, wc], style [n, c, hs, ws], out [n, c, hc, wc]. */
int ast_adain_f32(const float* content, const float* style, float* out,
                  int n, int c, int hc, int wc, int hs, int ws,
                  double alpha, int swap_style_stats, void* stream);

/* out = (x - mean[p]) / std[p] per plane (mean_variance_norm, models.py:64-68, given stats). */
int ast_plane_normalize_f32(const float* x, const float* mean, const float* std, float* out,
                            long long planes, long long hw, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AST_HIP_H */
