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
 *
 * Determinism: every result is bitwise reproducible run to run on the same device and shapes.
 * No floating-point partial sum meets another through an atomic: reductions split across
 * workgroups write their partials into a caller-provided `workspace` (size from the matching
 * *_workspace_floats query; device memory, 16-byte aligned) and are summed in a fixed order, and
 * scalar losses accumulate into a loss accumulator (below).
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

/* Loss accumulator: AST_LOSS_ACC_FLOATS device floats, zeroed once by the caller. [0] holds the
 * accumulated value; [1] is an arrival counter that every launch leaves at 0; [2..] hold one
 * partial per workgroup of the running launch, summed in workgroup order by the last workgroup
 * to finish. One stream at a time per accumulator. */
#define AST_LOSS_SLOTS 4096
#define AST_LOSS_ACC_FLOATS (2 + AST_LOSS_SLOTS)
int ast_loss_acc_floats(void);

/* ---------------------------------------------------------------------------------------------
 * 3x3 convolution, stride 1, "same" size, as an MFMA-fp32 implicit GEMM.
 * Replaces nn.Conv2d(k=3, padding=1) + ReLU (+ MaxPool2d(2,2)) of PretrainedEncoder
 * (models.py:199-224, forward :230-240) and ReflectionPad2d(1) + Conv2d + ReLU (+ the preceding
 * nn.Upsample(x2, nearest)) of the mirrored decoder (models.py:598-628).
 * ------------------------------------------------------------------------------------------ */

/* Number of floats of the packed weight buffer for a [cout, cin, 3, 3] filter bank. */
size_t ast_conv3x3_packed_numel(int cout, int cin);

/* Repack w[cout][cin][3][3] into the kernel layout (zero padded). The packed buffer holds the
 * fp32 pack [cin_pad8][9][cout_pad64] followed by the split-bf16 pack of the same weights (three
 * bf16 terms per value, w = hi + mid + lo exactly) that the fp32-accurate bf16-MFMA kernel reads. */
int ast_conv3x3_pack_weights_f32(const float* w, float* w_packed, int cout, int cin, void* stream);

/* (Re)build the split-bf16 part of a packed buffer from its fp32 part (the pack functions call it). */
int ast_conv3x3_pack_split_f32(float* w_packed, int cout, int cin, void* stream);

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

/* AdaIN with precomputed style statistics (one-style-many-contents mode, SURVEY §8e: the rank
 * owning the style image computes them and broadcasts 2*C floats). style_mean/style_std are
 * indexed [n * style_stride_n + c]; style_stride_n = 0 shares one style across the batch.
 * std is the unbiased standard deviation (channel_stats, model_util.py:3-8). */
int ast_adain_stats_f32(const float* content, const float* style_mean, const float* style_std,
                        float* out, int n, int c, int hc, int wc, int style_stride_n, double alpha,
                        int swap_style_stats, void* stream);

/* Backward of ast_adain_f32: d_content and/or d_style (either may be NULL) from grad_out. */
int ast_adain_backward_f32(const float* content, const float* style, const float* grad_out,
                           float* d_content, float* d_style, int n, int c, int hc, int wc,
                           int hs, int ws, double alpha, int swap_style_stats, void* stream);

/* out = (x - mean[p]) / std[p] per plane (mean_variance_norm, models.py:64-68, given stats). */
int ast_plane_normalize_f32(const float* x, const float* mean, const float* std, float* out,
                            long long planes, long long hw, void* stream);

/* ---------------------------------------------------------------------------------------------
 * 3x3 conv backward (training step). Input gradients run ast_conv3x3_fwd_f32_cfg on a
 * transposed+flipped pack of the filter (cin' = cout, cout' = cin, zero padding):
 * dgrad_same(dy) = gradient of the padded input at its interior.
 * ------------------------------------------------------------------------------------------ */

/* transpose_flip = 0: same as ast_conv3x3_pack_weights_f32. transpose_flip = 1: pack
 * W'[ci][co][ky][kx] = W[co][ci][2-ky][2-kx] / (in_scale ? in_scale[ci] : 1) (in_scale folds
 * the conv_1 normalisation's 1/std into the image gradient); its packed size is
 * ast_conv3x3_packed_numel(cin, cout). */
int ast_conv3x3_pack_weights_ex_f32(const float* w, float* w_packed, int cout, int cin,
                                    int transpose_flip, const float* in_scale, void* stream);

/* Backward of y_pre -> ReLU -> [MaxPool2d(2,2)] (models.py:216-218):
 * dy = g_pre + (pre > 0) * (g_act + unpool(g_pool)); any of g_pre/g_act/g_pool may be NULL.
 * pre [planes, h, w], g_pool [planes, h/2, w/2]. */
int ast_conv_act_backward_f32(const float* pre, const float* g_pre, const float* g_act,
                              const float* g_pool, float* dy, long long planes, int h, int w,
                              void* stream);

/* out = mask > 0 ? g : 0 (ReLU backward given the ReLU output). */
int ast_relu_mask_f32(const float* g, const float* mask, float* out, long long n, void* stream);

/* Decoder dgrad, step 1: out_pad [planes, h+2, pitch] = zero-padded (mask > 0 ? g : 0)
 * (g [planes, h, w]; mask = the layer's ReLU output, or NULL). A zero-padded same conv of
 * out_pad with the transposed+flipped filter is then the FULL gradient of the padded input. */
int ast_grad_pad_f32(const float* g, const float* mask, float* out_pad, long long planes,
                     int h, int w, int pitch, void* stream);

/* Decoder dgrad, step 3: adjoint of Upsample(x upsample, nearest) -> ReflectionPad2d(1): folds
 * the full padded-input gradient dp_full [planes, h_in*up+2, pitch] onto dx [planes, h_in, w_in]. */
int ast_pad_up_adjoint_f32(const float* dp_full, float* dx, long long planes, int h_in, int w_in,
                           int upsample, int pitch, void* stream);

/* Input gradient with a fused epilogue (round 5; replaces the grad_pad -> dgrad -> pad_up_adjoint
 * chain of the decoder and the ReLU backward of the layer below, models.py:216-218, 598-628).
 * For the forward y = conv3x3(pad(upsample(x))) with dy [n, cout, h, w] (h, w: the conv's output
 * grid, = upsample x the source grid): dx [n, cin, h/up, w/up] = epi(S(D)) where D = the zero-padded
 * same conv of dy with the transposed+flipped pack w_tf_packed (the interior of the padded-input
 * gradient), S = the 2x2 window sum when upsample == 2 (the nearest-upsample adjoint), and
 * epi(v) = mask > 0 ? add_post + (v + add_pre) : add_post per element of dx (mask, add_pre,
 * add_post [n, cin, h/up, w/up], each optional: no mask keeps every element, no add_post reads 0).
 * Reflect padding's border fold is ast_dgrad_reflect_border_f32, run after this.
 * The epilogue is the split-bf16 kernels' (cfg 24-35) and, for upsample 1, the cout <= 4 direct
 * kernels' (cfg 18-23) and the cout <= 3 split-bf16 ones' (cfg 42, 43; -1 = heuristic):
 * AST_E_UNSUPPORTED for any other configuration -- the
 * caller then runs ast_conv3x3_fwd_f32_cfg + ast_dgrad_finish_f32. */
int ast_conv3x3_dgrad_f32(int cfg, const float* dy, const float* w_tf_packed, float* dx,
                          const float* mask, const float* add_pre, const float* add_post, int n,
                          int cout, int h, int w, int cin, int upsample, void* stream);

/* The same epilogue as a separate pass over a plain input-gradient conv's output raw
 * [planes, h*up, w*up]: dx [planes, h, w] = epi(S(raw)). */
int ast_dgrad_finish_f32(const float* raw, float* dx, const float* mask, const float* add_pre,
                         const float* add_post, long long planes, int h, int w, int upsample,
                         void* stream);

/* Reflect-pad border of the input gradient of conv3x3(ReflectionPad2d(1)(upsample(x))): adds to
 * dx [n, cin, h, w_in] the padded-input gradient's four border lines (computed from dy [n, cout,
 * h*up, w_in*up] and the forward filter w [cout, cin, 3, 3] into the workspace, with dy's edge
 * columns made contiguous there first) folded as the
 * reflect pad and upsample map them, masked like the interior (mask [n, cin, h, w_in] > 0, or
 * NULL). workspace: ast_dgrad_reflect_border_workspace_floats floats. */
long long ast_dgrad_reflect_border_workspace_floats(int n, int cout, int cin, int h, int w_in, int upsample);
int ast_dgrad_reflect_border_f32(const float* dy, const float* w, float* dx, const float* mask,
                                 float* workspace, long long workspace_floats, int n, int cout,
                                 int cin, int h, int w_in, int upsample, void* stream);

/* dw [cout, cin, 3, 3] = sum over images/pixels of dy x pad(upsample(x)) (overwritten; split-bf16
 * MFMA, split over pixel tiles: each split's partial dW/db goes to the workspace, then one ordered
 * reduce); db [cout] = sum of dy (optional). workspace: ast_conv3x3_wgrad_workspace_floats floats. */
long long ast_conv3x3_wgrad_workspace_floats(int n, int cin, int h_in, int w_in, int cout, int upsample);
int ast_conv3x3_wgrad_f32(const float* x, const float* dy, float* dw, float* db,
                          int n, int cin, int h_in, int w_in, int cout,
                          int upsample, int pad_mode, float* workspace, long long workspace_floats,
                          void* stream);

/* Same with dy read through (pitch, plane stride, offset of element (0,0)) — e.g. the padded
 * gradient buffer of ast_grad_pad_f32 (pitch, (h+2)*pitch, pitch+1). dy_pitch = 0: dense. */
int ast_conv3x3_wgrad_ex_f32(const float* x, const float* dy, float* dw, float* db,
                             int n, int cin, int h_in, int w_in, int cout, int upsample,
                             int pad_mode, int dy_pitch, long long dy_plane, long long dy_offset,
                             float* workspace, long long workspace_floats, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Losses (losses.py). Loss values are ADDED into the loss accumulator `loss` (AST_LOSS_ACC_FLOATS
 * floats, value at [0]; may be NULL); gradients are written (accumulate=0) or added
 * (accumulate=1) into `dx` (may be NULL = value only). `weight` multiplies both; `gscale` (device
 * scalar or NULL) multiplies the gradient only (autograd's grad_output).
 * ------------------------------------------------------------------------------------------ */

/* gram_matrix (losses.py:105-109): gram[b] = scale * feat[b] feat[b]^T, feat [n, c, hw],
 * gram [n, c, c] (overwritten; split-K MFMA, the K-splits' partial tiles summed in order through
 * the workspace of ast_gram_workspace_floats floats, 0 when the launch needs no split). */
long long ast_gram_workspace_floats(int n, int c, long long hw);
int ast_gram_f32(const float* feat, float* gram, int n, int c, long long hw, float scale, float* workspace,
                 long long workspace_floats, void* stream);

/* dfeat[b] (+)= scale * (dgram[b] + dgram[b]^T) feat[b] + row_a[b,i] * feat[b,i,:] + row_b[b,i]
 * (the backward of gram_matrix, with compute_style_loss's mean/std gradients fused: row_a/row_b
 * from ast_style_moments_f32, or both NULL). */
int ast_gram_backward_f32(const float* feat, const float* dgram, float* dfeat,
                          const float* row_a, const float* row_b,
                          int n, int c, long long hw, float scale, const float* gscale,
                          int accumulate, void* stream);

/* compute_content_loss(mean_variance_norm(x), mean_variance_norm(y)) (losses.py:124-126,
 * models.py:64-68; train.py:225): loss += weight * mean(huber(mvn(x) - mvn(y))). With pstats
 * [planes, 6] (or NULL) it also keeps what the backward needs. */
int ast_mvn_huber_f32(const float* x, const float* y, long long planes, long long hw, float weight,
                      float* loss, float* pstats, void* stream);

/* The same, split over (chunk, plane) workgroups: partial moments and Huber sums of each chunk of
 * 8192 elements go to `workspace` (ast_plane_stats_workspace_floats(planes, hw) floats) and are
 * merged in chunk order, so few large planes fill the chip. Three launches; same outputs. */
long long ast_plane_stats_workspace_floats(long long planes, long long hw);
int ast_mvn_huber_ws_f32(const float* x, const float* y, long long planes, long long hw, float weight,
                         float* loss, float* pstats, float* workspace, long long workspace_floats,
                         void* stream);

/* d/dx of the above (y constant), from the forward's pstats: one pass over x and y. */
int ast_mvn_huber_backward_f32(const float* x, const float* y, const float* pstats, long long planes,
                               long long hw, float weight, const float* gscale, float* dx,
                               int accumulate, void* stream);

/* compute_content_loss(x, y) = F.huber_loss(x, y) (delta 1, mean). */
int ast_huber_f32(const float* x, const float* y, long long n, float weight, const float* gscale,
                  float* loss, float* dx, int accumulate, void* stream);

/* Mean/std part of compute_style_loss (losses.py:130-134):
 * loss += weight * 1.25 * (mean huber(mu_x - mu_y) + mean huber(sd_x - sd_y)) over planes,
 * stats [planes, 4] = (mu_x, sd_x, mu_y, sd_y); row_a/row_b [planes] = per-plane gradient
 * d/dx = row_a * x + row_b (NULL: value only). */
int ast_style_moments_f32(const float* x, const float* y, long long planes, long long hw, float weight,
                          const float* gscale, float* stats, float* loss, float* row_a, float* row_b,
                          void* stream);

/* The same with the plane moments split over (chunk, plane) workgroups through `workspace`
 * (ast_plane_stats_workspace_floats(planes, hw) floats; merged in chunk order). */
int ast_style_moments_ws_f32(const float* x, const float* y, long long planes, long long hw, float weight,
                             const float* gscale, float* stats, float* loss, float* row_a, float* row_b,
                             float* workspace, long long workspace_floats, void* stream);

/* Gram part of compute_style_loss (losses.py:135-137): loss += weight * 10 * mean(huber(gx-gy)),
 * dgram = d/dgx (NULL: value only). */
int ast_gram_huber_f32(const float* gx, const float* gy, long long n, float weight, const float* gscale,
                       float* loss, float* dgram, void* stream);

/* tv_loss (losses.py:90-103): loss += weight * tv(x); dx (+)= d/dx. x [planes, h, w]. */
int ast_tv_loss_f32(const float* x, long long planes, int h, int w, float weight, const float* gscale,
                    float* loss, float* dx, int accumulate, void* stream);

/* Backward of mean_variance_norm (models.py:64-68) given the output gradient g. */
int ast_mvn_backward_f32(const float* x, const float* g, float* dx, long long planes, long long hw,
                         float eps, void* stream);

/* Backward of channel_stats / calc_mean_std: dx (+)= dmean/N + dstd*(x-mean)/((N-unbiased)*std);
 * dmean or dstd may be NULL. */
int ast_channel_stats_backward_f32(const float* x, const float* mean, const float* std,
                                   const float* dmean, const float* dstd, float* dx,
                                   long long planes, long long hw, int unbiased, int accumulate,
                                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * Optimizer (train.py:287-300): clip_grad_norm_ + torch.optim.Adam over many tensors in two
 * launches. The caller builds a tensor table on the host (ast_optim_build_table, returns the
 * number of 64K-element chunks = workgroups), copies it to device memory once, and reuses it.
 * ------------------------------------------------------------------------------------------ */
size_t ast_optim_table_bytes(int ntensors);
long long ast_optim_build_table(void* host_table, int ntensors, float* const* params,
                                float* const* grads, float* const* exp_avg,
                                float* const* exp_avg_sq, const long long* numel);

/* state[0] = sqrt(sum of squared grads), state[1] = min(1, max_norm/(state[0]+1e-6))
 * (max_norm <= 0: coefficient 1). partial: nchunks floats of scratch. */
int ast_grad_norm_f32(const void* dev_table, int ntensors, long long nchunks, float* partial,
                      float max_norm, float* state, void* stream);

/* grads *= state[1] (the clip_grad_norm_ scaling alone). */
int ast_grad_scale_f32(const void* dev_table, int ntensors, long long nchunks, const float* state,
                       void* stream);

/* grads *= state[1] (if state) then one Adam step (step = 1-based count; lr, betas, eps as in
 * torch.optim.Adam, amsgrad off, no weight decay). */
int ast_adam_step_f32(const void* dev_table, int ntensors, long long nchunks, const float* state,
                      double lr, double beta1, double beta2, double eps, int step, void* stream);

/* The same step with its step count on the device (hipGraph replays): sched [4] floats =
 * [step count, skip flag, lr / bias_correction1, sqrt(bias_correction2)]; the call advances
 * sched[0] and computes the rest on the device. check_finite: a non-finite gradient norm state[0]
 * sets the skip flag and leaves parameters, moments, gradients and the step count unchanged (the
 * caller reads state[0] after the step and raises, as clip_grad_norm_(error_if_nonfinite)). */
int ast_adam_step_sched_f32(const void* dev_table, int ntensors, long long nchunks, const float* state,
                            double lr, double beta1, double beta2, double eps, float* sched, int check_finite,
                            void* stream);

/* ---------------------------------------------------------------------------------------------
 * MobileNet-style variant (config 5). dtype / dtype_in / dtype_out: 0 = fp32,
 * 1 = bf16 storage (fp32 accumulate). All maps NCHW contiguous. BatchNorm (eval) is folded into
 * the weights by the caller.
 * ------------------------------------------------------------------------------------------ */

/* DepthWiseConv.forward (mobilenetv2.py:153-165) up to the SE pool: the expand 1x1 conv
 * (w1p != NULL: packed [round_up(hid,16)][cin_pad] in dtype, cin_pad a multiple of 16 (bf16) or 4
 * (fp32), zero padded; b1 [hid]) + Hardswish, then the depthwise k x k conv (k 3|5, stride 1|2,
 * reflect pad (k-1)/2; wdw [hid][k*k], bdw [hid]) + Hardswish, written to d [n][hid][ho][wo];
 * pool [n][hid] receives the per-plane sums of d (overwritten: each output tile's sums go to the
 * workspace, [n][hid][tile], and one ordered reduce makes pool). w1p == NULL is the ratio-1 form
 * (mobilenetv2.py:103-116): hid == cin, k == 3, and up == 2 applies DecoderBlock's nearest
 * Upsample (models.py:264-266) to x first. x2 != NULL feeds channels [c1, cin) from a second
 * tensor (the torch.cat before ada_out, models.py:335). workspace: the floats returned by
 * ast_mb_expand_dw_workspace_floats for the same arguments (has_x2 = x2 != NULL,
 * expand = w1p != NULL); <= 0 means the shape is unsupported. d == NULL is the pool-only pass
 * of the fused block pair (ast_mb_expand_dw_pw): pool is made, nothing else is written (bf16, k 3,
 * stride 1, expand blocks; AST_E_UNSUPPORTED elsewhere). */
long long ast_mb_expand_dw_workspace_floats(int dtype, int has_x2, int c1, int n, int cin, int h, int w, int up,
                                            int expand, int hid, int cin_pad, int k, int stride, int ho, int wo);
int ast_mb_expand_dw(int dtype, const void* x1, const void* x2, int c1, int n, int cin, int h, int w,
                     int up, const void* w1p, const float* b1, int hid, int cin_pad,
                     const float* wdw, const float* bdw, int k, int stride, void* d, float* pool,
                     int ho, int wo, float* workspace, long long workspace_floats, void* stream);

/* The fused block pair (DepthWiseConv.forward, mobilenetv2.py:153-165, without its hidden-width
 * tensor in memory): after ast_mb_expand_dw(d = NULL) made pool and ast_mb_se_fold made wg, this
 * recomputes the expand + depthwise of x and applies wg directly: out[n][co] = sum_c wg[n][co][c] *
 * D[n][c] + b2[co] (+ res[n][co]) in bf16, bit-identical to ast_mb_expand_dw + ast_mb_pw. Shapes:
 * ast_mb_expand_dw_pw_supported (1 = supported: bf16, k 3, stride 1, up 1, no x2, and the
 * (cin_pad, hid, cout) combinations instantiated). b2 and res may be NULL; hid_pad =
 * round_up(hid, 32), cout_pad = round_up(cout, 16). */
int ast_mb_expand_dw_pw_supported(int dtype, int has_x2, int cin, int cin_pad, int hid, int cout, int k,
                                  int stride, int up, int ho, int wo);
int ast_mb_expand_dw_pw(int dtype, const void* x, int n, int cin, int h, int w, const void* w1p,
                        const float* b1, int hid, int cin_pad, const float* wdw, const float* bdw, int k,
                        const void* wg, int cout, int cout_pad, int hid_pad, const float* b2,
                        const void* res, void* out, void* stream);

/* SELayer (mobilenetv2.py:63-81) on the pooled sums (mean = pool / hw), folded into the pw-linear
 * weights w2 [cout][hid]: wg[n][co][c] = w2[co][c] * gate[n][c], written as dtype
 * [n][cout_pad][hid_pad] with zero padding. fc1w [red][hid], fc2w [hid][red]. */
int ast_mb_se_fold(int dtype, const float* pool, int n, int hid, long long hw, const float* fc1w,
                   const float* fc1b, int red, const float* fc2w, const float* fc2b, const float* w2,
                   int cout, int cout_pad, int hid_pad, void* wg, void* stream);

/* pw-linear conv: out[n][co] = sum_c wg[n*wg_stride + co*hid_pad + c] * d[n][c] + bias[co]
 * (+ res[n][co], or res at (y/2, x/2) when res_up: the upsampled identity of models.py:266).
 * hid_pad a multiple of 32, cout_pad a multiple of 16 (16..128, except 112). bias may be NULL. */
int ast_mb_pw(int dtype, const void* d, int n, int hid, int hid_pad, int h, int w, const void* wg,
              long long wg_stride, const float* bias, int cout, int cout_pad, const void* res,
              int res_up, void* out, void* stream);

/* The expand half of DepthWiseConv (mobilenetv2.py:170-173) on its own, for blocks whose input is
 * too wide for the fused expand+depthwise kernels (AutoEncoder/AST ada_out, models.py:335: 256 ->
 * 768): out[n][co] = Hardswish(sum_c w1p[co][c] * cat(x1, x2)[n][c] + b1[co]) in bf16 (dtype 1),
 * [n][hid][h][w]. The depthwise then runs as the ratio-1 form of ast_mb_expand_dw on out.
 * cin_pad a multiple of 32, hid a multiple of 128; x2 != NULL feeds channels [c1, cin). */
int ast_mb_expand_gemm(int dtype, const void* x1, const void* x2, int c1, int n, int cin, int h, int w,
                       const void* w1p, const float* b1, int hid, int cin_pad, void* out, void* stream);

/* Eval-mode BatchNorm folded into the conv before it (mobilenetv2.py:223-231 _fold, the planned
 * inference path of DepthWiseConv; reference layers mobilenetv2.py:146-160): w is [cout][k],
 * s = gamma / sqrt(var + eps), w_out[r][c] = w[r][c] * s[r] for r < cout, c < k and 0 in the padding
 * of the [rows_out][ld] output; b_out[r] = beta[r] - mean[r] * s[r] (NULL: not written). has_bn 0:
 * a padded copy and a zero bias. Same roundings as the torch expression. */
int ast_mb_fold_bn_f32(const float* w, int cout, int k, const float* gamma, const float* beta, const float* mean,
                       const float* var, float eps, int has_bn, float* w_out, int ld, int rows_out, float* b_out,
                       void* stream);

/* Dense 3x3 reflect-pad convs of the variant: block 0 (conv_3x3_bn, mobilenetv2.py:38-43:
 * cin 3 -> cout 16, no bias, act 1 = Hardswish, fp32 input) and the decoder output conv
 * (models.py:300-316: cin 16 -> cout 3 + bias, fp32 output, act 2 = Hardtanh(0,1) when exporting,
 * act 0 otherwise). wt [cout][cin][3][3]. */
int ast_mb_conv3x3_dense(int dtype_in, int dtype_out, const void* x, const float* wt,
                         const float* bias, void* y, int n, int cin, int cout, int h, int w, int act,
                         void* stream);

/* AdaIN (as ast_adain_f32) on bf16 maps, fp32 statistics. */
int ast_adain_bf16(const void* content, const void* style, void* out, int n, int c, int hc, int wc,
                   int hs, int ws, double alpha, int swap_style_stats, void* stream);

/* ---------------------------------------------------------------------------------------------
 * AdaAttN (models.py:70-115; SURVEY §8f "next" #1): attention-weighted style statistics.
 *   q = W_q(IN(content)), k = W_k(IN(style)), v = W_v(style)     (1x1 convs, no bias)
 *   A = softmax over style pixels of q^T k; mean = A v; std = sqrt(relu(A v^2 - mean^2))
 *   out = std * IN(content) + mean,   IN = InstanceNorm2d (biased var, eps 1e-5, no affine)
 * content [n][c][hc][wc], style [n][c][hs][ws], out like content (dtype 0 = fp32);
 * wq/wk/wv [c][c] fp32 (the Conv2d weights [c][c][1][1]). c <= 128.
 * workspace: device scratch of ast_adaattn_workspace_bytes() bytes (Q, K, V, statistics). */
/* ---------------------------------------------------------------------------------------------
 * AdaAttN backward stages (csrc/adaattn_bwd.hip; the GEMMs between them are ast_mbt_gemm_f32).
 * Notation per image: C channels, N content pixels, M style pixels; O = [mean | ex2] [N][2C].
 * ------------------------------------------------------------------------------------------ */
/* s[r][:] = softmax(s[r][:]) in place, rows x cols (nn.Softmax(dim=-1), models.py:97-99). */
int ast_softmax_rows_f32(float* s, long long rows, int cols, void* stream);
/* From O [n][N][2C], G = dL/dout [n][C][N] and IN(c) [n][C][N]: dO [n][N][2C] (d mean | d ex2 of
 * out = sqrt(relu(ex2 - mean^2)) IN(c) + mean, models.py:101-115), D[n*N] = rowsum(dO * O) and
 * optionally std [n][C][N]. */
int ast_adaattn_dstats_f32(const float* o2, const float* g, const float* chat, float* do2, float* drow,
                           float* std_out, int n, int c, int npix, void* stream);
/* dS = P * (dP - D[row]) in place in dp (softmax backward), rows x cols. */
int ast_softmax_backward_f32(const float* p, float* dp, const float* drow, long long rows, int cols,
                             void* stream);
/* vv [n][2][cm]: vv[b][1] = vv[b][0]^2 (the [V; V^2] operand). */
int ast_adaattn_square_f32(float* vv, int n, long long cm, void* stream);
/* dv [n][cm] = dvv[b][0] + 2 vv[b][0] * dvv[b][1]. */
int ast_adaattn_dv_f32(const float* dvv, const float* vv, float* dv, int n, long long cm, void* stream);
/* InstanceNorm2d backward (no affine) per plane, given the forward's mean / std = sqrt(var + eps)
 * (biased var): dx (=|+=) (dxh - mean(dxh) - xh mean(dxh xh)) / std. */
int ast_instance_norm_backward_f32(const float* x, const float* mean, const float* std, const float* dxh,
                                   float* dx, long long planes, long long hw, int accumulate, void* stream);
/* dst += a * b elementwise. */
int ast_fma_inplace_f32(float* dst, const float* a, const float* b, long long n, void* stream);
/* Flash-style AdaAttN backward (csrc/adaattn_flash.hip; replaces the materialised P / dS of the
 * calls above for large maps). q [n][C][N], k [n][C][M], vv [n][2C][M] ([V; V^2]) as above;
 * C a multiple of 16, at most 128, not 80 or 112 (ast_adaattn_flash_supported).
 * stats: o2 [n][N][2C] = softmax(Q^T K) [V; V^2]^T and lse2 [n][N] (log2-domain row log-sum-exp).
 * bwd_kv: dk [n][C][M] = Q dS, dvv [n][2C][M] = dO^T P, from do2 / drow of ast_adaattn_dstats_f32.
 * bwd_q: dq [n][C][N] = K dS^T. Deterministic (one lane sums each output in a fixed order). */
int ast_adaattn_flash_supported(int c);
int ast_adaattn_flash_stats_f32(const float* q, const float* k, const float* vv, float* o2, float* lse2, int n, int c,
                                int nq, int nk, void* stream);
int ast_adaattn_flash_bwd_kv_f32(const float* q, const float* k, const float* vv, const float* do2, const float* lse2,
                                 const float* drow, float* dk, float* dvv, int n, int c, int nq, int nk, void* stream);
int ast_adaattn_flash_bwd_q_f32(const float* q, const float* k, const float* vv, const float* do2, const float* lse2,
                                const float* drow, float* dq, int n, int c, int nq, int nk, void* stream);

size_t ast_adaattn_workspace_bytes(int dtype, int n, int c, int hc, int wc, int hs, int ws);
int ast_adaattn_fwd(int dtype, const void* content, const void* style, const float* wq,
                    const float* wk, const float* wv, void* out, void* workspace,
                    size_t workspace_bytes, int n, int c, int hc, int wc, int hs, int ws,
                    void* stream);

/* ---------------------------------------------------------------------------------------------
 * Remaining train.py loss terms (SURVEY §8f "next" #2). Scalars are added into the loss
 * accumulator `loss` (AST_LOSS_ACC_FLOATS floats, zeroed once by the caller); gscale (device
 * scalar, may be NULL = 1) scales gradients.
 * ------------------------------------------------------------------------------------------ */

/* SingleDimHistLayer (losses.py:40-57): hist[b][k] = inv_norm * sum_i phi_k(x[b][i]) over the
 * m = C*H*W values of image b (m < 2^30), K = 256 bins, L = 1/256, W = L/2.5 (inv_norm = 1/(C*H):
 * the reference divides by x.size(1)*x.size(2)). hist [n][256] is overwritten. The bin sums are
 * exact 32.32 fixed-point integers (order-independent), kept in the workspace of
 * ast_soft_hist_workspace_floats(n) floats. */
long long ast_soft_hist_workspace_floats(int n);
int ast_soft_hist_f32(const float* x, int n, long long m, float inv_norm, float* hist, float* workspace,
                      long long workspace_floats, void* stream);

/* EarthMoversDistanceLoss (losses.py:8-22) of two histograms [n][256], mean over n
 * (compute_hist_loss, losses.py:84-87): *loss += weight * mean_b sum_t (cdf_x - cdf_y)^2;
 * ghist [n][256] (may be NULL) = gscale * d/dhx. */
int ast_emd_loss_f32(const float* hx, const float* hy, int n, float weight, const float* gscale,
                     float* loss, float* ghist, void* stream);

/* Backward of ast_soft_hist_f32: dx (+)= inv_norm * sum_k ghist[b][k] * dphi_k/dx. */
int ast_soft_hist_backward_f32(const float* x, int n, long long m, float inv_norm,
                               const float* ghist, float* dx, int accumulate, void* stream);

/* out_of_range_loss (train.py:259): *loss += weight * mean huber(x - clip(x, 0, 1)) (the clipped
 * copy is detached); dx (+)= its gradient. */
int ast_range_loss_f32(const float* x, long long numel, float weight, const float* gscale,
                       float* loss, float* dx, int accumulate, void* stream);

/* *loss += weight * mean((x - y)^2) (org_img_loss pixel term, train.py:268); dx (+)= d/dx. */
int ast_sqdiff_mean_f32(const float* x, const float* y, long long numel, float weight,
                        const float* gscale, float* loss, float* dx, int accumulate, void* stream);

/* ---------------------------------------------------------------------------------------------
 * On-device augmentation (SURVEY §8f "next" #3): the get_transform pipeline of data_loader.py:110-135
 * on [C][H][W] fp32 images (torchvision tensor semantics). Random parameters are drawn by the caller.
 * ------------------------------------------------------------------------------------------ */

/* transforms.ToTensor: uint8 [h][w][cs] (cs >= 3; RGB first) -> fp32 [3][h][w] / 255. */
int ast_aug_to_tensor(const unsigned char* src, int h, int w, int cs, float* dst, void* stream);

/* Integer-affine gather (torch.rot90 / hflip / vflip, data_loader.py:14-24, :115-116):
 * dst[c][y][x] = src[c][sy][sx], sy = coef[0]*y + coef[1]*x + coef[2], sx = coef[3]*y + coef[4]*x +
 * coef[5]; coef is a HOST array of 6 ints; every (y, x) must map inside src. */
int ast_aug_remap_f32(const float* src, int c, int hi, int wi, float* dst, int ho, int wo,
                      const int* coef, void* stream);

/* acc[0] = sum over pixels of rgb_to_grayscale(img) (adjust_contrast's mean * h*w); acc is a loss
 * accumulator (AST_LOSS_ACC_FLOATS floats, zeroed once by the caller; [0] is overwritten here). */
int ast_aug_gray_sum_f32(const float* img, int h, int w, float* acc, void* stream);

/* ColorJitter's adjustments and RandomGrayscale on a 3-channel image: op 0 brightness, 1 contrast
 * (gray_sum from ast_aug_gray_sum_f32), 2 saturation, 3 hue (factor in [-0.5, 0.5]), 4 grayscale. */
int ast_aug_color_f32(const float* src, int h, int w, int op, float factor, const float* gray_sum,
                      float* dst, void* stream);

/* Resize / RandomResizedCrop: the crop [y0, y0+crop_h) x [x0, x0+crop_w) of src resized to ho x wo
 * with antialiased bilinear weights (torch upsample aa, align_corners=False). tmp: device scratch
 * of ast_aug_resize_workspace_floats(c, crop_h, wo) floats. */
size_t ast_aug_resize_workspace_floats(int c, int crop_h, int wo);
int ast_aug_resize_f32(const float* src, int c, int h, int w, int y0, int x0, int crop_h, int crop_w,
                       float* dst, int ho, int wo, float* tmp, void* stream);

/* GaussianBlur: separable normalised taps (HOST array of k floats, k odd <= 15), reflect padding;
 * tmp: device scratch of c*h*w floats. */
int ast_aug_blur_f32(const float* src, int c, int h, int w, const float* taps, int k, float* dst,
                     float* tmp, void* stream);

/* ---------------------------------------------------------------------------------------------
 * MobileNet-variant training (SURVEY §8f "next" #4: AutoEncoder training, train_autoencoder.py),
 * fp32, composable kernels with their backward (csrc/mbtrain.hip).
 * ------------------------------------------------------------------------------------------ */

/* Side-by-side packing for small-plane zero-padded 3x3 convs (csrc/pack.hip; ops.conv3x3):
 * xp[ceil(n/G)][c][h][G*(w+gap)-gap] holds images x[0..n1) then x2[0..n2), G per row band,
 * `gap` zero columns between them; unpack reads image i at column (i%G)*sp of packed plane i/G. */
int ast_pack_images_f32(const float* x, int n1, const float* x2, int n2, int c, int h, int w, int G,
                        int gap, float* xp, void* stream);
int ast_unpack_images_f32(const float* yp, int n, int c, int h, int w, int G, int sp, int wp,
                          float* out, void* stream);

/* C[b][m][n] (+)= sum_k A[b][m][k] B[b][k][n] with element strides (1x1 convs and their grads).
 * ksplit > 1 splits K across workgroups, and sCb == 0 with batch > 1 shares C across the batch:
 * then every (image, K-split) tile goes to the workspace (ast_mbt_gemm_workspace_floats floats,
 * 0 when neither applies) and one ordered reduce writes / adds C.
 * foldN = P > 0 (batch 1, B n-contiguous): column n is pixel n % P of image n / P, reached through
 * the image strides sBb / sCb; foldK = P > 0 (batch 1, A and B k-contiguous): the same for K. */
long long ast_mbt_gemm_workspace_floats(int M, int N, int batch, int ksplit, long long sCb);
int ast_mbt_gemm_f32(const float* A, const float* B, float* C, int M, int N, int K, int batch,
                     long long sAb, long long sAm, long long sAk, long long sBb, long long sBk,
                     long long sBn, long long sCb, long long sCm, long long sCn, int ksplit,
                     int accumulate, int foldK, int foldN, float* workspace, long long workspace_floats,
                     void* stream);

/* Depthwise k x k conv (k 3|5, stride 1|2, reflect pad (k-1)/2; mobilenetv2.py:148-149, :116-117),
 * LDS-tiled (csrc/mbt_dw.hip): mode 0 out = conv(x, w); 1 out = dx from g (overwritten, one pass,
 * no workspace); 2 out = dw [c][k*k] from x, g (overwritten; the workspace holds one partial row
 * per (channel, image, tile group), summed in that order). Mode 2 needs
 * ast_mbt_dw_workspace_floats floats of workspace (modes 0 and 1 ignore it). */
long long ast_mbt_dw_workspace_floats(int n, int c, int h, int wd, int k);
int ast_mbt_dw_f32(int mode, const float* x, const float* w, const float* g, float* out, int n,
                   int c, int h, int wd, int k, int s, float* workspace, long long workspace_floats,
                   void* stream);
/* The same with DepthWiseConv's Hardswish -> depthwise conv pair fused (mobilenetv2.py:144-149):
 * act 1 means the conv's input is hardswish(x) with x the stored pre-activation -- modes 0 and 2
 * apply it while staging x, mode 1 (x required then) returns the gradient w.r.t. x, taken on
 * through the Hardswish. Bit-identical to the materialised activation. act 0 = ast_mbt_dw_f32. */
int ast_mbt_dw_act_f32(int mode, const float* x, const float* w, const float* g, float* out, int n,
                       int c, int h, int wd, int k, int s, int act, float* workspace,
                       long long workspace_floats, void* stream);

/* BatchNorm2d in training mode (batch statistics, biased var + eps; running stats updated with
 * momentum and the unbiased variance when run_mean/run_var are given). mean/invstd [c] saved.
 * workspace: ast_mbt_bn_workspace_floats(n, c, hw) floats of per-segment partial statistics.
 * The composites below are stats -> merge(1 part) -> apply and bwd_sums -> bwd_apply; SyncBatchNorm
 * (data-parallel AutoEncoder training, dp.convert_sync_batchnorm) calls the stages itself with a
 * gather of the per-rank stats and an all-reduce of the backward sums in between. */
long long ast_mbt_bn_workspace_floats(int n, int c, long long hw);
int ast_mbt_bn_fwd_f32(const float* x, int n, int c, long long hw, const float* gamma,
                       const float* beta, float eps, float momentum, float* mean, float* invstd,
                       float* run_mean, float* run_var, float* y, float* workspace,
                       long long workspace_floats, void* stream);
int ast_mbt_bn_bwd_f32(const float* x, const float* dy, int n, int c, long long hw,
                       const float* mean, const float* invstd, const float* gamma, float* dgamma,
                       float* dbeta, float* dx, float* workspace, long long workspace_floats,
                       void* stream);
/* this process's per-channel (count, mean, M2) as double [c][3] */
int ast_mbt_bn_stats_f32(const float* x, int n, int c, long long hw, float* workspace,
                         long long workspace_floats, double* stats, void* stream);
/* merge [parts][c][3] stats (Chan) -> mean, invstd, running stats (nullable), 1/count [1] (nullable) */
int ast_mbt_bn_merge_f32(const double* stats, int parts, int c, float eps, float momentum, float* mean,
                         float* invstd, float* run_mean, float* run_var, float* inv_count, void* stream);
int ast_mbt_bn_apply_f32(const float* x, int n, int c, long long hw, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, float* y,
                         void* stream);
/* sums [2][c]: sum(dy), sum(dy * xhat) over this process's images */
int ast_mbt_bn_bwd_sums_f32(const float* x, const float* dy, int n, int c, long long hw,
                            const float* mean, const float* invstd, float* workspace,
                            long long workspace_floats, float* sums, void* stream);
/* dx from (all-reduced) sums and the device 1/count written by ast_mbt_bn_merge_f32 */
int ast_mbt_bn_bwd_apply_f32(const float* x, const float* dy, int n, int c, long long hw,
                             const float* mean, const float* invstd, const float* gamma,
                             const float* sums, const float* inv_count, float* dx, void* stream);

/* The same stages with DepthWiseConv's BatchNorm2d -> Hardswish pair (mobilenetv2.py:122-126,
 * :150-153) fused: act 1 makes y = hardswish(BN(x)) in the apply pass, and the backward takes dy as
 * the gradient of that output (through the Hardswish at the recomputed BN output, bit-identical to
 * the forward's); act 0 is plain BatchNorm (the entries above are these with act 0). beta is needed
 * by the backward only when act is 1. */
int ast_mbt_bn_act_fwd_f32(const float* x, int n, int c, long long hw, const float* gamma,
                           const float* beta, float eps, float momentum, float* mean, float* invstd,
                           float* run_mean, float* run_var, int act, float* y, float* workspace,
                           long long workspace_floats, void* stream);
int ast_mbt_bn_act_apply_f32(const float* x, int n, int c, long long hw, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, int act, float* y,
                             void* stream);
int ast_mbt_bn_act_bwd_f32(const float* x, const float* dy, int n, int c, long long hw,
                           const float* mean, const float* invstd, const float* gamma, const float* beta,
                           int act, float* dgamma, float* dbeta, float* dx, float* workspace,
                           long long workspace_floats, void* stream);
int ast_mbt_bn_act_bwd_sums_f32(const float* x, const float* dy, int n, int c, long long hw,
                                const float* mean, const float* invstd, const float* gamma,
                                const float* beta, int act, float* workspace, long long workspace_floats,
                                float* sums, void* stream);
int ast_mbt_bn_act_bwd_apply_f32(const float* x, const float* dy, int n, int c, long long hw,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, int act, const float* sums, const float* inv_count,
                                 float* dx, void* stream);

/* op 0 y = hardswish(a); 1 y = hardswish'(a) * b; 2 y = a + b; 3 y = nearest-upsample x2 of a
 * (n planes of h x w); 4 its backward (a = grad of the 2h x 2w planes). */
int ast_mbt_eltwise_f32(int op, const float* a, const float* b, float* y, long long n, int h,
                        int w, void* stream);

/* op 0 out[p] = mean(x[p]) (AdaptiveAvgPool2d(1)); 1 out[p] = sum(x[p] * y[p]);
 * 2 out = x * gate[p] (+ gadd[p]) over planes of hw elements. */
int ast_mbt_plane_f32(int op, const float* x, const float* y, const float* gate, const float* gadd,
                      float* out, long long planes, long long hw, void* stream);
/* ops 0-2 as above, plus the Hardswish -> SELayer pair over the stored pre-activation
 * (mobilenetv2.py:151-156): 3 out[p] = mean(hardswish(x[p])); 4 out[p] = sum(x[p] * hardswish(y[p]));
 * 5 out = hardswish(x) * gate[p]; 6 out = hardswish'(a) * (x * gate[p] + gadd[p]) (a: the
 * pre-activation). Bit-identical to the materialised activation. */
int ast_mbt_plane_act_f32(int op, const float* x, const float* y, const float* gate, const float* gadd,
                          const float* a, float* out, long long planes, long long hw, void* stream);

/* SELayer MLP (mobilenetv2.py:63-81): hid = relu(W1 pool + b1), z = W2 hid + b2, gate = clamp(z,0,1);
 * backward from dgate: parameter gradients (overwritten, summed over images in image order) and
 * dpool / hw; workspace n * (c + red) floats (the per-image dz, dh). */
int ast_mbt_se_fc_fwd_f32(const float* pool, const float* w1, const float* b1, const float* w2,
                          const float* b2, int n, int c, int red, float* hid, float* z, float* gate,
                          void* stream);
int ast_mbt_se_fc_bwd_f32(const float* dgate, const float* z, const float* hid, const float* pool,
                          const float* w1, const float* w2, int n, int c, int red, long long hw,
                          float* dw1, float* db1, float* dw2, float* db2, float* dpool, float* workspace,
                          long long workspace_floats, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AST_HIP_H */
