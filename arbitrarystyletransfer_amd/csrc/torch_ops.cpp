// PyTorch custom-op registration of the hot ops: torch.ops.ast_hip.* ("What the
// C++ side exports"), a thin shim over the C ABI of libast_hip.so (include/ast_hip.h). Each op
// checks its arguments with TORCH_CHECK (RuntimeError in Python), allocates outputs with the
// caching allocator, and enqueues the same kernel the ctypes binding (_lib.py) launches, on
// PyTorch's current HIP stream. Meta kernels give shapes for tracing / fake tensors.
//
// Built by csrc/Makefile into libast_torch_ops.so (linked against libast_hip.so and libtorch);
// loaded with torch.ops.load_library (arbitrarystyletransfer_amd/torch_ops.py).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <tuple>

#include "../../include/ast_hip.h"

namespace {

void* cur_stream(const at::Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

const char* err_name(int code) {
  switch (code) {
    case AST_E_NULLPTR: return "null pointer";
    case AST_E_SHAPE: return "bad shape";
    case AST_E_UNSUPPORTED: return "unsupported configuration";
    default: return "hipError_t";
  }
}

#define AST_CALL(what, expr)                                                                    \
  do {                                                                                          \
    const int _c = (expr);                                                                      \
    TORCH_CHECK(_c == 0, what " failed: ", err_name(_c), " (", _c, ")");                        \
  } while (0)

at::Tensor dev_f32(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be on a HIP device (arbitrarystyletransfer_amd has no CPU path), got ",
              t.device());
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32, got ", t.scalar_type());
  return t.contiguous();
}

const float* fptr(const c10::optional<at::Tensor>& t) { return t ? t->data_ptr<float>() : nullptr; }

// Every tensor argument of an op must live on the device of its first input (whose stream the
// launch uses): a pointer from another GPU would be read as if it were local.
void same_device(const at::Tensor& ref, const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.device() == ref.device(), name, " is on ", t.device(), " but the op runs on ", ref.device());
}

// ---- AdaIN (models.py:43-51) + alpha blend (models.py:471) ----------------------------------
at::Tensor adain(const at::Tensor& content_, const at::Tensor& style_, double alpha, bool swap_style_stats) {
  at::Tensor content = dev_f32(content_, "content_map"), style = dev_f32(style_, "style_map");
  TORCH_CHECK(content.dim() == 4 && style.dim() == 4 && content.size(0) == style.size(0) &&
                  content.size(1) == style.size(1),
              "AdaIN needs NCHW maps with equal (N, C): ", content.sizes(), " vs ", style.sizes());
  same_device(content, style, "style_map");
  const c10::DeviceGuard guard(content.device());
  at::Tensor out = at::empty_like(content);
  AST_CALL("adain", ast_adain_f32(content.data_ptr<float>(), style.data_ptr<float>(), out.data_ptr<float>(),
                                  (int)content.size(0), (int)content.size(1), (int)content.size(2),
                                  (int)content.size(3), (int)style.size(2), (int)style.size(3), alpha,
                                  swap_style_stats ? 1 : 0, cur_stream(content)));
  return out;
}

at::Tensor adain_meta(const at::Tensor& content, const at::Tensor& style, double, bool) {
  TORCH_CHECK(content.dim() == 4 && style.dim() == 4 && content.size(0) == style.size(0) &&
                  content.size(1) == style.size(1),
              "AdaIN needs NCHW maps with equal (N, C): ", content.sizes(), " vs ", style.sizes());
  return at::empty_like(content);
}

// ---- channel_stats (model_util.py:3-8) / calc_mean_std (models.py:54-62) --------------------
std::tuple<at::Tensor, at::Tensor> channel_stats(const at::Tensor& x_, bool unbiased, double eps) {
  at::Tensor x = dev_f32(x_, "x");
  TORCH_CHECK(x.dim() == 4, "channel_stats expects NCHW, got ", x.sizes());
  const c10::DeviceGuard guard(x.device());
  at::Tensor mean = at::empty({x.size(0), x.size(1), 1, 1}, x.options());
  at::Tensor std_ = at::empty_like(mean);
  AST_CALL("channel_stats", ast_channel_stats_f32(x.data_ptr<float>(), mean.data_ptr<float>(), std_.data_ptr<float>(),
                                                  x.size(0) * x.size(1), x.size(2) * x.size(3), unbiased ? 1 : 0,
                                                  (float)eps, cur_stream(x)));
  return {mean, std_};
}

std::tuple<at::Tensor, at::Tensor> channel_stats_meta(const at::Tensor& x, bool, double) {
  TORCH_CHECK(x.dim() == 4, "channel_stats expects NCHW, got ", x.sizes());
  at::Tensor mean = at::empty({x.size(0), x.size(1), 1, 1}, x.options());
  return {mean, at::empty_like(mean)};
}

// ---- conv3x3: weight packing + the fused forward (PretrainedEncoder / VGG decoder convs) -----
at::Tensor conv3x3_pack(const at::Tensor& w_) {
  at::Tensor w = dev_f32(w_, "weight");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "conv3x3 weight must be [cout, cin, 3, 3], got ",
              w.sizes());
  const int cout = (int)w.size(0), cin = (int)w.size(1);
  const c10::DeviceGuard guard(w.device());
  at::Tensor out = at::empty({(int64_t)ast_conv3x3_packed_numel(cout, cin)}, w.options());
  AST_CALL("conv3x3_pack", ast_conv3x3_pack_weights_f32(w.data_ptr<float>(), out.data_ptr<float>(), cout, cin,
                                                        cur_stream(w)));
  return out;
}

at::Tensor conv3x3_pack_meta(const at::Tensor& w) {
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "conv3x3 weight must be [cout, cin, 3, 3], got ",
              w.sizes());
  return at::empty({(int64_t)ast_conv3x3_packed_numel((int)w.size(0), (int)w.size(1))}, w.options());
}

struct ConvShape {
  int64_t n, cin, h_in, w_in, H, W;
};

ConvShape conv_shape(const at::Tensor& x, const at::Tensor& w_packed, int64_t cout, int64_t upsample,
                     int64_t pad_mode, bool want_pre, bool want_act, bool want_pool) {
  TORCH_CHECK(x.dim() == 4, "x must be NCHW, got ", x.sizes());
  TORCH_CHECK(upsample == 1 || upsample == 2, "upsample must be 1 or 2");
  TORCH_CHECK(pad_mode == 0 || pad_mode == 1, "pad_mode must be 0 (zeros) or 1 (reflect)");
  TORCH_CHECK(want_pre || want_act || want_pool, "conv3x3: no output requested");
  TORCH_CHECK(cout > 0, "cout must be positive");
  ConvShape s{x.size(0), x.size(1), x.size(2), x.size(3), x.size(2) * upsample, x.size(3) * upsample};
  TORCH_CHECK(w_packed.numel() == (int64_t)ast_conv3x3_packed_numel((int)cout, (int)s.cin),
              "packed weight does not match (cout, cin)");
  TORCH_CHECK(!want_pool || (s.H >= 2 && s.W >= 2), "max-pool needs H, W >= 2");
  return s;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> conv3x3_fwd(
    const at::Tensor& x_, const at::Tensor& w_packed_, const c10::optional<at::Tensor>& bias_, int64_t cout,
    int64_t upsample, int64_t pad_mode, const c10::optional<at::Tensor>& in_mean_,
    const c10::optional<at::Tensor>& in_std_, bool want_pre, bool want_act, bool want_pool, int64_t cfg) {
  at::Tensor x = dev_f32(x_, "x"), w_packed = dev_f32(w_packed_, "w_packed");
  same_device(x, w_packed, "w_packed");
  const ConvShape s = conv_shape(x, w_packed, cout, upsample, pad_mode, want_pre, want_act, want_pool);
  c10::optional<at::Tensor> bias, in_mean, in_std;
  if (bias_) {
    bias = dev_f32(*bias_, "bias");
    same_device(x, *bias, "bias");
    TORCH_CHECK(bias->numel() == cout, "bias size mismatch");
  }
  TORCH_CHECK(in_mean_.has_value() == in_std_.has_value(), "in_mean and in_std go together");
  if (in_mean_) {
    in_mean = dev_f32(*in_mean_, "in_mean");
    in_std = dev_f32(*in_std_, "in_std");
    same_device(x, *in_mean, "in_mean");
    same_device(x, *in_std, "in_std");
    TORCH_CHECK(in_mean->numel() == s.cin && in_std->numel() == s.cin, "normalisation stats must have cin entries");
  }
  const c10::DeviceGuard guard(x.device());
  auto mk = [&](bool want, int64_t h, int64_t w) {
    return want ? at::empty({s.n, cout, h, w}, x.options()) : at::empty({0}, x.options());
  };
  at::Tensor pre = mk(want_pre, s.H, s.W), act = mk(want_act, s.H, s.W), pool = mk(want_pool, s.H / 2, s.W / 2);
  AST_CALL("conv3x3", ast_conv3x3_fwd_f32_cfg(
                          (int)cfg, x.data_ptr<float>(), nullptr, 0, w_packed.data_ptr<float>(), fptr(bias),
                          want_pre ? pre.data_ptr<float>() : nullptr, want_act ? act.data_ptr<float>() : nullptr,
                          want_pool ? pool.data_ptr<float>() : nullptr, fptr(in_mean), fptr(in_std), (int)s.n,
                          (int)s.cin, (int)s.h_in, (int)s.w_in, (int)cout, (int)upsample, (int)pad_mode,
                          cur_stream(x)));
  return {pre, act, pool};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> conv3x3_fwd_meta(
    const at::Tensor& x, const at::Tensor& w_packed, const c10::optional<at::Tensor>&, int64_t cout,
    int64_t upsample, int64_t pad_mode, const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&,
    bool want_pre, bool want_act, bool want_pool, int64_t) {
  const ConvShape s = conv_shape(x, w_packed, cout, upsample, pad_mode, want_pre, want_act, want_pool);
  auto mk = [&](bool want, int64_t h, int64_t w) {
    return want ? at::empty({s.n, cout, h, w}, x.options()) : at::empty({0}, x.options());
  };
  return {mk(want_pre, s.H, s.W), mk(want_act, s.H, s.W), mk(want_pool, s.H / 2, s.W / 2)};
}

// ---- gram_matrix (losses.py:105-109) --------------------------------------------------------
at::Tensor gram(const at::Tensor& f_) {
  at::Tensor f = dev_f32(f_, "tensor");
  TORCH_CHECK(f.dim() == 4, "gram_matrix expects [B, C, H, W], got ", f.sizes());
  const int64_t b = f.size(0), c = f.size(1), hw = f.size(2) * f.size(3);
  const c10::DeviceGuard guard(f.device());
  at::Tensor g = at::empty({b, c, c}, f.options());
  const long long wsf = ast_gram_workspace_floats((int)b, (int)c, hw);
  at::Tensor ws = at::empty({wsf > 0 ? wsf : 1}, f.options());
  AST_CALL("gram", ast_gram_f32(f.data_ptr<float>(), g.data_ptr<float>(), (int)b, (int)c, hw,
                                (float)(1.0 / (double)(c * hw)), ws.data_ptr<float>(), wsf, cur_stream(f)));
  return g;
}

at::Tensor gram_meta(const at::Tensor& f) {
  TORCH_CHECK(f.dim() == 4, "gram_matrix expects [B, C, H, W], got ", f.sizes());
  return at::empty({f.size(0), f.size(1), f.size(1)}, f.options());
}

}  // namespace

TORCH_LIBRARY(ast_hip, m) {
  m.def("adain(Tensor content_map, Tensor style_map, float alpha=1.0, bool swap_style_stats=True) -> Tensor");
  m.def("channel_stats(Tensor x, bool unbiased=True, float eps=0.0) -> (Tensor, Tensor)");
  m.def("conv3x3_pack(Tensor weight) -> Tensor");
  m.def("conv3x3_fwd(Tensor x, Tensor w_packed, Tensor? bias, int cout, int upsample=1, int pad_mode=0, "
        "Tensor? in_mean=None, Tensor? in_std=None, bool want_pre=False, bool want_act=True, bool want_pool=False, "
        "int cfg=-1) -> (Tensor, Tensor, Tensor)");
  m.def("gram(Tensor feat) -> Tensor");
}

TORCH_LIBRARY_IMPL(ast_hip, CUDA, m) {   // HIP tensors dispatch on the CUDA key in PyTorch-ROCm
  m.impl("adain", &adain);
  m.impl("channel_stats", &channel_stats);
  m.impl("conv3x3_pack", &conv3x3_pack);
  m.impl("conv3x3_fwd", &conv3x3_fwd);
  m.impl("gram", &gram);
}

TORCH_LIBRARY_IMPL(ast_hip, Meta, m) {
  m.impl("adain", &adain_meta);
  m.impl("channel_stats", &channel_stats_meta);
  m.impl("conv3x3_pack", &conv3x3_pack_meta);
  m.impl("conv3x3_fwd", &conv3x3_fwd_meta);
  m.impl("gram", &gram_meta);
}
