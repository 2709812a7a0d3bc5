"""ctypes binding of libast_hip.so (the C ABI declared in include/ast_hip.h).

The library is built in-tree (`python -c "import __graft_entry__ as g; g.build()"`). There is no
fallback: if the library is missing, or a tensor is not on a HIP device, calls raise.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads PyTorch's HIP runtime first, so the library binds to the same one)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AST_HIP_LIB") or os.path.join(_HERE, "libast_hip.so")  # override: A/B kernel builds

_c_float_p = ctypes.c_void_p
_i = ctypes.c_int
_ll = ctypes.c_longlong
_p = ctypes.c_void_p
_f = ctypes.c_float
_d = ctypes.c_double

# name -> (restype, argtypes); must match include/ast_hip.h exactly (tests/test_capi.py checks it)
SIGNATURES = {
    "ast_version": (ctypes.c_char_p, []),
    "ast_loss_acc_floats": (_i, []),
    "ast_conv3x3_packed_numel": (ctypes.c_size_t, [_i, _i]),
    "ast_conv3x3_pack_weights_f32": (_i, [_p, _p, _i, _i, _p]),
    "ast_conv3x3_pack_split_f32": (_i, [_p, _i, _i, _p]),
    "ast_conv3x3_fwd_f32": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ast_conv3x3_num_configs": (_i, []),
    "ast_conv3x3_fwd_f32_cfg": (_i, [_i, _p, _p, _i, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ast_channel_stats_f32": (_i, [_p, _p, _p, _ll, _ll, _i, ctypes.c_float, _p]),
    "ast_adain_f32": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _i, ctypes.c_double, _i, _p]),
    "ast_plane_normalize_f32": (_i, [_p, _p, _p, _p, _ll, _ll, _p]),
    "ast_adain_backward_f32": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _d, _i, _p]),
    "ast_adain_stats_f32": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _d, _i, _p]),
    "ast_conv3x3_pack_weights_ex_f32": (_i, [_p, _p, _i, _i, _i, _p, _p]),
    "ast_conv_act_backward_f32": (_i, [_p, _p, _p, _p, _p, _ll, _i, _i, _p]),
    "ast_relu_mask_f32": (_i, [_p, _p, _p, _ll, _p]),
    "ast_grad_pad_f32": (_i, [_p, _p, _p, _ll, _i, _i, _i, _p]),
    "ast_pad_up_adjoint_f32": (_i, [_p, _p, _ll, _i, _i, _i, _i, _p]),
    "ast_conv3x3_dgrad_f32": (_i, [_i, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p]),
    "ast_dgrad_finish_f32": (_i, [_p, _p, _p, _p, _p, _ll, _i, _i, _i, _p]),
    "ast_dgrad_reflect_border_workspace_floats": (_ll, [_i, _i, _i, _i, _i, _i]),
    "ast_dgrad_reflect_border_f32": (_i, [_p, _p, _p, _p, _p, _ll, _i, _i, _i, _i, _i, _i, _p]),
    "ast_conv3x3_wgrad_workspace_floats": (_ll, [_i, _i, _i, _i, _i, _i]),
    "ast_conv3x3_wgrad_f32": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _ll, _p]),
    "ast_conv3x3_wgrad_ex_f32": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _ll, _ll, _p, _ll, _p]),
    "ast_gram_workspace_floats": (_ll, [_i, _i, _ll]),
    "ast_gram_f32": (_i, [_p, _p, _i, _i, _ll, _f, _p, _ll, _p]),
    "ast_gram_backward_f32": (_i, [_p, _p, _p, _p, _p, _i, _i, _ll, _f, _p, _i, _p]),
    "ast_mvn_huber_f32": (_i, [_p, _p, _ll, _ll, _f, _p, _p, _p]),
    "ast_plane_stats_workspace_floats": (_ll, [_ll, _ll]),
    "ast_mvn_huber_ws_f32": (_i, [_p, _p, _ll, _ll, _f, _p, _p, _p, _ll, _p]),
    "ast_style_moments_ws_f32": (_i, [_p, _p, _ll, _ll, _f, _p, _p, _p, _p, _p, _p, _ll, _p]),
    "ast_mvn_huber_backward_f32": (_i, [_p, _p, _p, _ll, _ll, _f, _p, _p, _i, _p]),
    "ast_huber_f32": (_i, [_p, _p, _ll, _f, _p, _p, _p, _i, _p]),
    "ast_style_moments_f32": (_i, [_p, _p, _ll, _ll, _f, _p, _p, _p, _p, _p, _p]),
    "ast_gram_huber_f32": (_i, [_p, _p, _ll, _f, _p, _p, _p, _p]),
    "ast_tv_loss_f32": (_i, [_p, _ll, _i, _i, _f, _p, _p, _p, _i, _p]),
    "ast_mvn_backward_f32": (_i, [_p, _p, _p, _ll, _ll, _f, _p]),
    "ast_channel_stats_backward_f32": (_i, [_p, _p, _p, _p, _p, _p, _ll, _ll, _i, _i, _p]),
    "ast_optim_table_bytes": (ctypes.c_size_t, [_i]),
    "ast_optim_build_table": (_ll, [_p, _i, _p, _p, _p, _p, _p]),
    "ast_grad_norm_f32": (_i, [_p, _i, _ll, _p, _f, _p, _p]),
    "ast_grad_scale_f32": (_i, [_p, _i, _ll, _p, _p]),
    "ast_adam_step_f32": (_i, [_p, _i, _ll, _p, _d, _d, _d, _d, _i, _p]),
    "ast_adam_step_sched_f32": (_i, [_p, _i, _ll, _p, _d, _d, _d, _d, _p, _i, _p]),
    "ast_mb_expand_dw_workspace_floats": (_ll, [_i] * 15),
    "ast_mb_expand_dw": (_i, [_i, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _i, _i, _p, _p, _i, _i, _p, _p,
                              _i, _i, _p, _ll, _p]),
    "ast_mb_se_fold": (_i, [_i, _p, _i, _i, _ll, _p, _p, _i, _p, _p, _p, _i, _i, _i, _p, _p]),
    "ast_mb_pw": (_i, [_i, _p, _i, _i, _i, _i, _i, _p, _ll, _p, _i, _i, _p, _i, _p, _p]),
    "ast_mb_expand_gemm": (_i, [_i, _p, _p, _i, _i, _i, _i, _i, _p, _p, _i, _i, _p, _p]),
    "ast_mb_fold_bn_f32": (_i, [_p, _i, _i, _p, _p, _p, _p, ctypes.c_float, _i, _p, _i, _i, _p, _p]),
    "ast_mb_expand_dw_pw_supported": (_i, [_i] * 11),
    "ast_mb_expand_dw_pw": (_i, [_i, _p, _i, _i, _i, _i, _p, _p, _i, _i, _p, _p, _i, _p, _i, _i, _i, _p, _p, _p, _p]),
    "ast_mb_conv3x3_dense": (_i, [_i, _i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p]),
    "ast_adain_bf16": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _i, _d, _i, _p]),
    "ast_softmax_rows_f32": (_i, [_p, _ll, _i, _p]),
    "ast_adaattn_dstats_f32": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "ast_softmax_backward_f32": (_i, [_p, _p, _p, _ll, _i, _p]),
    "ast_adaattn_square_f32": (_i, [_p, _i, _ll, _p]),
    "ast_adaattn_dv_f32": (_i, [_p, _p, _p, _i, _ll, _p]),
    "ast_instance_norm_backward_f32": (_i, [_p, _p, _p, _p, _p, _ll, _ll, _i, _p]),
    "ast_fma_inplace_f32": (_i, [_p, _p, _p, _ll, _p]),
    "ast_adaattn_flash_supported": (_i, [_i]),
    "ast_adaattn_flash_stats_f32": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "ast_adaattn_flash_bwd_kv_f32": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "ast_adaattn_flash_bwd_q_f32": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "ast_adaattn_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i, _i, _i, _i]),
    "ast_adaattn_fwd": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, ctypes.c_size_t, _i, _i, _i, _i, _i, _i, _p]),
    "ast_soft_hist_workspace_floats": (_ll, [_i]),
    "ast_soft_hist_f32": (_i, [_p, _i, _ll, _f, _p, _p, _ll, _p]),
    "ast_emd_loss_f32": (_i, [_p, _p, _i, _f, _p, _p, _p, _p]),
    "ast_soft_hist_backward_f32": (_i, [_p, _i, _ll, _f, _p, _p, _i, _p]),
    "ast_range_loss_f32": (_i, [_p, _ll, _f, _p, _p, _p, _i, _p]),
    "ast_sqdiff_mean_f32": (_i, [_p, _p, _ll, _f, _p, _p, _p, _i, _p]),
    "ast_aug_to_tensor": (_i, [_p, _i, _i, _i, _p, _p]),
    "ast_aug_remap_f32": (_i, [_p, _i, _i, _i, _p, _i, _i, _p, _p]),
    "ast_aug_gray_sum_f32": (_i, [_p, _i, _i, _p, _p]),
    "ast_aug_color_f32": (_i, [_p, _i, _i, _i, _f, _p, _p, _p]),
    "ast_aug_resize_workspace_floats": (ctypes.c_size_t, [_i, _i, _i]),
    "ast_aug_resize_f32": (_i, [_p, _i, _i, _i, _i, _i, _i, _i, _p, _i, _i, _p, _p]),
    "ast_aug_blur_f32": (_i, [_p, _i, _i, _i, _p, _i, _p, _p, _p]),
    "ast_pack_images_f32": (_i, [_p, _i, _p, _i, _i, _i, _i, _i, _i, _p, _p]),
    "ast_unpack_images_f32": (_i, [_p, _i, _i, _i, _i, _i, _i, _i, _p, _p]),
    "ast_mbt_gemm_workspace_floats": (_ll, [_i, _i, _i, _i, _ll]),
    "ast_mbt_gemm_f32": (_i, [_p, _p, _p, _i, _i, _i, _i, _ll, _ll, _ll, _ll, _ll, _ll, _ll, _ll, _ll, _i, _i, _i, _i, _p,
                              _ll, _p]),
    "ast_mbt_dw_workspace_floats": (_ll, [_i, _i, _i, _i, _i]),
    "ast_mbt_dw_f32": (_i, [_i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _ll, _p]),
    "ast_mbt_dw_act_f32": (_i, [_i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _ll, _p]),
    "ast_mbt_bn_workspace_floats": (_ll, [_i, _i, _ll]),
    "ast_mbt_bn_fwd_f32": (_i, [_p, _i, _i, _ll, _p, _p, _f, _f, _p, _p, _p, _p, _p, _p, _ll, _p]),
    "ast_mbt_bn_bwd_f32": (_i, [_p, _p, _i, _i, _ll, _p, _p, _p, _p, _p, _p, _p, _ll, _p]),
    "ast_mbt_bn_stats_f32": (_i, [_p, _i, _i, _ll, _p, _ll, _p, _p]),
    "ast_mbt_bn_merge_f32": (_i, [_p, _i, _i, _f, _f, _p, _p, _p, _p, _p, _p]),
    "ast_mbt_bn_apply_f32": (_i, [_p, _i, _i, _ll, _p, _p, _p, _p, _p, _p]),
    "ast_mbt_bn_bwd_sums_f32": (_i, [_p, _p, _i, _i, _ll, _p, _p, _p, _ll, _p, _p]),
    "ast_mbt_bn_bwd_apply_f32": (_i, [_p, _p, _i, _i, _ll, _p, _p, _p, _p, _p, _p, _p]),
    "ast_mbt_bn_act_fwd_f32": (_i, [_p, _i, _i, _ll, _p, _p, _f, _f, _p, _p, _p, _p, _i, _p, _p, _ll, _p]),
    "ast_mbt_bn_act_apply_f32": (_i, [_p, _i, _i, _ll, _p, _p, _p, _p, _i, _p, _p]),
    "ast_mbt_bn_act_bwd_f32": (_i, [_p, _p, _i, _i, _ll, _p, _p, _p, _p, _i, _p, _p, _p, _p, _ll, _p]),
    "ast_mbt_bn_act_bwd_sums_f32": (_i, [_p, _p, _i, _i, _ll, _p, _p, _p, _p, _i, _p, _ll, _p, _p]),
    "ast_mbt_bn_act_bwd_apply_f32": (_i, [_p, _p, _i, _i, _ll, _p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "ast_mbt_eltwise_f32": (_i, [_i, _p, _p, _p, _ll, _i, _i, _p]),
    "ast_mbt_plane_f32": (_i, [_i, _p, _p, _p, _p, _p, _ll, _ll, _p]),
    "ast_mbt_plane_act_f32": (_i, [_i, _p, _p, _p, _p, _p, _p, _ll, _ll, _p]),
    "ast_mbt_se_fc_fwd_f32": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p]),
    "ast_mbt_se_fc_bwd_f32": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _ll, _p, _p, _p, _p, _p, _p, _ll, _p]),
}

ERRORS = {-1: "null pointer", -2: "bad shape", -3: "unsupported configuration"}

_lib = None


class HipOpError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipOpError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(code: int, what: str) -> None:
    if code != 0:
        msg = ERRORS.get(code, f"hipError_t {code}")
        raise HipOpError(f"{what} failed: {msg}")


def stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def workspace(nfloats: int, device) -> "torch.Tensor":
    """Device scratch of a deterministic reduction (the *_workspace_floats queries of ast_hip.h):
    taken from the caching allocator per call, so stream order alone keeps calls apart."""
    return torch.empty((max(1, int(nfloats)),), device=device, dtype=torch.float32)


_ACC_FLOATS = None


_ACC_POOL = None   # [chunk, next row] while an accumulator_pool() scope is active


def loss_accumulator(device, pooled: bool = True) -> "torch.Tensor":
    """A zeroed loss accumulator (AST_LOSS_ACC_FLOATS floats; the value is element 0). Inside an
    accumulator_pool() scope it is a row of a chunk of 64 zeroed at once -- not for the outputs of
    torch.ops custom operators (pooled=False), which must not share storage with each other."""
    global _ACC_FLOATS
    if _ACC_FLOATS is None:
        _ACC_FLOATS = int(lib().ast_loss_acc_floats())
    pool = _ACC_POOL if pooled else None
    if pool is not None:
        chunk, i = pool.get(device, (None, 64))
        if i == 64:
            chunk, i = torch.zeros((64, _ACC_FLOATS), device=device, dtype=torch.float32), 0
        pool[device] = (chunk, i + 1)
        return chunk[i]
    return torch.zeros((_ACC_FLOATS,), device=device, dtype=torch.float32)


class accumulator_pool:
    """Scope of one training step: its loss accumulators come from chunks of 64 zeroed by one
    launch each (~40 loss terms per ASTTrainer step, each a zero fill before). Every scope takes
    fresh chunks, so values a caller keeps from an earlier step are never overwritten."""

    def __enter__(self):
        global _ACC_POOL
        self.prev, _ACC_POOL = _ACC_POOL, {}
        return self

    def __exit__(self, *exc):
        global _ACC_POOL
        _ACC_POOL = self.prev
