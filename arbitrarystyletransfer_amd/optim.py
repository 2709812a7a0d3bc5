"""Optimizer step of train.py:287-300 on HIP: clip_grad_norm_(params, max_norm,
error_if_nonfinite) + torch.optim.Adam, as two multi-tensor launches (optim.hip).

FusedAdam keeps torch.optim.Adam's param_groups/state layout ('step', 'exp_avg', 'exp_avg_sq'),
so `ast_optim` state dicts interchange with the reference's checkpoints (train.py:103-115).
"""
from __future__ import annotations

import ctypes

import torch

from . import ops
from ._lib import check, lib, ptr, stream_ptr


class _Table:
    """Device copy of the (param, grad, exp_avg, exp_avg_sq, numel) table, staged through a
    pinned host buffer (one small H2D copy on the stream, no host sync in steady state)."""

    def __init__(self):
        self.host = None
        self.dev = None
        self.event = None

    def build(self, params, grads, ms, vs, device):
        L = lib()
        n = len(params)
        nbytes = int(L.ast_optim_table_bytes(n))
        if self.host is None or self.host.numel() < nbytes:
            self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        if self.event is not None:
            self.event.synchronize()  # previous copy out of the pinned buffer has finished
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() if t is not None else 0 for t in ts])  # noqa: E731
        numel = (ctypes.c_longlong * n)(*[t.numel() for t in params])
        nchunks = L.ast_optim_build_table(ctypes.c_void_p(self.host.data_ptr()), n, arr(params), arr(grads),
                                          arr(ms) if ms is not None else None,
                                          arr(vs) if vs is not None else None, numel)
        if nchunks < 0:
            raise RuntimeError("optimizer table: null tensor")
        self.dev[:nbytes].copy_(self.host[:nbytes], non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record(torch.cuda.current_stream(device))
        return nchunks


def _grad_norm_state(table, n, nchunks, max_norm, device):
    partial = torch.empty(nchunks, device=device, dtype=torch.float32)
    state = torch.empty(2, device=device, dtype=torch.float32)
    check(lib().ast_grad_norm_f32(ptr(table.dev), n, nchunks, ptr(partial), float(max_norm), ptr(state),
                                  stream_ptr(device)), "grad_norm")
    return state


def _check_finite(norm):
    v = float(norm.item())
    if v != v or v in (float("inf"), float("-inf")):
        raise RuntimeError(f"The total norm of order 2.0 for gradients from `parameters` is non-finite ({v}), "
                           "so it cannot be clipped (error_if_nonfinite=True, train.py:292)")


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad off, no weight decay) with an optional fused
    clip_grad_norm_(max_grad_norm, error_if_nonfinite) in front, all on HIP."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm=None, error_if_nonfinite=False):
        if weight_decay != 0.0:
            raise ValueError("FusedAdam: weight_decay is not supported (the reference uses 0)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        self.max_grad_norm = max_grad_norm
        self.error_if_nonfinite = error_if_nonfinite
        self._tables = {}
        self.last_grad_norm = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        groups = []
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if params:
                groups.append((gi, group, params))
        if not groups:
            return loss
        dev = groups[0][2][0].device
        for _, _, params in groups:
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        tables = []
        for gi, group, params in groups:
            table = self._tables.setdefault(gi, _Table())
            grads = [ops._dev(p.grad, "grad") for p in params]
            nchunks = table.build([p.data for p in params], grads, [self.state[p]["exp_avg"] for p in params],
                                  [self.state[p]["exp_avg_sq"] for p in params], dev)
            tables.append((table, nchunks))
        state = None
        if self.max_grad_norm is not None:
            # clip_grad_norm_(all parameters): ONE norm over every group (train.py:292 clips
            # self.ast.parameters() as a whole)
            if len(groups) == 1:
                table, nchunks = tables[0]
                n_all = len(groups[0][2])
            else:
                table = self._tables.setdefault("all", _Table())
                allp = [p for _, _, ps in groups for p in ps]
                n_all = len(allp)
                nchunks = table.build([p.data for p in allp], [ops._dev(p.grad, "grad") for p in allp], None, None,
                                      dev)
            state = _grad_norm_state(table, n_all, nchunks, self.max_grad_norm, dev)
            self.last_grad_norm = state[0]
            if self.error_if_nonfinite:
                _check_finite(state[0])   # raises before any state changes (as torch's clip_grad_norm_)
        for (gi, group, params), (table, nchunks) in zip(groups, tables):
            for p in params:
                self.state[p]["step"] += 1
            step = int(self.state[params[0]]["step"].item())
            b1, b2 = group["betas"]
            check(lib().ast_adam_step_f32(ptr(table.dev), len(params), nchunks, ptr(state), float(group["lr"]),
                                          float(b1), float(b2), float(group["eps"]), step, stream_ptr(dev)),
                  "adam_step")
        ops.bump_weights_epoch([p for _, _, ps in groups for p in ps])
        return loss

    # ---- graph-capturable step (hipGraph replays: no host sync, no allocation, device step count) --
    def prepare_static(self):
        """Before capture: moments, device tables (contents filled by fill_static once the
        gradients' storage is known), the norm / schedule scratch and the device step count."""
        self._static = []
        dev = None
        for group in self.param_groups:
            params = list(group["params"])
            dev = params[0].device
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            table = _Table()
            nbytes = int(lib().ast_optim_table_bytes(len(params)))
            table.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            table.dev = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            nchunks = sum(-(-p.numel() // 65536) for p in params)
            sched = torch.zeros(4, device=dev, dtype=torch.float32)
            sched[0] = float(self.state[params[0]]["step"])
            self._static.append((group, params, table, nchunks, sched))
        allp = [p for _, ps, _, _, _ in self._static for p in ps]
        if len(self._static) == 1:
            self._static_norm = (self._static[0][2], len(allp), self._static[0][3])
        else:
            t = _Table()
            nbytes = int(lib().ast_optim_table_bytes(len(allp)))
            t.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            t.dev = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            self._static_norm = (t, len(allp), sum(-(-p.numel() // 65536) for p in allp))
        self._static_partial = torch.empty(self._static_norm[2], device=dev, dtype=torch.float32)
        self._static_state = torch.zeros(2, device=dev, dtype=torch.float32)

    def fill_static(self):
        """After capture: write the tables (every parameter now holds its persistent gradient)."""
        dev = None
        for group, params, table, nchunks, _ in self._static:
            if any(p.grad is None for p in params):
                raise RuntimeError("FusedAdam.fill_static: a parameter has no gradient after the captured backward")
            dev = params[0].device
            n = table.build([p.data for p in params], [ops._dev(p.grad, "grad") for p in params],
                            [self.state[p]["exp_avg"] for p in params], [self.state[p]["exp_avg_sq"] for p in params],
                            dev)
            assert n == nchunks
        if len(self._static) > 1:
            t, n_all, nchunks = self._static_norm
            allp = [p for _, ps, _, _, _ in self._static for p in ps]
            assert t.build([p.data for p in allp], [p.grad for p in allp], None, None, dev) == nchunks
        torch.cuda.current_stream(dev).synchronize()   # the pinned tables have reached the device

    def static_hyper(self):
        """The hyper-parameters step_static bakes into its launches (StepGraph recaptures on change)."""
        return (tuple((float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"])) for g in self.param_groups),
                self.max_grad_norm, self.error_if_nonfinite)

    def step_static(self):
        """clip_grad_norm_ + Adam on the static tables, capturable: a non-finite norm skips the
        update on the device (the caller checks last_grad_norm after the replay and raises)."""
        dev = self._static[0][1][0].device
        state = None
        if self.max_grad_norm is not None:
            table, n_all, nchunks = self._static_norm
            check(lib().ast_grad_norm_f32(ptr(table.dev), n_all, nchunks, ptr(self._static_partial),
                                          float(self.max_grad_norm), ptr(self._static_state), stream_ptr(dev)),
                  "grad_norm")
            state = self._static_state
            self.last_grad_norm = state[0]
        for group, params, table, nchunks, sched in self._static:
            b1, b2 = group["betas"]
            check(lib().ast_adam_step_sched_f32(ptr(table.dev), len(params), nchunks, ptr(state), float(group["lr"]),
                                                float(b1), float(b2), float(group["eps"]), ptr(sched),
                                                1 if self.error_if_nonfinite else 0, stream_ptr(dev)), "adam_step")

    def after_static_step(self):
        """Host bookkeeping of one replayed step (after the caller's non-finite check)."""
        for _, params, _, _, _ in self._static:
            for p in params:
                self.state[p]["step"] += 1
        ops.bump_weights_epoch([p for _, ps, _, _, _ in self._static for p in ps])


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    """torch.nn.utils.clip_grad_norm_ for L2 on HIP: returns the total norm (device scalar) and
    scales the gradients in place by min(1, max_norm / (norm + 1e-6))."""
    if norm_type != 2.0:
        raise ValueError("only the L2 norm is implemented")
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.tensor(0.0)
    dev = params[0].device
    table = _Table()
    grads = [ops._dev(p.grad, "grad") for p in params]
    nchunks = table.build(grads, grads, None, None, dev)
    state = _grad_norm_state(table, len(params), nchunks, max_norm, dev)
    if error_if_nonfinite:
        _check_finite(state[0])
    # scale: an Adam step with lr 0 would also touch moments; use the scale-only path instead
    check(lib().ast_grad_scale_f32(ptr(table.dev), len(params), nchunks, ptr(state), stream_ptr(dev)), "grad_scale")
    return state[0]
