"""AdaIN training step on HIP: the counterpart of the reference's ASTTrainer (train.py:50-401)
for the VGG AdaIN network (BASELINE.json configs 3-4).

Per step (train.py:191-300, AdaIN version):
  stylised = decoder(AdaIN(enc(content), enc(style)))            (encoder frozen, under no_grad)
  content_map, style_map, t_cs_map = lossnet(content|style|stylised)   (VGG19 to relu_15)
  content = sum_i huber(mvn(t_cs_map[i]), mvn(content_map[i])) + 0.1 * pixel term     (:217-227, :258)
  style   = sum_i w_i * style_loss(t_cs_map[i], style_map[i]) + style_loss(stylised, style)  (:230-245, :271)
            w = 1, 1, 1, 1, 0.75, 0.5
  lf      = huber(mvn(t), mvn(enc(stylised).detach()))           (:276-277; no gradient: t is constant)
  tv      = tv_loss(stylised)                                      (:282)
  loss    = 1.25*content + 0.5*style + 1.0*lf + 6e-4*tv            (:283, defaults :416-425)
  Adam(lr 2e-4, betas (0.9, 0.999), eps 1e-5) after clip_grad_norm_(2.0, error_if_nonfinite).
With `full_losses=True` (SURVEY.md §8f "next" #2) the step also carries the remaining terms of
train.py:248-283, as the reference adds them to the loss:
  org_out      = decoder(content features)                        (the AST's org_out, models.py:474)
  org_img      = org_img_lam * (sum_i huber(lossnet(org_out)[i], content_map[i])
                                + 100 * mean((content - org_out)^2))          (:248-256, :268-269)
  out_of_range = 1e8 * huber(stylised, clip(stylised.detach(), 0, 1))          (:259)
  hist         = 1e-5 * compute_hist_loss(stylised, style)                     (:261)
  loss        += hist + org_img + out_of_range                                 (:283)

Data parallel (config 4): one process per GPU, each with its own shard of the global batch
(`args.batch_size` is the global batch, as the reference's --batch_size is the batch of one step;
dp.shard_range). Decoder gradients land in one flat buffer (dp.FlatGradArena) and are SUMMED with a
single all-reduce (RCCL over xGMI) before clip + Adam. Each rank back-propagates its batch-mean
terms weighted by local/global images and the batch-sum term (tv, losses.py:90-103 sums over the
batch) unweighted, so the reduced gradient is exactly the full-batch gradient of train.py's loss,
for uneven shards too.
"""
from __future__ import annotations

import argparse
import gc
import json
import os

import torch
import torch.distributed as dist

from . import _lib, dp
from . import losses as L
from . import mbtrain, models, ops
from .conf import enc_out_layers
from .optim import FusedAdam

class StepGraph:
    """One training step captured in a hipGraph (torch.cuda.CUDAGraph is the HIP graph on ROCm):
    forward, backward, the gradient-arena reduction and clip + Adam replay with no Python, no
    launch latency and no host sync (every C-ABI call is capture-safe: no allocation, no sync).
    Inputs are copied into static buffers before each replay; the outputs are the captured
    step's static tensors. Gradients live in a flat arena (dp.FlatGradArena) so the optimizer's
    device tables point at storage that stays put; its step count and bias corrections are
    computed on the device (optim.FusedAdam.step_static). The one host sync left is the
    non-finite gradient-norm check (train.py:292, clip_grad_norm_(error_if_nonfinite))."""

    def __init__(self, optim, arena, params, body, frozen=()):
        self.optim, self.arena, self.params, self.body = optim, arena, list(params), body
        self.frozen = list(frozen)   # frozen networks whose weight packs are built once, outside the graph
        self.graph = None
        self.key = None   # (input shapes, optimizer hyper-parameters) the graph was captured for

    def _key(self, inputs):
        # the captured clip + Adam launches carry lr, betas, eps and max_grad_norm as kernel
        # arguments: a change (a scheduler, load() resetting the lr, train.py:94-98) recaptures
        return ([tuple(x.shape) for x in inputs], self.optim.static_hyper())

    def _capture(self, inputs):
        # a recapture (new input shapes or optimizer hyper-parameters) first drops the old graph,
        # its static buffers and outputs (the caller holds copies), so nothing of the old graph's
        # memory pool is released while the new capture is underway
        self.graph = self.out = self.static = None
        gc.collect()
        for net in self.frozen:
            net.prepack()
        self.optim.zero_grad(set_to_none=True)
        self.arena.reset()
        # every trainable weight's pack is rebuilt inside the graph (replays update the weights)
        ops.bump_weights_epoch(self.params)
        self.optim.prepare_static()
        self.static = [torch.empty_like(x) for x in inputs]
        for s_, x in zip(self.static, inputs):
            s_.copy_(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        gc.disable()   # no finalizer of unrelated garbage may run (and free or sync) inside the capture
        try:
            with torch.cuda.graph(g):
                self.out = self.body(*self.static)
        finally:
            gc.enable()
        self.optim.fill_static()
        self.graph = g
        self.key = self._key(inputs)

    def run(self, *inputs):
        """One replayed step. The returned tensors are copies: the next replay overwrites the
        captured step's own outputs in place, so a caller keeping a step's results (to log or show
        them later) gets what eager mode gives."""
        if self.graph is None or self.key != self._key(inputs):
            self._capture(inputs)
        for s_, x in zip(self.static, inputs):
            s_.copy_(x)
        self.graph.replay()
        if self.optim.error_if_nonfinite:
            v = float(self.optim.last_grad_norm.item())   # the one host sync per step
            if v != v or v in (float("inf"), float("-inf")):
                raise RuntimeError(f"The total norm of order 2.0 for gradients from `parameters` is non-finite ({v}), "
                                   "so it cannot be clipped (error_if_nonfinite=True, train.py:292); the step was "
                                   "not applied")
        self.optim.after_static_step()
        out = {k: _detached_copy(v) for k, v in self.out.items()}
        out["grad_norm"] = self.optim.last_grad_norm.clone()
        return out


def _detached_copy(v):
    if isinstance(v, torch.Tensor):
        return v.detach().clone()
    if isinstance(v, (list, tuple)):
        return type(v)(_detached_copy(x) for x in v)
    return v


STYLE_WEIGHTS = (1.0, 1.0, 1.0, 1.0, 0.75, 0.5)   # train.py:232-238 for the 6 loss-network layers
LOSSNET_LAYERS = ["conv_1", "conv_3", "conv_5", "conv_9", "conv_13", "relu_15"]   # models.py:187
# the loss network also emits relu_9 (= relu4_1, the AdaIN encoder output): with shared weights
# one pass over content+style yields both the loss targets and the AdaIN inputs, and the pass over
# the stylised batch yields enc(stylised) for the lf term.
_TAPS = ["conv_1", "conv_3", "conv_5", "conv_9", "relu_9", "conv_13", "relu_15"]
_LOSS_IDX = [0, 1, 2, 3, 5, 6]
_RELU9 = 4


def default_args(**kw):
    a = dict(train_iter=10, batch_size=8, lr=2e-4, content_lam=1.25, style_lam=0.5, tv_lam=0.0006, lf_lam=1.0,
             org_img_lam=0.5, save_dir="models/ast/", load=False, image_size=512, full_losses=False)
    a.update(kw)
    return argparse.Namespace(**a)


class AdaINTrainer:
    def __init__(self, args=None, device=None, net=None, lossnet=None, grad_hook=None):
        self.args = args or default_args()
        self.device = torch.device(device or "cuda")
        self.net = (net or models.AdaINStyleTransfer()).to(self.device)
        self.net.encoder.requires_grad_(False).eval()
        self.lossnet = (lossnet or models.PretrainedEncoder(_TAPS)).to(self.device).eval()
        self.lossnet.requires_grad_(False)
        self.lossnet._content_layers = set(_TAPS)
        # The AdaIN encoder is VGG19 to relu4_1 — the first 9 convs of the loss network. When the
        # weights agree (the reference's setup: both pretrained VGG19), share them so one pass
        # serves both; otherwise encode separately.
        enc_convs, loss_convs = self.net.encoder.convs(), self.lossnet.convs()[:9]
        self.shared = all(a.weight.shape == b.weight.shape and torch.equal(a.weight, b.weight) and
                          torch.equal(a.bias, b.bias) for a, b in zip(enc_convs, loss_convs))
        self.params = [p for p in self.net.decoder.parameters()]
        self.optim = FusedAdam(self.params, lr=self.args.lr, betas=(0.9, 0.999), eps=1e-5, max_grad_norm=2.0,
                               error_if_nonfinite=True)
        self.grad_hook = grad_hook  # called between backward and the optimizer step
        self.rank, self.world = 0, 1
        self.grad_arena = None
        if dp.active():   # any world size: a world of 1 runs the same collectives
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
            dp.shard_range(self.args.batch_size, self.rank, self.world)   # raises on an empty shard
            self.grad_arena = dp.FlatGradArena(self.params, average=False)
        self.train_dict = {"content_loss": [], "style_loss": [], "lf_loss": [], "tv_loss": [], "org_img_loss": []}
        self.save_file = os.path.join(self.args.save_dir, "ast.pth")
        self.train_dict_file = os.path.join(self.args.save_dir, "ast_train_dict.json")

    # ---- one step ----------------------------------------------------------------------------
    def compute_losses(self, content, style):
        a = self.args
        b = content.shape[0]
        with torch.no_grad():
            taps = self.lossnet(content, style)                  # both batches in the same launches
            if self.shared:
                f_c, f_s = taps[_RELU9][:b], taps[_RELU9][b:]
            else:
                f_c, f_s = self.net.encode_pair(content, style)
            t = self.net.adain(f_c, f_s)
            style_map = [taps[i][b:] for i in _LOSS_IDX]
            content_map = [taps[i][:b] for i in _LOSS_IDX]
        stylized = self.net.decoder(t)
        s_taps = self.lossnet(stylized)
        t_cs_map = [s_taps[i] for i in _LOSS_IDX]
        with torch.no_grad():
            enc_stylized = s_taps[_RELU9].detach() if self.shared else self.net.encoder(stylized.detach())[0]
            lf_loss = L.content_mvn_loss(t, enc_stylized)

        # content and style terms of each tap (and of the image) from one op: one input gradient each
        pairs = [L.content_style_loss(t_cs_map[i], content_map[i], style_map[i], 1.0, STYLE_WEIGHTS[i])
                 for i in range(len(t_cs_map))]
        pairs.append(L.content_style_loss(stylized, content, style, 0.1, 1.0))
        content_terms = [p[0] for p in pairs]
        style_terms = [p[1] for p in pairs]
        tv = L.tv_loss(stylized)
        content_loss = torch.stack(content_terms).sum()
        style_loss = torch.stack(style_terms).sum()
        mean_terms = a.content_lam * content_loss + a.style_lam * style_loss + a.lf_lam * lf_loss
        loss = mean_terms + a.tv_lam * tv
        out = {"loss": loss, "content_loss": content_loss, "style_loss": style_loss, "lf_loss": lf_loss,
               "tv_loss": tv, "stylized": stylized, "t": t}
        if getattr(a, "full_losses", False):
            org_out = self.net.decoder(f_c)
            o_taps = self.lossnet(org_out)
            org_terms = [L.compute_content_loss(o_taps[j], content_map[i]) for i, j in enumerate(_LOSS_IDX)]
            org_terms.append(L.pixel_mse_loss(org_out, content, 100.0))
            org_img_loss = torch.stack(org_terms).sum() * a.org_img_lam
            range_loss = L.out_of_range_loss(stylized, 1e8)
            hist_loss = L.compute_hist_loss(stylized, style, 1e-5)
            mean_terms = mean_terms + hist_loss + org_img_loss + range_loss
            out["loss"] = loss + hist_loss + org_img_loss + range_loss
            out.update(org_img_loss=org_img_loss, out_of_range_loss=range_loss, hist_loss=hist_loss, org_out=org_out)
        out["_mean_terms"] = mean_terms
        return out

    def shard_weight(self, local_n):
        """local / global images of this rank's shard (1.0 in a single process)."""
        if self.world == 1:
            return 1.0
        a, b = dp.shard_range(self.args.batch_size, self.rank, self.world)
        if local_n != b - a:
            raise ValueError(f"rank {self.rank} holds {local_n} images, its shard of the global batch "
                             f"{self.args.batch_size} over {self.world} ranks is {b - a}")
        return (b - a) / self.args.batch_size

    def train_step(self, content, style, record=False):
        with _lib.accumulator_pool():
            out = self.compute_losses(content, style)
        self.optim.zero_grad(set_to_none=True)
        w = self.shard_weight(content.shape[0])
        if w == 1.0:
            out["loss"].backward()
        else:   # batch-mean terms carry local/global, the batch-sum tv term is already additive
            (w * out["_mean_terms"] + self.args.tv_lam * out["tv_loss"]).backward()
        if self.grad_arena is not None:
            self.grad_arena.all_reduce()
        if self.grad_hook is not None:
            self.grad_hook(self.params)
        self.optim.step()
        out["grad_norm"] = self.optim.last_grad_norm
        if record:  # device -> host syncs, as train.py:302-306 does every step
            keys = ("content_loss", "style_loss", "lf_loss", "tv_loss") + (("org_img_loss",) if "org_img_loss" in out else ())
            vals = dp.global_terms({k: out[k] for k in keys}, {k: w for k in keys if k != "tv_loss"})
            for k in ("content_loss", "style_loss", "lf_loss", "tv_loss"):
                self.train_dict[k].append(float(vals[k].item()))
            self.train_dict["org_img_loss"].append(float(vals["org_img_loss"].item()) if "org_img_loss" in vals else 0.0)
        return out

    # ---- checkpoints (train.py:103-133) -------------------------------------------------------
    def save(self):
        """Rank 0 writes (every rank holds the same parameters after the reduced step); the others
        wait at a barrier so no rank reads a half-written file."""
        if dp.is_main():
            os.makedirs(self.args.save_dir, exist_ok=True)
            torch.save({"ast": self.net.state_dict(), "ast_optim": self.optim.state_dict()}, self.save_file)
            with open(self.train_dict_file, "w") as f:
                json.dump(self.train_dict, f)
        dp.barrier()

    def load(self):
        d = torch.load(self.save_file, map_location=self.device, weights_only=True)
        self.net.load_state_dict(d["ast"])
        self.optim.load_state_dict(d["ast_optim"])
        with open(self.train_dict_file) as f:
            self.train_dict = json.load(f)


# ------------------------------------------------------------------------------------------------
# The reference's own trainer: ASTTrainer (train.py:50-401) over the MobileNet AST with AdaAttN
# ------------------------------------------------------------------------------------------------

def default_ast_args(**kw):
    """train.py:405-440 defaults (batch_size, lr and the loss weights)."""
    a = dict(train_iter=10000, batch_size=8, lr=2e-4, content_lam=1.25, style_lam=0.5, tv_lam=0.0006, lf_lam=1.0,
             org_img_lam=0.5, save_dir="models/ast/", load=False, ae_model="models/auto_encoder/ae.pth")
    a.update(kw)
    return argparse.Namespace(**a)


class ASTTrainer:
    """ASTTrainer (train.py:50-401) on HIP: models.AST(attention=True) -- MobileNet encoder,
    AdaAttN at enc_out_layers (ada_att_1 / ada_att_2), ada_out, decoder -- trained end to end in
    train mode after load_ae (train.py:135-144), every parameter in one Adam (train.py:61).

    Per step (train.py:186-300):
      stylized, t, org_out = ast(content, style)          (t = the per-layer stylised maps)
      content/style/t_cs/org_out maps = lossnet(...)      (VGG19 to relu_15, frozen)
      enc_stylized = ast._enc(stylized)                   (train mode: BN running stats update)
      content = sum_i huber(mvn(t_cs_map_i), mvn(content_map_i)) + 0.1 huber(mvn(stylized), mvn(content))
      style   = sum_i w_i style_loss(t_cs_map_i, style_map_i) + style_loss(stylized, style)
      org_img = org_img_lam (sum_i huber(org_out_map_i, content_map_i) + 100 mean((content - org_out)^2))
      lf      = sum_i huber(mvn(t_i), mvn(enc_stylized_i))  (gradient into AdaAttN)
      loss = content_lam content + style_lam style + lf_lam lf + tv_lam tv + 1e-5 hist + org_img + 1e8 out_of_range
      clip_grad_norm_(2.0, error_if_nonfinite) + Adam(lr, (0.9, 0.999), 1e-5)
    Data parallel as AdaINTrainer (args.batch_size = global batch, shard-weighted batch-mean terms,
    one SUM all-reduce of the flat gradient arena) plus SyncBatchNorm for the train-mode encoder."""

    def __init__(self, args=None, device=None, ast=None, lossnet=None, content_iter=None, grad_hook=None,
                 graph=None):
        self.args = args or default_ast_args()
        self.device = torch.device(device or "cuda")
        self.ast = (ast or models.AST(attention=True)).to(self.device).train()
        self.pretrained_enc = (lossnet or models.PretrainedEncoder()).to(self.device).eval()
        self.pretrained_enc.requires_grad_(False)
        self.content_iter = content_iter
        if ast is None and not self.args.load and self.args.ae_model and os.path.exists(self.args.ae_model):
            self.load_ae()
        self.params = list(self.ast.parameters())
        self.ast_optim = FusedAdam(self.params, lr=self.args.lr, betas=(0.9, 0.999), eps=1e-5, max_grad_norm=2.0,
                                   error_if_nonfinite=True)
        self.grad_hook = grad_hook
        self.rank, self.world = 0, 1
        self.grad_arena = None
        if dp.active():   # any world size: a world of 1 runs the same collectives
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
            dp.shard_range(self.args.batch_size, self.rank, self.world)
            dp.convert_sync_batchnorm(self.ast)
            self.grad_arena = dp.FlatGradArena(self.params, average=False)
        # graph mode (default on in one process: the step is launch-bound at the reference's 160^2
        # training size): the whole step replays as one hipGraph (StepGraph); grad_hook is then not
        # called. Off by default under data parallelism: gloo stages every collective through the
        # host (a synchronising copy, which a capture refuses), and capturing the RCCL all-reduce
        # and SyncBatchNorm's all-gather at world size > 1 has not been verified.
        if graph is None:
            graph = getattr(self.args, "graph", self.world == 1)
        graph = graph and grad_hook is None   # a grad_hook needs the eager step
        if graph and self.world > 1:
            raise ValueError("ASTTrainer(graph=True) runs in one process only: gloo collectives stage through "
                             "the host and cannot be captured, and a captured RCCL all-reduce / SyncBatchNorm "
                             "all-gather at world size > 1 has not been checked against the eager step")
        self.graph = graph
        self._step_graph = None
        if self.graph:
            if self.grad_arena is None:   # persistent gradient storage for the captured optimizer tables
                self.grad_arena = dp.FlatGradArena(self.params, average=False)
            self._step_graph = StepGraph(self.ast_optim, self.grad_arena, self.params, self._step_body,
                                         frozen=[self.pretrained_enc])
        self.train_dict = {"content_loss": [], "style_loss": [], "lf_loss": [], "tv_loss": [], "org_img_loss": []}
        self.save_file = os.path.join(self.args.save_dir, "ast.pth")
        self.train_dict_file = os.path.join(self.args.save_dir, "ast_train_dict.json")
        if self.args.load:
            self.load()

    def load_ae(self, path=None):
        """train.py:135-144: the pretrained AutoEncoder's encoder / ada_out / decoder into the AST."""
        d = torch.load(path or self.args.ae_model, map_location=self.device, weights_only=True)
        ae = models.AutoEncoder()
        ae.load_state_dict(d["AE"])
        self.ast._enc.load_state_dict(ae.encoder.state_dict())
        self.ast.ada_out.load_state_dict(ae.ada_out.state_dict())
        self.ast._dec.load_state_dict(ae.decoder.state_dict())

    def compute_losses(self, content, style):
        a = self.args
        b = content.shape[0]
        stylized, t, org_out = self.ast(content, style)                                 # train.py:191
        with torch.no_grad():
            if content.shape == style.shape:                                            # :193-194, one pass
                both = self.pretrained_enc(content, style)
                content_map, style_map = [m[:b] for m in both], [m[b:] for m in both]
            else:
                content_map, style_map = self.pretrained_enc(content), self.pretrained_enc(style)
            # :198 (the reference records autograd here but only ever uses the result detached)
            enc_stylized = self.ast._enc(stylized.detach(), out_layers=enc_out_layers)
        if stylized.shape == org_out.shape:
            # :195-196 in ONE pass over both batches: the loss network's small maps (20^2, 10^2 at
            # 512 channels) fill twice the workgroups per launch; every conv is per image, so each
            # half equals its own pass (the frozen network has no weight gradient to mix them)
            both_maps = self.pretrained_enc(torch.cat([stylized, org_out]))
            halves = [m.split(b) for m in both_maps]
            t_cs_map, org_out_map = [h[0] for h in halves], [h[1] for h in halves]
        else:
            t_cs_map = self.pretrained_enc(stylized)                                    # :195
            org_out_map = self.pretrained_enc(org_out)                                  # :196
        # :217-227 content and :230-245 style terms per tap, :258 / :271 on the image, pairwise fused
        pairs = [L.content_style_loss(x, yc, ys, 1.0, w) for x, yc, ys, w in zip(t_cs_map, content_map, style_map,
                                                                                STYLE_WEIGHTS)]
        pairs.append(L.content_style_loss(stylized, content, style, 0.1, 1.0))
        content_terms = [p[0] for p in pairs]
        style_terms = [p[1] for p in pairs]
        org_terms = [L.compute_content_loss(x, y) for x, y in zip(org_out_map, content_map)]           # :248-256
        org_terms.append(L.pixel_mse_loss(org_out, content, 100.0))                                    # :268
        content_loss = torch.stack(content_terms).sum()
        style_loss = torch.stack(style_terms).sum()
        org_img_loss = torch.stack(org_terms).sum() * a.org_img_lam                                    # :269
        range_loss = L.out_of_range_loss(stylized, 1e8)                                                # :259
        hist_loss = L.compute_hist_loss(stylized, style, 1e-5)                                         # :261
        lf_loss = torch.stack([L.content_mvn_loss(x, y) for x, y in zip(t, enc_stylized)]).sum()       # :275-277
        tv = L.tv_loss(stylized)                                                                       # :282
        mean_terms = (a.content_lam * content_loss + a.style_lam * style_loss + a.lf_lam * lf_loss + hist_loss
                      + org_img_loss + range_loss)
        loss = mean_terms + a.tv_lam * tv                                                              # :283
        return {"loss": loss, "_mean_terms": mean_terms, "content_loss": content_loss, "style_loss": style_loss,
                "lf_loss": lf_loss, "tv_loss": tv, "org_img_loss": org_img_loss, "hist_loss": hist_loss,
                "out_of_range_loss": range_loss, "stylized": stylized, "t": t, "org_out": org_out}

    def _backward(self, out, n_local):
        if self.world == 1:
            out["loss"].backward()                                                      # :288
        else:
            a, b = dp.shard_range(self.args.batch_size, self.rank, self.world)
            if n_local != b - a:
                raise ValueError(f"rank {self.rank} holds {n_local} images, its shard is {b - a}")
            ((b - a) / self.args.batch_size * out["_mean_terms"] + self.args.tv_lam * out["tv_loss"]).backward()
        if self.grad_arena is not None:
            self.grad_arena.all_reduce()

    def _step_body(self, content, style):
        """The captured step (StepGraph): losses, backward, reduction, clip + Adam."""
        with mbtrain.deferred_bn_counters():
            out = self.compute_losses(content, style)
        self._backward(out, content.shape[0])
        self.ast_optim.step_static()
        return out

    def train_step(self, content, style, record=False):
        if self.graph:
            out = self._step_graph.run(content, style)
        else:
            with mbtrain.deferred_bn_counters():
                out = self.compute_losses(content, style)
            self.ast_optim.zero_grad(set_to_none=True)                                  # :287
            self._backward(out, content.shape[0])
            if self.grad_hook is not None:
                self.grad_hook(self.params)
            self.ast_optim.step()                                                       # :292, :300
            out["grad_norm"] = self.ast_optim.last_grad_norm
        if record:                                                                      # :302-306
            keys = ("content_loss", "style_loss", "lf_loss", "tv_loss", "org_img_loss")
            w = 1.0 if self.world == 1 else dp.shard_weight(self.args.batch_size, self.rank, self.world)
            vals = dp.global_terms({k: out[k] for k in keys}, {k: w for k in keys if k != "tv_loss"})
            for k in keys:
                self.train_dict[k].append(float(vals[k].item()))
        return out

    def train(self):
        for cur_iter in range(self.args.train_iter):                                    # :150
            content, style = next(self.content_iter)
            self.train_step(content.to(self.device), style.to(self.device), record=True)
            if (cur_iter + 1) % 32 == 0:                                                # :313
                self.save()

    def save(self):
        if dp.is_main():   # rank 0 writes, the others wait (identical parameters after the reduced step)
            os.makedirs(self.args.save_dir, exist_ok=True)
            torch.save({"ast": self.ast.state_dict(), "ast_optim": self.ast_optim.state_dict()}, self.save_file)
            with open(self.train_dict_file, "w") as f:
                json.dump(self.train_dict, f)
        dp.barrier()

    def load(self):
        d = torch.load(self.save_file, map_location=self.device, weights_only=True)
        self.ast.load_state_dict(d["ast"])
        self.ast_optim.load_state_dict(d["ast_optim"])
        for g in self.ast_optim.param_groups:                                           # train.py:94-98
            g["betas"], g["lr"], g["eps"] = (0.9, 0.999), self.args.lr, 1e-5
        with open(self.train_dict_file) as f:
            self.train_dict = json.load(f)


# ------------------------------------------------------------------------------------------------
# AutoEncoder training (train_autoencoder.py:16-148; SURVEY.md §8f "next" #4)
# ------------------------------------------------------------------------------------------------

def default_ae_args(**kw):
    """train_autoencoder.py:250-264 defaults."""
    a = dict(train_iter=8192, batch_size=16, lr=2e-4, save_dir="models/auto_encoder/", load=False,
             recon_lam=100.0, perp_lam=0.01)
    a.update(kw)
    return argparse.Namespace(**a)


class AutoencoderTrainer:
    """AutoencoderTrainer (train_autoencoder.py:16-148) on HIP: the MobileNet AutoEncoder in
    training mode (BatchNorm batch statistics, mbtrain.py), reconstruction Huber loss plus the
    perceptual Huber loss over the frozen VGG loss network's six layers, clip_grad_norm_(10) and
    Adam(betas (0.9, 0.99), eps 1e-7), fused (optim.FusedAdam). Checkpoint and train_dict.json
    layout as the reference (ae.pth {"AE", "optim"}; train_loss / val_loss / perp_loss)."""

    def __init__(self, args=None, content_iter=None, val_loader=None, device=None, model=None, lossnet=None):
        self.args = args or default_ae_args()
        self.device = torch.device(device or "cuda")
        self.content_iter, self.val_loader = content_iter, val_loader
        self.model = (model or models.AutoEncoder()).to(self.device).train()
        self.pretrained_mobnet = (lossnet or models.PretrainedEncoder()).to(self.device).eval()
        self.pretrained_mobnet.requires_grad_(False)
        self.ae_optim = FusedAdam(list(self.model.parameters()), lr=self.args.lr, betas=(0.9, 0.99), eps=1e-7,
                                  max_grad_norm=10.0)
        # data-parallel (one process per GPU, batch-sharded): SyncBatchNorm keeps the reference's
        # whole-batch statistics, one all-reduce averages the gradient arena before clip + Adam
        # (args.batch_size = the global batch; each rank back-propagates its batch-mean losses
        # weighted by local/global images and the arena SUMS: the full-batch gradient, uneven
        # shards included)
        self.grad_arena = None
        self.rank, self.world = 0, 1
        if dp.active():   # any world size: a world of 1 runs the same collectives
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
            dp.shard_range(self.args.batch_size, self.rank, self.world)   # raises on an empty shard
            dp.convert_sync_batchnorm(self.model)
            self.grad_arena = dp.FlatGradArena(list(self.model.parameters()), average=False)
        self.save_file = os.path.join(self.args.save_dir, "ae.pth")
        self.train_dict_file = os.path.join(self.args.save_dir, "train_dict.json")
        self.train_dict = {"train_loss": [], "val_loss": [], "perp_loss": []}

    def compute_losses(self, content_imgs):
        recon_imgs = self.model(content_imgs)
        recon_loss = L.compute_content_loss(recon_imgs, content_imgs)                  # nn.HuberLoss(), :129
        with torch.no_grad():
            content_maps = self.pretrained_mobnet(content_imgs)                        # :132
        recon_maps = self.pretrained_mobnet(recon_imgs)                                # :133
        terms = [L.compute_content_loss(r, c) for r, c in zip(recon_maps, content_maps)]   # :137-151
        content_loss = torch.stack(terms).sum()
        loss = self.args.recon_lam * recon_loss + self.args.perp_lam * content_loss   # :156
        return {"loss": loss, "recon_loss": recon_loss, "content_loss": content_loss, "recon": recon_imgs}

    def train_step(self, content_imgs, record=True):
        with mbtrain.deferred_bn_counters():
            out = self.compute_losses(content_imgs)
        self.ae_optim.zero_grad(set_to_none=True)
        if self.world == 1:
            out["loss"].backward()
        else:
            a, b = dp.shard_range(self.args.batch_size, self.rank, self.world)
            if content_imgs.shape[0] != b - a:
                raise ValueError(f"rank {self.rank} holds {content_imgs.shape[0]} images, its shard of the global "
                                 f"batch {self.args.batch_size} is {b - a}")
            ((b - a) / self.args.batch_size * out["loss"]).backward()
        if self.grad_arena is not None:
            self.grad_arena.all_reduce()
        self.ae_optim.step()                                                           # clip 10 + Adam, :159-165
        out["grad_norm"] = self.ae_optim.last_grad_norm
        if record:   # full-batch values (shard-weighted sums over ranks)
            w = 1.0 if self.world == 1 else dp.shard_weight(self.args.batch_size, self.rank, self.world)
            vals = dp.global_terms({"recon_loss": out["recon_loss"], "content_loss": out["content_loss"]},
                                   {"recon_loss": w, "content_loss": w})
            self.train_dict["train_loss"].append(float(vals["recon_loss"].item()))
            self.train_dict["perp_loss"].append(float(vals["content_loss"].item()))
        return out

    def train(self):
        for cur_iter in range(self.args.train_iter):
            if (cur_iter + 1) % 32 == 0:
                self.save()
                if (cur_iter + 1) % 64 == 0 and self.val_loader is not None:
                    self.validate()
            self.train_step(next(self.content_iter).to(self.device))

    @torch.no_grad()
    def validate(self):
        """train_autoencoder.py:71-82 (mean absolute reconstruction error per image; a logged metric)."""
        val_imgs = next(self.val_loader).to(self.device)
        self.model.eval()
        recon_imgs = self.model(val_imgs)
        self.train_dict["val_loss"].append(float((val_imgs - recon_imgs).abs().mean().item()) / val_imgs.shape[0])
        self.model.train()

    def save(self):
        if dp.is_main():   # rank 0 writes, the others wait (identical parameters after the reduced step)
            os.makedirs(self.args.save_dir, exist_ok=True)
            torch.save({"AE": self.model.state_dict(), "optim": self.ae_optim.state_dict()}, self.save_file)
            with open(self.train_dict_file, "w") as f:
                json.dump(self.train_dict, f)
        dp.barrier()

    def load(self):
        d = torch.load(self.save_file, map_location=self.device, weights_only=True)
        self.model.load_state_dict(d["AE"])
        self.ae_optim.load_state_dict(d["optim"])
        with open(self.train_dict_file) as f:
            self.train_dict = json.load(f)
