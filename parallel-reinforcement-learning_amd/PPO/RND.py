"""Random Network Distillation — drop-in for the reference's PPO/RND.py:8-115.

Same modules, parameter names, initialisation and optimiser as the reference (target_net and
pred_net are independent re-initialisations of Linear(D,64) -> GroupNorm(8,64) -> SiLU ->
Linear(64,D); target frozen; AdamW lr 1e-3 + MSE for the predictor).  The intrinsic-reward
forward (the hot part: every learn() call runs it over all N transitions) is one fused HIP
kernel on fp32 MFMA (prl_rnd_forward); the predictor update's forward / backward stay PyTorch
(north star), replayed as one HIP graph per minibatch on one GPU with the native AdamW
(prl_flat_adamw) stepping flat views of the predictor's state.
"""
from __future__ import annotations

import os
from copy import deepcopy
from types import SimpleNamespace

import torch
from torch import nn, optim

import prl_native

from .layers import GroupNormSiLU, Linear


class _MSELoss(torch.autograd.Function):
    """nn.MSELoss()(preds, targets) (mean reduction) for update_pred's [mb, D] batches: the
    difference is formed once and kept for the backward (2 (p - t) / numel), and the mean of its
    squares is one rocBLAS dot instead of PyTorch-ROCm's generic reduction (~140 us per
    65,536 x 348 batch, RND.py:112 at C5's mini_batch).  Float32, same value up to summation
    order."""

    @staticmethod
    def forward(ctx, preds, targets):
        d = (preds - targets).contiguous()
        ctx.save_for_backward(d)
        flat = d.view(-1)
        return torch.dot(flat, flat) / float(flat.numel())

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d * (g * (2.0 / float(d.numel()))), None


class _MaskedMSELoss(torch.autograd.Function):
    """The graphed update's MSE: the rows past the minibatch's (mask 0: a ragged minibatch padded
    to the graph's static shape) contribute nothing, and inv = 1 / (rows x D) is a device scalar,
    so one captured graph serves every minibatch size.  With mask = 1 it is _MSELoss: the same
    gradient bits (2 * inv is exact), the loss up to multiplying by 1/numel instead of dividing."""

    @staticmethod
    def forward(ctx, preds, targets, mask, inv):
        d = (preds - targets).mul_(mask)
        ctx.save_for_backward(d, inv)
        flat = d.view(-1)
        return torch.dot(flat, flat) * inv

    @staticmethod
    def backward(ctx, g):
        d, inv = ctx.saved_tensors
        return d * (g * 2.0 * inv), None, None, None


def mse_loss(preds, targets):
    if preds.is_cuda and preds.dtype == torch.float32 and preds.shape == targets.shape:
        return _MSELoss.apply(preds, targets)
    return nn.functional.mse_loss(preds, targets)


class RND(nn.Module):
    def __init__(self, in_features: int, out_features: int, beta: float = 0.001, device=None):
        super().__init__()
        model = nn.Sequential(Linear(in_features, 64), GroupNormSiLU(8, 64), nn.Identity(),
                              Linear(64, out_features))
        self.target_net = deepcopy(model)
        self.pred_net = deepcopy(model)
        del model
        self.init_weights()
        for p in self.target_net.parameters():
            p.requires_grad = False
        self.beta = beta
        self.loss_fn = nn.MSELoss()
        self.optimizer = optim.AdamW(params=self.pred_net.parameters(), lr=0.001)
        self.eval()
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.to(device)

    def init_weights(self):  # RND.py:43-57
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.normal_(m.bias, mean=0, std=0.01)
            elif isinstance(m, nn.GroupNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    @staticmethod
    def _params(net):
        return (net[0].weight, net[0].bias, net[1].weight, net[1].bias, net[3].weight, net[3].bias)

    @staticmethod
    def _concat(values):
        if isinstance(values, torch.Tensor):
            return values
        values = list(values)
        return values[0] if len(values) == 1 else torch.cat(values, dim=0)

    @torch.no_grad()
    def compute_intrinsic_reward(self, values) -> torch.Tensor:
        """RND.py:71-94: beta * ||pred(x) - target(x)||_2 per row.  `values` is the reference's
        list of minibatches (PPO.batch_packer) or one [N, D] tensor; rows keep their order."""
        x = self._concat(values)
        dev = self.target_net[0].weight.device
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        out = torch.empty(x.shape[0], dtype=torch.float32, device=dev)
        tp = [p.detach().contiguous() for p in self._params(self.target_net)]
        pp = [p.detach().contiguous() for p in self._params(self.pred_net)]
        prl_native.rnd_forward(x, tp, pp, float(self.beta), out)
        return out

    # ------------------------------------------------------------------ graphed update (one GPU)
    def _flat_state(self):
        """The predictor's parameters, gradients and AdamW state as flat vectors (views, as the
        policy's: update.FlatAdamState), so one native AdamW launch steps them."""
        from .update import FlatAdamState
        params = list(self.pred_net.parameters())
        fa = getattr(self, "_fa", None)
        # rebuilt when the parameters OR the optimizer object were replaced: the flat state holds
        # the optimizer it was built for, and a new one must get its moments / step count
        if (fa is None or fa.ppo.optimizer is not self.optimizer or len(fa.params) != len(params)
                or any(a is not b for a, b in zip(fa.params, params))):
            fa = self._fa = FlatAdamState(SimpleNamespace(policy=self.pred_net, optimizer=self.optimizer))
            self._fgrad = torch.zeros_like(fa.flat)
            self._graph = None
        else:
            fa.prepare()
        off = 0
        base = self._fgrad.data_ptr()
        for p in params:   # every .grad a view of the flat gradient (re-attached if replaced)
            if p.grad is None or p.grad.data_ptr() != base + 4 * off:
                p.grad = self._fgrad[off:off + p.numel()].view_as(p)
            off += p.numel()
        return fa

    def _step_body(self, x, fa, mask=None, inv=None):
        """One update_pred step on rows x: MSE(pred(x), target(x)) backward into the flat
        gradient, then AdamW (no clipping: max_norm = inf gives the coefficient 1).  mask / inv:
        the graphed step's row mask and 1 / (rows x D) (rows past the minibatch are padding)."""
        self._fgrad.zero_()
        with torch.no_grad():
            targets = self.target_net(x)
        preds = self.pred_net(x)
        if mask is not None:
            loss = _MaskedMSELoss.apply(preds, targets, mask, inv)
        else:
            loss = (mse_loss(preds, targets)
                    if isinstance(self.loss_fn, nn.MSELoss) and self.loss_fn.reduction == "mean"
                    else self.loss_fn(preds, targets))
        loss.backward()
        group = self.optimizer.param_groups[0]
        beta1, beta2 = group["betas"]
        prl_native.flat_adamw(fa.flat, fa.m, fa.v, fa.step, self._fgrad, group["lr"], beta1, beta2,
                              group["eps"], group["weight_decay"], float("inf"), fa.total_norm)

    def _flat_optimizer_ok(self) -> bool:
        """The native flat AdamW stands in for self.optimizer / self.loss_fn only when they are
        exactly what it computes: one-group torch AdamW (no amsgrad / maximize), f32 parameters
        on the GPU, and the reference's nn.MSELoss(reduction='mean') (RND.py:45)."""
        w = self.pred_net[0].weight
        if not (w.is_cuda and w.dtype == torch.float32) or type(self.optimizer) is not optim.AdamW:
            return False
        if len(self.optimizer.param_groups) != 1:
            return False
        group = self.optimizer.param_groups[0]
        if group.get("amsgrad") or group.get("maximize"):
            return False
        return isinstance(self.loss_fn, nn.MSELoss) and self.loss_fn.reduction == "mean"

    def _flat_dp_ok(self) -> bool:
        # rank-invariant inputs only (optimizer, loss_fn, parameter device / dtype): the flat and
        # the per-parameter loops issue different numbers of collectives per step, so every rank
        # must take the same one whatever its own minibatches look like
        return self._flat_optimizer_ok()

    def _native_ok(self, values) -> bool:
        """The fused predictor-gradient kernel (prl_rnd_pred_grad) runs every step when the loss
        and optimizer are the reference's (_flat_optimizer_ok), D % 4 == 0 and the minibatches are
        contiguous f32 device rows (PRL_RND_NATIVE=0: the graphed / PyTorch steps).  Rank-invariant
        on data-parallel ranks except for the minibatches, which only choose between two paths
        that issue the same single all-reduce per step."""
        if os.environ.get("PRL_RND_NATIVE", "1") == "0" or not torch.cuda.is_available():
            return False
        if not self._flat_optimizer_ok():
            return False
        D = self.pred_net[0].weight.shape[1]
        if D % 4 != 0 or self.pred_net[3].weight.shape[0] != D:
            return False
        return all(v.is_cuda and v.dtype == torch.float32 and v.dim() == 2 and v.shape[1] == D
                   for v in values)

    def _update_native(self, values, all_reduce=None, counts=None) -> None:
        """update_pred with the fused gradient kernel: per minibatch ONE prl_rnd_pred_grad (both
        forwards, MSE, the predictor's backward, written into the flat gradient the parameters'
        .grad view) and the native flat AdamW launch (max_norm = inf), plus, on data-parallel ranks, one
        all-reduce of the flat gradient (each rank's rows scaled by 2 / (union rows D): the
        union's mean).  Same steps in the same order as the loops below."""
        fa = self._flat_state()
        group = self.optimizer.param_groups[0]
        beta1, beta2 = group["betas"]
        D = self.pred_net[0].weight.shape[1]

        tnet = [p.detach().contiguous() for p in self._params(self.target_net)]
        pnet = [p.detach().contiguous() for p in self._params(self.pred_net)]
        mb = max([v.shape[0] for v in values] + [1])
        need = prl_native.rnd_pred_grad_ws_floats(mb, D)
        part = getattr(self, "_rg_partial", None)
        if part is None or part.numel() < need or part.device != fa.flat.device:
            self._rg_partial = part = torch.empty(max(need, 1), dtype=torch.float32,
                                                  device=fa.flat.device)
        steps = len(values) if counts is None else len(counts)
        for j in range(steps):
            if j < len(values):
                x = values[j] if values[j].is_contiguous() else values[j].contiguous()
                rows = x.shape[0] if counts is None else counts[j]
                prl_native.rnd_pred_grad(x, tnet, pnet, 2.0 / (rows * D), part, self._fgrad)
            else:
                self._fgrad.zero_()
            if all_reduce is not None:
                all_reduce(self._fgrad)
            prl_native.flat_adamw(fa.flat, fa.m, fa.v, fa.step, self._fgrad, group["lr"], beta1,
                                  beta2, group["eps"], group["weight_decay"], float("inf"),
                                  fa.total_norm)
        fa.sync()

    def _graphed_ok(self, values, all_reduce, counts) -> bool:
        if all_reduce is not None or counts is not None or os.environ.get("PRL_RND_GRAPH", "1") == "0":
            return False
        if not values or not torch.cuda.is_available():
            return False
        if not self._flat_optimizer_ok():
            return False
        return all(v.is_cuda and v.dtype == torch.float32 and v.dim() == 2 for v in values)

    def _update_graphed(self, values) -> None:
        """update_pred on one GPU: every minibatch replays ONE captured HIP graph of the step
        (forward of both nets, masked MSE, backward, native AdamW) on a static input buffer the
        minibatch is copied into; a ragged last minibatch fills the buffer's first rows and a
        row mask zeroes the rest's contribution (the padding rows hold the previous minibatch's
        finite values, so 0 x them is 0).  The first minibatch of a new shape runs eagerly on a
        side stream (PyTorch's warm-up before a capture, a real step) and is then captured.  Same
        steps in the same order as the loop below; the ragged step sums the same products with
        zero rows added (float32 rounding only); AdamW's arithmetic is prl_flat_adamw's (torch's
        up to fused multiply-adds)."""
        fa = self._flat_state()
        mb = max(v.shape[0] for v in values)
        D = values[0].shape[1]
        # the captured AdamW launch holds the hyper-parameters as constants: a changed lr / betas /
        # eps / weight decay (a scheduler, a user edit of param_groups) re-captures
        group = self.optimizer.param_groups[0]
        hyper = (float(group["lr"]), tuple(float(b) for b in group["betas"]), float(group["eps"]),
                 float(group["weight_decay"]))
        if getattr(self, "_graph_hyper", None) != hyper:
            self._graph = None
            self._graph_hyper = hyper
        for v in values:
            v = v.contiguous()
            rows = v.shape[0]
            g = self._graph
            if g is None or self._graph_x.shape != (mb, D):
                # warm-up (a real step, unpadded) and capture on a side stream, as PyTorch requires
                self._graph_x = torch.zeros(mb, D, dtype=torch.float32, device=v.device)
                self._graph_mask = torch.ones(mb, 1, dtype=torch.float32, device=v.device)
                self._graph_inv = torch.full((), 1.0 / (mb * D), dtype=torch.float32, device=v.device)
                self._graph_rows = mb
                g = torch.cuda.CUDAGraph()
                cur = torch.cuda.current_stream()
                s = torch.cuda.Stream()
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    self._step_body(v, fa)
                    with torch.cuda.graph(g, stream=s):
                        self._step_body(self._graph_x, fa, self._graph_mask, self._graph_inv)
                cur.wait_stream(s)
                self._graph = g
                continue
            if rows != self._graph_rows:
                self._graph_mask[:rows].fill_(1.0)
                self._graph_mask[rows:].fill_(0.0)
                self._graph_inv.fill_(1.0 / (rows * D))
                self._graph_rows = rows
            self._graph_x[:rows].copy_(v)
            g.replay()
        fa.sync()

    def update_pred(self, values, all_reduce=None, counts=None) -> None:
        """RND.py:96-115: one MSE/AdamW pass of the predictor over the minibatches (PyTorch).

        Data-parallel ranks (all_reduce, counts given): minibatch j is the union of the ranks'
        j-th minibatches, counts[j] its rows.  Each rank weights its MSE by its share of the union
        (the union's MSE is the row-weighted mean of the ranks'), the predictor's gradient is
        all-reduced (SUM) and every rank takes the same AdamW step; len(counts) steps on every
        rank, ranks past their last minibatch contribute zero gradients (lockstep)."""
        self.pred_net.train()
        values = list(values)
        if self._native_ok(values):
            self._update_native(values, all_reduce, counts)
            self.pred_net.eval()
            return
        if self._graphed_ok(values, all_reduce, counts):
            self._update_graphed(values)
            self.pred_net.eval()
            return
        steps = len(values) if counts is None else len(counts)
        if all_reduce is not None and self._flat_dp_ok():
            # data-parallel ranks on the GPU: the gradient is ONE flat buffer (the parameters'
            # .grad are views of it), so each step is one all-reduce instead of one per parameter
            # tensor, and AdamW is the native flat launch (max_norm = inf: no clipping)
            fa = self._flat_state()
            group = self.optimizer.param_groups[0]
            beta1, beta2 = group["betas"]
            for j in range(steps):
                self._fgrad.zero_()
                if j < len(values):
                    i = values[j]
                    with torch.no_grad():
                        targets = self.target_net(i)
                    preds = self.pred_net(i)
                    loss = mse_loss(preds, targets)
                    if counts is not None:
                        loss = loss * (i.shape[0] / counts[j])
                    loss.backward()
                all_reduce(self._fgrad)
                prl_native.flat_adamw(fa.flat, fa.m, fa.v, fa.step, self._fgrad, group["lr"], beta1,
                                      beta2, group["eps"], group["weight_decay"], float("inf"),
                                      fa.total_norm)
            fa.sync()
            self.pred_net.eval()
            return
        params = list(self.pred_net.parameters())
        for j in range(steps):
            self.optimizer.zero_grad()
            if j < len(values):
                i = values[j]
                with torch.no_grad():
                    targets = self.target_net(i)
                preds = self.pred_net(i)
                loss = (mse_loss(preds, targets)
                        if isinstance(self.loss_fn, nn.MSELoss) and self.loss_fn.reduction == "mean"
                        else self.loss_fn(preds, targets))
                if counts is not None:
                    loss = loss * (i.shape[0] / counts[j])
                loss.backward()
            if all_reduce is not None:
                for p in params:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                    all_reduce(p.grad)
            self.optimizer.step()
        self.pred_net.eval()
