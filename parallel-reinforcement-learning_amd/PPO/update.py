"""Graph-captured PPO optimizer step (PPO/PPO.py:219-255).

The reference runs k_epochs x ceil(N / mini_batch_size) optimizer steps in sequence (22,528 at
N = 2^20, mb = 512): at that size each step is a few dozen tiny kernels, so the loop is bound by
launch overhead, not by the GPU.  Here ONE full step — minibatch gather (device cursor) ->
policy forward (PyTorch GEMMs, HIP GroupNorm+SiLU and Categorical) -> HIP surrogate -> autograd
backward -> [RCCL all-reduce of the flat gradient] -> clip_grad_norm_(2.0) -> capturable AdamW ->
cursor += 1 — is captured once per learn() into a HIP graph and replayed for every full
minibatch, in order.  With world_size > 1 the step is two graphs (forward/backward/flatten, then
clip/AdamW) and the RCCL all-reduce of the flat gradient is issued eagerly between the two
replays: no collective is ever captured.  The first two minibatches of epoch 0 run eagerly on a side stream (the
warm-up PyTorch requires before capture) and are real steps, so the sequence of updates is the
reference's exactly.  Ragged / uneven minibatches (the last partial one, or ranks with fewer rows)
run through PPO._eager_step.
"""
from __future__ import annotations

import os

import torch
from torch import nn

import prl_native


def wide_info(ppo, D: int):
    """prl_ppo_wide_grad's (params, partial floats, grid) for this policy, or None when the wide
    step does not apply (shape outside it, use_fused off, or PRL_WIDE=0)."""
    if os.environ.get("PRL_WIDE", "1") != "1" or not getattr(ppo, "use_fused", True):
        return None
    info = prl_native.ppo_wide_info(D, ppo.action_dim, not ppo.is_continuous,
                                    ppo.mini_batch_size)
    n_params = sum(p.numel() for p in ppo.policy.parameters())
    if info is None or info[0] != n_params or n_params != sum(
            p.numel() for p in ppo.policy.parameters() if p.requires_grad):
        return None
    return info


class FlatAdamState:
    """The policy's parameters, gradients and AdamW state as flat f32 vectors in parameters()
    order, for prl_flat_adamw (clip_grad_norm_(2.0) + AdamW.step() in two launches, PPO.py:248-250):
    every Parameter's .data, every .grad (PPO._ensure_flat_grads) and the optimizer's exp_avg /
    exp_avg_sq state tensors are VIEWS of these buffers, so torch's own optimizer, state_dict()
    and save_weights see the same copy (as engine.FusedUpdate does for the persistent engine).
    The step count lives in one device scalar; sync() writes it into the optimizer's per-param
    state."""

    def __init__(self, ppo):
        self.ppo = ppo
        self.params = [p for p in ppo.policy.parameters()]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step = torch.zeros(1, dtype=torch.float32, device=dev)
        # [0] clip_grad_norm_'s value, [1] prl_flat_adamw's arrival counter (kept at zero)
        self.total_norm = torch.zeros(2, dtype=torch.float32, device=dev)
        self._bind()

    def _views(self, buf):
        out, off = [], 0
        for p in self.params:
            out.append(buf[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out

    def _bind(self):
        opt = self.ppo.optimizer
        self._opt = opt   # the optimizer these moments belong to (a replaced one re-binds)
        self.step.zero_()
        with torch.no_grad():
            for p, fv, mv, vv in zip(self.params, self._views(self.flat), self._views(self.m),
                                     self._views(self.v)):
                fv.copy_(p.data)
                p.data = fv
                st = opt.state.get(p)
                if st and "exp_avg" in st:
                    mv.copy_(st["exp_avg"])
                    vv.copy_(st["exp_avg_sq"])
                    self.step.copy_(torch.as_tensor(st["step"], dtype=torch.float32).reshape(1))
                    st["exp_avg"], st["exp_avg_sq"] = mv, vv
                else:
                    mv.zero_()
                    vv.zero_()

    def bound(self) -> bool:
        opt = self.ppo.optimizer
        if opt is not self._opt:
            return False
        for p, fv, mv in zip(self.params, self._views(self.flat), self._views(self.m)):
            if p.data.data_ptr() != fv.data_ptr():
                return False
            st = opt.state.get(p)
            if st and "exp_avg" in st and st["exp_avg"].data_ptr() != mv.data_ptr():
                return False
        return True

    def prepare(self):
        """Before a learn's first step: re-bind if the parameters or the optimizer state were
        replaced, else take the optimizer's step count (torch may have stepped in between)."""
        if not self.bound():
            self._bind()
            return
        st = self.ppo.optimizer.state.get(self.params[0])
        if st and "step" in st:
            self.step.copy_(torch.as_tensor(st["step"], dtype=torch.float32).reshape(1))

    def launch(self, grad, max_norm=2.0):
        group = self.ppo.optimizer.param_groups[0]
        beta1, beta2 = group["betas"]
        prl_native.flat_adamw(self.flat, self.m, self.v, self.step, grad, group["lr"], beta1,
                              beta2, group["eps"], group["weight_decay"], max_norm, self.total_norm)

    def sync(self):
        """The optimizer's state = this one's: moments as views, step counts = ours."""
        opt = self.ppo.optimizer
        group = opt.param_groups[0]
        on_device = bool(group.get("capturable") or group.get("fused"))
        host_step = None   # torch's default AdamW keeps host step counts: ONE device read for all
        for p, mv, vv in zip(self.params, self._views(self.m), self._views(self.v)):
            st = opt.state[p]
            st["exp_avg"], st["exp_avg_sq"] = mv, vv
            if "step" in st and torch.is_tensor(st["step"]) and st["step"].is_cuda:
                st["step"].copy_(self.step.reshape(st["step"].shape))
            elif on_device:
                st["step"] = self.step.reshape(()).clone()
            else:
                if host_step is None:
                    host_step = float(self.step.item())
                if "step" in st and torch.is_tensor(st["step"]):
                    st["step"].fill_(host_step)
                else:
                    st["step"] = torch.tensor(host_step)


def flat_adam_ok(optimizer) -> bool:
    """prl_flat_adamw computes one-group torch AdamW without amsgrad / maximize: anything else
    (another optimizer type, extra groups) keeps torch's clip_grad_norm_ + optimizer.step()."""
    if type(optimizer) is not torch.optim.AdamW or len(optimizer.param_groups) != 1:
        return False
    group = optimizer.param_groups[0]
    return not (group.get("amsgrad") or group.get("maximize"))


def flat_adam_state(ppo):
    """ppo's FlatAdamState (built once per policy and optimizer), re-armed for this learn()."""
    fa = getattr(ppo, "_flat_adam", None)
    params = list(ppo.policy.parameters())
    if fa is None or len(fa.params) != len(params) or any(a is not b for a, b in zip(fa.params, params)):
        fa = ppo._flat_adam = FlatAdamState(ppo)
    else:
        fa.prepare()
    return fa


class GraphedUpdate:
    WARMUP = 2

    def __init__(self, ppo, S, A, old_logp, adv, ret, scales=None):
        from .PPO import SurrogateLoss
        self.ppo = ppo
        self.SurrogateLoss = SurrogateLoss
        mb = ppo.mini_batch_size
        dev = S.device
        self.mb = mb
        self.cursor = torch.zeros(1, dtype=torch.int64, device=dev)
        A2 = A if A.dim() == 2 else A.view(-1, 1)
        self.sources = [S.contiguous(), A2.contiguous(), old_logp.contiguous(), adv.contiguous(),
                        ret.contiguous()]
        self.S_mb = torch.empty(mb, S.shape[1], dtype=torch.float32, device=dev)
        self.A_mb = torch.empty(mb, A2.shape[1], dtype=torch.float32, device=dev)
        self.old_mb = torch.empty(mb, dtype=torch.float32, device=dev)
        self.adv_mb = torch.empty(mb, dtype=torch.float32, device=dev)
        self.ret_mb = torch.empty(mb, dtype=torch.float32, device=dev)
        self.gather = prl_native.MinibatchGather(
            self.sources, [self.S_mb, self.A_mb, self.old_mb, self.adv_mb, self.ret_mb],
            self.cursor, mb)
        self.A_eval = self.A_mb if A.dim() == 2 else self.A_mb.view(-1)
        self.scales = scales          # device [n_steps] f32, world > 1 only
        self.params = [p for p in ppo.policy.parameters() if p.requires_grad]
        self.sizes = [p.numel() for p in self.params]
        self.flat = torch.zeros(sum(self.sizes), dtype=torch.float32, device=dev)
        self.graph_b = None
        self.loss_out = torch.zeros((), dtype=torch.float32, device=dev)
        self.graph = None
        self.replays = 0
        prl_native.reserve_workspace(mb, dev)
        # wide nets (outside the persistent engine, e.g. C5's D = 348, A = 17): the step's
        # forward + loss + backward is prl_ppo_wide_grad (two HIP launches reading the minibatch
        # in place) instead of ~60 PyTorch / hipBLASLt kernels.  Part of the native path
        # (ppo.use_fused); PRL_WIDE=0 or use_fused = False keeps the autograd step
        self.wide = None
        self.fa = None
        info = wide_info(ppo, S.shape[1])
        if info is not None:
            self.wide = info
            self.part = torch.empty(info[1], dtype=torch.float32, device=dev)
            # the eager steps' minibatch indices as one device arange: step j reads the view
            # [j : j + 1] (no fill kernel per step; the kernel takes the index from the device)
            nbj = -(-S.shape[0] // mb)
            self.cursor_all = torch.arange(max(nbj, 1), dtype=torch.int64, device=dev)
            self.sources[1] = self.sources[1].float().contiguous()
            # parameters / gradient / AdamW state as flat vectors: the kernel reads the
            # parameters in place and clip_grad_norm_ + AdamW are one launch (prl_flat_adamw);
            # PRL_WIDE_ADAM=0 keeps torch's clip_grad_norm_ + fused AdamW
            if os.environ.get("PRL_WIDE_ADAM", "1") != "0" and flat_adam_ok(ppo.optimizer):
                self.fa = flat_adam_state(ppo)
            else:
                self.pflat = torch.empty(info[0], dtype=torch.float32, device=dev)

    def _wide_grad(self, cursor, scales):
        """Gradient of minibatch `cursor` into the flat gradient buffer (p.grad views) or, on
        data-parallel ranks, into self.flat (the all-reduce buffer); loss into loss_out."""
        ppo = self.ppo
        grads = ppo._ensure_flat_grads()
        if self.fa is not None:
            pflat = self.fa.flat          # the parameters themselves (views of it)
        else:
            pflat = self.pflat
            torch.cat([p.detach().reshape(-1) for p in self.params], out=pflat)
        S, A2, old, adv, ret = self.sources
        prl_native.ppo_wide_grad(pflat, S.shape[1], ppo.action_dim, not ppo.is_continuous,
                                 S, A2, old, adv, ret, self.mb, cursor, scales, ppo.policy_clip,
                                 ppo.value_coef, ppo.entropy_coef,
                                 self.flat if scales is not None else grads, self.loss_out,
                                 self.part)

    def wide_step(self, j: int):
        """One eager optimizer step on minibatch j through the wide kernel (single rank: the
        ragged last minibatch of an epoch)."""
        self._wide_grad(self.cursor_all[j:j + 1], None)
        if self.fa is not None:
            self.fa.launch(self.ppo._flat_grad)
        else:
            nn.utils.clip_grad_norm_(self.params, 2.0)
            self.ppo.optimizer.step()
        return self.loss_out

    def _forward_backward(self):
        ppo = self.ppo
        if self.wide is not None:
            self._wide_grad(self.cursor, self.scales)
            return
        self.gather()
        logp, V, H = ppo.policy.get_evaluate(self.S_mb, self.A_eval)
        loss = self.SurrogateLoss.apply(logp, self.old_mb, self.adv_mb, V, self.ret_mb, H,
                                        ppo.policy_clip, ppo.value_coef, ppo.entropy_coef,
                                        ppo._ops)
        if self.scales is not None:
            (loss * self.scales.index_select(0, self.cursor).reshape(())).backward()
            torch.cat([p.grad.reshape(-1) for p in self.params], out=self.flat)
        else:
            loss.backward()
        self.loss_out.copy_(loss.detach())

    def _apply(self):
        if self.fa is not None:   # the all-reduced buffer on data-parallel ranks
            self.fa.launch(self.flat if self.scales is not None else self.ppo._flat_grad)
            self.cursor.add_(1)
            return
        if self.scales is not None:
            grads = [p.grad for p in self.params]
            torch._foreach_copy_(grads, [f.view_as(g) for f, g in
                                         zip(self.flat.split(self.sizes), grads)])
        nn.utils.clip_grad_norm_(self.params, 2.0)
        self.ppo.optimizer.step()
        self.cursor.add_(1)

    def finish(self):
        """After the learn's last step: the optimizer's state reflects the native steps."""
        if self.fa is not None:
            self.fa.sync()

    def _step_eager(self):
        if self.fa is None:
            self.ppo.optimizer.zero_grad(set_to_none=True)
        self._forward_backward()
        if self.scales is not None:
            self.ppo.all_reduce(self.flat)
        self._apply()

    def _replay(self):
        self.replays += 1
        if self.scales is None:
            self.graph.replay()
        else:  # the collective stays outside the graphs (eager RCCL between two replays)
            self.graph.replay()
            self.ppo.all_reduce(self.flat)
            self.graph_b.replay()

    def run_epoch(self, n_steps: int) -> int:
        """Run minibatches 0 .. n_steps-1 of one epoch; returns n_steps."""
        self.cursor.zero_()
        done = 0
        if self.graph is None:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(min(self.WARMUP, n_steps)):
                    self._step_eager()
                    done += 1
            torch.cuda.current_stream().wait_stream(side)
            if done == n_steps:
                return done
            if self.fa is None:
                self.ppo.optimizer.zero_grad(set_to_none=True)
            self.graph = torch.cuda.CUDAGraph()
            if self.scales is None:
                with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                    self._forward_backward()
                    self._apply()
            else:
                with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                    self._forward_backward()
                self.graph_b = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_b, pool=self.graph.pool(),
                                      capture_error_mode="thread_local"):
                    self._apply()
        for _ in range(n_steps - done):
            self._replay()
        return n_steps
