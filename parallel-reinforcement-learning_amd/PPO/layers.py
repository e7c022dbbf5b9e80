"""Hidden-block layer shared by ActorCritic and RND: GroupNorm(8, 64) fused with the SiLU that
follows it in every block of the reference (PPO/ActorCritic.py:19-60, PPO/RND.py:25-30).

Device tensors run one HIP kernel each way (prl_gn_silu_fwd / prl_gn_silu_bwd).  This is not only
fewer launches: PyTorch-ROCm's nn.GroupNorm backward in this image returns wrong weight/bias
gradients once a batch has >= 512 rows (tools/diag_groupnorm.py), which would silently corrupt
every PPO update.  The module subclasses nn.GroupNorm, so its parameters and state_dict keys
(`<block>.1.weight`, `<block>.1.bias`) are the reference's; the SiLU slot becomes nn.Identity.
CPU-resident modules (no GPU present) and non-float32 tensors evaluate nn.functional.group_norm +
silu, as the reference does on the CPU.
"""
import torch
import torch.nn.functional as F
from torch import nn

import prl_native


class _GroupNormSiLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x = x.contiguous()
        w = weight.detach().contiguous()
        b = bias.detach().contiguous()
        out = torch.empty_like(x)
        prl_native.gn_silu_fwd(x, w, b, eps, True, out)
        ctx.save_for_backward(x, w, b)
        ctx.eps = eps
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, b = ctx.saved_tensors
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        db = torch.empty_like(b)
        prl_native.gn_silu_bwd(x, dout.contiguous(), w, b, ctx.eps, True, dx, dw, db)
        return dx, dw, db, None


class GroupNormSiLU(nn.GroupNorm):
    def __init__(self, num_groups: int = 8, num_channels: int = 64, eps: float = 1e-5):
        super().__init__(num_groups, num_channels, eps)
        if (num_groups, num_channels) != (8, 64):
            raise ValueError("only GroupNorm(8, 64) has a HIP kernel")

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.float32 and self.weight.dtype == torch.float32:
            return _GroupNormSiLU.apply(x, self.weight, self.bias, self.eps)
        # CPU, or another dtype (tests' float64 copies of a device policy): torch's own ops
        return F.silu(F.group_norm(x, self.num_groups, self.weight, self.bias, self.eps))


SPLIT_ROWS = 4096        # rows per split-K chunk of a weight gradient
SPLIT_MIN_ROWS = 16384   # below this the plain GEMM already fills the chip


class _SplitKLinear(torch.autograd.Function):
    """y = x W^T + b whose backward forms dW = dy^T x (and db = 1^T dy) split over row chunks:
    one batched GEMM [k, out, 4096] x [k, 4096, in] + a sum over k.  At the per-step update's
    65,536-row minibatches the library GEMM for dW (output 64 x 348, K = 65,536) runs on 12
    workgroups of 256 CUs (~210 us); the batched form gives it k x the tiles.  db on the device
    by prl_colsum_f32 (PyTorch's dim-0 column sum of a [65,536, 348] gradient took ~170 us, a
    batched GEMM with a ones column ~36 us); elsewhere through that batched GEMM.  Float32
    throughout; only the summation order differs from the plain GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy @ weight if ctx.needs_input_grad[0] else None
        dw = db = None
        n = x.shape[0]
        k = n // SPLIT_ROWS
        main = k * SPLIT_ROWS
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dyT = dy[:main].view(k, SPLIT_ROWS, -1).transpose(1, 2)          # [k, out, rows]
        if ctx.needs_input_grad[1]:
            dw = torch.bmm(dyT, x[:main].view(k, SPLIT_ROWS, -1)).sum(0)
            if main < n:
                dw = dw + dy[main:].t() @ x[main:]
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if dy.is_cuda and dy.dtype == torch.float32:
                db = prl_native.colsum(dy)       # deterministic two-pass HIP column sum
            else:
                ones = torch.ones(k, SPLIT_ROWS, 1, dtype=dy.dtype, device=dy.device)
                db = torch.bmm(dyT, ones).sum(0).reshape(-1)
                if main < n:
                    db = db + dy[main:].sum(0)
        return dx, dw, db


class Linear(nn.Linear):
    """nn.Linear (same parameters and state_dict keys) whose weight / bias gradients are formed
    split-K on large device batches (_SplitKLinear); otherwise exactly F.linear."""

    def forward(self, x):
        if (x.is_cuda and x.dim() == 2 and x.shape[0] >= SPLIT_MIN_ROWS and torch.is_grad_enabled()
                and (self.weight.requires_grad or x.requires_grad)):
            return _SplitKLinear.apply(x.contiguous(), self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)


def hidden_block(in_features: int, out_features: int = 64, bias: bool = False):
    """[Linear, GroupNorm(8,64)+SiLU, Identity] — the reference's [Linear, GroupNorm, SiLU]."""
    return [Linear(in_features, out_features, bias=bias), GroupNormSiLU(8, 64), nn.Identity()]
