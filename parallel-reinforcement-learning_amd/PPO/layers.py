"""Hidden-block layer shared by ActorCritic and RND: GroupNorm(8, 64) fused with the SiLU that
follows it in every block of the reference (PPO/ActorCritic.py:19-60, PPO/RND.py:25-30).

Device tensors run one HIP kernel each way (prl_gn_silu_fwd / prl_gn_silu_bwd).  This is not only
fewer launches: PyTorch-ROCm's nn.GroupNorm backward in this image returns wrong weight/bias
gradients once a batch has >= 512 rows (tools/diag_groupnorm.py), which would silently corrupt
every PPO update.  The module subclasses nn.GroupNorm, so its parameters and state_dict keys
(`<block>.1.weight`, `<block>.1.bias`) are the reference's; the SiLU slot becomes nn.Identity.
CPU-resident modules (no GPU present) evaluate nn.functional.group_norm + silu, as the
reference does on the CPU.
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
        if x.is_cuda:
            return _GroupNormSiLU.apply(x, self.weight, self.bias, self.eps)
        return F.silu(F.group_norm(x, self.num_groups, self.weight, self.bias, self.eps))


def hidden_block(in_features: int, out_features: int = 64, bias: bool = False):
    """[Linear, GroupNorm(8,64)+SiLU, Identity] — the reference's [Linear, GroupNorm, SiLU]."""
    return [nn.Linear(in_features, out_features, bias=bias), GroupNormSiLU(8, 64), nn.Identity()]
