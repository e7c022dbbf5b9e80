"""Diagnostic: nn.GroupNorm(8, 64) forward/backward on [N, 64] inputs, PyTorch GPU vs CPU vs a
float64 restatement (what the actor-critic's trunk/heads compute, ActorCritic.py:19-60)."""
import torch
import torch.nn.functional as F


def manual(x, w, b, G=8, eps=1e-5):
    N, C = x.shape
    g = x.view(N, G, C // G)
    mu = g.mean(-1, keepdim=True)
    var = g.var(-1, unbiased=False, keepdim=True)
    y = ((g - mu) / torch.sqrt(var + eps)).view(N, C)
    return y * w + b


def grads(fn, x, w, b, dy):
    x = x.clone().requires_grad_(True)
    w = w.clone().requires_grad_(True)
    b = b.clone().requires_grad_(True)
    y = fn(x, w, b)
    y.backward(dy)
    return y.detach(), x.grad, w.grad, b.grad


torch.manual_seed(0)
for N in (1, 7, 512, 65536):
    x = torch.randn(N, 64) * 3 + 1
    w = torch.randn(64) * 0.5 + 1
    b = torch.randn(64) * 0.1
    dy = torch.randn(N, 64)
    ref = grads(manual, x.double(), w.double(), b.double(), dy.double())
    cpu = grads(lambda x, w, b: F.group_norm(x, 8, w, b, 1e-5), x, w, b, dy)
    gpu = grads(lambda x, w, b: F.group_norm(x, 8, w, b, 1e-5), x.cuda(), w.cuda(), b.cuda(),
                dy.cuda())
    gpu3 = grads(lambda x, w, b: F.group_norm(x.unsqueeze(-1), 8, w, b, 1e-5).squeeze(-1),
                 x.cuda(), w.cuda(), b.cuda(), dy.cuda())
    man_gpu = grads(manual, x.cuda(), w.cuda(), b.cuda(), dy.cuda())
    for name, res in (("cpu", cpu), ("gpu", gpu), ("gpu[N,C,1]", gpu3), ("gpu-manual", man_gpu)):
        errs = [float((a.double().cpu() - r).abs().max() / (r.abs().max() + 1e-30))
                for a, r in zip(res, ref)]
        print(f"N={N:6d} {name:11s} rel err  y {errs[0]:.2e}  dx {errs[1]:.2e}  "
              f"dw {errs[2]:.2e}  db {errs[3]:.2e}")
