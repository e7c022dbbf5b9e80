"""TEST-ONLY stand-in for prl_native's learn() entry points, backed by the CPU oracle.

PPO.learn() calls its HIP ops through `ppo._ops` (prl_native in the product).  CPU tests swap
in this object to exercise learn()'s orchestration — chunked evaluation, GAE wiring, global
advantage statistics, minibatch order, gradient all-reduce weighting under gloo — on machines
without a GPU.  It is never reachable from the product path.
"""
import numpy as np
import torch

import oracle as O


class FakeOps:
    calls = None

    def __init__(self):
        self.calls = {"gae": 0, "adv_normalize": 0, "surrogate_fwd": 0, "surrogate_bwd": 0}

    def gae(self, r, d, V, next_value, gamma, lam, ret, adv=None, sums=None):
        self.calls["gae"] += 1
        Vn = V.detach().cpu().numpy()
        nv = float(next_value.reshape(-1)[0]) if next_value is not None else float(Vn[-1])
        rr = O.gae(r.cpu().numpy(), d.cpu().numpy(), Vn, nv, gamma, lam)
        ret.copy_(torch.from_numpy(rr))
        if adv is not None:
            a = (rr - Vn).astype(np.float32)
            adv.copy_(torch.from_numpy(a))
            a64 = a.astype(np.float64)
            sums.copy_(torch.tensor([a64.sum(), (a64 * a64).sum()], dtype=torch.float64))

    def adv_normalize(self, x, sums, count, eps, out):
        self.calls["adv_normalize"] += 1
        s = sums.cpu().numpy()
        mean = s[0] / count
        var = (s[1] - s[0] * mean) / (count - 1)
        xn = x.cpu().numpy()
        y = (xn - np.float32(mean)) / (np.float32(np.sqrt(max(var, 0.0))) + np.float32(eps))
        out.copy_(torch.from_numpy(y.astype(np.float32)))

    def surrogate_fwd(self, logp, old_logp, adv, V, ret, entropy, clip, vf_coef, ent_coef, loss,
                      dlogp=None, dV=None):
        self.calls["surrogate_fwd"] += 1
        lo, dl, dv = O.surrogate(logp.detach().cpu().numpy(), old_logp.cpu().numpy(),
                                 adv.cpu().numpy(), V.detach().cpu().numpy(), ret.cpu().numpy(),
                                 float(entropy), clip, vf_coef, ent_coef)
        loss.fill_(float(lo))
        if dlogp is not None:
            dlogp.copy_(torch.from_numpy(dl.astype(np.float32)))
        if dV is not None:
            dV.copy_(torch.from_numpy(dv.astype(np.float32)))

    def surrogate_bwd(self, grad_out, dlogp_unit, dV_unit, dlogp, dV):
        self.calls["surrogate_bwd"] += 1
        g = float(grad_out)
        dlogp.copy_(dlogp_unit * g)
        dV.copy_(dV_unit * g)
