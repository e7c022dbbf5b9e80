"""RND intrinsic-reward forward (prl_rnd_forward): the persistent fast kernel vs the round-1
kernel (PRL_RND_GENERIC=1) at C5's shape (D = 348), HIP-event timed, checked against a float64
torch restatement of RND.py:71-94 on a row subset.  Prints one JSON line per (kernel, N)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))
import prl_native  # noqa: E402

D = int(os.environ.get("RND_D", 348))
rng = np.random.default_rng(0)


def net():
    p = dict(w1=rng.normal(0, (2 / (D + 64)) ** .5, (64, D)), b1=rng.normal(0, .01, 64),
             gw=np.ones(64), gb=np.zeros(64), w2=rng.normal(0, (2 / (D + 64)) ** .5, (D, 64)),
             b2=rng.normal(0, .01, D))
    return [torch.from_numpy(p[k].astype(np.float32)).cuda() for k in ("w1", "b1", "gw", "gb", "w2", "b2")]


def ref64(x, t, p, beta):
    def f(n):
        w1, b1, gw, gb, w2, b2 = [a.double() for a in n]
        h = x.double() @ w1.T + b1
        h = torch.nn.functional.group_norm(h, 8, gw, gb, 1e-5)
        h = h * torch.sigmoid(h)
        return h @ w2.T + b2
    return beta * torch.linalg.norm(f(p) - f(t), dim=-1)


tn, pn = net(), net()
for N in [int(a) for a in (sys.argv[1:] or ["323584", "1048576"])]:
    x = torch.randn(N, D, device="cuda")
    out = torch.empty(N, device="cuda")
    for kern in ("fast", "generic"):
        if kern == "generic":
            os.environ["PRL_RND_GENERIC"] = "1"
        else:
            os.environ.pop("PRL_RND_GENERIC", None)
        prl_native.rnd_forward(x, tn, pn, 1e-3, out)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 10
        ev[0].record()
        for _ in range(reps):
            prl_native.rnd_forward(x, tn, pn, 1e-3, out)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        sub = torch.arange(0, N, max(1, N // 4096), device="cuda")
        r = ref64(x[sub], tn, pn, 1e-3)
        err = float(((out[sub].double() - r).abs() / r.abs().clamp_min(1e-30)).max())
        flops = 512.0 * D * N
        print(json.dumps({"kernel": kern, "D": D, "N": N, "ms": round(ms, 4),
                          "tflops": round(flops / ms / 1e9, 2), "frac_f32_mfma": round(flops / ms / 1e9 / 157.3, 4),
                          "max_rel_err_vs_f64": err}), flush=True)
