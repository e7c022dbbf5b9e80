"""Continuous learn(): fused vs per-step after n optimizer steps (k = 1, N = 512 n): function-space
distance and the largest relative difference of AdamW's moments per tensor."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tests")]
from test_engine_gpu import _data, _outputs, _run  # noqa: E402

cont = True
data = _data(512 * 8, 3, cont)
for n in (1, 2, 3, 4, 6, 8):
    d = tuple(x[:512 * n] for x in data)
    f = _run(True, cont, d, 512, 1, lr=3e-4, clip=1e3)
    g = _run(False, cont, d, 512, 1, lr=3e-4, clip=1e3)
    (lf, vf), (lg, vg) = _outputs(f, d[0][:1024], d[1][:1024]), _outputs(g, d[0][:1024], d[1][:1024])
    worst_m, worst_v = {}, {}
    for (name, pf), pg in zip(f.policy.named_parameters(), g.policy.parameters()):
        sf, sg = f.optimizer.state[pf], g.optimizer.state[pg]
        for key, dst in (("exp_avg", worst_m), ("exp_avg_sq", worst_v)):
            a, b = sf[key].double(), sg[key].double()
            dst[name] = float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)
    wm = max(worst_m, key=worst_m.get)
    wv = max(worst_v, key=worst_v.get)
    print(n, "steps: logp", float((lf - lg).abs().max()), "V", float((vf - vg).abs().max()),
          "| m", wm, f"{worst_m[wm]:.1e}", "| v", wv, f"{worst_v[wv]:.1e}",
          "| step", float(f.optimizer.state[next(f.policy.parameters())]["step"]),
          float(g.optimizer.state[next(g.policy.parameters())]["step"]), flush=True)
