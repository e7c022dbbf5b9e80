"""Diagnostic: the wide step (prl_ppo_wide_grad) on the reference's learn_rnd_c5 fixture.

Per parameter tensor: the wide kernel's minibatch-0 gradient vs float64 autograd of the reference
loss (tests/test_wide_gpu._grad64) elementwise — the worst error relative to each ELEMENT (AdamW's
first step moves every element by lr * sign(g), so an element's sign matters, not only the
tensor's largest entry) — and the post-learn() weights of the wide path vs the reference."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tests", "golden")]
from test_rnd_learn_gpu import _inputs, _ppo_from_fixture, _sub  # noqa: E402
from test_wide_gpu import _grad64, _wide  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "learn_rnd_c5"
g = np.load(os.path.join(ROOT, "tests", "golden", f"{tag}.npz"))
D, A, mb = int(g["D"]), int(g["A_dim"]), int(g["mb"])
S, Aa = _inputs(g)
S = torch.from_numpy(np.ascontiguousarray(S)).cuda()
Aa = torch.from_numpy(np.ascontiguousarray(Aa)).cuda()
old = torch.from_numpy(g["old_logp"]).cuda()
adv = torch.from_numpy(g["adv"]).cuda()
ret = torch.from_numpy(g["returns"]).cuda()
from PPO.ActorCritic import ActorCritic  # noqa: E402
pol = ActorCritic(True, D, A, device=torch.device("cuda"))
pol.load_state_dict(_sub(g, "init/"))
hi = min(mb, S.shape[0])
g64, l64 = _grad64(pol, True, S[:hi], Aa[:hi], old[:hi], adv[:hi], ret[:hi])
gw, lw = _wide(pol, True, D, A, S, Aa, old, adv, ret, mb, 0)
rows = {}
for (name, _), a, b in zip(pol.named_parameters(), gw, g64):
    a, b = a.double().flatten(), b.double().flatten()
    big = b.abs() > 1e-8
    rel = ((a - b).abs() / b.abs().clamp_min(1e-30))[big]
    sign = ((a * b) < 0) & big
    idx = int(((a - b).abs() / b.abs().clamp_min(1e-12)).argmax())
    rows[name] = dict(tensor_rel=float((a - b).abs().max() / (b.abs().max() + 1e-30)),
                      elem_rel_max=float(rel.max()) if big.any() else 0.0,
                      sign_flips=int(sign.sum()), n=int(b.numel()),
                      worst=dict(i=idx, wide=float(a[idx]), f64=float(b[idx])))
print(json.dumps({"loss": [lw, l64], "grad": rows}, indent=1), flush=True)

p = _ppo_from_fixture(g, "wide")
p.learn()
torch.cuda.synchronize()
ref = _sub(g, "final/")
init = _sub(g, "init/")
sd = p.policy.state_dict()
out = {}
for k in ref:
    d = (sd[k].cpu().double() - ref[k].double()).abs().flatten()
    i = int(d.argmax())
    out[k] = dict(max=float(d.max()), n_over_1e5=int((d > 1e-5).sum()), i=i,
                  ours=float(sd[k].cpu().flatten()[i]), ref=float(ref[k].flatten()[i]),
                  init=float(init[k].flatten()[i]))
print(json.dumps({"weights_vs_reference": out}, indent=1), flush=True)
