"""Diagnostic: the runtime-layout engine on a non-specialised shape vs float64 autograd, per
tensor (one step at lr = 0, exp_avg = 0.1 * clipped gradient)."""
import copy
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tests")]
import test_engine_gpu as T  # noqa: E402

for cont, D, A in ((False, 6, 3), (False, 4, 3), (False, 6, 2), (True, 5, 2), (True, 3, 2)):
    rng = np.random.default_rng(41)
    N = 512
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    Aa = (torch.from_numpy((np.tanh(rng.normal(size=(N, A))) * 2).astype(np.float32)).cuda() if cont
          else torch.from_numpy(rng.integers(0, A, N).astype(np.float32)).cuda())
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.05).astype(np.float32)).cuda()
    Dn[-1] = 1
    p = T._run(True, cont, (S, Aa, R, Dn), 512, 1, D=D, A=A, lr=0.0)
    S_, A_, old, adv, ret = p._last_update_inputs
    lv, _ = p._engine.evaluate(p.policy, S_, A_)
    g64 = T._grad_f64(p, (S_, A_, old, adv, ret), logp_val=lv)
    print(f"cont={cont} D={D} A={A}")
    for (name, prm), gr in zip(p.policy.named_parameters(), g64):
        m = p.optimizer.state[prm]["exp_avg"].double().cpu() / 0.1
        err = float((m - gr).abs().max()) / (float(gr.abs().max()) + 1e-30)
        extra = ""
        if err > 1e-3 and m.numel() <= 8:
            extra = f" engine {m.flatten().tolist()} ref {gr.flatten().tolist()}"
        print(f"   {name:24s} {err:.2e}{extra}")
