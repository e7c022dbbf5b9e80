"""Time prl_ppo_wide_grad (the wide-net optimizer step's gradient, csrc/prl_ppo_wide.hip) on a
C5-shaped minibatch (D = 348, A = 17 continuous, mb = 65,536) with HIP events, and print workgroup
0's per-stage split (s_memrealtime, us per step).  python tools/wide_bench.py [--mb N] [--reps R]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "parallel-reinforcement-learning_amd"))
import prl_native  # noqa: E402
from PPO.ActorCritic import ActorCritic  # noqa: E402

STAGES = ("stage X", "trunk", "heads fwd", "outputs", "loss", "heads bwd", "dW1+dF+GN0", "dW0")

ap = argparse.ArgumentParser()
ap.add_argument("--D", type=int, default=348)
ap.add_argument("--A", type=int, default=17)
ap.add_argument("--mb", type=int, default=65536)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(0)
pol = ActorCritic(True, a.D, a.A, device=dev)
N = a.mb
S = torch.randn(N, a.D, device=dev) * 0.5
with torch.no_grad():
    act = pol.get_dist(S).sample().contiguous()
    old, _, _ = pol.get_evaluate(S, act)
adv, ret = torch.randn(N, device=dev), torch.randn(N, device=dev)
n_params, part_floats, grid = prl_native.ppo_wide_info(a.D, a.A, False, a.mb)
flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
grad = torch.empty(n_params, device=dev)
loss = torch.zeros(1, device=dev)
part = torch.empty(part_floats, device=dev)
cur = torch.zeros(1, dtype=torch.int64, device=dev)
args = (flat, a.D, a.A, False, S, act, old.contiguous(), adv, ret, a.mb, cur, None, 0.2, 0.5, 0.01,
        grad, loss, part)
for _ in range(3):
    prl_native.ppo_wide_grad(*args)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.reps):
    prl_native.ppo_wide_grad(*args)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / a.reps
prof = torch.zeros(8, dtype=torch.int64, device=dev)
for _ in range(a.reps):
    prl_native.ppo_wide_grad(*args, prof=prof)
torch.cuda.synchronize()
stages = {n: round(float(v) * 0.01 / a.reps, 1) for n, v in zip(STAGES, prof.tolist())}
flop_row = 2 * (a.D * 64 + 3 * 64 * 64 + (2 * a.A + 1) * 64) * 2 + 2 * (3 * 64 * 64 + (2 * a.A + 1) * 64)
tf = flop_row * a.mb / (us * 1e-6) / 1e12
print(json.dumps({"D": a.D, "A": a.A, "mb": a.mb, "grid": grid, "us_per_step": round(us, 1),
                  "linear_tflops": round(tf, 2), "frac_f32_mfma_peak": round(tf / 157.3, 4),
                  "wg0_stage_us": stages}))
