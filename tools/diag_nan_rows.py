"""Replay the saved C5 NaN case (tools/exp/nan_case.pt): does a non-finite observation row leak
into another row's prl_ppo_wide_dist output?"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))
import prl_native  # noqa: E402

d = torch.load(os.path.join(ROOT, "tools", "exp", "nan_case.pt"), weights_only=True)
obs0, flat = d["obs"].cuda(), d["flat"].cuda()


def run(obs):
    out = torch.empty(obs.shape[0], 34, device="cuda")
    prl_native.ppo_wide_dist(flat, 348, 17, False, obs.contiguous(), out)
    torch.cuda.synchronize()
    return torch.nonzero(~torch.isfinite(out).all(-1)).flatten().tolist()


print("as saved:", run(obs0))
z = obs0.clone(); z[18] = 0; z[102] = 0
print("rows 18/102 zeroed:", run(z))
for val in (float("nan"), float("inf"), 3e38, 1e30):
    y = z.clone(); y[102, 5] = val
    print(f"row 102 col 5 = {val}:", run(y))
for col in (0, 100, 347):
    y = z.clone(); y[102, col] = float("nan")
    print(f"row 102 col {col} = nan:", run(y))
for row in (96, 97, 100, 103, 111):
    y = z.clone(); y[row, 7] = float("nan")
    print(f"row {row} col 7 = nan:", run(y))
