"""Diagnostic: the C5 graphed rollout with the caching allocator poisoned by NaN-filled freed
blocks (as earlier GPU tests leave it): does the warm-up capture + replay at the end of the
first rollout read memory nobody wrote?  Prints the reward sum around the capture and replay."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))
from AsyncTools.AsyncPPO import AsyncPPO  # noqa: E402
from PPO import PPO  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 200
poison = [torch.full((n,), float("nan"), device="cuda") for n in
          [256, 1024, 4096, 16384, 65536, 262144] * 8 + [1 << 22, 1 << 24, 1 << 26]]
del poison
os.environ["PRL_WIDE_ROLLOUT"] = "0"
os.environ["PRL_ROLLOUT_GRAPH"] = "1"
torch.manual_seed(0)
p = PPO(True, 348, 17, action_scaling=1.0, batch_size=10**9, mini_batch_size=512)
a = AsyncPPO("SyntheticHumanoid-v0", p, num_envs=E, seed=5)
orig_cap = a._capture_step


def cap(seed, scaling):
    tr = a._traj
    torch.cuda.synchronize()
    print(f"  before capture: reward_sum {float(tr.reward_sum.item()):.4f}", flush=True)
    g = orig_cap(seed, scaling)
    torch.cuda.synchronize()
    print(f"  after capture: reward_sum {float(tr.reward_sum.item()):.4f} k_dev {a._k_dev.tolist()}",
          flush=True)
    if g is not None:
        orig_replay = g.replay

        def replay():
            orig_replay()
            torch.cuda.synchronize()
            print(f"  after a replay: reward_sum {float(tr.reward_sum.item()):.4f} "
                  f"k_dev {a._k_dev.tolist()} terminal {int(a.env.terminal.sum())}/{E}", flush=True)
        g.replay = replay
    return g


a._capture_step = cap
for it in range(2):
    a.reward_score = 0.0
    n = a.worker()
    print(f"it{it}: N={n} reward_score={float(a.reward_score):.4f}", flush=True)
    p.memory.clear()
