"""Diagnostic: the C5 per-step eager rollout (PRL_WIDE_ROLLOUT=0, PRL_ROLLOUT_GRAPH=0) at E envs,
before and after a persistent wide rollout (prl_wide_rollout) in the same process: where do
non-finite actions / rewards / observations / reward sums appear.  Usage: diag_wide_rollout.py [E]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))
from AsyncTools.AsyncPPO import AsyncPPO  # noqa: E402
from PPO import PPO  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 300


def run(tag, fused, reset_score=True):
    os.environ["PRL_WIDE_ROLLOUT"] = fused
    os.environ["PRL_ROLLOUT_GRAPH"] = "0"
    torch.manual_seed(0)
    p = PPO(True, 348, 17, action_scaling=1.0, batch_size=10**9, mini_batch_size=512)
    a = AsyncPPO("SyntheticHumanoid-v0", p, num_envs=E, seed=5)
    first_bad = []
    orig = a._step_kernel

    def checked(k, dist, seed, scaling, active_after):
        orig(k, dist, seed, scaling, active_after)
        if not first_bad:
            torch.cuda.synchronize()
            rs = float(a._traj.reward_sum.item())
            if rs != rs:
                tr = a._traj
                live = (tr.ep_len >= k + 1)
                first_bad.append(k)
                print(f"  {tag}: reward_sum NaN after vector step {k}; dist finite rows "
                      f"{int(torch.isfinite(dist).all(-1).sum())}/{dist.shape[0]}, live rows with a "
                      f"non-finite dist {int((~torch.isfinite(dist).all(-1) & live).sum())}, "
                      f"non-finite rewards at k among live {int((~torch.isfinite(tr.rew[k]) & live).sum())}",
                      flush=True)
    a._step_kernel = checked
    for it in range(3):
        if reset_score:
            a.reward_score = 0.0
        n = a.worker()
        tr = a._traj
        T = int(tr.ep_len.max())
        live = torch.arange(T, device="cuda")[:, None] < tr.ep_len[None, :]
        bad_a = (~torch.isfinite(tr.act[:T]).all(-1)) & live
        bad_r = (~torch.isfinite(tr.rew[:T])) & live
        bad_o = (~torch.isfinite(tr.obs[:T]).all(-1)) & live
        print(f"{tag} it{it}: N={n} reward_score={float(a.reward_score):.3f} "
              f"reward_sum={float(tr.reward_sum.item()):.3f} T={T} bad actions {int(bad_a.sum())} "
              f"bad rewards {int(bad_r.sum())} bad obs {int(bad_o.sum())}", flush=True)
        p.memory.clear()


run("eager", "0")
run("eager-noreset", "0", reset_score=False)
run("fused", "1")
run("eager-after", "0")
