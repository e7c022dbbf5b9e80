"""Diagnostic: the C5 per-step eager rollout (PRL_WIDE_ROLLOUT=0, PRL_ROLLOUT_GRAPH=0) at E=300,
before and after a persistent wide rollout (prl_wide_rollout) in the same process: where do
non-finite actions / rewards / observations appear.  Usage: diag_wide_rollout.py [E]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))
from AsyncTools.AsyncPPO import AsyncPPO  # noqa: E402
from PPO import PPO  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 300


def run(tag, fused):
    os.environ["PRL_WIDE_ROLLOUT"] = fused
    os.environ["PRL_ROLLOUT_GRAPH"] = "0"
    torch.manual_seed(0)
    p = PPO(True, 348, 17, action_scaling=1.0, batch_size=10**9, mini_batch_size=512)
    a = AsyncPPO("SyntheticHumanoid-v0", p, num_envs=E, seed=5)
    for it in range(3):
        a.reward_score = 0.0
        n = a.worker()
        tr = a._traj
        T = int(tr.ep_len.max())
        live = torch.arange(T, device="cuda")[:, None] < tr.ep_len[None, :]
        act = tr.act[:T]
        bad_a = (~torch.isfinite(act).all(-1)) & live
        bad_r = (~torch.isfinite(tr.rew[:T])) & live
        obs = tr.obs[:T]
        bad_o = (~torch.isfinite(obs).all(-1)) & live
        msg = (f"{tag} it{it}: N={n} reward={float(a.reward_score):.3f} T={T} "
               f"bad actions {int(bad_a.sum())} bad rewards {int(bad_r.sum())} bad obs {int(bad_o.sum())}")
        if bad_a.any():
            t, e = [int(x) for x in torch.nonzero(bad_a)[0]]
            d = p.dist_params(tr.obs[t].contiguous())
            msg += (f" | first bad (t={t}, e={e}): obs finite {bool(torch.isfinite(tr.obs[t, e]).all())}"
                    f" dist finite rows {int(torch.isfinite(d).all(-1).sum())}/{E},"
                    f" row e finite {bool(torch.isfinite(d[e]).all())}")
            with torch.no_grad():
                ref = p.policy_old.dist_params(tr.obs[t].contiguous())
            msg += f" torch dist row e finite {bool(torch.isfinite(ref[e]).all())}"
        print(msg, flush=True)
        p.memory.clear()


run("eager", "0")
run("fused", "1")
run("eager-after", "0")
