"""Host-side time of one C5 learn() (GPU box): where the Python side of learn() spends its time
before the GPU work it enqueues hides it.  Runs two untimed AsyncPPO iterations of bench.py's c5
configuration, then a third whose learn() is under cProfile (no extra synchronisation inside it),
and prints the wall time until learn() returns, the time until the GPU is done, and the top
functions by cumulative host time.

    python tools/learn_host_profile.py [--config c5] [--top 30]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5", choices=sorted(bench.CONFIGS))
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    from AsyncTools.AsyncPPO import AsyncPPO
    from AsyncTools.envs import make
    from PPO import PPO
    spec = make(cfg["env"])
    torch.manual_seed(1234)
    ppo = PPO(is_continuous=cfg["cont"], observ_dim=spec.obs_dim, action_dim=spec.act_dim,
              action_scaling=cfg["scaling"], lr=1e-3, k_epochs=cfg["k_epochs"], policy_clip=0.2,
              GAE_lambda=0.95, gamma=0.995, batch_size=cfg["batch_size"],
              mini_batch_size=cfg["mb"], use_RND=cfg["rnd"], beta=1e-3)
    ppo.show_progress = False
    runner = AsyncPPO(spec, ppo, num_envs=cfg["num_envs"], seed=1000)
    for it in range(4):
        runner.step_score, runner.reward_score = 0, 0
        n = runner.worker()
        torch.cuda.synchronize()
        prof = cProfile.Profile() if it == 3 else None
        t0 = time.perf_counter()
        if prof is not None:
            prof.enable()
        ppo.learn()
        if prof is not None:
            prof.disable()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"iteration {it}: {n} transitions, learn() returned after {1e3 * (t1 - t0):.2f} ms, "
              f"GPU done after {1e3 * (t2 - t0):.2f} ms", flush=True)
    pstats.Stats(prof).sort_stats("cumulative").print_stats(args.top)


if __name__ == "__main__":
    main()
