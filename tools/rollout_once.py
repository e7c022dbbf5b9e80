"""One CartPole device rollout through AsyncPPO.worker() (the one-launch prl_cartpole_rollout) on a
fresh policy, for counter passes: prints the transitions it collected, so a per-dispatch counter
mean (one cp_rollout_kernel dispatch) divides into bytes per env-step.
Usage: rollout_once.py [num_envs]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd")]
from AsyncTools.AsyncPPO import AsyncPPO  # noqa: E402
from PPO import PPO  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
torch.manual_seed(0)
p = PPO(False, 4, 2)
p.show_progress = False
a = AsyncPPO("CartPole-v1", p, num_envs=E, seed=1)
n = a.worker()
torch.cuda.synchronize()
print(json.dumps({"num_envs": E, "env_steps": int(n), "vector_steps": int(a.last_vector_steps)}), flush=True)
