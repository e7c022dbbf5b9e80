"""Rollout (AsyncPPO device worker) time per iteration, eager launches vs the captured vector-step
graph, and the cost of one capture, for a config of bench.py (default c2)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parallel-reinforcement-learning_amd")]
from bench import CONFIGS  # noqa: E402
from AsyncTools.AsyncPPO import AsyncPPO  # noqa: E402
from AsyncTools.envs import make  # noqa: E402
from PPO import PPO  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
spec = make(cfg["env"])
for mode in ("0", "1"):
    os.environ["PRL_ROLLOUT_GRAPH"] = mode
    torch.manual_seed(0)
    p = PPO(cfg["cont"], spec.obs_dim, spec.act_dim, action_scaling=cfg["scaling"],
            batch_size=10**12, use_RND=False)
    a = AsyncPPO(spec, p, num_envs=cfg["num_envs"], seed=3)
    a.worker()
    torch.cuda.synchronize()
    times, n = [], 0
    for _ in range(3):
        p.memory.clear()
        t0 = time.perf_counter()
        n = a.worker()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    rec = {"graph": mode, "rollout_ms": [round(t * 1e3, 2) for t in times], "transitions": n,
           "vector_steps": a.last_vector_steps}
    if mode == "1":
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a._capture_step(123, 1.0)
        torch.cuda.synchronize()
        rec["capture_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    print(json.dumps(rec), flush=True)
