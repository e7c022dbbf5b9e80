"""Fused update engine: learn() time and workgroup 0's per-phase breakdown (us per step) on the
survey's C2 learn workload (2^20 synthetic CartPole transitions), at several mini_batch sizes.
Usage: engine_profile.py [N] [mb,mb,...] [cartpole|pendulum]  (pendulum: C3's net, D 3 / A 1
continuous, actions ~ 2 tanh(N(0,1)), rewards ~ -|N(5,3)|, 200-step episodes)."""
import json
import os
import sys
import time

import torch

os.environ.setdefault("PRL_UPD_PROFILE", "1")   # the engine's phase marks (off by default)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from learn_bench import synthetic_batch  # noqa: E402
from PPO import PPO  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
MBS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else (512, 2048, 65536)
NET = sys.argv[3] if len(sys.argv) > 3 else "cartpole"
if NET == "pendulum":
    import numpy as np
    rng = np.random.default_rng(0)
    S = rng.normal(size=(N, 3)).astype(np.float32)
    A = (2.0 * np.tanh(rng.normal(size=(N, 1)))).astype(np.float32)
    R = (-np.abs(rng.normal(5, 3, N))).astype(np.float32)
    D = np.zeros(N, np.float32)
    D[199::200] = 1
    D[-1] = 1
    batch = [torch.from_numpy(x).cuda() for x in (S, A, R, D)]
    cont, dims = True, (3, 1)
else:
    batch = synthetic_batch(N)
    cont, dims = False, (4, 2)
for mb in MBS:
    for k in (11,):
        torch.manual_seed(0)
        p = PPO(cont, *dims, action_scaling=2.0 if cont else None, lr=1e-3, k_epochs=k,
                batch_size=1, mini_batch_size=mb)
        p.show_progress = False
        p.memory.push_device(*batch)
        p.learn()                                   # warm-up (engine creation, workspaces)
        p.memory.push_device(*batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.learn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = k * -(-N // mb)
        print(json.dumps({"net": NET, "mb": mb, "grid": p._engine.grid, "learn_ms": round(dt * 1e3, 1),
                          "us_per_step": round(dt / steps * 1e6, 2),
                          "phases_us": p._engine.profile()}), flush=True)
