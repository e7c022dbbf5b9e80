"""C2's rollout at full occupancy: 65,536 CartPole envs for ~500 vector steps, without training.

The policy's real MLP forward runs every vector step (so the timing is the trained C2 rollout's),
but its probabilities are then overwritten by a balancing controller (push toward the pole's
lean, p(right) = sigmoid(40 (theta + 0.5 theta_dot + 0.02 x_dot))), so every env stays up for
most of the TimeLimit's 500 steps, as the bench's trained policy does by iteration ~20.

Prints one JSON line: rollout wall time, vector steps, env-steps/s, GPU time per vector step
(HIP events between consecutive steps), and the isolated costs of the policy forward and the
step kernel.  Usage: python tools/c2_rollout_breakdown.py [E]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd")]
from AsyncTools.AsyncPPO import AsyncPPO  # noqa: E402
from PPO import PPO  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
torch.manual_seed(0)
ppo = PPO(False, 4, 2, lr=1e-3, k_epochs=11, batch_size=1 << 20, mini_batch_size=512)
ppo.show_progress = False
real = ppo.dist_params
mode = os.environ.get("C2RB_MODE", "controller")   # "controller" | "policy" (untrained: short episodes)


def controlled(obs):
    probs = real(obs)
    if mode != "controller":
        return probs
    z = 40.0 * (obs[:, 2] + 0.5 * obs[:, 3] + 0.02 * obs[:, 1])
    p1 = torch.sigmoid(z)
    return torch.stack([1.0 - p1, p1], dim=1)


ppo.dist_params = controlled
a = AsyncPPO("CartPole-v1", ppo, num_envs=E, seed=0)
out = {"E": E, "mode": mode}
for it in range(3):   # 0: warm-up (eager + first capture), then graphed rollouts
    a.step_score, a.reward_score = 0, 0
    ppo.memory.clear() if hasattr(ppo.memory, "clear") else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = a.worker()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[f"rollout{it}"] = {"transitions": int(n), "vector_steps": int(a.last_vector_steps),
                           "wall_ms": round(dt * 1e3, 2),
                           "env_steps_per_s": round(n / dt / 1e6, 2)}
    ppo.memory.clear()

# isolated costs on E rows: the policy forward (dist_params, eager and graphed), the step kernel
obs = torch.randn(E, 4, device="cuda") * 0.05


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


with torch.no_grad():
    out["policy_forward_eager_us"] = round(timeit(lambda: real(obs)), 1)
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        real(obs)
        with torch.cuda.graph(g, stream=st):
            real(obs)
    torch.cuda.current_stream().wait_stream(st)
    out["policy_forward_graph_us"] = round(timeit(g.replay), 1)
    gc = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        controlled(obs)
        with torch.cuda.graph(gc, stream=st):
            controlled(obs)
    torch.cuda.current_stream().wait_stream(st)
    out["forward_plus_controller_graph_us"] = round(timeit(gc.replay), 1)
print(json.dumps(out), flush=True)
