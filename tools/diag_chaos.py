"""Three float32 implementations of the same continuous learn() (fused engine, per-step GPU
path, CPU PyTorch + oracle ops): pairwise function-space distance after 3 epochs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]
from fake_ops import FakeOps  # noqa: E402
from test_engine_gpu import _data, _outputs, _run  # noqa: E402
from PPO import PPO  # noqa: E402


def dist(p, q, S, A):
    (lf, vf), (lg, vg) = _outputs(p, S, A), _outputs(q, S, A)
    return (round(float((lf - lg).abs().max()) / (float(lg.abs().max()) + 1), 5),
            round(float((vf - vg).abs().max()) / (float(vg.abs().max()) + 1), 5))


for cont, kw in ((True, dict(clip=1e3, lr=3e-4)), (True, dict(clip=0.2, lr=1e-3)),
                 (False, dict(clip=0.2, lr=1e-3))):
    data = _data(6037, 3 if cont else 4, cont)
    f = _run(True, cont, data, 512, 3, **kw)
    g = _run(False, cont, data, 512, 3, **kw)
    # CPU: the same PPO object model on CPU tensors with the oracle's GAE/normalise/surrogate
    torch.manual_seed(0)
    D, A = (3, 1) if cont else (4, 2)
    c = PPO(cont, D, A, action_scaling=2.0 if cont else None, lr=kw["lr"], k_epochs=3,
            batch_size=64, mini_batch_size=512, policy_clip=kw["clip"])
    c.show_progress = False
    c.policy.cpu(); c.policy_old.cpu()
    c.device = torch.device("cpu")
    c.optimizer = torch.optim.AdamW(c.policy.parameters(), lr=kw["lr"])
    c._ops = FakeOps()
    c.memory.push_device(*(x.cpu() for x in data))
    c.learn()
    S, Aa = data[0][:2048], data[1][:2048]
    print("cont" if cont else "disc", kw, "fused-graph", dist(f, g, S, Aa), "fused-cpu",
          dist(f, c, S, Aa), "graph-cpu", dist(g, c, S, Aa), flush=True)
