"""Is PPO._evaluate_old (PyTorch GEMMs + HIP GroupNorm/Categorical) bit-repeatable across fresh,
identically seeded PPO objects in one process?"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tests")]
from test_engine_gpu import _data  # noqa: E402
from PPO import PPO  # noqa: E402

S, A, R, Dn = _data(6037, 4, False)
outs = []
for i in range(4):
    torch.manual_seed(0)
    p = PPO(False, 4, 2, k_epochs=1, batch_size=64, mini_batch_size=512)
    lp, V = p._evaluate_old(S, A)
    torch.cuda.synchronize()
    outs.append((lp.clone(), V.clone()))
    print(i, "logp eq first", torch.equal(lp, outs[0][0]), "V eq first", torch.equal(V, outs[0][1]),
          "max dV", float((V - outs[0][1]).abs().max()), flush=True)
# raw GEMM repeatability at the shapes involved
x = torch.randn(6037, 64, device="cuda")
w = torch.randn(64, 64, device="cuda")
ys = [torch.nn.functional.linear(x, w) for _ in range(3)]
print("linear 6037x64x64 repeat:", [torch.equal(ys[0], y) for y in ys[1:]], flush=True)
