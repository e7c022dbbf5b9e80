"""learn() bit-reproducibility: fresh PPO (same seed) + a fresh copy of the same synthetic memory,
learn() once, several times; compare the engine's inputs (old_logp, adv, ret) and final params."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from learn_bench import synthetic_batch  # noqa: E402
from PPO import PPO  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
base = [x.clone() for x in synthetic_batch(N)]
runs = []
for r in range(4):
    torch.manual_seed(0)
    p = PPO(False, 4, 2, lr=1e-3, k_epochs=11, batch_size=1, mini_batch_size=512)
    p.show_progress = False
    p.memory.push_device(*[x.clone() for x in base])
    p.learn()
    torch.cuda.synchronize()
    ins = [x.detach().cpu().clone() for x in p._last_update_inputs]
    runs.append((ins, p._engine.flat.detach().cpu().clone()))
names = ["S", "A", "old_logp", "adv", "ret"]
for r in range(1, len(runs)):
    print(json.dumps({"run": r, **{n: bool(torch.equal(a, b)) for n, a, b in zip(names, runs[0][0], runs[r][0])},
                      "params": bool(torch.equal(runs[0][1], runs[r][1]))}), flush=True)
print(json.dumps({"base_unchanged": all(torch.equal(a.cpu(), b.cpu()) for a, b in zip(base, synthetic_batch(N)))}))
