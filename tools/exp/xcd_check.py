"""One-XCD engine mode (PRL_UPD_XCD=1) vs the default spread mode: same bits after a long
learn() (the exchange is deterministic, so any stale read would show), and us per step of each."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from learn_bench import synthetic_batch  # noqa: E402
from PPO import PPO  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "0", "1"]
batch = synthetic_batch(N)
res = {}
for mode in modes:
    os.environ["PRL_UPD_XCD"] = mode
    torch.manual_seed(0)
    p = PPO(False, 4, 2, lr=1e-3, k_epochs=11, batch_size=1, mini_batch_size=512)
    p.show_progress = False
    p.memory.push_device(*batch)
    p.learn()
    p.memory.push_device(*batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p.learn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    flat = p._engine.flat.detach().cpu().clone()
    same = None
    if mode in res:
        same = bool(torch.equal(flat, res[mode]))
    res[mode] = flat
    steps = 11 * -(-N // 512)
    print(json.dumps({"mode": mode, "us_per_step": round(dt / steps * 1e6, 2),
                      "equal_to_mode0": bool(torch.equal(flat, res["0"])) if "0" in res else None,
                      "repeat_equal": same}), flush=True)
