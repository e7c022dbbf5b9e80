"""Engine reproducibility on learn()'s own captured inputs vs random inputs, same engine, same
starting state restored before every run."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from learn_bench import synthetic_batch  # noqa: E402
from PPO import PPO  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
torch.manual_seed(0)
p = PPO(False, 4, 2, lr=1e-3, k_epochs=11, batch_size=1, mini_batch_size=512)
p.show_progress = False
eng = p._fused_engine()
init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
p.memory.push_device(*synthetic_batch(N))
p.learn()
torch.cuda.synchronize()
learn_ins = [x.clone() for x in p._last_update_inputs]
g = torch.Generator().manual_seed(1)
rnd_ins = [(0.05 * torch.randn(N, 4, generator=g)).cuda(), (torch.rand(N, generator=g) < 0.5).float().cuda(),
           (-0.69 + 0.01 * torch.randn(N, generator=g)).cuda(), torch.randn(N, generator=g).cuda(),
           torch.randn(N, generator=g).cuda()]
for name, ins in (("learn_inputs", learn_ins), ("random_inputs", rnd_ins), ("learn_inputs", learn_ins)):
    outs = []
    for r in range(4):
        for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
            dst.copy_(src)
        eng.run(*ins, 11)
        torch.cuda.synchronize()
        outs.append(eng.flat.cpu().clone())
    print(json.dumps({"inputs": name, "equal_to_first": [bool(torch.equal(outs[0], o)) for o in outs[1:]],
                      "maxdiff": [float((outs[0] - o).abs().max()) for o in outs[1:]],
                      "nan": bool(torch.isnan(outs[0]).any())}), flush=True)
print(json.dumps({k: [float(x.float().min()), float(x.float().max())] for k, x in zip(["S", "A", "old", "adv", "ret"], learn_ins)}))
