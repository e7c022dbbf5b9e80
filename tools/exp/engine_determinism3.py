"""First optimizer step where repeated engine runs (same start, learn()'s own inputs) diverge."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from learn_bench import synthetic_batch  # noqa: E402
from PPO import PPO  # noqa: E402

N = 1 << 18
torch.manual_seed(0)
p = PPO(False, 4, 2, lr=1e-3, k_epochs=11, batch_size=1, mini_batch_size=512)
p.show_progress = False
eng = p._fused_engine()
init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
p.memory.push_device(*synthetic_batch(N))
p.learn()
torch.cuda.synchronize()
ins = [x.clone() for x in p._last_update_inputs]
for m in (1, 2, 3, 4, 8, 16, 32, 64, 128, 512):
    sub = [x[:512 * m].contiguous() for x in ins]
    outs = []
    for r in range(6):
        for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
            dst.copy_(src)
        loss = eng.run(*sub, 1)
        torch.cuda.synchronize()
        outs.append((eng.flat.cpu().clone(), eng.m.cpu().clone(), float(loss)))
    eqp = [bool(torch.equal(outs[0][0], o[0])) for o in outs[1:]]
    eqm = [bool(torch.equal(outs[0][1], o[1])) for o in outs[1:]]
    nd = [int((outs[0][1] != o[1]).sum()) for o in outs[1:]]
    print(json.dumps({"steps": m, "params_equal": eqp, "m_equal": eqm, "m_words_differing": nd,
                      "loss": [o[2] for o in outs]}), flush=True)
