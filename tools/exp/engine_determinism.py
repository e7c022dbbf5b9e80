"""Is the persistent engine bit-reproducible?  The same inputs and starting state through
FusedUpdate.run several times per mode (PRL_UPD_XCD=0 spread / 1 one-XCD), final flat params,
moments and loss compared bitwise; also the step at which two runs first diverge (k_epochs=1
chunks)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd")]
from PPO import PPO  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 17
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = torch.Generator().manual_seed(1)
S = (0.05 * torch.randn(N, 4, generator=g)).cuda()
A = (torch.rand(N, generator=g) < 0.5).float().cuda()
old = (-0.69 + 0.01 * torch.randn(N, generator=g)).cuda()
adv = torch.randn(N, generator=g).cuda()
ret = torch.randn(N, generator=g).cuda()
torch.manual_seed(0)
p = PPO(False, 4, 2, lr=1e-3, k_epochs=11, batch_size=1, mini_batch_size=512)
eng = p._fused_engine()
start = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
out = {}
for mode in ("0", "1"):
    os.environ["PRL_UPD_XCD"] = mode
    finals = []
    for r in range(reps):
        for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), start):
            dst.copy_(src)
        loss = eng.run(S, A, old, adv, ret, 11)
        torch.cuda.synchronize()
        finals.append((eng.flat.cpu().clone(), eng.m.cpu().clone(), eng.v.cpu().clone(), float(loss)))
    eq = [all(torch.equal(a, b) for a, b in zip(finals[0][:3], f[:3])) and finals[0][3] == f[3] for f in finals[1:]]
    out[mode] = finals[0]
    print(json.dumps({"mode": mode, "reps_equal_to_first": eq,
                      "max_abs_diff_vs_first": [float((finals[0][0] - f[0]).abs().max()) for f in finals[1:]]}), flush=True)
print(json.dumps({"mode0_vs_mode1_equal": bool(torch.equal(out["0"][0], out["1"][0])),
                  "max_abs_diff": float((out["0"][0] - out["1"][0]).abs().max())}))
