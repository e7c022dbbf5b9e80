"""One optimizer step, repeated from the same start on learn()'s inputs: which exchange buffer
differs between runs?  Reads the workspace: norm pieces sq[NW G], reduced gradient red[Qtot*4],
partials part[G][Qtot*4] (layout of upd_ws_carve)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
import prl_native  # noqa: E402
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
ins = [x[:512].contiguous().clone() for x in p._last_update_inputs]
L4 = prl_native.ppo_image_floats(4, 2, True)
Qtot = L4 // 4
G = eng.grid


def take(off, nbytes):
    return off + ((nbytes + 255) & ~255)


o_ctr = 0
o_prof = take(o_ctr, 4 * 544)
o_sq = take(o_prof, 256)
o_red = take(o_sq, 2048 * 4)
o_part = take(o_red, Qtot * 16)
ws = eng.ws
outs = []
for r in range(5):
    for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
        dst.copy_(src)
    eng.ws.zero_()
    eng.run(*ins, 1)
    torch.cuda.synchronize()
    b = ws.cpu()
    sq = b[o_sq:o_sq + 4 * 4 * G].view(torch.float32).clone()
    red = b[o_red:o_red + Qtot * 16].view(torch.float32).clone()
    part = b[o_part:o_part + G * Qtot * 16].view(torch.float32).view(G, Qtot * 4).clone()
    outs.append((sq, red, part, eng.m.cpu().clone()))
    img_m = torch.zeros(L4, device="cuda")
    img_p = torch.zeros(L4, device="cuda")
    img_v = torch.zeros(L4, device="cuda")
    prl_native.ppo_image(4, 2, True, eng.flat, eng.m, eng.v, img_p, img_m, img_v, True)
    mi = img_m.cpu()[:-4]
    g = red[:-4]
    nz = g != 0
    ratio = (mi[nz].double() / (0.1 * g[nz].double()))
    n2 = float((g.double() ** 2).sum())
    print(json.dumps({"rep": r, "implied_clip_min": float(ratio.min()), "implied_clip_max": float(ratio.max()),
                      "host_clip": min(1.0, 2.0 / (n2 ** 0.5 + 1e-6)), "sq_sum": float(sq.double().sum()),
                      "red_norm2": n2}), flush=True)
for r in range(1, 5):
    sq0, red0, part0, m0 = outs[0]
    sq1, red1, part1, m1 = outs[r]
    print(json.dumps({"run": r, "sq_equal": bool(torch.equal(sq0, sq1)), "red_equal": bool(torch.equal(red0, red1)),
                      "part_equal": bool(torch.equal(part0, part1)),
                      "part_rows_differing": [int(i) for i in (part0 != part1).any(1).nonzero().flatten()][:40],
                      "sq_diff_idx": [int(i) for i in (sq0 != sq1).nonzero().flatten()][:40],
                      "m_equal": bool(torch.equal(m0, m1)),
                      "norm2_from_red": [float((red0[:-4].double() ** 2).sum()), float((red1[:-4].double() ** 2).sum())],
                      "norm2_from_sq": [float(sq0.double().sum()), float(sq1.double().sum())]}), flush=True)
