"""Hunt an intermittent divergence: repeat identical work many times and report the first stage
that differs from the first run.  (1) learn() alternating fused / per-step; (2) prl_gae under a
concurrent load on another stream; (3) the fused update kernel alone on fixed inputs."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tests")]
import prl_native  # noqa: E402
from test_engine_gpu import _data, _run  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
data = _data(6037, 4, False)

if which in ("all", "learn"):
    ref = {}
    bad = 0
    for i in range(24):
        fused = i % 2 == 0
        p = _run(fused, False, data, 512, 3, clip=10.0)
        S, A, old, adv, ret = p._last_update_inputs
        sd = {k: v.clone() for k, v in p.policy.state_dict().items()}
        cur = dict(old=old.clone(), adv=adv.clone(), ret=ret.clone())
        tag = "F" if fused else "G"
        if tag not in ref:
            ref[tag] = (cur, sd)
            continue
        rc, rsd = ref[tag]
        diffs = {k: not torch.equal(cur[k], rc[k]) for k in cur}
        wd = max(float((sd[k] - rsd[k]).abs().max()) for k in sd)
        if any(diffs.values()) or wd > 0:
            bad += 1
            print("learn run", i, tag, "stage differs:", diffs, "weights", wd, flush=True)
    print("learn: runs differing from the first of their path:", bad, flush=True)

if which in ("all", "gae"):
    r, d, V = data[2], data[3], torch.randn(6037, device="cuda")
    def call():
        ret, adv = torch.empty_like(V), torch.empty_like(V)
        sums = torch.zeros(2, dtype=torch.float64, device="cuda")
        prl_native.gae(r, d, V, V[-1:], 0.995, 0.95, ret, adv, sums)
        return ret, adv, sums
    r0 = [x.clone() for x in call()]
    side = torch.cuda.Stream()
    big = torch.empty(64 << 20, device="cuda")
    bad = 0
    for i in range(2000):
        if i % 3 == 0:
            with torch.cuda.stream(side):
                big.mul_(1.0001)          # uneven load from another stream
        out = call()
        if i % 50 == 49:
            torch.cuda.synchronize()
        if not all(torch.equal(a, b) for a, b in zip(out, r0)):
            bad += 1
            if bad < 8:
                ws = prl_native._ws.get(prl_native.OP_GAE, 0, V.device)
                ctr = ws[:16].view(torch.int32).tolist()
                def wsb(nt):
                    ng = (nt + 63) // 64
                    return 64 + 64 * ng + ((8 * nt + 15) // 16) * 16 + 16 * nt + 16 * ng + 64
                nb_ = ws.numel()
                nt = max(1, int((nb_ - 216) / 25.25))
                while nt > 1 and wsb(nt) > nb_:
                    nt -= 1
                ng = (nt + 63) // 64
                o_ts = 64 + 64 * ng + ((8 * nt + 15) // 16) * 16
                tsums = ws[o_ts:o_ts + 16 * 3].view(torch.float64).tolist()
                o_gs = o_ts + 16 * nt
                gsums = ws[o_gs:o_gs + 16].view(torch.float64).tolist()
                print("   tile sums", tsums, "group", gsums, flush=True)
                print("gae call", i, "sums", out[2].tolist(), "ref", r0[2].tolist(), "ctrs", ctr,
                      "group_ctr0", ws[64:68].view(torch.int32).tolist(),
                      "host", [float(out[1].double().sum()), float((out[1].double() ** 2).sum())],
                      flush=True)
    torch.cuda.synchronize()
    print("gae: differing calls:", bad, "lookaheads:", flush=True)

if which in ("all", "kernel"):
    p = _run(True, False, data, 512, 1, clip=10.0)
    eng = p._engine
    S, A, old, adv, ret = p._last_update_inputs
    init = (eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone())
    outs = None
    bad = 0
    for i in range(100):
        eng.flat.copy_(init[0]); eng.m.copy_(init[1]); eng.v.copy_(init[2]); eng.step.copy_(init[3])
        eng.run(S, A, old, adv, ret, 3)
        cur = (eng.flat.clone(), eng.m.clone(), eng.v.clone())
        if outs is None:
            outs = cur
        elif not all(torch.equal(a, b) for a, b in zip(cur, outs)):
            bad += 1
            if bad < 5:
                print("kernel run", i, "max diff", float((cur[0] - outs[0]).abs().max()), flush=True)
    print("kernel: differing runs:", bad, flush=True)
