"""Per-workgroup phase durations of the GAE kernel (instrumented build, tools/exp/gae_phases.hip)
on the bench-sized input: load, local scan, tail resolve, carry wait, stores, statistics."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parallel-reinforcement-learning_amd")]
import prl_native  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("GAE_PHASES_LIB", "libgae_phases.so")))
P = ctypes.c_void_p
CASES = [(int(a), int(b)) for a, b in (x.split(":") for x in sys.argv[1].split(","))] if len(sys.argv) > 1 else [(8_269_824, 126), (2_277_376, 35)]
for n, seg in CASES:
    g = torch.Generator(device="cuda").manual_seed(1)
    r = torch.ones(n, device="cuda")
    V = torch.randn(n, device="cuda", generator=g)
    if seg < 0:   # every -seg-th transition ends an episode (trained CartPole: 500, Pendulum: 200)
        d = torch.zeros(n, device="cuda")
        d[-seg - 1::-seg] = 1
    else:
        d = (torch.rand(n, device="cuda", generator=g) < 1.0 / seg).float()
    d[-1] = 1
    ret, adv = torch.empty_like(V), torch.empty_like(V)
    sums = torch.zeros(2, dtype=torch.float64, device="cuda")
    nt = -(-n // 2048)
    prof = torch.zeros((nt + 8192) * 16,   # grid = R * Q can exceed the tile count
                        dtype=torch.int64, device="cuda")
    assert lib.gae_prof_set(P(prof.data_ptr())) == 0
    nbytes = prl_native.workspace_bytes(prl_native.OP_GAE, n)
    ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    flush = torch.ones(128 << 20, device="cuda")
    for rep in range(3):
        flush.sum()
        torch.cuda._sleep(2_000_000)
        rc = lib.prl_gae(P(r.data_ptr()), P(d.data_ptr()), P(V.data_ptr()), None,
                         ctypes.c_int64(n), ctypes.c_double(0.995), ctypes.c_double(0.95),
                         P(ret.data_ptr()), P(adv.data_ptr()), P(sums.data_ptr()),
                         P(ws.data_ptr()), ctypes.c_int64(nbytes),
                         P(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert rc == 0
    tf = prof.view(-1, 16).cpu().numpy().astype(np.int64)
    tf = tf[tf[:, 0] > 0]   # blocks past the last stream's end record nothing
    t = tf[:, :7]
    t0 = t[:, 0].min()
    dur = np.diff(t, axis=1) * 10.0 / 1000.0   # us
    names = ["load", "local", "tail", "carry wait", "stores", "stats+arrive"]
    out = {"n": n, "tiles": nt, "kernel_span_us": round(float((t[:, 6].max() - t0) * 0.01), 2),
           "wg_lifetime_us_mean": round(float(((t[:, 6] - t[:, 0]) * 0.01).mean()), 2),
           "start_spread_us": round(float((t[:, 0].max() - t0) * 0.01), 2)}
    for i, nm in enumerate(names):
        out[nm] = {"mean": round(float(dur[:, i].mean()), 3), "p99": round(float(np.percentile(dur[:, i], 99)), 3)}
    tl = tf[:, 8:11]
    has = tl[:, 0] > 0   # tiles whose tail thread ran (chunk 255 does not end in a break)
    if has.any():
        x = tl[has]
        out["tail_thread"] = {"tiles": int(has.sum()),
                              "start_after_local_us": round(float(((x[:, 0] - t[has, 2]) * 0.01).mean()), 3),
                              "granule_wait_us": round(float(((x[:, 1] - x[:, 0]) * 0.01).mean()), 3),
                              "walk_us": round(float(((x[:, 2] - x[:, 1]) * 0.01).mean()), 3),
                              "walk_p99_us": round(float(np.percentile((x[:, 2] - x[:, 1]) * 0.01, 99)), 3)}
    print(json.dumps(out), flush=True)
