"""Per-step cost of the data-parallel (stepped) engine on one GPU: grad kernel -> all-reduce ->
AdamW kernel per optimizer step on the C2 learn workload (2^20 synthetic CartPole transitions),
with (a) no collective, (b) a one-rank RCCL all_reduce through torch.distributed — the host
and launch overhead the N > 1 runs pay on top of the collective's own latency — and (c) the
native loop (prl_ppo_update_dp: the steps enqueued from C, ncclAllReduce on a one-rank
communicator of the engine's own)."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from learn_bench import synthetic_batch  # noqa: E402
from PPO import PPO  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29611")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
N, mb, k = 1 << 20, 512, 11
batch = synthetic_batch(N)
import prl_native  # noqa: E402
prl_native.dp_rccl_open()
# host-side enqueue time of the native loop: if it approaches the GPU time, the loop is host-bound
_enq = []


def _timed(fn):
    def wrap(*a, **k):
        t = time.perf_counter()
        r = fn(*a, **k)
        _enq.append(time.perf_counter() - t)
        return r
    return wrap


prl_native.ppo_update_dp = _timed(prl_native.ppo_update_dp)
comm = prl_native.dp_comm_init(prl_native.dp_unique_id(), 1, 0)
MODES = (("identity", lambda t: t, None, {}), ("rccl-1rank", dist.all_reduce, None, {}),
         ("native-stepped-rccl-1rank", None, comm, {}))
for label, ar, cm, env in MODES:
    os.environ.update(env)
    torch.manual_seed(0)
    p = PPO(False, 4, 2, lr=1e-3, k_epochs=k, batch_size=1, mini_batch_size=mb)
    p.show_progress = False
    p.memory.push_device(*batch)
    S, A, R, Dn = p.memory.device_tensors(p.device)
    old, V = p._evaluate_old(S, A)
    adv = torch.randn_like(V)
    ret = torch.randn_like(V)
    eng = p._fused_engine()
    eng.run_stepped(S[:8192], A[:8192], old[:8192], adv[:8192], ret[:8192], 1, [8192], ar,
                    comm=cm)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run_stepped(S, A, old, adv, ret, k, [N], ar, comm=cm)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = k * -(-N // mb)
    rec = {"all_reduce": label, "learn_update_ms_per_1M": round(dt * 1e3, 1),
           "us_per_step": round(dt / steps * 1e6, 2)}
    if cm is not None and _enq:   # the timed (last) call of this mode
        rec["host_enqueue_us_per_step"] = round(_enq[-1] / steps * 1e6, 2)
    print(json.dumps(rec), flush=True)
prl_native.dp_comm_destroy(comm)
dist.destroy_process_group()
