"""Kernel-level timings of the two HBM-bound hot kernels, cold cache (512 MiB read before every
launch), HIP events on the launching stream.  Run alone, or under rocprofv3 (--kernel-trace
--stats, or one --pmc pass per counter group) to read the same launches' counters.

  GAE scan (prl_gae, gae_kernel<true>): 20 B per transition (r, d, V in; ret, adv out)
  CartPole fused rollout step (rollout_step_kernel<CartPole>): 111 B per env-step
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parallel-reinforcement-learning_amd")]
import prl_native  # noqa: E402
from bench import ENV_STEP_BYTES, GAE_BYTES_PER_TRANSITION, HBM_PEAK_GBS, time_kernel  # noqa

CARTPOLE_STEP_BYTES = ENV_STEP_BYTES["CartPole-v1"]


def gae_case(n, pd=0.05, seg=None, reps=10):
    g = torch.Generator(device="cuda").manual_seed(n)
    r = torch.ones(n, device="cuda")
    V = torch.randn(n, device="cuda", generator=g)
    if seg:
        d = torch.zeros(n, device="cuda")
        d[seg - 1::seg] = 1
    else:
        d = (torch.rand(n, device="cuda", generator=g) < pd).float()
        d[-1] = 1
    ret, adv = torch.empty_like(V), torch.empty_like(V)
    sums = torch.zeros(2, dtype=torch.float64, device="cuda")
    med, mn = time_kernel(lambda: prl_native.gae(r, d, V, None, 0.995, 0.95, ret, adv, sums),
                          reps=reps)
    gbs = GAE_BYTES_PER_TRANSITION * n / (med * 1e-3) / 1e9
    return {"kernel": "gae", "n": n, "us": round(med * 1e3, 2), "min_us": round(mn * 1e3, 2),
            "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def gae_file_case(path, reps=10):
    x = torch.load(path, weights_only=True)
    r, d, V = (x[k].cuda() for k in ("r", "d", "V"))
    nv = x["next_value"].cuda() if x["next_value"] is not None else None
    n = V.numel()
    ret, adv = torch.empty_like(V), torch.empty_like(V)
    sums = torch.zeros(2, dtype=torch.float64, device="cuda")
    med, mn = time_kernel(lambda: prl_native.gae(r, d, V, nv, x["gamma"], x["lam"], ret, adv, sums),
                          reps=reps)
    gbs = GAE_BYTES_PER_TRANSITION * n / (med * 1e-3) / 1e9
    return {"kernel": "gae", "n": n, "source": path, "us": round(med * 1e3, 2),
            "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def cartpole_step_case(E, reps=10):
    from AsyncTools.AsyncPPO import DeviceTrajectory, EnvVectorizer
    vec = EnvVectorizer("CartPole-v1", E, seed=0)
    tr = DeviceTrajectory(E, vec.spec, vec.device)
    probs = torch.full((E, 2), 0.5, device="cuda")

    def launch():  # step 0 from a fresh reset: every env active
        vec.reset_device(tr.obs[0])
        torch.cuda._sleep(1_000_000)
        prl_native.rollout_step(0, 0, vec.phys, vec.t_elapsed, vec.terminal, probs, 1.0, 1, tr.T,
                                tr.obs, tr.act, tr.rew, tr.done, tr.ep_len, tr.active_after,
                                tr.reward_sum)

    # time only the step: reset + sleep go before the start event
    flush = torch.ones(128 << 20, dtype=torch.float32, device="cuda")   # read-only flush
    ms = []
    for _ in range(reps):
        vec.reset_device(tr.obs[0])
        flush.sum()
        torch.cuda._sleep(2_000_000)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        prl_native.rollout_step(0, 0, vec.phys, vec.t_elapsed, vec.terminal, probs, 1.0, 1, tr.T,
                                tr.obs, tr.act, tr.rew, tr.done, tr.ep_len, tr.active_after,
                                tr.reward_sum)
        e.record()
        e.synchronize()
        ms.append(s.elapsed_time(e))
    ms.sort()
    med = ms[len(ms) // 2]
    gbs = CARTPOLE_STEP_BYTES * E / (med * 1e-3) / 1e9
    return {"kernel": "cartpole_rollout_step", "envs": E, "us": round(med * 1e3, 2),
            "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "env_steps_per_s": round(E / (med * 1e-3), 1)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--gae-n", type=int, default=0, help="only the GAE scan at this size")
    ap.add_argument("--gae-seg", type=int, default=0, help="with --gae-n: fixed segment length")
    ap.add_argument("--gae-file", default=None, help="only the GAE scan on bench.py --dump-gae")
    ap.add_argument("--env-e", type=int, default=0, help="only the CartPole rollout step at E envs")
    a = ap.parse_args()
    if a.env_e:
        print(json.dumps(cartpole_step_case(a.env_e, reps=a.reps)), flush=True)
        sys.exit(0)
    if a.gae_file:
        print(json.dumps(gae_file_case(a.gae_file, reps=a.reps)), flush=True)
        sys.exit(0)
    if a.gae_n:
        print(json.dumps(gae_case(a.gae_n, seg=a.gae_seg or None, reps=a.reps)), flush=True)
        sys.exit(0)
    out = []
    sizes = [1 << 20] if a.quick else [1 << 20, 2_300_000, 65536 * 200]
    for n in sizes:
        out.append(gae_case(n, reps=a.reps))
    out.append(gae_case(65536 * 200, seg=200, reps=a.reps))
    for E in ([65536] if a.quick else [65536, 1 << 22]):
        out.append(cartpole_step_case(E, reps=a.reps))
    for o in out:
        print(json.dumps(o), flush=True)
