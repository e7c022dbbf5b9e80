"""Per-optimizer-step time of the data-parallel persistent engine (prl_ppo_update_dpx) on W ranks
sharing ONE GPU (gloo for the IPC-handle exchange), against the single-GPU engine
(prl_ppo_update) on the same per-rank rows.  CartPole shape, mb 512, k 2.

  python tools/dp_persistent_bench.py [world] [rows_per_rank]
"""
import json
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATHS = [ROOT, os.path.join(ROOT, "parallel-reinforcement-learning_amd")]


def _data(n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    S = torch.randn(n, 4, device="cuda", generator=g) * 0.5
    A = (torch.rand(n, device="cuda", generator=g) < 0.5).float().reshape(-1, 1)
    old = torch.randn(n, device="cuda", generator=g) * 0.1 - 0.7
    adv = torch.randn(n, device="cuda", generator=g)
    ret = torch.randn(n, device="cuda", generator=g)
    return S, A, old, adv, ret


def _worker(rank, world, port, n, out):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PRL_DP_PERSISTENT="1")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from PPO import PPO
        torch.manual_seed(0)
        p = PPO(False, 4, 2, lr=3e-4, k_epochs=2, batch_size=1, mini_batch_size=512)
        eng = p._fused_engine()
        data = _data(n, 100 + rank)
        k, mb = 2, 512
        steps = k * (-(-n // mb))
        res = {}
        for name in ("dpx", "single"):
            ts = []
            for rep in range(3):
                torch.distributed.barrier()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                if name == "dpx":
                    eng.run_dp_persistent(*data, k, [n] * world, p.all_reduce)
                elif rank == 0:   # the single-GPU engine alone (the other ranks wait)
                    eng.run(*data, k)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e))
            res[name] = round(min(ts) * 1e3 / steps, 2)
            if os.environ.get("PRL_UPD_PROFILE") == "1" and (name == "dpx" or rank == 0):
                res[name + "_phases"] = eng.profile()
        torch.distributed.barrier()
        if rank == 0:
            with open(out, "w") as f:
                json.dump({"world": world, "rows_per_rank": n, "steps": steps,
                           "us_per_step_dpx": res["dpx"], "us_per_step_single_engine": res["single"],
                           **{k: v for k, v in res.items() if k.endswith("_phases")}}, f)
        eng.close()
    finally:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18
    out = os.path.join(ROOT, "gpurun_out", f"dpx_w{world}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    mp.spawn(_worker, args=(world, 29990, n, out), nprocs=world, join=True)
    print(open(out).read(), flush=True)
