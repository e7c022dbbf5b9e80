"""pytest-run diagnostic (run after tests/test_kernels_gpu.py, where the full suite saw it): the
C5 graphed rollout's first (eager + warm-up capture) rollout, reward sum and live rows' dist
checked after every vector step, around the capture and after the replay."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-reinforcement-learning_amd"))


def test_diag_graph_nan(monkeypatch):
    from AsyncTools.AsyncPPO import AsyncPPO
    from PPO import PPO
    monkeypatch.setenv("PRL_WIDE_ROLLOUT", "0")
    monkeypatch.setenv("PRL_ROLLOUT_GRAPH", "1")
    E = 200
    torch.manual_seed(0)
    p = PPO(True, 348, 17, action_scaling=1.0, batch_size=10**9, mini_batch_size=512)
    a = AsyncPPO("SyntheticHumanoid-v0", p, num_envs=E, seed=5)
    log = []
    orig_step = a._step_kernel

    def step(k, dist, seed, scaling, active_after):
        if not isinstance(k, torch.Tensor):
            torch.cuda.synchronize()
            tr = a._traj
            live = a.env.terminal == 0
            bad = (~torch.isfinite(dist).all(-1)) & live
            before = float(tr.reward_sum.item())
        orig_step(k, dist, seed, scaling, active_after)
        if not isinstance(k, torch.Tensor):
            torch.cuda.synchronize()
            after = float(tr.reward_sum.item())
            if int(bad.sum()) and not os.path.exists(os.path.join(ROOT, "gpurun_out", "nan_case.pt")):
                os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
                obs = a._traj.obs[k].clone()
                flat = p._dist_flat_buf.clone()
                again = torch.empty_like(dist)
                import prl_native
                prl_native.ppo_wide_dist(flat, 348, 17, False, obs, again)
                torch.cuda.synchronize()
                torch.save({"obs": obs.cpu(), "flat": flat.cpu(), "dist": dist.cpu(), "again": again.cpu(),
                            "live": live.cpu(), "k": k}, os.path.join(ROOT, "gpurun_out", "nan_case.pt"))
                log.append(f"saved nan_case.pt: recomputed dist finite rows "
                           f"{int(torch.isfinite(again).all(-1).sum())}/{again.shape[0]}")
            if int(bad.sum()) or after != after or k < 5:
                e = int(torch.nonzero(bad)[0]) if int(bad.sum()) else -1
                log.append(f"k={k}: live rows with non-finite dist {int(bad.sum())} (first e={e}), "
                           f"reward_sum {before} -> {after}, obs row finite "
                           f"{bool(torch.isfinite(a._traj.obs[k, e]).all()) if e >= 0 else None}")
    a._step_kernel = step
    orig_dist = p.dist_params
    seen = {"n": 0}

    def dist_params(obs):
        tr = a._traj
        torch.cuda.synchronize()
        b = float(tr.reward_sum.item())
        flat_ptr = getattr(p, "_dist_flat_buf", None)
        out = orig_dist(obs)
        torch.cuda.synchronize()
        c = float(tr.reward_sum.item())
        seen["calls"] = seen.get("calls", 0) + 1
        if seen["calls"] <= 6:
            log.append(f"dist_params call {seen['calls']}: reward_sum {b} -> {c}")
        if (b == b) != (c == c) and seen["n"] < 3:
            seen["n"] += 1
            rs = tr.reward_sum
            log.append(f"dist_params flipped reward_sum {b} -> {c}: reward_sum ptr {rs.data_ptr():#x}, "
                       f"out ptr {out.data_ptr():#x} bytes {out.numel() * 4}, obs ptr {obs.data_ptr():#x}, "
                       f"flat ptr {p._dist_flat_buf.data_ptr():#x} bytes {p._dist_flat_buf.numel() * 4}")
        return out
    p.dist_params = dist_params
    import AsyncTools.AsyncPPO as AP
    RealEvent = torch.cuda.Event
    flips = {"n": 0}

    class Ev(RealEvent):   # recorded right after the loop's pinned copy of active_after[k]
        def record(self, stream=None):
            tr = a._traj
            torch.cuda.synchronize()
            v = float(tr.reward_sum.item())
            flips["calls"] = flips.get("calls", 0) + 1
            if flips["calls"] <= 6:
                log.append(f"event record {flips['calls']}: reward_sum {v}")
            if v != v and flips["n"] < 2:
                flips["n"] += 1
                log.append(f"NaN right after the pinned copy: reward_sum ptr {tr.reward_sum.data_ptr():#x}, "
                           f"active_after ptr {tr.active_after.data_ptr():#x}, pinned ptr "
                           f"{tr.pinned.data_ptr():#x} is_pinned {tr.pinned.is_pinned()}, "
                           f"ep_len ptr {tr.ep_len.data_ptr():#x}, offsets ptr {tr.offsets.data_ptr():#x}")
            return super().record(stream) if stream is not None else super().record()
    monkeypatch.setattr(AP.torch.cuda, "Event", Ev)
    orig_cap = a._capture_step

    def cap(seed, scaling):
        tr = a._traj
        torch.cuda.synchronize()
        b = float(tr.reward_sum.item())
        g = orig_cap(seed, scaling)
        torch.cuda.synchronize()
        log.append(f"capture: reward_sum {b} -> {float(tr.reward_sum.item())}")
        if g is not None:
            orig_replay = g.replay

            def replay():
                r0 = float(tr.reward_sum.item())
                orig_replay()
                torch.cuda.synchronize()
                r1 = float(tr.reward_sum.item())
                if r1 != r1 or len(log) < 40:
                    log.append(f"replay: reward_sum {r0} -> {r1}, k_dev {a._k_dev.tolist()}")
            g.replay = replay
        return g
    a._capture_step = cap
    n = a.worker()
    print("\n".join(log[:60]))
    print(f"it0: N={n} reward_score={float(a.reward_score)}")
