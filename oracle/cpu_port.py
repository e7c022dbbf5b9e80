"""CPU PORT of one AsyncPPO iteration — test/bench infrastructure only (bench.py cpu_baseline).

The reference's algorithm on the host (AsyncTools/AsyncPPO.py:117-165, PPO/PPO.py:122-260):
  rollout: per-env sequential CartPole stepping over the active envs, one episode per env,
           env-major flatten (C, prl_oracle.c:or_cartpole_rollout; the policy is a fixed
           distribution here, so policy inference is NOT in the rollout time);
  learn:   policy_old evaluation, sequential float32 GAE (C, O(N) — the reference's list.insert
           makes it O(N^2)), advantage normalisation, k_epochs x unshuffled minibatches of the
           clipped surrogate + 0.5 SmoothL1 - 0.01 H with AdamW and clip_grad_norm_(2.0),
           all in PyTorch on the CPU.
"""
import ctypes
import time

import numpy as np
import torch
from torch import nn, optim

import oracle as O


def cartpole_rollout(E, seed=0, p1=0.5, tmax=500):
    rng_states = np.stack([np.random.default_rng(seed + e).uniform(-0.05, 0.05, 4)
                           for e in range(E)]).astype(np.float64)
    s_work = np.empty_like(rng_states)
    term = np.zeros(E, np.uint8)
    lens = np.zeros(E, np.int32)
    traj_obs = np.zeros((tmax, E, 4), np.float32)
    traj_act = np.zeros((tmax, E), np.int32)
    cap = E * 64
    S = np.zeros((cap, 4), np.float32)
    A = np.zeros(cap, np.float32)
    R = np.zeros(cap, np.float32)
    Dn = np.zeros(cap, np.float32)
    p = O._p
    t0 = time.perf_counter()
    n = O.lib().or_cartpole_rollout(E, p(rng_states), seed, ctypes.c_float(p1), tmax, p(s_work),
                                    p(term), p(lens), p(traj_obs), p(S), p(A), p(R), p(Dn),
                                    p(traj_act))
    dt = time.perf_counter() - t0
    assert n <= cap
    return dt, S[:n], A[:n], R[:n], Dn[:n]


def _policy(obs_dim, act_dim):
    def block(i, o):
        return [nn.Linear(i, o, bias=False), nn.GroupNorm(8, 64), nn.SiLU()]
    trunk = nn.Sequential(*block(obs_dim, 64))
    actor = nn.Sequential(*block(64, 64), nn.Linear(64, act_dim), nn.Softmax(-1))
    critic = nn.Sequential(*block(64, 64), nn.Linear(64, 1))
    return trunk, actor, critic


def learn_port(S, A, R, Dn, mb=512, k_epochs=11, gamma=0.995, lam=0.95, lr=1e-3):
    torch.manual_seed(0)
    trunk, actor, critic = _policy(S.shape[1], 2)
    params = list(trunk.parameters()) + list(actor.parameters()) + list(critic.parameters())
    opt = optim.AdamW(params, lr=lr)
    St, At = torch.from_numpy(S), torch.from_numpy(A)
    t0 = time.perf_counter()
    with torch.no_grad():
        lp_old, v_old = [], []
        for lo in range(0, len(S), mb):
            f = trunk(St[lo:lo + mb])
            d = torch.distributions.Categorical(actor(f))
            lp_old.append(d.log_prob(At[lo:lo + mb]))
            v_old.append(critic(f).squeeze(-1))
        lp_old, v_old = torch.cat(lp_old), torch.cat(v_old)
    V = v_old.numpy()
    ret = torch.from_numpy(O.gae(R, Dn, V, V[-1], gamma, lam))
    adv = ret - v_old
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    sl1 = nn.SmoothL1Loss()
    for _ in range(k_epochs):
        for lo in range(0, len(S), mb):
            f = trunk(St[lo:lo + mb])
            d = torch.distributions.Categorical(actor(f))
            lp = d.log_prob(At[lo:lo + mb])
            v = critic(f).squeeze(-1)
            H = d.entropy().mean().detach()
            ratio = torch.exp(torch.clamp(lp - lp_old[lo:lo + mb], -20, 20))
            a = adv[lo:lo + mb]
            loss = -torch.min(ratio * a, torch.clamp(ratio, 0.8, 1.2) * a) \
                + 0.5 * sl1(v, ret[lo:lo + mb]) - 0.01 * H
            opt.zero_grad()
            loss.mean().backward()
            nn.utils.clip_grad_norm_(params, 2.0)
            opt.step()
    return time.perf_counter() - t0


def cpu_iteration(E=8192, mb=512, k_epochs=11, seed=0):
    """Returns (env_steps, rollout_s, learn_s, threads)."""
    t_roll, S, A, R, Dn = cartpole_rollout(E, seed)
    t_learn = learn_port(S, A, R, Dn, mb=mb, k_epochs=k_epochs)
    return len(S), t_roll, t_learn, torch.get_num_threads()
