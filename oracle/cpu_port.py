"""CPU PORT of one AsyncPPO iteration — test/bench infrastructure only (bench.py cpu_baseline).

The reference's CPU path, step for step, on the GPU box's host (it cannot travel there itself):
  rollout  AsyncPPO.worker (AsyncTools/AsyncPPO.py:117-146): per vector step the policy MLP in
           torch-CPU samples actions for the active envs (PPO.get_action, PPO.py:81-96), the
           active envs step one by one (CartPole-v1 physics in C, prl_oracle.c: FASTER than the
           reference's per-env gymnasium Python step, so this leg flatters the CPU), every
           transition is appended to per-env Python lists (utils.buffer_append, utils.py:17-36),
           the envs_active mask is updated (utils.py:38-43);
  flatten  utils.buffer_to_target_buffer_transfer's sum(list, []) (utils.py:45-51): O(E * N);
  learn    PPO.learn (PPO.py:122-260): memory stacked to tensors, batch_packer = DataLoader
           minibatches (PPO.py:98-105), policy_old evaluation, compute_gae as the reference's
           Python loop with list.insert(0) (PPO.py:107-120, O(N^2): oracle.gae_python), advantage
           normalisation, k_epochs x unshuffled minibatches of the clipped surrogate + 0.5
           SmoothL1 - 0.01 H, clip_grad_norm_(2.0), AdamW — torch on the CPU.
Each leg is timed on its own, so bench.py can extrapolate the sample to the GPU run's workload
with the measured complexities (rollout and learn ~ N, flatten ~ E * N, GAE ~ N^2).
"""
import os
import time

import numpy as np
import torch
from torch import nn, optim
from torch.utils.data import DataLoader

import oracle as O


def _policy(obs_dim, act_dim):
    def block(i, o):
        return [nn.Linear(i, o, bias=False), nn.GroupNorm(8, 64), nn.SiLU()]
    trunk = nn.Sequential(*block(obs_dim, 64))
    actor = nn.Sequential(*block(64, 64), nn.Linear(64, act_dim), nn.Softmax(-1))
    critic = nn.Sequential(*block(64, 64), nn.Linear(64, 1))
    return trunk, actor, critic


def worker_port(E, trunk, actor, seed=0):
    """One episode per env (AsyncPPO.worker).  Returns per-env lists and the rollout time."""
    env = O.CartPoleOracle(E)
    env.seed(np.arange(E) + seed)
    states = env.reset()
    terminal = np.zeros(E, bool)                      # envs_active (True = terminal)
    buf = [([], [], [], []) for _ in range(E)]
    t0 = time.perf_counter()
    while True:
        idx = np.where(~terminal)[0]
        with torch.no_grad():                         # PPO.get_action on the CPU
            probs = actor(trunk(torch.from_numpy(states)))
            actions = torch.distributions.Categorical(probs).sample().numpy()
        nxt, r, term, trunc = env.step_envs(idx, actions)
        done = term | trunc
        for i, e in enumerate(idx):                   # utils.buffer_append + VecMemory.push
            b = buf[e]
            b[0].append(states[i].astype(np.float32))
            b[1].append(np.float32(actions[i]))
            b[2].append(np.float32(r[i]))
            b[3].append(np.float32(done[i]))
        states = nxt[~done]                           # utils.inactive_states_dropout
        terminal[idx] = done                          # utils.update_active_environments_list
        if np.all(terminal):
            break
    return buf, time.perf_counter() - t0


def flatten_port(buf):
    """utils.buffer_to_target_buffer_transfer: env-major concatenation with sum(list, [])."""
    t0 = time.perf_counter()
    mem = [sum([b[k] for b in buf], []) for k in range(4)]
    return mem, time.perf_counter() - t0


def learn_port(mem, trunk, actor, critic, mb=512, k_epochs=11, gamma=0.995, lam=0.95, lr=1e-3):
    """PPO.learn on the CPU.  Returns (gae_seconds, rest_seconds)."""
    params = list(trunk.parameters()) + list(actor.parameters()) + list(critic.parameters())
    opt = optim.AdamW(params, lr=lr)
    t0 = time.perf_counter()
    S = torch.from_numpy(np.array(mem[0])).float()
    A = torch.from_numpy(np.array(mem[1])).float()
    batches = lambda x: list(DataLoader(x, mb))      # noqa: E731  PPO.batch_packer
    with torch.no_grad():
        lp_old, v_old = [], []
        for s, a in zip(batches(S), batches(A)):
            f = trunk(s)
            lp_old.append(torch.distributions.Categorical(actor(f)).log_prob(a))
            v_old.append(critic(f).squeeze(-1))
        lp_old, v_old = torch.cat(lp_old), torch.cat(v_old)
    R, Dn = np.array(mem[2]), np.array(mem[3])
    V = v_old.numpy()
    t1 = time.perf_counter()
    ret = O.gae_python(R, Dn, V, V[-1], gamma, lam)   # the reference's O(N^2) loop
    t2 = time.perf_counter()
    ret = torch.from_numpy(ret)
    adv = ret - v_old
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    sl1 = nn.SmoothL1Loss()
    data = [batches(x) for x in (S, A, lp_old, adv, ret)]
    for _ in range(k_epochs):
        for s, a, old, ad, rt in zip(*data):
            f = trunk(s)
            d = torch.distributions.Categorical(actor(f))
            lp = d.log_prob(a)
            v = critic(f).squeeze(-1)
            H = d.entropy().mean().detach()
            ratio = torch.exp(torch.clamp(lp - old, -20, 20))
            loss = -torch.min(ratio * ad, torch.clamp(ratio, 0.8, 1.2) * ad) \
                + 0.5 * sl1(v, rt) - 0.01 * H
            opt.zero_grad()
            loss.mean().backward()
            nn.utils.clip_grad_norm_(params, 2.0)
            opt.step()
    return t2 - t1, (t1 - t0) + (time.perf_counter() - t2)


def cpu_iteration(E=4096, mb=512, k_epochs=11, seed=0):
    """One CartPole AsyncPPO iteration (rollout + learn) of the reference's CPU path.  Returns a
    dict: N transitions, seconds per leg, torch threads used, host cores in the affinity mask."""
    torch.manual_seed(0)
    trunk, actor, critic = _policy(4, 2)
    buf, t_roll = worker_port(E, trunk, actor, seed)
    mem, t_flat = flatten_port(buf)
    t_gae, t_learn = learn_port(mem, trunk, actor, critic, mb=mb, k_epochs=k_epochs)
    return {"E": E, "N": len(mem[0]), "rollout_s": t_roll, "flatten_s": t_flat, "gae_s": t_gae,
            "learn_s": t_learn, "threads": torch.get_num_threads(),
            "affinity_cores": len(os.sched_getaffinity(0))}


def extrapolate(rec, E_target, N_target):
    """Seconds for one iteration of E_target envs / N_target transitions, scaling each leg by its
    complexity in the reference: rollout and learn ~ N, flatten ~ E * N, GAE ~ N^2."""
    n = N_target / rec["N"]
    e = E_target / rec["E"]
    return (rec["rollout_s"] * n + rec["flatten_s"] * e * n + rec["gae_s"] * n * n
            + rec["learn_s"] * n)


EXTRAPOLATION_RULE = ("t(E, N) = rollout_s * N/N0 + flatten_s * (E/E0)(N/N0) + gae_s * (N/N0)^2 "
                      "+ learn_s * N/N0 (reference complexities: per-transition rollout and "
                      "update, sum(list, []) flatten O(E N), list.insert(0) GAE O(N^2))")
