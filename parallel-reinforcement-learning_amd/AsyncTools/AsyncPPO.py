"""AsyncPPO / EnvVectorizer / VecMemory — drop-in for the reference's AsyncTools/AsyncPPO.py.

Reference semantics kept (AsyncPPO.py:11-165):
  * EnvVectorizer holds num_envs envs; `envs_active[e]` is True when env e is TERMINAL; reset()
    resets every env and clears the mask; step(actions) steps only the non-terminal envs in
    ascending index order, the i-th action going to the i-th active env, and returns
    obs / rewards / dones / truncates / infos compacted to the active envs.
  * AsyncPPO.worker() runs ONE episode per env until every env is terminal, records
    (pre-step state, action, reward, done|truncated) per env and appends the rollout to
    ppo.memory env-major; run() alternates worker() and ppo.learn() until `steps` transitions.

MI355X design: the envs are one structure-of-arrays batch in HBM stepped by HIP kernels
(libprl_hip.so).  With a PPO from this package, worker() is DEVICE-RESIDENT: per vector step,
the policy MLP (PyTorch) reads the contiguous time-major slice traj_obs[t], and one fused kernel
(prl_rollout_step) samples the actions, steps the physics, writes the transition, updates the
mask and the score counters.  No per-step host<->device copy: the host only polls a pinned
"envs still active" counter a few steps behind, and ends the loop when it reaches zero.  The
finished rollout is flattened env-major on the device (prl_exclusive_scan_i32 +
prl_flatten_env_major) and handed to ppo.memory as device tensors.  Any other duck-typed `ppo`
(get_action/memory/learn) runs through the compat path (numpy API, same HIP env kernels).
"""
from __future__ import annotations

import os
import warnings

import numpy as np
import torch
import torch.distributed as tdist
from tqdm import tqdm

import AsyncTools.utils as utils
import prl_native
from AsyncTools.envs import resolve


class VecMemory:  # AsyncPPO.py:11-33
    def __init__(self, num_envs: int):
        self.states = [[] for _ in range(num_envs)]
        self.actions = [[] for _ in range(num_envs)]
        self.rewards = [[] for _ in range(num_envs)]
        self.dones = [[] for _ in range(num_envs)]

    def push(self, idx: int, state, action, reward, done):
        self.states[idx].append(np.asarray(state).astype(np.float32))
        self.actions[idx].append(np.asarray(action).astype(np.float32))
        self.rewards[idx].append(np.asarray(reward).astype(np.float32))
        self.dones[idx].append(np.asarray(done).astype(np.float32))

    def clear(self):
        for i in range(len(self.states)):
            del self.states[i][:]
            del self.actions[i][:]
            del self.rewards[i][:]
            del self.dones[i][:]


def _rank_world():
    if tdist.is_available() and tdist.is_initialized():
        return tdist.get_rank(), tdist.get_world_size()
    return 0, 1


class EnvVectorizer:  # AsyncPPO.py:35-102
    """num_envs copies of one env as a device batch.  seed: int -> env i is seeded with
    seed + i (+ rank * num_envs under torch.distributed), like gymnasium's reset(seed=...);
    None -> fresh OS entropy, like an unseeded gymnasium env."""

    def __init__(self, env, num_envs: int = 1, seed=None, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("EnvVectorizer runs on the GPU through libprl_hip.so; no GPU visible")
        self.spec = resolve(env)
        self.num_envs = num_envs
        self.action_space = self.spec.action_space
        self.observation_space = self.spec.observation_space
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        E, dev = num_envs, self.device
        self.phys = torch.zeros(E, self.spec.phys_dim, dtype=torch.float64, device=dev)
        self.rng = torch.zeros(E, 4, dtype=torch.int64, device=dev)
        self.t_elapsed = torch.zeros(E, dtype=torch.int32, device=dev)
        self.terminal = torch.zeros(E, dtype=torch.uint8, device=dev)
        self.obs = torch.zeros(E, self.spec.obs_dim, dtype=torch.float32, device=dev)
        self._idx = torch.zeros(E, dtype=torch.int64, device=dev)
        self._cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        self.seed(seed)

    # the reference exposes the deep-copied env list (AsyncPPO.py:39)
    @property
    def envs(self):
        return [self.spec] * self.num_envs

    def seed(self, seed=None):
        rank, _ = _rank_world()
        if seed is None:
            seeds = np.frombuffer(os.urandom(8 * self.num_envs), dtype=np.uint64) >> np.uint64(1)
        else:
            seeds = np.arange(self.num_envs, dtype=np.uint64) + np.uint64(seed) + np.uint64(
                rank * self.num_envs)
        s = torch.from_numpy(seeds.astype(np.int64)).to(self.device)
        prl_native.pcg64_seed(s, self.rng)

    @property
    def envs_active(self):
        return self.terminal.cpu().numpy().astype(bool)

    @envs_active.setter
    def envs_active(self, mask):
        m = torch.as_tensor(np.asarray(mask, dtype=np.uint8)).to(self.device)
        self.terminal.copy_(m)

    def reset_device(self, obs_out=None):
        """Reset every env on the device; obs written to obs_out ([E, D] view) or self.obs."""
        out = self.obs if obs_out is None else obs_out
        prl_native.env_reset(self.spec.kind, self.phys, self.rng, self.t_elapsed, self.terminal,
                             out, out.stride(0))
        return out

    def reset(self, seed=None):
        if seed is not None:
            self.seed(seed)
        obs = self.reset_device()
        return obs.cpu().numpy(), [{} for _ in range(self.num_envs)]

    def step(self, actions):
        prl_native.active_indices(self.terminal, self._idx, self._cnt)
        n = int(self._cnt.item())
        if self.spec.discrete:
            act = torch.as_tensor(np.asarray(actions)).to(self.device, torch.int64).reshape(-1)
        else:
            act = torch.as_tensor(np.asarray(actions, dtype=np.float32)).to(self.device)
            act = act.reshape(-1, self.spec.act_dim)
        act = act.contiguous()
        if act.shape[0] < n:
            raise IndexError(f"{act.shape[0]} actions for {n} active environments")
        obs = torch.empty(n, self.spec.obs_dim, dtype=torch.float32, device=self.device)
        rew = torch.empty(n, dtype=torch.float64, device=self.device)
        term = torch.empty(n, dtype=torch.uint8, device=self.device)
        trunc = torch.empty(n, dtype=torch.uint8, device=self.device)
        prl_native.env_step_compact(self.spec.kind, self.phys, self.t_elapsed, self._idx, n, act,
                                    obs, rew, term, trunc)
        infos = np.array([{} for _ in range(n)], dtype=object)
        return (obs.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy().astype(bool),
                trunc.cpu().numpy().astype(bool), infos)

    def close(self):
        pass


class DeviceTrajectory:
    """Time-major rollout buffers in HBM (one row of E envs per vector step)."""

    def __init__(self, E, spec, device):
        T, D = spec.max_episode_steps, spec.obs_dim
        adim = 1 if spec.discrete else spec.act_dim
        self.T, self.E, self.adim = T, E, adim
        self.obs = torch.empty(T + 1, E, D, dtype=torch.float32, device=device)
        self.act = torch.empty(T, E, adim, dtype=torch.float32, device=device)
        self.rew = torch.empty(T, E, dtype=torch.float32, device=device)
        self.done = torch.empty(T, E, dtype=torch.uint8, device=device)
        self.ep_len = torch.zeros(E, dtype=torch.int32, device=device)
        self.active_after = torch.zeros(T, dtype=torch.int32, device=device)
        self.reward_sum = torch.zeros(1, dtype=torch.float64, device=device)
        self.offsets = torch.zeros(E + 1, dtype=torch.int64, device=device)
        self.pinned = torch.zeros(T, dtype=torch.int32, pin_memory=True)


def sample_key(seed, rank=None):
    """The Philox key of the in-kernel action sampling.  Under torch.distributed the rank is
    mixed in (as EnvVectorizer.seed offsets the env seeds by rank * num_envs), so ranks given the
    same seed draw independent exploration noise; rank 0 keeps the single-process key."""
    if seed is None:
        return int.from_bytes(os.urandom(8), "little")
    if rank is None:
        rank = _rank_world()[0]
    key = (int(seed) * 0x9E3779B97F4A7C15 + 0x1234567) & (2**64 - 1)
    return (key + rank * 0xBF58476D1CE4E5B9) & (2**64 - 1)


class AsyncPPO:  # AsyncPPO.py:104-165
    def __init__(self, env, ppo: object, num_envs: int = 32, steps: int = 100000, seed=None,
                 poll_lag: int = 4):
        self.env = EnvVectorizer(env, num_envs, seed=seed)
        self.num_envs = num_envs
        self.steps = steps
        self.ppo = ppo
        self.step_score = np.array(0, dtype=np.int32)
        self.reward_score = np.array(0.0, dtype=np.float32)
        self.buffer = VecMemory(num_envs)
        self.poll_lag = poll_lag
        self.sample_seed = sample_key(seed)
        self._rollouts = 0
        self._evals = 0
        self._warm = False      # one eager rollout first (warm-up before graph capture)
        self._graph = None
        self._traj = None
        self.last_vector_steps = 0

    # ------------------------------------------------------------------ worker
    def worker(self):
        if hasattr(self.ppo, "dist_params"):
            return self._device_worker()
        return self._compat_worker()

    def _compat_worker(self):
        """The reference's worker loop verbatim over the numpy API (AsyncPPO.py:117-146)."""
        states = self.env.reset()[0]
        while True:
            actions = self.ppo.get_action(torch.from_numpy(states))
            next_states, rewards, dones, truncates, _ = self.env.step(actions)
            utils.buffer_append(self.buffer, states, actions, rewards, dones | truncates,
                                self.env.envs_active, self.num_envs)
            self.reward_score += np.sum(rewards)
            self.step_score += np.sum(~self.env.envs_active)
            states = utils.inactive_states_dropout(next_states, dones | truncates)
            self.env.envs_active = utils.update_active_environments_list(self.env.envs_active,
                                                                         dones | truncates)
            if np.all(self.env.envs_active):
                utils.buffer_to_target_buffer_transfer(self.buffer, self.ppo.memory)
                break

    def _device_worker(self):
        seed = (self.sample_seed + self._rollouts * 0xD1B54A32D192ED03) & (2**64 - 1)
        self._rollouts += 1
        k = self._device_rollout(seed)
        return self._device_collect(k)

    def _device_rollout(self, seed):
        """One episode per env on the device (fused rollout step kernel per vector step, policy
        on traj_obs[t]); returns the index of the last vector step taken.  From the second
        rollout of this runner on, one vector step (policy forward + rollout step kernel) is a
        captured HIP graph replayed per step (PRL_ROLLOUT_GRAPH=0: eager launches)."""
        env, spec = self.env, self.env.spec
        E = self.num_envs
        if self._traj is None:
            self._traj = DeviceTrajectory(E, spec, env.device)
        tr = self._traj
        scaling = float(getattr(self.ppo, "action_scaling", None) or 1.0)
        env.reset_device(tr.obs[0])
        tr.active_after.zero_()
        tr.reward_sum.zero_()
        k = self._fused_rollout(seed, scaling)
        if k is not None:
            self._warm = True
            self.last_vector_steps = k + 1
            return k
        stream = torch.cuda.current_stream()
        graph = None
        if (self._warm and not getattr(self, "_graph_failed", False)
                and os.environ.get("PRL_ROLLOUT_GRAPH", "1") != "0"):
            graph = self._capture_step(seed, scaling)
        events = []
        checked = -1           # last step whose counter has been read
        finished = False
        k = 0
        with torch.no_grad():
            for k in range(tr.T):
                if graph is not None:
                    graph.replay()
                else:
                    self._vector_step(k, tr.obs[k], seed, scaling, tr.active_after)
                tr.pinned[k:k + 1].copy_(tr.active_after[k:k + 1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                events.append(ev)
                # poll completed steps without blocking; block only when too far ahead
                while checked < k and (k - checked > self.poll_lag or events[checked + 1].query()):
                    events[checked + 1].synchronize()
                    checked += 1
                    if int(tr.pinned[checked]) == 0:
                        finished = True
                        break
                if finished:
                    break
            if (not self._warm and not getattr(self, "_graph_failed", False)
                    and os.environ.get("PRL_ROLLOUT_GRAPH", "1") != "0"):
                # every env is terminal now: capture and replay the step once (a no-op for
                # terminal envs) so the first capture's one-time cost (~85 ms at C2) falls in
                # this warm-up rollout, not in the first graphed one
                g = self._capture_step(seed, scaling)
                if g is not None:
                    g.replay()
        self._warm = True
        self.last_vector_steps = k + 1
        return k

    def _fused_rollout(self, seed, scaling):
        """The whole rollout as ONE persistent launch (prl_wide_rollout: each wave steps 16 envs to
        the end of their episodes with policy_old's actor in LDS) where it applies — the wide
        continuous nets on the synthetic env (C5); PRL_WIDE_ROLLOUT=0 keeps the per-step path.
        Returns the index of the last vector step (max episode length - 1), or None."""
        if os.environ.get("PRL_WIDE_ROLLOUT", "1") == "0":
            return None
        params_fn = getattr(self.ppo, "rollout_params", None)
        spec, env, tr = self.env.spec, self.env, self._traj
        if params_fn is None or not prl_native.wide_rollout_supported(
                spec.kind, spec.obs_dim, spec.act_dim, spec.discrete):
            return None
        with torch.no_grad():
            flat = params_fn(tr.obs[0])
        if flat is None:
            return None
        prl_native.wide_rollout(spec.kind, flat, spec.obs_dim, spec.act_dim, spec.discrete,
                                env.phys, env.t_elapsed, env.terminal, scaling, seed, tr.T,
                                tr.obs, tr.act, tr.rew, tr.done, tr.ep_len, tr.active_after,
                                tr.reward_sum)
        return max(int(tr.ep_len.max().item()) - 1, 0)

    def _vector_step(self, k, obs, seed, scaling, active_after):
        """Policy forward on this step's observations + the fused rollout step kernel."""
        self._step_kernel(k, self.ppo.dist_params(obs), seed, scaling, active_after)

    def _step_kernel(self, k, dist, seed, scaling, active_after):
        """The fused rollout step kernel on this step's distribution rows (k: the step index, an
        int, or a device int64 [1] tensor for the captured step)."""
        spec, env, tr = self.env.spec, self.env, self._traj
        if dist.dtype != torch.float32 or not dist.is_contiguous():
            dist = dist.float().contiguous()
        step = prl_native.rollout_step_at if isinstance(k, torch.Tensor) else prl_native.rollout_step
        step(spec.kind, k, env.phys, env.t_elapsed, env.terminal, dist, scaling, seed, tr.T,
             tr.obs, tr.act, tr.rew, tr.done, tr.ep_len, active_after, tr.reward_sum)

    def _capture_step(self, seed, scaling):
        """One vector step as a HIP graph for this rollout's sampling key: the step index k lives
        on the device (k_dev, advanced by the graph), the policy reads traj_obs[k_dev] (in place
        for the wide nets, prl_ppo_wide_dist_at; through a gather otherwise), the step kernel
        counts the still-active envs into active_after[k_dev] and advances k_dev itself
        (prl_rollout_step_at; the graph is the policy's kernels + one step kernel).
        PRL_ROLLOUT_STEP_AT=0 keeps round 3's form: the count goes to a scalar the graph copies
        to active_after[k_dev], then an increment node.  Same per-row arithmetic as the eager
        step, so the same bits.  None if capture fails (eager then)."""
        tr, E, D = self._traj, self.num_envs, self.env.spec.obs_dim
        dev = tr.obs.device
        if getattr(self, "_k_dev", None) is None:
            self._k_dev = torch.zeros(2, dtype=torch.int64, device=dev)   # {k, arrivals}
            self._active_now = torch.zeros(1, dtype=torch.int32, device=dev)
        k_dev, now = self._k_dev, self._active_now
        k1 = k_dev[:1]
        self._graph = None
        k_dev.zero_()
        g = torch.cuda.CUDAGraph()
        try:
            # thread_local: other threads' HIP calls (e.g. the nccl process group's watchdog
            # querying its events on data-parallel ranks) must not invalidate this capture
            # wide nets: the distribution kernel reads traj_obs[k_dev] in place (no per-step
            # copy of the E x D rows; policy_old's flat parameters gathered once per rollout)
            at = (getattr(self.ppo, "dist_params_at", None)
                  if os.environ.get("PRL_ROLLOUT_DIST_AT", "1") != "0" else None)
            if at is not None:
                with torch.no_grad():
                    self.ppo.refresh_dist_params(tr.obs[0])
            # the step kernel adds its still-active count to active_after[k_dev] (zeroed at
            # rollout start) and its last block advances k_dev: no scalar fill, index copy or
            # increment node (graphed == eager: test_graphed_rollout_equals_eager_rollout)
            with torch.no_grad(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                dist = at(tr.obs, k1, E) if at is not None else None
                if dist is None:
                    obs = tr.obs.index_select(0, k1).view(E, D)
                    dist = self.ppo.dist_params(obs)
                if os.environ.get("PRL_ROLLOUT_STEP_AT", "1") != "0":
                    self._step_kernel(k_dev, dist, seed, scaling, tr.active_after)
                else:   # the count goes to a scalar the graph copies to active_after[k_dev]
                    now.zero_()
                    self._step_kernel(0, dist, seed, scaling, now)
                    tr.active_after.index_copy_(0, k1, now)
                    k1.add_(1)
        except RuntimeError as e:   # e.g. a host sync inside a duck-typed policy
            warnings.warn(f"rollout step not capturable ({e}); eager launches")
            self._graph_failed = True
            return None
        self._graph = g
        return g

    def _device_collect(self, k):
        env, spec, tr = self.env, self.env.spec, self._traj
        E = self.num_envs
        # env-major flatten straight into learn()'s input tensors
        prl_native.exclusive_scan_i32(tr.ep_len, tr.offsets)
        N = int(tr.offsets[E].item())
        D = spec.obs_dim
        S = torch.empty(N, D, dtype=torch.float32, device=env.device)
        A = torch.empty(N, tr.adim, dtype=torch.float32, device=env.device)
        R = torch.empty(N, dtype=torch.float32, device=env.device)
        Dn = torch.empty(N, dtype=torch.float32, device=env.device)
        prl_native.flatten_env_major(tr.offsets, N, tr.obs, tr.act, tr.rew, tr.done, S, A, R, Dn)
        self.ppo.memory.push_device(S, A[:, 0] if spec.discrete else A, R, Dn)
        self.step_score = self.step_score + N
        self.reward_score = self.reward_score + float(tr.reward_sum.item())
        return N

    # ------------------------------------------------------------------ evaluation
    def evaluate(self):
        """Test.py:19-35 without rendering, batched: one episode per env with the current
        policy (the duck-typed ppo's dist_params, i.e. policy_old as in get_action), nothing
        pushed to ppo.memory and the score counters untouched.  Returns (episode returns f64
        [num_envs], episode lengths int [num_envs]) — Test.py's `reward_per_episode` and step
        count of each env's episode.  Sampling keys come from a stream of their own, so
        evaluating does not change the keys of later training rollouts."""
        if not hasattr(self.ppo, "dist_params"):
            raise RuntimeError("evaluate() needs the device policy path (ppo.dist_params)")
        seed = (self.sample_seed ^ 0x5851F42D4C957F2D) + self._evals * 0xD1B54A32D192ED03
        self._evals += 1
        k = self._device_rollout(seed & (2**64 - 1))
        tr = self._traj
        T = k + 1
        live = (torch.arange(T, device=tr.ep_len.device)[:, None] < tr.ep_len[None, :])
        returns = torch.where(live, tr.rew[:T].double(), torch.zeros((), dtype=torch.float64,
                                                                     device=live.device))
        return returns.sum(0).cpu().numpy(), tr.ep_len.cpu().numpy().astype(np.int64)

    # ------------------------------------------------------------------ run
    def run(self):  # AsyncPPO.py:148-165
        rank, _ = _rank_world()
        pbar = tqdm(total=self.steps, unit="step", disable=rank != 0)
        while pbar.n < self.steps:
            self.step_score = 0
            self.reward_score = 0
            self.worker()
            mean_reward = self.reward_score / self.num_envs
            pbar.update(min(pbar.total - pbar.n, int(self.step_score)))
            pbar.set_description(f"Mean reward {float(mean_reward): .1f}")
            self.ppo.learn()
        pbar.close()
        self.env.close()
