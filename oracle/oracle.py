"""CPU ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

The product (parallel-reinforcement-learning_amd/) never imports this module.  It restates the
reference's hot path on the CPU so the HIP path can be checked against it:

  * gymnasium==1.1.1 CartPole-v1 / Pendulum-v1 (+TimeLimit) behind EnvVectorizer
    (AsyncTools/AsyncPPO.py:35-102): resets draw from numpy's PCG64 exactly as gymnasium's
    ``env.reset(seed=s)`` (``np.random.default_rng(s).uniform``), physics in C (prl_oracle.c);
  * the envs_active mask utilities (AsyncTools/utils.py:3-51) in numpy, op for op;
  * PPO.compute_gae (PPO/PPO.py:107-120) sequential float32 loop (C) and the advantage
    normalisation (PPO.py:198-199);
  * the clipped surrogate loss and its gradient (PPO.py:225-249) in float64 numpy;
  * RND.compute_intrinsic_reward (PPO/RND.py:71-94) in float64 numpy.

Pinning: tests/test_oracle.py checks these against golden vectors produced by importing the
reference itself (tests/golden/make_golden.py).  The env physics is pinned against a numpy
restatement of gymnasium's code (gymnasium is not installed here): parity of the physics with
gymnasium proper is documented as "parity unpinned" in DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(HERE, "liboracle.so")
        src = os.path.join(HERE, "prl_oracle.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(so)
        P = ctypes.c_void_p
        i64, u64, i32, u32, f32, f64 = (ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32,
                                        ctypes.c_uint32, ctypes.c_float, ctypes.c_double)
        sig = {
            "or_sin": (f64, [f64]), "or_cos": (f64, [f64]),
            "or_sin_cos_array": (None, [P, i64, P, P]),
            "or_philox": (None, [P, u32, u32, P]),
            "or_sample_categorical": (ctypes.c_int, [P, ctypes.c_int, u64, u32, u32]),
            "or_sample_normal": (f32, [u64, u32, u32, u32]),
            "or_sample_categorical_batch": (None, [P, i64, ctypes.c_int, u64, P, P]),
            "or_cartpole_step1": (ctypes.c_int, [P, ctypes.c_int]),
            "or_cartpole_step": (None, [P, P, i64, P]),
            "or_pendulum_step1": (f64, [P, f32]),
            "or_pendulum_step": (None, [P, P, i64, P]),
            "or_synth_episode_len": (u32, [u64]),
            "or_synth_obs": (None, [u64, u32, P]),
            "or_gae": (None, [P, P, P, f32, i64, f64, f64, P]),
            "or_cartpole_rollout": (i64, [i64, P, u64, f32, i32, P, P, P, P, P, P, P, P, P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    assert a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.c_void_p)


# ------------------------------------------------------------------------------------ trig
def sin_cos(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float64)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib().or_sin_cos_array(_p(x), x.size, _p(s), _p(c))
    return s, c


# ------------------------------------------------------------------------------------ RNG
def pcg64_state_words(seed: int) -> np.ndarray:
    """numpy's PCG64(SeedSequence(seed)) state as {state_hi, state_lo, inc_hi, inc_lo}."""
    st = np.random.PCG64(seed).state["state"]
    m = (1 << 64) - 1
    return np.array([st["state"] >> 64, st["state"] & m, st["inc"] >> 64, st["inc"] & m],
                    dtype=np.uint64)


def sample_categorical(probs: np.ndarray, seed: int, t: np.ndarray) -> np.ndarray:
    probs = np.ascontiguousarray(probs, dtype=np.float32)
    E, A = probs.shape
    t = np.ascontiguousarray(t, dtype=np.int32)
    out = np.empty(E, dtype=np.int32)
    lib().or_sample_categorical_batch(_p(probs), E, A, seed, _p(t), _p(out))
    return out


def sample_normal(seed: int, e: int, t: int, j: int) -> float:
    return float(lib().or_sample_normal(seed, e, t, j))


# ------------------------------------------------------------------------------------ envs
class CartPoleOracle:
    """gymnasium CartPole-v1 + TimeLimit(500), E copies (AsyncPPO.py:39 deep copies)."""
    D, A, TMAX, discrete = 4, 2, 500, True

    def __init__(self, E: int):
        self.E = E
        self.state = np.zeros((E, 4), np.float64)
        self.t = np.zeros(E, np.int32)
        self.rngs = [None] * E

    def seed(self, seeds):
        self.rngs = [np.random.default_rng(int(s)) for s in seeds]

    def reset(self, mask=None):
        for e in range(self.E):
            if mask is None or mask[e]:
                self.state[e] = self.rngs[e].uniform(low=-0.05, high=0.05, size=(4,))
                self.t[e] = 0
        return self.obs()

    def obs(self):
        return self.state.astype(np.float32)

    def step_envs(self, idx: np.ndarray, actions: np.ndarray):
        """Step envs idx (ascending) with actions; returns compacted obs, r, term, trunc."""
        idx = np.asarray(idx, np.int64)
        s = np.ascontiguousarray(self.state[idx])
        a = np.ascontiguousarray(np.asarray(actions).reshape(-1), dtype=np.int64)
        term = np.zeros(len(idx), np.uint8)
        lib().or_cartpole_step(_p(s), _p(a), len(idx), _p(term))
        self.state[idx] = s
        self.t[idx] += 1
        trunc = self.t[idx] >= self.TMAX
        return s.astype(np.float32), np.ones(len(idx)), term.astype(bool), trunc


class PendulumOracle:
    """gymnasium Pendulum-v1 (g=10.0) + TimeLimit(200)."""
    D, A, TMAX, discrete = 3, 1, 200, False

    def __init__(self, E: int):
        self.E = E
        self.state = np.zeros((E, 2), np.float64)
        self.t = np.zeros(E, np.int32)
        self.rngs = [None] * E

    def seed(self, seeds):
        self.rngs = [np.random.default_rng(int(s)) for s in seeds]

    def reset(self, mask=None):
        high = np.array([np.pi, 1.0])
        for e in range(self.E):
            if mask is None or mask[e]:
                self.state[e] = self.rngs[e].uniform(low=-high, high=high)
                self.t[e] = 0
        return self.obs()

    def obs(self, state=None):
        st = self.state if state is None else state
        s, c = sin_cos(st[:, 0])
        return np.stack([c, s, st[:, 1]], axis=1).astype(np.float32)

    def step_envs(self, idx, actions):
        idx = np.asarray(idx, np.int64)
        s = np.ascontiguousarray(self.state[idx])
        u = np.ascontiguousarray(np.asarray(actions, np.float32).reshape(len(idx), -1)[:, 0])
        r = np.zeros(len(idx), np.float64)
        lib().or_pendulum_step(_p(s), _p(u), len(idx), _p(r))
        self.state[idx] = s
        self.t[idx] += 1
        trunc = self.t[idx] >= self.TMAX
        return self.obs(s), r, np.zeros(len(idx), bool), trunc


class SynthOracle:
    """Synthetic Humanoid-v5-shaped env (obs 348, act 17); semantics in DESIGN.md."""
    D, A, TMAX, discrete = 348, 17, 1000, False

    def __init__(self, E: int):
        self.E = E
        self.key = np.zeros(E, np.uint64)
        self.L = np.zeros(E, np.int64)
        self.t = np.zeros(E, np.int32)
        self.bitgens = [None] * E

    def seed(self, seeds):
        self.bitgens = [np.random.PCG64(int(s)) for s in seeds]

    def _obs1(self, key, t):
        o = np.empty(348, np.float32)
        lib().or_synth_obs(int(key), int(t), _p(o))
        return o

    def reset(self, mask=None):
        out = np.zeros((self.E, 348), np.float32)
        for e in range(self.E):
            if mask is None or mask[e]:
                k = int(self.bitgens[e].random_raw())
                self.key[e] = k
                self.L[e] = lib().or_synth_episode_len(k)
                self.t[e] = 0
            out[e] = self._obs1(self.key[e], self.t[e])
        return out

    def step_envs(self, idx, actions):
        idx = np.asarray(idx, np.int64)
        acts = np.asarray(actions, np.float32).reshape(len(idx), 17)
        obs = np.zeros((len(idx), 348), np.float32)
        r = np.zeros(len(idx), np.float64)
        term = np.zeros(len(idx), bool)
        for i, e in enumerate(idx):
            self.t[e] += 1
            obs[i] = self._obs1(self.key[e], self.t[e])
            acc = np.float32(0)
            for j in range(17):
                acc = np.float32(acc + np.float32(acts[i, j] * acts[i, j]))
            r[i] = float(np.float32(np.float32(1.0) - np.float32(0.01) * acc))
            term[i] = self.t[e] >= self.L[e]
        trunc = self.t[idx] >= self.TMAX
        return obs, r, term, trunc


ENV_ORACLES = {"CartPole-v1": CartPoleOracle, "Pendulum-v1": PendulumOracle,
               "SyntheticHumanoid-v0": SynthOracle}


# ------------------------------------------------------------------------------------ utils.py
def indexes_of_active_environments(num_envs, is_env_terminal):          # utils.py:3-4
    return np.arange(num_envs)[~is_env_terminal]


def number_of_active_environments(is_env_terminal):                      # utils.py:6-7
    return np.sum(~is_env_terminal)


def inactive_states_dropout(states, dones):                              # utils.py:14-15
    return states[~dones]


def update_active_environments_list(is_env_terminal, dones):             # utils.py:38-43
    m = is_env_terminal.copy()
    m[np.where(~m)[0]] = dones
    return m


def flatten_env_major(episodes):                                         # utils.py:45-51
    """episodes: list over envs of lists of per-step items -> env-major concatenation."""
    return [x for ep in episodes for x in ep]


class EnvVectorizerOracle:
    """EnvVectorizer semantics (AsyncPPO.py:35-102) over an env oracle."""

    def __init__(self, env_oracle):
        self.env = env_oracle
        self.envs_active = np.zeros(env_oracle.E, bool)  # True = terminal

    def reset(self):
        obs = self.env.reset()
        self.envs_active = np.zeros(self.env.E, bool)
        return obs

    def step(self, actions):
        idx = np.arange(self.env.E)[~self.envs_active]
        return self.env.step_envs(idx, actions)


def worker_oracle(env_oracle, action_fn, max_steps=10_000):
    """AsyncPPO.worker (AsyncPPO.py:117-146) with a deterministic action function
    action_fn(states_compact, active_idx, t) -> actions.  Returns the env-major flattened memory
    (states, actions, rewards, dones as float32 arrays), the per-step masks and the scores."""
    vec = EnvVectorizerOracle(env_oracle)
    states = vec.reset()
    E = env_oracle.E
    buf = [[] for _ in range(E)]
    masks = []
    step_score, reward_score = 0, 0.0
    for t in range(max_steps):
        idx = np.arange(E)[~vec.envs_active]
        actions = action_fn(states, idx, t)
        nxt, r, d, tr, = vec.step(actions)[:4]
        done = d | tr
        for i, e in enumerate(idx):       # buffer_append (utils.py:17-36)
            buf[e].append((states[i].astype(np.float32), np.asarray(actions[i]).astype(np.float32),
                           np.float32(r[i]), np.float32(done[i])))
        reward_score += float(np.sum(r))
        step_score += int(np.sum(~vec.envs_active))
        states = nxt[~done]
        vec.envs_active = update_active_environments_list(vec.envs_active, done)
        masks.append(vec.envs_active.copy())
        if np.all(vec.envs_active):
            break
    flat = flatten_env_major(buf)
    S = np.stack([x[0] for x in flat]).astype(np.float32)
    A = np.stack([x[1] for x in flat]).astype(np.float32)
    R = np.array([x[2] for x in flat], np.float32)
    Dn = np.array([x[3] for x in flat], np.float32)
    return dict(S=S, A=A, R=R, D=Dn, masks=np.array(masks), lengths=np.array([len(b) for b in buf]),
                step_score=step_score, reward_score=reward_score)


# ------------------------------------------------------------------------------------ learn()
def gae(r, d, V, next_value, gamma, lam):
    """PPO.compute_gae (PPO.py:107-120), float32 sequential loop in C."""
    r = np.ascontiguousarray(r, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    V = np.ascontiguousarray(V, np.float32)
    out = np.empty_like(V)
    lib().or_gae(_p(r), _p(d), _p(V), float(np.float32(next_value)), len(V), float(gamma),
                 float(lam), _p(out))
    return out


def gae_python(rewards, dones, state_values, next_value, gamma, lam):
    """Pure-Python restatement of the same loop (small N only) — pins or_gae's op order."""
    gae_ = 0
    out = []
    for step in reversed(range(len(state_values))):
        delta = rewards[step] + gamma * next_value * (1 - dones[step]) - state_values[step]
        gae_ = delta + gamma * lam * (1 - dones[step]) * gae_
        out.insert(0, gae_ + state_values[step])
        next_value = state_values[step]
    return np.array(out, np.float32)


def adv_normalize(ret, V, eps=1e-8):
    """PPO.py:198-199 with float64 statistics (the reference reduces in float32)."""
    adv = (ret.astype(np.float32) - V.astype(np.float32)).astype(np.float32)
    a64 = adv.astype(np.float64)
    mean = a64.mean()
    std = a64.std(ddof=1) if len(a64) > 1 else np.nan
    return ((adv - np.float32(mean)) / (np.float32(std) + np.float32(eps))).astype(np.float32), adv


def surrogate(logp, old_logp, adv, V, ret, entropy, clip=0.2, vf_coef=0.5, ent_coef=0.01):
    """PPO.py:225-249 loss and d(loss)/d(logp), d(loss)/d(V) with torch's gradient rules."""
    logp, old_logp, adv, V, ret = (np.asarray(x, np.float64) for x in (logp, old_logp, adv, V, ret))
    mb = len(logp)
    diff = logp - old_logp
    cl = np.clip(diff, -20, 20)
    ratio = np.exp(cl)
    s1 = ratio * adv
    rc = np.clip(ratio, 1 - clip, 1 + clip)
    s2 = rc * adv
    m = np.minimum(s1, s2)
    x = V - ret
    ax = np.abs(x)
    sl1 = np.where(ax < 1, 0.5 * x * x, ax - 0.5)
    loss = np.mean(-m) + vf_coef * np.mean(sl1) - ent_coef * float(entropy)
    w1 = np.where(s1 < s2, 1.0, np.where(s2 < s1, 0.0, 0.5))
    w2 = 1.0 - w1
    in_clip = ((ratio >= 1 - clip) & (ratio <= 1 + clip)).astype(np.float64)
    in_20 = ((diff >= -20) & (diff <= 20)).astype(np.float64)
    dlogp = -(1.0 / mb) * (w1 * adv + w2 * adv * in_clip) * ratio * in_20
    dV = vf_coef * (1.0 / mb) * np.clip(x, -1, 1)
    return loss, dlogp, dV


def rnd_forward(x, tnet, pnet, beta):
    """RND.compute_intrinsic_reward (RND.py:71-94) in float64.  nets: dicts of numpy arrays
    with keys w1 [64,D], b1, gw, gb, w2 [D,64], b2."""
    x = np.asarray(x, np.float64)

    def net(p):
        h = x @ p["w1"].T.astype(np.float64) + p["b1"]
        g = h.reshape(len(x), 8, 8)
        mu = g.mean(-1, keepdims=True)
        var = g.var(-1, keepdims=True)
        h = ((g - mu) / np.sqrt(var + 1e-5)).reshape(len(x), 64) * p["gw"] + p["gb"]
        h = h / (1 + np.exp(-h))
        return h @ p["w2"].T.astype(np.float64) + p["b2"]

    return beta * np.linalg.norm(net(pnet) - net(tnet), axis=-1)
