"""Env registry for the batched HIP environments.

The reference hands EnvVectorizer a gymnasium env object (train.py:8 `gym.make('CartPole-v1')`,
AsyncTools/AsyncPPO.py:36) and deep-copies it num_envs times (:39).  Here the envs live on the GPU
as one structure-of-arrays batch, so the vectorizer needs only the env's identity: `make(id)`
returns a light spec; a gymnasium env object (if gymnasium is installed) or a plain id string
is accepted too and resolved through its `spec.id`.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import prl_native


@dataclass
class Discrete:
    n: int
    shape: tuple = ()


@dataclass
class Box:
    shape: tuple
    low: float = float("-inf")
    high: float = float("inf")


@dataclass
class EnvSpec:
    id: str
    kind: int
    obs_dim: int
    act_dim: int
    phys_dim: int
    max_episode_steps: int
    discrete: bool
    observation_space: Box = field(init=False)
    action_space: object = field(init=False)

    def __post_init__(self):
        self.observation_space = Box(shape=(self.obs_dim,))
        self.action_space = Discrete(self.act_dim) if self.discrete else Box(
            shape=(self.act_dim,), low=-2.0 if self.id == "Pendulum-v1" else -1.0,
            high=2.0 if self.id == "Pendulum-v1" else 1.0)

    @property
    def spec(self):  # gymnasium-style `env.spec.id`
        return self

    def close(self):
        pass


REGISTRY = tuple(prl_native.ENV_KINDS)


def make(env_id: str) -> EnvSpec:
    """gymnasium.make() stand-in for the envs that have HIP kernels."""
    if env_id not in prl_native.ENV_KINDS:
        raise ValueError(f"unknown env id {env_id!r}; available: {', '.join(REGISTRY)}")
    kind = prl_native.ENV_KINDS[env_id]
    d = prl_native.env_dims(kind)
    return EnvSpec(env_id, kind, d["obs_dim"], d["act_dim"], d["phys_dim"],
                   d["max_episode_steps"], d["discrete"])


def resolve(env) -> EnvSpec:
    if isinstance(env, EnvSpec):
        return env
    if isinstance(env, str):
        return make(env)
    spec = getattr(env, "spec", None)
    env_id = getattr(spec, "id", None)
    if env_id is None:
        unwrapped = getattr(env, "unwrapped", env)
        env_id = {"CartPoleEnv": "CartPole-v1", "PendulumEnv": "Pendulum-v1"}.get(
            type(unwrapped).__name__)
    if env_id is None:
        raise TypeError(f"cannot map {type(env).__name__} to a HIP env; use AsyncTools.envs.make()")
    return make(env_id)
