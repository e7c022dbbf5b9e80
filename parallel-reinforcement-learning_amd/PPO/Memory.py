"""Rollout memory — drop-in for the reference's PPO/Memory.py:7-30.

The reference keeps four Python lists of float32 numpy arrays and PPO.learn() stacks ALL of
them (PPO.py:127-128).  Here the same four fields exist for host-side `push()` (compat path),
but the device-resident worker hands over whole rollouts as device tensors
(`push_device`, env-major rows straight out of prl_flatten_env_major), so learn() never touches
per-transition Python objects.  `len(memory)` / `len(memory.states)` count both.
"""
from __future__ import annotations

import numpy as np
import torch


class _Field(list):
    """A list (host transitions) that also counts the rows held in device segments."""

    def __init__(self, owner, idx):
        super().__init__()
        self._owner = owner
        self._idx = idx

    def __len__(self):
        return list.__len__(self) + self._owner._device_rows()

    def host_len(self):
        return list.__len__(self)

    def __iadd__(self, other):
        self.extend(other)
        return self


class Memory:
    def __init__(self):
        self._segments = []  # [(S [n,D], A [n] or [n,A], R [n], Dn [n]) float32 device tensors]
        self.states = _Field(self, 0)
        self.actions = _Field(self, 1)
        self.rewards = _Field(self, 2)
        self.dones = _Field(self, 3)

    def _device_rows(self):
        return sum(int(s[0].shape[0]) for s in self._segments)

    def __len__(self):
        return len(self.states)

    # -- reference API (Memory.py:14-24) ----------------------------------------------------
    def push(self, state, action, reward, done):
        self.states.append(np.asarray(state).astype(np.float32))
        self.actions.append(np.asarray(action).astype(np.float32))
        self.rewards.append(np.asarray(reward).astype(np.float32))
        self.dones.append(np.asarray(done).astype(np.float32))

    def clear(self):
        for f in (self.states, self.actions, self.rewards, self.dones):
            list.clear(f)
        self._segments.clear()

    # -- device path -----------------------------------------------------------------------
    def push_device(self, S, A, R, Dn):
        """Append a whole env-major rollout (float32 device tensors)."""
        n = S.shape[0]
        if not (A.shape[0] == R.shape[0] == Dn.shape[0] == n):
            raise ValueError("push_device: row counts differ")
        self._segments.append((S, A, R, Dn))

    def device_tensors(self, device):
        """All transitions (host pushes first, then device segments, in push order) as four
        contiguous float32 tensors on `device`."""
        parts = []
        if self.states.host_len():
            parts.append(tuple(
                torch.from_numpy(np.array(list(f), dtype=np.float32)).to(device)
                for f in (self.states, self.actions, self.rewards, self.dones)))
        parts.extend(self._segments)
        if not parts:
            raise ValueError("memory is empty")
        if len(parts) == 1:
            return tuple(p.to(device).contiguous() for p in parts[0])
        return tuple(torch.cat([p[i].to(device) for p in parts]).contiguous() for i in range(4))
