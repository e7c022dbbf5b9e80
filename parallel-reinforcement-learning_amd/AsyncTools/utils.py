"""envs_active mask utilities — drop-in for the reference's AsyncTools/utils.py.

Same names, arguments and results as the reference (utils.py:3-51).  `is_env_terminal` is the
vectorizer's `envs_active` array, where True means TERMINAL (the reference's naming, kept).
The mask / index / compaction work runs in libprl_hip.so (ordered scans and compaction) on the
GPU: numpy inputs are moved to the device and the result is returned as numpy; device tensors
stay on the device.  buffer_append / buffer_to_target_buffer_transfer move Python objects
between the list-based VecMemory/Memory buffers (host bookkeeping, kept for API compatibility);
the device-resident AsyncPPO.worker replaces both with prl_rollout_step + prl_flatten_env_major.
"""
from __future__ import annotations

import numpy as np
import torch

import prl_native


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("AsyncTools.utils runs on the GPU (libprl_hip.so); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _mask_to_dev(mask):
    if isinstance(mask, torch.Tensor):
        t = mask.to(_device()) if not mask.is_cuda else mask
        return t.to(torch.uint8).contiguous(), False
    return torch.from_numpy(np.ascontiguousarray(mask, dtype=np.uint8)).to(_device()), True


def _active(is_env_terminal):
    term, was_np = _mask_to_dev(is_env_terminal)
    E = term.numel()
    idx = torch.empty(max(E, 1), dtype=torch.int64, device=term.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=term.device)
    prl_native.active_indices(term, idx, cnt)
    n = int(cnt.item())
    return idx[:n], n, was_np


def indexes_of_active_environments(num_envs: int, is_env_terminal):
    """utils.py:3-4 — np.arange(num_envs)[~is_env_terminal]."""
    if len(is_env_terminal) != num_envs:
        raise IndexError(f"boolean index did not match: mask of {len(is_env_terminal)} for "
                         f"{num_envs} envs")
    idx, _, was_np = _active(is_env_terminal)
    return idx.cpu().numpy() if was_np else idx


def number_of_active_environments(is_env_terminal):
    """utils.py:6-7 — np.sum(~is_env_terminal)."""
    _, n, was_np = _active(is_env_terminal)
    return np.int64(n) if was_np else n


def range_of_active_environments(is_env_terminal):
    """utils.py:9-12 — np.arange(number_of_active_environments(...))."""
    _, n, was_np = _active(is_env_terminal)
    return np.arange(n) if was_np else torch.arange(n, device=_device())


def inactive_states_dropout(states, dones):
    """utils.py:14-15 — states[~dones] (order kept)."""
    was_np = not isinstance(states, torch.Tensor)
    src = torch.from_numpy(np.ascontiguousarray(states)).to(_device()) if was_np else states
    src = src.contiguous()
    drop, _ = _mask_to_dev(dones)
    if drop.numel() != src.shape[0]:
        raise IndexError(f"boolean index did not match: {drop.numel()} vs {src.shape[0]} rows")
    dst = torch.empty_like(src)
    cnt = torch.zeros(1, dtype=torch.int64, device=src.device)
    prl_native.compact_rows(src, drop, dst, cnt)
    out = dst[: int(cnt.item())]
    return out.cpu().numpy() if was_np else out


def buffer_append(buffer, states, actions, rewards, dones, is_env_terminal, num_envs: int):
    """utils.py:17-36 — the k-th row goes to the k-th active env's per-env lists."""
    idxs = indexes_of_active_environments(num_envs, is_env_terminal)
    if isinstance(idxs, torch.Tensor):
        idxs = idxs.cpu().numpy()
    for i_, idx_ in enumerate(idxs):
        buffer.push(int(idx_), states[i_], actions[i_], rewards[i_], dones[i_])


def update_active_environments_list(is_env_terminal, dones):
    """utils.py:38-43 — is_env_terminal[where(~is_env_terminal)] = dones, in place; returned."""
    term, was_np = _mask_to_dev(is_env_terminal)
    d, _ = _mask_to_dev(dones)
    n_active = int((term == 0).sum().item())
    if d.numel() != n_active and d.numel() != 1:
        raise ValueError(f"shape mismatch: value array of shape ({d.numel()},) could not be "
                         f"broadcast to indexing result of shape ({n_active},)")
    if d.numel() == 1 and n_active != 1:
        d = d.expand(n_active).contiguous()
    prl_native.mask_update(term, d)
    if was_np:
        is_env_terminal[...] = term.cpu().numpy().astype(bool)
        return is_env_terminal
    if is_env_terminal.data_ptr() != term.data_ptr():
        is_env_terminal.copy_(term.to(is_env_terminal.dtype))
    return is_env_terminal


def buffer_to_target_buffer_transfer(buffer, target_buffer):
    """utils.py:45-51 — env-major concatenation into the target, then buffer.clear().
    O(N) list extension (the reference's sum(list, []) is O(E*N))."""
    for name in ("states", "actions", "rewards", "dones"):
        dst = getattr(target_buffer, name)
        for per_env in getattr(buffer, name):
            dst.extend(per_env)
    buffer.clear()
