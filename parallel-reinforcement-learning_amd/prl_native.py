"""ctypes binding of libprl_hip.so (include/prl_abi.h) for torch device tensors.

This is the only way the Python drop-in packages (`PPO`, `AsyncTools`) reach the GPU hot path.
There is no fallback: if the library is missing or no GPU is visible, calls raise.  Tensors are
passed as raw device pointers (`tensor.data_ptr()`) on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PRL_HIP_LIB", os.path.join(_HERE, "libprl_hip.so"))

ENV_KINDS = {"CartPole-v1": 0, "Pendulum-v1": 1, "SyntheticHumanoid-v0": 2}
OP_GAE, OP_SURROGATE, OP_SCAN, OP_STATS, OP_GN = 0, 1, 2, 3, 4

_P = ctypes.c_void_p
_I64, _I32, _U64, _F32, _F64, _INT = (ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64,
                                      ctypes.c_float, ctypes.c_double, ctypes.c_int)
# symbol -> argtypes (restype int unless listed in _RESTYPES)
# the update engines' scalars: clip, vf_coef, ent_coef, lr, beta1, beta2, eps, weight_decay,
# max_norm — the AdamW betas as doubles (1 - beta2 formed from a float32 0.999 is 1.3e-5 off the
# reference's Python-double 1 - 0.999)
_UPD_SCALARS = [_F32] * 4 + [_F64] * 2 + [_F32] * 3

SIGNATURES = {
    "prl_abi_version": [],
    "prl_last_error": [],
    "prl_workspace_bytes": [_INT, _I64],
    "prl_env_dims": [_INT, _P, _P, _P, _P, _P],
    "prl_pcg64_seed": [_P, _I64, _P, _P],
    "prl_env_reset": [_INT, _I64, _P, _P, _P, _P, _P, _P, _I64, _P],
    "prl_env_step_compact": [_INT, _I64, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
    "prl_rollout_step": [_INT, _I64, _I32, _P, _P, _P, _P, _I64, _F32, _U64, _I32, _P, _P, _P,
                         _P, _P, _P, _P, _P],
    "prl_rollout_step_at": [_INT, _I64, _P, _P, _P, _P, _P, _I64, _F32, _U64, _I32, _P, _P, _P,
                         _P, _P, _P, _P, _P],
    "prl_wide_rollout_supported": [_INT, _I32, _I32, _I32],
    "prl_wide_rollout": [_INT, _P, _I32, _I32, _I32, _I64, _P, _P, _P, _F32, _U64, _I32, _P, _P,
                         _P, _P, _P, _P, _P, _P],
    "prl_cartpole_rollout": [_P, _I64, _P, _P, _P, _U64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "prl_active_indices": [_P, _I64, _P, _P, _P, _P],
    "prl_mask_update": [_P, _I64, _P, _I64, _P, _P],
    "prl_compact_rows": [_P, _I64, _I64, _P, _P, _P, _P, _P],
    "prl_exclusive_scan_i32": [_P, _I64, _P, _P, _P],
    "prl_flatten_env_major": [_I64, _I32, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P,
                              _P],
    "prl_gae": [_P, _P, _P, _P, _I64, _F64, _F64, _P, _P, _P, _P, _I64, _P],
    "prl_adv_stats": [_P, _I64, _P, _P, _I64, _P],
    "prl_adv_normalize": [_P, _I64, _P, _F64, _F32, _P, _P],
    "prl_ppo_surrogate_fwd": [_P, _P, _P, _P, _P, _P, _I64, _F32, _F32, _F32, _P, _P, _P, _P,
                              _I64, _P],
    "prl_ppo_surrogate_bwd": [_P, _P, _P, _I64, _P, _P, _P],
    "prl_rnd_forward": [_P, _I64, _I32] + [_P] * 12 + [_F32, _P, _P],
    "prl_rnd_pred_grad": [_P, _I64, _I32] + [_P] * 12 + [_F32, _P, _I64, _P, _P],
    "prl_rnd_pred_grad_ws_floats": [_I64, _I32],
    "prl_gn_silu_fwd": [_P, _I64, _I32, _I32, _P, _P, _F32, _I32, _P, _P],
    "prl_gn_silu_bwd": [_P, _P, _I64, _I32, _I32, _P, _P, _F32, _I32, _P, _P, _P, _P, _I64, _P],
    "prl_gather_minibatch": [_P, _P, _P, _I32, _P, _I64, _I64, _P],
    "prl_ppo_wide_info": [_I32, _I32, _I32, _I64, _P, _P, _P],
    "prl_ppo_wide_grad": [_P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64, _I64, _P, _P, _F32,
                          _F32, _F32, _P, _P, _P, _I64, _P],
    "prl_ppo_wide_grad_prof": [_P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64, _I64, _P, _P,
                               _F32, _F32, _F32, _P, _P, _P, _I64, _P, _P],
    "prl_ppo_wide_evaluate": [_P, _I32, _I32, _I32, _P, _P, _I64, _P, _P, _P],
    "prl_ppo_wide_dist": [_P, _I32, _I32, _I32, _P, _I64, _P, _P],
    "prl_ppo_wide_dist_at": [_P, _I32, _I32, _I32, _P, _I64, _I64, _P, _P, _P],
    "prl_categorical_fwd": [_P, _P, _I64, _I32, _P, _P, _P],
    "prl_categorical_bwd": [_P, _P, _P, _I64, _I32, _P, _P],
    "prl_ppo_update_info": [_I32, _I32, _I32, _I64, _P, _P, _P],
    "prl_ppo_update": [_P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64, _I32, _I32]
                      + _UPD_SCALARS + [_P, _P, _I64, _P],
    "prl_ppo_update_status_ptr": [_P, _P],
    "prl_ppo_update_profile_ptr": [_P, _P],
    "prl_dp_rccl_open": [ctypes.c_char_p],
    "prl_dp_unique_id": [_P, _I64],
    "prl_dp_comm_init": [_P, _I64, _I32, _I32, _P],
    "prl_dp_comm_destroy": [_P],
    "prl_ppo_update_dp": [_P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64, _I32, _I32,
                          _I64, _P, _I64] + _UPD_SCALARS + [_P, _P, _P, _I64, _P, _P],
    "prl_ppo_update_dpx": [_P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64, _I32,
                           _I32, _I32, _P] + _UPD_SCALARS + [_P, _I32, _I32, _P, _I64, _I32, _P,
                                                           _I64, _P],
    "prl_dp_xbuf_bytes": [_I32, _I32, _I32, _I32],
    "prl_dp_set_spin_limit": [ctypes.c_uint32],
    "prl_ppo_update_set_tp": [_I32],
    "prl_ppo_update_set_repl": [_I32],
    "prl_ppo_update_set_split": [_I32],
    "prl_ppo_update_wb_check": [_I32, _I32, _I32],
    "prl_ppo_update_dp_split": [_I32, _I32, _I32, _I32],
    "prl_debug_fill_lds": [_F32, _P],
    "prl_ppo_update_last_plan": [_P],
    "prl_source_id": [],
    "prl_dp_xbuf_alloc": [_I64, _P, _P],
    "prl_dp_xbuf_free": [_P],
    "prl_dp_ipc_handle": [_P, _P, _I64],
    "prl_dp_ipc_open": [_P, _I64, _P],
    "prl_dp_ipc_close": [_P],
    "prl_ppo_evaluate": [_P, _I32, _I32, _I32, _P, _P, _I64, _P, _P, _P, _P],
    "prl_ppo_image_floats": [_I32, _I32, _I32],
    "prl_ppo_image": [_I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _I32, _P],
    "prl_ppo_grad_step": [_P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64, _I32, _I64, _F32, _F32,
                          _F32, _P, _P, _I64, _P],
    # lr, beta1, beta2, eps, weight_decay, max_norm, inv_count, vf_coef, ent_coef
    "prl_ppo_adam_step": [_P, _P, _P, _I32, _I32, _I32, _P, _I64, _F32, _F64, _F64] + [_F32] * 6
                         + [_P, _P],
    "prl_colsum_partial_floats": [_I64, _I32],
    "prl_colsum_f32": [_P, _I64, _I32, _P, _P, _I64, _P],
    "prl_flat_adamw": [_P, _P, _P, _P, _P, _I64, _F32, _F64, _F64, _F32, _F32, _F32, _P, _P],
    "prl_ppo_grad_fold_step": [_P] * 7 + [_I64, _F32, _I32, _I32, _I32] + [_P] * 5
                              + [_I64, _I32, _I64, _F32] + _UPD_SCALARS + [_P, _P, _P, _I64, _P],
}
_RESTYPES = {"prl_last_error": ctypes.c_char_p, "prl_source_id": ctypes.c_char_p,
             "prl_ppo_update_last_plan": None, "prl_workspace_bytes": _I64,
             "prl_rnd_pred_grad_ws_floats": _I64, "prl_dp_xbuf_bytes": _I64,
             "prl_dp_set_spin_limit": ctypes.c_uint32, "prl_ppo_update_set_tp": _I32,
             "prl_ppo_update_set_repl": _I32, "prl_ppo_update_set_split": _I32,
             "prl_ppo_update_wb_check": _I32,
             "prl_ppo_update_dp_split": _I32,
             "prl_ppo_image_floats": _I64, "prl_colsum_partial_floats": _I64}

_lib = None
_lock = threading.Lock()
ABI_VERSION = 2   # include/prl_abi.h PRL_ABI_VERSION (2: prl_ppo_update_last_plan writes 8 entries)


def _sources_id():
    """The stamp the in-tree sources would give (csrc/build.py source_id), or None when the
    library is not the in-tree one or the sources are not next to it."""
    csrc = os.path.join(_HERE, "csrc")
    if "PRL_HIP_LIB" in os.environ or not os.path.exists(os.path.join(csrc, "build.py")):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_prl_csrc_build", os.path.join(csrc, "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    # a package shipped with csrc/ but without every stamped file (e.g. the repo-level include/
    # dir): no stamp to compare against, so the check is skipped rather than failing to load
    if not all(os.path.exists(os.path.join(csrc, f)) for f in mod.SOURCES + mod.HEADERS):
        return None
    return mod.source_id(csrc)


def lib():
    """Load libprl_hip.so once.  Raises RuntimeError if it is missing (build it with
    `python -c "import __graft_entry__ as g; g.build()"` or csrc/build.py)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"libprl_hip.so not found at {LIB_PATH}: build it with "
                                       "parallel-reinforcement-learning_amd/csrc/build.py")
                L = ctypes.CDLL(LIB_PATH)
                for name, args in SIGNATURES.items():
                    try:
                        fn = getattr(L, name)
                    except AttributeError:
                        # an explicit PRL_HIP_LIB (an older build for a same-box A/B) may lack
                        # symbols added since; the in-tree library must export every one
                        if "PRL_HIP_LIB" in os.environ:
                            continue
                        raise
                    fn.argtypes = args
                    fn.restype = _RESTYPES.get(name, ctypes.c_int)
                if L.prl_abi_version() != ABI_VERSION:
                    raise RuntimeError(f"libprl_hip.so ABI version {L.prl_abi_version()}, this "
                                       f"package needs {ABI_VERSION}: rebuild it")
                want = _sources_id()
                got = L.prl_source_id().decode()
                if want is not None and got != want:
                    raise RuntimeError(
                        f"{LIB_PATH} was built from other sources (stamp {got[:12]}, sources "
                        f"{want[:12]}): rebuild it with parallel-reinforcement-learning_amd/csrc/"
                        "build.py")
                _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().prl_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def _dev(t: torch.Tensor | None, dtype=None, name="tensor"):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# ------------------------------------------------------------------------- workspace
class _Workspace:
    """Per-(op, device) scratch, zero-initialised when (re)allocated, grown never shrunk.
    The GAE / statistics / surrogate kernels keep their in-launch synchronisation state here
    and leave it re-armed after every launch (include/prl_abi.h), so each op owns its buffer.
    Callers that capture graphs reserve first (reserve_workspace)."""

    def __init__(self):
        self.buf = {}

    def get(self, op: int, nbytes: int, device) -> torch.Tensor:
        dev = torch.device(device)
        key = (op, dev.type, dev.index)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
            self.buf[key] = b
        return b


_ws = _Workspace()


def workspace_bytes(op: int, n: int) -> int:
    return int(lib().prl_workspace_bytes(op, int(n)))


def workspace(op: int, n: int, device) -> torch.Tensor:
    return _ws.get(op, workspace_bytes(op, n), device)


def reserve_workspace(n: int, device):
    """Pre-grow every op's scratch for n elements so later calls (e.g. under graph capture)
    do not allocate."""
    for op in (OP_GAE, OP_SURROGATE, OP_SCAN, OP_STATS, OP_GN):
        workspace(op, n, device)


# ------------------------------------------------------------------------- envs
def env_dims(kind: int):
    o = [ctypes.c_int() for _ in range(5)]
    _check(lib().prl_env_dims(kind, *[ctypes.byref(x) for x in o]), "prl_env_dims")
    D, A, P, T, disc = (x.value for x in o)
    return dict(obs_dim=D, act_dim=A, phys_dim=P, max_episode_steps=T, discrete=bool(disc))


def pcg64_seed(seeds: torch.Tensor, rng: torch.Tensor):
    E = seeds.numel()
    _check(lib().prl_pcg64_seed(_dev(seeds, torch.int64, "seeds"), E,
                                _dev(rng, torch.int64, "rng"), _stream()), "prl_pcg64_seed")


def env_reset(kind, phys, rng, t_elapsed, terminal, obs, obs_stride, reset_mask=None):
    E = t_elapsed.numel()
    _check(lib().prl_env_reset(kind, E, _dev(phys, torch.float64, "phys"),
                               _dev(rng, torch.int64, "rng"), _dev(t_elapsed, torch.int32, "t"),
                               _dev(terminal, torch.uint8, "terminal"),
                               _dev(reset_mask, torch.uint8, "reset_mask"),
                               _dev(obs, torch.float32, "obs"), int(obs_stride), _stream()),
           "prl_env_reset")


def env_step_compact(kind, phys, t_elapsed, active_idx, n, actions, obs_out, reward_out,
                     terminated_out, truncated_out):
    E = t_elapsed.numel()
    _check(lib().prl_env_step_compact(kind, E, _dev(phys, torch.float64, "phys"),
                                      _dev(t_elapsed, torch.int32, "t"),
                                      _dev(active_idx, torch.int64, "active_idx"), int(n),
                                      _dev(actions, None, "actions"),
                                      _dev(obs_out, torch.float32, "obs_out"),
                                      _dev(reward_out, torch.float64, "reward_out"),
                                      _dev(terminated_out, torch.uint8, "terminated_out"),
                                      _dev(truncated_out, torch.uint8, "truncated_out"),
                                      _stream()), "prl_env_step_compact")


def rollout_step(kind, step, phys, t_elapsed, terminal, dist, action_scaling, seed, t_max,
                 traj_obs, traj_act, traj_rew, traj_done, ep_len, active_after, reward_sum):
    E = t_elapsed.numel()
    _check(lib().prl_rollout_step(kind, E, int(step), _dev(phys, torch.float64, "phys"),
                                  _dev(t_elapsed, torch.int32, "t"),
                                  _dev(terminal, torch.uint8, "terminal"),
                                  _dev(dist, torch.float32, "dist"), int(dist.stride(0)),
                                  float(action_scaling), int(seed) & (2**64 - 1), int(t_max),
                                  _dev(traj_obs, torch.float32, "traj_obs"),
                                  _dev(traj_act, torch.float32, "traj_act"),
                                  _dev(traj_rew, torch.float32, "traj_rew"),
                                  _dev(traj_done, torch.uint8, "traj_done"),
                                  _dev(ep_len, torch.int32, "ep_len"),
                                  _dev(active_after, torch.int32, "active_after"),
                                  _dev(reward_sum, torch.float64, "reward_sum"), _stream()),
           "prl_rollout_step")


def rollout_step_at(kind, step_dev, phys, t_elapsed, terminal, dist, action_scaling, seed, t_max,
                    traj_obs, traj_act, traj_rew, traj_done, ep_len, active_after, reward_sum):
    """rollout_step with the step index on the device (step_dev: int64 [2] = {k, arrivals},
    arrivals 0); the still-active count goes to active_after[k] and the kernel advances k by one
    (the captured vector step)."""
    E = t_elapsed.numel()
    if step_dev.numel() < 2:
        raise ValueError("step_dev must hold {k, arrivals} (int64 [2])")
    _check(lib().prl_rollout_step_at(kind, E, _dev(step_dev, torch.int64, "step_dev"),
                                     _dev(phys, torch.float64, "phys"),
                                     _dev(t_elapsed, torch.int32, "t"),
                                     _dev(terminal, torch.uint8, "terminal"),
                                     _dev(dist, torch.float32, "dist"), int(dist.stride(0)),
                                     float(action_scaling), int(seed) & (2**64 - 1), int(t_max),
                                     _dev(traj_obs, torch.float32, "traj_obs"),
                                     _dev(traj_act, torch.float32, "traj_act"),
                                     _dev(traj_rew, torch.float32, "traj_rew"),
                                     _dev(traj_done, torch.uint8, "traj_done"),
                                     _dev(ep_len, torch.int32, "ep_len"),
                                     _dev(active_after, torch.int32, "active_after"),
                                     _dev(reward_sum, torch.float64, "reward_sum"), _stream()),
           "prl_rollout_step_at")


def wide_rollout_supported(kind, D, A, discrete) -> bool:
    return bool(lib().prl_wide_rollout_supported(int(kind), int(D), int(A), int(bool(discrete))))


def wide_rollout(kind, params, D, A, discrete, phys, t_elapsed, terminal, action_scaling, seed,
                 t_max, traj_obs, traj_act, traj_rew, traj_done, ep_len, active_after, reward_sum):
    """The whole rollout of the wide continuous actor in one persistent launch (prl_wide_rollout):
    every non-terminal env stepped to the end of its episode."""
    E = t_elapsed.numel()
    _check(lib().prl_wide_rollout(kind, _dev(params, torch.float32, "params"), int(D), int(A),
                                  int(bool(discrete)), E, _dev(phys, torch.float64, "phys"),
                                  _dev(t_elapsed, torch.int32, "t"),
                                  _dev(terminal, torch.uint8, "terminal"), float(action_scaling),
                                  int(seed) & (2**64 - 1), int(t_max),
                                  _dev(traj_obs, torch.float32, "traj_obs"),
                                  _dev(traj_act, torch.float32, "traj_act"),
                                  _dev(traj_rew, torch.float32, "traj_rew"),
                                  _dev(traj_done, torch.uint8, "traj_done"),
                                  _dev(ep_len, torch.int32, "ep_len"),
                                  _dev(active_after, torch.int32, "active_after"),
                                  _dev(reward_sum, torch.float64, "reward_sum"), _stream()),
           "prl_wide_rollout")


def cartpole_rollout(params, phys, t_elapsed, terminal, seed, t_max, traj_obs, traj_act, traj_rew,
                     traj_done, ep_len, active_after, reward_sum, probs_out=None):
    """The whole CartPole rollout of the discrete actor in one launch (prl_cartpole_rollout): every
    non-terminal env stepped to the end of its episode; probs_out ([t_max, E, 2] f32, tests)
    receives the probabilities each step sampled from."""
    E = t_elapsed.numel()
    _check(lib().prl_cartpole_rollout(_dev(params, torch.float32, "params"), E,
                                      _dev(phys, torch.float64, "phys"),
                                      _dev(t_elapsed, torch.int32, "t"),
                                      _dev(terminal, torch.uint8, "terminal"),
                                      int(seed) & (2**64 - 1), int(t_max),
                                      _dev(traj_obs, torch.float32, "traj_obs"),
                                      _dev(traj_act, torch.float32, "traj_act"),
                                      _dev(traj_rew, torch.float32, "traj_rew"),
                                      _dev(traj_done, torch.uint8, "traj_done"),
                                      _dev(ep_len, torch.int32, "ep_len"),
                                      _dev(active_after, torch.int32, "active_after"),
                                      _dev(reward_sum, torch.float64, "reward_sum"),
                                      _dev(probs_out, torch.float32, "probs_out"), _stream()),
           "prl_cartpole_rollout")


# ------------------------------------------------------------------------- masks / buffers
def active_indices(terminal: torch.Tensor, idx_out: torch.Tensor, count_out: torch.Tensor):
    E = terminal.numel()
    ws = workspace(OP_SCAN, E, terminal.device)
    _check(lib().prl_active_indices(_dev(terminal, torch.uint8, "terminal"), E,
                                    _dev(idx_out, torch.int64, "idx_out"),
                                    _dev(count_out, torch.int64, "count_out"), _dev(ws),
                                    _stream()), "prl_active_indices")


def mask_update(terminal: torch.Tensor, dones: torch.Tensor):
    E = terminal.numel()
    ws = workspace(OP_SCAN, E, terminal.device)
    _check(lib().prl_mask_update(_dev(terminal, torch.uint8, "terminal"), E,
                                 _dev(dones, torch.uint8, "dones"), dones.numel(), _dev(ws),
                                 _stream()), "prl_mask_update")


def compact_rows(src: torch.Tensor, drop: torch.Tensor, dst: torch.Tensor, count_out: torch.Tensor):
    rows = src.shape[0]
    row_bytes = src[0].numel() * src.element_size() if rows else 0
    ws = workspace(OP_SCAN, rows, src.device)
    _check(lib().prl_compact_rows(_dev(src), rows, row_bytes, _dev(drop, torch.uint8, "drop"),
                                  _dev(dst), _dev(count_out, torch.int64, "count_out"), _dev(ws),
                                  _stream()), "prl_compact_rows")


def exclusive_scan_i32(x: torch.Tensor, offsets: torch.Tensor):
    n = x.numel()
    ws = workspace(OP_SCAN, n, x.device)
    _check(lib().prl_exclusive_scan_i32(_dev(x, torch.int32, "x"), n,
                                        _dev(offsets, torch.int64, "offsets"), _dev(ws),
                                        _stream()), "prl_exclusive_scan_i32")


def flatten_env_major(offsets, N, traj_obs, traj_act, traj_rew, traj_done, S, A, R, Dn):
    T1, E, D = traj_obs.shape
    Adim = traj_act.shape[2] if traj_act.dim() == 3 else 1
    _check(lib().prl_flatten_env_major(E, traj_rew.shape[0], D, Adim,
                                       _dev(offsets, torch.int64, "offsets"), int(N),
                                       _dev(traj_obs, torch.float32, "traj_obs"),
                                       _dev(traj_act, torch.float32, "traj_act"),
                                       _dev(traj_rew, torch.float32, "traj_rew"),
                                       _dev(traj_done, torch.uint8, "traj_done"),
                                       _dev(S, torch.float32, "S"), _dev(A, torch.float32, "A"),
                                       _dev(R, torch.float32, "R"),
                                       _dev(Dn, torch.float32, "Dn"), _stream()),
           "prl_flatten_env_major")


# ------------------------------------------------------------------------- learn()
def gae(r, d, V, next_value, gamma, lam, ret, adv=None, sums=None):
    n = V.numel()
    ws = workspace(OP_GAE, n, V.device)
    _check(lib().prl_gae(_dev(r, torch.float32, "r"), _dev(d, torch.float32, "d"),
                         _dev(V, torch.float32, "V"),
                         _dev(next_value, torch.float32, "next_value"), n, float(gamma),
                         float(lam), _dev(ret, torch.float32, "ret"),
                         _dev(adv, torch.float32, "adv"), _dev(sums, torch.float64, "sums"),
                         _dev(ws), ws.numel(), _stream()), "prl_gae")


def adv_stats(x, sums):
    n = x.numel()
    ws = workspace(OP_STATS, n, x.device)
    _check(lib().prl_adv_stats(_dev(x, torch.float32, "x"), n, _dev(sums, torch.float64, "sums"),
                               _dev(ws), ws.numel(), _stream()), "prl_adv_stats")


def adv_normalize(x, sums, count, eps, out):
    _check(lib().prl_adv_normalize(_dev(x, torch.float32, "x"), x.numel(),
                                   _dev(sums, torch.float64, "sums"), float(count), float(eps),
                                   _dev(out, torch.float32, "out"), _stream()),
           "prl_adv_normalize")


def surrogate_fwd(logp, old_logp, adv, V, ret, entropy, clip, vf_coef, ent_coef, loss_out,
                  dlogp=None, dV=None):
    mb = logp.numel()
    ws = workspace(OP_SURROGATE, mb, logp.device)
    _check(lib().prl_ppo_surrogate_fwd(
        _dev(logp, torch.float32, "logp"), _dev(old_logp, torch.float32, "old_logp"),
        _dev(adv, torch.float32, "adv"), _dev(V, torch.float32, "V"),
        _dev(ret, torch.float32, "ret"), _dev(entropy, torch.float32, "entropy"), mb,
        float(clip), float(vf_coef), float(ent_coef), _dev(loss_out, torch.float32, "loss"),
        _dev(dlogp, torch.float32, "dlogp"), _dev(dV, torch.float32, "dV"), _dev(ws),
        ws.numel(), _stream()), "prl_ppo_surrogate_fwd")


def surrogate_bwd(grad_out, dlogp_unit, dV_unit, dlogp, dV):
    _check(lib().prl_ppo_surrogate_bwd(_dev(grad_out, torch.float32, "grad_out"),
                                       _dev(dlogp_unit, torch.float32, "dlogp_unit"),
                                       _dev(dV_unit, torch.float32, "dV_unit"), dlogp_unit.numel(),
                                       _dev(dlogp, torch.float32, "dlogp"),
                                       _dev(dV, torch.float32, "dV"), _stream()),
           "prl_ppo_surrogate_bwd")


def rnd_forward(x, tnet, pnet, beta, out):
    """tnet/pnet: sequences (w1, b1, gw, gb, w2, b2) of contiguous float32 device tensors."""
    n, D = x.shape
    ptrs = [_dev(p.contiguous() if not p.is_contiguous() else p, torch.float32, "rnd param")
            for p in (*tnet, *pnet)]
    _check(lib().prl_rnd_forward(_dev(x, torch.float32, "x"), n, D, *ptrs, float(beta),
                                 _dev(out, torch.float32, "out"), _stream()), "prl_rnd_forward")


def rnd_pred_grad_ws_floats(n: int, D: int) -> int:
    return int(lib().prl_rnd_pred_grad_ws_floats(int(n), int(D)))


def rnd_pred_grad(x, tnet, pnet, scale, partial, grad):
    """RND.update_pred's predictor gradient for the minibatch x (prl_rnd_pred_grad): grad (flat,
    the predictor's parameters() order) = d/dpred MSE('mean') scaled so that scale = 2 / (rows D)
    is the reference's mean.  tnet / pnet: (w1, b1, gw, gb, w2, b2) float32 device tensors."""
    n, D = x.shape
    ptrs = [_dev(p, torch.float32, "rnd param") for p in (*tnet, *pnet)]
    _check(lib().prl_rnd_pred_grad(_dev(x, torch.float32, "x"), n, D, *ptrs, float(scale),
                                   _dev(partial, torch.float32, "partial"), partial.numel(),
                                   _dev(grad, torch.float32, "grad"), _stream()), "prl_rnd_pred_grad")


# ------------------------------------------------------------------------- GroupNorm + SiLU
def gn_silu_fwd(x, w, b, eps, silu, out):
    N = x.shape[0]
    _check(lib().prl_gn_silu_fwd(_dev(x, torch.float32, "x"), N, x.shape[1], 8,
                                 _dev(w, torch.float32, "w"), _dev(b, torch.float32, "b"),
                                 float(eps), int(bool(silu)), _dev(out, torch.float32, "out"),
                                 _stream()), "prl_gn_silu_fwd")


def gn_silu_bwd(x, dout, w, b, eps, silu, dx, dw, db):
    N = x.shape[0]
    ws = workspace(OP_GN, N, x.device)
    _check(lib().prl_gn_silu_bwd(_dev(x, torch.float32, "x"), _dev(dout, torch.float32, "dout"),
                                 N, x.shape[1], 8, _dev(w, torch.float32, "w"),
                                 _dev(b, torch.float32, "b"), float(eps), int(bool(silu)),
                                 _dev(dx, torch.float32, "dx"), _dev(dw, torch.float32, "dw"),
                                 _dev(db, torch.float32, "db"), _dev(ws), ws.numel(), _stream()),
           "prl_gn_silu_bwd")


# ------------------------------------------------------------------------- optimizer step
class MinibatchGather:
    """prl_gather_minibatch bound to fixed source / destination tensors (graph-capturable)."""

    def __init__(self, sources, dests, cursor, mb):
        if not 1 <= len(sources) <= 6 or len(sources) != len(dests):
            raise ValueError("1..6 source/destination pairs")
        for s_, d_ in zip(sources, dests):
            _dev(s_, torch.float32, "source")
            _dev(d_, torch.float32, "dest")
        self._keep = (list(sources), list(dests), cursor)
        n = len(sources)
        self.srcs = (ctypes.c_void_p * n)(*[s_.data_ptr() for s_ in sources])
        self.dsts = (ctypes.c_void_p * n)(*[d_.data_ptr() for d_ in dests])
        self.widths = (ctypes.c_int32 * n)(*[int(s_[0].numel()) if s_.dim() > 1 else 1
                                             for s_ in sources])
        self.n = n
        self.cursor = cursor
        self.mb = int(mb)
        self.nrows = int(sources[0].shape[0])

    def __call__(self):
        _check(lib().prl_gather_minibatch(self.srcs, self.dsts, self.widths, self.n,
                                          _dev(self.cursor, torch.int64, "cursor"), self.mb,
                                          self.nrows, _stream()), "prl_gather_minibatch")


def colsum(x: torch.Tensor) -> torch.Tensor:
    """Column sums of a 2-D f32 device matrix (1^T x), deterministic (prl_colsum_f32)."""
    rows, cols = x.shape
    x = x.contiguous()
    out = torch.empty(cols, dtype=torch.float32, device=x.device)
    npart = int(lib().prl_colsum_partial_floats(int(rows), int(cols)))
    part = torch.empty(max(npart, 1), dtype=torch.float32, device=x.device)
    _check(lib().prl_colsum_f32(_dev(x, torch.float32, "x"), int(rows), int(cols),
                                _dev(out, torch.float32, "out"), _dev(part, torch.float32, "part"),
                                npart, _stream()), "prl_colsum_f32")
    return out


def categorical_fwd(probs, actions, logp, entropy=None):
    n, A = probs.shape
    _check(lib().prl_categorical_fwd(_dev(probs, torch.float32, "probs"),
                                     _dev(actions, torch.float32, "actions"), n, A,
                                     _dev(logp, torch.float32, "logp"),
                                     _dev(entropy, torch.float32, "entropy"), _stream()),
           "prl_categorical_fwd")


def categorical_bwd(probs, actions, dlogp, dprobs):
    n, A = probs.shape
    _check(lib().prl_categorical_bwd(_dev(probs, torch.float32, "probs"),
                                     _dev(actions, torch.float32, "actions"),
                                     _dev(dlogp, torch.float32, "dlogp"), n, A,
                                     _dev(dprobs, torch.float32, "dprobs"), _stream()),
           "prl_categorical_bwd")


def ppo_update_info(D: int, A: int, discrete: bool, mini_batch: int):
    """(n_params, workspace_bytes, grid) of the fused update engine, or None when the shape is
    outside it (the caller then uses the graph-replayed PyTorch step)."""
    n_params, ws, grid = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
    rc = lib().prl_ppo_update_info(int(D), int(A), int(bool(discrete)), int(mini_batch),
                                   ctypes.byref(n_params), ctypes.byref(ws), ctypes.byref(grid))
    if rc != 0:
        return None
    return n_params.value, ws.value, grid.value


def ppo_wide_info(D: int, A: int, discrete: bool, mini_batch: int):
    """(n_params, part_floats, grid) of the wide-net gradient kernel (prl_ppo_wide_grad), or None
    when the shape is outside it."""
    n_params, part, grid = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
    rc = lib().prl_ppo_wide_info(int(D), int(A), int(bool(discrete)), int(mini_batch),
                                 ctypes.byref(n_params), ctypes.byref(part), ctypes.byref(grid))
    if rc != 0:
        return None
    return n_params.value, part.value, grid.value


def ppo_wide_grad(params, D, A, discrete, S, actions, old_logp, adv, ret, mini_batch, cursor,
                  scales, clip, vf_coef, ent_coef, grad, loss_out, part, prof=None):
    """Gradient (flat, torch parameters() order) and loss of ONE optimizer step's minibatch
    (rows cursor*mb .. of S, ...) for the wide nets, in two HIP launches (prl_ppo_wide_grad).
    Graph-capturable: the minibatch index is read from the device `cursor` (int64)."""
    N = int(S.shape[0])
    fn = lib().prl_ppo_wide_grad if prof is None else lib().prl_ppo_wide_grad_prof
    extra = () if prof is None else (_dev(prof, torch.int64, "prof"),)
    _check(fn(
        _dev(params, torch.float32, "params"), int(D), int(A), int(bool(discrete)),
        _dev(S, torch.float32, "S"), _dev(actions, torch.float32, "actions"),
        _dev(old_logp, torch.float32, "old_logp"), _dev(adv, torch.float32, "adv"),
        _dev(ret, torch.float32, "ret"), N, int(mini_batch), _dev(cursor, torch.int64, "cursor"),
        _dev(scales, torch.float32, "scales"), float(clip), float(vf_coef), float(ent_coef),
        _dev(grad, torch.float32, "grad"), _dev(loss_out, torch.float32, "loss_out"),
        _dev(part, torch.float32, "part"), part.numel(), *extra, _stream()), "prl_ppo_wide_grad")


def ppo_wide_evaluate(params, D, A, discrete, S, actions, logp, V):
    """ActorCritic.get_evaluate's log_prob and value over all rows with the wide step's forward
    arithmetic (prl_ppo_wide_evaluate)."""
    _check(lib().prl_ppo_wide_evaluate(
        _dev(params, torch.float32, "params"), int(D), int(A), int(bool(discrete)),
        _dev(S, torch.float32, "S"), _dev(actions, torch.float32, "actions"), int(S.shape[0]),
        _dev(logp, torch.float32, "logp"), _dev(V, torch.float32, "V"), _stream()),
        "prl_ppo_wide_evaluate")


def ppo_wide_dist(params, D, A, discrete, S, out):
    """ActorCritic.dist_params for the wide nets (prl_ppo_wide_dist): out = [N][A] probs or
    [N][2A] = [mu | std], from the wide kernel's forward."""
    _check(lib().prl_ppo_wide_dist(
        _dev(params, torch.float32, "params"), int(D), int(A), int(bool(discrete)),
        _dev(S, torch.float32, "S"), int(S.shape[0]), _dev(out, torch.float32, "out"), _stream()),
        "prl_ppo_wide_dist")


def ppo_wide_dist_at(params, D, A, discrete, S, rows, step_dev, out):
    """prl_ppo_wide_dist on rows [k*rows, (k+1)*rows) of S with k = step_dev[0] (a device int64):
    the rollout graph's sampling input straight from traj_obs[k], no per-step copy.  S is any
    contiguous [..., D] store (e.g. traj_obs [T+1][E][D])."""
    if S.shape[-1] != D:
        raise ValueError(f"S's last dimension {S.shape[-1]} != D {D}")
    _check(lib().prl_ppo_wide_dist_at(
        _dev(params, torch.float32, "params"), int(D), int(A), int(bool(discrete)),
        _dev(S, torch.float32, "S"), int(S.numel() // int(D)), int(rows),
        _dev(step_dev, torch.int64, "step_dev"), _dev(out, torch.float32, "out"), _stream()),
        "prl_ppo_wide_dist_at")


def ppo_update(params, exp_avg, exp_avg_sq, adam_step, D, A, discrete, S, actions, old_logp, adv,
               ret, mini_batch, k_epochs, clip, vf_coef, ent_coef, lr, beta1, beta2, eps,
               weight_decay, max_norm, loss_out, workspace):
    N = int(S.shape[0])
    _check(lib().prl_ppo_update(
        _dev(params, torch.float32, "params"), _dev(exp_avg, torch.float32, "exp_avg"),
        _dev(exp_avg_sq, torch.float32, "exp_avg_sq"), _dev(adam_step, torch.float32, "adam_step"),
        int(D), int(A), int(bool(discrete)), _dev(S, torch.float32, "S"),
        _dev(actions, torch.float32, "actions"), _dev(old_logp, torch.float32, "old_logp"),
        _dev(adv, torch.float32, "adv"), _dev(ret, torch.float32, "ret"), N, int(mini_batch),
        int(k_epochs), float(clip), float(vf_coef), float(ent_coef), float(lr), float(beta1),
        float(beta2), float(eps), float(weight_decay), float(max_norm),
        _dev(loss_out, torch.float32, "loss_out"), _dev(workspace, torch.uint8, "workspace"),
        workspace.numel(), _stream()), "prl_ppo_update")


def ppo_update_status(workspace) -> torch.Tensor:
    """Device i32 view of the engine's status words: [0] last launch (0 ok, 1 in-kernel timeout),
    [1] sticky timeout flag over all launches on this workspace."""
    ptr = ctypes.c_void_p()
    _check(lib().prl_ppo_update_status_ptr(_dev(workspace, torch.uint8, "workspace"),
                                           ctypes.byref(ptr)), "prl_ppo_update_status_ptr")
    return workspace[12:20].view(torch.int32)


def ppo_update_profile(workspace) -> torch.Tensor:
    """Device i64 view of the engine's 32 timing words (engine.FusedUpdate.profile)."""
    ptr = ctypes.c_void_p()
    _check(lib().prl_ppo_update_profile_ptr(_dev(workspace, torch.uint8, "workspace"),
                                            ctypes.byref(ptr)), "prl_ppo_update_profile_ptr")
    off = int(ptr.value) - workspace.data_ptr()
    return workspace[off:off + 256].view(torch.int64)


# ------------------------------------------------------------- data-parallel step loop (RCCL)
RCCL_UNIQUE_ID_BYTES = 128


def dp_rccl_open(path: str | None = None):
    """Resolve RCCL's entry points from the library torch loaded (one RCCL per process)."""
    if path is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    _check(lib().prl_dp_rccl_open(path.encode()), "prl_dp_rccl_open")


def dp_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(RCCL_UNIQUE_ID_BYTES)
    _check(lib().prl_dp_unique_id(ctypes.cast(buf, ctypes.c_void_p), RCCL_UNIQUE_ID_BYTES),
           "prl_dp_unique_id")
    return buf.raw


def dp_comm_init(uid: bytes, nranks: int, rank: int) -> ctypes.c_void_p:
    buf = ctypes.create_string_buffer(bytes(uid), RCCL_UNIQUE_ID_BYTES)
    comm = ctypes.c_void_p()
    _check(lib().prl_dp_comm_init(ctypes.cast(buf, ctypes.c_void_p), RCCL_UNIQUE_ID_BYTES,
                                  int(nranks), int(rank), ctypes.byref(comm)), "prl_dp_comm_init")
    return comm


def dp_comm_destroy(comm):
    if comm:
        lib().prl_dp_comm_destroy(comm)


def ppo_update_dp(img_p, img_m, img_v, D, A, discrete, S, A_, old_logp, adv, ret, mini_batch,
                  k_epochs, counts, step0, clip, vf_coef, ent_coef, lr, beta1, beta2, eps, wd,
                  max_norm, grad, loss_out, workspace, comm):
    """The stepped engine's whole loop enqueued natively (prl_ppo_update_dp): per optimizer step
    gradient kernel -> ncclAllReduce(grad) -> AdamW kernel on torch's current stream."""
    import numpy as np
    cnt = np.ascontiguousarray(np.asarray(counts, dtype=np.int64))
    N = int(S.shape[0])
    _check(lib().prl_ppo_update_dp(
        _dev(img_p, torch.float32, "img_p"), _dev(img_m, torch.float32, "img_m"),
        _dev(img_v, torch.float32, "img_v"), int(D), int(A), int(bool(discrete)),
        _dev(S, torch.float32, "S"), _dev(A_, torch.float32, "actions"),
        _dev(old_logp, torch.float32, "old_logp"), _dev(adv, torch.float32, "adv"),
        _dev(ret, torch.float32, "ret"), N, int(mini_batch), int(k_epochs), int(cnt.size),
        cnt.ctypes.data_as(ctypes.c_void_p), int(step0), clip, vf_coef, ent_coef, lr, beta1,
        beta2, eps, wd, max_norm, _dev(grad, torch.float32, "grad"),
        _dev(loss_out, torch.float32, "loss"), _dev(workspace, torch.uint8, "workspace"),
        workspace.numel(), comm, _stream()), "prl_ppo_update_dp")


# -------------------------------------- data-parallel persistent engine (IPC slice buffers)
IPC_HANDLE_BYTES = 64


def dp_xbuf_bytes(D, A, discrete, mini_batch) -> int:
    n = int(lib().prl_dp_xbuf_bytes(int(D), int(A), int(bool(discrete)), int(mini_batch)))
    if n <= 0:
        raise ValueError(f"prl_dp_xbuf_bytes: shape D={D} A={A} not on the fused engine")
    return n


def dp_set_spin_limit(polls: int) -> int:
    """Polls of the data-parallel launch's cross-rank wait before it times out (0: default);
    returns the previous value."""
    return int(lib().prl_dp_set_spin_limit(int(polls)))


def ppo_update_set_tp(mode: int) -> int:
    """Form of the fused update engine: 0 latency form, 1 throughput form (launches of >= 2
    steps), 2 auto (default); returns the previous mode.  Both forms give the same bits."""
    return int(lib().prl_ppo_update_set_tp(int(mode)))


def debug_fill_lds(value: float) -> None:
    """Fill every CU's LDS with `value` on the current stream (tests: kernels must not read LDS
    they did not write in their own launch)."""
    _check(lib().prl_debug_fill_lds(float(value), _stream()), "prl_debug_fill_lds")


def ppo_update_set_repl(replicas: int) -> int:
    """Workgroups per 16-row tile group of the engine's latency form (each publishes its share of
    the tile's partial gradient); returns the previous value.  Every value gives the same bits."""
    return int(lib().prl_ppo_update_set_repl(int(replicas)))


def ppo_update_set_split(mode: int) -> int:
    """The engine's head-split latency form for the two-head CartPole shape (1, the default) or
    the 8-wave kernel (0); returns the previous value.  The two agree to float32 rounding."""
    return int(lib().prl_ppo_update_set_split(int(mode)))


def flat_adamw(params, exp_avg, exp_avg_sq, step, grad, lr, beta1, beta2, eps, weight_decay,
               max_norm, total_norm=None):
    """clip_grad_norm_(max_norm) + AdamW.step() over flat f32 vectors (one launch up to 262,144
    parameters, two above).  total_norm: a two-entry f32 device workspace, zeroed before its
    first use ([0] the gradient's norm, clip_grad_norm_'s return value; [1] the launch's arrival
    counter, left at zero by every call; a new one unless passed).  A caller's buffer is zeroed
    here on its first use (torch.empty or a reused buffer would otherwise leave the counter
    dirty: no workgroup would see itself last, so the gradient would stay unclipped and the
    step count unadvanced, silently).  Returns total_norm[:1]."""
    P = int(params.numel())
    for t, n in ((exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq"), (grad, "grad")):
        if t.numel() != P:
            raise ValueError(f"{n} has {t.numel()} entries, params {P}")
    if total_norm is None:
        total_norm = torch.zeros(2, dtype=torch.float32, device=params.device)
    if total_norm.numel() < 2:
        raise ValueError("total_norm must hold 2 entries (the norm and an arrival counter)")
    if not getattr(total_norm, "_prl_fa_zeroed", False):
        total_norm.zero_()
        total_norm._prl_fa_zeroed = True
    _check(lib().prl_flat_adamw(
        _dev(params, torch.float32, "params"), _dev(exp_avg, torch.float32, "exp_avg"),
        _dev(exp_avg_sq, torch.float32, "exp_avg_sq"), _dev(step, torch.float32, "step"),
        _dev(grad, torch.float32, "grad"), P, float(lr), float(beta1), float(beta2), float(eps),
        float(weight_decay), float(max_norm), _dev(total_norm, torch.float32, "total_norm"),
        _stream()), "prl_flat_adamw")
    return total_norm[:1]


def ppo_update_last_plan() -> dict:
    """What the last prl_ppo_update / _dpx launch in this process ran: form ("throughput" /
    "latency"), waves per workgroup, workgroups, 16-row tiles per workgroup and step, whether
    the kernel was a compile-time-layout specialisation, and the workgroups per tile group (the
    latency form's replicated tiles; the split form: its two head roles), and whether the
    head-split latency form ran (csrc/prl_ppo_split.h) and whether in its slice-owner variant
    ("owner": AdamW by the slice owners, PRL_UPD_SPL_OWN), and the split form's phase-B helper
    workgroups (launched beside "grid")."""
    out = (ctypes.c_int32 * 8)()
    lib().prl_ppo_update_last_plan(out)
    tp, nw, G, tiles, spec, repl, split, helpers = list(out)
    return {"form": {1: "throughput", 0: "latency"}.get(tp), "waves": nw, "grid": G,
            "tiles": tiles, "specialised": bool(spec == 1), "replicas": repl,
            "split": bool(split >= 1), "owner": bool(split == 2), "helpers": helpers}


XBUF_KINDS = {"auto": 0, "uncached": 1, "fine": 2}


def dp_xbuf_alloc(nbytes: int, kind: str = "auto"):
    """A zeroed device allocation of its own (shareable by IPC handle): uncached memory, or
    fine-grained memory as the fallback ("auto"); kind "uncached" / "fine" forces one.  Returns
    (pointer, "uncached" | "fine")."""
    p = ctypes.c_void_p()
    k = ctypes.c_int32(XBUF_KINDS[kind])
    _check(lib().prl_dp_xbuf_alloc(int(nbytes), ctypes.byref(k), ctypes.byref(p)),
           "prl_dp_xbuf_alloc")
    return p, {1: "uncached", 2: "fine"}[k.value]


def dp_xbuf_free(p):
    if p:
        _check(lib().prl_dp_xbuf_free(p), "prl_dp_xbuf_free")


def dp_ipc_handle(p) -> bytes:
    buf = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
    _check(lib().prl_dp_ipc_handle(p, ctypes.cast(buf, ctypes.c_void_p), IPC_HANDLE_BYTES),
           "prl_dp_ipc_handle")
    return buf.raw


def dp_ipc_open(handle: bytes) -> ctypes.c_void_p:
    buf = ctypes.create_string_buffer(bytes(handle), IPC_HANDLE_BYTES)
    p = ctypes.c_void_p()
    _check(lib().prl_dp_ipc_open(ctypes.cast(buf, ctypes.c_void_p), IPC_HANDLE_BYTES,
                                 ctypes.byref(p)), "prl_dp_ipc_open")
    return p


def dp_ipc_close(p):
    if p:
        _check(lib().prl_dp_ipc_close(p), "prl_dp_ipc_close")


def ppo_update_dp_split(D, A, discrete, mini_batch) -> bool:
    """Would a data-parallel launch of this shape run the head-split kernel in this process?
    (The ranks vote: the kernel form must be the same on every rank.)"""
    return bool(lib().prl_ppo_update_dp_split(int(D), int(A), int(bool(discrete)), int(mini_batch)))


def ppo_update_dpx(params, exp_avg, exp_avg_sq, adam_step, D, A, discrete, S, actions, old_logp,
                   adv, ret, mini_batch, k_epochs, nb_union, inv_count, clip, vf_coef, ent_coef,
                   lr, beta1, beta2, eps, weight_decay, max_norm, loss_out, world, rank, xbufs,
                   seq0, workspace, fine_grained=False, push=False, split=True):
    """The persistent engine as one data-parallel rank: the cross-rank gradient sum runs inside
    the launch over the ranks' IPC-mapped slice buffers `xbufs` (rank order); fine_grained: any
    rank's buffer is fine-grained memory (the flags are then fenced); push: the push form of the
    exchange (every rank writes its slice and flag into every rank's buffer and polls its own;
    the head-split kernel only, else the pull form runs); split=False forces the 8-wave kernel
    (the ranks' vote, ppo_update_dp_split) — every rank must pass the same."""
    N = int(S.shape[0])
    arr = (ctypes.c_void_p * len(xbufs))(*[ctypes.c_void_p(getattr(x, "value", x)) for x in xbufs])
    _check(lib().prl_ppo_update_dpx(
        _dev(params, torch.float32, "params"), _dev(exp_avg, torch.float32, "exp_avg"),
        _dev(exp_avg_sq, torch.float32, "exp_avg_sq"), _dev(adam_step, torch.float32, "adam_step"),
        int(D), int(A), int(bool(discrete)), _dev(S, torch.float32, "S"),
        _dev(actions, torch.float32, "actions"), _dev(old_logp, torch.float32, "old_logp"),
        _dev(adv, torch.float32, "adv"), _dev(ret, torch.float32, "ret"), N, int(mini_batch),
        int(k_epochs), int(nb_union), _dev(inv_count, torch.float32, "inv_count"), float(clip),
        float(vf_coef), float(ent_coef), float(lr), float(beta1), float(beta2), float(eps),
        float(weight_decay), float(max_norm), _dev(loss_out, torch.float32, "loss_out"),
        int(world), int(rank), ctypes.cast(arr, ctypes.c_void_p), int(seq0),
        int(bool(fine_grained)) | (int(bool(push)) << 1) | (0 if split else 4),
        _dev(workspace, torch.uint8, "workspace"),
        workspace.numel(),
        _stream()),
        "prl_ppo_update_dpx")


def ppo_image_floats(D, A, discrete) -> int:
    return int(lib().prl_ppo_image_floats(int(D), int(A), int(bool(discrete))))


def ppo_image(D, A, discrete, params, exp_avg, exp_avg_sq, img_p, img_m, img_v, to_image):
    _check(lib().prl_ppo_image(int(D), int(A), int(bool(discrete)),
                               _dev(params, torch.float32, "params"),
                               _dev(exp_avg, torch.float32, "exp_avg"),
                               _dev(exp_avg_sq, torch.float32, "exp_avg_sq"),
                               _dev(img_p, torch.float32, "img_p"), _dev(img_m, torch.float32, "img_m"),
                               _dev(img_v, torch.float32, "img_v"), int(bool(to_image)), _stream()),
           "prl_ppo_image")


def ppo_evaluate(params, D, A, discrete, S, actions, logp, V, entropy=None):
    """ActorCritic.get_evaluate over all rows with the fused engine's forward arithmetic."""
    N = int(S.shape[0])
    _check(lib().prl_ppo_evaluate(_dev(params, torch.float32, "params"), int(D), int(A),
                                  int(bool(discrete)), _dev(S, torch.float32, "S"),
                                  _dev(actions, torch.float32, "actions"), N,
                                  _dev(logp, torch.float32, "logp"), _dev(V, torch.float32, "V"),
                                  _dev(entropy, torch.float32, "entropy"), _stream()),
           "prl_ppo_evaluate")
