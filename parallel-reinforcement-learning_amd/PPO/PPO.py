"""PPO — drop-in for the reference's PPO/PPO.py:13-283 on MI355X.

Same constructor (14 kwargs, same defaults), attributes and methods.  What changes is where the
work runs in learn() (PPO.py:122-260):
  * the rollout memory is already env-major on the device (no per-transition numpy stacking);
  * policy_old's log-probs / values are evaluated in large chunks (per-row MLP: same values);
  * RND intrinsic reward: fused HIP kernel (prl_rnd_forward);
  * GAE(lambda) + advantages: one single-pass HIP segmented scan (prl_gae), bit-exact with the
    reference's float32 loop, which is O(N^2) there (list.insert(0), PPO.py:116);
  * advantage normalisation: f64 statistics from the GAE pass + HIP normalise (prl_adv_normalize);
  * the clipped surrogate + value loss forward/backward: HIP (prl_ppo_surrogate_fwd/bwd) behind
    a torch.autograd.Function; the MLP backward, clip_grad_norm_(2.0) and AdamW stay PyTorch;
  * minibatches are zero-copy slices of the device tensors, sequential and unshuffled, last
    partial batch kept (the reference's DataLoader semantics, PPO.py:98-105).
Data parallel (torch.distributed, one process per GPU, RCCL): every rank learns on its own
rollout; advantage statistics and the flat gradient of every optimizer step are all-reduced,
and global minibatch j is the union of the ranks' j-th slices (multi-GPU).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.distributed as tdist
from torch import nn, optim
from tqdm import tqdm

import prl_native

from .ActorCritic import ActorCritic
from .Memory import Memory
from .RND import RND

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _require_gpu(what):
    if not torch.cuda.is_available():
        raise RuntimeError(f"{what} runs on the GPU through libprl_hip.so; no GPU is visible")


class SurrogateLoss(torch.autograd.Function):
    """PPO.py:225-249 as one HIP forward (loss + per-sample gradient) and one HIP scale in
    backward.  Returns the minibatch mean loss (what the reference back-propagates)."""

    @staticmethod
    def forward(ctx, logp, old_logp, adv, V, ret, entropy, clip, vf_coef, ent_coef, ops):
        logp = logp.contiguous()
        V = V.contiguous()
        loss = torch.empty((), dtype=torch.float32, device=logp.device)
        dl = torch.empty_like(logp)
        dv = torch.empty_like(V)
        ops.surrogate_fwd(logp, old_logp.contiguous(), adv.contiguous(), V, ret.contiguous(),
                          entropy.reshape(()).contiguous(), clip, vf_coef, ent_coef, loss, dl, dv)
        ctx.save_for_backward(dl, dv)
        ctx.ops = ops
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        dl, dv = ctx.saved_tensors
        gl = torch.empty_like(dl)
        gv = torch.empty_like(dv)
        ctx.ops.surrogate_bwd(grad_out.reshape(()).contiguous(), dl, dv, gl, gv)
        return gl, None, None, gv, None, None, None, None, None, None


class PPO:
    def __init__(self, is_continuous: bool, observ_dim: int, action_dim: int,
                 action_scaling: float = None, lr: float = 0.001, k_epochs: int = 7,
                 policy_clip: float = 0.2, GAE_lambda: float = 0.95, gamma: float = 0.995,
                 batch_size: int = 1024, mini_batch_size: int = 64, use_RND: bool = False,
                 beta: float = 0.001):
        self.device = device
        self.policy = ActorCritic(is_continuous, observ_dim, action_dim, device=self.device)
        self.policy_old = ActorCritic(is_continuous, observ_dim, action_dim, device=self.device)
        if use_RND:
            self.rnd = RND(in_features=observ_dim, out_features=observ_dim, beta=beta,
                           device=self.device)
        self.memory = Memory()
        self.policy_old.load_state_dict(self.policy.state_dict())
        self.policy.train()
        self.policy_old.eval()
        if use_RND:
            self.rnd.eval()
        self.loss_fn = nn.SmoothL1Loss()
        self.optimizer = self._make_optimizer(lr)

        self.is_continuous = is_continuous
        self.action_scaling = action_scaling
        self.use_RND = use_RND
        self.beta = beta
        self.lr = lr
        self.policy_clip = policy_clip
        self.k_epochs = k_epochs
        self.GAE_lambda = GAE_lambda
        self.gamma = gamma
        self.batch_size = batch_size
        self.mini_batch_size = mini_batch_size
        self.observ_dim = observ_dim
        self.action_dim = action_dim

        # engine knobs (not in the reference API)
        self.eval_chunk = 1 << 18          # rows per policy_old evaluation chunk
        self.value_coef, self.entropy_coef = 0.5, 0.01  # PPO.py:245
        self.show_progress = True
        self.last_loss = None
        self._ops = prl_native              # HIP entry points (tests may substitute a fake)
        self.use_fused = True               # whole update loop in one persistent HIP kernel
        self.use_fused_dp = True            # world > 1: stepped engine + all-reduce per step
        self.use_graphs = True              # else: replay one captured optimizer step per minibatch
        self.graph_min_steps = 16           # below this many graphable steps, stay eager
        self._flat_grad = None
        self._sync_initial_weights()

    def _make_optimizer(self, lr):
        """AdamW (PPO.py:53-56).  On the GPU: capturable (step count on device, so the step can
        live in a HIP graph) and the fused single-kernel implementation when available."""
        params = list(self.policy.parameters())
        if params[0].is_cuda:
            for kw in (dict(capturable=True, fused=True), dict(capturable=True, foreach=True)):
                try:
                    return optim.AdamW(params=params, lr=lr, **kw)
                except (RuntimeError, TypeError, ValueError):
                    continue
        return optim.AdamW(params=params, lr=lr)

    # ---------------------------------------------------------------- data parallel helpers
    @staticmethod
    def _world():
        return tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1

    @staticmethod
    def _device_collectives():
        return tdist.get_backend() == "nccl"   # RCCL on ROCm: device tensors directly

    @classmethod
    def all_reduce(cls, t):
        """SUM over ranks in place (RCCL on device tensors; gloo through a host copy)."""
        if cls._device_collectives() or not t.is_cuda:
            tdist.all_reduce(t)
        else:
            h = t.cpu()
            tdist.all_reduce(h)
            t.copy_(h)
        return t

    def _sync_initial_weights(self):
        if self._world() > 1:
            for m in (self.policy, self.policy_old) + ((self.rnd,) if self.use_RND else ()):
                for t in list(m.parameters()) + list(m.buffers()):
                    if self._device_collectives() or not t.is_cuda:
                        tdist.broadcast(t.data, src=0)
                    else:
                        h = t.data.cpu()
                        tdist.broadcast(h, src=0)
                        t.data.copy_(h)

    def _ensure_flat_grads(self):
        """Make every policy gradient a view of one flat buffer: one all-reduce per step."""
        params = [p for p in self.policy.parameters() if p.requires_grad]
        total = sum(p.numel() for p in params)
        if self._flat_grad is None or self._flat_grad.numel() != total:
            self._flat_grad = torch.zeros(total, dtype=torch.float32, device=params[0].device)
        off = 0
        base = self._flat_grad.data_ptr()
        for p in params:  # re-attach views a set_to_none / graph epoch may have replaced
            if p.grad is None or p.grad.data_ptr() != base + 4 * off:
                p.grad = self._flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        return self._flat_grad

    # ---------------------------------------------------------------- reference API
    @torch.no_grad()
    def get_action(self, state: torch.Tensor) -> np.ndarray:  # PPO.py:81-96
        state = state.to(dtype=torch.float32, device=self.device)
        dist = self.policy_old.get_dist(state)
        action = dist.sample()
        if self.is_continuous:
            action = torch.tanh(action).mul(self.action_scaling)
        return action.cpu().numpy()

    @torch.no_grad()
    def dist_params(self, obs: torch.Tensor) -> torch.Tensor:
        """Distribution rows for the fused device worker step (probs, or [mu | std]).  Wide nets
        (outside the persistent engine: C5's D = 348) on the native path: one prl_ppo_wide_dist
        launch instead of ~12 PyTorch / hipBLASLt kernels per vector step."""
        flat = self._dist_flat(obs)
        if flat is None:
            return self.policy_old.dist_params(obs)
        A = self.action_dim
        out = torch.empty(obs.shape[0], A if not self.is_continuous else 2 * A,
                          dtype=torch.float32, device=obs.device)
        prl_native.ppo_wide_dist(flat, obs.shape[1], A, not self.is_continuous,
                                 obs.contiguous(), out)
        return out

    @torch.no_grad()
    def dist_params_at(self, traj_obs: torch.Tensor, step_dev: torch.Tensor, rows: int):
        """dist_params(traj_obs[k]) with k = step_dev[0] read on the device (AsyncPPO's captured
        vector step): the wide nets' prl_ppo_wide_dist_at reads the rows in place.  The flat
        parameter buffer is NOT re-gathered here: the caller refreshes it once per rollout
        (refresh_dist_params).  None when the native distribution path does not apply."""
        D = traj_obs.shape[-1]
        S = traj_obs.reshape(-1, D)
        flat = self._dist_flat(S[:rows], gather=False)
        if flat is None:
            return None
        A = self.action_dim
        out = torch.empty(rows, A if not self.is_continuous else 2 * A,
                          dtype=torch.float32, device=S.device)
        prl_native.ppo_wide_dist_at(flat, D, A, not self.is_continuous, S, rows, step_dev, out)
        return out

    @torch.no_grad()
    def refresh_dist_params(self, obs: torch.Tensor) -> None:
        """Gather policy_old's current parameters into the flat buffer dist_params_at reads."""
        self._dist_flat(obs)

    def rollout_params(self, obs: torch.Tensor):
        """policy_old's parameters as one flat vector for AsyncPPO's persistent rollouts
        (prl_wide_rollout: the wide continuous nets, same rule as dist_params_at; and the CartPole
        net, prl_cartpole_rollout), gathered now; None when neither applies (PRL_CP_ROLLOUT=0
        keeps CartPole on the per-step path)."""
        with torch.no_grad():
            if (not self.is_continuous and self.observ_dim == 4 and self.action_dim == 2
                    and obs.is_cuda and os.environ.get("PRL_CP_ROLLOUT", "1") != "0"
                    and type(self.policy_old).dist_params is ActorCritic.dist_params):
                params = [p.detach().reshape(-1) for p in self.policy_old.parameters()]
                if sum(p.numel() for p in params) != 9027 or params[0].dtype != torch.float32:
                    return None
                flat = getattr(self, "_cp_flat", None)
                if flat is None or flat.device != params[0].device:
                    flat = self._cp_flat = torch.empty(9027, dtype=torch.float32, device=params[0].device)
                torch.cat(params, out=flat)
                return flat
            return self._dist_flat(obs)

    def _dist_flat(self, obs, gather: bool = True):
        """policy_old's parameters gathered into one persistent flat buffer for
        prl_ppo_wide_dist, or None when the native distribution path does not apply.  The gather
        runs on every dist_params call (one small kernel) so a CUDA graph that captured it
        always reads the current weights; dist_params_at (gather=False) leaves it to the caller."""
        if (not obs.is_cuda or obs.dtype != torch.float32 or obs.dim() != 2
                or os.environ.get("PRL_WIDE_DIST", "1") != "1"):
            return None
        from .update import wide_info
        if wide_info(self, obs.shape[1]) is None:
            return None
        # the persistent engine's small nets (C2 / C3: D <= 64) keep the PyTorch forward: the
        # wide tile kernel (16-row tiles over 256 workgroups) took 61.5 us per C2 vector step,
        # the rollout 151 -> 143 M env-steps/s (profiles/r03_final_bench_kernel_stats.md)
        if prl_native.ppo_update_info(obs.shape[1], self.action_dim, not self.is_continuous,
                                      self.mini_batch_size) is not None:
            return None
        params = [p.detach().reshape(-1) for p in self.policy_old.parameters()]
        n = sum(p.numel() for p in params)
        flat = getattr(self, "_dist_flat_buf", None)
        if flat is None or flat.numel() != n or flat.device != obs.device:
            flat = torch.empty(n, dtype=torch.float32, device=obs.device)
            self._dist_flat_buf = flat
            gather = True
        if gather:
            torch.cat(params, out=flat)
        return flat

    def batch_packer(self, values, batch_size: int):  # PPO.py:98-105 (DataLoader, no shuffle)
        def split(v):
            if not isinstance(v, torch.Tensor):
                v = torch.as_tensor(np.asarray(v))
            return list(v.split(batch_size))
        if isinstance(values, torch.Tensor):
            return split(values)
        if isinstance(values, list):
            return [split(v) for v in values]
        return split(values)

    def compute_gae(self, rewards, dones, state_values, next_value):  # PPO.py:107-120
        """Same float32 results as the reference loop, from one HIP scan.  numpy inputs ->
        list of np.float32 (the reference's return type); device tensors -> tensor."""
        _require_gpu("PPO.compute_gae")
        as_list = not isinstance(state_values, torch.Tensor)
        dev = self.device

        def t(x):
            return torch.as_tensor(np.asarray(x, dtype=np.float32) if as_list else x,
                                   dtype=torch.float32).to(dev).contiguous()
        r, d, V = t(rewards), t(dones), t(state_values)
        nv = t(np.asarray([next_value], np.float32) if as_list else
               torch.as_tensor(next_value, dtype=torch.float32).reshape(1))
        ret = torch.empty_like(V)
        self._ops.gae(r, d, V, nv, self.gamma, self.GAE_lambda, ret)
        if as_list:
            return list(ret.cpu().numpy())
        return ret

    def _fused_path(self, world):
        """The fused engine runs the update (one persistent launch on one GPU; stepped, with an
        all-reduce per optimizer step, on several)."""
        return self.use_fused and self.device.type == "cuda" and (world == 1 or self.use_fused_dp)

    @torch.no_grad()
    def _evaluate_old(self, S, A, world=1):
        """policy_old.get_evaluate over the batch (PPO.py:127-154).  When the fused engine runs
        the update, it also evaluates here, so both log-probs come from the same arithmetic and
        the first minibatch sees ratio == 1 exactly, as in the reference.  The same holds for
        the wide nets (prl_ppo_wide_evaluate) on every minibatch the wide step runs: all of them
        on one GPU; with world > 1, the graphed full minibatches only — the ragged tail after
        n_graph runs _eager_step's autograd forward, whose first-step ratios are 1 to float32
        rounding (~1e-7), not bit-exactly."""
        if self._fused_path(world) and S.is_cuda:
            eng = self._fused_engine()
            if eng is not None:
                return eng.evaluate(self.policy_old, S, A)
        if S.is_cuda and self.use_graphs:
            from .update import wide_info
            if wide_info(self, S.shape[1]) is not None:
                # the wide step updates on these rows: its own forward arithmetic here too
                flat = torch.cat([p.detach().reshape(-1) for p in self.policy_old.parameters()])
                A2 = (A if A.dim() == 2 else A.reshape(-1, 1)).float().contiguous()
                logp = torch.empty(S.shape[0], dtype=torch.float32, device=S.device)
                V = torch.empty_like(logp)
                prl_native.ppo_wide_evaluate(flat, S.shape[1], self.action_dim,
                                             not self.is_continuous, S.contiguous(), A2, logp, V)
                return logp, V
        lps, vs = [], []
        for lo in range(0, S.shape[0], self.eval_chunk):
            lp, v, _ = self.policy_old.get_evaluate(S[lo:lo + self.eval_chunk],
                                                    A[lo:lo + self.eval_chunk])
            lps.append(lp)
            vs.append(v)
        cat = (lambda x: x[0]) if len(lps) == 1 else torch.cat
        return cat(lps).float().contiguous(), cat(vs).float().contiguous()

    def learn(self):  # PPO.py:122-260
        world = self._world()
        n_local = len(self.memory)
        if world > 1:
            ns = torch.tensor([n_local], dtype=torch.int64,
                              device=self.device if self._device_collectives() else "cpu")
            gathered = [torch.zeros_like(ns) for _ in range(world)]
            tdist.all_gather(gathered, ns)
            n_ranks = [int(x.item()) for x in gathered]
        else:
            n_ranks = [n_local]
        if sum(n_ranks) < self.batch_size:
            return
        _require_gpu("PPO.learn") if self._ops is prl_native else None
        S, A, R, Dn = self.memory.device_tensors(self.device)
        N = S.shape[0]
        old_logp, old_V = self._evaluate_old(S, A, world)

        if self.use_RND:
            r_int = self.rnd.compute_intrinsic_reward(S)
            R = R + r_int                                   # PPO.py:171 (float32 add)
            if world > 1:   # union minibatches over the ranks, predictor gradient all-reduced
                mb = self.mini_batch_size
                nbr = max(-(-n // mb) for n in n_ranks)
                counts = [sum(min(mb, max(0, n - j * mb)) for n in n_ranks) for j in range(nbr)]
                self.rnd.update_pred(self.batch_packer(S, mb), self.all_reduce, counts)
            else:
                self.rnd.update_pred(self.batch_packer(S, self.mini_batch_size))
        self.memory.clear()

        returns = torch.empty_like(old_V)
        adv = torch.empty_like(old_V)
        sums = torch.zeros(2, dtype=torch.float64, device=self.device)
        self._ops.gae(R, Dn, old_V, old_V[-1:], self.gamma, self.GAE_lambda, returns, adv, sums)
        if world > 1:
            self.all_reduce(sums)
        self._ops.adv_normalize(adv, sums, float(sum(n_ranks)), 1e-8, adv)

        self._update(S, A, old_logp, adv, returns, n_ranks)
        self.policy_old.load_state_dict(self.policy.state_dict())

    def _fused_engine(self):
        """The fused update engine for this policy / mini_batch (None: shape outside it)."""
        eng = getattr(self, "_engine", None)
        if eng is not None and eng.mini_batch == self.mini_batch_size:
            return eng
        if eng is not None:   # mini_batch changed: release its RCCL comm / slice buffers first
            eng.close()
        from .engine import FusedUpdate
        try:
            self._engine = FusedUpdate(self, self.mini_batch_size)
        except ValueError:
            self._engine = None
        return self._engine

    def _update(self, S, A, old_logp, adv, returns, n_ranks):
        """k_epochs x sequential minibatches (PPO.py:219-255).  One GPU: the whole loop is one
        persistent HIP kernel (engine.py).  Otherwise full minibatches that every rank has replay
        one captured HIP graph (update.py); the rest run eagerly, in order."""
        mb = self.mini_batch_size
        world = len(n_ranks)
        self._last_update_inputs = (S, A, old_logp, adv, returns)   # references (tests, debugging)
        if self._fused_path(world) and S.is_cuda:
            eng = self._fused_engine()
            if eng is not None:
                if world == 1:
                    self.last_loss = eng.run(S, A, old_logp, adv, returns, self.k_epochs).clone()
                    self.last_update_path = "fused"
                else:
                    comm = eng.dp_comm()
                    self.last_loss = eng.run_stepped(S, A, old_logp, adv, returns, self.k_epochs,
                                                     n_ranks, self.all_reduce, comm=comm).clone()
                    self.last_update_path = ("fused-dp" + ("-native" if comm is not None else "")
                                             + ("-persistent" if getattr(eng, "_xbufs", None)
                                                else ""))
                self.last_graph_replays = 0
                return
        self.last_update_path = "graph" if self.use_graphs else "eager"
        nb = max(-(-n // mb) for n in n_ranks)
        counts = [sum(min(mb, max(0, n - j * mb)) for n in n_ranks) for j in range(nb)]
        n_graph = min(n // mb for n in n_ranks)
        from .update import GraphedUpdate, wide_info
        # nets the wide step covers (C5's D = 348 / A = 17) always go through it, however few
        # steps there are (GraphedUpdate captures a graph only past its two eager warm-up steps)
        use_graph = (self.use_graphs and S.is_cuda
                     and (self.k_epochs * n_graph >= self.graph_min_steps
                          or wide_info(self, S.shape[1]) is not None))
        graphed = None
        if use_graph:
            scales = None
            if world > 1:
                scales = torch.tensor([mb / counts[j] for j in range(n_graph)],
                                      dtype=torch.float32, device=S.device)
            graphed = GraphedUpdate(self, S, A, old_logp, adv, returns, scales)
        self._last_graphed = graphed        # (bench.py re-times its wide step)
        pbar = tqdm(total=sum(n_ranks) * self.k_epochs, leave=False,
                    disable=not self.show_progress or (world > 1 and tdist.get_rank() != 0))
        loss = None
        # one GPU, wide step: every minibatch is a few native launches whose ~250 us of GPU time
        # hides their host enqueue, so they run eagerly in order (no warm-up steps, no capture
        # per learn); the captured graph stays for data-parallel ranks (all-reduce per step)
        eager_wide = (graphed is not None and graphed.wide is not None and world == 1
                      and os.environ.get("PRL_WIDE_GRAPH", "0") != "1")
        for _ in range(self.k_epochs):
            j0 = 0
            if eager_wide:
                pass
            elif graphed is not None:
                j0 = graphed.run_epoch(n_graph)
                loss = graphed.loss_out
                pbar.update(sum(counts[:j0]))
            for j in range(j0, nb):
                if graphed is not None and graphed.wide is not None and world == 1:
                    loss = graphed.wide_step(j)
                    pbar.update(counts[j])
                    continue
                fa = graphed.fa if graphed is not None else None
                if fa is not None:   # torch's AdamW takes this step: hand it the native state
                    fa.sync()
                out = self._eager_step(S, A, old_logp, adv, returns, j, counts[j], world)
                if fa is not None:
                    fa.prepare()
                loss = out if out is not None else loss
                pbar.update(counts[j])
        if graphed is not None:
            graphed.finish()
        self.last_loss = loss.detach().clone() if loss is not None else None
        self.last_graph_replays = graphed.replays if graphed is not None else 0
        if loss is not None and self.show_progress:
            pbar.set_description(f"Loss: {float(self.last_loss): .6f}")
        pbar.close()

    def _eager_step(self, S, A, old_logp, adv, returns, j, count_j, world):
        """One optimizer step on minibatch j (this rank's rows [j*mb, (j+1)*mb) ∩ [0, N))."""
        mb = self.mini_batch_size
        lo, hi = j * mb, min((j + 1) * mb, S.shape[0])
        params = [p for p in self.policy.parameters() if p.requires_grad]
        flat = self._ensure_flat_grads() if world > 1 else None
        if flat is not None:
            flat.zero_()
        else:
            self.optimizer.zero_grad()
        loss = None
        if lo < hi:
            logp, V, H = self.policy.get_evaluate(S[lo:hi], A[lo:hi])
            loss = SurrogateLoss.apply(logp, old_logp[lo:hi], adv[lo:hi], V, returns[lo:hi], H,
                                       self.policy_clip, self.value_coef, self.entropy_coef,
                                       self._ops)
            (loss * ((hi - lo) / count_j) if world > 1 else loss).backward()
        if flat is not None:
            self.all_reduce(flat)
        nn.utils.clip_grad_norm_(params, 2.0)
        self.optimizer.step()
        return loss

    def load_weights(self, path: str):  # PPO.py:262-277
        try:
            self.policy.load_state_dict(torch.load(os.path.join(path, "Policy_weights.pth"),
                                                   weights_only=True, map_location=self.device))
            self.policy_old.load_state_dict(self.policy.state_dict())
            if self.use_RND:
                self.rnd.load_state_dict(torch.load(os.path.join(path, "RND_weights.pth"),
                                                    weights_only=True, map_location=self.device))
        except FileNotFoundError:
            pass

    def save_weights(self, path: str):  # PPO.py:279-283
        torch.save(self.policy.state_dict(), os.path.join(path, "Policy_weights.pth"))
        if self.use_RND:
            torch.save(self.rnd.state_dict(), os.path.join(path, "RND_weights.pth"))
