"""Actor-critic MLP — stays in PyTorch-ROCm (BASELINE.json north star).

Same module tree, parameter names and initialisation as the reference's PPO/ActorCritic.py:13-80
so `Policy_weights.pth` state_dicts load either way (SURVEY.md §3.5 keys):
  model = Linear(obs, 64, bias=False) -> GroupNorm(8, 64) -> SiLU
  discrete: actor  = Linear(64,64,nobias) -> GN -> SiLU -> Linear(64, A) -> Softmax
  continuous: mu_head / log_std_head = Linear(64,64,nobias) -> GN -> SiLU -> Linear(64, A)
  critic = Linear(64,64,nobias) -> GN -> SiLU -> Linear(64, 1)
The continuous policy is the reference's MultivariateNormal(mu, diag(std^2)) with
std = softplus(clamp(log_std, -2, 2)) (ActorCritic.py:90-102); it is evaluated as the equivalent
diagonal Normal (Independent(Normal(mu, std), 1)): identical density/entropy, no batched
Cholesky per minibatch.  GroupNorm + SiLU run as one fused HIP op (layers.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import distributions, nn

import prl_native

from .layers import GroupNormSiLU, Linear, hidden_block as _block


class _CategoricalLogProb(torch.autograd.Function):
    """Categorical(probs).log_prob(actions) + per-row entropy in one HIP kernel each way
    (prl_categorical_fwd/bwd): same formulas as torch.distributions.Categorical, no host sync
    (torch validates the simplex constraint with a host round trip), graph-capturable."""

    @staticmethod
    def forward(ctx, probs, actions):
        probs = probs.contiguous()
        actions = actions.to(torch.float32).contiguous()
        logp = torch.empty(probs.shape[0], dtype=torch.float32, device=probs.device)
        ent = torch.empty_like(logp)
        prl_native.categorical_fwd(probs, actions, logp, ent)
        ctx.save_for_backward(probs, actions)
        ctx.mark_non_differentiable(ent)
        return logp, ent

    @staticmethod
    def backward(ctx, dlogp, dent):
        probs, actions = ctx.saved_tensors
        dprobs = torch.empty_like(probs)
        prl_native.categorical_bwd(probs, actions, dlogp.contiguous(), dprobs)
        return dprobs, None


class ActorCritic(nn.Module):
    def __init__(self, is_continuous: bool, observ_dim: int, action_dim: int, device=None):
        super().__init__()
        self.is_continuous = is_continuous
        self.model = nn.Sequential(*_block(observ_dim, 64))
        if is_continuous:
            self.mu_head = nn.Sequential(*_block(64, 64), Linear(64, action_dim))
            self.log_std_head = nn.Sequential(*_block(64, 64), Linear(64, action_dim))
        else:
            self.actor = nn.Sequential(*_block(64, 64), Linear(64, action_dim),
                                       nn.Softmax(dim=-1))
        self.critic = nn.Sequential(*_block(64, 64), Linear(64, 1))
        self.init_weights()
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.to(device)

    def init_weights(self):  # ActorCritic.py:66-80
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.normal_(m.bias, mean=0, std=0.01)
            elif isinstance(m, (nn.GroupNorm, GroupNormSiLU)):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, state):
        raise NotImplementedError

    # -- distribution parameters (device-resident worker: fed to prl_rollout_step) ----------
    def dist_params(self, state: torch.Tensor) -> torch.Tensor:
        """[n, A] probabilities (discrete) or [n, 2A] = [mu | std] (continuous), contiguous."""
        features = self.model(state)
        if self.is_continuous:
            mu = self.mu_head(features)
            std = F.softplus(torch.clamp(self.log_std_head(features), min=-2, max=2))
            return torch.cat([mu, std], dim=-1)
        return self.actor(features).contiguous()

    def _dist(self, features):
        if self.is_continuous:
            mu = self.mu_head(features)
            std = F.softplus(torch.clamp(self.log_std_head(features), min=-2, max=2))
            return distributions.Independent(
                distributions.Normal(mu, std, validate_args=False), 1, validate_args=False)
        return distributions.Categorical(self.actor(features))

    def get_dist(self, state: torch.Tensor):  # ActorCritic.py:85-110
        return self._dist(self.model(state))

    def get_state_value(self, state: torch.Tensor):  # :112-116
        return self.critic(self.model(state)).squeeze(-1)

    def get_evaluate(self, states: torch.Tensor, actions: torch.Tensor):  # :118-146
        features = self.model(states)
        if not self.is_continuous and features.is_cuda:
            log_probs, ent = _CategoricalLogProb.apply(self.actor(features), actions)
            dist_entropy = ent.mean().detach()
        else:
            dist = self._dist(features)
            log_probs = dist.log_prob(actions)
            dist_entropy = dist.entropy().mean().detach()
        state_value = self.critic(features).squeeze(-1)
        return log_probs, state_value, dist_entropy
