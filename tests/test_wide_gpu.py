"""The wide-net optimizer step (csrc/prl_ppo_wide.hip, C-ABI prl_ppo_wide_grad) for shapes outside
the persistent engine — C5's D = 348 / A = 17 continuous net — against
float64 autograd of the reference loss (PPO/PPO.py:216-249: -min(surr1, surr2) + 0.5 SmoothL1 -
0.01 H, mean, backward) on the same parameters and rows.  Gradients differ only by float32
rounding / summation order: each tensor is checked at 1e-4 of its largest entry (the persistent
engine's bar, tests/test_engine_gpu.py); the loss at 1e-5 relative."""
import copy

import numpy as np
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


def _policy(cont, D, A, seed=0):
    from PPO.ActorCritic import ActorCritic
    torch.manual_seed(seed)
    return ActorCritic(cont, D, A, device=torch.device("cuda"))


def _sample(pol, S, seed=9):
    """Actions sampled from the policy's own Gaussian.  Far off-distribution actions (narrow
    std, |a - mu| ~ 1) give |log p| ~ 500 for A = 17, whose float32 rounding alone moves every
    ratio by ~1e-4 (the same conditioning limit as the persistent engine's test)."""
    torch.manual_seed(seed)
    with torch.no_grad():
        return pol.get_dist(S).sample().float().contiguous()


def _rows(pol, cont, N, D, A, spread, seed=3, clip=0.2):
    """Random states / actions, advantages, returns; old log-probs = float64 log-probs + noise of
    `spread` (0: on-policy), nudged 1e-2 away from the clip kinks (the gradient jumps there)."""
    rng = np.random.default_rng(seed)
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.7).astype(np.float32)).cuda()
    if cont:   # actions drawn from the policy, as a rollout stores them: |log p| stays O(A)
        act = _sample(pol, S)
    else:
        act = torch.from_numpy(rng.integers(0, A, size=(N, 1)).astype(np.float32)).cuda()
    adv = torch.from_numpy(rng.normal(size=N).astype(np.float32)).cuda()
    ret = torch.from_numpy(rng.normal(0.3, 1.5, size=N).astype(np.float32)).cuda()
    p64 = copy.deepcopy(pol).cpu().double()
    with torch.no_grad():
        l64, _, _ = p64.get_evaluate(S.cpu().double(), act.cpu().double() if cont else
                                     act.cpu().double().reshape(-1))
    old = l64 + torch.from_numpy(rng.normal(size=N) * spread)
    r = torch.exp(l64 - old)
    near = ((r - (1 - clip)).abs() < 1e-3) | ((r - (1 + clip)).abs() < 1e-3)
    old = torch.where(near, old + 1e-2, old)
    return S, act, old.float().cuda(), adv, ret


def _grad64(pol, cont, S, act, old, adv, ret, clip=0.2, vf=0.5, ent=0.01):
    p64 = copy.deepcopy(pol).cpu().double()
    a = act.cpu().double() if cont else act.cpu().double().reshape(-1)
    logp, V, H = p64.get_evaluate(S.cpu().double(), a)
    ratio = torch.exp(torch.clamp(logp - old.cpu().double(), -20, 20))
    A_ = adv.cpu().double()
    s1, s2 = ratio * A_, torch.clamp(ratio, 1 - clip, 1 + clip) * A_
    loss = (-torch.min(s1, s2) + vf * nn.SmoothL1Loss()(V, ret.cpu().double()) - ent * H).mean()
    loss.backward()
    return [p.grad for p in p64.parameters()], float(loss.detach())


def _wide(pol, cont, D, A, S, act, old, adv, ret, mb, j):
    import prl_native
    info = prl_native.ppo_wide_info(D, A, not cont, mb)
    assert info is not None
    n_params, part_floats, grid = info
    params = list(pol.parameters())
    assert n_params == sum(p.numel() for p in params)
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    grad = torch.full((n_params,), float("nan"), device="cuda")
    loss = torch.zeros(1, device="cuda")
    part = torch.full((part_floats,), float("nan"), device="cuda")
    cur = torch.tensor([j], dtype=torch.int64, device="cuda")
    prl_native.ppo_wide_grad(flat, D, A, not cont, S, act, old, adv, ret, mb, cur, None, 0.2, 0.5,
                             0.01, grad, loss, part)
    torch.cuda.synchronize()
    out, off = [], 0
    for p in params:
        out.append(grad[off:off + p.numel()].view_as(p).double().cpu())
        off += p.numel()
    return out, float(loss)


CASES = [
    # cont, D, A, N, mb, spread     (C5's net; a ragged minibatch; discrete; D % 4 != 0)
    (True, 348, 17, 1000, 512, 0.3),
    (True, 348, 17, 300, 4096, 0.0),
    (False, 100, 5, 700, 256, 0.5),
    (True, 201, 3, 530, 512, 1.0),
    (False, 66, 30, 257, 128, 0.3),
]


@pytest.mark.parametrize("cont,D,A,N,mb,spread", CASES)
def test_wide_gradient_matches_float64_autograd(cont, D, A, N, mb, spread):
    pol = _policy(cont, D, A)
    S, act, old, adv, ret = _rows(pol, cont, N, D, A, spread)
    nb = -(-N // mb)
    for j in range(nb):
        lo, hi = j * mb, min(N, (j + 1) * mb)
        g64, l64 = _grad64(pol, cont, S[lo:hi], act[lo:hi], old[lo:hi], adv[lo:hi], ret[lo:hi])
        gw, lw = _wide(pol, cont, D, A, S, act, old, adv, ret, mb, j)
        errs = {}
        for (name, _), a, b in zip(pol.named_parameters(), gw, g64):
            assert torch.isfinite(a).all(), name
            errs[name] = float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)
        worst = max(errs.values())
        top = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
        print(j, {k: f"{v:.1e}" for k, v in top})
        assert worst <= 1e-4, (j, [(k, f"{v:.1e}") for k, v in top])
        assert abs(lw - l64) <= 1e-5 * max(1.0, abs(l64)), (lw, l64)


def test_wide_deterministic_and_info_bounds():
    import prl_native
    assert prl_native.ppo_wide_info(348, 17, False, 65536) is not None
    assert prl_native.ppo_wide_info(353, 4, False, 512) is None      # D > 352
    assert prl_native.ppo_wide_info(64, 24, False, 512) is None      # 49 outputs > 48
    pol = _policy(True, 348, 17)
    S, act, old, adv, ret = _rows(pol, True, 4096 + 77, 348, 17, 0.3)
    g1, l1 = _wide(pol, True, 348, 17, S, act, old, adv, ret, 4096, 0)
    g2, l2 = _wide(pol, True, 348, 17, S, act, old, adv, ret, 4096, 0)
    assert l1 == l2
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)


def test_wide_learn_matches_autograd_step_path():
    """learn() on a C5-shaped net through the wide kernel (graphed + the ragged minibatch) against
    the PyTorch autograd step path (PRL_WIDE=0) in function space: log-probs / values on probe
    states after 2 epochs agree to 1e-3 (the persistent engine's function-space bar, in its
    smooth regime: clip 1e3, on-policy actions)."""
    import os
    from PPO import PPO
    D, A = 348, 17
    rng = np.random.default_rng(11)
    N, mb = 3 * 1024 + 200, 1024
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.02).astype(np.float32)).cuda()
    Dn[-1] = 1
    Aa = _sample(_policy(True, D, A), S)   # PPO(...) below builds the same net from seed 0
    out = {}
    for wide in ("1", "0"):
        os.environ["PRL_WIDE"] = wide
        try:
            torch.manual_seed(0)
            p = PPO(True, D, A, action_scaling=1.0, lr=3e-4, k_epochs=2, batch_size=64,
                    mini_batch_size=mb, policy_clip=1e3)   # smooth surrogate (no clip kinks)
            p.show_progress = False
            p.graph_min_steps = 1
            p.memory.push_device(S, Aa, R, Dn)
            p.learn()
            assert p.last_update_path == "graph"
            pol = copy.deepcopy(p.policy).cpu().double()
            with torch.no_grad():
                lp, V, _ = pol.get_evaluate(S[:512].cpu().double(), Aa[:512].cpu().double())
            out[wide] = (lp, V, float(p.last_loss))
        finally:
            os.environ.pop("PRL_WIDE", None)
    (l1, v1, L1), (l0, v0, L0) = out["1"], out["0"]
    el = float((l1 - l0).abs().max()) / (float(l0.abs().max()) + 1.0)
    ev = float((v1 - v0).abs().max()) / (float(v0.abs().max()) + 1.0)
    assert el <= 1e-3 and ev <= 1e-3, (el, ev)
    assert abs(L1 - L0) <= 1e-3 * max(1.0, abs(L0)), (L1, L0)


def test_wide_learn_clip02_relational_to_cpu():
    """The reference's policy_clip = 0.2 on C5's net (D 348, A 17), end to end through learn():
    ratios crossing 0.8 / 1.2 flip single rows' gradient terms, so two valid float32 paths drift
    apart (the persistent engine's test (iii), tests/test_engine_gpu.py).  The check is
    relational: the wide kernel must be (about) as close to the CPU path (PyTorch-CPU autograd +
    AdamW with the oracle's GAE / surrogate, i.e. the reference's arithmetic) as the GPU
    autograd step path (PRL_WIDE=0) is."""
    import os
    from fake_ops import FakeOps
    from PPO import PPO
    from test_engine_gpu import _fdist
    D, A = 348, 17
    rng = np.random.default_rng(12)
    N, mb, k = 3 * 1024 + 200, 1024, 2
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.02).astype(np.float32)).cuda()
    Dn[-1] = 1
    Aa = _sample(_policy(True, D, A), S)

    def make():
        torch.manual_seed(0)
        p = PPO(True, D, A, action_scaling=1.0, lr=3e-4, k_epochs=k, batch_size=64,
                mini_batch_size=mb, policy_clip=0.2)
        p.show_progress = False
        p.graph_min_steps = 1        # the autograd arm graph-replays its steps too
        return p

    runs = {}
    for wide in ("1", "0"):
        os.environ["PRL_WIDE"] = wide
        try:
            p = make()
            p.memory.push_device(S, Aa, R, Dn)
            p.learn()
            torch.cuda.synchronize()
            assert p.last_update_path == "graph"
            assert (p._last_graphed.wide is not None) == (wide == "1")
            runs[wide] = p
        finally:
            os.environ.pop("PRL_WIDE", None)
    c = make()
    c.policy.cpu()
    c.policy_old.cpu()
    c.device = torch.device("cpu")
    c.optimizer = torch.optim.AdamW(c.policy.parameters(), lr=3e-4)
    c._ops = FakeOps()
    c.memory.push_device(S.cpu(), Aa.cpu(), R.cpu(), Dn.cpu())
    c.learn()
    data = (S, Aa)
    d_wc, d_gc = _fdist(runs["1"], c, data), _fdist(runs["0"], c, data)
    print(f"function distance to the CPU path: wide {d_wc:.2e}, autograd {d_gc:.2e}")
    assert d_wc <= 2.0 * d_gc + 1e-4, (d_wc, d_gc)


@pytest.mark.parametrize("cont,D,A", [(True, 348, 17), (False, 100, 5), (True, 201, 3)])
def test_wide_evaluate_matches_get_evaluate_and_row_placement(cont, D, A):
    """prl_ppo_wide_evaluate (learn()'s policy_old pass for the wide nets, PPO.py:127-154) against
    float64 get_evaluate: log-probs within 2e-6 of max |logp| and values within 2e-6 of max |V|
    (float32 rounding; the persistent engine's evaluate bar).  Every row's result depends only on
    that row: the same rows evaluated at other tile positions (a 5-row shift, a ragged count)
    give the same bits — the wide step's loss uses this same arithmetic on the same rows, so the
    first minibatch of learn() sees ratio == 1 exactly, as in the reference."""
    import prl_native
    pol = _policy(cont, D, A, seed=4)
    N = 1000
    S, act, _, _, _ = _rows(pol, cont, N, D, A, 0.0)
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])

    def ev(lo):
        Ss, As = S[lo:].contiguous(), act[lo:].contiguous()
        lp = torch.full((N - lo,), float("nan"), device="cuda")
        V = torch.full((N - lo,), float("nan"), device="cuda")
        prl_native.ppo_wide_evaluate(flat, D, A, not cont, Ss, As, lp, V)
        return lp, V

    lp, V = ev(0)
    lp5, V5 = ev(5)
    torch.cuda.synchronize()
    assert torch.equal(lp[5:], lp5) and torch.equal(V[5:], V5)
    p64 = copy.deepcopy(pol).cpu().double()
    with torch.no_grad():
        l64, v64, _ = p64.get_evaluate(S.cpu().double(), act.cpu().double() if cont else
                                       act.cpu().double().reshape(-1))
    el = float((lp.cpu().double() - l64).abs().max()) / (1.0 + float(l64.abs().max()))
    ev_ = float((V.cpu().double() - v64).abs().max()) / (1.0 + float(v64.abs().max()))
    print(f"logp {el:.1e}, V {ev_:.1e}")
    assert el <= 2e-6 and ev_ <= 2e-6, (el, ev_)


@pytest.mark.parametrize("cont,D,A,N", [(True, 348, 17, 1000), (True, 348, 17, 7),
                                        (False, 100, 5, 1000), (True, 201, 3, 1)])
def test_wide_dist_matches_dist_params(cont, D, A, N):
    """prl_ppo_wide_dist (the rollout's sampling input for the wide nets, AsyncPPO's vector step)
    against float64 ActorCritic.dist_params: probabilities / [mu | std] within 2e-6 of the
    largest entry (float32 rounding); every row depends only on itself (a shifted slice gives
    the same bits)."""
    import prl_native
    pol = _policy(cont, D, A, seed=5)
    torch.manual_seed(11)
    S = torch.randn(N, D, device="cuda")
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    W = 2 * A if cont else A

    def dist(lo):
        out = torch.full((N - lo, W), float("nan"), device="cuda")
        prl_native.ppo_wide_dist(flat, D, A, not cont, S[lo:].contiguous(), out)
        return out

    out = dist(0)
    if N > 3:
        out3 = dist(3)
        torch.cuda.synchronize()
        assert torch.equal(out[3:], out3)
    p64 = copy.deepcopy(pol).cpu().double()
    with torch.no_grad():
        ref = p64.dist_params(S.cpu().double())
    err = float((out.cpu().double() - ref).abs().max()) / (1.0 + float(ref.abs().max()))
    print(f"dist {err:.1e}")
    assert err <= 2e-6, err


def test_ppo_dist_params_native_and_graph_sees_new_weights():
    """PPO.dist_params routes the wide nets through prl_ppo_wide_dist; a CUDA graph that captured
    it (AsyncPPO's vector step) reads policy_old's current weights after load_state_dict."""
    from PPO.PPO import PPO
    ppo = PPO(True, 348, 17, action_scaling=1.0, mini_batch_size=512)
    assert ppo._dist_flat(torch.zeros(2, 348, device="cuda")) is not None
    # the persistent engine's nets (C2 CartPole, C3 Pendulum) keep the PyTorch forward
    assert PPO(False, 4, 2, mini_batch_size=512)._dist_flat(torch.zeros(2, 4, device="cuda")) is None
    assert PPO(True, 3, 1, mini_batch_size=512)._dist_flat(torch.zeros(2, 3, device="cuda")) is None
    torch.manual_seed(2)
    S = torch.randn(64, 348, device="cuda")
    with torch.no_grad():
        ref = ppo.policy_old.dist_params(S)
    assert float((ppo.dist_params(S) - ref).abs().max()) <= 2e-6 * (1 + float(ref.abs().max()))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ppo.dist_params(S)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = ppo.dist_params(S)
    with torch.no_grad():
        for p in ppo.policy.parameters():
            p.add_(0.05 * torch.randn_like(p))
    ppo.policy_old.load_state_dict(ppo.policy.state_dict())
    g.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        ref2 = ppo.policy_old.dist_params(S)
    assert not torch.allclose(ref, ref2)
    assert float((out - ref2).abs().max()) <= 2e-6 * (1 + float(ref2.abs().max()))


def test_wide_dist_at_reads_the_step_in_place():
    """prl_ppo_wide_dist_at (AsyncPPO's captured vector step for the wide nets): rows
    [k*E, (k+1)*E) of the whole [T+1][E][D] observation store with k read on the device give
    exactly prl_ppo_wide_dist's bits on that slice; a k past the store writes nothing."""
    import prl_native
    pol = _policy(True, 348, 17, seed=3)
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    T1, E, D, W = 5, 300, 348, 34
    torch.manual_seed(4)
    S = torch.randn(T1, E, D, device="cuda")
    k_dev = torch.zeros(1, dtype=torch.int64, device="cuda")
    for k in (0, 2, T1 - 1):
        k_dev.fill_(k)
        out = torch.full((E, W), float("nan"), device="cuda")
        prl_native.ppo_wide_dist_at(flat, D, 17, False, S, E, k_dev, out)
        ref = torch.full((E, W), float("nan"), device="cuda")
        prl_native.ppo_wide_dist(flat, D, 17, False, S[k].contiguous(), ref)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), k
    k_dev.fill_(T1)
    out = torch.full((E, W), float("nan"), device="cuda")
    prl_native.ppo_wide_dist_at(flat, D, 17, False, S, E, k_dev, out)
    torch.cuda.synchronize()
    assert bool(torch.isnan(out).all())


def test_wide_graphed_rollout_equals_eager_rollout(monkeypatch):
    """C5's net on the synthetic env: the graphed rollout (distribution read from traj_obs[k] in
    place, parameters gathered once per rollout) gives the eager rollout's memory and scores
    bit for bit, including after learn() changed policy_old between rollouts.  (The per-step
    path: PRL_WIDE_ROLLOUT=0; by default C5 rolls out in one persistent launch, tested below.)"""
    from AsyncTools.AsyncPPO import AsyncPPO
    from PPO import PPO
    outs = []
    monkeypatch.setenv("PRL_WIDE_ROLLOUT", "0")
    for graphed in ("1", "0"):
        monkeypatch.setenv("PRL_ROLLOUT_GRAPH", graphed)
        torch.manual_seed(0)
        p = PPO(True, 348, 17, action_scaling=1.0, batch_size=10**9, mini_batch_size=512)
        a = AsyncPPO("SyntheticHumanoid-v0", p, num_envs=200, seed=5)
        rec = []
        for it in range(3):
            n = a.worker()
            rec.append((n, float(a.reward_score)))
            if it == 1:   # new policy_old weights before the third rollout
                with torch.no_grad():
                    for q in p.policy.parameters():
                        q.add_(0.02 * torch.randn_like(q))
                p.policy_old.load_state_dict(p.policy.state_dict())
        assert (a._graph is not None) == (graphed == "1")
        outs.append((rec, [x.cpu() for x in p.memory.device_tensors("cuda")]))
    (r1, m1), (r0, m0) = outs
    assert r1 == r0
    for x, y in zip(m1, m0):
        assert torch.equal(x, y)


@pytest.mark.parametrize("scale", [1e-3, 1e2])
def test_flat_adamw_matches_torch_clip_and_adamw(scale):
    """prl_flat_adamw (the wide step's optimizer tail: clip_grad_norm_(2.0) + AdamW.step() in one
    launch over flat buffers, PPO.py:248-250; ~37 K parameters = 10 workgroups, the last of which
    clips the gradient and advances the step) against torch's own clip_grad_norm_ + AdamW
    (the reference's defaults: bias corrections from Python doubles) on C5's parameter shapes
    over four steps.  scale 1e-3: norm < 2, no clipping;
    1e2: clipping every step.  The two differ only in float32 rounding (norm summed in float64
    here, the AdamW division as rcp + one Newton step): moments within 1e-5 relative and the
    clipped gradient within 1e-6 relative.  Parameters: the native tail rounds each step's update with fused multiply-adds
    (p * decay, then fma(-step_size, m / denom, p)) where torch rounds mul_ and addcdiv_
    separately: up to ~2 ulps of the parameter per step, so 4 steps stay within 16 ulps of the
    largest parameter (2.4e-7 measured on MI355X at |p| <= 0.3)."""
    import prl_native
    pol = _policy(True, 348, 17)
    shapes = [p.shape for p in pol.parameters()]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in pol.parameters()]
    opt = torch.optim.AdamW(ref, lr=1e-3)   # the reference's AdamW (PPO.py:51-54): defaults
    P = sum(p.numel() for p in ref)
    flat = torch.cat([p.detach().reshape(-1) for p in ref]).contiguous()
    m, v = torch.zeros_like(flat), torch.zeros_like(flat)
    step = torch.zeros(1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(4):
        grad = torch.randn(P, device="cuda", generator=g) * scale
        off = 0
        for p, sh in zip(ref, shapes):
            p.grad = grad[off:off + p.numel()].view(sh).clone()
            off += p.numel()
        tn = torch.nn.utils.clip_grad_norm_(ref, 2.0)
        opt.step()
        gbuf = grad.clone()
        got_n = prl_native.flat_adamw(flat, m, v, step, gbuf, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 2.0)
        torch.cuda.synchronize()
        want_g = torch.cat([p.grad.reshape(-1) for p in ref])
        assert float((gbuf - want_g).abs().max()) <= 1e-6 * float(want_g.abs().max())
        assert abs(float(got_n) - float(tn)) <= 1e-6 * float(tn)   # clip_grad_norm_'s return value
    want = torch.cat([p.detach().reshape(-1) for p in ref])
    ulp = float(torch.finfo(torch.float32).eps) * float(want.abs().max())
    assert float((flat - want).abs().max()) <= 16 * ulp, float((flat - want).abs().max())
    wm = torch.cat([opt.state[p]["exp_avg"].reshape(-1) for p in ref])
    wv = torch.cat([opt.state[p]["exp_avg_sq"].reshape(-1) for p in ref])
    assert float((m - wm).abs().max()) <= 1e-5 * float(wm.abs().max())
    assert float((v - wv).abs().max()) <= 1e-5 * float(wv.abs().max())
    assert float(step.item()) == 4.0


@pytest.mark.parametrize("P", [262_144, 300_003])
def test_flat_adamw_one_and_two_launch_forms(P):
    """prl_flat_adamw at the fused form's largest size (64 workgroups: the last one clips and
    advances the step) and above it (the separate clip launch; P % 4 = 3 exercises the tail)
    against torch's clip_grad_norm_(2.0) + AdamW on one flat Parameter over three clipping steps:
    the same bounds as test_flat_adamw_matches_torch_clip_and_adamw.  The arrival counter
    (total_norm[1]) is back at zero after every call."""
    import prl_native
    g = torch.Generator(device="cuda").manual_seed(9)
    p0 = (torch.rand(P, device="cuda", generator=g) - 0.5) * 0.6
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-3)
    flat = p0.clone()
    m, v = torch.zeros_like(flat), torch.zeros_like(flat)
    step = torch.zeros(1, device="cuda")
    ws = torch.zeros(2, device="cuda")
    for _ in range(3):
        grad = torch.randn(P, device="cuda", generator=g) * 0.1
        ref.grad = grad.clone()
        tn = torch.nn.utils.clip_grad_norm_([ref], 2.0)
        opt.step()
        gbuf = grad.clone()
        got_n = prl_native.flat_adamw(flat, m, v, step, gbuf, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 2.0, ws)
        torch.cuda.synchronize()
        assert float(tn) > 2.0
        assert float((gbuf - ref.grad).abs().max()) <= 1e-6 * float(ref.grad.abs().max())
        assert abs(float(got_n) - float(tn)) <= 1e-6 * float(tn)
        assert int(ws[1:].view(torch.int32).item()) == 0
    ulp = float(torch.finfo(torch.float32).eps) * float(ref.detach().abs().max())
    assert float((flat - ref.detach()).abs().max()) <= 16 * ulp
    wm, wv = opt.state[ref]["exp_avg"], opt.state[ref]["exp_avg_sq"]
    assert float((m - wm).abs().max()) <= 1e-5 * float(wm.abs().max())
    assert float((v - wv).abs().max()) <= 1e-5 * float(wv.abs().max())
    assert float(step.item()) == 3.0


def test_flat_adamw_graph_replay_equals_eager():
    """The one-launch flat AdamW captured in a HIP graph (the data-parallel wide step replays it
    per minibatch): three replays give the same bits as three eager calls — parameters, moments,
    the clipped gradient, the norm and the step — and the arrival counter is zero after each."""
    import prl_native
    P = 37_347   # C5's policy: 10 workgroups, a P % 4 tail of 3
    g = torch.Generator(device="cuda").manual_seed(13)
    p0 = (torch.rand(P, device="cuda", generator=g) - 0.5) * 0.6
    grads = [torch.randn(P, device="cuda", generator=g) * 0.5 for _ in range(3)]

    def fresh():
        return [p0.clone(), torch.zeros(P, device="cuda"), torch.zeros(P, device="cuda"),
                torch.zeros(1, device="cuda"), torch.zeros(2, device="cuda")]

    e = fresh()
    e_g = []
    for gr in grads:
        gb = gr.clone()
        prl_native.flat_adamw(e[0], e[1], e[2], e[3], gb, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 2.0, e[4])
        e_g.append(gb)
    c = fresh()
    gbuf = torch.empty(P, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            prl_native.flat_adamw(c[0], c[1], c[2], c[3], gbuf, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 2.0,
                                  c[4])
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for i, gr in enumerate(grads):
        gbuf.copy_(gr)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(gbuf, e_g[i])
        assert int(c[4][1:].view(torch.int32).item()) == 0
    for a, b in zip(c, e):
        assert torch.equal(a[:1] if a.numel() == 2 else a, b[:1] if b.numel() == 2 else b)
    assert float(c[3].item()) == 3.0


def test_wide_learn_native_adam_equals_torch_adam(monkeypatch):
    """learn() on C5's net through the wide step with the native optimizer tail (default) and
    with torch's clip_grad_norm_ + fused AdamW (PRL_WIDE_ADAM=0): same data, two epochs with a
    ragged minibatch; the learned function agrees (log-probs / values on probe states, 1e-3 as
    the wide step's other learn() comparisons: continuous log-probs amplify float32 rounding), the
    optimizer's step count and state tensors stay consistent across two learn() calls."""
    from PPO import PPO
    rng = np.random.default_rng(2)
    N, D, A = 3 * 512 + 77, 348, 17
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    Aa = torch.from_numpy(np.tanh(rng.normal(size=(N, A))).astype(np.float32)).cuda()
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.05).astype(np.float32)).cuda()
    Dn[-1] = 1
    outs = []
    for native in ("1", "0"):
        monkeypatch.setenv("PRL_WIDE_ADAM", native)
        torch.manual_seed(0)
        p = PPO(True, D, A, action_scaling=1.0, k_epochs=2, batch_size=64, mini_batch_size=512)
        p.show_progress = False
        for _ in range(2):
            p.memory.push_device(S, Aa, R, Dn)
            p.learn()
        torch.cuda.synchronize()
        assert p._last_graphed.wide is not None
        assert (p._last_graphed.fa is not None) == (native == "1")
        st = p.optimizer.state[next(p.policy.parameters())]
        assert float(st["step"]) == 2 * 2 * 4
        with torch.no_grad():
            lp, V, _ = copy.deepcopy(p.policy).double().get_evaluate(S[:1024].double(),
                                                                     Aa[:1024].double())
        outs.append((lp.cpu(), V.cpu()))
    (l1, v1), (l0, v0) = outs
    assert float((l1 - l0).abs().max()) <= 1e-3 * (1 + float(l0.abs().max()))
    assert float((v1 - v0).abs().max()) <= 1e-3 * (1 + float(v0.abs().max()))


@pytest.mark.parametrize("E,stride,team", [(300, 7, "1"), (5000, 211, "1"), (300, 7, "8"), (300, 7, "0")])
def test_persistent_wide_rollout_matches_per_step_rollout(monkeypatch, E, stride, team):
    """prl_wide_rollout (the whole C5 rollout in ONE launch, each wave stepping 16 envs to the end
    of their episodes) against the per-step path (prl_ppo_wide_dist + prl_rollout_step per vector
    step, PRL_WIDE_ROLLOUT=0, eager) on the same runner seeds and policy, three rollouts with a
    new policy_old before the third: observations, done flags and episode lengths bit for bit (the
    synthetic env's do not depend on the actions); actions to float32 rounding of the two forward
    orders (<= 2e-5 absolute, actions in [-1, 1]); rewards (1 - 0.01 sum a^2) to 1e-5.  The fused
    actions are also checked against a float64 forward of policy_old with the same Philox
    normals (oracle.sample_normal): tanh(mu + std z) to 2e-5.  E = 300: 19 workgroups of 16 envs,
    the last one ragged; E = 5000: 256 workgroups of 20 envs each, so every workgroup refills
    its lanes from its queue as episodes end (the team form's env queue).  team: the launch's
    form (PRL_WIDE_ROLLOUT_TEAM: 1 four waves per tile, the default; 8 eight; 0 one wave per tile)."""
    monkeypatch.setenv("PRL_WIDE_ROLLOUT_TEAM", team)
    import oracle as O
    from AsyncTools.AsyncPPO import AsyncPPO
    from PPO import PPO
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("PRL_WIDE_ROLLOUT", fused)
        monkeypatch.setenv("PRL_ROLLOUT_GRAPH", "0")
        torch.manual_seed(0)
        p = PPO(True, 348, 17, action_scaling=1.0, batch_size=10**9, mini_batch_size=512)
        a = AsyncPPO("SyntheticHumanoid-v0", p, num_envs=E, seed=5)
        rec, mems, pols = [], [], []
        for it in range(3):
            if it == 2:
                with torch.no_grad():
                    for q in p.policy.parameters():
                        q.add_(0.02 * torch.randn_like(q))
                p.policy_old.load_state_dict(p.policy.state_dict())
            seed = (a.sample_seed + a._rollouts * 0xD1B54A32D192ED03) & (2**64 - 1)
            n = a.worker()
            rec.append((n, float(a.reward_score)))
            mems.append([x.cpu().clone() for x in p.memory.device_tensors("cuda")])
            pols.append((copy.deepcopy(p.policy_old).cpu().double(), seed,
                         a.env.t_elapsed.cpu().clone()))
            p.memory.clear()
        outs.append((rec, mems, pols))
    (rf, mf, pf), (rs, ms, _) = outs
    for it in range(3):
        assert rf[it][0] == rs[it][0]
        assert abs(rf[it][1] - rs[it][1]) <= 1e-6 * max(1.0, abs(rs[it][1]))
        (S1, A1, R1, D1), (S0, A0, R0, D0) = mf[it], ms[it]
        assert torch.equal(S1, S0) and torch.equal(D1, D0)
        assert float((A1 - A0).abs().max()) <= 2e-5
        assert float((R1 - R0).abs().max()) <= 1e-5
        # fused actions vs a float64 forward with the kernel's Philox normals
        pol, seed, lens = pf[it]
        lens = lens.numpy().astype(np.int64)
        e_of = np.repeat(np.arange(E), lens)
        t_of = np.concatenate([np.arange(L) for L in lens])
        idx = np.arange(0, len(e_of), stride)      # a sample of the transitions
        with torch.no_grad():
            feats = pol.model(S1[idx].double())
            mu = pol.mu_head(feats)
            sd = torch.nn.functional.softplus(torch.clamp(pol.log_std_head(feats), -2, 2))
        z = torch.tensor([[O.sample_normal(seed, int(e_of[i]), int(t_of[i]), k) for k in range(17)]
                          for i in idx], dtype=torch.float64)
        want = torch.tanh(mu + sd * z)
        assert float((A1[idx].double() - want).abs().max()) <= 2e-5


@pytest.mark.parametrize("N", [200, 1000])
def test_wide_dist_reads_no_stale_lds(N):
    """prl_ppo_wide_dist after every CU's LDS was filled with NaN and after it was filled with 0
    (prl_debug_fill_lds): the same bits, and no NaN — the kernel reads no LDS it did not write in
    its own launch.  (The full GPU suite once saw one row's [mu | std] come out NaN in a C5
    rollout after earlier tests; the row's observations were finite.)"""
    import prl_native
    pol = _policy(True, 348, 17, seed=5)
    torch.manual_seed(3)
    S = torch.randn(N, 348, device="cuda")
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    outs = []
    for fill in (float("nan"), 0.0, float("inf")):
        prl_native.debug_fill_lds(fill)
        out = torch.empty(N, 34, device="cuda")
        prl_native.ppo_wide_dist(flat, 348, 17, False, S, out)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    assert bool(torch.isfinite(outs[1]).all())
    for o in (outs[0], outs[2]):
        bad = ~(o == outs[1]).all(1)
        assert not bool(bad.any()), f"rows differing after a poisoned LDS: {torch.nonzero(bad)[:8].tolist()}"


def test_wide_dist_rows_independent_of_nonfinite_neighbours():
    """A non-finite observation row (a terminal env's never-written row of traj_obs[k], which the
    rollout's distribution pass covers too) leaves every other row's [mu | std] bit for bit
    unchanged.  D = 348 = 16 x 21 + 12: the trunk's last column group reads 4 columns past the
    row end (the next row's first columns under the unpadded row stride); they are zeroed, since
    their zero weights would still turn a NaN there into a NaN output (found in the full GPU suite:
    row 101 of a C5 rollout went NaN through row 102's column 0)."""
    import prl_native
    pol = _policy(True, 348, 17, seed=5)
    torch.manual_seed(4)
    N = 200
    S = torch.randn(N, 348, device="cuda")
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])

    def dist(x):
        out = torch.empty(N, 34, device="cuda")
        prl_native.ppo_wide_dist(flat, 348, 17, False, x, out)
        torch.cuda.synchronize()
        return out.cpu()

    clean = dist(S)
    P = S.clone()
    P[102, :4] = float("nan")
    P[18] = float("nan")
    P[111, 0] = float("inf")
    out = dist(P)
    keep = torch.ones(N, dtype=torch.bool)
    keep[[18, 102, 111]] = False
    assert torch.equal(out[keep], clean[keep])
