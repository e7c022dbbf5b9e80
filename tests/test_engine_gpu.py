"""The fused update engine (csrc/prl_ppo_update.hip, PPO/engine.py) against the per-step path
(PyTorch autograd + HIP GroupNorm/Categorical/surrogate kernels, graph-replayed) on the same
seeded policy and data.  Both follow PPO.py:216-255; they differ only in float32 summation
order (GEMM / gradient reductions), so weights agree to a tolerance, stated per test.
The reference's own learn() is matched by test_stack_gpu::test_learn_on_gpu_matches_reference_learn
(path "fused")."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ATOL = 3e-5   # weights after tens of AdamW steps (lr 1e-3): reduction-order differences only


class _split:
    """Run the block with the engine's head-split latency form on (1) or off (0: the 8-wave
    kernel), restoring the previous setting (prl_ppo_update_set_split)."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        import prl_native
        self.prev = prl_native.ppo_update_set_split(self.mode)

    def __exit__(self, *exc):
        import prl_native
        prl_native.ppo_update_set_split(self.prev)


def _data(N, D, cont, seed=5):
    rng = np.random.default_rng(seed)
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    A = (torch.from_numpy((np.tanh(rng.normal(size=(N, 1))) * 2).astype(np.float32)).cuda() if cont
         else torch.from_numpy((rng.random(N) < 0.5).astype(np.float32)).cuda())
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.05).astype(np.float32)).cuda()
    Dn[-1] = 1
    return S, A, R, Dn


def _run(fused, cont, data, mb, k, learns=1, D=None, A=None, lr=1e-3, clip=0.2):
    from PPO import PPO
    D = D or (3 if cont else 4)
    A = A or (1 if cont else 2)
    torch.manual_seed(0)
    p = PPO(cont, D, A, action_scaling=2.0 if cont else None, lr=lr, k_epochs=k, batch_size=64,
            mini_batch_size=mb, policy_clip=clip)
    p.show_progress = False
    p.use_fused = fused
    for _ in range(learns):
        p.memory.push_device(*data)
        p.learn()
        assert p.last_update_path == ("fused" if fused else "graph")
    return p


def _outputs(p, S, A):
    """log_prob and value of the learned policy on probe states, in float64 on the CPU (the same
    evaluation for both paths)."""
    import copy
    pol = copy.deepcopy(p.policy).cpu().double()
    with torch.no_grad():
        logp, V, _ = pol.get_evaluate(S.cpu().double(), A.cpu().double())
    return logp, V


def _compare_function(pf, pg, data, rtol=1e-4):
    """Adam turns near-zero gradients (e.g. GroupNorm's scale-invariant directions) into
    +-lr steps whose sign is float32 noise, so after a few steps some WEIGHTS differ by O(lr)
    between two equally valid float32 paths although the learned FUNCTION does not: compare
    log-probs and values on probe states."""
    S, A = data[0][:2048], data[1][:2048]
    (lf, vf), (lg, vg) = _outputs(pf, S, A), _outputs(pg, S, A)
    el = float((lf - lg).abs().max()) / (float(lg.abs().max()) + 1.0)
    ev = float((vf - vg).abs().max()) / (float(vg.abs().max()) + 1.0)
    assert el <= rtol and ev <= rtol, (el, ev)


def _compare(pf, pg, atol=ATOL, loss_rtol=1e-4):
    sf, sg = pf.policy.state_dict(), pg.policy.state_dict()
    worst = 0.0
    for key in sf:
        d = float((sf[key] - sg[key]).abs().max())
        worst = max(worst, d)
        assert d <= atol, (key, d)
    lf, lg = float(pf.last_loss), float(pg.last_loss)
    assert abs(lf - lg) <= loss_rtol * max(1.0, abs(lg)), (lf, lg)
    return worst


def _grad_f64(ppo, data, clip_eps=0.2, vf=0.5, ent=0.01, logp_val=None):
    """float64 CPU autograd of the reference loss (PPO.py:216-249) for ONE minibatch = all rows,
    with old_logp / adv / ret recomputed exactly as learn() does (GAE oracle on the GPU's f32
    old values is not needed: the same device tensors are reused).  logp_val: use these
    (float32) log-prob VALUES in the ratio (the gradient flows through the f64 log-probs)."""
    import copy
    from torch import nn
    S, A, old_logp, adv, ret = data
    pol = copy.deepcopy(ppo.policy).cpu().double()
    logp, V, H = pol.get_evaluate(S.cpu().double(), A.cpu().double())
    if logp_val is not None:
        logp = logp - logp.detach() + logp_val.cpu().double()
    ratio = torch.exp(torch.clamp(logp - old_logp.cpu().double(), -20, 20))
    a = adv.cpu().double()
    s1 = ratio * a
    s2 = torch.clamp(ratio, 1 - clip_eps, 1 + clip_eps) * a
    loss = -torch.min(s1, s2) + vf * nn.SmoothL1Loss()(V, ret.cpu().double()) - ent * H
    loss.mean().backward()
    grads = [p.grad.clone() for p in pol.parameters()]
    norm = torch.sqrt(sum((g * g).sum() for g in grads))
    coef = min(2.0 / (float(norm) + 1e-6), 1.0)
    return [g * coef for g in grads]


@pytest.mark.parametrize("cont", [False, True])
def test_fused_gradient_matches_autograd(cont):
    """One optimizer step at lr = 0: parameters stay put and AdamW's first moment is exactly
    (1 - beta1) * clip_coef * grad.  Both GPU paths are compared with a float64 autograd of the
    reference loss on the same minibatch (error relative to each tensor's largest entry)."""
    S, Aa, R, Dn = _data(512, 3 if cont else 4, cont)
    errs = {}
    for fused in (True, False):
        p = _run(fused, cont, (S, Aa, R, Dn), 512, 1, lr=0.0)
        cap = p._last_update_inputs
        # each path's float32 log-prob values in the ratio (see test_fused_gradient_off_policy);
        # on-policy they reproduce old_logp, i.e. ratio == 1 as in the reference
        with torch.no_grad():
            lv = (p._engine.evaluate(p.policy, cap[0], cap[1])[0] if fused
                  else p.policy.get_evaluate(cap[0], cap[1])[0])
        g64 = _grad_f64(p, cap, logp_val=lv)
        per = {}
        for (name, prm), g in zip(p.policy.named_parameters(), g64):
            m = p.optimizer.state[prm]["exp_avg"].double().cpu() / 0.1
            scale = float(g.abs().max()) + 1e-30
            per[name] = float((m - g).abs().max()) / scale
        errs["fused" if fused else "graph"] = per
    print({k: {n: f"{e:.1e}" for n, e in v.items()} for k, v in errs.items()})
    worst = {k: max(v.values()) for k, v in errs.items()}
    assert worst["fused"] <= 1e-4 and worst["graph"] <= 1e-4, worst


def _away_from_kinks(ppo, S, A, old, clip=0.2, gap=1e-3):
    """The surrogate's gradient jumps where a ratio crosses 1 +- clip (or the log-ratio crosses
    the +-20 clamp): a row within float32 noise of a kink may take either branch in any valid
    float32 implementation (continuous log-probs reach |logp| ~ 100, so that noise is ~1e-5 in
    the ratio).  Nudge such rows' old log-probs off the kink (float64 ratios)."""
    import copy
    pol = copy.deepcopy(ppo.policy).cpu().double()
    with torch.no_grad():
        logp, _, _ = pol.get_evaluate(S.cpu().double(), A.cpu().double())
    old64 = old.cpu().double()
    for _ in range(4):
        diff = logp - old64
        ratio = torch.exp(torch.clamp(diff, -20, 20))
        near = ((ratio - (1 - clip)).abs() < gap) | ((ratio - (1 + clip)).abs() < gap) | \
               ((diff.abs() - 20).abs() < gap)
        if not bool(near.any()):
            break
        old64 = torch.where(near, old64 + 10 * gap, old64)
    return old64.to(old.dtype).to(old.device)


@pytest.mark.parametrize("cont", [False, True])
@pytest.mark.parametrize("spread,rows", [(0.3, 512), (3.0, 512), (30.0, 512), (3.0, 405),
                                         (3.0, 100)])
def test_fused_gradient_off_policy(cont, spread, rows):
    """One engine step with old_logp = logp + noise(spread): ratios span the clip range, both
    sides of it and (spread 30) the +-20 log-ratio clamp, so every branch of the surrogate's
    gradient is exercised; rows < mini_batch is the ragged last minibatch (workgroups with a
    partial chunk or none).  Compared with float64 autograd of the reference loss."""
    S, Aa, R, Dn = _data(rows, 3 if cont else 4, cont, seed=21)
    p = _run(True, cont, (S, Aa, R, Dn), 512, 1, lr=0.0)
    S_, A_, old, adv, ret = p._last_update_inputs
    g = torch.Generator(device="cuda").manual_seed(3)
    old2 = _away_from_kinks(p, S_, A_, old + spread * torch.randn(old.shape, device="cuda", generator=g))
    eng = p._engine
    eng.m.zero_()
    eng.v.zero_()
    eng.step.zero_()
    # Continuous log-probs reach |logp| ~ 100 (narrow sigma): their float32 rounding (~5e-5
    # absolute, the same for CPU float32) moves every ratio by ~5e-5 relative, which the
    # cancelling sums of the mu gradients amplify past 1e-4.  So the forward is checked on its
    # own (log-prob error relative to max |logp|, CPU float32 reaches 4e-7 here) and the
    # backward against float64 autograd of the loss at the engine's own log-prob values.
    logp_eng, _ = eng.evaluate(p.policy, S_, A_)
    import copy
    with torch.no_grad():
        l64, _, _ = copy.deepcopy(p.policy).cpu().double().get_evaluate(S_.cpu().double(),
                                                                          A_.cpu().double())
    fwd = float((logp_eng.cpu().double() - l64).abs().max()) / (1.0 + float(l64.abs().max()))
    assert fwd <= 2e-6, fwd
    eng.run(S_, A_, old2, adv, ret, 1)
    import prl_native
    # CartPole at mb 512 runs the head-split latency form by default (csrc/prl_ppo_split.h)
    import os
    want_split = not cont and os.environ.get("PRL_UPD_SPLIT", "1") != "0"
    assert prl_native.ppo_update_last_plan()["split"] == want_split
    g64 = _grad_f64(p, (S_, A_, old2, adv, ret), logp_val=logp_eng)
    per = {}
    for (name, prm), gr in zip(p.policy.named_parameters(), g64):
        m = p.optimizer.state[prm]["exp_avg"].double().cpu() / 0.1
        per[name] = float((m - gr).abs().max()) / (float(gr.abs().max()) + 1e-30)
    assert max(per.values()) <= 1e-4, per


@pytest.mark.parametrize("cont", [False, True])
def test_fused_matches_per_step_path_smooth(cont):
    """A large policy_clip keeps every ratio inside the clip range (no kink in the surrogate;
    continuous log-probs move fast, hence clip 1e3 and a smaller lr there), so the two paths stay
    within float32 reduction-order noise over all 36 steps."""
    N = 6000 + 37                               # ragged last minibatch
    data = _data(N, 3 if cont else 4, cont)
    kw = dict(clip=1e3, lr=3e-4) if cont else dict(clip=10.0)
    pf = _run(True, cont, data, 512, 3, **kw)
    pg = _run(False, cont, data, 512, 3, **kw)
    # continuous: |logp| reaches ~100 (narrow sigma), d logp / d mu ~ 1e2: measured spread
    # between the GPU per-step and CPU paths themselves is 4e-4
    _compare_function(pf, pg, data, rtol=1e-3 if cont else 1e-4)
    if not cont:
        _compare(pf, pg)                      # discrete: the weights themselves agree too


def _cpu_run(cont, data, mb, k, lr=1e-3, clip=0.2):
    """The same learn() on CPU tensors with the oracle's GAE / normalisation / surrogate (the
    reference's arithmetic, PyTorch-CPU autograd and AdamW)."""
    from fake_ops import FakeOps
    from PPO import PPO
    torch.manual_seed(0)
    D, A = (3, 1) if cont else (4, 2)
    c = PPO(cont, D, A, action_scaling=2.0 if cont else None, lr=lr, k_epochs=k, batch_size=64,
            mini_batch_size=mb, policy_clip=clip)
    c.show_progress = False
    c.policy.cpu()
    c.policy_old.cpu()
    c.device = torch.device("cpu")
    c.optimizer = torch.optim.AdamW(c.policy.parameters(), lr=lr)
    c._ops = FakeOps()
    c.memory.push_device(*(x.cpu() for x in data))
    c.learn()
    return c


def _fdist(p, q, data):
    S, A = data[0][:2048], data[1][:2048]
    (lf, vf), (lg, vg) = _outputs(p, S, A), _outputs(q, S, A)
    return max(float((lf - lg).abs().max()) / (float(lg.abs().max()) + 1.0),
               float((vf - vg).abs().max()) / (float(vg.abs().max()) + 1.0))


@pytest.mark.parametrize("cont", [False, True])
def test_fused_matches_per_step_path(cont):
    """The reference's policy_clip = 0.2.  A ratio landing on the other side of 0.8 / 1.2 flips
    that sample's gradient term, and continuous PPO amplifies it: the per-step GPU path and the
    CPU path themselves end ~2 % apart.  So the check is relational: the fused engine must be
    (about) as close to the CPU path as the per-step GPU path is."""
    N = 6000 + 37
    data = _data(N, 3 if cont else 4, cont)
    pf = _run(True, cont, data, 512, 3)
    pg = _run(False, cont, data, 512, 3)
    pc = _cpu_run(cont, data, 512, 3)
    d_fc, d_gc = _fdist(pf, pc, data), _fdist(pg, pc, data)
    assert d_fc <= 2.0 * d_gc + 1e-4, (d_fc, d_gc)


def test_fused_large_minibatch_multichunk():
    """mb 4096 -> 256 workgroups x 16 rows (two 8-row chunks each); mb > N on the last epoch."""
    data = _data(9000, 4, False, seed=7)
    pf = _run(True, False, data, 4096, 2, clip=10.0)
    pg = _run(False, False, data, 4096, 2, clip=10.0)
    _compare(pf, pg)


def test_fused_small_minibatch_and_batch_smaller_than_grid():
    data = _data(700, 4, False, seed=9)
    pf = _run(True, False, data, 64, 2, clip=10.0)   # 8 workgroups, 11 steps per epoch
    pg = _run(False, False, data, 64, 2, clip=10.0)
    _compare(pf, pg)


def test_fused_state_continuity_over_learns_and_paths():
    """Two learn() calls: the AdamW moments and step count carry over (engine <-> torch state),
    and a fused learn followed by a per-step learn matches two per-step learns."""
    data = _data(3000, 4, False, seed=11)
    pf = _run(True, False, data, 512, 2, learns=2, clip=10.0)
    pg = _run(False, False, data, 512, 2, learns=2, clip=10.0)
    _compare(pf, pg)
    opt = pf.optimizer
    st = opt.state[next(iter(pf.policy.parameters()))]
    assert float(st["step"]) == 2 * 2 * 6
    # mixed: fused then per-step
    from PPO import PPO  # noqa: F401
    torch.manual_seed(0)
    pm = _run(True, False, data, 512, 2, learns=1, clip=10.0)
    pm.use_fused = False
    pm.memory.push_device(*data)
    pm.learn()
    _compare(pm, pg)


def test_fused_parameters_alias_and_save_load(tmp_path):
    data = _data(2048, 4, False)
    p = _run(True, False, data, 512, 1)
    eng = p._engine
    assert eng.bound()
    p.save_weights(str(tmp_path))
    sd = {k: v.clone() for k, v in p.policy.state_dict().items()}
    from PPO import PPO
    q = PPO(False, 4, 2)
    q.load_weights(str(tmp_path))
    for k, v in q.policy.state_dict().items():
        torch.testing.assert_close(v, sd[k], rtol=0, atol=0)
    # policy_old was refreshed from the updated policy
    for k, v in p.policy_old.state_dict().items():
        torch.testing.assert_close(v, sd[k], rtol=0, atol=0)


@pytest.mark.parametrize("cont", [False, True])
def test_engine_evaluate_matches_get_evaluate(cont):
    """prl_ppo_evaluate (policy_old pass of learn()) vs ActorCritic.get_evaluate in float64."""
    from PPO import PPO
    torch.manual_seed(0)
    D, A = (3, 1) if cont else (4, 2)
    p = PPO(cont, D, A, action_scaling=2.0 if cont else None, mini_batch_size=512)
    S, Aa, _, _ = _data(3000 + 5, D, cont, seed=13)
    eng = p._fused_engine()
    logp, V = eng.evaluate(p.policy_old, S, Aa)
    l64, v64 = _outputs(p, S, Aa)
    torch.testing.assert_close(logp.double().cpu(), l64, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(V.double().cpu(), v64, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cont", [False, True])
def test_stepped_engine_matches_persistent(cont):
    """The stepped engine (world_size > 1 path: grad kernel -> all-reduce -> AdamW kernel per
    step) with an identity all-reduce equals the persistent kernel up to float32 summation
    order (the gradient norm is summed in a different order)."""
    N = 4000 + 11
    data = _data(N, 3 if cont else 4, cont, seed=17)
    kw = dict(clip=1e3, lr=3e-4) if cont else dict(clip=10.0)
    pf = _run(True, cont, data, 512, 2, **kw)
    from PPO import PPO
    torch.manual_seed(0)
    D, A = (3, 1) if cont else (4, 2)
    ps = PPO(cont, D, A, action_scaling=2.0 if cont else None, lr=kw.get("lr", 1e-3), k_epochs=2,
             batch_size=64, mini_batch_size=512, policy_clip=kw["clip"])
    ps.show_progress = False
    ps.memory.push_device(*data)
    # drive learn()'s stepped branch with a one-rank "all-reduce"
    ps._world = staticmethod(lambda: 1)
    orig = ps._update

    def stepped_update(S, A_, old, adv, ret, n_ranks):
        eng = ps._fused_engine()
        ps._last_update_inputs = (S, A_, old, adv, ret)
        ps.last_loss = eng.run_stepped(S, A_, old, adv, ret, ps.k_epochs, n_ranks, lambda t: t)
        ps.last_update_path = "fused-dp"
    ps._update = stepped_update
    ps.learn()
    ps._update = orig
    _compare_function(pf, ps, data, rtol=1e-3 if cont else 1e-4)
    assert float(ps.optimizer.state[next(ps.policy.parameters())]["step"]) == 2 * 8
    if not cont:
        _compare(pf, ps)


@pytest.mark.parametrize("cont", [False, True])
def test_native_dp_loop_equals_python_loop(cont):
    """prl_ppo_update_dp (the stepped loop enqueued from C with ncclAllReduce, here on a one-rank
    RCCL communicator: the all-reduce is an identity) gives the same bits as the Python loop
    with an identity all-reduce: parameters, both moments, step count and loss."""
    import prl_native
    from PPO import PPO
    N = 3000 + 7
    data = _data(N, 3 if cont else 4, cont, seed=29)
    D, A = (3, 1) if cont else (4, 2)
    prl_native.dp_rccl_open()
    comm = prl_native.dp_comm_init(prl_native.dp_unique_id(), 1, 0)
    outs = []
    try:
        for native in (False, True):
            torch.manual_seed(0)
            p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=3, batch_size=64,
                    mini_batch_size=512)
            p.show_progress = False
            p.memory.push_device(*data)
            p._world = staticmethod(lambda: 1)

            def stepped_update(S, A_, old, adv, ret, n_ranks, p=p, native=native):
                eng = p._fused_engine()
                p.last_loss = eng.run_stepped(S, A_, old, adv, ret, p.k_epochs, n_ranks,
                                              lambda t: t, comm=comm if native else None)
            p._update = stepped_update
            p.learn()
            torch.cuda.synchronize()
            eng = p._engine
            outs.append((eng.flat.cpu(), eng.m.cpu(), eng.v.cpu(), float(eng.step.item()),
                         float(p.last_loss)))
    finally:
        prl_native.dp_comm_destroy(comm)
    (f0, m0, v0, s0, l0), (f1, m1, v1, s1, l1) = outs
    assert torch.equal(f0, f1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    assert s0 == s1 == 3 * 6 and l0 == l1


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("cont", [False, True])
def test_dpx_one_rank_equals_engine(cont, split):
    """The data-parallel persistent kernel (prl_ppo_update_dpx) with ONE rank — its own slice
    buffer, inv_count = float(1 / rows) — gives the single-GPU engine's bits (parameters, both
    moments, step count, loss) over two learn() calls on one buffer set: its in-GPU part is the
    engine's, the cross-rank phase adds only the rank-order sum.  split: both sides run the
    head-split form (CartPole) or both the 8-wave kernel."""
    if cont and split == 0:
        pytest.skip("the split setting applies to the two-head CartPole shape only")
    with _split(split):
        _dpx_one_rank_equals_engine(cont)


def _dpx_one_rank_equals_engine(cont):
    import prl_native
    from PPO import PPO
    N = 3000 + 7
    data = _data(N, 3 if cont else 4, cont, seed=31)
    D, A = (3, 1) if cont else (4, 2)
    outs = []
    for dpx in (False, True):
        torch.manual_seed(0)
        p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=3, batch_size=64,
                mini_batch_size=512)
        p.show_progress = False
        state = {"xb": None, "seq": 0}
        if dpx:
            def upd(S, A_, old, adv, ret, n_ranks, p=p, state=state):
                eng = p._fused_engine()
                if state["xb"] is None:
                    state["xb"], _ = prl_native.dp_xbuf_alloc(
                        prl_native.dp_xbuf_bytes(eng.D, eng.A, eng.discrete, eng.mini_batch))
                n, mb = int(S.shape[0]), eng.mini_batch
                nb = -(-n // mb)
                inv = torch.tensor([1.0 / min(mb, n - j * mb) for j in range(nb)],
                                   dtype=torch.float32, device=S.device)
                group = p.optimizer.param_groups[0]
                prl_native.ppo_update_dpx(
                    eng.flat, eng.m, eng.v, eng.step, D, A, eng.discrete, S.contiguous(),
                    (A_ if A_.dim() == 2 else A_.reshape(-1, 1)).contiguous(), old.contiguous(),
                    adv.contiguous(), ret.contiguous(), mb, p.k_epochs, nb, inv, p.policy_clip,
                    p.value_coef, p.entropy_coef, group["lr"], group["betas"][0],
                    group["betas"][1], group["eps"], group["weight_decay"], 2.0, eng.loss, 1, 0,
                    [state["xb"]], state["seq"], eng.ws)
                state["seq"] += p.k_epochs * nb
                eng._sync_optimizer_state()
                p.last_loss = eng.loss.reshape(()).clone()
                p.last_update_path = "dpx1"
            p._update = upd
        for _ in range(2):
            p.memory.push_device(*data)
            p.learn()
        torch.cuda.synchronize()
        eng = p._engine
        assert max(prl_native.ppo_update_status(eng.ws).tolist()) == 0
        outs.append((eng.flat.cpu(), eng.m.cpu(), eng.v.cpu(), float(eng.step.item()),
                     float(p.last_loss)))
        if state["xb"] is not None:
            prl_native.dp_xbuf_free(state["xb"])
    (f0, m0, v0, s0, l0), (f1, m1, v1, s1, l1) = outs
    assert torch.equal(f0, f1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    assert s0 == s1 == 2 * 3 * 6 and l0 == l1


@pytest.mark.parametrize("cont,D,A", [(False, 6, 3), (True, 5, 2)])
def test_generic_shape_engine_gradient(cont, D, A):
    """Shapes outside the specialised kernels run the runtime-layout engine (KD = -1): one step at
    lr = 0, its forward against float64 and its gradient against float64 autograd of the
    reference loss at the engine's own log-prob values (as test_fused_gradient_off_policy)."""
    import copy
    rng = np.random.default_rng(41)
    N = 512 - 37        # one ragged minibatch: the float64 reference is one step over all rows
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    Aa = (torch.from_numpy((np.tanh(rng.normal(size=(N, A))) * 2).astype(np.float32)).cuda() if cont
          else torch.from_numpy(rng.integers(0, A, N).astype(np.float32)).cuda())
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.05).astype(np.float32)).cuda()
    Dn[-1] = 1
    p = _run(True, cont, (S, Aa, R, Dn), 512, 1, D=D, A=A, lr=0.0)
    S_, A_, old, adv, ret = p._last_update_inputs
    eng = p._engine
    logp_eng, _ = eng.evaluate(p.policy, S_, A_)
    with torch.no_grad():
        l64, _, _ = copy.deepcopy(p.policy).cpu().double().get_evaluate(S_.cpu().double(),
                                                                          A_.cpu().double())
    fwd = float((logp_eng.cpu().double() - l64).abs().max()) / (1.0 + float(l64.abs().max()))
    assert fwd <= 2e-6, fwd
    g = torch.Generator(device="cuda").manual_seed(5)
    old2 = _away_from_kinks(p, S_, A_, old + 0.5 * torch.randn(old.shape, device="cuda", generator=g))
    eng.m.zero_()
    eng.v.zero_()
    eng.step.zero_()
    eng.run(S_, A_, old2, adv, ret, 1)
    g64 = _grad_f64(p, (S_, A_, old2, adv, ret), logp_val=logp_eng)
    per = {}
    for (name, prm), gr in zip(p.policy.named_parameters(), g64):
        m = p.optimizer.state[prm]["exp_avg"].double().cpu() / 0.1
        per[name] = float((m - gr).abs().max()) / (float(gr.abs().max()) + 1e-30)
    assert max(per.values()) <= 1e-4, per


def _unfolded_stepped(eng, S, A, old, adv, ret, k_epochs, n_ranks):
    """The stepped loop in its unfolded form (prl_ppo_grad_step -> identity all-reduce ->
    prl_ppo_adam_step per optimizer step): the reference for the folded launch."""
    import ctypes
    import prl_native
    ppo = eng.ppo
    group = ppo.optimizer.param_groups[0]
    beta1, beta2 = group["betas"]
    L = prl_native.ppo_image_floats(eng.D, eng.A, eng.discrete)
    img = [torch.zeros(L, device="cuda") for _ in range(3)]
    grad = torch.zeros(L, device="cuda")
    prl_native.ppo_image(eng.D, eng.A, eng.discrete, eng.flat, eng.m, eng.v, *img, True)
    mb = eng.mini_batch
    nb = max(-(-n // mb) for n in n_ranks)
    counts = [sum(min(mb, max(0, n - j * mb)) for n in n_ranks) for j in range(nb)]
    A2 = (A if A.dim() == 2 else A.reshape(-1, 1)).contiguous()
    tens = [S.contiguous(), A2, old.contiguous(), adv.contiguous(), ret.contiguous()]
    P, lib = ctypes.c_void_p, prl_native.lib()
    stream = P(torch.cuda.current_stream().cuda_stream)
    step = int(round(float(eng.step.item())))
    for _ in range(k_epochs):
        for j in range(nb):
            inv = ctypes.c_float(1.0 / counts[j])
            assert lib.prl_ppo_grad_step(P(img[0].data_ptr()), eng.D, eng.A, int(eng.discrete),
                                         *(P(x.data_ptr()) for x in tens), int(S.shape[0]), mb, j,
                                         inv, ctypes.c_float(ppo.policy_clip),
                                         ctypes.c_float(ppo.value_coef), P(grad.data_ptr()),
                                         P(eng.ws.data_ptr()), eng.ws.numel(), stream) == 0
            step += 1
            assert lib.prl_ppo_adam_step(*(P(x.data_ptr()) for x in img), eng.D, eng.A,
                                         int(eng.discrete), P(grad.data_ptr()), step,
                                         ctypes.c_float(group["lr"]), ctypes.c_double(beta1),
                                         ctypes.c_double(beta2),
                                         *(ctypes.c_float(x) for x in (
                                             group["eps"], group["weight_decay"], 2.0)), inv,
                                         ctypes.c_float(ppo.value_coef),
                                         ctypes.c_float(ppo.entropy_coef),
                                         P(eng.loss.data_ptr()), stream) == 0
    torch.cuda.synchronize()
    return [x.cpu() for x in img], grad.cpu(), float(eng.loss.item())


@pytest.mark.parametrize("cont,D,A", [(False, 4, 2), (True, 3, 1), (False, 6, 3)])
def test_folded_step_equals_grad_then_adam(cont, D, A):
    """prl_ppo_grad_fold_step (previous step's AdamW folded in front of the next gradient,
    double-buffered state) gives the same bits as the unfolded prl_ppo_grad_step ->
    prl_ppo_adam_step sequence: parameter / moment images, last gradient and loss.  Covers the
    compile-time layouts (all loads before the norm) and the runtime layout (D=6, A=3)."""
    import prl_native
    from PPO import PPO
    N = 2500 + 3
    data = _data(N, D, cont, seed=31)
    torch.manual_seed(0)
    p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=2, batch_size=64,
            mini_batch_size=512)
    p.show_progress = False
    p.memory.push_device(*data)
    p._world = staticmethod(lambda: 1)
    captured = {}

    def stepped_update(S, A_, old, adv, ret, n_ranks):
        eng = p._fused_engine()
        if not eng.bound():
            eng._bind()
        captured["ref"] = _unfolded_stepped(eng, S, A_, old, adv, ret, p.k_epochs, n_ranks)
        p.last_loss = eng.run_stepped(S, A_, old, adv, ret, p.k_epochs, n_ranks, lambda t: t)
        torch.cuda.synchronize()
        captured["fold"] = ([x.cpu() for x in eng.img], eng.grad.cpu(), float(eng.loss.item()))
    p._update = stepped_update
    p.learn()
    (ri, rg, rl), (fi, fg, fl) = captured["ref"], captured["fold"]
    for a, b in zip(ri, fi):
        assert torch.equal(a, b)
    assert torch.equal(rg, fg) and rl == fl
    assert float(p._engine.step.item()) == 2 * 5




@pytest.mark.parametrize("cont", [False, True])
def test_engine_bit_reproducible(cont):
    """The persistent engine is deterministic: learn() from the same seed and memory gives the
    same bits twice, and re-running the engine from a restored state on learn()'s own inputs
    (workspace refilled by a plain-store kernel in between) gives them again.  Round 1's engine
    failed this: its clip coefficient came from 4-B norm pieces that workgroups sometimes read
    stale (tools/exp/engine_determinism4.py); the norm is now formed from the reduced gradient."""
    from PPO import PPO
    N = 512 * 24 + 7
    data = _data(N, 3 if cont else 4, cont, seed=41)
    D, A = (3, 1) if cont else (4, 2)
    flats = []
    for _ in range(2):
        torch.manual_seed(0)
        p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=3, batch_size=64,
                mini_batch_size=512)
        p.show_progress = False
        eng = p._fused_engine()
        init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
        p.memory.push_device(*data)
        p.learn()
        torch.cuda.synchronize()
        flats.append(eng.flat.cpu().clone())
    assert torch.equal(flats[0], flats[1])
    ins = [x.clone() for x in p._last_update_inputs]
    for _ in range(3):
        for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
            dst.copy_(src)
        eng.ws.fill_(0)
        eng.run(*ins, 3)
        torch.cuda.synchronize()
        assert torch.equal(eng.flat.cpu(), flats[0])


@pytest.mark.parametrize("cont", [False, True])
@pytest.mark.parametrize("mb,N", [(512, 512 * 6 + 7), (8192, 8192 * 3 + 300), (65536, 65536 + 5000)])
def test_throughput_form_equals_latency_form(cont, mb, N):
    """The persistent kernel's two forms (prl_ppo_update_set_tp): the latency form (gradient
    image in LDS, AdamW moments in registers) and the throughput form (gradient in registers,
    moments streamed through the workspace by the slice owners), at one tile per workgroup
    (mb 512, the form forced), two (mb 8192) and sixteen (mb 65536, ragged last minibatch).
    CartPole: both run the 8-wave kernel with the same tiles, order and per-tile sums, so
    parameters, moments, step count and loss are the same BITS (the head-split latency form is
    off here; test_split_form_matches_8wave_form covers it).  Pendulum: the throughput form
    runs 8 waves (the latency form's LDS image does not fit with 8), so the clip norm is summed
    in another order (and dW1 accumulates across tiles in the MFMA): float32 rounding apart,
    checked on the learned function (log-probs / values on probe states, rtol 1e-4) and the
    moments."""
    import copy
    import types

    import prl_native
    from PPO import PPO
    D, A = (3, 1) if cont else (4, 2)
    data = _data(N, D, cont, seed=43)
    torch.manual_seed(0)
    p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=2, batch_size=64,
            mini_batch_size=mb)
    p.show_progress = False
    eng = p._fused_engine()
    init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
    p.memory.push_device(*data)
    p.learn()
    torch.cuda.synchronize()
    ins = [x.clone() for x in p._last_update_inputs]
    outs, pols = {}, {}
    for mode in (0, 1):
        prev = prl_native.ppo_update_set_tp(mode)
        prev_split = prl_native.ppo_update_set_split(0)
        try:
            for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
                dst.copy_(src)
            eng.ws.fill_(0)
            loss = eng.run(*ins, 2)
            torch.cuda.synchronize()
            outs[mode] = [t.cpu().clone() for t in (eng.flat, eng.m, eng.v, eng.step, loss)]
            # (the policy's parameters alias eng.flat: snapshot them)
            pols[mode] = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
        finally:
            prl_native.ppo_update_set_tp(prev)
            prl_native.ppo_update_set_split(prev_split)
    assert not torch.equal(outs[0][0], init[0].cpu())
    names = ("params", "exp_avg", "exp_avg_sq", "step", "loss")
    if not cont:
        for a, b, name in zip(outs[0], outs[1], names):
            assert torch.equal(a, b), (name, float((a.double() - b.double()).abs().max()))
        return
    _compare_function(pols[0], pols[1], data, rtol=1e-4)
    assert torch.equal(outs[0][3], outs[1][3])
    for k in (1, 2):   # moments: float32 rounding of the same steps
        a, b = outs[0][k].double(), outs[1][k].double()
        assert float((a - b).abs().max()) <= 1e-3 * float(a.abs().max()) + 1e-12, names[k]
    assert abs(float(outs[0][4]) - float(outs[1][4])) <= 1e-4 * max(1.0, abs(float(outs[0][4])))


@pytest.mark.parametrize("cont", [False, True])
@pytest.mark.parametrize("mb,N", [(512, 512 * 5 + 77), (1000, 1000 * 3 + 1)])
def test_replicated_tiles_equal_single(cont, mb, N):
    """The latency form's replicated tiles (prl_ppo_update_set_repl): with X workgroups per
    16-row tile group, each publishing 1/X of the group's partial gradient and phase B cut into
    X times more slices, every replica computes the same partial bits and the slice sums run over
    the same partials in the same order, so parameters, moments, step count and loss are the same
    BITS as with one workgroup per tile.  mb 1000: 63 tile groups (the grid capped at one
    workgroup per CU: 4 replicas fit, 8 do not)."""
    import prl_native
    from PPO import PPO
    D, A = (3, 1) if cont else (4, 2)
    data = _data(N, D, cont, seed=47)
    torch.manual_seed(0)
    p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=2, batch_size=64,
            mini_batch_size=mb)
    p.show_progress = False
    eng = p._fused_engine()
    init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
    p.memory.push_device(*data)
    p.learn()
    torch.cuda.synchronize()
    ins = [x.clone() for x in p._last_update_inputs]
    Gt = -(-mb // 16)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    outs = {}
    for x in (1, 2, 3, 4, 8):
        prev = prl_native.ppo_update_set_repl(x)
        prev_split = prl_native.ppo_update_set_split(0)   # replicas are the 8-wave form's
        try:
            for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
                dst.copy_(src)
            eng.ws.fill_(0)
            loss = eng.run(*ins, 2)
            torch.cuda.synchronize()
            plan = prl_native.ppo_update_last_plan()
            want = max(r for r in range(1, x + 1) if Gt * r <= cus)
            assert plan["form"] == "latency" and plan["replicas"] == want, plan
            assert plan["grid"] == Gt * want, plan
            outs[x] = [t.cpu().clone() for t in (eng.flat, eng.m, eng.v, eng.step, loss)]
        finally:
            prl_native.ppo_update_set_repl(prev)
            prl_native.ppo_update_set_split(prev_split)
    assert not torch.equal(outs[1][0], init[0].cpu())
    names = ("params", "exp_avg", "exp_avg_sq", "step", "loss")
    for x in (2, 3, 4, 8):
        for a, b, name in zip(outs[1], outs[x], names):
            assert torch.equal(a, b), (x, name, float((a.double() - b.double()).abs().max()))


@pytest.mark.parametrize("mb,N", [(512, 512 * 6 + 7), (64, 700), (1000, 1000 * 3 + 1),
                                  (2048, 2048 * 2 + 33)])
def test_split_form_matches_8wave_form(mb, N):
    """The head-split latency form (csrc/prl_ppo_split.h: actor and critic head of a 16-row tile
    on two workgroups, 2 Gt workgroups of 4 waves) against the 8-wave kernel, from the same state
    on the same learn() inputs: the trunk gradient is summed per head and then across heads in
    float64 (not inside one MFMA chain), so the two agree to float32 rounding — the learned
    function (probe log-probs / values, rtol 1e-4), weights (3e-5), moments (1e-3 relative),
    step count and loss.  mb 64 / 1000 / 2048: few tile groups, a ragged tile group (1000 =
    62 x 16 + 8) and the largest grid that fits (2 x 128 workgroups)."""
    import copy
    import types

    import prl_native
    from PPO import PPO
    data = _data(N, 4, False, seed=53)
    torch.manual_seed(0)
    p = PPO(False, 4, 2, k_epochs=2, batch_size=64, mini_batch_size=mb)
    p.show_progress = False
    eng = p._fused_engine()
    init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
    p.memory.push_device(*data)
    p.learn()
    torch.cuda.synchronize()
    ins = [x.clone() for x in p._last_update_inputs]
    Gt = -(-mb // 16)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    outs, pols = {}, {}
    for mode in (0, 1):
        with _split(mode):
            for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
                dst.copy_(src)
            eng.ws.fill_(0)
            loss = eng.run(*ins, 2)
            torch.cuda.synchronize()
            plan = prl_native.ppo_update_last_plan()
            assert plan["form"] == "latency" and plan["split"] == bool(mode and 2 * Gt <= cus), plan
            if plan["split"]:
                assert plan["waves"] in (4, 8) and plan["grid"] == 2 * Gt, plan   # (8: PRL_UPD_SPL_WAVES)
            outs[mode] = [t.cpu().clone() for t in (eng.flat, eng.m, eng.v, eng.step, loss)]
            pols[mode] = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
    assert not torch.equal(outs[1][0], init[0].cpu())
    _compare_function(pols[0], pols[1], data, rtol=1e-4)
    worst = float((outs[0][0] - outs[1][0]).abs().max())
    assert worst <= ATOL, worst
    for k in (1, 2):
        a, b = outs[0][k].double(), outs[1][k].double()
        assert float((a - b).abs().max()) <= 1e-3 * float(a.abs().max()) + 1e-12, k
    assert torch.equal(outs[0][3], outs[1][3])
    assert abs(float(outs[0][4]) - float(outs[1][4])) <= 1e-4 * max(1.0, abs(float(outs[0][4])))



@pytest.mark.parametrize("adv_scale", [1e-3, 1e3])
def test_split_owner_form_matches_workgroup_adamw(monkeypatch, adv_scale):
    """The split form's slice-owner variant (prl_ppo_split.h OWN, PRL_UPD_SPL_OWN=1: each
    slice owner runs AdamW on its quads and publishes the new weights; the clip norm from
    per-wave pieces) against its workgroup-AdamW variant (PRL_UPD_SPL_OWN=0) from the same
    state on the same inputs.  adv x 1e-3: no step clips, so the same AdamW on the same gradient
    values gives the same bits (weights, both moments, step count, loss).  adv x 1e3: EVERY step
    clips (engine profile: clipped_steps_frac 1), so every step takes the owner variant's
    redo + counter-C hand-off; the norm is summed in another order than the workgroup
    variant's, so the two agree to float32 rounding of the clip coefficient (weights 3e-5)."""
    import prl_native
    from PPO import PPO
    N, mb = 512 * 5 + 9, 512
    data = _data(N, 4, False, seed=61)
    torch.manual_seed(0)
    p = PPO(False, 4, 2, k_epochs=2, batch_size=64, mini_batch_size=mb)
    p.show_progress = False
    eng = p._fused_engine()
    init = [eng.flat.clone(), eng.m.clone(), eng.v.clone(), eng.step.clone()]
    p.memory.push_device(*data)
    p.learn()
    torch.cuda.synchronize()
    S, A, old, adv, ret = [x.clone() for x in p._last_update_inputs]
    adv = adv * adv_scale
    if adv_scale < 1:
        # returns = the initial policy's own values (the policy's parameters are views of the
        # engine's flat buffer): a near-zero value gradient, so no step clips
        eng.flat.copy_(init[0])
        _, V0 = eng.evaluate(p.policy, S, A)
        ret = V0.clone()
    outs = {}
    monkeypatch.setenv("PRL_UPD_PROFILE", "1")
    for own in ("1", "0"):
        monkeypatch.setenv("PRL_UPD_SPL_OWN", own)
        for dst, src in zip((eng.flat, eng.m, eng.v, eng.step), init):
            dst.copy_(src)
        eng.ws.fill_(0)
        loss = eng.run(S, A, old, adv, ret, 3)
        torch.cuda.synchronize()
        plan = prl_native.ppo_update_last_plan()
        assert plan["split"] and plan["owner"] == (own == "1"), plan
        frac = eng.profile()["clipped_steps_frac"]
        assert frac == (1.0 if adv_scale > 1 else 0.0), frac
        outs[own] = [t.cpu().clone() for t in (eng.flat, eng.m, eng.v, eng.step, loss)]
    assert not torch.equal(outs["1"][0], init[0].cpu())
    if adv_scale < 1:
        for a, b in zip(outs["1"], outs["0"]):
            assert torch.equal(a, b)
    else:
        worst = float((outs["1"][0] - outs["0"][0]).abs().max())
        assert worst <= ATOL, worst
        for k in (1, 2):
            a, b = outs["1"][k].double(), outs["0"][k].double()
            assert float((a - b).abs().max()) <= 1e-3 * float(a.abs().max()) + 1e-12, k
        assert torch.equal(outs["1"][3], outs["0"][3])
