"""Kernel parity through the C-ABI (libprl_hip.so) against the CPU oracle and the reference's
golden vectors.  Integer / mask / index work and the reference-ordered float recurrences are
checked BIT-EXACT; float reductions and transcendental paths within the stated tolerances."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def native():
    import prl_native
    return prl_native


def T(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


# ---------------------------------------------------------------------------------- GAE
@pytest.mark.parametrize("case", list("abcde"))
def test_gae_bit_exact_vs_reference_fixture(golden, case):
    N = native()
    g = golden("gae")
    r, d, V = (T(g[f"{case}_{k}"]) for k in "rdV")
    nv = T(np.array([g[f"{case}_nv"]], np.float32))
    ret = torch.empty_like(V)
    adv = torch.empty_like(V)
    sums = torch.zeros(2, dtype=torch.float64, device=DEV)
    N.gae(r, d, V, nv, float(g[f"{case}_gamma"]), float(g[f"{case}_lam"]), ret, adv, sums)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(bits(ret.cpu().numpy()), bits(g[f"{case}_ret"]))
    adv_ref = (g[f"{case}_ret"] - g[f"{case}_V"]).astype(np.float32)
    np.testing.assert_array_equal(bits(adv.cpu().numpy()), bits(adv_ref))
    s = sums.cpu().numpy()
    a64 = adv_ref.astype(np.float64)
    assert s[0] == pytest.approx(a64.sum(), rel=1e-12, abs=1e-9)
    assert s[1] == pytest.approx((a64 * a64).sum(), rel=1e-12)


@pytest.mark.parametrize("n,pd,seed", [(1, 1.0, 0), (7, 0.3, 1), (2048, 0.05, 2), (2049, 0.05, 3),
                                       (100_003, 0.05, 4), (1 << 20, 0.05, 5), (300_000, 0.0, 6),
                                       (250_000, 0.002, 7), (65_536 * 200 // 8, -1, 8),
                                       (2048 * 37, 0.0, 10), (2048 * 300 + 5, -5000, 11),
                                       (2048 * 3000, -500, 12)])
def test_gae_bit_exact_vs_oracle(n, pd, seed):
    """Random breaks, none at all (a full last tile: the chain starts at gae = 0 past the end),
    fixed segments of 200 (Pendulum), 500 (trained CartPole, > 1 round of tiles) and 5000 steps
    (runs over break-free tiles: the stream heads' multi-tile look-ahead)."""
    N = native()
    rng = np.random.default_rng(seed)
    if pd < 0:                                 # fixed segments (-1: Pendulum's 200 steps)
        seg = 200 if pd == -1 else int(-pd)
        d = np.zeros(n, np.float32)
        d[seg - 1::seg] = 1
    else:
        d = (rng.random(n) < pd).astype(np.float32)
    r = rng.normal(1, 0.5, n).astype(np.float32)
    V = rng.normal(0, 3, n).astype(np.float32)
    ref = O.gae(r, d, V, V[-1], 0.995, 0.95)
    ret = torch.empty(n, dtype=torch.float32, device=DEV)
    N.gae(T(r), T(d), T(V), None, 0.995, 0.95, ret)
    np.testing.assert_array_equal(bits(ret.cpu().numpy()), bits(ref))


def test_gae_unaligned_views():
    N = native()
    rng = np.random.default_rng(9)
    n = 50_001
    r = rng.normal(size=n + 1).astype(np.float32)
    d = (rng.random(n + 1) < 0.04).astype(np.float32)
    V = rng.normal(size=n + 1).astype(np.float32)
    rt, dt_, Vt = T(r), T(d), T(V)
    ret = torch.empty(n + 1, dtype=torch.float32, device=DEV)
    N.gae(rt[1:], dt_[1:], Vt[1:], None, 0.99, 0.9, ret[1:])   # 4-B offset: scalar path
    ref = O.gae(r[1:], d[1:], V[1:], V[-1], 0.99, 0.9)
    np.testing.assert_array_equal(bits(ret[1:].cpu().numpy()), bits(ref))


def test_gae_large_properties():
    """Full-size (N = 13.1 M, config 3 shape) checks: a spot-checked oracle slice per segment
    and determinism across runs."""
    N = native()
    n = 65_536 * 200
    g = torch.Generator(device=DEV).manual_seed(0)
    r = torch.randn(n, device=DEV, generator=g)
    V = torch.randn(n, device=DEV, generator=g)
    d = torch.zeros(n, device=DEV)
    d[199::200] = 1
    ret1 = torch.empty_like(V)
    ret2 = torch.empty_like(V)
    N.gae(r, d, V, None, 0.995, 0.95, ret1)
    N.gae(r, d, V, None, 0.995, 0.95, ret2)
    assert torch.equal(ret1.view(torch.int32), ret2.view(torch.int32))
    for seg in (0, 1234, 40_000, 65_535):   # segments are independent (d = 1 ends)
        sl = slice(seg * 200, seg * 200 + 200)
        ref = O.gae(r[sl].cpu().numpy(), d[sl].cpu().numpy(), V[sl].cpu().numpy(),
                    float(V[sl][-1]), 0.995, 0.95)
        np.testing.assert_array_equal(bits(ret1[sl].cpu().numpy()), bits(ref))


def test_adv_stats_and_normalize(golden):
    N = native()
    g = golden("learn")
    ret = T(g["returns"])
    V = T(g["old_V"])
    adv = torch.empty_like(V)
    sums = torch.zeros(2, dtype=torch.float64, device=DEV)
    out = torch.empty_like(V)
    N.gae(T(g["R"]), T(g["Dn"]), V, None, 0.995, 0.95, torch.empty_like(V), adv, sums)
    N.adv_normalize(adv, sums, adv.numel(), 1e-8, out)
    # north_star: 1e-5 relative, 1e-6 absolute guard near zero (normalised units)
    np.testing.assert_allclose(out.cpu().numpy(), g["adv"], rtol=1e-5, atol=1e-6)
    sums2 = torch.zeros(2, dtype=torch.float64, device=DEV)
    N.adv_stats(adv, sums2)
    np.testing.assert_allclose(sums2.cpu().numpy(), sums.cpu().numpy(), rtol=1e-12)
    assert torch.equal(ret, ret)  # (returns checked bit-exact in the GAE tests)


# ---------------------------------------------------------------------------------- surrogate
@pytest.mark.parametrize("tag", ["learn", "learn_cont"])
def test_surrogate_vs_reference_autograd(golden, tag):
    N = native()
    g = golden(tag)
    mb, n = int(g["mb"]), int(g["N"])
    nsteps = int(g["k_epochs"]) * (-(-n // mb))
    old = np.tile(g["old_logp"], int(g["k_epochs"]))
    off = 0
    for s in range(nsteps):
        k = min(mb, n - (s % (-(-n // mb))) * mb)
        sl = slice(off, off + k)
        args = [T(x[sl]) for x in (g["step_logp"], old, g["step_adv"], g["step_V"], g["step_ret"])]
        H = T(np.array(g["step_H"][s], np.float32).reshape(()))
        loss = torch.empty((), dtype=torch.float32, device=DEV)
        dl = torch.empty(k, dtype=torch.float32, device=DEV)
        dv = torch.empty(k, dtype=torch.float32, device=DEV)
        N.surrogate_fwd(*args, H, 0.2, 0.5, 0.01, loss, dl, dv)
        ref_loss = np.mean(-g["step_min"][sl].astype(np.float64)) + 0.5 * float(g["step_sl1"][s]) \
            - 0.01 * float(g["step_H"][s])
        assert float(loss) == pytest.approx(ref_loss, rel=2e-5, abs=1e-6)
        scale = np.abs(g["step_dlogp"][sl]).max() + 1e-30
        np.testing.assert_allclose(dl.cpu().numpy(), g["step_dlogp"][sl], rtol=4e-6,
                                   atol=1e-7 * scale)
        np.testing.assert_allclose(dv.cpu().numpy(), g["step_dV"][sl], rtol=1e-5, atol=1e-9)
        # backward: upstream gradient scales the unit gradients
        go = torch.tensor(2.5, device=DEV)
        dl2, dv2 = torch.empty_like(dl), torch.empty_like(dv)
        N.surrogate_bwd(go, dl, dv, dl2, dv2)
        torch.testing.assert_close(dl2, dl * 2.5, rtol=0, atol=0)
        torch.testing.assert_close(dv2, dv * 2.5, rtol=0, atol=0)
        off += k


@pytest.mark.parametrize("mb", [1, 513, 4096, 65_536, 300_001])
def test_surrogate_multiblock_vs_oracle(mb):
    N = native()
    rng = np.random.default_rng(mb)
    lp = rng.normal(-0.7, 0.3, mb).astype(np.float32)
    old = (lp + rng.normal(0, 0.2, mb)).astype(np.float32)
    old[::97] = lp[::97]                       # exact ties: ratio == 1
    adv = rng.normal(0, 1, mb).astype(np.float32)
    V = rng.normal(0, 2, mb).astype(np.float32)
    ret = rng.normal(0, 2, mb).astype(np.float32)
    H = 0.69
    loss_ref, dl_ref, dv_ref = O.surrogate(lp, old, adv, V, ret, H)
    loss = torch.empty((), dtype=torch.float32, device=DEV)
    dl = torch.empty(mb, dtype=torch.float32, device=DEV)
    dv = torch.empty(mb, dtype=torch.float32, device=DEV)
    N.surrogate_fwd(T(lp), T(old), T(adv), T(V), T(ret), T(np.float32(H).reshape(())), 0.2, 0.5,
                    0.01, loss, dl, dv)
    assert float(loss) == pytest.approx(loss_ref, rel=1e-5, abs=1e-6)
    np.testing.assert_allclose(dl.cpu().numpy(), dl_ref, rtol=4e-6, atol=1e-8 / mb)
    np.testing.assert_allclose(dv.cpu().numpy(), dv_ref, rtol=1e-5, atol=1e-9)


# ---------------------------------------------------------------------------------- RND
def test_rnd_forward_vs_reference(golden):
    N = native()
    g = golden("rnd")
    for D in (4, 348):
        nets = []
        for name in ("target_net", "pred_net"):
            nets.append([T(g[f"D{D}/{name}.{k}"]) for k in
                         ("0.weight", "0.bias", "1.weight", "1.bias", "3.weight", "3.bias")])
        x = T(g[f"D{D}_x"])
        out = torch.empty(x.shape[0], dtype=torch.float32, device=DEV)
        N.rnd_forward(x, nets[0], nets[1], 0.001, out)
        np.testing.assert_allclose(out.cpu().numpy(), g[f"D{D}_r"], rtol=2e-5, atol=1e-8)


def test_rnd_forward_ragged_rows():
    N = native()
    rng = np.random.default_rng(0)
    D = 17
    nets_np, nets = [], []
    for _ in range(2):
        p = dict(w1=rng.normal(0, .3, (64, D)), b1=rng.normal(0, .01, 64), gw=rng.normal(1, .1, 64),
                 gb=rng.normal(0, .1, 64), w2=rng.normal(0, .3, (D, 64)), b2=rng.normal(0, .01, D))
        p = {k: v.astype(np.float32) for k, v in p.items()}
        nets_np.append(p)
        nets.append([T(p[k]) for k in ("w1", "b1", "gw", "gb", "w2", "b2")])
    for n in (1, 63, 64, 65, 1000):
        x = rng.normal(size=(n, D)).astype(np.float32)
        out = torch.empty(n, dtype=torch.float32, device=DEV)
        N.rnd_forward(T(x), nets[0], nets[1], 0.5, out)
        np.testing.assert_allclose(out.cpu().numpy(), O.rnd_forward(x, nets_np[0], nets_np[1], 0.5),
                                   rtol=3e-5, atol=1e-7)


@pytest.mark.parametrize("D,n", [(348, 70001), (348, 257), (12, 33000), (4, 1)])
def test_rnd_forward_persistent_blocks(D, n, monkeypatch):
    """The persistent fast kernel (D % 4 == 0: 128-row blocks, every workgroup looping over
    several when n > 128 x CUs, chunks prefetched across the layer and block boundaries) against
    the oracle on a row subset and against the round-1 kernel (PRL_RND_GENERIC=1) on all rows."""
    N = native()
    rng = np.random.default_rng(D + n)
    nets_np, nets = [], []
    for _ in range(2):
        p = dict(w1=rng.normal(0, .1, (64, D)), b1=rng.normal(0, .01, 64), gw=rng.normal(1, .1, 64),
                 gb=rng.normal(0, .1, 64), w2=rng.normal(0, .1, (D, 64)), b2=rng.normal(0, .01, D))
        p = {k: v.astype(np.float32) for k, v in p.items()}
        nets_np.append(p)
        nets.append([T(p[k]) for k in ("w1", "b1", "gw", "gb", "w2", "b2")])
    x = rng.normal(size=(n, D)).astype(np.float32)
    fast = torch.empty(n, dtype=torch.float32, device=DEV)
    N.rnd_forward(T(x), nets[0], nets[1], 0.001, fast)
    monkeypatch.setenv("PRL_RND_GENERIC", "1")
    gen = torch.empty(n, dtype=torch.float32, device=DEV)
    N.rnd_forward(T(x), nets[0], nets[1], 0.001, gen)
    f, gn = fast.cpu().numpy(), gen.cpu().numpy()
    np.testing.assert_allclose(f, gn, rtol=2e-5, atol=1e-9)
    sub = np.unique(np.r_[np.arange(0, n, max(1, n // 997)), n - 1])
    np.testing.assert_allclose(f[sub], O.rnd_forward(x[sub], nets_np[0], nets_np[1], 0.001),
                               rtol=2e-5, atol=1e-9)


# ---------------------------------------------------------------------------------- envs
def _make_env_state(kind, E, seeds, D):
    N = native()
    dims = N.env_dims(kind)
    phys = torch.zeros(E, dims["phys_dim"], dtype=torch.float64, device=DEV)
    rng = torch.zeros(E, 4, dtype=torch.int64, device=DEV)
    t = torch.zeros(E, dtype=torch.int32, device=DEV)
    term = torch.zeros(E, dtype=torch.uint8, device=DEV)
    obs = torch.zeros(E, D, dtype=torch.float32, device=DEV)
    N.pcg64_seed(T(np.asarray(seeds, np.int64)), rng)
    return phys, rng, t, term, obs


def test_pcg64_seed_matches_numpy():
    N = native()
    seeds = np.array([0, 1, 7, 12345, 2**32 + 5, 2**40 + 3, 987654321], np.int64)
    rng = torch.zeros(len(seeds), 4, dtype=torch.int64, device=DEV)
    N.pcg64_seed(T(seeds), rng)
    got = rng.cpu().numpy().view(np.uint64)
    for i, s in enumerate(seeds):
        np.testing.assert_array_equal(got[i], O.pcg64_state_words(int(s)))


@pytest.mark.parametrize("name,kind,cls", [("cartpole", 0, O.CartPoleOracle),
                                           ("pendulum", 1, O.PendulumOracle)])
def test_env_compact_step_bit_exact_vs_oracle(name, kind, cls):
    """EnvVectorizer.step semantics: compacted actions/results, physics bit-exact (fp64 state),
    TimeLimit truncation, and resets that continue each env's numpy PCG64 stream."""
    N = native()
    E = 3000
    seeds = np.arange(E) + 77
    orc = cls(E)
    orc.seed(seeds)
    o_ref = orc.reset()
    phys, rng, t, term, obs = _make_env_state(kind, E, seeds, orc.D)
    N.env_reset(kind, phys, rng, t, term, obs, orc.D)
    np.testing.assert_array_equal(obs.cpu().numpy(), o_ref)
    np.testing.assert_array_equal(phys.cpu().numpy(), orc.state)
    arng = np.random.default_rng(5)
    mask = np.zeros(E, bool)
    n_reset = 0
    for step in range(650):
        idx = np.where(~mask)[0]
        if len(idx) == 0 or (step % 97 == 96):
            rm = mask.copy() if len(idx) else np.ones(E, bool)
            o_ref = orc.reset(rm)
            N.env_reset(kind, phys, rng, t, term, obs, orc.D, reset_mask=T(rm.astype(np.uint8)))
            mask[rm] = False
            n_reset += 1
            np.testing.assert_array_equal(obs.cpu().numpy()[rm], o_ref[rm])
            continue
        n = len(idx)
        if orc.discrete:
            acts = (arng.random(n) < 0.5).astype(np.int64)
        else:
            acts = arng.uniform(-2.5, 2.5, (n, 1)).astype(np.float32)
            acts[::50] = np.nan if step == 3 else acts[::50]
        o_r, r_r, d_r, tr_r = orc.step_envs(idx, acts)
        o_out = torch.empty(n, orc.D, dtype=torch.float32, device=DEV)
        r_out = torch.empty(n, dtype=torch.float64, device=DEV)
        d_out = torch.empty(n, dtype=torch.uint8, device=DEV)
        tr_out = torch.empty(n, dtype=torch.uint8, device=DEV)
        N.env_step_compact(kind, phys, t, T(idx), n, T(acts), o_out, r_out, d_out, tr_out)
        np.testing.assert_array_equal(bits(phys.cpu().numpy()), bits(orc.state))
        np.testing.assert_array_equal(bits(o_out.cpu().numpy()), bits(o_r))
        np.testing.assert_array_equal(bits(r_out.cpu().numpy()), bits(np.asarray(r_r, np.float64)))
        np.testing.assert_array_equal(d_out.cpu().numpy().astype(bool), d_r)
        np.testing.assert_array_equal(tr_out.cpu().numpy().astype(bool), tr_r)
        mask[idx] = d_r | tr_r
    assert n_reset >= 3


def test_synth_env_vs_oracle():
    N = native()
    E = 300
    seeds = np.arange(E) + 5
    orc = O.SynthOracle(E)
    orc.seed(seeds)
    o_ref = orc.reset()
    phys, rng, t, term, obs = _make_env_state(2, E, seeds, 348)
    N.env_reset(2, phys, rng, t, term, obs, 348)
    np.testing.assert_array_equal(obs.cpu().numpy(), o_ref)
    np.testing.assert_array_equal(phys.cpu().numpy()[:, 0], orc.L.astype(np.float64))
    arng = np.random.default_rng(1)
    mask = np.zeros(E, bool)
    for step in range(40):
        idx = np.where(~mask)[0]
        if len(idx) == 0:
            break
        n = len(idx)
        acts = arng.uniform(-1, 1, (n, 17)).astype(np.float32)
        o_r, r_r, d_r, tr_r = orc.step_envs(idx, acts)
        o_out = torch.empty(n, 348, dtype=torch.float32, device=DEV)
        r_out = torch.empty(n, dtype=torch.float64, device=DEV)
        d_out = torch.empty(n, dtype=torch.uint8, device=DEV)
        tr_out = torch.empty(n, dtype=torch.uint8, device=DEV)
        N.env_step_compact(2, phys, t, T(idx), n, T(acts), o_out, r_out, d_out, tr_out)
        np.testing.assert_array_equal(o_out.cpu().numpy(), o_r)
        np.testing.assert_array_equal(r_out.cpu().numpy(), r_r)
        np.testing.assert_array_equal(d_out.cpu().numpy().astype(bool), d_r)
        mask[idx] = d_r | tr_r


def _run_rollout(kind, E, seeds, seed, probs_fn, scaling=1.0, at=False):
    """Drive prl_rollout_step with host-provided distribution rows; returns device results.
    at=True: prl_rollout_step_at with the step index {k, arrivals} on the device (the kernel
    advances k), checked against the host's k after every step."""
    N = native()
    dims = N.env_dims(kind)
    D, A, TM = dims["obs_dim"], dims["act_dim"], dims["max_episode_steps"]
    Adim = 1 if dims["discrete"] else A
    phys, rng, t, term, _ = _make_env_state(kind, E, seeds, D)
    traj_obs = torch.zeros(TM + 1, E, D, dtype=torch.float32, device=DEV)
    traj_act = torch.zeros(TM, E, Adim, dtype=torch.float32, device=DEV)
    traj_rew = torch.zeros(TM, E, dtype=torch.float32, device=DEV)
    traj_done = torch.zeros(TM, E, dtype=torch.uint8, device=DEV)
    ep_len = torch.zeros(E, dtype=torch.int32, device=DEV)
    active_after = torch.zeros(TM, dtype=torch.int32, device=DEV)
    rsum = torch.zeros(1, dtype=torch.float64, device=DEV)
    N.env_reset(kind, phys, rng, t, term, traj_obs[0], D)
    dists = []
    k_dev = torch.zeros(2, dtype=torch.int64, device=DEV)
    for k in range(TM):
        dist = T(probs_fn(k))
        dists.append(dist)
        if at:
            N.rollout_step_at(kind, k_dev, phys, t, term, dist, scaling, seed, TM, traj_obs,
                              traj_act, traj_rew, traj_done, ep_len, active_after, rsum)
            assert k_dev.tolist() == [k + 1, 0]
        else:
            N.rollout_step(kind, k, phys, t, term, dist, scaling, seed, TM, traj_obs, traj_act,
                           traj_rew, traj_done, ep_len, active_after, rsum)
        if k % 16 == 15 and int(active_after[k]) == 0:
            break
    torch.cuda.synchronize()
    return dict(traj_obs=traj_obs, traj_act=traj_act, traj_rew=traj_rew, traj_done=traj_done,
                ep_len=ep_len, active_after=active_after, rsum=rsum, term=term, steps=k + 1,
                dims=dims)


def test_cartpole_rollout_step_bit_exact_vs_oracle():
    """The fused device worker step: sampling (Philox), physics, TimeLimit, trajectory writes,
    envs_active mask, scores — replayed by the oracle env-by-env, bit-exact."""
    E = 4099
    seeds = np.arange(E) * 3 + 11
    prng = np.random.default_rng(4)
    probs = [prng.dirichlet([1, 1], E).astype(np.float32) for _ in range(500)]
    seed = 0xDEADBEEF12345
    out = _run_rollout(0, E, seeds, seed, lambda k: probs[k])
    orc = O.CartPoleOracle(E)
    orc.seed(seeds)
    obs = orc.reset()
    ep_len = np.zeros(E, np.int32)
    mask = np.zeros(E, bool)
    tobs = out["traj_obs"].cpu().numpy()
    tact = out["traj_act"].cpu().numpy()[:, :, 0]
    tdone = out["traj_done"].cpu().numpy()
    np.testing.assert_array_equal(tobs[0], obs)
    active_after = []
    for k in range(out["steps"]):
        idx = np.where(~mask)[0]
        if len(idx) == 0:
            active_after.append(0)
            continue
        a = O.sample_categorical(probs[k], seed, np.full(E, k, np.int32))[idx]
        np.testing.assert_array_equal(tact[k, idx], a.astype(np.float32))
        o, r, d, tr = orc.step_envs(idx, a)
        done = d | tr
        np.testing.assert_array_equal(tobs[k + 1, idx], o)
        np.testing.assert_array_equal(tdone[k, idx].astype(bool), done)
        ep_len[idx] = k + 1
        mask[idx] = done
        active_after.append(int(np.sum(~mask)))
    np.testing.assert_array_equal(out["ep_len"].cpu().numpy(), ep_len)
    np.testing.assert_array_equal(out["term"].cpu().numpy().astype(bool), mask)
    np.testing.assert_array_equal(out["active_after"].cpu().numpy()[: out["steps"]], active_after)
    assert float(out["rsum"]) == float(ep_len.sum())


@pytest.mark.parametrize("kind,E", [(0, 4099), (1, 700), (2, 37)])
def test_rollout_step_at_equals_rollout_step(kind, E):
    """prl_rollout_step_at (the captured vector step: k read on the device, advanced by the
    launch's last block) writes the same bits as prl_rollout_step with k from the host, every
    buffer; and a stale k past the store (k >= t_max) adds nothing to active_after."""
    N = native()
    seeds = np.arange(E) * 5 + 3
    dims = N.env_dims(kind)
    width = 2 if kind != 2 else 2 * dims["act_dim"]
    prng = np.random.default_rng(9)
    rows = [(prng.dirichlet([1, 1], E) if kind == 0 else
             np.concatenate([prng.normal(0, 1, (E, width // 2)),
                             np.full((E, width // 2), 0.5)], 1)).astype(np.float32)
            for _ in range(dims["max_episode_steps"])]
    a = _run_rollout(kind, E, seeds, 77, lambda k: rows[k], scaling=2.0 if kind == 1 else 1.0)
    b = _run_rollout(kind, E, seeds, 77, lambda k: rows[k], scaling=2.0 if kind == 1 else 1.0,
                     at=True)
    assert a["steps"] == b["steps"]
    for key in ("traj_obs", "traj_act", "traj_rew", "traj_done", "ep_len", "active_after", "term"):
        assert torch.equal(a[key], b[key]), key
    # the episode reward sum: one float64 atomic add per block, in whatever order the blocks
    # finish (Pendulum's rewards are not integers): equal to float64 rounding, not bit for bit
    ra, rb = float(a["rsum"]), float(b["rsum"])
    assert abs(ra - rb) <= 1e-12 * max(1.0, abs(ra)), (ra, rb)
    # k beyond the store: the launch counts nothing, still advances k
    TM = dims["max_episode_steps"]
    phys, rng, t, term, _ = _make_env_state(kind, E, seeds, dims["obs_dim"])
    traj = [torch.zeros(TM + 1, E, dims["obs_dim"], device=DEV),
            torch.zeros(TM, E, 1 if dims["discrete"] else dims["act_dim"], device=DEV),
            torch.zeros(TM, E, device=DEV), torch.zeros(TM, E, dtype=torch.uint8, device=DEV),
            torch.zeros(E, dtype=torch.int32, device=DEV)]
    store = torch.zeros(TM + 8, dtype=torch.int32, device=DEV)   # guard words past [0, TM)
    N.env_reset(kind, phys, rng, t, term, traj[0][0], dims["obs_dim"])
    k_dev = torch.tensor([TM, 0], dtype=torch.int64, device=DEV)
    N.rollout_step_at(kind, k_dev, phys, t, term, T(rows[0]), 1.0, 77, TM, *traj, store[:TM],
                      torch.zeros(1, dtype=torch.float64, device=DEV))
    torch.cuda.synchronize()
    assert k_dev.tolist() == [TM + 1, 0] and int(store.abs().sum()) == 0


def test_pendulum_rollout_step_vs_oracle():
    """Continuous sampling uses ocml logf/cosf/tanhf (tolerance); given the device's sampled
    actions, the physics, truncation and trajectory are bit-exact."""
    E = 1024
    seeds = np.arange(E) + 500
    mu = np.random.default_rng(2).normal(0, 0.5, (E, 1)).astype(np.float32)
    dist = np.concatenate([mu, np.full((E, 1), 0.6, np.float32)], axis=1)
    seed = 99
    out = _run_rollout(1, E, seeds, seed, lambda k: dist, scaling=2.0)
    assert out["steps"] == 208 or int(out["active_after"][199]) == 0
    tact = out["traj_act"].cpu().numpy()[:, :, 0]
    tobs = out["traj_obs"].cpu().numpy()
    trew = out["traj_rew"].cpu().numpy()
    orc = O.PendulumOracle(E)
    orc.seed(seeds)
    np.testing.assert_array_equal(tobs[0], orc.reset())
    idx = np.arange(E)
    for k in range(200):
        # sampled action vs the oracle's libm Box-Muller + tanhf
        for e in (0, 17, 1023):
            z = O.sample_normal(seed, e, k, 0)
            ref = np.float32(np.tanh(np.float32(mu[e, 0] + np.float32(0.6) * np.float32(z)))) * 2
            assert tact[k, e] == pytest.approx(float(ref), rel=2e-6, abs=2e-6)
        o, r, d, tr = orc.step_envs(idx, tact[k][:, None])
        np.testing.assert_array_equal(tobs[k + 1], o)
        np.testing.assert_array_equal(trew[k], r.astype(np.float32))
    assert (out["ep_len"].cpu().numpy() == 200).all()
    assert int(out["traj_done"][199].sum()) == E and int(out["traj_done"][198].sum()) == 0


def test_synth_rollout_step_masks_vs_oracle():
    E = 512
    seeds = np.arange(E) + 1
    dist = np.zeros((E, 34), np.float32)
    dist[:, 17:] = 0.3
    out = _run_rollout(2, E, seeds, 3, lambda k: dist, scaling=1.0)
    orc = O.SynthOracle(E)
    orc.seed(seeds)
    orc.reset()
    np.testing.assert_array_equal(out["ep_len"].cpu().numpy(), orc.L.astype(np.int32))
    tobs = out["traj_obs"].cpu().numpy()
    for e in (0, 5, 511):
        for k in range(int(orc.L[e]) + 1):
            np.testing.assert_array_equal(tobs[k, e], orc._obs1(orc.key[e], k))


# ---------------------------------------------------------------------------------- utils
def test_mask_utils_bit_exact():
    N = native()
    rng = np.random.default_rng(3)
    for E in (1, 5, 2047, 2048, 2049, 100_000):
        m = rng.random(E) < 0.37
        term = T(m.astype(np.uint8))
        idx = torch.empty(E, dtype=torch.int64, device=DEV)
        cnt = torch.empty(1, dtype=torch.int64, device=DEV)
        N.active_indices(term, idx, cnt)
        c = int(cnt)
        assert c == int(O.number_of_active_environments(m))
        np.testing.assert_array_equal(idx[:c].cpu().numpy(), O.indexes_of_active_environments(E, m))
        d = rng.random(c) < 0.5
        N.mask_update(term, T(d.astype(np.uint8)))
        np.testing.assert_array_equal(term.cpu().numpy().astype(bool),
                                      O.update_active_environments_list(m, d))
        states = rng.normal(size=(E, 3)).astype(np.float32)
        drop = rng.random(E) < 0.5
        dst = torch.empty(E, 3, dtype=torch.float32, device=DEV)
        N.compact_rows(T(states), T(drop.astype(np.uint8)), dst, cnt)
        k = int(cnt)
        np.testing.assert_array_equal(dst[:k].cpu().numpy(), O.inactive_states_dropout(states, drop))


def test_scan_and_flatten_vs_reference_worker(golden):
    """Env-major flatten (buffer_to_target_buffer_transfer) of time-major trajectories whose
    episode lengths are the reference worker fixture's, against the reference's own memory."""
    N = native()
    g = golden("worker")
    L = g["L"].astype(np.int32)
    E = len(L)
    TM = int(L.max())
    # rebuild the scripted trajectories time-major, exactly as the device worker stores them
    obs = np.zeros((TM + 1, E, 4), np.float32)
    act = np.zeros((TM, E, 1), np.float32)
    rew = np.zeros((TM, E), np.float32)
    done = np.zeros((TM, E), np.uint8)
    for e in range(E):
        for t in range(L[e] + 1):
            a_prev = float((e + t - 1) % 2) if t > 0 else 0.0
            obs[t, e] = [e, t, a_prev, e * 0.5 + t] if t > 0 else [e, 0, 0, 0]
        for t in range(L[e]):
            act[t, e, 0] = (e + t) % 2
            rew[t, e] = np.float32(float(e) * 0.25 + (t + 1) * 0.5)
            done[t, e] = 1 if t == L[e] - 1 else 0
    offsets = torch.empty(E + 1, dtype=torch.int64, device=DEV)
    N.exclusive_scan_i32(T(L), offsets)
    n = int(offsets[-1])
    assert n == int(L.sum())
    S = torch.empty(n, 4, dtype=torch.float32, device=DEV)
    A = torch.empty(n, 1, dtype=torch.float32, device=DEV)
    R = torch.empty(n, dtype=torch.float32, device=DEV)
    Dn = torch.empty(n, dtype=torch.float32, device=DEV)
    N.flatten_env_major(offsets, n, T(obs), T(act), T(rew), T(done), S, A, R, Dn)
    np.testing.assert_array_equal(S.cpu().numpy(), g["S"])
    np.testing.assert_array_equal(A.cpu().numpy()[:, 0], g["A"])
    np.testing.assert_array_equal(R.cpu().numpy(), g["R"])
    np.testing.assert_array_equal(Dn.cpu().numpy(), g["D"])


@pytest.mark.parametrize("E,D", [(65_536, 4), (3, 3), (1000, 348), (500, 350)])
def test_flatten_large_vs_numpy(E, D):
    N = native()
    rng = np.random.default_rng(E)
    TM = 60
    L = rng.integers(1, TM + 1, E).astype(np.int32)
    L[::7] = 0 if E > 7 else L[::7]   # zero-length envs are skipped
    obs = rng.normal(size=(TM + 1, E, D)).astype(np.float32)
    act = rng.normal(size=(TM, E, 2)).astype(np.float32)
    rew = rng.normal(size=(TM, E)).astype(np.float32)
    done = (rng.random((TM, E)) < 0.5).astype(np.uint8)
    offsets = torch.empty(E + 1, dtype=torch.int64, device=DEV)
    N.exclusive_scan_i32(T(L), offsets)
    n = int(L.sum())
    np.testing.assert_array_equal(offsets.cpu().numpy(), np.concatenate([[0], np.cumsum(L)]))
    S = torch.empty(n, D, dtype=torch.float32, device=DEV)
    A = torch.empty(n, 2, dtype=torch.float32, device=DEV)
    R = torch.empty(n, dtype=torch.float32, device=DEV)
    Dn = torch.empty(n, dtype=torch.float32, device=DEV)
    N.flatten_env_major(offsets, n, T(obs), T(act), T(rew), T(done), S, A, R, Dn)
    e_of = np.repeat(np.arange(E), L)
    t_of = np.concatenate([np.arange(x) for x in L])
    np.testing.assert_array_equal(S.cpu().numpy(), obs[t_of, e_of])
    np.testing.assert_array_equal(A.cpu().numpy(), act[t_of, e_of])
    np.testing.assert_array_equal(R.cpu().numpy(), rew[t_of, e_of])
    np.testing.assert_array_equal(Dn.cpu().numpy(), done[t_of, e_of].astype(np.float32))


# ---------------------------------------------------------------------------------- GroupNorm
def _gn_silu_f64(x, w, b, dout, eps=1e-5):
    x = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    w = torch.tensor(w, dtype=torch.float64, requires_grad=True)
    b = torch.tensor(b, dtype=torch.float64, requires_grad=True)
    N = x.shape[0]
    g = x.view(N, 8, 8)
    mu = g.mean(-1, keepdim=True)
    var = g.var(-1, unbiased=False, keepdim=True)
    y = ((g - mu) / torch.sqrt(var + eps)).view(N, 64) * w + b
    z = y * torch.sigmoid(y)
    z.backward(torch.tensor(dout, dtype=torch.float64))
    return z.detach().numpy(), x.grad.numpy(), w.grad.numpy(), b.grad.numpy()


@pytest.mark.parametrize("N", [1, 7, 31, 512, 513, 7681, 65_536])
def test_gn_silu_fwd_bwd_vs_float64(N):
    """The fused GroupNorm(8,64)+SiLU against a float64 restatement — including N >= 512, where
    PyTorch-ROCm's own GroupNorm backward returns wrong dw/db (tools/diag_groupnorm.py)."""
    N_ = native()
    rng = np.random.default_rng(N)
    x = (rng.normal(size=(N, 64)) * 3 + 1).astype(np.float32)
    w = (rng.normal(size=64) * 0.5 + 1).astype(np.float32)
    b = (rng.normal(size=64) * 0.1).astype(np.float32)
    dz = rng.normal(size=(N, 64)).astype(np.float32)
    z_ref, dx_ref, dw_ref, db_ref = _gn_silu_f64(x, w, b, dz)
    out = torch.empty(N, 64, dtype=torch.float32, device=DEV)
    N_.gn_silu_fwd(T(x), T(w), T(b), 1e-5, True, out)
    dx = torch.empty_like(out)
    dw = torch.empty(64, dtype=torch.float32, device=DEV)
    db = torch.empty(64, dtype=torch.float32, device=DEV)
    for _ in range(2):   # twice: the multi-block hand-off re-arms its workspace
        N_.gn_silu_bwd(T(x), T(dz), T(w), T(b), 1e-5, True, dx, dw, db)
    rel = lambda a, r: float(np.abs(a - r).max() / (np.abs(r).max() + 1e-30))  # noqa: E731
    assert rel(out.cpu().numpy(), z_ref) < 2e-6
    assert rel(dx.cpu().numpy(), dx_ref) < 1e-5
    assert rel(dw.cpu().numpy(), dw_ref) < 2e-5
    assert rel(db.cpu().numpy(), db_ref) < 2e-5


def test_gn_silu_module_grads_match_cpu_reference():
    from PPO.layers import GroupNormSiLU
    torch.manual_seed(0)
    m_cpu = torch.nn.Sequential(torch.nn.Linear(4, 64, bias=False), torch.nn.GroupNorm(8, 64),
                                torch.nn.SiLU())
    m_gpu = torch.nn.Sequential(torch.nn.Linear(4, 64, bias=False), GroupNormSiLU(8, 64),
                                torch.nn.Identity()).cuda()
    m_gpu.load_state_dict(m_cpu.state_dict())
    x = torch.randn(2048, 4)
    (m_cpu(x) ** 2).sum().backward()
    (m_gpu(x.cuda()) ** 2).sum().backward()
    for (n, a), (_, g) in zip(m_cpu.named_parameters(), m_gpu.named_parameters()):
        torch.testing.assert_close(g.grad.cpu(), a.grad, rtol=2e-5, atol=2e-5, msg=n)


def test_gae_statistics_exact_size_workspace_every_tile_count():
    """Regression: the workspace layout is carved from the buffer's size; an exact-size buffer
    (prl_workspace_bytes(n), fresh) must hold every tile's carry granule AND statistics record.
    A rounding error once carved one tile too few, so the last tile's granule overwrote tile 0's
    sum of advantages — only when that block happened to finish late, so the check runs under a
    concurrent load on another stream and repeats each size."""
    import ctypes
    import prl_native as P
    side = torch.cuda.Stream()
    big = torch.empty(32 << 20, device="cuda")
    for nt in list(range(1, 70)) + [127, 128, 129, 700]:
        n = nt * 2048 - 5
        g = torch.Generator(device="cuda").manual_seed(nt)
        r = torch.randn(n, device="cuda", generator=g)
        V = torch.randn(n, device="cuda", generator=g)
        d = (torch.rand(n, device="cuda", generator=g) < 0.05).float()
        d[-1] = 1
        nbytes = P.workspace_bytes(P.OP_GAE, n)
        ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
        for rep in range(3):
            with torch.cuda.stream(side):
                big.mul_(1.0001)
            ret, adv = torch.empty_like(V), torch.empty_like(V)
            sums = torch.zeros(2, dtype=torch.float64, device="cuda")
            rc = P.lib().prl_gae(ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(d.data_ptr()),
                                 ctypes.c_void_p(V.data_ptr()), None, n, 0.995, 0.95,
                                 ctypes.c_void_p(ret.data_ptr()), ctypes.c_void_p(adv.data_ptr()),
                                 ctypes.c_void_p(sums.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                 nbytes, P._stream())
            assert rc == 0, P.lib().prl_last_error()
            a = adv.double()
            host = torch.stack([a.sum(), (a * a).sum()])
            torch.testing.assert_close(sums, host, rtol=1e-12, atol=1e-9,
                                       msg=f"nt={nt} rep={rep}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("fin,fout,bias", [(348, 64, False), (348, 64, True), (64, 348, True)])
def test_split_k_linear_grads_vs_float64(fin, fout, bias):
    """PPO.layers.Linear on a large device batch (65,536 + 123 rows: 16 split-K chunks of 4,096
    plus a remainder) gives the float64 input / weight / bias gradients of x W^T + b to float32
    accumulation accuracy, and the same forward as F.linear (bit-exact)."""
    from PPO.layers import Linear
    torch.manual_seed(3)
    N = 65536 + 123
    lin = Linear(fin, fout, bias=bias).cuda()
    x = torch.randn(N, fin, device="cuda", requires_grad=True)
    dy = torch.randn(N, fout, device="cuda")
    y = lin(x)
    assert torch.equal(y.detach(), torch.nn.functional.linear(x.detach(), lin.weight.detach(),
                                                            None if lin.bias is None else lin.bias.detach()))
    y.backward(dy)
    x64, dy64, w64 = x.detach().double().cpu(), dy.double().cpu(), lin.weight.detach().double().cpu()
    gw = dy64.t() @ x64
    gx = dy64 @ w64
    torch.testing.assert_close(lin.weight.grad.double().cpu(), gw, rtol=0, atol=2e-5 * float(gw.abs().max()))
    torch.testing.assert_close(x.grad.double().cpu(), gx, rtol=0, atol=2e-5 * float(gx.abs().max()))
    if bias:
        gb = dy64.sum(0)
        torch.testing.assert_close(lin.bias.grad.double().cpu(), gb, rtol=0,
                                   atol=2e-5 * float(dy64.abs().sum(0).max()))


@pytest.mark.parametrize("mb", [512, 4096 + 4])
def test_gather_minibatch_every_cursor_bit_exact(mb):
    """prl_gather_minibatch (graph-step input copy) for every minibatch index incl. the ragged
    last one (zero-filled past the end): widths 1, 3, 348 (16-B rows), 5 (element path) and an
    odd row offset, against torch slicing."""
    import prl_native
    g = torch.Generator(device="cuda").manual_seed(9)
    nrows = 3 * mb + 37
    widths = [1, 3, 348, 5]
    srcs = [torch.randn(nrows, w, device="cuda", generator=g) if w > 1
            else torch.randn(nrows, device="cuda", generator=g) for w in widths]
    dsts = [torch.full((mb, w) if w > 1 else (mb,), float("nan"), device="cuda") for w in widths]
    cursor = torch.zeros(1, dtype=torch.int64, device="cuda")
    gat = prl_native.MinibatchGather(srcs, dsts, cursor, mb)
    for j in range(-(-nrows // mb)):
        cursor.fill_(j)
        gat()
        torch.cuda.synchronize()
        for s_, d_ in zip(srcs, dsts):
            ref = torch.zeros_like(d_)
            part = s_[j * mb:(j + 1) * mb]
            ref[:part.shape[0]] = part
            assert torch.equal(d_, ref), (j, s_.shape)


@pytest.mark.parametrize("rows,cols", [(0, 5), (1, 1), (65536 + 123, 1), (65536, 17), (1000, 64),
                                       (65536, 348), (7, 1024), (1 << 20, 348)])
def test_colsum_vs_float64_and_deterministic(rows, cols):
    """prl_colsum_f32 (the large-batch Linear's bias gradient) against float64 column sums, and
    bit-identical across two calls (fixed reduction order)."""
    import prl_native
    g = torch.Generator(device="cuda").manual_seed(rows + cols)
    x = torch.randn(rows, cols, device="cuda", generator=g)
    a = prl_native.colsum(x)
    b = prl_native.colsum(x)
    assert torch.equal(a, b)
    ref = x.double().sum(0).cpu()
    scale = x.double().abs().sum(0).cpu().clamp_min(1e-30)
    assert float(((a.double().cpu() - ref).abs() / scale).max() if rows else a.abs().max()) < 1e-6
