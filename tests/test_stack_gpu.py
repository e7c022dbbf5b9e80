"""The drop-in API on the GPU: EnvVectorizer / utils / AsyncPPO.worker / PPO.learn against the
reference's golden vectors and the oracle."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def test_env_vectorizer_vs_reference_fixture(golden):
    """The reference's EnvVectorizer over (restated) gymnasium envs, same seeds, same actions:
    compacted outputs and envs_active masks; masks exact, observations within trig ulps."""
    from AsyncTools.AsyncPPO import EnvVectorizer
    g = golden("envs")
    for name, env_id in (("cartpole", "CartPole-v1"), ("pendulum", "Pendulum-v1")):
        seeds = g[f"{name}_seeds"]
        vec = EnvVectorizer(env_id, len(seeds), seed=int(seeds[0]))
        vec.reset()                        # the reset(seed=...) draw
        obs0, infos = vec.reset()          # EnvVectorizer.reset(): second draw
        np.testing.assert_array_equal(obs0, g[f"{name}_obs0"])
        assert len(infos) == len(seeds)
        off = 0
        for step, n in enumerate(g[f"{name}_nact"]):
            n = int(n)
            if n < 0:
                o, _ = vec.reset()
                np.testing.assert_array_equal(o, g[f"{name}_obs"][off:off - n])
                off += -n
                continue
            acts = g[f"{name}_act"][off:off + n]
            if name == "cartpole":
                acts = acts[:, 0].astype(np.int64)
            o, r, d, tr, inf = vec.step(acts)
            sl = slice(off, off + n)
            assert o.shape == (n, g[f"{name}_obs"].shape[1]) and len(inf) == n
            np.testing.assert_allclose(o, g[f"{name}_obs"][sl], rtol=0, atol=1e-5)
            np.testing.assert_allclose(r, g[f"{name}_rew"][sl], rtol=1e-9, atol=1e-9)
            np.testing.assert_array_equal(d, g[f"{name}_term"][sl])
            np.testing.assert_array_equal(tr, g[f"{name}_trunc"][sl])
            m = vec.envs_active
            m[np.where(~m)[0]] = d | tr
            vec.envs_active = m
            np.testing.assert_array_equal(vec.envs_active, g[f"{name}_mask"][step])
            off += n


def test_utils_numpy_api_vs_oracle():
    import AsyncTools.utils as U
    rng = np.random.default_rng(0)
    for E in (1, 4, 33, 5000):
        m = rng.random(E) < 0.4
        np.testing.assert_array_equal(U.indexes_of_active_environments(E, m),
                                      O.indexes_of_active_environments(E, m))
        assert U.number_of_active_environments(m) == O.number_of_active_environments(m)
        np.testing.assert_array_equal(U.range_of_active_environments(m),
                                      np.arange(O.number_of_active_environments(m)))
        s = rng.normal(size=(E, 4))
        d = rng.random(E) < 0.5
        np.testing.assert_array_equal(U.inactive_states_dropout(s, d), O.inactive_states_dropout(s, d))
        n = int(np.sum(~m))
        dn = rng.random(n) < 0.3
        ref = O.update_active_environments_list(m, dn)
        out = U.update_active_environments_list(m, dn)
        assert out is m                                # in place, like the reference
        np.testing.assert_array_equal(out, ref)


class _DetPPO:
    """Duck-typed ppo for the compat worker: deterministic actions from the observation."""

    def __init__(self):
        from PPO import Memory
        self.memory = Memory()

    def get_action(self, states):
        s = states.numpy()
        return (s[:, 2] + 0.1 * s[:, 3] > 0).astype(np.int64)

    def learn(self):
        pass


def test_compat_worker_vs_oracle_worker():
    from AsyncTools.AsyncPPO import AsyncPPO
    E, seed = 300, 42
    ppo = _DetPPO()
    a = AsyncPPO("CartPole-v1", ppo, num_envs=E, seed=seed)
    a.step_score, a.reward_score = 0, 0
    a.worker()
    orc = O.CartPoleOracle(E)
    orc.seed(np.arange(E) + seed)
    ref = O.worker_oracle(orc, lambda s, idx, t: (s[:, 2] + 0.1 * s[:, 3] > 0).astype(np.int64))
    np.testing.assert_array_equal(np.array(ppo.memory.states), ref["S"])
    np.testing.assert_array_equal(np.array(ppo.memory.actions), ref["A"])
    np.testing.assert_array_equal(np.array(ppo.memory.dones), ref["D"])
    assert int(a.step_score) == ref["step_score"] == len(ref["S"])


class _FixedDist:
    def __init__(self, rows, scaling=None):
        from PPO import Memory
        self.memory = Memory()
        self.rows = rows
        self.action_scaling = scaling

    def dist_params(self, obs):
        return self.rows


@pytest.mark.parametrize("E", [1, 2048, 65536])
def test_device_worker_bit_exact_vs_oracle_worker(E):
    from AsyncTools.AsyncPPO import AsyncPPO
    seed = 7
    probs = np.random.default_rng(E).dirichlet([2, 2], E).astype(np.float32)
    stub = _FixedDist(torch.from_numpy(probs).cuda())
    a = AsyncPPO("CartPole-v1", stub, num_envs=E, seed=seed)
    n = a.worker()
    S, A, R, Dn = (x.cpu().numpy() for x in stub.memory.device_tensors("cuda"))
    orc = O.CartPoleOracle(E)
    orc.seed(np.arange(E) + seed)
    ss = a.sample_seed
    ref = O.worker_oracle(orc, lambda s, idx, t: O.sample_categorical(
        probs, ss, np.full(E, t, np.int32))[idx])
    assert n == len(ref["S"]) == int(a.step_score)
    np.testing.assert_array_equal(S, ref["S"])
    np.testing.assert_array_equal(A, ref["A"])
    np.testing.assert_array_equal(R, ref["R"])
    np.testing.assert_array_equal(Dn, ref["D"])
    assert float(a.reward_score) == float(ref["reward_score"])
    # a second rollout reuses the buffers, continues every env's PCG64 stream
    a.worker()
    assert len(stub.memory) == n + len(stub.memory._segments[1][0])


@pytest.mark.parametrize("E", [1, 2048, 65536])
def test_cartpole_persistent_rollout_matches_oracle_given_its_probs(E):
    """The whole CartPole rollout as one launch (prl_cartpole_rollout: one thread per env runs
    the actor's forward, Categorical sampling, the float64 step and the trajectory push to the end
    of its episode), through AsyncPPO.worker() with the real policy.  Its forward sums in another
    order than the per-step path's PyTorch GEMMs, so the check is: (1) its probabilities at EVERY
    step of every env (the row of probs_out it sampled from) against a float64 forward of
    policy_old on the state the env was in (the memory's env-major rows: 1e-5), and (2) given the
    probabilities it sampled
    from at every step (probs_out), the oracle worker (AsyncPPO.py:117-146 with the oracle's
    Philox sampling and gymnasium 1.1.1 physics) reproduces the memory bit for bit — states,
    actions, rewards, done flags, lengths and the score counters."""
    import copy

    import prl_native
    from AsyncTools.AsyncPPO import AsyncPPO
    from PPO import PPO
    torch.manual_seed(3)
    seed = 5
    ppo = PPO(False, 4, 2)
    ppo.show_progress = False
    T = 500
    probs = torch.zeros(T, E, 2, dtype=torch.float32, device="cuda")
    calls = []
    orig = prl_native.wide_rollout

    def wrapped(kind, flat, D, A, discrete, phys, t, term, scaling, sd, t_max, *rest):
        calls.append(kind)
        prl_native.cartpole_rollout(flat, phys, t, term, sd, t_max, *rest, probs_out=probs)

    a = AsyncPPO("CartPole-v1", ppo, num_envs=E, seed=seed)
    S0 = None
    prl_native.wide_rollout = wrapped
    try:
        n = a.worker()
    finally:
        prl_native.wide_rollout = orig
    assert calls == [prl_native.ENV_KINDS["CartPole-v1"]]
    S, A, R, Dn = (x.cpu().numpy() for x in ppo.memory.device_tensors("cuda"))
    P = probs.cpu().numpy()
    orc = O.CartPoleOracle(E)
    orc.seed(np.arange(E) + seed)
    ss = a.sample_seed

    def act(states, idx, t):
        return O.sample_categorical(P[t], ss, np.full(E, t, np.int32))[idx]

    ref = O.worker_oracle(orc, act)
    assert n == len(ref["S"]) == int(a.step_score)
    np.testing.assert_array_equal(S, ref["S"])
    np.testing.assert_array_equal(A, ref["A"])
    np.testing.assert_array_equal(R, ref["R"])
    np.testing.assert_array_equal(Dn, ref["D"])
    assert float(a.reward_score) == float(ref["reward_score"])
    # (1) every step's probabilities against a float64 forward of policy_old: memory row k of
    # env e (env-major) is env e's state at step t = k - (its first row), sampled from P[t, e]
    lens = ref["lengths"]
    env_of = np.repeat(np.arange(E), lens)
    t_of = np.arange(n) - np.repeat(np.cumsum(lens) - lens, lens)
    pol = copy.deepcopy(ppo.policy_old).cpu().double()
    with torch.no_grad():
        p64 = pol.actor(pol.model(torch.from_numpy(S).double())).numpy()
    assert t_of.max() > 8     # the check reaches well past the reset neighbourhood
    np.testing.assert_allclose(P[t_of, env_of].astype(np.float64), p64, rtol=0, atol=1e-5)


def test_evaluate_matches_oracle_episodes():
    """AsyncPPO.evaluate() (Test.py:19-35 batched, no render): per-env episode returns and
    lengths equal the oracle's replay of the same rollout (same PCG64 resets, the evaluation's
    own Philox key); nothing is pushed to memory and the score counters stay untouched; a
    training rollout afterwards uses the same keys as without the evaluation."""
    from AsyncTools.AsyncPPO import AsyncPPO
    E, seed = 512, 11
    probs = np.random.default_rng(3).dirichlet([2, 2], E).astype(np.float32)
    stub = _FixedDist(torch.from_numpy(probs).cuda())
    a = AsyncPPO("CartPole-v1", stub, num_envs=E, seed=seed)
    ret, lens = a.evaluate()
    assert len(stub.memory) == 0 and int(a.step_score) == 0 and float(a.reward_score) == 0.0
    orc = O.CartPoleOracle(E)
    orc.seed(np.arange(E) + seed)
    es = ((a.sample_seed ^ 0x5851F42D4C957F2D) + 0) & (2**64 - 1)
    ref = O.worker_oracle(orc, lambda s, idx, t: O.sample_categorical(
        probs, es, np.full(E, t, np.int32))[idx])
    ends = np.flatnonzero(ref["D"] == 1)
    ref_len = np.diff(np.concatenate([[-1], ends]))
    assert len(ref_len) == E
    np.testing.assert_array_equal(lens, ref_len)
    ref_ret = np.add.reduceat(ref["R"].astype(np.float64), np.concatenate([[0], ends[:-1] + 1]))
    np.testing.assert_array_equal(ret, ref_ret)
    # training keys unaffected: the first worker() after evaluate() samples with sample_seed
    b = AsyncPPO("CartPole-v1", _FixedDist(torch.from_numpy(probs).cuda()), num_envs=E, seed=seed)
    b.evaluate()
    n = b.worker()
    orc2 = O.CartPoleOracle(E)
    orc2.seed(np.arange(E) + seed)
    O.worker_oracle(orc2, lambda s, idx, t: O.sample_categorical(
        probs, es, np.full(E, t, np.int32))[idx])          # the evaluation's episode
    ref2 = O.worker_oracle(orc2, lambda s, idx, t: O.sample_categorical(
        probs, b.sample_seed, np.full(E, t, np.int32))[idx])
    assert n == len(ref2["S"])
    S = b.ppo.memory.device_tensors("cuda")[0].cpu().numpy()
    np.testing.assert_array_equal(S, ref2["S"])


def test_device_worker_pendulum_shapes_and_truncation():
    from AsyncTools.AsyncPPO import AsyncPPO
    E = 4096
    rows = torch.zeros(E, 2, device="cuda")
    rows[:, 1] = 0.5
    stub = _FixedDist(rows, scaling=2.0)
    a = AsyncPPO("Pendulum-v1", stub, num_envs=E, seed=3)
    n = a.worker()
    assert n == 200 * E
    S, A, R, Dn = stub.memory.device_tensors("cuda")
    assert S.shape == (n, 3) and A.shape == (n, 1)
    assert float(A.abs().max()) <= 2.0
    d = Dn.view(E, 200)
    assert int(d[:, -1].sum()) == E and int(d[:, :-1].sum()) == 0
    assert a.last_vector_steps <= 200 + a.poll_lag + 1


@pytest.mark.parametrize("path", ["fused", "graph"])
def test_learn_on_gpu_matches_reference_learn(golden, path):
    """PPO.learn() through libprl_hip.so vs the reference's learn(): same seeded policy, same
    memory -> same updated weights (GPU float32 GEMMs differ from CPU ones in rounding).
    path "fused": the whole update loop in the persistent engine; "graph": per-step graphs."""
    from PPO import PPO
    for tag, cont in (("learn", False), ("learn_cont", True)):
        g = golden(tag)
        torch.manual_seed(0)
        D, A = (3, 1) if cont else (4, 2)
        p = PPO(is_continuous=cont, observ_dim=D, action_dim=A,
                action_scaling=2.0 if cont else None, lr=1e-3, k_epochs=int(g["k_epochs"]),
                policy_clip=0.2, GAE_lambda=0.95, gamma=0.995, batch_size=1024,
                mini_batch_size=int(g["mb"]))
        p.show_progress = False
        p.use_fused = path == "fused"
        for i in range(int(g["N"])):
            p.memory.push(g["S"][i], g["A"][i] if cont else np.asarray(g["A"][i]), g["R"][i],
                          g["Dn"][i])
        p.learn()
        assert p.last_update_path == path
        sd = p.policy.state_dict()
        for k in sd:
            np.testing.assert_allclose(sd[k].cpu().numpy(), g["final/" + k], rtol=0, atol=2e-6,
                                       err_msg=f"{tag}:{k}")


def test_learn_c1_hyperparameters_match_reference_learn(golden):
    """C1 at its own hyper-parameters (README.md:35-49; BASELINE configs[0]): batch 1,024,
    mini_batch 512, k_epochs 11 — 33 sequential optimizer steps over a 1,500-row CartPole memory
    (two full minibatches and a ragged third) through the fused engine's latency form, against
    the reference's own learn() (tests/golden/learn_c1.npz, make_golden.py), at the CartPole
    2e-6 bound of test_learn_on_gpu_matches_reference_learn."""
    import prl_native
    from PPO import PPO
    g = golden("learn_c1")
    assert (int(g["mb"]), int(g["k_epochs"]), int(g["N"])) == (512, 11, 1500)
    torch.manual_seed(0)
    p = PPO(is_continuous=False, observ_dim=4, action_dim=2, lr=1e-3, k_epochs=11,
            policy_clip=0.2, GAE_lambda=0.95, gamma=0.995, batch_size=1024, mini_batch_size=512)
    p.show_progress = False
    init = {k[len("init/"):]: torch.from_numpy(g[k]) for k in g.files if k.startswith("init/")}
    for k, v in p.policy.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), init[k].numpy(), err_msg=k)
    for i in range(int(g["N"])):
        p.memory.push(g["S"][i], np.asarray(g["A"][i]), g["R"][i], g["Dn"][i])
    p.learn()
    torch.cuda.synchronize()
    assert p.last_update_path == "fused"
    plan = prl_native.ppo_update_last_plan()
    assert plan["form"] == "latency" and plan["specialised"], plan
    _, _, _, adv, returns = p._last_update_inputs
    ret_ref = g["returns"].astype(np.float64)
    assert np.all(np.abs(returns.cpu().double().numpy() - ret_ref) <= 1e-5 * np.abs(ret_ref) + 1e-5)
    sd = p.policy.state_dict()
    worst = max(float(np.abs(sd[k].cpu().numpy() - g["final/" + k]).max()) for k in sd)
    moved = max(float(np.abs(g["final/" + k] - init[k].numpy()).max()) for k in sd)
    print(f"learn_c1: max |w - w_ref| {worst:.3e} (33 steps moved weights by up to {moved:.3e})")
    for k in sd:
        np.testing.assert_allclose(sd[k].cpu().numpy(), g["final/" + k], rtol=0, atol=2e-6,
                                   err_msg=f"learn_c1:{k}")


def test_compute_gae_api_returns_reference_list(golden):
    from PPO import PPO
    g = golden("gae")
    p = PPO(False, 4, 2, gamma=float(g["c_gamma"]), GAE_lambda=float(g["c_lam"]))
    out = p.compute_gae(g["c_r"], g["c_d"], g["c_V"], g["c_nv"])
    assert isinstance(out, list) and isinstance(out[0], np.float32)
    np.testing.assert_array_equal(np.array(out).view(np.uint32), g["c_ret"].view(np.uint32))


def test_rnd_module_matches_reference(golden):
    from PPO import RND
    g = golden("rnd")
    for D in (4, 348):
        r = RND(D, D, beta=0.001)
        sd = {k[len(f"D{D}/"):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(f"D{D}/")}
        r.load_state_dict(sd)
        x = torch.from_numpy(g[f"D{D}_x"]).cuda()
        out = r.compute_intrinsic_reward(list(x.split(64)))
        np.testing.assert_allclose(out.cpu().numpy(), g[f"D{D}_r"], rtol=2e-5, atol=1e-8)
        # must run: the native prl_rnd_pred_grad + prl_flat_adamw step (its numbers are checked
        # in test_rnd_learn_gpu.py)
        r.update_pred(list(x.split(64)))


def test_gae_graph_capture_replay():
    """One prl_gae call is one kernel launch with a self-re-arming workspace: capture it in a
    HIP graph and replay it; every replay is bit-exact."""
    import prl_native
    n = 300_000
    g = torch.Generator(device="cuda").manual_seed(1)
    r = torch.randn(n, device="cuda", generator=g)
    V = torch.randn(n, device="cuda", generator=g)
    d = (torch.rand(n, device="cuda", generator=g) < 0.05).float()
    ret = torch.empty_like(V)
    adv = torch.empty_like(V)
    sums = torch.zeros(2, dtype=torch.float64, device="cuda")
    prl_native.gae(r, d, V, None, 0.995, 0.95, ret, adv, sums)   # warm + allocate workspace
    ref = O.gae(r.cpu().numpy(), d.cpu().numpy(), V.cpu().numpy(), float(V[-1]), 0.995, 0.95)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            prl_native.gae(r, d, V, None, 0.995, 0.95, ret, adv, sums)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        ret.zero_()
        graph.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(ret.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    a64 = (ref - V.cpu().numpy()).astype(np.float32).astype(np.float64)
    assert float(sums[0]) == pytest.approx(a64.sum(), rel=1e-10, abs=1e-6)


def test_training_improves_cartpole():
    """End to end: AsyncPPO.run() with the device worker learns CartPole (episode length grows)."""
    from AsyncTools.AsyncPPO import AsyncPPO
    from PPO import PPO
    torch.manual_seed(0)
    ppo = PPO(False, 4, 2, lr=1e-3, k_epochs=4, batch_size=4096, mini_batch_size=4096)
    ppo.show_progress = False
    a = AsyncPPO("CartPole-v1", ppo, num_envs=1024, seed=0)
    lens = []
    for _ in range(12):
        a.step_score, a.reward_score = 0, 0
        n = a.worker()
        lens.append(n / 1024)
        ppo.learn()
    assert np.mean(lens[-3:]) > 1.5 * np.mean(lens[:2]), lens


@pytest.mark.parametrize("cont", [False, True])
def test_graphed_update_equals_eager_update(cont):
    """The HIP-graph optimizer step (replayed per minibatch, device cursor) produces exactly the
    eager step's updates: same kernels, same order, same minibatches."""
    from PPO import PPO
    rng = np.random.default_rng(5)
    N, D, A = 20_000 + 77, (3 if cont else 4), 1 if cont else 2
    S = torch.from_numpy((rng.normal(size=(N, D)) * 0.5).astype(np.float32)).cuda()
    Aa = (torch.from_numpy(np.tanh(rng.normal(size=(N, 1))).astype(np.float32) * 2).cuda() if cont
          else torch.from_numpy((rng.random(N) < 0.5).astype(np.float32)).cuda())
    R = torch.from_numpy(rng.normal(1, 0.5, N).astype(np.float32)).cuda()
    Dn = torch.from_numpy((rng.random(N) < 0.05).astype(np.float32)).cuda()
    Dn[-1] = 1
    results = []
    for graphs in (False, True):
        torch.manual_seed(0)
        p = PPO(cont, D, A, action_scaling=2.0 if cont else None, k_epochs=3, batch_size=1024,
                mini_batch_size=256)
        p.show_progress = False
        p.use_fused = False            # this test is about the per-step graph path
        p.use_graphs = graphs
        p.memory.push_device(S, Aa, R, Dn)
        p.learn()
        results.append({k: v.clone() for k, v in p.policy.state_dict().items()})
        results.append(p.last_loss.clone())
    sd_e, loss_e, sd_g, loss_g = results
    for k in sd_e:
        torch.testing.assert_close(sd_g[k], sd_e[k], rtol=0, atol=0, msg=k)
    assert float(loss_g) == float(loss_e)


@pytest.mark.parametrize("env,cont,step_at", [("CartPole-v1", False, "1"), ("Pendulum-v1", True, "1"),
                                              ("CartPole-v1", False, "0")])
def test_graphed_rollout_equals_eager_rollout(env, cont, step_at, monkeypatch):
    """From the second rollout on, the device worker replays one captured HIP graph per vector
    step (policy forward + rollout step kernel, step index on the device).  Three rollouts with a
    real PPO policy: the graphed runner's memory and scores equal an eager runner's
    (PRL_ROLLOUT_GRAPH=0) bit for bit.  step_at "1" (default): the captured step kernel counts
    into active_after[k] and advances k itself (prl_rollout_step_at); "0": round 3's scalar +
    index copy + increment nodes (PRL_ROLLOUT_STEP_AT=0)."""
    monkeypatch.setenv("PRL_ROLLOUT_STEP_AT", step_at)
    # the per-step path (CartPole's real policy otherwise runs the one-launch rollout,
    # test_cartpole_persistent_rollout_matches_oracle_given_its_probs)
    monkeypatch.setenv("PRL_CP_ROLLOUT", "0")
    from AsyncTools.AsyncPPO import AsyncPPO
    from PPO import PPO
    outs = []
    for graphed in ("1", "0"):
        monkeypatch.setenv("PRL_ROLLOUT_GRAPH", graphed)
        torch.manual_seed(0)
        p = PPO(cont, 3 if cont else 4, 1 if cont else 2, action_scaling=2.0 if cont else None,
                batch_size=10**9)
        a = AsyncPPO(env, p, num_envs=3000, seed=5)
        rec = []
        for _ in range(3):
            n = a.worker()
            rec.append((n, float(a.reward_score)))   # (vector steps taken depend on poll timing)
        assert (a._graph is not None) == (graphed == "1")
        outs.append((rec, [x.cpu() for x in p.memory.device_tensors("cuda")]))
    (r1, m1), (r0, m0) = outs
    assert r1 == r0
    for x, y in zip(m1, m0):
        assert torch.equal(x, y)
