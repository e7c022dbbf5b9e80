"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.npz, produced by
tests/golden/make_golden.py importing the reference).  CPU only."""
import math

import numpy as np
import pytest

import oracle as O


# ---------------------------------------------------------------------------------- GAE
@pytest.mark.parametrize("case", list("abcde"))
def test_gae_oracle_bit_exact_vs_reference(golden, case):
    g = golden("gae")
    ret = O.gae(g[f"{case}_r"], g[f"{case}_d"], g[f"{case}_V"], g[f"{case}_nv"],
                float(g[f"{case}_gamma"]), float(g[f"{case}_lam"]))
    np.testing.assert_array_equal(ret.view(np.uint32), g[f"{case}_ret"].view(np.uint32))


def test_gae_python_restatement_matches_c(golden):
    g = golden("gae")
    r, d, V = g["a_r"][:300], g["a_d"][:300].copy(), g["a_V"][:300]
    d[-1] = 1
    a = O.gae_python(r, d, V, V[-1], 0.995, 0.95)
    b = O.gae(r, d, V, V[-1], 0.995, 0.95)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


# ---------------------------------------------------------------------------------- learn
@pytest.mark.parametrize("tag", ["learn", "learn_cont", "learn_rnd", "learn_rnd_c5", "learn_rnd_big",
                                 "learn_c1"])
def test_learn_gae_and_advantages(golden, tag):
    """GAE returns and ret - V bit-exact (with use_RND the rewards are R + r_int, PPO.py:171);
    normalised advantages within north_star's 1e-5 relative, with a 1e-6 absolute guard (in
    units of the normalised scale) for values near zero: the reference's float32 torch mean/std
    vs our float64 statistics (measured max |diff| 4.8e-7)."""
    g = golden(tag)
    V = g["old_V"]
    R = g["R"] + g["r_int"] if "r_int" in g.files else g["R"]
    ret = O.gae(R, g["Dn"], V, V[-1], 0.995, 0.95)
    np.testing.assert_array_equal(ret.view(np.uint32), g["returns"].view(np.uint32))
    adv_n, adv_raw = O.adv_normalize(ret, V)
    np.testing.assert_array_equal(adv_raw.view(np.uint32), g["adv_raw"].view(np.uint32))
    np.testing.assert_allclose(adv_n, g["adv"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tag", ["learn", "learn_cont"])
def test_surrogate_grads_vs_reference_autograd(golden, tag):
    g = golden(tag)
    mb, N = int(g["mb"]), int(g["N"])
    nsteps = int(g["k_epochs"]) * (-(-N // mb))
    lp, V, H = g["step_logp"], g["step_V"], g["step_H"]
    old = np.tile(g["old_logp"], int(g["k_epochs"]))
    assert len(lp) == int(g["k_epochs"]) * N and len(H) == nsteps
    off = 0
    for s in range(nsteps):
        n = min(mb, N - (s % (-(-N // mb))) * mb)
        sl = slice(off, off + n)
        loss, dlogp, dV = O.surrogate(lp[sl], old[sl], g["step_adv"][sl], V[sl], g["step_ret"][sl],
                                      H[s])
        scale = np.abs(g["step_dlogp"][sl]).max() + 1e-30
        np.testing.assert_allclose(dlogp, g["step_dlogp"][sl], rtol=2e-6, atol=1e-7 * scale)
        np.testing.assert_allclose(dV, g["step_dV"][sl], rtol=1e-5, atol=1e-9)
        # the loss the reference back-propagated, rebuilt from its own captured pieces
        ref_loss = np.mean(-g["step_min"][sl].astype(np.float64)) + 0.5 * float(g["step_sl1"][s]) \
            - 0.01 * float(H[s])
        assert loss == pytest.approx(ref_loss, rel=2e-5, abs=1e-6)
        off += n


def test_rnd_oracle_vs_reference(golden):
    g = golden("rnd")
    for D in (4, 348):
        nets = {}
        for name in ("target_net", "pred_net"):
            p = lambda k: g[f"D{D}/{name}.{k}"]  # noqa: E731
            nets[name] = dict(w1=p("0.weight"), b1=p("0.bias"), gw=p("1.weight"), gb=p("1.bias"),
                              w2=p("3.weight"), b2=p("3.bias"))
        r = O.rnd_forward(g[f"D{D}_x"], nets["target_net"], nets["pred_net"], 0.001)
        np.testing.assert_allclose(r, g[f"D{D}_r"], rtol=2e-5, atol=1e-8)


# ---------------------------------------------------------------------------------- worker
class ScriptedOracle:
    """The scripted env of make_golden.py in the oracle's batched-env interface."""

    def __init__(self, L):
        self.E = len(L)
        self.L = np.asarray(L)
        self.t = np.zeros(self.E, np.int64)

    def reset(self):
        self.t[:] = 0
        return np.stack([np.array([e, 0, 0, 0], np.float32) for e in range(self.E)])

    def step_envs(self, idx, actions):
        obs, rew, term, trunc = [], [], [], []
        for i, e in enumerate(idx):
            self.t[e] += 1
            end = self.t[e] >= self.L[e]
            tr = end and e % 5 == 3
            a = float(actions[i])
            obs.append(np.array([e, self.t[e], a, e * 0.5 + self.t[e]], np.float32))
            rew.append(float(e) * 0.25 + self.t[e] * 0.5)
            term.append(end and not tr)
            trunc.append(tr)
        return np.array(obs), np.array(rew), np.array(term), np.array(trunc)


def test_worker_oracle_matches_reference_worker(golden):
    g = golden("worker")
    env = ScriptedOracle(g["L"])

    def act(states, idx, t):
        return ((states[:, 0].astype(np.int64) + states[:, 1].astype(np.int64)) % 2)

    out = O.worker_oracle(env, act)
    np.testing.assert_array_equal(out["masks"], g["masks"])
    for k in ("S", "A", "R", "D"):
        np.testing.assert_array_equal(out[k].reshape(g[k].shape), g[k])
    assert out["step_score"] == int(g["step_score"])
    assert out["reward_score"] == pytest.approx(float(g["reward_score"]))
    np.testing.assert_array_equal(out["lengths"], g["L"])


def test_mask_utils_restatement():
    rng = np.random.default_rng(0)
    for _ in range(50):
        E = int(rng.integers(1, 300))
        m = rng.random(E) < 0.4
        n = int(np.sum(~m))
        d = rng.random(n) < 0.3
        ref = m.copy()
        ref[np.where(~ref)[0]] = d
        np.testing.assert_array_equal(O.update_active_environments_list(m, d), ref)
        np.testing.assert_array_equal(O.indexes_of_active_environments(E, m), np.where(~m)[0])


# ---------------------------------------------------------------------------------- envs
def _run_env_fixture(g, name, oracle_cls):
    seeds = g[f"{name}_seeds"]
    E = len(seeds)
    env = oracle_cls(E)
    env.seed(seeds)
    env.reset()                      # reset(seed=...) draw
    obs0 = env.reset()               # EnvVectorizer.reset(): the second draw
    np.testing.assert_array_equal(obs0, g[f"{name}_obs0"])
    vec = O.EnvVectorizerOracle(env)
    vec.envs_active = np.zeros(E, bool)
    nact = g[f"{name}_nact"]
    off = 0
    max_obs_err = 0.0
    mism_term = 0
    for step, n in enumerate(nact):
        n = int(n)
        if n < 0:
            o = env.reset()
            vec.envs_active[:] = False
            np.testing.assert_array_equal(o, g[f"{name}_obs"][off:off - n])
            off += -n
            continue
        acts = g[f"{name}_act"][off:off + n]
        if name == "cartpole":
            acts = acts[:, 0].astype(np.int64)
        o, r, d, tr = vec.step(acts)
        sl = slice(off, off + n)
        max_obs_err = max(max_obs_err, float(np.max(np.abs(o - g[f"{name}_obs"][sl]))))
        np.testing.assert_allclose(r, g[f"{name}_rew"][sl], rtol=1e-12, atol=1e-12)
        mism_term += int(np.sum(d != g[f"{name}_term"][sl]))
        np.testing.assert_array_equal(tr, g[f"{name}_trunc"][sl])
        vec.envs_active[np.where(~vec.envs_active)[0]] = d | tr
        np.testing.assert_array_equal(vec.envs_active, g[f"{name}_mask"][step])
        off += n
    assert mism_term == 0
    return max_obs_err


def test_cartpole_oracle_vs_gymnasium_restatement(golden):
    err = _run_env_fixture(golden("envs"), "cartpole", O.CartPoleOracle)
    assert err <= 1e-6  # fdlibm vs glibc trig: at most a few float32 ulps on the observation


def test_pendulum_oracle_vs_gymnasium_restatement(golden):
    err = _run_env_fixture(golden("envs"), "pendulum", O.PendulumOracle)
    assert err <= 1e-5


def test_fdlibm_trig_within_one_ulp_of_libm():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-0.25, 0.25, 50000), rng.uniform(-120, 120, 50000)])
    s, c = O.sin_cos(x)
    ms = np.array([math.sin(v) for v in x])
    mc = np.array([math.cos(v) for v in x])
    ulp_s = np.abs(s - ms) / np.spacing(np.abs(ms))
    ulp_c = np.abs(c - mc) / np.spacing(np.abs(mc))
    assert ulp_s.max() <= 1.0 and ulp_c.max() <= 1.0
    # most arguments agree bit for bit
    assert np.mean(s == ms) > 0.95 and np.mean(c == mc) > 0.95  # measured: ~97.9 %


def test_pcg64_seeding_restatement_matches_numpy():
    # the state words the GPU kernel must produce (prl_pcg64_seed), from numpy itself
    for seed in (0, 1, 7, 2**32 + 5, 123456789):
        w = O.pcg64_state_words(seed)
        g = np.random.PCG64(seed)
        st = g.state["state"]
        assert (int(w[0]) << 64 | int(w[1])) == st["state"]
        assert (int(w[2]) << 64 | int(w[3])) == st["inc"]
