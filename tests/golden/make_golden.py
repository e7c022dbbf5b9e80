"""Generate the golden fixtures in tests/golden/*.npz by IMPORTING THE REFERENCE.

Run in the development container only (the reference is not on the GPU box):
    python tests/golden/make_golden.py [--ref /root/reference]

The reference (Raven4567/Parallel-Reinforcement-Learning) is pure Python.  Its `PPO` package
imports as-is.  `AsyncTools.AsyncPPO` imports `gymnasium` (requirements.txt:4), which is not
installed and cannot be fetched; EnvVectorizer only subclasses `gym.Env` (AsyncPPO.py:35), so a
module object carrying a bare `Env` class is put in sys.modules, and the envs behind the
vectorizer are gym_restated.py (numpy restatement of gymnasium 1.1.1) or a scripted env.

Fixtures (every array is produced by the reference's own code paths, instrumented, never
re-implemented here):
  gae.npz      PPO.compute_gae (PPO/PPO.py:107-120) on seeded inputs, N in {1024, 16384, ...}
  learn.npz    one PPO.learn() (PPO.py:122-260): old log-probs / values, GAE returns, normalised
               advantages, per-minibatch surrogate inputs, the loss pieces and d loss/d logp,
               d loss/d V captured by autograd hooks, initial + final policy state_dict
  rnd.npz      RND.compute_intrinsic_reward (PPO/RND.py:71-94) for D in {4, 348}
  learn_rnd.npz, learn_rnd_c5.npz
               PPO.learn() with use_RND=True (PPO.py:157-178): the above plus the intrinsic
               rewards, the RND state before and after update_pred; ckpt_<tag>/ holds the
               reference's own save_weights() files (Policy_weights.pth, RND_weights.pth)
  worker.npz   AsyncPPO.worker (AsyncTools/AsyncPPO.py:117-146) over a scripted env: per-step
               envs_active masks, env-major memory, scores
  envs.npz     EnvVectorizer.reset/step (AsyncPPO.py:48-102) over gym_restated CartPole/Pendulum
"""
import argparse
import copy
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gym_restated  # noqa: E402
from learn_inputs import digest, learn_inputs  # noqa: E402


def import_reference(ref):
    sys.path.insert(0, ref)
    gym = types.ModuleType("gymnasium")

    class Env:  # AsyncPPO.py:35 subclasses gym.Env and calls super().__init__() / close()
        def __init__(self, *a, **k):
            pass

        def close(self):
            pass

    gym.Env = Env
    sys.modules["gymnasium"] = gym
    import torch
    import PPO as ppo_pkg
    import AsyncTools
    import AsyncTools.AsyncPPO as apo
    import AsyncTools.utils as utils
    return torch, ppo_pkg, AsyncTools, apo, utils


def sd_to_np(sd):
    return {k: v.detach().cpu().numpy().copy() for k, v in sd.items()}


# ------------------------------------------------------------------------------------ GAE
def make_gae(ppo_pkg):
    out = {}
    rng = np.random.default_rng(20250725)
    cases = {
        "a": dict(N=1024, gamma=0.995, lam=0.95, pd=0.05, endone=True, rew="ones"),
        "b": dict(N=16384, gamma=0.995, lam=0.95, pd=0.05, endone=True, rew="normal"),
        "c": dict(N=1000, gamma=0.99, lam=0.9, pd=0.1, endone=False, rew="normal", nv=0.37),
        "d": dict(N=4000, gamma=0.995, lam=0.95, pd=None, endone=True, rew="pendulum"),
        "e": dict(N=3000, gamma=0.995, lam=0.95, pd=0.0, endone=False, rew="normal", nv=-1.25),
    }
    for k, c in cases.items():
        N = c["N"]
        if c["pd"] is None:
            d = np.zeros(N, np.float32)
            d[199::200] = 1.0
        else:
            d = (rng.random(N) < c["pd"]).astype(np.float32)
        if c["endone"]:
            d[-1] = 1.0
        if c["rew"] == "ones":
            r = np.ones(N, np.float32)
        elif c["rew"] == "pendulum":
            r = (-np.abs(rng.normal(5, 3, N))).astype(np.float32)
        else:
            r = rng.normal(1.0, 0.5, N).astype(np.float32)
        V = (rng.normal(0, 1, N) * 5).astype(np.float32)
        nv = np.float32(c["nv"]) if "nv" in c else V[-1]
        ppo = ppo_pkg.PPO(is_continuous=False, observ_dim=4, action_dim=2, gamma=c["gamma"],
                          GAE_lambda=c["lam"])
        ret = np.array(ppo.compute_gae(r, d, V, nv), dtype=np.float32)
        assert ret.dtype == np.float32
        out.update({f"{k}_r": r, f"{k}_d": d, f"{k}_V": V, f"{k}_nv": np.float32(nv),
                    f"{k}_gamma": c["gamma"], f"{k}_lam": c["lam"], f"{k}_ret": ret})
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **out)


# ------------------------------------------------------------------------------------ learn
class _TorchProxy:
    """Stands in for the reference module's `torch as t` to observe the surrogate's tensors."""

    def __init__(self, torch, rec):
        self._t = torch
        self._rec = rec

    def __getattr__(self, name):
        return getattr(self._t, name)

    def clamp(self, *a, **k):
        out = self._t.clamp(*a, **k)
        if k.get("min") == -20:
            self._rec["diff"].append(k["input"].detach().clone())
        return out

    def exp(self, x):
        out = self._t.exp(x)
        self._rec["ratio"].append(out.detach().clone())
        return out

    def mul(self, a, b):
        if len(self._rec["adv_mb"]) < len(self._rec["ratio"]):
            self._rec["adv_mb"].append(b.detach().clone())
        return self._t.mul(a, b)

    def min(self, a, b):
        out = self._t.min(a, b)
        self._rec["min"].append(out.detach().clone())
        return out

    def sub(self, a, b):
        out = self._t.sub(a, b)
        self._rec["adv_raw"].append(out.detach().clone())
        return out


def make_learn(torch, ppo_pkg, continuous=False, tag="learn", N=1500, mb=512, k_epochs=2,
               use_rnd=False, D=None, A=None, ckpt=False, store_inputs=True, light=False):
    ppo_mod = sys.modules["PPO.PPO"]  # the package re-exports the class under the same name
    torch.manual_seed(0)
    if D is None:
        D, A = (3, 1) if continuous else (4, 2)
    ppo = ppo_pkg.PPO(is_continuous=continuous, observ_dim=D, action_dim=A,
                      action_scaling=2.0 if continuous else None, lr=1e-3, k_epochs=k_epochs,
                      policy_clip=0.2, GAE_lambda=0.95, gamma=0.995, batch_size=min(1024, N),
                      mini_batch_size=mb, use_RND=use_rnd, beta=0.001)
    rnd_rec = {}
    if use_rnd:   # PPO.learn's RND section (PPO.py:157-178): reward, then update_pred
        rnd_rec["init"] = sd_to_np(ppo.rnd.state_dict())
        orig_cir, orig_up = ppo.rnd.compute_intrinsic_reward, ppo.rnd.update_pred

        def cir(values):
            out = orig_cir(values)
            rnd_rec["r_int"] = out.detach().cpu().numpy().copy()
            return out

        def up(values):
            out = orig_up(values)
            rnd_rec["after_update"] = sd_to_np(ppo.rnd.state_dict())
            return out

        ppo.rnd.compute_intrinsic_reward, ppo.rnd.update_pred = cir, up
    S, Aa, R, Dn = learn_inputs(N, D, A, continuous)
    for i in range(N):
        ppo.memory.push(S[i], np.asarray(Aa[i]), np.float64(R[i]), np.asarray(Dn[i]))
    init_sd = sd_to_np(ppo.policy.state_dict())

    rec = {k: [] for k in ["diff", "ratio", "adv_mb", "min", "adv_raw", "old_logp", "old_V",
                           "logp", "V", "H", "dlogp", "dV", "sl1_in_V", "sl1_in_R", "sl1",
                           "gae_ret"]}
    orig_eval_old = ppo.policy_old.get_evaluate

    def eval_old(s, a):
        lp, v, h = orig_eval_old(s, a)
        rec["old_logp"].append(lp.detach().clone())
        rec["old_V"].append(v.detach().clone())
        return lp, v, h

    ppo.policy_old.get_evaluate = eval_old
    orig_eval = ppo.policy.get_evaluate

    def eval_new(s, a):
        lp, v, h = orig_eval(s, a)
        rec["logp"].append(lp.detach().clone())
        rec["V"].append(v.detach().clone())
        rec["H"].append(h.detach().clone())
        lp.register_hook(lambda g: rec["dlogp"].append(g.detach().clone()))
        v.register_hook(lambda g: rec["dV"].append(g.detach().clone()))
        return lp, v, h

    ppo.policy.get_evaluate = eval_new
    orig_loss = ppo.loss_fn

    def loss_fn(v, r):
        out = orig_loss(v, r)
        rec["sl1_in_V"].append(v.detach().clone())
        rec["sl1_in_R"].append(r.detach().clone())
        rec["sl1"].append(out.detach().clone())
        return out

    ppo.loss_fn = loss_fn
    orig_gae = ppo.compute_gae

    def gae(*a):
        out = orig_gae(*a)
        rec["gae_ret"].append(np.array(out, np.float32))
        return out

    ppo.compute_gae = gae
    real_t = ppo_mod.t
    ppo_mod.t = _TorchProxy(torch, rec)
    try:
        ppo.learn()
    finally:
        ppo_mod.t = real_t
    final_sd = sd_to_np(ppo.policy.state_dict())

    cat = lambda L: torch.cat(L).numpy()  # noqa: E731
    out = {"S": S, "A": Aa.astype(np.float32)} if store_inputs else {
        "inputs_sha256": digest(S, Aa.astype(np.float32))}   # regenerate: learn_inputs.py
    out.update({
        "R": R, "Dn": Dn.astype(np.float32), "D": D, "A_dim": A, "continuous": int(continuous),
        "mb": mb, "k_epochs": k_epochs, "N": N,
        "old_logp": cat(rec["old_logp"]), "old_V": cat(rec["old_V"]),
        "returns": rec["gae_ret"][0], "adv_raw": rec["adv_raw"][0].numpy(),
        "adv": cat(rec["adv_mb"][: -(-N // mb)]),
    })
    if not light:   # per optimizer step (k_epochs * ceil(N/mb) of them), concatenated
        out.update({
        "step_logp": cat(rec["logp"]), "step_V": cat(rec["V"]),
        "step_H": torch.stack(rec["H"]).numpy(), "step_diff": cat(rec["diff"]),
        "step_ratio": cat(rec["ratio"]), "step_min": cat(rec["min"]),
        "step_sl1": torch.stack(rec["sl1"]).numpy(), "step_dlogp": cat(rec["dlogp"]),
        "step_dV": cat(rec["dV"]), "step_ret": cat(rec["sl1_in_R"]),
        "step_adv": cat(rec["adv_mb"]),
        })
    for k, v in init_sd.items():
        out["init/" + k] = v
    for k, v in final_sd.items():
        out["final/" + k] = v
    if use_rnd:
        out["use_rnd"] = 1
        out["r_int"] = rnd_rec["r_int"]
        for k, v in rnd_rec["init"].items():
            out["rnd_init/" + k] = v
        for k, v in rnd_rec["after_update"].items():
            out["rnd_final/" + k] = v
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    if ckpt:   # the reference's own checkpoint files (PPO.save_weights, PPO.py:279-283)
        d = os.path.join(HERE, f"ckpt_{tag}")
        os.makedirs(d, exist_ok=True)
        ppo.save_weights(d)


# ------------------------------------------------------------------------------------ RND
def make_rnd(torch, ppo_pkg):
    out = {}
    for D, seed in ((4, 1), (348, 2)):
        torch.manual_seed(seed)
        rnd = ppo_pkg.RND(in_features=D, out_features=D, beta=0.001)
        x = torch.randn(300, D)
        r = rnd.compute_intrinsic_reward(list(torch.utils.data.DataLoader(x, 64)))
        out[f"D{D}_x"] = x.numpy()
        out[f"D{D}_r"] = r.numpy()
        for k, v in sd_to_np(rnd.state_dict()).items():
            out[f"D{D}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "rnd.npz"), **out)


# ------------------------------------------------------------------------------------ worker
class ScriptedEnv:
    """Deterministic env for the worker fixture.  The k-th reset() call gets id k (EnvVectorizer
    resets its deep copies in index order, AsyncPPO.py:52-53); its episode lasts L[id] steps and
    ends by termination, or by truncation when id % 5 == 3."""
    L = None
    counter = [0]

    def __init__(self):
        self.observation_space = gym_restated._Space(shape=(4,))
        self.action_space = gym_restated._Space(n=2)
        self.id = -1
        self.t = 0

    def reset(self):
        self.id = ScriptedEnv.counter[0]
        ScriptedEnv.counter[0] += 1
        self.t = 0
        return np.array([self.id, 0, 0, 0], np.float32), {}

    def step(self, action):
        self.t += 1
        end = self.t >= ScriptedEnv.L[self.id]
        trunc = end and self.id % 5 == 3
        obs = np.array([self.id, self.t, float(action), self.id * 0.5 + self.t], np.float32)
        return obs, float(self.id) * 0.25 + self.t * 0.5, end and not trunc, trunc, {}

    def close(self):
        pass


class ScriptedPPO:
    def __init__(self, ppo_pkg):
        self.memory = ppo_pkg.Memory()

    def get_action(self, states):
        s = states.numpy()
        return ((s[:, 0].astype(np.int64) + s[:, 1].astype(np.int64)) % 2).astype(np.int64)

    def learn(self):
        pass


def make_worker(apo, utils, ppo_pkg):
    E = 37
    rng = np.random.default_rng(11)
    ScriptedEnv.L = rng.integers(1, 40, E)
    ScriptedEnv.counter[0] = 0
    masks = []
    orig = utils.update_active_environments_list

    def rec_update(m, d):
        out = orig(m, d)
        masks.append(out.copy())
        return out

    utils.update_active_environments_list = rec_update
    try:
        ppo = ScriptedPPO(ppo_pkg)
        a = apo.AsyncPPO(env=ScriptedEnv(), ppo=ppo, num_envs=E, steps=10)
        a.step_score = 0
        a.reward_score = 0
        a.worker()
    finally:
        utils.update_active_environments_list = orig
    m = ppo.memory
    np.savez_compressed(
        os.path.join(HERE, "worker.npz"), L=ScriptedEnv.L, masks=np.array(masks),
        S=np.array(m.states, np.float32), A=np.array(m.actions, np.float32),
        R=np.array(m.rewards, np.float32), D=np.array(m.dones, np.float32),
        step_score=np.int64(a.step_score), reward_score=np.float64(a.reward_score))


# ------------------------------------------------------------------------------------ envs
def make_envs(apo):
    out = {}
    rng = np.random.default_rng(3)
    for name, ctor, E, steps in (("cartpole", gym_restated.CartPoleEnv, 24, 700),
                                 ("pendulum", gym_restated.PendulumEnv, 8, 450)):
        vec = apo.EnvVectorizer(ctor(), E)
        seeds = np.arange(E) + 1000
        for i in range(E):  # seed each deep copy as gymnasium's reset(seed=...) would
            vec.envs[i].reset(seed=int(seeds[i]))
        obs0, _ = vec.reset()  # second draw from each env's generator
        recs = {k: [] for k in ("obs", "rew", "term", "trunc", "mask", "act", "nact")}
        for t in range(steps):
            n = int(np.sum(~vec.envs_active))
            if n == 0:
                # every env finished: reset everything (next episode draws continue the RNG)
                obs_r, _ = vec.reset()
                recs["obs"].append(obs_r)
                recs["rew"].append(np.zeros(E))
                recs["term"].append(np.zeros(E, bool))
                recs["trunc"].append(np.zeros(E, bool))
                recs["act"].append(np.zeros((E, 1), np.float32))
                recs["nact"].append(-E)  # marks a reset row
                recs["mask"].append(vec.envs_active.copy())
                continue
            if name == "cartpole":
                acts = (rng.random(n) < 0.5).astype(np.int64)
            else:
                acts = rng.uniform(-2.5, 2.5, (n, 1)).astype(np.float32)
            o, r, d, tr, _ = vec.step(acts)
            done = d | tr
            vec.envs_active[np.where(~vec.envs_active)[0]] = done
            recs["obs"].append(o)
            recs["rew"].append(np.asarray(r, np.float64))
            recs["term"].append(np.asarray(d, bool))
            recs["trunc"].append(np.asarray(tr, bool))
            recs["act"].append(np.asarray(acts, np.float32).reshape(n, -1))
            recs["nact"].append(n)
            recs["mask"].append(vec.envs_active.copy())
        out[f"{name}_seeds"] = seeds
        out[f"{name}_obs0"] = obs0
        out[f"{name}_nact"] = np.array(recs["nact"])
        out[f"{name}_mask"] = np.array(recs["mask"])
        for k in ("obs", "rew", "term", "trunc", "act"):
            out[f"{name}_{k}"] = np.concatenate(recs[k], axis=0)
    np.savez_compressed(os.path.join(HERE, "envs.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated fixture names to (re)generate")
    args = ap.parse_args()
    torch, ppo_pkg, _, apo, utils = import_reference(args.ref)
    torch.set_num_threads(4)
    jobs = {
        "gae": lambda: make_gae(ppo_pkg),
        "learn": lambda: make_learn(torch, ppo_pkg, continuous=False, tag="learn"),
        "learn_cont": lambda: make_learn(torch, ppo_pkg, continuous=True, tag="learn_cont",
                                         N=1200, mb=256, k_epochs=1),
        # learn(use_RND=True): CartPole shapes (mb not dividing N), and C5's shapes (D 348,
        # A 17, continuous) at a CPU-sized N; both also write the reference's save_weights()
        "learn_rnd": lambda: make_learn(torch, ppo_pkg, continuous=False, tag="learn_rnd",
                                        N=1100, mb=256, k_epochs=2, use_rnd=True, ckpt=True),
        "learn_rnd_c5": lambda: make_learn(torch, ppo_pkg, continuous=True, tag="learn_rnd_c5",
                                           N=700, mb=256, k_epochs=1, use_rnd=True, D=348,
                                           A=17, ckpt=True),
        # mini_batch >= layers.SPLIT_MIN_ROWS: the split-K weight gradients and the colsum bias
        # gradients of the policy and of update_pred, end to end (inputs not stored: 28 MB)
        "learn_rnd_big": lambda: make_learn(torch, ppo_pkg, continuous=True, tag="learn_rnd_big",
                                            N=20000, mb=16384, k_epochs=1, use_rnd=True, D=348,
                                            A=17, store_inputs=False),
        # C5's own mini_batch (65,536 rows, the bench's) with a ragged second minibatch and two
        # epochs: the wide step at full size against the reference's post-learn() weights
        # (inputs regenerated by learn_inputs.py; per-step arrays not stored)
        "learn_rnd_c5mb": lambda: make_learn(torch, ppo_pkg, continuous=True,
                                             tag="learn_rnd_c5mb", N=65536 + 3000, mb=65536,
                                             k_epochs=2, use_rnd=True, D=348, A=17,
                                             store_inputs=False, light=True),
        # the large-minibatch update C2's second row and C3 run (mini_batch 65,536: the engine's
        # throughput form, 256 workgroups x 16 tiles): two full minibatches and a ragged third,
        # two epochs, CartPole and Pendulum (inputs regenerated by learn_inputs.py)
        "learn_mb65536": lambda: make_learn(torch, ppo_pkg, continuous=False, tag="learn_mb65536",
                                            N=2 * 65536 + 9000, mb=65536, k_epochs=2,
                                            store_inputs=False, light=True),
        "learn_cont_mb65536": lambda: make_learn(torch, ppo_pkg, continuous=True,
                                                 tag="learn_cont_mb65536", N=2 * 65536 + 9000,
                                                 mb=65536, k_epochs=2, store_inputs=False,
                                                 light=True),
        # C1 at its own hyper-parameters (README.md:35-49: batch 1,024, mini_batch 512,
        # k_epochs 11): a CartPole memory of N = 1,500 (two full minibatches and a ragged third),
        # 33 optimizer steps through the latency form of the engine
        "learn_c1": lambda: make_learn(torch, ppo_pkg, continuous=False, tag="learn_c1", N=1500,
                                       mb=512, k_epochs=11, light=True),
        "rnd": lambda: make_rnd(torch, ppo_pkg),
        "worker": lambda: make_worker(apo, utils, ppo_pkg),
        "envs": lambda: make_envs(apo),
    }
    only = [x for x in args.only.split(",") if x]
    for name, job in jobs.items():
        if not only or name in only:
            job()
    import torch as _t
    with open(os.path.join(HERE, "VERSIONS.txt"), "w") as f:
        f.write(f"numpy {np.__version__}\ntorch {_t.__version__}\n"
                f"python {sys.version.split()[0]}\nreference {args.ref} @ 2025-07-25\n")
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
