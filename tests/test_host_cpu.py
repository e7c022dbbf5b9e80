"""Host-side tests that run without a GPU: the C-ABI library loads and exports every declared
symbol, the drop-in API surface matches the reference (names, state_dict keys, seeded init,
batch_packer / Memory / VecMemory semantics), and learn()'s orchestration reproduces the
reference's own learn() when its HIP entry points are replaced by the CPU oracle (fake_ops)."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT


# ---------------------------------------------------------------------------------- C-ABI
def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "prl_abi.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|uint32_t|void|const char\*)\s+(prl_\w+)\s*\(", hdr, re.M)))


def test_abi_library_exports_every_declared_symbol():
    import prl_native
    L = prl_native.lib()
    syms = _declared_symbols()
    assert len(syms) == len(prl_native.SIGNATURES) == 70
    for s in syms:
        assert hasattr(L, s), s
        assert s in prl_native.SIGNATURES, f"{s} has no ctypes signature"
    assert L.prl_abi_version() == prl_native.ABI_VERSION == 2
    # the library was built from the sources next to it (csrc/build.py stamps them)
    assert L.prl_source_id().decode() == prl_native._sources_id()


def test_abi_host_calls_without_gpu():
    import prl_native
    d = prl_native.env_dims(0)
    assert d == dict(obs_dim=4, act_dim=2, phys_dim=4, max_episode_steps=500, discrete=True)
    assert prl_native.env_dims(1)["max_episode_steps"] == 200
    assert prl_native.env_dims(2)["obs_dim"] == 348
    assert prl_native.workspace_bytes(prl_native.OP_GAE, 1 << 20) > 0
    assert prl_native.workspace_bytes(prl_native.OP_SCAN, 65536) >= 8 * 65536
    assert prl_native.lib().prl_workspace_bytes(99, 10) == -1
    with pytest.raises(RuntimeError, match="unknown env kind"):
        prl_native.env_dims(7)


def test_split_wave_block_lists_cover_the_net():
    """The head-split kernel's wave-block AdamW / publish lists (csrc/prl_ppo_split.h
    spl_wb_quad) partition each role's parameter quads (trunk + its head, padding aside) among
    its four waves, within the moment slots a lane holds: checked on the host for the CartPole
    shape the kernel runs (D 4, A 2, discrete), and refused for a shape it does not."""
    import prl_native
    L = prl_native.lib()
    assert L.prl_ppo_update_wb_check(4, 2, 1) == 1
    assert L.prl_ppo_update_wb_check(64, 8, 1) == 0      # W0 blocks past the 5 slots per lane
    assert L.prl_ppo_update_wb_check(3, 1, 0) == 0       # three heads: not a split-form shape


def test_product_refuses_cpu_tensors():
    import prl_native
    with pytest.raises(ValueError, match="device tensor"):
        x = torch.zeros(4)
        prl_native.gae(x, x, x, None, 0.99, 0.95, x)


# ---------------------------------------------------------------------------------- API surface
def test_reference_api_names():
    import AsyncTools
    import AsyncTools.utils as U
    from AsyncTools.AsyncPPO import AsyncPPO, EnvVectorizer, VecMemory  # noqa: F401
    from PPO import PPO, ActorCritic, RND, Memory  # noqa: F401
    for f in ("indexes_of_active_environments", "number_of_active_environments",
              "range_of_active_environments", "inactive_states_dropout", "buffer_append",
              "update_active_environments_list", "buffer_to_target_buffer_transfer"):
        assert callable(getattr(U, f))
    for m in ("get_action", "batch_packer", "compute_gae", "learn", "save_weights",
              "load_weights"):
        assert callable(getattr(PPO, m))
    assert AsyncTools.envs.make("Pendulum-v1").action_space.shape == (1,)


@pytest.mark.parametrize("tag,cont", [("learn", False), ("learn_cont", True)])
def test_seeded_init_and_state_dict_keys_match_reference(golden, tag, cont):
    from PPO import PPO
    g = golden(tag)
    torch.manual_seed(0)
    D, A = (3, 1) if cont else (4, 2)
    p = PPO(is_continuous=cont, observ_dim=D, action_dim=A, action_scaling=2.0 if cont else None)
    sd = p.policy.state_dict()
    ref_keys = sorted(k[5:] for k in g.files if k.startswith("init/"))
    assert sorted(sd.keys()) == ref_keys
    for k in ref_keys:
        np.testing.assert_array_equal(sd[k].cpu().numpy(), g["init/" + k])


def test_rnd_state_dict_keys(golden):
    from PPO import RND
    g = golden("rnd")
    r = RND(4, 4)
    assert sorted(r.state_dict().keys()) == sorted(k[3:] for k in g.files if k.startswith("D4/"))


def test_batch_packer_matches_dataloader():
    from PPO import PPO
    p = PPO(False, 4, 2)
    x = torch.randn(227, 4)
    got = p.batch_packer(x, 32)
    ref = list(torch.utils.data.DataLoader(x, 32))
    assert len(got) == len(ref) == 8
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    vals = [torch.randn(227, 4), torch.randint(0, 2, (227,)), torch.rand(227)]
    got = p.batch_packer(vals, 50)
    assert len(got) == 3 and all(len(v) == 5 for v in got)
    assert got[1][4].shape == (27,)


def test_memory_semantics():
    from PPO import Memory
    m = Memory()
    for i in range(10):
        m.push(np.random.randn(4), np.random.randint(0, 2, size=()), np.random.rand(), True)
    assert len(m.states) == 10 and m.states[0].dtype == np.float32
    m.push_device(torch.zeros(5, 4), torch.zeros(5), torch.ones(5), torch.zeros(5))
    assert len(m) == 15 and len(m.states) == 15
    S, A, R, Dn = m.device_tensors("cpu")
    assert S.shape == (15, 4) and A.shape == (15,) and float(R[-1]) == 1.0
    m.clear()
    assert len(m) == 0 and len(m.actions) == 0


def test_vecmemory_semantics():
    from AsyncTools.AsyncPPO import VecMemory
    v = VecMemory(4)
    v.push(2, np.random.randn(1), np.random.randint(0, 2, (1,)), np.random.rand(1), True)
    assert len(v.states[2]) == 1 and v.dones[2][0].dtype == np.float32
    v.clear()
    assert all(len(s) == 0 for s in v.states)


def test_buffer_transfer_is_env_major():
    from AsyncTools.AsyncPPO import VecMemory
    from AsyncTools.utils import buffer_to_target_buffer_transfer
    from PPO import Memory
    v = VecMemory(3)
    for e, L in enumerate((2, 0, 3)):
        for t in range(L):
            v.push(e, np.array([e, t]), np.array(0), np.array(1.0), np.array(t == L - 1))
    m = Memory()
    buffer_to_target_buffer_transfer(v, m)
    assert [tuple(s) for s in m.states] == [(0, 0), (0, 1), (2, 0), (2, 1), (2, 2)]
    assert all(len(x) == 0 for x in v.states)


# ---------------------------------------------------------------------------------- learn()
def _ppo_from_fixture(g, cont, fake):
    from PPO import PPO
    torch.manual_seed(0)
    D, A = (3, 1) if cont else (4, 2)
    p = PPO(is_continuous=cont, observ_dim=D, action_dim=A, action_scaling=2.0 if cont else None,
            lr=1e-3, k_epochs=int(g["k_epochs"]), policy_clip=0.2, GAE_lambda=0.95, gamma=0.995,
            batch_size=1024, mini_batch_size=int(g["mb"]))
    p._ops = fake
    p.show_progress = False
    N = int(g["N"])
    for i in range(N):
        a = g["A"][i] if cont else np.asarray(g["A"][i])
        p.memory.push(g["S"][i], a, g["R"][i], g["Dn"][i])
    return p


@pytest.mark.parametrize("tag,cont", [("learn", False), ("learn_cont", True)])
def test_learn_orchestration_matches_reference_learn(golden, tag, cont):
    """Our learn() (oracle-backed ops on CPU) vs the reference's learn() on the same seeded
    policy and memory: every updated policy weight agrees to 1e-6 (measured max 1.8e-7)."""
    from fake_ops import FakeOps
    g = golden(tag)
    fake = FakeOps()
    p = _ppo_from_fixture(g, cont, fake)
    p.learn()
    steps = int(g["k_epochs"]) * -(-int(g["N"]) // int(g["mb"]))
    assert fake.calls["gae"] == 1 and fake.calls["surrogate_fwd"] == steps
    assert fake.calls["surrogate_bwd"] == steps
    assert len(p.memory) == 0
    sd = p.policy.state_dict()
    worst = 0.0
    for k in sd:
        ref = g["final/" + k]
        diff = np.abs(sd[k].cpu().numpy() - ref)
        worst = max(worst, float(diff.max()))
        np.testing.assert_allclose(sd[k].cpu().numpy(), ref, rtol=0, atol=1e-6)
    old = p.policy_old.state_dict()
    for k in sd:
        assert torch.equal(old[k], sd[k])


def test_learn_below_batch_size_is_a_noop():
    from fake_ops import FakeOps
    from PPO import PPO
    p = PPO(False, 4, 2, batch_size=100)
    p._ops = FakeOps()
    for _ in range(50):
        p.memory.push(np.zeros(4), np.array(0), 1.0, False)
    before = {k: v.clone() for k, v in p.policy.state_dict().items()}
    p.learn()
    assert len(p.memory) == 50 and p._ops.calls["gae"] == 0
    for k, v in p.policy.state_dict().items():
        assert torch.equal(v, before[k])


def test_save_load_weights_roundtrip(tmp_path):
    from PPO import PPO
    a = PPO(True, 3, 1, action_scaling=2.0, use_RND=True)
    a.save_weights(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["Policy_weights.pth", "RND_weights.pth"]
    b = PPO(True, 3, 1, action_scaling=2.0, use_RND=True)
    b.load_weights(str(tmp_path))
    for k, v in a.policy.state_dict().items():
        assert torch.equal(v, b.policy.state_dict()[k])
        assert torch.equal(v, b.policy_old.state_dict()[k])
    b.load_weights(str(tmp_path / "missing"))  # FileNotFoundError swallowed (PPO.py:276-277)


def test_kernel_bench_tool_imports():
    """tools/kernel_bench.py (the PMC passes of tools/gpu_benchprof.sh) binds bench.py's
    constants at import: keep the two in step (no GPU needed to import)."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("kernel_bench", os.path.join(root, "tools", "kernel_bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.CARTPOLE_STEP_BYTES == 111 and mod.GAE_BYTES_PER_TRANSITION == 20


def test_bench_traffic_comes_from_recorded_workloads():
    """bench.py's roofline `traffic` fields read committed PMC summaries (profiles/*_pmc.json):
    scaled per unit from the workload the summary records, the update engine's only at the
    minibatch size it was profiled at (None otherwise), and labelled with where it came from."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    per, src = bench.update_pmc_traffic("ppo_update_split_kernel", 1000, 512)
    assert per is not None and 2e9 < per < 5e9 and "per optimizer step at mb 512" in src
    assert bench.update_pmc_traffic("ppo_update_split_kernel", 1000, 65536) == (None, None)
    assert bench.update_pmc_traffic("ppo_update_kernel", 1000, 512) == (None, None)
    env, src = bench.unit_pmc_traffic("*rollout_step_pmc.json", "rollout_step_kernel",
                                      "env_steps_per_dispatch")
    assert 100 < env < 130 and "B per env-step" in src      # 111 B algorithmic
    cpr, _ = bench.unit_pmc_traffic("*cp_rollout_pmc.json", "cp_rollout_kernel", "env_steps_per_dispatch")
    assert 20 < cpr < 111                                   # the one-launch rollout keeps state in registers
    assert bench.unit_pmc_traffic("*no_such_pmc.json", "x", "y") == (None, None)
    wide, _ = bench.wide_pmc_traffic()
    assert 2e8 < wide < 4e8
    gae, _ = bench.pmc_traffic(1 << 20)
    assert 20 * (1 << 20) <= gae < 24 * (1 << 20)           # 20 B per transition algorithmic


@pytest.mark.parametrize("n", [3 * 64, 3 * 64 + 5])
def test_split_k_linear_function_vs_autograd(monkeypatch, n):
    """PPO.layers._SplitKLinear (the large-batch Linear's split-K weight / bias gradient) is plain
    torch code: on CPU tensors with 64-row chunks it gives F.linear's forward and autograd's
    gradients in float64 (chunked sums, with and without a remainder)."""
    from PPO import layers
    monkeypatch.setattr(layers, "SPLIT_ROWS", 64)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(n, 7, dtype=torch.float64, generator=g, requires_grad=True)
    w = torch.randn(5, 7, dtype=torch.float64, generator=g, requires_grad=True)
    b = torch.randn(5, dtype=torch.float64, generator=g, requires_grad=True)
    dy = torch.randn(n, 5, dtype=torch.float64, generator=g)
    y = layers._SplitKLinear.apply(x, w, b)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), dy)
    x2, w2, b2 = (t.detach().clone().requires_grad_() for t in (x, w, b))
    y2 = torch.nn.functional.linear(x2, w2, b2)
    rx, rw, rb = torch.autograd.grad(y2, (x2, w2, b2), dy)
    assert torch.equal(y, y2)
    torch.testing.assert_close(gx, rx, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(gw, rw, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(gb, rb, rtol=1e-12, atol=1e-12)
    # no bias, weight only
    y3 = layers._SplitKLinear.apply(x, w, None)
    (gw3,) = torch.autograd.grad(y3, (w,), dy)
    torch.testing.assert_close(gw3, rw, rtol=1e-12, atol=1e-12)


def test_sample_key_mixes_rank():
    """data-parallel ranks given the same seed must not share the sampling key; rank 0
    keeps the single-process key (so 1-rank results are unchanged)."""
    from AsyncTools.AsyncPPO import sample_key
    k0 = sample_key(123, rank=0)
    assert k0 == sample_key(123)            # no process group: rank 0
    keys = {sample_key(123, rank=r) for r in range(8)}
    assert len(keys) == 8 and all(0 <= k < 2**64 for k in keys)
    assert sample_key(124, rank=0) != k0


@pytest.mark.parametrize("tag", ["learn_rnd", "learn_rnd_c5"])
def test_checkpoint_files_match_reference_format(tmp_path, tag):
    """§8 f3 on the CPU: the reference's save_weights() files (weights_only loads) and ours carry
    the same keys, shapes and dtypes, for the policy and for RND."""
    import os
    from PPO import PPO
    ref_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"ckpt_{tag}")
    cont, D, A = (False, 4, 2) if tag == "learn_rnd" else (True, 348, 17)
    p = PPO(cont, D, A, action_scaling=2.0 if cont else None, use_RND=True)
    p.save_weights(str(tmp_path))
    for name in ("Policy_weights.pth", "RND_weights.pth"):
        ref = torch.load(os.path.join(ref_dir, name), weights_only=True)
        ours = torch.load(os.path.join(str(tmp_path), name), weights_only=True)
        assert list(ref) == list(ours), name
        for k in ref:
            assert ref[k].shape == ours[k].shape and ref[k].dtype == ours[k].dtype, (name, k)
    q = PPO(cont, D, A, action_scaling=2.0 if cont else None, use_RND=True)
    q.load_weights(ref_dir)                 # the reference's files load into ours (CPU)
    ref = torch.load(os.path.join(ref_dir, "Policy_weights.pth"), weights_only=True)
    for k, v in q.policy.state_dict().items():
        assert torch.equal(v.cpu(), ref[k])
