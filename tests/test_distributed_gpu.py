"""Data-parallel learn() on the GPU: two ranks sharing cuda:0 (gloo for the host exchange), real
HIP kernels and the graph-captured optimizer step (PPO/update.py, world > 1: two graphs with the
gradient all-reduce issued eagerly between them).

Checked: both ranks end bit-identical; the result equals ONE process learning (also graphed) on
the interleaved union with minibatch 2*mb, to atol 2e-5 (the gradient is summed in a different
order: per-rank partial sums then the all-reduce); the graphs were actually replayed.
On 8 GPUs the same code runs with RCCL (backend "nccl") and device tensors.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_distributed_cpu import PATHS, _shard

pytestmark = pytest.mark.gpu


def _make_ppo(mb, k):
    from PPO import PPO
    torch.manual_seed(0)
    p = PPO(False, 4, 2, lr=1e-3, k_epochs=k, batch_size=1, mini_batch_size=mb)
    p.show_progress = False
    return p


def _worker(rank, world, port, mb, nb, k, out_dir, fused):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PRL_DP_PERSISTENT="0")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        torch.manual_seed(1234 + rank)
        p = _make_ppo(mb, k)
        p.use_fused = fused
        S, A, R, D = _shard(rank, mb, nb)
        p.memory.push_device(*(torch.from_numpy(x).cuda() for x in (S, A, R, D)))
        p.learn()
        torch.cuda.synchronize()
        sd = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **sd,
                 _replays=np.int64(p.last_graph_replays),
                 _path=np.array(p.last_update_path))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("fused", [True, False])
def test_two_ranks_graphed_equal_one_process_on_the_union(tmp_path, fused):
    """fused: the stepped engine (grad kernel -> all-reduce -> AdamW kernel per step) on both
    ranks vs one process running the persistent engine on the union (function space, since the
    gradient sums differ in order); graph: per-step graphs on both sides (weights, 2e-5)."""
    mb, nb, k = 64, 5, 4
    mp.spawn(_worker, args=(2, 29547 + int(fused), mb, nb, k, str(tmp_path), fused), nprocs=2,
             join=True)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    assert str(outs[0]["_path"]) == ("fused-dp" if fused else "graph")
    if not fused:
        assert int(outs[0]["_replays"]) == k * nb - 2       # all but the 2 warm-up steps
    shards = [_shard(r, mb, nb) for r in range(2)]
    cols = [np.concatenate([shards[r][c][j * mb:(j + 1) * mb] for j in range(nb) for r in range(2)])
            for c in range(4)]
    torch.manual_seed(1234)
    p = _make_ppo(2 * mb, k)
    p.use_fused = fused
    p.memory.push_device(*(torch.from_numpy(x).cuda() for x in cols))
    p.learn()
    ref = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
    for key in ref:
        if not key.startswith("_"):
            np.testing.assert_array_equal(outs[0][key], outs[1][key])
    if fused:
        import copy
        import types
        q = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
        q.policy.load_state_dict({kk: torch.from_numpy(outs[0][kk]) for kk in ref})
        S = torch.from_numpy(np.concatenate([cols[0][:256]])).cuda()
        A = torch.from_numpy(np.concatenate([cols[1][:256]])).cuda()
        from test_engine_gpu import _outputs
        (l1, v1), (l2, v2) = _outputs(q, S, A), _outputs(p, S, A)
        assert float((l1 - l2).abs().max()) <= 1e-4 and float((v1 - v2).abs().max()) <= 1e-4
        return
    assert p.last_graph_replays == k * nb - 2
    for key in ref:
        np.testing.assert_allclose(outs[0][key], ref[key], rtol=0, atol=2e-5, err_msg=key)


def _dpx_worker(rank, world, port, mb, nb, k, out_dir, xbuf="auto", push=False):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PRL_DP_PERSISTENT="1",
                      PRL_DP_XBUF=xbuf, PRL_DP_PUSH="1" if push else "0")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        p = _make_ppo(mb, k)
        S, A, R, D = _shard(rank, mb, nb)
        if rank == 1:   # unequal shards: rank 1 has one minibatch less (zero rows in the last)
            S, A, R, D = (x[:-mb] for x in (S, A, R, D))
        p.memory.push_device(*(torch.from_numpy(x).cuda() for x in (S, A, R, D)))
        p.learn()
        p.learn()       # a second launch on the same slice buffers (flags carry global steps)
        torch.cuda.synchronize()
        sd = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
        import prl_native
        tag = ('' if xbuf == 'auto' else xbuf) + ('push' if push else '')
        np.savez(os.path.join(out_dir, f"{tag}rank{rank}.npz"), **sd,
                 _path=np.array(p.last_update_path), _loss=np.float32(p.last_loss.item()),
                 _kinds=np.array(p._engine.dp_xbuf_kinds), _push=np.int32(p._engine._dp_push),
                 _split=np.int32(prl_native.ppo_update_last_plan()["split"]))
        p._engine.close()
    finally:
        torch.distributed.destroy_process_group()


def _stepped_worker(rank, world, port, mb, nb, k, out_dir):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PRL_DP_PERSISTENT="0")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        p = _make_ppo(mb, k)
        S, A, R, D = _shard(rank, mb, nb)
        if rank == 1:
            S, A, R, D = (x[:-mb] for x in (S, A, R, D))
        p.memory.push_device(*(torch.from_numpy(x).cuda() for x in (S, A, R, D)))
        p.learn()
        p.learn()
        torch.cuda.synchronize()
        sd = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
        np.savez(os.path.join(out_dir, f"stepped{rank}.npz"), **sd,
                 _path=np.array(p.last_update_path))
    finally:
        torch.distributed.destroy_process_group()


def test_two_ranks_persistent_dp_engine(tmp_path):
    """prl_ppo_update_dpx on 2 ranks sharing cuda:0 (opt-in PRL_DP_PERSISTENT=1): one persistent
    launch per rank per learn(), the per-step gradient summed across the ranks INSIDE the
    kernels over IPC-mapped slice buffers.  Unequal shards, two learn() calls.  Both ranks end
    bit-identical, and equal the stepped data-parallel loop (grad kernel -> all-reduce -> AdamW
    per step) in function space: the two sum the gradient norm in different orders
    (test_stepped_engine_matches_persistent), so bits are not expected to match."""
    import random
    mb, nb, k = 64, 5, 3
    port = 29960 + random.randint(0, 30)
    mp.spawn(_dpx_worker, args=(2, port, mb, nb, k, str(tmp_path)), nprocs=2, join=True)
    mp.spawn(_stepped_worker, args=(2, port + 40, mb, nb, k, str(tmp_path)), nprocs=2, join=True)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    ref = np.load(os.path.join(tmp_path, "stepped0.npz"))
    assert str(outs[0]["_path"]) == "fused-dp-persistent"
    assert str(ref["_path"]) == "fused-dp"
    keys = [kk for kk in outs[0].files if not kk.startswith("_")]
    for key in keys:
        np.testing.assert_array_equal(outs[0][key], outs[1][key], err_msg=key)
    assert np.isfinite(outs[0]["_loss"])
    import copy
    import types
    p = _make_ppo(mb, k)
    q1 = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
    q2 = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
    q1.policy.load_state_dict({kk: torch.from_numpy(outs[0][kk]) for kk in keys})
    q2.policy.load_state_dict({kk: torch.from_numpy(ref[kk]) for kk in keys})
    S, A, _, _ = _shard(0, mb, nb)
    from test_engine_gpu import _outputs
    (l1, v1), (l2, v2) = (_outputs(q, torch.from_numpy(S[:256]).cuda(),
                                   torch.from_numpy(A[:256]).cuda()) for q in (q1, q2))
    assert float((l1 - l2).abs().max()) <= 1e-4 and float((v1 - v2).abs().max()) <= 1e-4


def test_two_ranks_persistent_dp_engine_fine_grained_buffers(tmp_path):
    """The data-parallel persistent launch on prl_dp_xbuf_alloc's FALLBACK memory (fine-grained,
    forced with PRL_DP_XBUF=fine): the flag store then follows a system-scope release and the
    slice loads a system-scope acquire (args.dp_fine).  Same 2-rank workload as above; the
    fences change no arithmetic, so both ranks end with exactly the bits of the default
    (uncached) buffers."""
    import random
    mb, nb, k = 64, 5, 3
    port = 29700 + random.randint(0, 30)
    mp.spawn(_dpx_worker, args=(2, port, mb, nb, k, str(tmp_path), "auto"), nprocs=2, join=True)
    mp.spawn(_dpx_worker, args=(2, port + 40, mb, nb, k, str(tmp_path), "fine"), nprocs=2,
             join=True)
    auto = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    fine = [np.load(os.path.join(tmp_path, f"finerank{r}.npz")) for r in range(2)]
    assert [str(x) for x in fine[0]["_kinds"]] == ["fine", "fine"]
    assert [str(x) for x in auto[0]["_kinds"]] == ["uncached", "uncached"]
    assert str(fine[0]["_path"]) == "fused-dp-persistent"
    for key in auto[0].files:
        if key.startswith("_"):
            continue
        for r in range(2):
            np.testing.assert_array_equal(fine[r][key], auto[0][key], err_msg=key)
    assert float(fine[0]["_loss"]) == float(auto[0]["_loss"])


@pytest.mark.parametrize("xbuf", ["auto", "fine"])
def test_two_ranks_persistent_dp_engine_push_form(tmp_path, xbuf):
    """The PUSH form of the cross-rank exchange (PRL_DP_PUSH=1, the head-split kernel): each
    workgroup writes its reduced slice into EVERY rank's receive slot and raises its flag there,
    then polls only its own buffer — against the pull form on the same 2-rank
    workload (unequal shards, two learn() calls): the same rank-order float32 sums, so both ranks
    end with exactly the pull form's bits, on uncached and on fine-grained buffers."""
    import random
    mb, nb, k = 64, 5, 3
    port = 29800 + random.randint(0, 30)
    mp.spawn(_dpx_worker, args=(2, port, mb, nb, k, str(tmp_path), xbuf, False), nprocs=2, join=True)
    mp.spawn(_dpx_worker, args=(2, port + 40, mb, nb, k, str(tmp_path), xbuf, True), nprocs=2,
             join=True)
    tag = '' if xbuf == 'auto' else xbuf
    pull = [np.load(os.path.join(tmp_path, f"{tag}rank{r}.npz")) for r in range(2)]
    push = [np.load(os.path.join(tmp_path, f"{tag}pushrank{r}.npz")) for r in range(2)]
    assert int(push[0]["_push"]) == 1 and int(pull[0]["_push"]) == 0
    assert int(push[0]["_split"]) == 1 and str(push[0]["_path"]) == "fused-dp-persistent"
    for key in pull[0].files:
        if key.startswith("_"):
            continue
        for r in range(2):
            np.testing.assert_array_equal(push[r][key], pull[0][key], err_msg=key)
    assert float(push[0]["_loss"]) == float(pull[0]["_loss"])


def test_four_ranks_persistent_dp_engine_push_equals_pull(tmp_path):
    """4 data-parallel ranks sharing cuda:0 (4 x 8 split workgroups at mb 64), unequal shards
    (rank 1 one minibatch short), two learn() calls: the push form (the default) gives exactly
    the pull form's bits, and all four ranks end bit-identical — the exchange's rank-order sums
    at more than two ranks, as the 8-rank node runs them."""
    import random
    mb, nb, k, world = 64, 5, 3, 4
    port = 29600 + random.randint(0, 30)
    mp.spawn(_dpx_worker, args=(world, port, mb, nb, k, str(tmp_path), "auto", False), nprocs=world,
             join=True)
    mp.spawn(_dpx_worker, args=(world, port + 40, mb, nb, k, str(tmp_path), "auto", True),
             nprocs=world, join=True)
    pull = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    push = [np.load(os.path.join(tmp_path, f"pushrank{r}.npz")) for r in range(world)]
    assert int(push[0]["_push"]) == 1 and int(pull[0]["_push"]) == 0
    assert int(push[0]["_split"]) == 1 and str(push[0]["_path"]) == "fused-dp-persistent"
    for key in pull[0].files:
        if key.startswith("_"):
            continue
        for r in range(world):
            np.testing.assert_array_equal(pull[r][key], pull[0][key], err_msg=key)
            np.testing.assert_array_equal(push[r][key], pull[0][key], err_msg=key)
    assert float(push[0]["_loss"]) == float(pull[0]["_loss"])


def _nccl_one_rank_worker(port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PRL_DP_NATIVE="1")
    sys.path[:0] = PATHS
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1,
                                         device_id=torch.device("cuda", 0))
    p = _make_ppo(512, 2)
    eng = p._fused_engine()
    comm = eng.dp_comm()
    ok = bool(comm)
    eng.close()
    ok = ok and not eng._comm and eng.dp_comm() is None
    # rollouts with the nccl process group (and its watchdog thread) alive: the vector-step
    # graph is captured and replayed (thread-local capture mode; the per-step path, not the
    # one-launch CartPole rollout)
    os.environ["PRL_CP_ROLLOUT"] = "0"
    from AsyncTools.AsyncPPO import AsyncPPO
    a = AsyncPPO("CartPole-v1", p, num_envs=4096, seed=1)
    for _ in range(3):
        a.worker()
    torch.cuda.synchronize()
    ok = ok and a._graph is not None and not getattr(a, "_graph_failed", False)
    torch.distributed.destroy_process_group()
    with open(os.path.join(out_dir, "ok"), "w") as f:
        f.write("1" if ok else "0")


def test_engine_rccl_communicator_build_and_close(tmp_path):
    """On the nccl backend the engine builds its own RCCL communicator (one rank here) and
    close() destroys it before destroy_process_group (bench.py's teardown order); device-worker
    rollouts capture and replay their vector-step graph with the process group alive."""
    import random
    port = 29700 + random.randint(0, 200)
    ctx = mp.get_context("spawn")
    proc = ctx.Process(target=_nccl_one_rank_worker, args=(port, str(tmp_path)))
    proc.start()
    proc.join(90)
    if proc.is_alive():
        proc.kill()
        pytest.fail("one-rank nccl worker hung")
    assert proc.exitcode == 0
    assert (tmp_path / "ok").read_text() == "1"


def _config_worker(rank, world, port, cfg, out_dir):
    """One rank of a BASELINE config's per-GPU shape: a device rollout of cfg['E'] envs (rank-
    offset env seeds, rank-mixed sampling key), then learn() as data-parallel rank."""
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from AsyncTools.AsyncPPO import AsyncPPO
        from PPO import PPO
        torch.manual_seed(0)                      # same initial weights on every rank
        p = PPO(cfg["cont"], cfg["D"], cfg["A"], action_scaling=1.0 if cfg["cont"] else None,
                lr=1e-3, k_epochs=cfg["k"], batch_size=1, mini_batch_size=cfg["mb"],
                use_RND=cfg["rnd"])
        p.show_progress = False
        a = AsyncPPO(cfg["env"], p, num_envs=cfg["E"], seed=7)   # same seed: rank offsets apply
        a.worker()
        S = p.memory.device_tensors("cuda")[0]
        n = S.shape[0]
        head = S[:64].cpu().numpy()
        p.learn()
        torch.cuda.synchronize()
        sd = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
        if cfg["rnd"]:
            sd.update({"rnd." + kk: v.cpu().numpy() for kk, v in p.rnd.state_dict().items()})
        import prl_native
        plan = prl_native.ppo_update_last_plan()
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **sd, _n=np.int64(n), _head=head,
                 _key=np.uint64(a.sample_seed), _loss=np.float32(p.last_loss.item()),
                 _path=np.array(p.last_update_path), _split=np.int32(plan["split"]),
                 _grid=np.int32(plan["grid"]))
        if getattr(p, "_engine", None) is not None:
            p._engine.close()
    finally:
        torch.distributed.destroy_process_group()


# BASELINE.json configs[3] (C4: CartPole, 65,536 envs per rank) and configs[4] (C5: synthetic
# D 348 / A 17 + RND, 16,384 envs per rank), on 2 ranks sharing cuda:0, k_epochs 1
C4 = dict(env="CartPole-v1", E=65536, cont=False, D=4, A=2, mb=512, k=1, rnd=False)
C5 = dict(env="SyntheticHumanoid-v0", E=16384, cont=True, D=348, A=17, mb=65536, k=1, rnd=True)


@pytest.mark.parametrize("name,cfg", [("c4", C4), ("c5", C5)])
def test_two_ranks_at_config_per_rank_shape(tmp_path, name, cfg):
    """C4 / C5 per-rank shapes end to end on 2 ranks: independent rollouts (different envs and
    sampling keys per rank), one data-parallel learn() (C4: the data-parallel persistent engine,
    the default; C5: graphed per-step path + RND update_pred with its gradient all-reduced); both ranks
    end with bit-identical policy (and predictor) weights and finite losses."""
    import random
    port = 29800 + random.randint(0, 150)
    mp.spawn(_config_worker, args=(2, port, cfg, str(tmp_path)), nprocs=2, join=True)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    assert int(outs[0]["_key"]) != int(outs[1]["_key"])              # rank-mixed sampling keys
    assert not np.array_equal(outs[0]["_head"], outs[1]["_head"])    # different rollouts
    assert min(int(o["_n"]) for o in outs) >= cfg["E"]               # >= one step per env
    assert str(outs[0]["_path"]) == ("fused-dp-persistent" if name == "c4" else "graph")
    for key in outs[0].files:
        if not key.startswith("_"):
            np.testing.assert_array_equal(outs[0][key], outs[1][key], err_msg=key)
    assert all(np.isfinite(o["_loss"]) for o in outs)   # each rank reports its own rows


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,cfg", [("c4", C4), ("c5", C5)])
def test_eight_ranks_at_config_per_rank_shape(tmp_path, name, cfg):
    """The WHOLE C4 (8 x 65,536 CartPole envs) and C5 (8 x 16,384 synthetic envs + RND)
    workloads as 8 data-parallel ranks sharing cuda:0 (the 8-GPU node's rank layout rehearsed on
    one GPU; gloo for the host exchange): independent rollouts, one learn() each, the assertions
    of test_two_ranks_at_config_per_rank_shape.  C4 runs the data-parallel persistent engine;
    8 ranks x 64 split workgroups exceed one GPU's CUs, so the ranks' co-residency vote
    (PPO/engine.py dp_slices) picks the 8-wave kernel (8 x 32 workgroups) — on a node each rank
    has a GPU of its own and the split kernel runs.  C5: the wide step + the RND predictor's
    all-reduced update.  All 8 ranks end bit-identical."""
    import random
    port = 28800 + random.randint(0, 150)
    world = 8
    mp.spawn(_config_worker, args=(world, port, cfg, str(tmp_path)), nprocs=world, join=True)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    assert len({int(o["_key"]) for o in outs}) == world                # rank-mixed sampling keys
    for r in range(1, world):
        assert not np.array_equal(outs[0]["_head"], outs[r]["_head"])  # different rollouts
    assert min(int(o["_n"]) for o in outs) >= cfg["E"]                 # >= one step per env
    if name == "c4":
        assert all(str(o["_path"]) == "fused-dp-persistent" for o in outs)
        assert all(int(o["_split"]) == 0 and int(o["_grid"]) == 32 for o in outs)   # 8 x 32 CUs
    else:
        assert all(str(o["_path"]) == "graph" for o in outs)
    for key in outs[0].files:
        if not key.startswith("_"):
            for r in range(1, world):
                np.testing.assert_array_equal(outs[0][key], outs[r][key], err_msg=f"{key} rank {r}")
    assert all(np.isfinite(o["_loss"]) for o in outs)


@pytest.mark.timeout(300)
def test_eight_ranks_persistent_dp_engine_push_equals_pull(tmp_path):
    """8 data-parallel ranks sharing cuda:0 at mb 64 (8 x 8 split workgroups: the head-split
    kernel fits, so this is the DEFAULT push form of the exchange at the node's rank count):
    unequal shards (rank 1 one minibatch short), two learn() calls; the push form gives exactly
    the pull form's bits and all 8 ranks end bit-identical."""
    import random
    mb, nb, k, world = 64, 5, 3, 8
    port = 28500 + random.randint(0, 30)
    mp.spawn(_dpx_worker, args=(world, port, mb, nb, k, str(tmp_path), "auto", False), nprocs=world,
             join=True)
    mp.spawn(_dpx_worker, args=(world, port + 40, mb, nb, k, str(tmp_path), "auto", True),
             nprocs=world, join=True)
    pull = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    push = [np.load(os.path.join(tmp_path, f"pushrank{r}.npz")) for r in range(world)]
    assert int(push[0]["_push"]) == 1 and int(pull[0]["_push"]) == 0
    assert all(int(o["_split"]) == 1 for o in push + pull)
    assert all(str(o["_path"]) == "fused-dp-persistent" for o in push + pull)
    for key in pull[0].files:
        if key.startswith("_"):
            continue
        for r in range(world):
            np.testing.assert_array_equal(pull[r][key], pull[0][key], err_msg=key)
            np.testing.assert_array_equal(push[r][key], pull[0][key], err_msg=key)
    assert float(push[0]["_loss"]) == float(pull[0]["_loss"])


def _wide_shard(rank, mb, nb, D=348, A=17):
    rng = np.random.default_rng(100 + rank)
    n = mb * nb
    S = (rng.normal(size=(n, D)) * 0.5).astype(np.float32)
    Aa = (np.tanh(rng.normal(size=(n, A))) * 0.3).astype(np.float32)
    R = rng.normal(1, 0.5, n).astype(np.float32)
    Dn = (rng.random(n) < 0.02).astype(np.float32)
    Dn[mb - 1::mb] = 1      # episodes end at every minibatch block: GAE equal on the union
    return S, Aa, R, Dn


def _make_wide_ppo(mb, k):
    from PPO import PPO
    torch.manual_seed(0)
    p = PPO(True, 348, 17, action_scaling=1.0, lr=3e-4, k_epochs=k, batch_size=1,
            mini_batch_size=mb, policy_clip=1e3)     # smooth surrogate: compare in function space
    p.show_progress = False
    p.graph_min_steps = 1
    return p


def _wide_worker(rank, world, port, mb, nb, k, out_dir):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        p = _make_wide_ppo(mb, k)
        p.memory.push_device(*(torch.from_numpy(x).cuda() for x in _wide_shard(rank, mb, nb)))
        p.learn()
        torch.cuda.synchronize()
        sd = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **sd,
                 _wide=np.int64(p._last_graphed is not None and p._last_graphed.wide is not None),
                 _path=np.array(p.last_update_path))
    finally:
        torch.distributed.destroy_process_group()


def test_two_ranks_wide_step_equal_one_process_on_the_union(tmp_path):
    """C5's net (D 348, A 17) on 2 ranks through the wide step (prl_ppo_wide_grad into the
    all-reduce buffer, scaled by 1 / union rows) vs ONE process on the interleaved union with
    minibatch 2 mb: both ranks bit-identical, and the learned function equal to 1e-3 (the sums
    differ in order)."""
    import copy
    import random
    import types
    mb, nb, k = 256, 4, 2
    port = 29960 + random.randint(0, 30)
    mp.spawn(_wide_worker, args=(2, port, mb, nb, k, str(tmp_path)), nprocs=2, join=True)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    assert str(outs[0]["_path"]) == "graph" and int(outs[0]["_wide"]) == 1
    shards = [_wide_shard(r, mb, nb) for r in range(2)]
    cols = [np.concatenate([shards[r][c][j * mb:(j + 1) * mb] for j in range(nb) for r in range(2)])
            for c in range(4)]
    p = _make_wide_ppo(2 * mb, k)
    p.memory.push_device(*(torch.from_numpy(x).cuda() for x in cols))
    p.learn()
    ref = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
    for key in ref:
        np.testing.assert_array_equal(outs[0][key], outs[1][key], err_msg=key)
    q = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
    q.policy.load_state_dict({kk: torch.from_numpy(outs[0][kk]) for kk in ref})
    S = torch.from_numpy(cols[0][:256]).cuda()
    A = torch.from_numpy(cols[1][:256]).cuda()
    from test_engine_gpu import _outputs
    (l1, v1), (l2, v2) = _outputs(q, S, A), _outputs(p, S, A)
    el = float((l1 - l2).abs().max()) / (float(l2.abs().max()) + 1.0)
    ev = float((v1 - v2).abs().max()) / (float(v2.abs().max()) + 1.0)
    assert el <= 1e-3 and ev <= 1e-3, (el, ev)


def _rnd_gpu_worker(rank, world, port, mb, rows, D, out_dir):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from PPO import PPO
        from PPO.RND import RND
        torch.manual_seed(7)                       # same initial predictor / target on every rank
        r = RND(D, D, device="cuda")
        x = torch.from_numpy(np.random.default_rng(100 + rank).normal(size=(rows[rank], D))
                             .astype(np.float32)).cuda()
        nb = max(-(-n // mb) for n in rows)
        counts = [sum(min(mb, max(0, n - j * mb)) for n in rows) for j in range(nb)]
        r.update_pred(list(x.split(mb)), PPO.all_reduce, counts)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"rnd{rank}.npz"),
                 **{k: v.cpu().numpy() for k, v in r.pred_net.state_dict().items()})
    finally:
        torch.distributed.destroy_process_group()


def test_rnd_update_pred_two_ranks_on_gpu_equal_one_process_on_the_union(tmp_path):
    """RND.update_pred (RND.py:96-115) on 2 data-parallel ranks sharing cuda:0, at
    C5's width (D = 348) with a first minibatch of 16,384 rows per rank, so the predictor's
    backward runs the HIP GroupNorm+SiLU kernels (layers.GroupNormSiLU) and, on rank 0, the
    split-K / colsum weight and bias gradients (layers.SPLIT_MIN_ROWS); rank 1 has fewer rows
    (unequal shards, lockstep).  Against ONE process on the CPU (the reference's own PyTorch-CPU
    arithmetic) whose minibatch j is [rank0 slice j | rank1 slice j]: both ranks bit-identical,
    weights within 1e-5 (3 AdamW steps of lr 1e-3 from different float32 summation orders —
    GEMMs, the MSE difference pass + rocBLAS dot, the split-K reduction: AdamW's first steps are
    ~lr * sign(g), so entries whose gradient is near zero move by up to a step on either side;
    1e-5 is 0.33 % of the 3e-3 a weight can move; 6.1e-6 measured on MI355X)."""
    import random
    from PPO.RND import RND
    D, mb, rows = 348, 16384, (16384 + 9000, 13000)
    port = 29900 + random.randint(0, 50)
    mp.spawn(_rnd_gpu_worker, args=(2, port, mb, rows, D, str(tmp_path)), nprocs=2, join=True)
    outs = [np.load(os.path.join(tmp_path, f"rnd{r}.npz")) for r in range(2)]
    xs = [np.random.default_rng(100 + r).normal(size=(rows[r], D)).astype(np.float32)
          for r in range(2)]
    nb = max(-(-n // mb) for n in rows)
    union = [torch.from_numpy(np.concatenate([x[j * mb:(j + 1) * mb] for x in xs]))
             for j in range(nb)]
    torch.manual_seed(7)
    r = RND(D, D, device="cpu")         # same (CPU-drawn) initial weights as the ranks
    r.update_pred(union)
    ref = r.pred_net.state_dict()
    worst = 0.0
    for key in ref:
        np.testing.assert_array_equal(outs[0][key], outs[1][key], err_msg=key)
        worst = max(worst, float(np.abs(outs[0][key] - ref[key].numpy()).max()))
    print(f"max |2-rank GPU predictor - CPU union| {worst:.2e}")
    assert worst <= 1e-5, worst


def _dpx_fail_worker(rank, world, port, mb, nb, k, out_dir, persistent):
    sys.path[:0] = PATHS
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      PRL_DP_PERSISTENT="1" if persistent else "0")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import prl_native
        torch.cuda.set_device(0)
        p = _make_ppo(mb, k)
        S, A, R, D = _shard(rank, mb, nb)
        if rank == 1:
            S, A, R, D = (x[:-mb] for x in (S, A, R, D))
        data = [torch.from_numpy(x).cuda() for x in (S, A, R, D)]
        p.memory.push_device(*data)
        p.learn()                                   # healthy launch (default wait limit)
        paths = [str(p.last_update_path)]
        if persistent:   # second learn: rank 1 launches 2 s late, the wait limit is ~ms
            import time
            prl_native.dp_set_spin_limit(1 << 12)
            p._engine.before_dp_launch = lambda r: time.sleep(2.0) if r == 1 else None
        p.memory.push_device(*data)
        p.learn()
        p._engine.before_dp_launch = None
        prl_native.dp_set_spin_limit(0)
        paths.append(str(p.last_update_path))
        torch.cuda.synchronize()
        sd = {kk: v.cpu().numpy() for kk, v in p.policy.state_dict().items()}
        np.savez(os.path.join(out_dir, f"{'dpx' if persistent else 'st'}{rank}.npz"), **sd,
                 _paths=np.array(paths), _fallbacks=np.int64(getattr(p._engine, "dp_fallbacks", 0)),
                 _step=np.float32(p._engine.step.item()))
        p._engine.close()
    finally:
        torch.distributed.destroy_process_group()


def test_dpx_timeout_restores_and_falls_back_to_stepped_loop(tmp_path):
    """The data-parallel persistent launch when a peer is late:
    the cross-rank wait limit lowered to ~ms (prl_dp_set_spin_limit) and rank 1 launching 2 s
    after rank 0.  Rank 0's wait times out; rank 1 then waits on rank 0's next step and times
    out too.  Every rank gathers (status, checksum) in one collective, restores the pre-launch
    parameters / moments / step count and re-runs the update on the stepped loop.  Checked:
    no hang, one fallback on each rank, the path recorded as the stepped one, both ranks
    bit-identical, the AdamW step count continuous, and the result equal to two learns on the
    stepped loop alone in function space (learn 1 ran persistent; the two forms sum the clip norm
    in different orders)."""
    import copy
    import random
    import types
    mb, nb, k = 64, 5, 3
    port = 29860 + random.randint(0, 30)
    mp.spawn(_dpx_fail_worker, args=(2, port, mb, nb, k, str(tmp_path), True), nprocs=2, join=True)
    mp.spawn(_dpx_fail_worker, args=(2, port + 40, mb, nb, k, str(tmp_path), False), nprocs=2,
             join=True)
    outs = [np.load(os.path.join(tmp_path, f"dpx{r}.npz")) for r in range(2)]
    ref = np.load(os.path.join(tmp_path, "st0.npz"))
    assert [str(x) for x in outs[0]["_paths"]] == ["fused-dp-persistent", "fused-dp"]
    assert [str(x) for x in ref["_paths"]] == ["fused-dp", "fused-dp"]
    assert int(outs[0]["_fallbacks"]) == 1 and int(outs[1]["_fallbacks"]) == 1
    assert float(outs[0]["_step"]) == float(ref["_step"]) == 2 * k * nb
    keys = [kk for kk in outs[0].files if not kk.startswith("_")]
    for key in keys:
        np.testing.assert_array_equal(outs[0][key], outs[1][key], err_msg=key)
    p = _make_ppo(mb, k)
    q1 = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
    q2 = types.SimpleNamespace(policy=copy.deepcopy(p.policy))
    q1.policy.load_state_dict({kk: torch.from_numpy(outs[0][kk]) for kk in keys})
    q2.policy.load_state_dict({kk: torch.from_numpy(ref[kk]) for kk in keys})
    S, A, _, _ = _shard(0, mb, nb)
    from test_engine_gpu import _outputs
    (l1, v1), (l2, v2) = (_outputs(q, torch.from_numpy(S[:256]).cuda(),
                                   torch.from_numpy(A[:256]).cuda()) for q in (q1, q2))
    assert float((l1 - l2).abs().max()) <= 1e-4 and float((v1 - v2).abs().max()) <= 1e-4
