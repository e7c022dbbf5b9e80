"""Fused update engine: PPO.learn's whole update loop (PPO/PPO.py:216-255) as ONE persistent HIP
kernel (csrc/prl_ppo_update.hip, C-ABI prl_ppo_update).

The kernel needs the policy's parameters and AdamW moments as flat vectors in torch
parameters() order.  FusedUpdate re-points every policy Parameter's .data at a view of one flat
buffer (Parameter objects, state_dict keys and the optimizer's param list are unchanged) and
makes the optimizer's `exp_avg` / `exp_avg_sq` state tensors views of two flat buffers, so the
engine and torch's AdamW share one copy of the state: an eager step taken afterwards (world > 1,
shapes outside the engine) continues exactly where the engine stopped.
"""
from __future__ import annotations

import os
import warnings

import torch

import prl_native


class FusedUpdate:
    # test injection point: called with this rank's index right before the data-parallel
    # persistent launch (tests make one rank late); None in production
    before_dp_launch = None

    def __init__(self, ppo, mini_batch: int):
        pol = ppo.policy
        self.ppo = ppo
        self.discrete = not ppo.is_continuous
        self.D, self.A = int(ppo.observ_dim), int(ppo.action_dim)
        info = prl_native.ppo_update_info(self.D, self.A, self.discrete, mini_batch)
        if info is None:
            raise ValueError("shape outside the fused engine")
        n_params, ws_bytes, self.grid = info
        self.params = [p for p in pol.parameters()]
        if sum(p.numel() for p in self.params) != n_params:
            raise ValueError("policy parameter count does not match the engine's layout")
        dev = self.params[0].device
        self.flat = torch.empty(n_params, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n_params, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n_params, dtype=torch.float32, device=dev)
        self.step = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
        self.mini_batch = int(mini_batch)
        self.events = None       # a list: (kernel, start, end, rows, optimizer steps) per launch
        self._bind()

    def _views(self, buf):
        out, off = [], 0
        for p in self.params:
            out.append(buf[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out

    def _bind(self):
        """Alias parameters and optimizer state onto the flat buffers (copies current values)."""
        opt = self.ppo.optimizer
        self._opt = opt   # the optimizer these moments belong to (a replaced one re-binds)
        with torch.no_grad():
            self.step.zero_()
            for p, fv, mv, vv in zip(self.params, self._views(self.flat), self._views(self.m),
                                     self._views(self.v)):
                fv.copy_(p.data)
                p.data = fv
                st = opt.state.get(p)
                if st and "exp_avg" in st:
                    mv.copy_(st["exp_avg"])
                    vv.copy_(st["exp_avg_sq"])
                    self.step.copy_(torch.as_tensor(st["step"], dtype=torch.float32).reshape(1))
                    st["exp_avg"], st["exp_avg_sq"] = mv, vv
                else:   # torch's AdamW starts a parameter without state from zero moments
                    mv.zero_()
                    vv.zero_()
        self._opt_views = (self._views(self.m), self._views(self.v))

    def bound(self) -> bool:
        """True while the policy parameters still live in the flat buffer and the optimizer is
        the one the moments were taken from."""
        if self.ppo.optimizer is not self._opt:
            return False
        return all(p.data.data_ptr() == fv.data_ptr()
                   for p, fv in zip(self.params, self._views(self.flat)))

    def _sync_optimizer_state(self):
        """Make the optimizer's state the engine's: moments as views, step counts = engine's."""
        opt = self.ppo.optimizer
        group = opt.param_groups[0]
        on_device = bool(group.get("capturable") or group.get("fused"))
        for p, mv, vv in zip(self.params, *self._opt_views):
            st = opt.state[p]
            st["exp_avg"], st["exp_avg_sq"] = mv, vv
            if "step" in st and torch.is_tensor(st["step"]):
                st["step"].copy_(self.step.reshape(st["step"].shape))
            else:
                st["step"] = (self.step.reshape(()).clone() if on_device
                              else torch.tensor(float(self.step.item())))

    def evaluate(self, module, S, A):
        """module.get_evaluate(S, A)'s log_prob and value for all rows (module: policy_old, same
        architecture) with the engine's forward arithmetic."""
        with torch.no_grad():
            flat = torch.cat([p.detach().reshape(-1) for p in module.parameters()])
        A2 = A if A.dim() == 2 else A.reshape(-1, 1)
        n = S.shape[0]
        logp = torch.empty(n, dtype=torch.float32, device=S.device)
        V = torch.empty(n, dtype=torch.float32, device=S.device)
        prl_native.ppo_evaluate(flat, self.D, self.A, self.discrete, S.contiguous(),
                                A2.contiguous(), logp, V)
        return logp, V

    def flops_per_row(self) -> int:
        """Algorithmic FLOPs of one row through the Linear layers: forward (2 MAC), weight
        gradients (2 MAC) and input gradients of every layer but the first (2 MAC); GroupNorm,
        SiLU, the loss and AdamW are not counted."""
        H = 64
        nh = 3 if not self.discrete else 2
        nout = self.A + 1 if self.discrete else 2 * self.A + 1
        trunk, heads, outs = self.D * H, nh * H * H, nout * H
        return 2 * (trunk + heads + outs) * 2 + 2 * (heads + outs)

    PHASES = ("forward+backward", "publish", "wait A", "slice reduce", "wait B", "norm",
              "AdamW")

    CHUNK_STAGES = ("forward", "barrier 1", "loss", "heads bwd + dW2", "barrier 2", "dW1",
                    "dF + trunk bwd", "dW0 + biases")

    def profile(self):
        """Workgroup 0's time per phase of the last launch, us per step (s_memrealtime, 100 MHz;
        recorded only with PRL_UPD_PROFILE=1 in the environment, zeros otherwise);
        'chunk' splits forward+backward by stage (summed over the step's 16-row tiles)."""
        p = prl_native.ppo_update_profile(self.ws).tolist()
        steps = max(p[7], 1)
        out = {name: round(p[i] * 0.01 / steps, 2) for i, name in enumerate(self.PHASES)}
        out["chunk"] = {name: round(p[8 + i] * 0.01 / steps, 2)
                        for i, name in enumerate(self.CHUNK_STAGES)}
        # sub-phase marks (time since the phase began): phase B's partial loads landed, its
        # slice stores issued; phase C's gradient loads landed
        out["sub"] = {name: round(p[16 + i] * 0.01 / steps, 2) for i, name in
                      enumerate(("B: partials landed", "B: slice stored", "C: gradient landed",
                                 "A: loop top to tile start"))}
        if p[24] > 0:   # the split form's arrival skew at counters A / B (every 16th step)
            n = p[24]
            out["skew"] = {"samples": n,
                           "A: last arrival - wg0": round(p[20] * 0.01 / n, 2),
                           "A: last - first": round(p[21] * 0.01 / n, 2),
                           "B: last arrival - wg0": round(p[22] * 0.01 / n, 2),
                           "B: last - first": round(p[23] * 0.01 / n, 2),
                           "A: last arriver critic frac": round(p[25] / n, 3)}
        if p[30] > 0:
            out["shader_clock_GHz"] = round(p[31] / (p[30] * 10.0), 3)
        out["clipped_steps_frac"] = round(p[28] / steps, 4)   # clip_grad_norm_ active
        return out

    def run(self, S, A, old_logp, adv, ret, k_epochs: int):
        """k_epochs x ceil(N / mini_batch) optimizer steps; returns the last step's loss (device)."""
        if not self.bound():
            self._bind()
        group = self.ppo.optimizer.param_groups[0]
        beta1, beta2 = group["betas"]
        A2 = A if A.dim() == 2 else A.reshape(-1, 1)
        if self.events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        prl_native.ppo_update(
            self.flat, self.m, self.v, self.step, self.D, self.A, self.discrete,
            S.contiguous(), A2.contiguous(), old_logp.contiguous(), adv.contiguous(),
            ret.contiguous(), self.mini_batch, k_epochs, self.ppo.policy_clip,
            self.ppo.value_coef, self.ppo.entropy_coef, group["lr"], beta1, beta2, group["eps"],
            group["weight_decay"], 2.0, self.loss, self.ws)
        if self.events is not None:
            ev[1].record()
            nb = -(-int(S.shape[0]) // self.mini_batch)
            kern = ("ppo_update_split_kernel" if prl_native.ppo_update_last_plan()["split"]
                    else "ppo_update_kernel")
            self.events.append((kern, ev[0], ev[1], int(S.shape[0]) * int(k_epochs),
                                int(k_epochs) * nb))
        self._sync_optimizer_state()
        status = max(prl_native.ppo_update_status(self.ws).tolist())
        if status != 0:
            # a launch that stopped part-way: start the next one from a clean workspace
            self.ws.zero_()
            raise RuntimeError(f"prl_ppo_update: in-kernel timeout (status {status}); the policy "
                               "parameters are undefined")
        return self.loss.reshape(())

    # ------------------------------------------------------------------ stepped (world_size > 1)
    def dp_comm(self):
        """This engine's own RCCL communicator for the native step loop (world > 1 on the nccl
        backend), or None: then run_stepped loops in Python with torch's all_reduce.  Every rank
        opens RCCL and votes; the communicator is built only if all ranks could open it.
        Opt-in (PRL_DP_NATIVE=1): it gives the Python loop's bits on one rank
        (test_native_dp_loop_equals_python_loop), but RCCL refuses two ranks on one GPU, so no
        test here has run it across ranks; until an 8-GPU run confirms it, the default is the
        Python loop (the 2-rank tests cover that one)."""
        if getattr(self, "_comm_tried", False):
            return self._comm
        self._comm_tried, self._comm = True, None
        if os.environ.get("PRL_DP_NATIVE", "0") != "1":
            return None
        import torch.distributed as tdist
        if not (tdist.is_available() and tdist.is_initialized() and tdist.get_backend() == "nccl"):
            return None
        dev = self.ws.device
        ok = torch.ones(1, dtype=torch.int32, device=dev)
        try:
            prl_native.dp_rccl_open()
        except (RuntimeError, OSError) as e:
            warnings.warn(f"native data-parallel loop unavailable ({e}); using the Python loop")
            ok.zero_()
        tdist.all_reduce(ok, op=tdist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            return None
        world, rank = tdist.get_world_size(), tdist.get_rank()
        uid = torch.zeros(prl_native.RCCL_UNIQUE_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(prl_native.dp_unique_id()), dtype=torch.uint8))
        tdist.broadcast(uid, src=0)
        self._comm = prl_native.dp_comm_init(bytes(uid.cpu().numpy().tobytes()), world, rank)
        return self._comm

    def close(self):
        """Destroy this engine's own RCCL communicator (if one was built) once the device is
        idle, and its data-parallel slice buffers (after every rank is idle: a peer may still be
        reading them); call on every rank before torch.distributed.destroy_process_group()."""
        comm = getattr(self, "_comm", None)
        if comm:
            torch.cuda.synchronize()
            prl_native.dp_comm_destroy(comm)
        self._comm = None
        xb = getattr(self, "_xbufs", None)
        if xb:
            import torch.distributed as tdist
            torch.cuda.synchronize()
            tdist.barrier()
            for r, ptr in enumerate(xb):
                if r != self._dp_rank:
                    prl_native.dp_ipc_close(ptr)
            tdist.barrier()
            prl_native.dp_xbuf_free(self._xbuf_own)
        self._xbufs, self._xb_tried = None, False

    # ---------------------------------- data-parallel persistent launch (world > 1, opt-in)
    def dp_slices(self):
        """Every rank's slice buffer for prl_ppo_update_dpx (this rank's own allocation and the
        peers' opened through IPC handles exchanged over torch.distributed), built once; None
        when PRL_DP_PERSISTENT=0, world > 8, or any rank could not build them or failed the
        self-test (a vote; then run_stepped's loop runs).  All ranks call it together.
        The self-test is one small launch on scratch copies of the optimizer state: it must end
        without an in-kernel timeout and leave bit-identical parameters on every rank.  Its
        2-rank GPU test runs both ranks on ONE GPU (IPC maps of the same device); on a node the
        maps are other GPUs' memory over xGMI, which the self-test checks before first use."""
        if getattr(self, "_xb_tried", False):
            return self._xbufs
        self._xb_tried, self._xbufs = True, None
        if os.environ.get("PRL_DP_PERSISTENT", "1") != "1":
            return None
        import torch.distributed as tdist
        if not (tdist.is_available() and tdist.is_initialized()):
            return None
        world, rank = tdist.get_world_size(), tdist.get_rank()
        own, handle, kind = None, b"", None
        if 1 < world <= 8:
            try:
                # PRL_DP_XBUF=fine forces the fine-grained fallback (tests), "uncached" forbids it
                own, kind = prl_native.dp_xbuf_alloc(
                    prl_native.dp_xbuf_bytes(self.D, self.A, self.discrete, self.mini_batch),
                    os.environ.get("PRL_DP_XBUF", "auto"))
                handle = prl_native.dp_ipc_handle(own)
            except (RuntimeError, ValueError) as e:
                warnings.warn(f"data-parallel slice buffer unavailable ({e})")
                own, handle, kind = None, b"", None
        handles = [None] * world
        tdist.all_gather_object(handles, (handle, kind))
        # the flags are fenced when ANY rank's buffer is fine-grained (prl_ppo_update_dpx)
        self._dp_fine = any(k == "fine" for _, k in handles)
        # the push form of the exchange (default; PRL_DP_PUSH=0 on any rank: the pull form) only
        # when every rank asks for it (one-GPU rehearsal: 17.1 vs 17.5 us per step at 2 ranks)
        push = [None] * world
        tdist.all_gather_object(push, os.environ.get("PRL_DP_PUSH", "1") != "0")
        self._dp_push = all(push)
        self.dp_xbuf_kinds = [k for _, k in handles]
        handles = [h for h, _ in handles]
        ptrs, ok = [], all(len(h) > 0 for h in handles)
        if ok:
            try:
                ptrs = [own if r == rank else prl_native.dp_ipc_open(h) for r, h in enumerate(handles)]
            except RuntimeError as e:
                warnings.warn(f"data-parallel peer slice buffers unavailable ({e})")
                ok = False
        votes = [None] * world
        tdist.all_gather_object(votes, ok)
        if not all(votes):
            for r, ptr in enumerate(ptrs):
                if r != rank:
                    prl_native.dp_ipc_close(ptr)
            tdist.barrier()
            prl_native.dp_xbuf_free(own)
            return None
        self._xbuf_own, self._xbufs, self._dp_rank, self._dp_seq = own, ptrs, rank, 0
        # every rank runs the same collectives whatever its local outcome: ONE gather of
        # (ok, checksum) per rank, then the same decision everywhere
        # co-residency: every rank's workgroups of one launch must be resident together, so ranks
        # that share a GPU (the one-GPU rehearsals) must fit its CUs between them — the split
        # kernel's 2 x tile groups per rank, else the 8-wave kernel's tile groups, else no
        # persistent launch at all (the stepped loop runs)
        votes = [None] * world
        tdist.all_gather_object(votes, (self._device_key(),
                                        prl_native.ppo_update_dp_split(self.D, self.A, self.discrete,
                                                                       self.mini_batch)))
        share = sum(1 for k, _ in votes if k == self._device_key())
        cus = torch.cuda.get_device_properties(self.flat.device).multi_processor_count
        fits = [None] * world
        tdist.all_gather_object(fits, (share * 2 * self.grid <= cus, share * self.grid <= cus))
        self._dp_split_fits = all(f for f, _ in fits)
        if not all(f for _, f in fits):
            warnings.warn("data-parallel persistent engine: the ranks sharing a GPU do not fit its "
                          "CUs together; using the stepped loop")
            self.close()
            self._xb_tried = True
            return None
        res = [None] * world
        tdist.all_gather_object(res, self._dp_selftest(
            world, all(s for _, s in votes) and self._dp_split_fits))
        sums = [c for _, c in res]
        if not (all(ok for ok, _ in res) and len(set(sums)) == 1 and sums[0] == sums[0]):
            warnings.warn("data-parallel persistent engine failed its self-test; using the "
                          "stepped loop")
            self.close()
            self._xb_tried = True
            return None
        return ptrs

    def _device_key(self):
        """Which physical GPU this rank's engine runs on (host + device UUID, or PCI location)."""
        import socket
        pr = torch.cuda.get_device_properties(self.flat.device)
        uid = str(getattr(pr, "uuid", "") or "")
        return (socket.gethostname(), uid or (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id))

    def _dp_checksum(self, flat) -> float:
        return float(flat.double().sum().item()) + float((flat.double() ** 2).sum().item())

    def _dp_selftest(self, world, split=True):
        """One small prl_ppo_update_dpx launch (2 minibatches per rank, k 1) on scratch copies
        of the state.  Local only (no collective): returns (ok, parameter checksum); the caller
        gathers every rank's pair at once."""
        try:
            mb = self.mini_batch
            n = 2 * mb
            dev = self.flat.device
            g = torch.Generator(device=dev).manual_seed(7 + self._dp_rank)
            S = torch.randn(n, self.D, device=dev, generator=g) * 0.5
            if self.discrete:
                A = (torch.rand(n, device=dev, generator=g) * self.A).floor().reshape(-1, 1)
            else:
                A = torch.randn(n, self.A, device=dev, generator=g) * 0.3
            old = torch.randn(n, device=dev, generator=g) * 0.1 - 0.7
            adv, ret = torch.randn(n, device=dev, generator=g), torch.randn(n, device=dev, generator=g)
            flat, m, v, step = self.flat.clone(), self.m.clone(), self.v.clone(), self.step.clone()
            loss = torch.zeros(1, dtype=torch.float32, device=dev)
            group = self.ppo.optimizer.param_groups[0]
            inv = torch.full((2,), 1.0 / (n // 2 * world), dtype=torch.float32, device=dev)
            prl_native.ppo_update_dpx(
                flat, m, v, step, self.D, self.A, self.discrete, S, A, old, adv, ret, mb, 1, 2,
                inv, self.ppo.policy_clip, self.ppo.value_coef, self.ppo.entropy_coef,
                group["lr"], group["betas"][0], group["betas"][1], group["eps"],
                group["weight_decay"], 2.0, loss, world, self._dp_rank, self._xbufs,
                self._dp_seq, self.ws, fine_grained=self._dp_fine, push=self._dp_push, split=split)
            self._dp_seq += 2
            torch.cuda.synchronize()
            status = max(prl_native.ppo_update_status(self.ws).tolist())
            if status != 0:
                # the sticky word stays set: clear the workspace so the engine's own runs start clean
                self.ws.zero_()
                return False, None
            return True, self._dp_checksum(flat)
        except RuntimeError as e:
            warnings.warn(f"data-parallel persistent self-test failed ({e})")
            return False, None

    def run_dp_persistent(self, S, A, old_logp, adv, ret, k_epochs: int, n_ranks, all_reduce):
        """run() as one data-parallel rank: ONE persistent launch for the whole loop; each step's
        gradient is summed over the ranks inside it (union minibatch j = every rank's rows
        j*mb .. (j+1)*mb, weighted 1 / union rows, as run_stepped).

        Failure handling: parameters, both moments and the step count (3 x 36 KB for CartPole)
        are snapshotted before the launch.  After it every rank gathers (status, checksum) in ONE
        collective.  If any rank's launch timed out in its cross-rank wait (a peer late or gone:
        prl_dp_set_spin_limit) or the checksums differ, every rank restores its snapshot, drops
        the slice buffers and re-runs this learn()'s update through the stepped loop
        (run_stepped: one grad launch + all-reduce per step), which later learns keep using."""
        import torch.distributed as tdist
        xb = self.dp_slices()
        if not self.bound():
            self._bind()
        world = tdist.get_world_size()
        snap = (self.flat.clone(), self.m.clone(), self.v.clone(), self.step.clone())
        group = self.ppo.optimizer.param_groups[0]
        beta1, beta2 = group["betas"]
        mb = self.mini_batch
        nb = max(-(-n // mb) for n in n_ranks)
        counts = [sum(min(mb, max(0, n - j * mb)) for n in n_ranks) for j in range(nb)]
        inv = torch.tensor([1.0 / c for c in counts], dtype=torch.float32, device=S.device)
        A2 = A if A.dim() == 2 else A.reshape(-1, 1)
        # the ranks' launches must overlap: line them up (the cross-rank wait also absorbs skew).
        # The gather doubles as the vote on the kernel form: the head-split kernel only when every
        # rank's process would pick it (its split mode and CU count are per process)
        torch.cuda.synchronize()
        votes = [None] * world
        tdist.all_gather_object(votes, prl_native.ppo_update_dp_split(self.D, self.A, self.discrete, mb))
        split = all(votes) and getattr(self, "_dp_split_fits", True)
        if self.before_dp_launch is not None:   # test injection point (a late rank)
            self.before_dp_launch(self._dp_rank)
        if self.events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        try:
            prl_native.ppo_update_dpx(
                self.flat, self.m, self.v, self.step, self.D, self.A, self.discrete,
                S.contiguous(), A2.contiguous(), old_logp.contiguous(), adv.contiguous(),
                ret.contiguous(), mb, k_epochs, nb, inv, self.ppo.policy_clip,
                self.ppo.value_coef, self.ppo.entropy_coef, group["lr"], beta1, beta2,
                group["eps"], group["weight_decay"], 2.0, self.loss, world, self._dp_rank, xb,
                self._dp_seq, self.ws, fine_grained=self._dp_fine, push=self._dp_push,
                split=split)
            launch_error = None
        except (RuntimeError, ValueError) as e:
            # this rank did not launch (e.g. an argument check): it still joins the gather
            # below with a nonzero status, so every rank takes the same restore / fallback
            launch_error = e
        self._dp_seq += int(k_epochs) * nb
        if self.events is not None:
            ev[1].record()
            self.events.append(("ppo_update_kernel_dp", ev[0], ev[1],
                                int(S.shape[0]) * int(k_epochs), int(k_epochs) * nb))
        status = (max(prl_native.ppo_update_status(self.ws).tolist()) if launch_error is None
                  else -1)
        res = [None] * world
        tdist.all_gather_object(res, (status, self._dp_checksum(self.flat) if status == 0 else None))
        sums = [c for _, c in res]
        if all(st == 0 for st, _ in res) and len(set(sums)) == 1:
            self._sync_optimizer_state()
            return self.loss.reshape(())
        # a rank timed out or the ranks diverged: restore, and take the stepped loop from here
        warnings.warn(f"data-parallel persistent launch failed (status / checksum per rank: "
                      f"{res}{'; this rank: ' + str(launch_error) if launch_error else ''}); restoring the pre-launch state and re-running this update on "
                      "the stepped loop")
        self.flat.copy_(snap[0])
        self.m.copy_(snap[1])
        self.v.copy_(snap[2])
        self.step.copy_(snap[3])
        self.ws.zero_()
        self.dp_fallbacks = getattr(self, "dp_fallbacks", 0) + 1
        self.close()
        self._xb_tried = True            # dp_slices() -> None from now on
        self._sync_optimizer_state()
        return self.run_stepped(S, A, old_logp, adv, ret, k_epochs, n_ranks, all_reduce)

    def run_stepped(self, S, A, old_logp, adv, ret, k_epochs: int, n_ranks, all_reduce,
                    comm=None):
        """The same update loop for data-parallel ranks.  Per optimizer step ONE launch,
        prl_ppo_grad_fold_step: the previous step's clip_grad_norm_ + AdamW (folded in front)
        then this rank's slice of the union minibatch j (scaled by 1 / union rows) -> its
        gradient image; then the all_reduce of that image (RCCL over xGMI on the GPU node).  The
        last step's AdamW is one prl_ppo_adam_step.  Parameters and moments stay in the engine's
        image layout in HBM for the whole loop, double-buffered (a launch reads one set while
        its workgroups write their slices of the other).  With `comm` (an RCCL communicator from
        dp_comm()) the loop is enqueued natively (prl_ppo_update_dp: no Python per step,
        ncclAllReduce on torch's stream); otherwise it runs here, calling `all_reduce` on the
        gradient image every step.  Both give the same bits."""
        import ctypes
        if k_epochs > 0 and comm is None and self.dp_slices() is not None:
            return self.run_dp_persistent(S, A, old_logp, adv, ret, k_epochs, n_ranks, all_reduce)
        if not self.bound():
            self._bind()
        group = self.ppo.optimizer.param_groups[0]
        beta1, beta2 = group["betas"]
        dev = S.device
        L = prl_native.ppo_image_floats(self.D, self.A, self.discrete)
        if getattr(self, "img", None) is None or self.img[0].numel() != L:
            self.img = [torch.zeros(L, dtype=torch.float32, device=dev) for _ in range(3)]
            self.grad = torch.zeros(L, dtype=torch.float32, device=dev)
            self.img_b = [torch.zeros(L, dtype=torch.float32, device=dev) for _ in range(3)]
            self.grad_b = torch.zeros(L, dtype=torch.float32, device=dev)
        img_p, img_m, img_v = self.img
        prl_native.ppo_image(self.D, self.A, self.discrete, self.flat, self.m, self.v,
                             img_p, img_m, img_v, True)
        mb = self.mini_batch
        nb = max(-(-n // mb) for n in n_ranks)
        counts = [sum(min(mb, max(0, n - j * mb)) for n in n_ranks) for j in range(nb)]
        A2 = (A if A.dim() == 2 else A.reshape(-1, 1)).contiguous()
        tens = [S.contiguous(), A2, old_logp.contiguous(), adv.contiguous(), ret.contiguous()]
        for x in tens:
            prl_native._dev(x, torch.float32, "update input")
        P = ctypes.c_void_p
        lib = prl_native.lib()
        stream = P(torch.cuda.current_stream().cuda_stream)
        # clip, vf_coef, ent_coef, lr, beta1, beta2, eps, weight_decay, max_norm (the betas as
        # doubles: prl_native._UPD_SCALARS)
        hyper = tuple(ctypes.c_float(x) for x in (
            self.ppo.policy_clip, self.ppo.value_coef, self.ppo.entropy_coef, group["lr"]))
        hyper += (ctypes.c_double(beta1), ctypes.c_double(beta2))
        hyper += tuple(ctypes.c_float(x) for x in (group["eps"], group["weight_decay"], 2.0))
        step = int(round(float(self.step.item())))
        n_local = int(S.shape[0])
        if comm is not None and k_epochs > 0:
            if self.events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            prl_native.ppo_update_dp(img_p, img_m, img_v, self.D, self.A, self.discrete, *tens,
                                     mb, k_epochs, counts, step, self.ppo.policy_clip,
                                     self.ppo.value_coef, self.ppo.entropy_coef, group["lr"],
                                     beta1, beta2, group["eps"], group["weight_decay"], 2.0,
                                     self.grad, self.loss, self.ws, comm)
            if self.events is not None:
                ev[1].record()
                self.events.append(("ppo_update_dp", ev[0], ev[1], n_local * k_epochs,
                                    k_epochs * nb))
            step += k_epochs * nb
            k_epochs = 0   # the Python loop below has nothing left to do
        sets = [self.img, self.img_b]
        grads = [self.grad, self.grad_b]
        cur, inv_prev, total = 0, 0.0, k_epochs * nb
        null = P()
        for s in range(total):
            j = s % nb
            inv = 1.0 / counts[j]
            if s > 0:
                fin, fout, gprev = sets[cur], sets[cur ^ 1], grads[(s - 1) & 1]
                fold = tuple(P(x.data_ptr()) for x in fin + fout) + (P(gprev.data_ptr()), step,
                                                                     ctypes.c_float(inv_prev))
                cur ^= 1
            else:
                fold = (P(sets[0][0].data_ptr()),) + (null,) * 6 + (0, ctypes.c_float(0.0))
            gout = grads[s & 1]
            if self.events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            rc = lib.prl_ppo_grad_fold_step(
                *fold, self.D, self.A, int(self.discrete), *(P(x.data_ptr()) for x in tens),
                n_local, mb, j, ctypes.c_float(inv), *hyper, P(self.loss.data_ptr()),
                P(gout.data_ptr()), P(self.ws.data_ptr()), self.ws.numel(), stream)
            if rc != 0:
                prl_native._check(rc, "prl_ppo_grad_fold_step")
            if self.events is not None:
                ev[1].record()
                self.events.append(("ppo_grad_kernel", ev[0], ev[1],
                                    min(mb, max(0, n_local - j * mb)), 1))
            all_reduce(gout)
            step += 1
            inv_prev = inv
        if total > 0:
            p_, m_, v_ = sets[cur]
            rc = lib.prl_ppo_adam_step(
                P(p_.data_ptr()), P(m_.data_ptr()), P(v_.data_ptr()), self.D, self.A,
                int(self.discrete), P(grads[(total - 1) & 1].data_ptr()), step, *hyper[3:],
                ctypes.c_float(inv_prev), hyper[1], hyper[2], P(self.loss.data_ptr()), stream)
            if rc != 0:
                prl_native._check(rc, "prl_ppo_adam_step")
            if cur != 0:
                for dst, src in zip(self.img, self.img_b):
                    dst.copy_(src)
            if (total - 1) & 1:
                self.grad.copy_(self.grad_b)
        prl_native.ppo_image(self.D, self.A, self.discrete, self.flat, self.m, self.v,
                             img_p, img_m, img_v, False)
        self.step.fill_(float(step))
        self._sync_optimizer_state()
        status = max(prl_native.ppo_update_status(self.ws).tolist())
        if status != 0:
            raise RuntimeError(f"prl_ppo_grad_step: in-kernel timeout (status {status})")
        return self.loss.reshape(())
