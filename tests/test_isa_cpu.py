"""The built code object's memory-instruction encodings (CPU only: llvm-objdump of
libprl_hip.so's gfx950 offload bundles).  This file names scalar-cache write instructions as
things that must NOT appear, so it is listed in .gpurunignore (no GPU run loads it)."""
import os
import re

import pytest


# ------------------------------------------------------------------ hand-off encodings (ISA)
def _kernel_memory_ops():
    """{kernel symbol: [(opcode, has_sc0, has_sc1), ...]} of every vector / scalar memory
    instruction in libprl_hip.so's gfx950 code objects (llvm-objdump of the offload bundles)."""
    import glob
    import shutil
    import subprocess
    import tempfile
    import prl_native
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not in this image")
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        lib = os.path.join(tmp, "libprl_hip.so")
        shutil.copy(prl_native.LIB_PATH, lib)
        subprocess.run([objdump, "--offloading", lib], check=True, capture_output=True)
        bundles = sorted(glob.glob(lib + ".*gfx950"))
        assert bundles, "no gfx950 code object in libprl_hip.so"
        for b in bundles:
            asm = subprocess.run([objdump, "-d", "--mcpu=gfx950", b], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for line in asm.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
                if m:
                    cur = m.group(1)
                    out.setdefault(cur, [])
                    continue
                ins = line.strip().split("//")[0].strip()
                if not ins or cur is None:
                    continue
                op = ins.split()[0]
                if re.match(r"(flat|global|buffer|scratch|s_load|s_store|s_buffer|s_atomic|s_dcache)_", op):
                    out[cur].append((op, bool(re.search(r"\bsc0\b", ins)),
                                     bool(re.search(r"\bsc1\b", ins))))
    return out


def test_handoff_isa():
    """The cross-workgroup hand-offs in the built code object have the encodings the MI355X
    guide's hand-off table is measured for (MI355X_MICROARCH.md, 'Valid forms' and the sc1
    table):
      * no flat_ atomic and no flat_ access with an sc0 / sc1 cache policy anywhere: hand-off
        words are global_ / buffer_ accesses (round 3 found the runtime-layout update kernel's
        counters, status words and data-parallel flags lowered to flat_ and fixed it);
      * no scalar-cache store, atomic or write-back anywhere (s_store / s_buffer_store /
        s_atomic / s_dcache_wb);
      * in the update engine (ppo_update_kernel*, ppo_grad_kernel*) every buffer_ access — the
        resource path that carries only the exchanged partials, slices and gradients — is sc1
        (agent scope) or sc0 sc1 (system scope, the data-parallel slices); arrivals are
        global_atomic_add; polls of the counters are global_load_dword sc1;
      * the head-split kernel (ppo_update_split_kernel*, the default at mb <= 2,048, its
        data-parallel instances included) likewise: every buffer_ access sc1 / sc0 sc1, arrivals
        global_atomic_add, polls global_load_dword sc1;
      * flat_adamw's one-launch tail: the last arriver is told by a RETURNING global_atomic_add
        (sc0) with acquire-release ordering (buffer_wbl2 sc1 before it, buffer_inv sc1 after
        it), so it rescales the gradient and advances the step only after every other
        workgroup's reads of them;
      * the RND gradient folds (rnd_grad_fold1 / 2) hand nothing over inside a launch: no atomic,
        no sc1 access (their inputs come across a kernel boundary);
      * the GAE carry granules are 8-B global_ sc1 stores and loads."""
    ops = _kernel_memory_ops()
    assert len(ops) > 20
    bad = [(k, op) for k, v in ops.items() for op, s0, s1 in v
           if op.startswith("flat_") and (s0 or s1 or "atomic" in op)]
    assert not bad, bad[:10]
    scal = [(k, op) for k, v in ops.items() for op, _, _ in v
            if op.startswith(("s_store", "s_buffer_store", "s_atomic", "s_dcache"))]
    assert not scal, scal[:10]
    engine = {k: v for k, v in ops.items()
              if "ppo_update_kernel" in k or "ppo_grad_kernel" in k or "ppo_update_split_kernel" in k}
    assert len(engine) >= 14, sorted(engine)
    split = [k for k in engine if "ppo_update_split_kernel" in k]
    assert len(split) >= 5, split     # 4 / 8 waves, single-GPU / data-parallel, slice-owner
    for k, v in engine.items():
        buf = [(op, s0, s1) for op, s0, s1 in v if op.startswith("buffer_")]
        assert buf and all(s1 for _, _, s1 in buf), (k, [b for b in buf if not b[2]][:5])
        assert any(op == "global_atomic_add" for op, _, _ in v), k
        assert any(op == "global_load_dword" and s1 for op, _, s1 in v), k
    adam = {k: v for k, v in ops.items() if "flat_adamw" in k}
    assert adam, "flat_adamw kernel not found"
    for k, v in adam.items():
        assert any(op == "global_atomic_add" and s0 for op, s0, _ in v), k      # returning add
        assert any(op == "buffer_wbl2" and s1 for op, _, s1 in v), k            # agent release
        assert any(op == "buffer_inv" and s1 for op, _, s1 in v), k             # agent acquire
    folds = {k: v for k, v in ops.items() if "rnd_grad_fold" in k}
    assert len(folds) == 2, sorted(folds)
    for k, v in folds.items():
        assert not any("atomic" in op or s1 for op, _, s1 in v), k
    gae = {k: v for k, v in ops.items() if "gae_kernel" in k}
    assert gae
    for k, v in gae.items():
        assert any(op == "global_store_dwordx2" and s1 for op, _, s1 in v), k
        assert any(op == "global_load_dwordx2" and s1 for op, _, s1 in v), k
