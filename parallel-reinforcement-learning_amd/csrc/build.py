"""Build libprl_hip.so (gfx950) in-tree with hipcc.  Usage: python build.py [-j N] [--force]

Every translation unit is compiled with -ffp-contract=off: the env physics, the GAE recurrence and
the surrogate follow the reference's float sequences operation for operation, so the compiler
must not fuse multiplies into adds behind our back (explicit fmaf/MFMA are unaffected).

The library carries a stamp of the sources it was built from (source_id(): sha256 over every
source and header, exported as prl_source_id); prl_native.lib() recomputes it from the files
next to it and refuses a library built from other sources.
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
SOURCES = ["prl_abi.hip", "prl_envs.hip", "prl_buffers.hip", "prl_gae.hip", "prl_loss.hip",
           "prl_rnd.hip", "prl_gn.hip",
           "prl_update.hip", "prl_ppo_update.hip", "prl_ppo_wide.hip", "prl_wide_rollout.hip"]
HEADERS = ["prl_common.h", "prl_envs.h", "prl_ppo_split.h", os.path.join("..", "..", "include", "prl_abi.h")]
LIB = os.path.join(PKG, "libprl_hip.so")
OBJDIR = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=off",
          "-fno-gpu-rdc", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
STAMPED = "prl_abi.hip"   # the translation unit that carries the source stamp


def source_id(csrc_dir=HERE) -> str:
    """sha256 over the sources and headers (name + bytes, fixed order)."""
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        h.update(name.encode())
        with open(os.path.join(csrc_dir, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def _compile(src, force, sid):
    obj = os.path.join(OBJDIR, src.replace(".hip", ".o"))
    deps = [os.path.join(HERE, src)] + [os.path.join(HERE, h) for h in HEADERS]
    extra = []
    if src == STAMPED:   # rebuilt whenever any source changes, so the stamp follows them
        deps = [os.path.join(HERE, s) for s in SOURCES] + [os.path.join(HERE, h) for h in HEADERS]
        extra = [f'-DPRL_SOURCE_ID="{sid}"']
    if not force and _mtime(obj) >= max(_mtime(d) for d in deps):
        return obj, None
    cmd = [HIPCC, *CFLAGS, *extra, *os.environ.get("PRL_EXTRA_CFLAGS", "").split(), "-c",
           os.path.join(HERE, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(jobs=None, force=False, verbose=False):
    os.makedirs(OBJDIR, exist_ok=True)
    sid = source_id()
    jobs = jobs or min(len(SOURCES), os.cpu_count() or 4, 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, sid), SOURCES))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    try:
        build(a.j, a.force, verbose=True)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
