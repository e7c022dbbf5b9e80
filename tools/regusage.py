"""Register / spill summary of the kernels of one HIP source (device-only compile for gfx950).

Usage: python tools/regusage.py [source.hip] [name-substring]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else os.path.join(
    ROOT, "parallel-reinforcement-learning_amd", "csrc", "prl_ppo_update.hip")
pat = sys.argv[2] if len(sys.argv) > 2 else "kernel"
with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17",
                        "-ffp-contract=off", "-fno-gpu-rdc", "--cuda-device-only", "-c", src,
                        "-o", os.path.join(d, "o.o"), "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, cwd=d)
txt = r.stdout + r.stderr
if r.returncode != 0:
    print("\n".join(l for l in txt.splitlines() if "error" in l)[:4000])
    sys.exit(1)
for blk in txt.split("Function Name: ")[1:]:
    name = blk.split()[0]
    if pat not in name:
        continue

    def g(k):
        m = re.search(k + r": (\d+)", blk)
        return m.group(1) if m else "?"
    scr = g(r"ScratchSize \[bytes/lane\]")
    print(f"{name[:72]:72s} V {g('VGPRs'):>3} A {g('AGPRs'):>3} Vspill {g('VGPRs Spill'):>3} "
          f"Sspill {g('SGPRs Spill'):>3} scratch {scr}")
