"""Time the GAE traffic-pattern floors (cold cache, same method as bench.time_kernel)."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "parallel-reinforcement-learning_amd"), os.path.join(ROOT, "tools")]
from bench import time_kernel  # noqa: E402
from kernel_bench import gae_case  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libgae_floor.so"))
P = ctypes.c_void_p
for n in (2_277_376, 8_269_824, 13_107_200):
    r, d, V = (torch.rand(n, device="cuda") for _ in range(3))
    o1, o2 = torch.empty_like(r), torch.empty_like(r)
    s = P(torch.cuda.current_stream().cuda_stream)
    out = {"n": n}
    for name, var, grid in (("v0_8consec", 0, 0), ("v1_coalesced_g1024", 1, 1024),
                            ("v1_coalesced_g2048", 1, 2048), ("v1_coalesced_g4096", 1, 4096)):
        med, _ = time_kernel(lambda: lib.run_copy(var, P(r.data_ptr()), P(d.data_ptr()),
                                                  P(V.data_ptr()), P(o1.data_ptr()),
                                                  P(o2.data_ptr()), ctypes.c_int64(n), grid, s))
        out[name] = round(20 * n / (med * 1e-3) / 1e9, 1)
    out["gae_kernel"] = gae_case(n)["GB/s"]
    import prl_native
    rr, dd = torch.ones(n, device="cuda"), (torch.rand(n, device="cuda") < 0.05).float()
    dd[-1] = 1
    VV = torch.randn(n, device="cuda")
    ret = torch.empty_like(VV)
    med, _ = time_kernel(lambda: prl_native.gae(rr, dd, VV, None, 0.995, 0.95, ret))
    out["gae_ret_only_GBs_16B"] = round(16 * n / (med * 1e-3) / 1e9, 1)
    print(json.dumps(out), flush=True)
