"""The seeded learn() memory every learn*.npz fixture was made from (numpy default_rng(7)).

Shared by make_golden.py (which feeds it to the reference's PPO.learn) and the tests (which feed
it to ours), so large fixtures need not store their inputs: they store a digest of them instead.
"""
import hashlib

import numpy as np


def learn_inputs(N, D, A, continuous, seed=7):
    rng = np.random.default_rng(seed)
    S = (rng.normal(0, 1, (N, D)) * 0.5).astype(np.float32)
    if continuous:
        Aa = np.tanh(rng.normal(0, 1, (N, A))).astype(np.float32) * 2.0
    else:
        Aa = (rng.random(N) < 0.5).astype(np.int64)
    R = rng.normal(1.0, 0.5, N).astype(np.float32)
    Dn = (rng.random(N) < 0.05)
    Dn[-1] = True
    return S, Aa, R, Dn


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
