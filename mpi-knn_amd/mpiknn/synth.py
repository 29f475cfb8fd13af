"""Synthetic corpora for the benchmark (no dataset can be fetched here).

mnist_like(): the MNIST-784 shape of BASELINE.json configs[1] -- 60000 rows
of 784 integer "pixels" in 0..255 stored as fp64, labels 1..10, from 10
smooth class prototypes with per-row contrast jitter and noise.  Integer
valued like the real train_X, so the engine runs the same (exact-integer)
mode it would on MNIST.  Deterministic in (m, n, seed).
"""
import numpy as np


def mnist_like(m=60000, n=784, seed=1234):
    rng = np.random.default_rng(seed)
    side = int(round(np.sqrt(n)))
    cell = max(side // 8, 1)
    protos = []
    for _ in range(10):
        g = rng.normal(0, 1, (8, 8))
        img = np.resize(np.kron(g, np.ones((cell, cell))), n)
        img = (img - img.min()) / (np.ptp(img) + 1e-9) * 255
        protos.append(img)
    protos = np.array(protos)
    y = rng.integers(0, 10, m)
    scale = rng.uniform(0.6, 1.0, (m, 1))
    X = protos[y] * scale + rng.normal(0, 40, (m, n))
    np.rint(X, out=X)
    np.clip(X, 0, 255, out=X)
    return X, (y + 1).astype(np.float64)
