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


def mnist_real(m=60000, n=784, seed=1234, noise_seed=0x5EA1):
    """The real-valued MNIST variant (mnist_train_svd.mat is
    real-valued): mnist_like(m, n, seed) / 255 + N(0, 1e-3) (numpy
    default_rng(noise_seed)), fp64.  Not integer, so the engine runs its
    GEMM mode: the split-fp16 filter + exact reference-order re-rank."""
    X, y = mnist_like(m, n, seed)
    X /= 255.0
    X += np.random.default_rng(noise_seed).normal(0, 1e-3, X.shape)
    return X, y


def sift_like(m=1_000_000, n=128, clusters=1024, seed=0x51F7, chunk=1 << 18):
    """BASELINE.json configs[3] shape: SIFT-like 1M x 128, a mixture of
    `clusters` Gaussian centres clipped to [0, 255] and rounded (integer
    valued like SIFT descriptors), returned as float32 row-major (the fvecs
    layout).  Generated in chunks so 1M+ rows stay cheap."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0, 160, (clusters, n)).astype(np.float32)
    X = np.empty((m, n), dtype=np.float32)
    for lo in range(0, m, chunk):
        hi = min(m, lo + chunk)
        lab = rng.integers(0, clusters, hi - lo)
        blk = centres[lab] + rng.normal(0, 25, (hi - lo, n)).astype(np.float32)
        np.rint(blk, out=blk)
        np.clip(blk, 0, 255, out=blk)
        X[lo:hi] = blk
    return X


def gist_like(m=4_000_000, n=960, clusters=256, seed=0x6157, chunk=1 << 16):
    """BASELINE.json configs[4] shape: GIST-like x 960 real-valued features
    in [0, 1) (mixture of `clusters` centres + N(0, 0.08)), float32
    row-major."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0.1, 0.6, (clusters, n)).astype(np.float32)
    X = np.empty((m, n), dtype=np.float32)
    top = np.nextafter(np.float32(1), np.float32(0))
    for lo in range(0, m, chunk):
        hi = min(m, lo + chunk)
        lab = rng.integers(0, clusters, hi - lo)
        blk = centres[lab] + rng.normal(0, 0.08, (hi - lo, n)).astype(np.float32)
        np.clip(blk, 0, top, out=blk)
        X[lo:hi] = blk
    return X
