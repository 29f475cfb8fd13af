"""Deterministic test corpora.  All inputs are synthetic or
the sklearn digits set shipped in the image; nothing is fetched."""
import numpy as np


def digits():
    """sklearn digits 1797x64, integers 0..16, labels 1..10."""
    from sklearn.datasets import load_digits
    d = load_digits()
    return d.data.astype(np.float64), (d.target + 1).astype(np.float64)


def digits_real():
    """digits/16 + N(0, 0.05) (numpy default_rng(7)) plus the first 3 rows
    appended as exact duplicates: 1800x64 real-valued.  The reference's
    serial vote gives Matches = 1631 on it (probed)."""
    X, y = digits()
    r = np.random.default_rng(7)
    Xr = X / 16 + r.normal(0, 0.05, X.shape)
    return np.vstack([Xr, Xr[:3]]), np.concatenate([y, y[:3]])


def mnist_like(m, n=784, seed=1234):
    """MNIST-shaped integer corpus: 10 smooth class prototypes in 0..255,
    per-row brightness/offset jitter and noise, clipped and rounded.  Labels
    1..10.  Integer-valued like MNIST pixels, so the engine runs its exact
    integer mode."""
    rng = np.random.default_rng(seed)
    side = int(round(np.sqrt(n)))
    protos = []
    for c in range(10):
        g = rng.normal(0, 1, (8, 8))
        img = np.kron(g, np.ones((max(side // 8, 1), max(side // 8, 1))))
        img = np.resize(img, n)
        img = (img - img.min()) / (np.ptp(img) + 1e-9) * 255
        protos.append(img)
    protos = np.array(protos)
    y = rng.integers(0, 10, m)
    scale = rng.uniform(0.6, 1.0, (m, 1))
    X = protos[y] * scale + rng.normal(0, 40, (m, n))
    X = np.clip(np.rint(X), 0, 255)
    return X.astype(np.float64), (y + 1).astype(np.float64)


def mnist_real(m, n=784, seed=1234, noise_seed=0x5EA1):
    """Real-valued MNIST-shaped corpus (mpiknn.synth.mnist_real): the integer
    corpus / 255 + N(0, 1e-3), fp64 -- the engine's GEMM mode."""
    X, y = mnist_like(m, n, seed)
    X = X / 255.0 + np.random.default_rng(noise_seed).normal(0, 1e-3, X.shape)
    return X, y


def sift_like(m, n=128, clusters=1024, seed=0x51F7):
    """BASELINE configs[3] shape (SIFT-like): Gaussian mixture of `clusters`
    centres, clipped to [0, 255] and rounded -- integer-valued, fp32."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0, 160, (clusters, n))
    lab = rng.integers(0, clusters, m)
    X = centres[lab] + rng.normal(0, 25, (m, n))
    return np.clip(np.rint(X), 0, 255).astype(np.float64)


def gist_like(m, n=960, clusters=256, seed=0x6157):
    """BASELINE configs[4] shape (GIST-like): mixture in [0, 1), real-valued."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0.1, 0.6, (clusters, n))
    lab = rng.integers(0, clusters, m)
    X = centres[lab] + rng.normal(0, 0.08, (m, n))
    return np.clip(X, 0.0, np.nextafter(1.0, 0.0)).astype(np.float64)
