"""GPU parity of the fp32 path (dtype "f32", include/knn.h 'Element type').

Contract: the fp32 path returns the EXACT k nearest neighbours of the
fp32-rounded points under the reference's semantics (serial:72-93: sqrt of
the j-ordered fp64 sum S, zeros excluded, ties by lower index).  So:
  * against the oracle run on the rounded points: bit-exact, every mode;
  * integer data (exactly representable): bit-exact to the fp64 reference,
    both in fp32 INT mode (n max^2 <= 2^23) and fp32 GEMM mode (re-rank);
  * against the oracle on the ORIGINAL points: every reported distance
    within the stated bound 2^-24 (|q| + |c|) + 1e-12 d of the reference's
    distance to that same neighbour.
"""
import numpy as np
import pytest

import datasets
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def rounded(X):
    return X.astype(np.float32).astype(np.float64)


def run_engine(X, k, dtype="f32"):
    """One-block search through the device API; returns (result, mode, unresolved)."""
    import torch
    import mpiknn.ring as ring
    m, n = X.shape
    dev = torch.device("cuda", 0)
    e = ring.GpuEngine(torch, 0, n, m, m, k, dtype=dtype)
    e.pack(torch.from_numpy(np.ascontiguousarray(X)).to(dev), layout_col=False, elements=True)
    e.begin(0)
    e.step(e.qb, m, 0)
    u = e.end()
    if u:
        e.step(e.qb, m, 0, rescan=True)
        e.rescan_end()
    mode, _ = e.ctx.info()
    return e.result(), mode, u


@pytest.mark.parametrize("m,n", [(3000, 128), (2000, 17)])
def test_f32_integer_exact_mode(knn, oracle, m, n):
    X = datasets.sift_like(m, n, clusters=64, seed=m + n)
    ref = oracle.knn(X, 30)
    got, mode, _ = run_engine(X, 30)
    assert mode == 0, "expected fp32 integer-exact mode"
    assert_same(got, ref, "sift_like f32 %dx%d" % (m, n))


def test_f32_digits_matches_f64(knn, oracle):
    X, y = datasets.digits()
    ref = oracle.knn(X, 30, labels=y)
    got, _ = knn.search(X, 30, labels=y, dtype="f32")
    assert_same(got, ref, "digits f32")
    assert knn.classify(got, y, 10, knn.VOTE_SERIAL)[1] == 1636


def test_f32_mnist_gemm_mode_integer(knn, oracle):
    # n = 784 pixels exceed the fp32 integer bound: fp32 GEMM filter + exact
    # fp64 re-rank, still bit-exact (integers round to themselves)
    X, _ = datasets.mnist_like(2500, 784, seed=21)
    ref = oracle.knn(X, 30)
    got, mode, u = run_engine(X, 30)
    assert mode == 1
    assert_same(got, ref, "mnist_like f32 gemm")
    print("f32 gemm mnist: %d of %d queries rescanned" % (u, len(X)))


@pytest.mark.parametrize("maker", ["digits_real", "gaussian", "gist_like"])
def test_f32_real_valued(knn, oracle, maker):
    if maker == "digits_real":
        X = datasets.digits_real()[0]
    elif maker == "gaussian":
        X = np.random.default_rng(11).normal(0, 1, (1500, 96))
    else:
        X = datasets.gist_like(1200, 960, clusters=32)
    Xr = rounded(X)
    ref_r = oracle.knn(Xr, 30)
    got, mode, u = run_engine(X, 30)
    assert mode == 1
    assert_same(got, ref_r, "%s f32 vs oracle on rounded points" % maker)
    # distance tolerance against the reference on the original points
    nrm = np.sqrt((X * X).sum(1))
    for q in range(0, len(X), 97):
        for slot in range(30):
            j = got["idx"][q, slot] - 1
            if j < 0:
                continue
            d_ref = np.sqrt(((X[q] - X[j]) ** 2).sum())
            tol = 2.0 ** -24 * (nrm[q] + nrm[j]) + 1e-12 * d_ref
            assert abs(got["distance"][q, slot] - d_ref) <= tol, (maker, q, slot)


def test_f32_duplicates_and_ties(knn, oracle):
    X, _ = datasets.digits()
    X = np.vstack([X, X[:40], X[:40]]) / 3.0
    ref = oracle.knn(rounded(X), 30)
    got, _, _ = run_engine(X, 30)
    assert_same(got, ref, "duplicates f32")
    rng = np.random.default_rng(5)
    B = rng.integers(0, 2, (1200, 12)).astype(np.float64)
    assert_same(run_engine(B, 30)[0], oracle.knn(B, 30), "binary ties f32")


@pytest.mark.parametrize("m,n,k", [(300, 20, 30), (2000, 24, 100)])
def test_f32_nonfinite_scan(knn, oracle, m, n, k):
    """SCAN mode: every query takes the exact rescan, chunked over the
    corpus rows (2000 rows: 8 chunks; k = 100 merges 128-slot lists)."""
    rng = np.random.default_rng(3)
    X = rng.normal(0, 1, (m, n))
    X[5, 3] = np.nan
    X[17, 0] = np.inf
    got, mode, u = run_engine(X, k)
    assert mode == 2 and u == m
    assert_same(got, oracle.knn(rounded(X), k), "nan/inf f32 k=%d" % k)


@pytest.mark.parametrize("what,k", [("gist_like", 100), ("sift_like", 64), ("gaussian", 128),
                                    ("gist_like", 31), ("mnist_like", 100), ("binary", 100),
                                    ("gaussian", 16), ("gaussian", 17), ("gaussian", 33),
                                    ("dups", 17), ("dups", 100), ("sift_like", 32)])
def test_f32_large_k(knn, oracle, what, k):
    """k > 16: the 64-slot (24-deep lane lists, k <= 32) and 128-slot
    (40-deep, k <= 128; BASELINE configs[4]: k = 100) states at their
    boundaries, in every engine mode; exact duplicates (S == 0 entries next
    to the merge's exact-S window)."""
    if what == "dups":
        X, _ = datasets.digits()
        X = np.vstack([X, X[:40], X[:40]]) / 3.0
    elif what == "gist_like":
        X = datasets.gist_like(1500, 960, clusters=24, seed=k)
    elif what == "sift_like":
        X = datasets.sift_like(2500, 128, clusters=32, seed=7)   # fp32 INT mode
    elif what == "mnist_like":
        X = datasets.mnist_like(1300, 784, seed=4)[0]            # GEMM, integers
    elif what == "binary":
        X = np.random.default_rng(9).integers(0, 2, (900, 10)).astype(np.float64)  # ties
    else:
        X = np.random.default_rng(12).normal(0, 1, (1800, 72))
    got, mode, u = run_engine(X, k)
    if what == "sift_like":
        assert mode == 0
    assert_same(got, oracle.knn(rounded(X), k), "%s f32 k=%d" % (what, k))
    print("%s k=%d: mode %d, %d rescanned" % (what, k, mode, u))


def test_f32_k_exceeds_m(knn, oracle):
    # fewer points than k: missing slots {INFINITY, 0, 0}
    X = datasets.gist_like(70, 40, clusters=4, seed=1)
    got, _ = knn.search(X, 100, dtype="f32")
    ref = oracle.knn(rounded(X), 100)
    assert_same(got, ref, "m < k f32")
    assert np.isinf(got["distance"][:, 69:]).all() and (got["idx"][:, 69:] == 0).all()


@pytest.mark.parametrize("k", [30, 100])
def test_f32_ring_blocks(knn, oracle, k):
    """fp32 blocks rotated as in the ring (simulated on one GPU, P = 3)."""
    import torch
    import mpiknn.ring as ring
    X = datasets.gist_like(1000, 300, clusters=16, seed=3)
    m, n = X.shape
    full = oracle.knn(rounded(X), k)
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(X).to(dev)
    P = 3
    R, blocks = ring.partition(m, P)
    engines = []
    for g in range(P):
        base, rows = blocks[g]
        e = ring.GpuEngine(torch, 0, n, R, rows, k, dtype="f32")
        e.pack(Xd[base:base + rows].float(), layout_col=False, elements=True)   # fp32 source
        engines.append(e)
    meta = torch.stack([e.meta for e in engines]).max(dim=0).values
    for g, e in enumerate(engines):
        e.meta.copy_(meta)
        base, rows = blocks[g]
        e.begin(base)
        for s in range(P):
            b = (g - s) % P
            e.step(engines[b].qb, blocks[b][1], blocks[b][0])
        if e.end():
            for s in range(P):
                b = (g - s) % P
                e.step(engines[b].qb, blocks[b][1], blocks[b][0], rescan=True)
            e.rescan_end()
        assert_same(e.result(), full[base:base + rows], "f32 ring rank %d" % g)


# ---- split fp16 filter (knn_ctx_split: fp32 GEMM mode) --------------------
# The filter only chooses candidates; the exact fp64 re-rank and the
# certificate (knn_cert_E with the split error bound) make the results those
# of the oracle on the fp32-rounded points, bit for bit, and byte-identical
# to the fp32 MFMA filter's (KNN_NO_SPLIT=1).

def _split_case(X, k, monkeypatch, oracle):
    import torch
    import mpiknn.ring as ring
    m, n = X.shape
    e = ring.GpuEngine(torch, 0, n, m, m, k, dtype="f32")
    e.pack(torch.from_numpy(np.ascontiguousarray(X.astype(np.float32))).to("cuda:0"), layout_col=False,
           elements=True)
    e.begin(0)
    assert e.ctx.split() == 1, "expected the split fp16 filter"
    got, _, u = run_engine(X.astype(np.float32), k)
    assert_same(got, oracle.knn(rounded(X), k), "split f32 %dx%d k=%d" % (m, n, k))
    monkeypatch.setenv("KNN_NO_SPLIT", "1")
    base, _, ub = run_engine(X.astype(np.float32), k)
    monkeypatch.delenv("KNN_NO_SPLIT")
    assert got.tobytes() == base.tobytes()
    return u, ub


@pytest.mark.parametrize("m,n,k", [(2500, 960, 100), (3000, 128, 32), (1500, 40, 16), (2000, 333, 100)])
def test_split_filter_gist_like(knn, oracle, monkeypatch, m, n, k):
    X = datasets.gist_like(m, n, seed=m + n + k)
    u, ub = _split_case(X, k, monkeypatch, oracle)
    # the split filter's error bound is ~3.5x the fp32 filter's: a few more
    # queries may miss the certificate (they take the exact rescan)
    assert u <= 3 * ub + max(2, m // 50), "%d of %d queries uncertified (fp32 filter: %d)" % (u, m, ub)


@pytest.mark.parametrize("scale", [1e-7, 3e-3, 1.0, 5e4, 2e9])
def test_split_filter_scales(knn, oracle, monkeypatch, scale):
    """The power-of-two pre-scale keeps hi in fp16 and lo normal for any
    data magnitude; signed values, a few exact duplicates and near ties."""
    rng = np.random.default_rng(5)
    X = (rng.standard_normal((1200, 64)) * scale).astype(np.float32).astype(np.float64)
    X[10] = X[3]
    X[11] = X[3] * (1 + 2 ** -22)
    _split_case(X, 30, monkeypatch, oracle)


def test_split_filter_small_values_subnormal_lo(knn, oracle, monkeypatch):
    """Values spanning 12 orders of magnitude: the lo halves of the small
    ones are fp16 subnormals (the certificate's absolute term)."""
    rng = np.random.default_rng(9)
    X = rng.random((1500, 96)) * 10.0 ** rng.integers(-10, 2, (1500, 96))
    _split_case(X, 24, monkeypatch, oracle)


def test_split_filter_ring_loopback(knn, oracle, monkeypatch):
    """P = 4 loopback ring (element blocks travel, each rank converts them to
    split shadow rows) against the oracle."""
    monkeypatch.setenv("KNN_RING_LOOPBACK", "1")
    X = datasets.gist_like(2400, 200, seed=3)
    got, _ = knn.search(X, 50, ngpus=4, dtype="f32")
    assert_same(got, oracle.knn(rounded(X), 50), "split ring P=4")


@pytest.mark.parametrize("m,n", [(3000, 784), (2000, 100)])
def test_split_filter_fp64_blocks(knn, oracle, monkeypatch, m, n):
    """fp64 GEMM mode (SURVEY C1's real-valued data) on the split filter:
    bit-exact vs the oracle (the reference's fp64 S) and byte-identical to
    the fp64 MFMA filter (KNN_NO_SPLIT=1)."""
    X, _ = datasets.mnist_real(m, n)
    import torch
    import mpiknn.ring as ring
    e = ring.GpuEngine(torch, 0, n, m, m, 30, dtype="f64")
    e.pack(torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0"), layout_col=False, elements=True)
    e.begin(0)
    assert e.ctx.split() == 1
    got, _, u = run_engine(X, 30, dtype="f64")
    assert_same(got, oracle.knn(X, 30), "split f64 %dx%d" % (m, n))
    monkeypatch.setenv("KNN_NO_SPLIT", "1")
    base, _, ub = run_engine(X, 30, dtype="f64")
    assert got.tobytes() == base.tobytes()
    assert u <= ub + max(2, m // 200)


def test_gemm_state_holds_near_ties(knn, oracle):
    """fp64 GEMM mode, k = 30: each of 50 centre rows has 40 rows at one
    distance (0.5, spread 1e-9 -- inside the certificate window E ~ 1e-3 of
    one another).  The 64-entry state (knn_kp_for, fp64 16 < k <= 32) keeps
    all 40, so the smallest value a merge drops (Td) lies past the window
    and every query is certified in the first pass; a 32-entry state
    dropped the 33rd inside the window and sent each centre to the exact
    rescan.  Bit-exact vs the oracle either way."""
    rng = np.random.default_rng(5)
    n, nc = 64, 50
    C = rng.uniform(0, 1, (nc, n))
    parts = [C]
    for i in range(nc):
        u = rng.normal(0, 1, (40, n))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        parts.append(C[i] + 0.5 * u * (1 + 1e-9 * rng.standard_normal((40, 1))))
    X = np.vstack(parts)
    got, mode, u = run_engine(X, 30, dtype="f64")
    assert mode == 1   # GEMM
    assert_same(got, oracle.knn(X, 30), "near-tie crowd f64")
    assert u == 0, u


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_gemm_merge_query_order(knn, oracle, monkeypatch, dtype):
    """The GEMM-mode merge in the query order of knn_order.hip (label
    propagation over the lists' heads, then a radix sort; forced with
    KNN_ORDER=1 -- by default only past 64 MB blocks) gives the same bytes
    as the merge in index order, and the oracle's neighbours."""
    X, _ = datasets.mnist_real(3000, 200)
    if dtype == "f32":
        X = rounded(X)
    monkeypatch.setenv("KNN_ORDER", "1")
    got, mode, _ = run_engine(X, 30, dtype=dtype)
    assert mode == 1
    monkeypatch.delenv("KNN_ORDER")
    monkeypatch.setenv("KNN_NO_ORDER", "1")
    base, _, _ = run_engine(X, 30, dtype=dtype)
    assert got.tobytes() == base.tobytes()
    assert_same(got, oracle.knn(X, 30), "ordered merge %s" % dtype)
