"""fp16-MFMA contraction (include/knn.h knn_ctx_contraction_bits): fp32
searches take it when every value is an integer with max|x| <= 2048 inside
the fp32 exact-integer range, fp64 searches when every value is an integer
with max|x| <= 256 (fp32 partial sums over 256 features stay exact, then
fp64 accumulation).  Either way the result must be bit-identical to the
oracle.
Run with KNN_NO_I8=1 (the int8 path has its own tests, test_gpu_i8.py).
Checked through bench's per-rank engine (mpiknn.ring.GpuEngine) so the
contraction actually used is visible."""
import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp16_path(monkeypatch):
    # 8-bit-window data now takes the int8 contraction (test_gpu_i8.py);
    # these cases pin the fp16 one
    monkeypatch.setenv("KNN_NO_I8", "1")


def run_engine(X, k, dtype="f32"):
    import torch
    import mpiknn.ring as ring
    m, n = X.shape
    eng = ring.GpuEngine(torch, 0, n, m, m, k, dtype=dtype)
    npdt = np.float32 if dtype == "f32" else np.float64
    eng.pack(torch.from_numpy(np.ascontiguousarray(X, dtype=npdt)).to("cuda:0"),
             layout_col=False)
    ring.ring_search(None, torch, eng, 0, 1, m, 0)
    return eng.result(), eng.ctx.contraction_bits()


def check(oracle, X, k, bits, dtype="f32"):
    got, b = run_engine(X, k, dtype)
    assert b == bits
    ref = oracle.knn(X.astype(np.float32).astype(np.float64) if dtype == "f32" else X, k)
    assert np.array_equal(got["idx"], ref["idx"])
    assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64))


def test_h16_sift_like(oracle):
    check(oracle, datasets.sift_like(20000, 128), 32, 16)


def test_h16_boundary_values(oracle):
    # max|x| = 2048 and n max^2 = 2^23 exactly: the largest eligible data
    rng = np.random.default_rng(3)
    X = rng.integers(0, 2049, (4000, 2)).astype(np.float64)
    X[:50, 0] = 2048.0
    X[100] = X[7]                                  # exact duplicate
    check(oracle, X, 16, 16)


def test_h16_signed_with_duplicates(oracle):
    rng = np.random.default_rng(4)
    X = rng.integers(-60, 61, (3000, 100)).astype(np.float64)
    X[200:260] = X[0]                              # a mass of duplicates
    check(oracle, X, 16, 16)
    check(oracle, X, 100, 16)                      # the k=33..128 variant


def test_h16_not_taken_above_2048(oracle):
    rng = np.random.default_rng(5)
    X = rng.integers(0, 2050, (3000, 1)).astype(np.float64)
    X[0, 0] = 2049.0
    check(oracle, X, 8, 32)


def test_h16_not_taken_real_valued(oracle, monkeypatch):
    """Real-valued data never takes the exact fp16 contraction: it runs the
    split fp16 filter (knn_ctx_split) or, without it, fp32 MFMA."""
    X = datasets.digits_real()[0]
    monkeypatch.setenv("KNN_NO_SPLIT", "1")
    check(oracle, X, 30, 32)


def test_h16_fp64_mnist_like(oracle):
    check(oracle, datasets.mnist_like(3000, 784, seed=21)[0], 30, 16, "f64")


def test_h16_fp64_signed_boundary(oracle):
    # |x| = 256 with 784 features: every 256-feature fp32 partial sum may
    # reach 2^24 exactly -- the largest eligible data
    rng = np.random.default_rng(8)
    X = rng.integers(-256, 257, (2500, 784)).astype(np.float64)
    X[:20] = 256.0
    X[20:40] = -256.0
    X[41] = X[40]
    check(oracle, X, 32, 16, "f64")


def test_h16_fp64_not_taken(oracle, monkeypatch):
    rng = np.random.default_rng(9)
    X = rng.integers(0, 258, (2000, 50)).astype(np.float64)
    X[0, 0] = 257.0
    check(oracle, X, 30, 64, "f64")
    monkeypatch.setenv("KNN_NO_SPLIT", "1")   # (real-valued: the split fp16 filter otherwise)
    check(oracle, datasets.digits_real()[0], 30, 64, "f64")


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_h16_fragment_conversion_path(oracle, monkeypatch, dtype):
    """KNN_NO_SHADOW=1: the fp16 operands are converted from the element
    fragments in the kernel instead of staged from fp16 shadow rows."""
    monkeypatch.setenv("KNN_NO_SHADOW", "1")
    X = datasets.mnist_like(2500, 784, seed=31)[0] if dtype == "f64" else datasets.sift_like(6000, 128)
    check(oracle, X, 30, 16, dtype)
