"""int8-MFMA contraction (knn_i8.hip; knn_ctx_contraction_bits() == 8).

Taken when the search is in exact-integer mode and every value lies in a
window of 256 integers (meta max(x)+ + max(-x)+ <= 255) with n <= 896:
x - o is an exact int8 and every dot product an exact int32, so d^2 equals
the reference's S (knn-serial.c:76-85) bit for bit.  Every case here is
compared with the oracle (oracle/knn_oracle.c, serial:72-93): index AND
distance bits, plus the contraction actually used."""
import numpy as np
import pytest

import datasets
from test_gpu_h16 import run_engine

pytestmark = pytest.mark.gpu


def check(oracle, X, k, bits=8, dtype="f64"):
    got, b = run_engine(X, k, dtype)
    assert b == bits
    ref = oracle.knn(X.astype(np.float32).astype(np.float64) if dtype == "f32" else X, k)
    assert np.array_equal(got["idx"], ref["idx"])
    assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64))


def test_i8_mnist_like(oracle):
    check(oracle, datasets.mnist_like(3000, 784, seed=21)[0], 30)


def test_i8_sift_like_f32(oracle):
    check(oracle, datasets.sift_like(20000, 128), 32, dtype="f32")


def test_i8_digits(oracle):
    check(oracle, datasets.digits()[0], 30)


@pytest.mark.parametrize("n", [1, 17, 32, 33, 128, 129, 800, 896])
def test_i8_feature_counts(oracle, n):
    rng = np.random.default_rng(n)
    X = rng.integers(0, 256, (1500, n)).astype(np.float64)
    X[11] = X[5]                                   # an exact duplicate
    check(oracle, X, 30 if n > 1 else 8)


def test_i8_signed_window_boundary(oracle):
    # lo = -100, hi = 155: range exactly 255, the widest eligible window
    rng = np.random.default_rng(3)
    X = rng.integers(-100, 156, (2500, 100)).astype(np.float64)
    X[:10] = -100.0
    X[10:20] = 155.0
    X[300:340] = X[0]                              # a mass of duplicates
    check(oracle, X, 30)


def test_i8_not_taken(oracle):
    rng = np.random.default_rng(4)
    X = rng.integers(-100, 157, (1200, 100)).astype(np.float64)
    X[0, 0] = 156.0                                # range 256: fp16 instead
    check(oracle, X, 30, bits=16)
    X = rng.integers(0, 256, (600, 897)).astype(np.float64)   # n > 896
    check(oracle, X, 30, bits=16)


@pytest.mark.parametrize("k", [1, 2, 31, 32])
def test_i8_k_range_f64(oracle, k):
    X = datasets.mnist_like(2000, 64, seed=40 + k)[0]
    check(oracle, X, k)


@pytest.mark.parametrize("k", [17, 33, 64, 100, 128])
def test_i8_k_range_f32(oracle, k):
    check(oracle, datasets.sift_like(6000, 128), k, dtype="f32")


def test_i8_small_m(oracle):
    rng = np.random.default_rng(6)
    for m in (1, 5, 40, 127, 129):
        X = rng.integers(0, 256, (m, 50)).astype(np.float64)
        check(oracle, X, 30)


def test_i8_binary_ties(oracle):
    # huge tie sets at the k boundary: the lower index must win every tie
    rng = np.random.default_rng(7)
    X = rng.integers(0, 2, (3000, 20)).astype(np.float64)
    check(oracle, X, 32)


def test_i8_single_split(oracle, monkeypatch):
    monkeypatch.setenv("KNN_SPLITS", "1")
    check(oracle, datasets.mnist_like(4000, 784, seed=9)[0], 30)


def test_i8_matches_fp16_path(oracle, monkeypatch):
    X = datasets.mnist_like(2500, 784, seed=13)[0]
    a, b8 = run_engine(X, 30, "f64")
    monkeypatch.setenv("KNN_NO_I8", "1")
    b, b16 = run_engine(X, 30, "f64")
    assert (b8, b16) == (8, 16)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("kl", ["12", "17"])
@pytest.mark.parametrize("case", ["mnist", "digits", "dups", "sift"])
def test_i8_lane_list_lengths(oracle, monkeypatch, kl, case):
    """Both lane-list lengths of the k <= 32 kernel (12 by default, 17 with
    KNN_I8_KL=17): with 12 entries only the 4-lane bound applies (2 x 12 <
    k + 1) and the published bound must still sit at or below every list's
    last entry (a full list drops candidates there); heavy ties, mass
    duplicates and k = 32 over few lanes exercise that."""
    monkeypatch.setenv("KNN_I8_KL", kl)
    if case == "mnist":
        check(oracle, datasets.mnist_like(2500, 784, seed=31)[0], 30)
    elif case == "digits":
        check(oracle, datasets.digits()[0], 30)
    elif case == "dups":
        rng = np.random.default_rng(8)
        X = rng.integers(0, 4, (2000, 24)).astype(np.float64)   # massive ties
        check(oracle, X, 30)
    else:
        check(oracle, datasets.sift_like(8000, 128, clusters=16, seed=3), 32, dtype="f32")


@pytest.mark.parametrize("m,k", [(1000, 32), (777, 10)])
def test_i8_two_query_groups_match_one(oracle, monkeypatch, m, k):
    """Rows of <= 4 K-steps run two query groups a wave (256-query
    workgroups, knn_i8_qg): a partial last block of 256 queries, bit-exact
    vs the oracle and byte-identical to the one-group kernel
    (KNN_I8_QG1=1)."""
    X = datasets.sift_like(m, 128).astype(np.float64)
    check(oracle, X, k)
    got2, _ = run_engine(X, k, "f64")
    monkeypatch.setenv("KNN_I8_QG1", "1")
    got1, b = run_engine(X, k, "f64")
    assert b == 8
    assert got1.tobytes() == got2.tobytes()
