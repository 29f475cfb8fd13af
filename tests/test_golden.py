"""Committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle reproduces the reference-run aggregates (reference_runs.json,
SURVEY.md sec.0/sec.4) and the committed neighbour fixtures.  GPU: libknn
through the C ABI reproduces the same fixtures bit for bit -- digits (integer
mode), the real-valued digits variant (GEMM filter + exact re-rank) and 48
sampled queries of the full 60000x784 MNIST-shaped corpus (configs[1]), in
its integer form and its real-valued form (SURVEY C1's svd variant is
real-valued: GEMM mode on the split-fp16 filter plus the exact fp64 re-rank,
at full size) -- and, at that size, every one of the 60000 rows against the
oracle's committed per-row hashes (*_rowhash.npz).
"""
import json
import os
import sys

import numpy as np
import pytest

import datasets

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
if GOLD not in sys.path:
    sys.path.insert(0, GOLD)
from rowhash import row_hashes  # noqa: E402  (the hash make_golden.py committed)


def load(name):
    with np.load(os.path.join(GOLD, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def runs():
    with open(os.path.join(GOLD, "reference_runs.json")) as f:
        return json.load(f)


def check_digits(nb, g):
    assert np.array_equal(nb["idx"], g["idx"].astype(np.int32))
    assert np.array_equal(nb["distance"], np.sqrt(g["d2"].astype(np.float64)))


def check_digits_real(nb, g):
    assert np.array_equal(nb["idx"], g["idx"].astype(np.int32))
    assert np.array_equal(nb["distance"].view(np.uint64), g["dist_bits"])


def check_mnist_rows(nb_rows, g):
    assert np.array_equal(nb_rows["idx"], g["idx"])
    assert np.array_equal(nb_rows["distance"], np.sqrt(g["d2"].astype(np.float64)))


def check_all_rows(nb, name):
    """every row of a full-size (60000, 30) result against the oracle's
    per-row hashes (`name`: "mnist_like" or "mnist_real"): knn-serial.c:72-93
    for all 60000 queries, not only the sampled ones"""
    g = load("%s_rowhash.npz" % name)
    assert nb.shape == (int(g["m"]), int(g["k"])), nb.shape
    bad = np.flatnonzero(row_hashes(nb) != g["hash"])
    assert bad.size == 0, "%d of %d rows differ from the oracle (first: %s)" % (bad.size, len(nb), bad[:8])


def test_oracle_reference_runs(oracle):
    r = runs()
    X, y = datasets.digits()
    nb = oracle.knn(X, 30)
    assert oracle.classify(nb, y, 10, oracle.VOTE_SERIAL)[1] == r["digits"]["matches_serial_rule"]
    assert oracle.classify(nb, y, 10, oracle.VOTE_MPI)[1] == r["digits"]["matches_mpi_rule"]
    assert oracle.classify(nb, y, 10, oracle.VOTE_MAJORITY)[1] == \
        r["digits"]["matches_true_majority"]
    Xr, yr = datasets.digits_real()
    nbr = oracle.knn(Xr, 30)
    assert oracle.classify(nbr, yr, 10, oracle.VOTE_SERIAL)[1] == \
        r["digits_real"]["matches_serial_rule"]


def test_oracle_matches_fixtures(oracle):
    X, y = datasets.digits()
    nb = oracle.knn(X, 30)
    g = load("digits_k30.npz")
    check_digits(nb, g)
    pred, _ = oracle.classify(nb, y, 10, oracle.VOTE_SERIAL)
    assert np.array_equal(np.asarray(pred), g["pred"].astype(np.asarray(pred).dtype))
    check_digits_real(oracle.knn(datasets.digits_real()[0], 30), load("digits_real_k30.npz"))


@pytest.mark.parametrize("name", ["mnist_like", "mnist_real"])
def test_oracle_matches_rowhash(oracle, name):
    """the committed per-row hashes against the oracle on a spread of rows
    (the CPU check of the fixture the GPU tests compare all rows with)"""
    X, _ = getattr(datasets, name)(60000)
    g = load("%s_rowhash.npz" % name)
    rows = np.unique(np.concatenate([[0, 1, 59999], np.arange(7, 60000, 4999)]))
    got = np.concatenate([oracle.knn(X, 30, rows=(int(r), 1)) for r in rows])
    assert np.array_equal(row_hashes(got), g["hash"][rows])
    # the 48 sampled fixture rows hash to the same entries
    s = load("%s_sample.npz" % name)
    nb = np.zeros(s["idx"].shape, dtype=oracle.NB_DTYPE)
    nb["idx"] = s["idx"]
    nb["distance"] = (np.sqrt(s["d2"].astype(np.float64)) if "d2" in s else s["dist_bits"].view(np.float64))
    assert np.array_equal(row_hashes(nb), g["hash"][s["rows"]])


def test_oracle_matches_mnist_sample(oracle):
    g = load("mnist_like_sample.npz")
    X, _ = datasets.mnist_like(60000)
    rows = g["rows"][::6]                        # a subset keeps the CPU suite quick
    got = np.concatenate([oracle.knn(X, 30, rows=(int(r), 1)) for r in rows])
    check_mnist_rows(got, {"idx": g["idx"][::6], "d2": g["d2"][::6]})


@pytest.mark.gpu
def test_gpu_digits_fixture(knn):
    X, y = datasets.digits()
    nb, _ = knn.search(X, 30)
    g = load("digits_k30.npz")
    check_digits(nb, g)
    pred, matches = knn.classify(nb, y, 10, knn.VOTE_SERIAL)
    assert matches == runs()["digits"]["matches_serial_rule"]
    assert np.array_equal(np.asarray(pred), g["pred"].astype(np.asarray(pred).dtype))


@pytest.mark.gpu
def test_gpu_digits_real_fixture(knn):
    nb, _ = knn.search(datasets.digits_real()[0], 30)
    check_digits_real(nb, load("digits_real_k30.npz"))


@pytest.mark.gpu
def test_gpu_mnist_full_size_fixture(knn):
    """configs[1] at full size (60000x784 fp64, k=30, col-major like the
    .mat); the 48 committed rows are compared bit-exact."""
    X, _ = datasets.mnist_like(60000)
    nb, _ = knn.search(np.asfortranarray(X), 30, layout="col")
    g = load("mnist_like_sample.npz")
    check_mnist_rows(nb[g["rows"]], g)
    check_all_rows(nb, "mnist_like")
    # size-independent properties over all 60000 rows: sorted, no self, no S=0
    d = nb["distance"]
    assert np.all(d[:, 1:] >= d[:, :-1]) and np.all(d > 0)
    assert not np.any(nb["idx"] == np.arange(1, 60001)[:, None])


@pytest.mark.gpu
def test_gpu_mnist_single_split_rescan(knn, monkeypatch):
    """One corpus split (KNN_SPLITS=1) leaves ~0.7% of the MNIST-shaped
    queries uncertified, so they take the exact rescan,
    chunked over the corpus (k_rescan_step grid.y + k_rescan_merge).  The
    result must be byte-identical to the default split count's."""
    X, _ = datasets.mnist_like(60000)
    base, _ = knn.search(X, 30)
    monkeypatch.setenv("KNN_SPLITS", "1")
    one, _ = knn.search(X, 30)
    assert base.tobytes() == one.tobytes()
    g = load("mnist_like_sample.npz")
    check_mnist_rows(one[g["rows"]], g)
    check_all_rows(one, "mnist_like")


def test_oracle_matches_mnist_real_sample(oracle):
    g = load("mnist_real_sample.npz")
    X, _ = datasets.mnist_real(60000)
    rows = g["rows"][::12]
    got = np.concatenate([oracle.knn(X, 30, rows=(int(r), 1)) for r in rows])
    assert np.array_equal(got["idx"], g["idx"][::12])
    assert np.array_equal(got["distance"].view(np.uint64), g["dist_bits"][::12])


@pytest.mark.gpu
def test_gpu_mnist_real_full_size_fixture(knn):
    """The real-valued 60000x784 corpus at full size through the C ABI (fp64
    GEMM mode: the split-fp16 filter k_dist_split, exact fp64 re-rank in
    k_merge, certificate): the 48 committed rows bit-exact (indices and
    distance bits), and every row against its committed hash."""
    X, _ = datasets.mnist_real(60000)
    nb, _ = knn.search(np.asfortranarray(X), 30, layout="col")
    g = load("mnist_real_sample.npz")
    got = nb[g["rows"]]
    assert np.array_equal(got["idx"], g["idx"])
    assert np.array_equal(got["distance"].view(np.uint64), g["dist_bits"])
    check_all_rows(nb, "mnist_real")
    d = nb["distance"]
    assert np.all(d[:, 1:] >= d[:, :-1]) and np.all(d > 0)


@pytest.mark.parametrize("name", ["mnist_like", "mnist_real"])
def test_bench_corpus_is_the_fixture_corpus(name):
    """bench.py's synthetic corpus (mpiknn/synth.py) is the one the row-hash
    fixtures were made from (tests/datasets.py), so its check_all_rows holds
    the bench's result to the oracle's"""
    from mpiknn import synth
    a, ya = getattr(synth, name)(60000)
    b, yb = getattr(datasets, name)(60000)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)) and np.array_equal(ya, yb)
