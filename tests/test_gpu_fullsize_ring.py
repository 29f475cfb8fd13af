"""Multi-rank parity at the BASELINE configs' full sizes (configs[2], [3]).

knn_ring.c's P = 8 schedules run through its loopback transport (8 virtual
ranks on device 0, every transfer a device copy; the same buffers, events,
lag rule and fused launches as over RCCL).  Rank g folds the blocks of
mpi-knn-parallel_blocking.c:217-242 for its own query rows -- every block
once (the reference visits r, r-2, ..., r-P), so each rank's
rows must carry the serial lists of knn-serial.c:72-93:

* mnist_like(60000) x 784 (configs[2]) and its real-valued form (fp64 GEMM
  mode, element blocks on the wire): all 60000 rows against the oracle's
  committed per-row hashes, the 48 golden rows bit for bit, and the whole
  result byte-identical to the one-GPU search; the integer form once more
  with every transfer through RCCL (self-loop communicator);
* a SIFT-shaped 1M x 128 fp32 corpus (configs[3]): 16 rows spread over the
  eight ranks against the oracle's scan.

Plus k_merge's two INT-mode argmin forms: packed (d^2 << 32 |
idx) keys when 4 max|x|^2 < 2^32, the (d^2, idx) double pair above it --
both on tie-heavy data against the oracle.
"""
import numpy as np
import pytest

import datasets
from test_golden import check_all_rows, check_mnist_rows, load
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _props(nb, m):
    d = nb["distance"]
    assert np.all(d[:, 1:] >= d[:, :-1]) and np.all(d > 0)
    assert not np.any(nb["idx"] == np.arange(1, m + 1)[:, None])


@pytest.mark.parametrize("schedule", ["direct", "ring"])
def test_mnist_full_size_p8_loopback(knn, monkeypatch, schedule):
    X, _ = datasets.mnist_like(60000)
    Xf = np.asfortranarray(X)
    one, _ = knn.search(Xf, 30, layout="col")
    monkeypatch.setenv("KNN_RING_LOOPBACK", "1")
    monkeypatch.setenv("KNN_RING_SCHEDULE", schedule)
    nb, _ = knn.search(Xf, 30, ngpus=8, layout="col")
    check_mnist_rows(nb[load("mnist_like_sample.npz")["rows"]], load("mnist_like_sample.npz"))
    check_all_rows(nb, "mnist_like")
    _props(nb, 60000)
    assert nb.tobytes() == one.tobytes(), "P=8 %s differs from the one-GPU search" % schedule


def test_mnist_full_size_p8_rccl_self(knn, monkeypatch):
    """configs[2] at full size with every transfer through RCCL (the
    one-device self-loop communicator of knn_ring.c, P = 8 virtual ranks):
    all 60000 rows against the oracle's per-row hashes"""
    X, _ = datasets.mnist_like(60000)
    monkeypatch.setenv("KNN_RING_LOOPBACK", "rccl")
    monkeypatch.setenv("KNN_RING_SCHEDULE", "direct")
    nb, _ = knn.search(np.asfortranarray(X), 30, ngpus=8, layout="col")
    check_all_rows(nb, "mnist_like")


def test_mnist_real_full_size_p8_loopback(knn, monkeypatch):
    X, _ = datasets.mnist_real(60000)
    Xf = np.asfortranarray(X)
    one, _ = knn.search(Xf, 30, layout="col")
    monkeypatch.setenv("KNN_RING_LOOPBACK", "1")
    monkeypatch.setenv("KNN_RING_SCHEDULE", "direct")
    nb, _ = knn.search(Xf, 30, ngpus=8, layout="col")
    g = load("mnist_real_sample.npz")
    assert np.array_equal(nb[g["rows"]]["idx"], g["idx"])
    assert np.array_equal(nb[g["rows"]]["distance"].view(np.uint64), g["dist_bits"])
    check_all_rows(nb, "mnist_real")
    _props(nb, 60000)
    assert nb.tobytes() == one.tobytes()


def test_sift_full_size_p8_loopback(knn, oracle, monkeypatch):
    X = datasets.sift_like(1_000_000, 128)
    monkeypatch.setenv("KNN_RING_LOOPBACK", "1")
    monkeypatch.setenv("KNN_RING_SCHEDULE", "direct")
    nb, _ = knn.search(X, 32, ngpus=8, dtype="f32")
    R = 125000
    rows = [g * R + o for g in range(8) for o in (0, 77777 % R)]
    X64 = X.astype(np.float32).astype(np.float64)
    for r in rows:
        assert_same(nb[r:r + 1], oracle.knn(X64, 32, rows=(r, 1)), "sift P=8 row %d" % r)
    d = nb["distance"]
    assert np.all(d[:, 1:] >= d[:, :-1]) and np.all(d > 0)


@pytest.mark.parametrize("amp,packed", [(8000, True), (20000, False)])
def test_merge_argmin_forms_on_ties(knn, oracle, amp, packed):
    """INT-mode fp64 data outside the int8/fp16 windows (fp64 MFMA
    contraction): values in {-amp, 0, amp}, n = 16, so distances repeat
    thousands of times.  amp = 8000: 4 max|x|^2 = 4.1e9 < 2^32, the packed
    u64 argmin; amp = 20000: d^2 up to 2.56e10 > 2^32, the double pair."""
    rng = np.random.default_rng(11)
    X = rng.choice(np.array([-amp, 0.0, amp]), size=(3000, 16))
    assert (4 * (X * X).sum(1).max() < 2 ** 32) == packed
    got, _ = knn.search(X, 30)
    assert_same(got, oracle.knn(X, 30), "amp %d" % amp)
