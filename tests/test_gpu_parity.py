"""GPU parity: libknn (HIP, gfx950) vs the CPU oracle on the same inputs.

The bar: neighbour indices bit-exact and distances
bit-exact (the reference's own fp64 sqrt(S), S accumulated in j order
without FMA) for every engine mode -- integer data (exact GEMM form),
real-valued data (GEMM filter + exact re-rank), non-finite data (exact
scan) -- and for every block count of the ring.
"""
import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu


def assert_same(got, ref, what=""):
    assert got.shape == ref.shape, what
    bad_i = np.nonzero(got["idx"] != ref["idx"])
    assert bad_i[0].size == 0, "%s: %d idx mismatches, first at %s: got %s ref %s" % (
        what, bad_i[0].size, (bad_i[0][0], bad_i[1][0]), got[bad_i[0][0]][:8], ref[bad_i[0][0]][:8])
    gd = got["distance"].view(np.uint64)
    rd = ref["distance"].view(np.uint64)
    nd = int((gd != rd).sum())
    assert nd == 0, "%s: %d distance bit mismatches" % (what, nd)


def test_digits_integer_mode(knn, oracle):
    X, y = datasets.digits()
    ref = oracle.knn(X, 30, labels=y)
    got, _ = knn.search(X, 30, labels=y)
    assert_same(got, ref, "digits")
    # pinned to the reference's own run
    assert knn.classify(got, y, 10, knn.VOTE_SERIAL)[1] == 1636
    assert knn.classify(got, y, 10, knn.VOTE_MPI)[1] == 1635
    assert knn.classify(got, y, 10, knn.VOTE_MAJORITY)[1] == 1742


def test_digits_colmajor_layout(knn, oracle):
    X, y = datasets.digits()
    ref = oracle.knn(X, 30)
    got, _ = knn.search(X, 30, layout="col")
    assert_same(got, ref, "digits col-major")


def test_digits_real_gemm_mode(knn, oracle):
    X, y = datasets.digits_real()
    ref = oracle.knn(X, 30, labels=y)
    got, _ = knn.search(X, 30, labels=y)
    assert_same(got, ref, "digits_real")
    assert knn.classify(got, y, 10, knn.VOTE_SERIAL)[1] == 1631


@pytest.mark.parametrize("m,n,k", [(3000, 784, 30), (1000, 100, 30), (700, 17, 5), (300, 1, 30)])
def test_mnist_like_integer(knn, oracle, m, n, k):
    X, y = datasets.mnist_like(m, n, seed=m + n)
    ref = oracle.knn(X, k)
    got, _ = knn.search(X, k)
    assert_same(got, ref, "mnist_like %dx%d k=%d" % (m, n, k))


@pytest.mark.parametrize("m,n", [(2000, 64), (513, 200), (129, 3)])
def test_gaussian_real(knn, oracle, m, n):
    rng = np.random.default_rng(m * 7 + n)
    X = rng.normal(0, 1, (m, n))
    ref = oracle.knn(X, 30)
    got, _ = knn.search(X, 30)
    assert_same(got, ref, "gaussian %dx%d" % (m, n))


@pytest.mark.parametrize("k", [1, 2, 31, 32])
def test_k_range_fp64(knn, oracle, k):
    """k from 1 to KNN_MAX_K in both exact modes, with duplicate rows (S == 0
    entries beside the merge's exact-S window) in the real-valued case."""
    X, _ = datasets.digits()
    X = np.vstack([X, X[:30], X[:30]])
    assert_same(knn.search(X, k)[0], oracle.knn(X, k), "digits+dups k=%d" % k)
    Xr = X / 7.0 + 0.001
    assert_same(knn.search(Xr, k)[0], oracle.knn(Xr, k), "real+dups k=%d" % k)


def test_fewer_rows_than_k(knn, oracle):
    X = np.arange(40, dtype=np.float64).reshape(10, 4)
    ref = oracle.knn(X, 30)
    got, _ = knn.search(X, 30)
    assert_same(got, ref, "m<k")
    assert (got["idx"][:, 9:] == 0).all() and np.isinf(got["distance"][:, 9:]).all()


def test_single_row(knn, oracle):
    X = np.ones((1, 5))
    got, _ = knn.search(X, 3)
    assert (got["idx"] == 0).all() and np.isinf(got["distance"]).all()


def test_duplicates_excluded(knn, oracle):
    X, _ = datasets.digits()
    X = np.vstack([X, X[:50], X[:50]])  # two extra copies of 50 rows
    ref = oracle.knn(X, 30)
    got, _ = knn.search(X, 30)
    assert_same(got, ref, "duplicates (int)")
    Xr = X / 7.0 + 0.001
    ref = oracle.knn(Xr, 30)
    got, _ = knn.search(Xr, 30)
    assert_same(got, ref, "duplicates (real)")


def test_heavy_ties(knn, oracle):
    # tiny integer alphabet: huge numbers of exact distance ties
    rng = np.random.default_rng(5)
    X = rng.integers(0, 2, (1500, 12)).astype(np.float64)
    ref = oracle.knn(X, 30)
    got, _ = knn.search(X, 30)
    assert_same(got, ref, "binary ties")


def test_nonfinite_scan_mode(knn, oracle):
    rng = np.random.default_rng(3)
    X = rng.normal(0, 1, (400, 20))
    X[5, 3] = np.nan
    X[17, 0] = np.inf
    ref = oracle.knn(X, 30)
    got, _ = knn.search(X, 30)
    assert_same(got, ref, "nan/inf")


def test_ring_blocks_match_single_device(knn, oracle):
    """The ring's per-rank work simulated on one GPU: for every block count
    each rank's lists equal the oracle's serial scan of its rows."""
    import torch
    import mpiknn.ring as ring

    for X in (datasets.mnist_like(2500, 784, seed=9)[0], datasets.digits_real()[0]):
        m, n = X.shape
        dev = torch.device("cuda", 0)
        Xd = torch.from_numpy(X).to(dev)
        for P in (2, 3, 8):
            R, blocks = ring.partition(m, P)
            engines = []
            for g in range(P):
                base, rows = blocks[g]
                e = ring.GpuEngine(torch, 0, n, R, rows, 30)
                e.pack(Xd[base:base + rows], layout_col=False, elements=True)
                engines.append(e)
            meta = torch.stack([e.meta for e in engines]).max(dim=0).values
            for g, e in enumerate(engines):
                e.meta.copy_(meta)
                base, rows = blocks[g]
                e.begin(base)
                for s in range(P):
                    b = (g - s) % P
                    e.step(engines[b].qb, blocks[b][1], blocks[b][0])
                u = e.end()
                if u:
                    for s in range(P):
                        b = (g - s) % P
                        e.step(engines[b].qb, blocks[b][1], blocks[b][0], rescan=True)
                    e.rescan_end()
                got = e.result()
                assert_same(got, oracle.knn(X, 30, rows=(base, rows)), "ring P=%d rank %d" % (P, g))


@pytest.mark.parametrize("schedule", ["ring", "direct", "direct-all", "ring-element"])
@pytest.mark.parametrize("P", [2, 3, 4, 8, 11])
@pytest.mark.parametrize("force_rescan", [False, True])
def test_ring_driver_loopback(knn, oracle, monkeypatch, P, force_rescan, schedule):
    """knn_ring.c's P >= 2 schedules with its loopback transport: P virtual
    ranks on device 0, every transfer a device copy on one fabric stream.
    "ring": ring_pass / ring_hop, the receive-buffer rotation and the rescan
    rotation; "direct": the all-at-once exchange and the fused fold of the
    received byte blocks (P = 11: launches of 8 + 2; "direct-all" with the
    own block in the fused launch); these move the search's shadow form,
    "ring-element" element blocks.  KNN_FORCE_RESCAN=1 sends
    every query through the exact rescan pass, so its element-block pass is
    checked too.  Against the oracle."""
    monkeypatch.setenv("KNN_RING_LOOPBACK", "1")
    monkeypatch.setenv("KNN_RING_SCHEDULE", "ring" if schedule.startswith("ring") else "direct")
    if schedule == "direct-all":
        monkeypatch.setenv("KNN_RING_FUSE", "all")
    if schedule == "ring-element":
        monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    if force_rescan:
        monkeypatch.setenv("KNN_FORCE_RESCAN", "1")
    for X in (datasets.mnist_like(1500, 784, seed=4)[0], datasets.digits_real()[0]):
        ref = oracle.knn(X, 30)
        got, _ = knn.search(X, 30, ngpus=P, layout="col")
        assert_same(got, ref, "loopback ring P=%d" % P)
    X = datasets.sift_like(3000, 128)
    ref = oracle.knn(X.astype(np.float32).astype(np.float64), 32)
    got, _ = knn.search(X, 32, ngpus=P, dtype="f32")
    assert_same(got, ref, "loopback ring f32 P=%d" % P)


def test_ring_driver_more_procs_than_gpus(knn, oracle):
    """The reference's `mpi-knn-parallel_blocking 4 4` on a box with fewer
    GPUs: knn_search runs on the GPUs present (results do not depend on the
    block count); m=9 with P=4 (an empty ceil-block) runs too."""
    X = datasets.mnist_like(1000, 784, seed=2)[0]
    got, _ = knn.search(X, 30, ngpus=64)
    assert_same(got, oracle.knn(X, 30), "ngpus=64")
    X9 = datasets.mnist_like(9, 20, seed=3)[0]
    got, _ = knn.search(X9, 5, ngpus=4)
    assert_same(got, oracle.knn(X9, 5), "m=9 P=4")


def test_rccl_ring_driver_one_gpu(knn, oracle, monkeypatch):
    """knn_ring.c (ncclCommInitAll, meta ncclAllReduce, ring passes) on the
    GPUs present; with KNN_FORCE_RING=1 it runs even for one GPU."""
    import torch
    ng = torch.cuda.device_count()
    monkeypatch.setenv("KNN_FORCE_RING", "1")
    for X in (datasets.mnist_like(1500, 784, seed=4)[0], datasets.digits_real()[0]):
        ref = oracle.knn(X, 30)
        for p in sorted({1, ng}):
            got, _ = knn.search(X, 30, ngpus=p, layout="col")
            assert_same(got, ref, "rccl ring P=%d" % p)


@pytest.mark.parametrize("what", ["fp64-int-no-i8", "real-split", "fp32-sift", "real-no-split"])
def test_xcd_grouped_order(knn, oracle, monkeypatch, what):
    """KNN_XCD_ORDER=1: the XCD-grouped workgroup order of k_dist_topk and
    k_dist_split (the split-major order is the default)
    gives the same lists -- the order only moves which workgroup folds which
    (query block, split), never the result (knn-serial.c:72-93)."""
    monkeypatch.setenv("KNN_XCD_ORDER", "1")
    if what == "fp64-int-no-i8":
        monkeypatch.setenv("KNN_NO_I8", "1")
        X = datasets.mnist_like(2000, 784, seed=21)[0]
        got, _ = knn.search(X, 30)
        ref = oracle.knn(X, 30)
    elif what in ("real-split", "real-no-split"):
        if what == "real-no-split":
            monkeypatch.setenv("KNN_NO_SPLIT", "1")
        X = datasets.digits_real()[0]
        got, _ = knn.search(X, 30)
        ref = oracle.knn(X, 30)
    else:
        monkeypatch.setenv("KNN_NO_I8", "1")
        X = datasets.sift_like(4000, 128)
        got, _ = knn.search(X, 32, dtype="f32")
        ref = oracle.knn(X.astype(np.float32).astype(np.float64), 32)
    assert_same(got, ref, "xcd order %s" % what)
