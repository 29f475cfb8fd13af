"""Bug-compatible mode (include/knn.h knn_search_mpi_compat).

CPU: oracle.mpi_compat (the block-fold restatement) against a literal
pure-Python replay of mpi-knn-parallel_blocking.c's data movement on tiny
inputs -- (n+2)-strided matrices, the short first hop (blk:130-146),
matrix_send's feature-only copy (blk:169,231), the ring (blk:187-244) and
the strict-< insert + stable distance-only sort (blk:24-31,172-178).
GPU: libknn's compat search against oracle.mpi_compat, bit-exact.
Parity with the reference binaries themselves is unpinned: their neighbour
dumps are not in the container.
"""
import math

import numpy as np
import pytest

import datasets


def literal_blocking(X, labels, P, NN):
    """Replay of blk:81-244 for P ranks (host memory of every rank)."""
    m, n = X.shape
    R = m // P
    W = n + 2
    matrix = [[0.0] * (R * W) for _ in range(P)]
    for r in range(P):
        for k in range(R):
            for i in range(n):
                matrix[r][k * W + i] = float(X[k + r * R, i])      # blk:104 (col-major read)
            matrix[r][k * W + n] = float(k + r * R + 1)            # blk:107
            matrix[r][k * W + n + 1] = float(labels[k + r * R])    # blk:108
    temp = [[0.0] * (R * W) for _ in range(P)]
    for r in range(P):                                             # blk:122-147: R*n doubles
        src = matrix[(r - 1) % P]
        temp[r][:R * n] = src[:R * n]
    send = [[0.0] * (R * W) for _ in range(P)]
    lists = [[[(math.inf, 0, 0)] * NN for _ in range(R)] for _ in range(P)]

    def fold(r, blk):
        for k in range(R):
            L = lists[r][k]
            for i in range(R):
                S = 0.0
                for j in range(n):
                    t = matrix[r][k * W + j] - blk[i * W + j]
                    S = S + t * t
                    send[r][i * W + j] = temp[r][i * W + j]        # blk:169 / 231
                d = math.sqrt(S)
                if d < L[NN - 1][0] and d != 0:
                    L[NN - 1] = (d, int(blk[i * W + n]), int(blk[i * W + n + 1]))
                    L.sort(key=lambda e: e[0])                     # stable, distance only

    for r in range(P):
        fold(r, matrix[r])                                         # blk:155-181: own block
    for _ in range(P - 1):                                         # blk:187-244
        new_temp = [list(send[(r - 1) % P]) for r in range(P)]
        for r in range(P):
            temp[r] = new_temp[r]
        for r in range(P):
            fold(r, temp[r])
    return lists


def as_arrays(lists):
    d = np.array([[e[0] for e in row] for rk in lists for row in rk])
    i = np.array([[e[1] for e in row] for rk in lists for row in rk])
    lab = np.array([[e[2] for e in row] for rk in lists for row in rk])
    return d, i, lab


@pytest.mark.parametrize("P,m,n,kind", [(2, 14, 3, "int"), (3, 20, 5, "int"), (4, 23, 2, "int"),
                                       (3, 19, 4, "real"), (2, 12, 1, "int")])
def test_oracle_compat_matches_literal_replay(oracle, P, m, n, kind):
    rng = np.random.default_rng(m * 10 + P)
    X = rng.integers(0, 4, (m, n)).astype(np.float64) if kind == "int" else rng.normal(0, 1, (m, n))
    X[5] = X[1]                                                   # an exact duplicate
    labels = rng.integers(1, 11, m).astype(np.float64)
    NN = 6
    got = oracle.mpi_compat(X, NN, P, labels=labels)
    d, i, lab = as_arrays(literal_blocking(X, labels, P, NN))
    assert np.array_equal(got["distance"], d)
    assert np.array_equal(got["idx"], i)
    assert np.array_equal(got["label"], lab)


def test_oracle_compat_shape_facts(oracle):
    X, y = datasets.digits()
    P = 4
    nb = oracle.mpi_compat(X, 30, P, labels=y)
    R = X.shape[0] // P
    assert nb.shape == (P * R, 30)
    for r in range(P):
        ids = nb["idx"][r * R:(r + 1) * R]
        real = ids[ids > 0]
        # only the own block ever carries real ids (F5)
        assert real.min() >= r * R + 1 and real.max() <= (r + 1) * R
        assert (ids == 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_gpu_compat_digits(knn, oracle, P):
    X, y = datasets.digits()
    got, _ = knn.search_mpi_compat(X, 30, P, labels=y, layout="col")
    ref = oracle.mpi_compat(X, 30, P, labels=y)
    assert np.array_equal(got["idx"], ref["idx"])
    assert np.array_equal(got["label"], ref["label"])
    assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64))


@pytest.mark.gpu
def test_gpu_compat_real_and_mnist(knn, oracle):
    for X, P in ((datasets.digits_real()[0], 3), (datasets.mnist_like(2000, 784, seed=3)[0], 4)):
        got, _ = knn.search_mpi_compat(X, 30, P)
        ref = oracle.mpi_compat(X, 30, P)
        assert np.array_equal(got["idx"], ref["idx"])
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64))
