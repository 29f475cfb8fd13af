"""The CPU oracle (oracle/knn_oracle.c) against the reference-run pins.

The reference cannot be built here (it needs MATLAB's mat.h / libmat /
libmx), so the restatement is pinned by the numbers SURVEY.md records from
the compiled reference (sec.0 F1/F7, sec.4): sklearn digits -> serial vote
Matches 1636, MPI tie rule 1635, true majority 1742, 106 queries with an
exact distance tie at the k = 30 boundary; the real-valued digits variant ->
1631.  Plus internal consistency: the literal "overwrite slot NN-1 + glibc
qsort" form (serial:86-91) equals the stable insertion, and folding blocks
in any order (the ring) equals the serial scan.
"""
import numpy as np
import pytest

import datasets


def test_digits_pins(oracle):
    X, y = datasets.digits()
    nb = oracle.knn(X, 30, labels=y)
    assert oracle.classify(nb, y, 10, oracle.VOTE_SERIAL)[1] == 1636
    assert oracle.classify(nb, y, 10, oracle.VOTE_MPI)[1] == 1635
    assert oracle.classify(nb, y, 10, oracle.VOTE_MAJORITY)[1] == 1742
    nb31 = oracle.knn(X, 31)
    assert int((nb31["distance"][:, 29] == nb31["distance"][:, 30]).sum()) == 106


def test_digits_real_pin(oracle):
    X, y = datasets.digits_real()
    nb = oracle.knn(X, 30, labels=y)
    assert oracle.classify(nb, y, 10, oracle.VOTE_SERIAL)[1] == 1631
    # F4: an exact duplicate is excluded like the point itself
    assert 1798 not in nb["idx"][0] and 1 not in nb["idx"][1797]


def test_literal_qsort_equals_stable_insertion(oracle):
    X, _ = datasets.digits()
    a = oracle.knn(X, 30, literal=False)
    b = oracle.knn(X, 30, literal=True, layout="col")
    assert np.array_equal(a, b)


def test_vote_quirk_vectors(oracle):
    """16 x label 1 + 14 x label 9 -> 9 with the reference rule."""
    labels = np.array([1.0] * 16 + [9.0] * 14 + [1.0], dtype=np.float64)  # row 31 is the query
    nb = np.zeros((1, 30), dtype=oracle.NB_DTYPE)
    nb["idx"][0] = np.arange(1, 31)
    nb["distance"][0] = np.arange(1, 31)
    pred, _ = oracle.classify(nb, labels, 10, oracle.VOTE_SERIAL, q0=30)
    assert pred[0] == 9
    pred, _ = oracle.classify(nb, labels, 10, oracle.VOTE_MAJORITY, q0=30)
    assert pred[0] == 1


def test_distance_is_reference_arithmetic(oracle):
    # S accumulates (a-b)^2 in j order with two roundings per term (no FMA)
    rng = np.random.default_rng(11)
    X = rng.normal(0, 1, (50, 33))
    nb = oracle.knn(X, 5)
    for q in range(0, 50, 7):
        i = nb["idx"][q, 0] - 1
        S = 0.0
        for j in range(33):
            t = X[q, j] - X[i, j]
            S = S + t * t
        assert nb["distance"][q, 0] == np.sqrt(S)


@pytest.mark.parametrize("P", [2, 3, 5])
def test_block_folding_any_order(oracle, P):
    X, _ = datasets.digits_real()
    m = X.shape[0]
    full = oracle.knn(X, 30)
    R = -(-m // P)
    rng = np.random.default_rng(P)
    for g in range(P):
        q0, q1 = g * R, min(m, (g + 1) * R)
        lists = oracle.lists_init(q1 - q0, 30)
        for b in rng.permutation(P):
            c0, c1 = b * R, min(m, (b + 1) * R)
            oracle.knn_block(X[q0:q1], q0, X[c0:c1], c0, lists)
        assert np.array_equal(lists[["distance", "idx"]], full[q0:q1][["distance", "idx"]])


def test_oracle_f32_entry_equals_f64_scan(oracle):
    """orc_knn_rows_f32 (configs[4]'s checker, no 8-byte copy of the
    corpus) is orc_knn_rows on the widened values, bit for bit."""
    rng = np.random.default_rng(17)
    X = rng.random((2500, 96)).astype(np.float32)
    X[9] = X[4]                                    # an exact duplicate
    a = oracle.knn_f32(X, 100, (0, 64))
    b = oracle.knn(X.astype(np.float64), 100, rows=(0, 64))
    assert a.tobytes() == b.tobytes()
