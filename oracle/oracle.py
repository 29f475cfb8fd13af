"""ctypes front-end of the CPU oracle (oracle/libknn_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  See
knn_oracle.h for what it restates and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libknn_oracle.so")

NB_DTYPE = np.dtype([("distance", "<f8"), ("idx", "<i4"), ("label", "<i4")])
COLMAJOR, ROWMAJOR = 0, 1
VOTE_SERIAL, VOTE_MPI, VOTE_MAJORITY = 0, 1, 2

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        p, sz, i, d = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
        L.orc_knn_rows.argtypes = [p, sz, sz, i, p, sz, sz, i, i, i, p]
        L.orc_knn_rows.restype = i
        L.orc_knn_rows_f32.argtypes = [p, sz, sz, p, sz, i, i, p]
        L.orc_knn_rows_f32.restype = i
        L.orc_knn_block.argtypes = [p, sz, sz, p, sz, sz, sz, p, i, i, p]
        L.orc_knn_block.restype = i
        L.orc_lists_init.argtypes = [p, sz, i]
        L.orc_lists_init.restype = None
        L.orc_classify.argtypes = [p, sz, sz, i, i, i, p, p]
        L.orc_classify.restype = ctypes.c_long
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def knn(X, k=30, labels=None, rows=None, literal=False, nthreads=0, layout="row"):
    """All-kNN with the reference's serial semantics (serial:57-93).

    X: (m, n) float64 array (row-major in memory unless layout="col", in which
    case X is the column-major buffer of an (m, n) matrix given as its (n, m)
    transpose view is NOT assumed: pass a Fortran-ordered array).
    rows: optional (q0, nq) query range.  Returns a structured array (nq, k).
    """
    X = np.asarray(X, dtype=np.float64)
    m, n = X.shape
    if layout == "col":
        buf = np.asfortranarray(X)
        lay = COLMAJOR
    else:
        buf = np.ascontiguousarray(X)
        lay = ROWMAJOR
    q0, nq = rows if rows is not None else (0, m)
    out = np.zeros((nq, k), dtype=NB_DTYPE)
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.float64)
    rc = lib().orc_knn_rows(_ptr(buf), m, n, lay, _ptr(lab), q0, nq, k,
                            int(bool(literal)), nthreads, _ptr(out))
    if rc:
        raise RuntimeError("orc_knn_rows failed rc=%d" % rc)
    return out


def knn_f32(X, k, rows, nthreads=0):
    """knn() of X.astype(float64) for a row-major float32 X without the
    float64 copy (orc_knn_rows_f32; the checker of the fp32 path at
    configs[4]'s size).  rows: (q0, nq) or a sequence of query row indices
    (one result row each, in that order)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    m, n = X.shape
    if isinstance(rows, tuple) and len(rows) == 2:
        qidx = np.arange(rows[0], rows[0] + rows[1], dtype=np.int64)
    else:
        qidx = np.ascontiguousarray(rows, dtype=np.int64)
    out = np.zeros((len(qidx), k), dtype=NB_DTYPE)
    rc = lib().orc_knn_rows_f32(_ptr(X), m, n, _ptr(qidx), len(qidx), k, nthreads, _ptr(out))
    if rc:
        raise RuntimeError("orc_knn_rows_f32 failed rc=%d" % rc)
    return out


def lists_init(nq, k):
    out = np.zeros((nq, k), dtype=NB_DTYPE)
    lib().orc_lists_init(_ptr(out), nq, k)
    return out


def knn_block(Q, q_base, C, c_base, lists, labels=None, nthreads=0):
    """Fold one corpus block into running lists (ring-step restatement)."""
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    C = np.ascontiguousarray(C, dtype=np.float64)
    assert lists.dtype == NB_DTYPE and lists.flags.c_contiguous
    nq, n = Q.shape
    nc = C.shape[0]
    k = lists.shape[1]
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.float64)
    rc = lib().orc_knn_block(_ptr(Q), nq, q_base, _ptr(C), nc, c_base, n,
                             _ptr(lab), k, nthreads, _ptr(lists))
    if rc:
        raise RuntimeError("orc_knn_block failed rc=%d" % rc)
    return lists


def mpi_compat(X, k=30, procs=2, labels=None):
    """What the reference MPI programs compute with `procs` ranks (SURVEY
    F5), restated from mpi-knn-parallel_blocking.c with the block fold above:

    * R = floor(m/procs) rows per rank, the remainder dropped (blk:81);
    * step 0 folds the rank's OWN block, real ids/labels (blk:155-181,
      matrix[i] not matrix_temp[i]; ids/labels blk:107-108);
    * the first hop sends R*n of R*(n+2) doubles (blk:130,137,146): the
      receiver's (n+2)-strided rows below q = R*n // (n+2) arrive whole,
      row q its first R*n - q*(n+2) doubles, later rows stay zero;
    * matrix_send copies only the n feature columns (blk:169,231): every
      forwarded block has id 0 / label 0 and keeps the truncation;
    * iteration p = 0..procs-2 (blk:187-244) folds block r-2-p.
    Ties keep scan order (strict <, stable distance-only qsort, blk:24-31):
    visits get scan-order ids (own block real ids, visit p m + p*R + row),
    then ids above m become idx 0 / label 0.
    """
    X = np.ascontiguousarray(X, dtype=np.float64)
    m, n = X.shape
    P = procs
    R = m // P
    out = np.zeros((P * R, k), dtype=NB_DTYPE)

    def trunc(b):
        B = X[b * R:(b + 1) * R].copy()
        sent, stride = R * n, n + 2
        q = sent // stride
        for i in range(q, R):
            got = sent - q * stride if i == q else 0
            B[i, min(got, n):] = 0.0
        return B

    for r in range(P):
        Q = X[r * R:(r + 1) * R]
        L = lists_init(R, k)
        knn_block(Q, r * R, Q, r * R, L)
        for p in range(P - 1):
            knn_block(Q, r * R, trunc((r - 2 - p) % P), m + p * R, L)
        fwd = L["idx"] > m
        L["idx"][fwd] = 0
        L["label"] = 0
        own = L["idx"] > 0
        if labels is not None:
            L["label"][own] = np.asarray(labels)[L["idx"][own] - 1].astype(np.int32)
        out[r * R:(r + 1) * R] = L
    return out


def classify(nb, labels, nclasses=10, rule=VOTE_SERIAL, q0=0):
    """Vote + Matches (serial:104-130 / blk:252-270).  Returns (pred, matches)."""
    nb = np.ascontiguousarray(nb)
    nq, k = nb.shape
    lab = np.ascontiguousarray(labels, dtype=np.float64)
    pred = np.zeros(nq, dtype=np.int32)
    matches = lib().orc_classify(_ptr(nb), nq, q0, k, nclasses, rule, _ptr(lab), _ptr(pred))
    return pred, int(matches)
