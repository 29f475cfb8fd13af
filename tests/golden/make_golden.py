#!/usr/bin/env python3
"""Regenerate the committed golden fixtures in tests/golden/.

  python tests/golden/make_golden.py

Provenance.  The reference (knn-serial.c, mpi-knn-parallel_*.c) cannot be
built here: it needs MATLAB's mat.h / libmat / libmx, which the image lacks,
and stand-ins may not be written.  Its only outputs on
record are the aggregate numbers SURVEY.md (sec.0 F1/F7, sec.4) took from
reference runs; they are written to reference_runs.json verbatim and pin the
oracle (tests/test_golden.py).  The per-neighbour fixtures below are produced
by the oracle (oracle/knn_oracle.c, serial:57-93 restated) once those pins
hold, so the GPU tests can check neighbour lists against committed data:

* digits_k30.npz      sklearn digits 1797x64, k=30: idx (u16, 1-based),
                      d2 = S (u16, exact integers), serial-rule prediction;
* digits_real_k30.npz digits_real() 1800x64, k=30: idx (u16) and the
                      distances' raw fp64 bits (u64);
* mnist_like_sample.npz  datasets.mnist_like(60000): 48 sampled queries
                      against the full 60000x784 corpus, k=30: rows, idx
                      (i32), d2 (u32, exact integers);
* mnist_real_sample.npz  datasets.mnist_real(60000) (real-valued, the GEMM
                      mode): the same 48 rows, k=30: rows, idx (i32), the
                      distances' raw fp64 bits (u64);
* mnist_like_rowhash.npz / mnist_real_rowhash.npz  EVERY row of the two
                      60000x784 corpora (configs[1]/[2]): a 64-bit hash per
                      row of its k=30 (idx i32 LE, distance fp64 bits LE)
                      record (row_hashes(); SURVEY sec.4's "sampled rows plus
                      per-row hashes"), so the GPU tests compare all 60000
                      rows, not only the 48 sampled ones.

  python tests/golden/make_golden.py [--only mnist_real|rowhash]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.dirname(HERE), HERE]

import datasets  # noqa: E402
import oracle  # noqa: E402
from rowhash import row_hashes  # noqa: E402  (the same hash the tests take)

REFERENCE_RUNS = {
    "_source": "SURVEY.md sec.0 (F1, F7) and sec.4: reference binaries run on these inputs",
    "digits": {"k": 30, "matches_serial_rule": 1636, "matches_mpi_rule": 1635,
               "matches_true_majority": 1742, "queries_tied_at_k_boundary": 106},
    "digits_real": {"k": 30, "matches_serial_rule": 1631},
}

MNIST_SAMPLE_SEED = 20260214


def exact_s(dist):
    """Integer S with sqrt(S) == dist bit-for-bit (integer data)."""
    s = np.rint(dist.astype(np.float64) ** 2)
    assert np.array_equal(np.sqrt(s), dist)
    return s.astype(np.uint64)


def mnist_sample_rows(m=60000, q=48):
    rng = np.random.default_rng(MNIST_SAMPLE_SEED)
    rows = np.sort(rng.choice(m, q - 2, replace=False))
    return np.concatenate([[0], rows, [m - 1]]).astype(np.int64)


def mnist_real_fixture():
    Xm, _ = datasets.mnist_real(60000)
    rows = mnist_sample_rows()
    idx = np.zeros((len(rows), 30), np.int32)
    bits = np.zeros((len(rows), 30), np.uint64)
    for i, r in enumerate(rows):
        nb = oracle.knn(Xm, 30, rows=(int(r), 1))
        idx[i] = nb["idx"][0]
        bits[i] = nb["distance"][0].view(np.uint64)
    np.savez_compressed(os.path.join(HERE, "mnist_real_sample.npz"), rows=rows, idx=idx,
                        dist_bits=bits)


def rowhash_fixtures():
    """the oracle's all-kNN of every row of both 60000x784 corpora (a few
    minutes each on the container's cores), kept as per-row hashes"""
    for name, make in (("mnist_like", datasets.mnist_like), ("mnist_real", datasets.mnist_real)):
        X, _ = make(60000)
        nb = oracle.knn(X, 30)
        np.savez_compressed(os.path.join(HERE, "%s_rowhash.npz" % name), k=np.int32(30),
                            m=np.int32(60000), hash=row_hashes(nb))
        print("wrote", name, flush=True)


def main():
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "mnist_real":
        mnist_real_fixture()
        return
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "rowhash":
        rowhash_fixtures()
        return
    with open(os.path.join(HERE, "reference_runs.json"), "w") as f:
        json.dump(REFERENCE_RUNS, f, indent=1)
        f.write("\n")

    X, y = datasets.digits()
    nb = oracle.knn(X, 30)
    pred, matches = oracle.classify(nb, y, 10, oracle.VOTE_SERIAL)
    assert matches == REFERENCE_RUNS["digits"]["matches_serial_rule"]
    d2 = exact_s(nb["distance"])
    np.savez_compressed(os.path.join(HERE, "digits_k30.npz"),
                        idx=nb["idx"].astype(np.uint16), d2=d2.astype(np.uint16),
                        pred=np.asarray(pred, dtype=np.uint8))

    Xr, yr = datasets.digits_real()
    nb = oracle.knn(Xr, 30)
    assert oracle.classify(nb, yr, 10, oracle.VOTE_SERIAL)[1] == \
        REFERENCE_RUNS["digits_real"]["matches_serial_rule"]
    np.savez_compressed(os.path.join(HERE, "digits_real_k30.npz"),
                        idx=nb["idx"].astype(np.uint16),
                        dist_bits=nb["distance"].view(np.uint64))

    Xm, _ = datasets.mnist_like(60000)
    rows = mnist_sample_rows()
    idx = np.zeros((len(rows), 30), np.int32)
    d2 = np.zeros((len(rows), 30), np.uint32)
    for i, r in enumerate(rows):
        nb = oracle.knn(Xm, 30, rows=(int(r), 1))
        idx[i] = nb["idx"][0]
        d2[i] = exact_s(nb["distance"][0])
    np.savez_compressed(os.path.join(HERE, "mnist_like_sample.npz"), rows=rows, idx=idx, d2=d2)
    mnist_real_fixture()
    rowhash_fixtures()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
