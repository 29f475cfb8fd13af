"""Per-row hashes of all-kNN results (the full-size fixtures *_rowhash.npz).

One 64-bit hash per query row: blake2b-64 of the row's k neighbour indices
(int32 LE) followed by its k distances' fp64 bits (LE).  make_golden.py
commits it for every row of the oracle's 60000x784 results; the GPU tests
(tests/test_golden.py::check_all_rows) and bench.py's post-timing check hash
libknn's rows the same way and compare all of them.
"""
import hashlib

import numpy as np


def row_hashes(nb):
    idx = np.ascontiguousarray(nb["idx"], dtype="<i4")
    bits = np.ascontiguousarray(nb["distance"], dtype="<f8").view("<u8")
    out = np.empty(len(idx), dtype=np.uint64)
    for r in range(len(idx)):
        h = hashlib.blake2b(idx[r].tobytes() + bits[r].tobytes(), digest_size=8)
        out[r] = np.frombuffer(h.digest(), dtype="<u8")[0]
    return out
