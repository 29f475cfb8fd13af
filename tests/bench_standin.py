"""CPU stand-in engine for bench.py's multi-rank path (TEST INFRASTRUCTURE).

bench.py loads it only when KNN_BENCH_TEST_ENGINE=bench_standin:make is set
(tests/test_bench_launch.py), so `bench.py --gpus N` can run its whole rank
path -- the launcher, the gloo process group, ring_search's exchange, the
barrier + max-over-ranks timing and rank 0's JSON line -- on a machine with
no GPU.  The per-block fold is the oracle's block restatement (as in
tests/test_ring_cpu.py::CpuEngine); the product bench never uses it.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(HERE, "..", "oracle"),):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import oracle  # noqa: E402


class _Ctx:
    """the knn_ctx queries bench.py makes after the timed region"""

    def __init__(self, eng):
        self.eng = eng

    def profile(self, enable=-1):
        if enable == 1:
            self.eng.steps = 0
            return 0.0, 0.0, 0
        return 0.0, 0.0, self.eng.steps

    def info(self):
        return 0, 1

    def contraction_bits(self):
        return 64

    def split(self):
        return 0


class StandinEngine:
    """The subset of mpiknn.ring.GpuEngine that ring_search and bench.py use;
    blocks are (R, n + 1) float64 CPU tensors (last column: the row count)."""

    def __init__(self, torch, n, R, nq, k, dtype):
        self.torch = torch
        self.n, self.R, self.nq, self.k = n, R, nq, k
        self.qb = torch.zeros((R, n + 1), dtype=torch.float64)
        self.rx = tuple(torch.zeros_like(self.qb) for _ in range(4))
        self.meta = torch.zeros(8, dtype=torch.float64)
        self.ctx = _Ctx(self)
        self.steps = 0
        self.lists = None

    def pack(self, src, layout_col=True):
        rows = src.shape[0]
        X = np.ascontiguousarray(src.numpy(), dtype=np.float64)
        self.qb.zero_()
        self.qb[:rows, : self.n] = self.torch.from_numpy(X)
        self.qb[0, self.n] = rows
        self.meta.zero_()
        self.meta[0] = float(np.abs(X).max()) if rows else 0.0

    def begin(self, q_base, h_meta=None):
        self.q_base = q_base
        self.lists = oracle.lists_init(self.nq, self.k)

    def step(self, buf, rows, base, rescan=False):
        assert int(buf[0, self.n]) == rows
        oracle.knn_block(self.qb[: self.nq, : self.n].numpy(), self.q_base,
                         buf[:rows, : self.n].numpy(), base, self.lists)

    def end(self):
        self.steps += 1
        return 0

    def result(self):
        return self.lists


def make(torch, n, R, nq, k, dtype):
    return StandinEngine(torch, n, R, nq, k, dtype)
