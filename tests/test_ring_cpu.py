"""The per-rank ring driver (mpiknn/ring.py) under gloo on CPU.

world_size 2, 3, 4 (and 8 for the direct exchange) processes run the real
ring_search() schedules -- meta
all-reduce, then either P-1 isend/irecv hops per pass with the query block
kept resident ("ring") or one exchange of every block with every rank
("direct"), and the rescan pass -- with a CPU stand-in engine whose per-block fold
is the oracle's block restatement (test-only; the product engine is HIP).
Every rank must end with exactly the serial-semantics lists of its rows and
must have folded every block exactly once per pass.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class CpuEngine:
    """Same interface as mpiknn.ring.GpuEngine; blocks are (R, n) float64."""

    def __init__(self, oracle, n, R, nq, k, force_rescan):
        self.O = oracle
        self.n, self.R, self.nq, self.k = n, R, nq, k
        self.qb = torch.zeros((R, n + 1), dtype=torch.float64)   # last column: row count
        self.rx = tuple(torch.zeros_like(self.qb) for _ in range(4))
        self.meta = torch.zeros(8, dtype=torch.float64)
        self.force_rescan = force_rescan
        self.visits = {False: [], True: []}
        self.h_metas = []

    def pack(self, src):
        rows = src.shape[0]
        self.qb.zero_()
        self.qb[:rows, : self.n] = src
        self.qb[0, self.n] = rows
        self.meta[0] = float(src.abs().max()) if rows else 0.0

    def begin(self, q_base, h_meta=None):
        self.q_base = q_base
        self.lists = self.O.lists_init(self.nq, self.k)
        self.h_metas.append(None if h_meta is None else np.array(h_meta))

    def meta_host(self, meta):
        # (GpuEngine: an asynchronous copy into pinned memory)
        return meta.clone()

    def step(self, buf, rows, base, rescan=False):
        assert int(buf[0, self.n]) == rows           # the block we were told we hold
        self.visits[rescan].append(base)
        target = self.rescan_lists if rescan else self.lists
        self.O.knn_block(self.qb[: self.nq, : self.n].numpy(), self.q_base,
                         buf[:rows, : self.n].numpy(), base, target)

    def end(self):
        self.rescan_lists = self.O.lists_init(self.nq, self.k)
        return 1 if self.force_rescan else 0

    def rescan_end(self):
        assert np.array_equal(self.rescan_lists, self.lists)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, force_rescan, q, m_rows=None):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, "..", "oracle"), os.path.join(here, "..", "mpi-knn_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import datasets
        import oracle
        from mpiknn.ring import partition, ring_search
        X, _ = datasets.digits_real()
        if m_rows:
            X = np.ascontiguousarray(X[:m_rows])
        m, n = X.shape
        R, blocks = partition(m, world)
        base, rows = blocks[rank]
        eng = CpuEngine(oracle, n, R, rows, 30, force_rescan)
        eng.pack(torch.from_numpy(X[base:base + rows]))
        ring_search(dist, torch, eng, rank, world, m, base)
        full = oracle.knn(X, 30, rows=(base, rows))
        ok = np.array_equal(eng.lists[["distance", "idx"]], full[["distance", "idx"]])
        nonempty = sorted(b for b, r in blocks if r > 0)
        every = sorted(eng.visits[False]) == nonempty
        every_rescan = (not force_rescan) or sorted(eng.visits[True]) == nonempty
        meta_ok = float(eng.meta[0]) == float(np.abs(X).max())
        q.put((rank, ok, every, every_rescan, meta_ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("schedule,world,force_rescan",
                         [(s, w, f) for s in ("ring", "direct") for w, f in ((2, False), (3, True), (4, True))] +
                         [("direct", 8, True)])
def test_ring_schedule_gloo(world, force_rescan, schedule, monkeypatch):
    monkeypatch.setenv("KNN_RING_SCHEDULE", schedule)   # inherited by the spawned ranks
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, force_rescan, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, every, every_rescan, meta_ok in sorted(res):
        assert ok, "rank %d lists differ from the serial scan" % rank
        assert every, "rank %d did not fold every block once" % rank
        assert every_rescan, "rank %d rescan pass missed a block" % rank
        assert meta_ok, "rank %d meta not max-reduced" % rank


def _hint_worker(rank, world, port, q):
    """three searches on one engine: the first from the reduced meta, the
    second from the first one's meta as the hint (verified after end()), the
    third on rescaled rows -- the hint no longer matches, every rank runs the
    search again from the reduced meta; every result the serial scan's"""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, "..", "oracle"), os.path.join(here, "..", "mpi-knn_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import datasets
        import oracle
        from mpiknn.ring import partition, ring_search
        X, _ = datasets.digits_real()
        m, n = X.shape
        R, blocks = partition(m, world)
        base, rows = blocks[rank]
        eng = CpuEngine(oracle, n, R, rows, 30, False)
        oks = []
        for Xs in (X, X, 3.0 * X):
            eng.visits = {False: [], True: []}
            eng.pack(torch.from_numpy(Xs[base:base + rows]))
            ring_search(dist, torch, eng, rank, world, m, base)
            full = oracle.knn(Xs, 30, rows=(base, rows))
            oks.append(np.array_equal(eng.lists[["distance", "idx"]], full[["distance", "idx"]]))
        # begins: reduced meta, the hint, the (stale) hint, then the redo
        hm = eng.h_metas
        shape = (len(hm) == 4 and hm[1] is not None and np.array_equal(hm[1], hm[0]) and
                 np.array_equal(hm[2], hm[0]) and not np.array_equal(hm[3], hm[0]))
        q.put((rank, all(oks), shape))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("schedule", ["direct", "ring"])
def test_ring_meta_hint_gloo(schedule, monkeypatch):
    """P > 1 searches after the first start from the last reduced meta
    (no host wait on the all-reduce); new data is caught after end() and
    searched again on every rank."""
    monkeypatch.setenv("KNN_RING_SCHEDULE", schedule)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_hint_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, shape in sorted(res):
        assert ok, "rank %d lists differ from the serial scan" % rank
        assert shape, "rank %d: begins did not follow reduced / hint / stale hint / redo" % rank


def test_partition_covers_all_rows():
    from mpiknn.ring import partition
    for m, P in [(60000, 8), (60000, 7), (10, 3), (9, 3)]:
        R, blocks = partition(m, P)
        assert sum(r for _, r in blocks) == m
        assert all(b == i * R for i, (b, _) in enumerate(blocks))


@pytest.mark.parametrize("schedule", ["ring", "direct"])
def test_ring_empty_last_block_gloo(schedule, monkeypatch):
    """m = 9 rows over P = 4 ranks: R = 3, so rank 3 owns no rows and its
    block is empty.  It still joins every exchange; nobody folds it."""
    monkeypatch.setenv("KNN_RING_SCHEDULE", schedule)
    from mpiknn.ring import partition
    assert partition(9, 4)[1][3] == (9, 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_worker, args=(r, world, port, True, q, 9)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, every, every_rescan, meta_ok in sorted(res):
        assert ok and every and every_rescan and meta_ok, rank


def _stall_worker(rank, world, port, schedule, timeout_s, q):
    """rank 0 runs ring_search; every other rank joins the meta all-reduce
    and then stalls (never posts its exchange), as a hung or dying peer."""
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, "..", "oracle"), os.path.join(here, "..", "mpi-knn_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import datasets
        import oracle
        from mpiknn.ring import RingError, partition, ring_search
        X, _ = datasets.digits_real()
        m, n = X.shape
        R, blocks = partition(m, world)
        base, rows = blocks[rank]
        eng = CpuEngine(oracle, n, R, rows, 30, False)
        eng.pack(torch.from_numpy(X[base:base + rows]))
        if rank != 0:
            dist.all_reduce(eng.meta, op=dist.ReduceOp.MAX)
            time.sleep(timeout_s + 20)
            q.put((rank, "stalled", 0.0))
            return
        t0 = time.perf_counter()
        try:
            ring_search(dist, torch, eng, rank, world, m, base, schedule=schedule, timeout_s=timeout_s)
            q.put((rank, "no error", time.perf_counter() - t0))
        except RingError as e:
            q.put((rank, "RingError: %s" % e, time.perf_counter() - t0))
    finally:
        q.close()
        q.join_thread()   # flush the result before the hard exit
        os._exit(0)       # the stalled peers' sockets die with them


@pytest.mark.parametrize("schedule,world", [("direct", 2), ("ring", 2), ("direct", 3)])
def test_ring_stalled_peer_raises_within_timeout(schedule, world):
    """a peer that stops participating after the meta
    all-reduce must turn into RingError on the surviving rank within the
    exchange bound (KNN_RING_TIMEOUT_S / timeout_s), not a hang."""
    timeout_s = 4.0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stall_worker, args=(r, world, port, schedule, timeout_s, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=120)
        assert got[0] == 0, got
        assert got[1].startswith("RingError"), got
        assert got[2] < timeout_s + 10.0, got
    finally:
        for p in procs:
            p.kill()
            p.join(timeout=30)
