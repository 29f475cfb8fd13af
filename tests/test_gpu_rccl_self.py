"""The ring's RCCL calls, executed on a one-GPU box.

The P >= 2 ring replaces the MPI rotation of mpi-knn-parallel_blocking.c:
187-214 / _non_blocking.c:198-230.  Its loopback tests (test_gpu_parity.py,
test_gpu_ring_rotation.py) move blocks with device copies; here every
transfer goes through RCCL instead:

* knn_ring.c with KNN_RING_LOOPBACK=rccl: P virtual ranks on device 0, a
  one-device communicator (ncclCommInitAll, ndev = 1), each hop / exchange
  one ncclGroupStart / ncclSend(to self) / ncclRecv(from self) /
  ncclGroupEnd group shaped like the multi-GPU transport's, the meta
  through ncclAllReduce, ring_drain polling ncclCommGetAsyncError;
* mpiknn/ring.py (what bench.py runs per rank) on a real world-size-1
  torch.distributed "nccl" (RCCL) process group: every irecv of the P-rank
  ring is an RCCL send-to-self of the block the left neighbour (or the
  peer) would send plus the receive into the rank's buffer, every isend an
  RCCL send-to-self into a sink, all in one batch_isend_irecv; the ring's
  _wait_all takes its stream-ordered nccl branch;
* the progress-bounded drain: a loopback transfer that never
  lands (KNN_RING_TEST_STALL=1) ends the search with KNN_ERR_RCCL after
  KNN_RING_TIMEOUT_S, and the process goes on.

Every rank's rows must equal the oracle's serial scan (knn-serial.c:72-93)
byte for byte.
"""
import time

import numpy as np
import pytest

import datasets
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("schedule", ["direct", "ring"])
@pytest.mark.parametrize("P", [2, 8])
@pytest.mark.parametrize("force_rescan", [False, True])
def test_ring_driver_rccl_self(knn, oracle, monkeypatch, P, schedule, force_rescan):
    monkeypatch.setenv("KNN_RING_LOOPBACK", "rccl")
    monkeypatch.setenv("KNN_RING_SCHEDULE", schedule)
    if force_rescan:
        monkeypatch.setenv("KNN_FORCE_RESCAN", "1")
    # mnist-shaped integers: int8 byte blocks on the link (element blocks in
    # the forced rescan pass); real-valued digits: element blocks
    for X in (datasets.mnist_like(1500, 784, seed=4)[0], datasets.digits_real()[0]):
        ref = oracle.knn(X, 30)
        got, _ = knn.search(X, 30, ngpus=P, layout="col")
        assert_same(got, ref, "rccl-self ring P=%d %s" % (P, schedule))


def test_ring_driver_rccl_self_element_blocks(knn, oracle, monkeypatch):
    """KNN_NO_SHADOW_RING=1: fp64 element blocks through RCCL, P = 8 fp32 sift."""
    monkeypatch.setenv("KNN_RING_LOOPBACK", "rccl")
    monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    X = datasets.mnist_like(1500, 784, seed=9)[0]
    got, _ = knn.search(X, 30, ngpus=8, layout="col")
    assert_same(got, oracle.knn(X, 30), "rccl-self element blocks")
    monkeypatch.delenv("KNN_NO_SHADOW_RING")
    X = datasets.sift_like(3000, 128)
    got, _ = knn.search(X, 32, ngpus=8, dtype="f32")
    assert_same(got, oracle.knn(X.astype(np.float32).astype(np.float64), 32), "rccl-self sift")


def test_ring_driver_stalled_transfer_times_out(knn, oracle, monkeypatch):
    """A loopback transfer that never lands: the drain gives up after
    KNN_RING_TIMEOUT_S (progress-bounded), returns KNN_ERR_RCCL, releases
    the stalled queue and tears down without hanging; the next search on
    the same process is correct."""
    X = datasets.mnist_like(800, 784, seed=2)[0]
    monkeypatch.setenv("KNN_RING_LOOPBACK", "1")
    monkeypatch.setenv("KNN_RING_TEST_STALL", "1")
    monkeypatch.setenv("KNN_RING_TIMEOUT_S", "2")
    for schedule in ("direct", "ring"):
        monkeypatch.setenv("KNN_RING_SCHEDULE", schedule)
        t0 = time.time()
        with pytest.raises(knn.KnnError) as ei:
            knn.search(X, 30, ngpus=4, layout="col")
        assert ei.value.status == knn.ERR_RCCL
        assert 1.5 < time.time() - t0 < 60
    monkeypatch.delenv("KNN_RING_TEST_STALL")
    got, _ = knn.search(X, 30, ngpus=4, layout="col")
    assert_same(got, oracle.knn(X, 30), "after a stalled search")


# ------------------------------------------------ ring.py over a real RCCL group

@pytest.fixture(scope="module")
def nccl1():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


class RcclSelfDist:
    """torch.distributed for virtual rank `rank` of a P-ring, with every
    transfer made by a world-size-1 RCCL process group (rank 0 sending to
    and receiving from itself).  An irecv from peer p gets block b's form of
    the receiving buffer's size (b = p for the direct exchange; the block
    that started on rank - h - 1 for ring hop h), sent by RCCL; an isend
    goes to a sink buffer through RCCL.  The works returned are the
    group's own (their wait() is stream-ordered)."""

    def __init__(self, dist, torch, rank, P, packed, metas, wires, engine, schedule):
        self.d, self.torch = dist, torch
        self.rank, self.P, self.schedule = rank, P, schedule
        self.packed, self.metas, self.wires, self.engine = packed, metas, wires, engine
        self.ReduceOp = dist.ReduceOp
        self.isend, self.irecv = "isend", "irecv"
        self.hop = 0
        self.shadows, self.sinks = {}, {}
        self.calls = 0

    def get_backend(self):
        return self.d.get_backend()

    def P2POp(self, fn, buf, peer):
        return (fn, buf, peer)

    def all_reduce(self, t, op):
        if op == self.d.ReduceOp.MAX and t.numel() == self.metas.shape[1]:
            t.copy_(self.metas.max(dim=0).values)
        self.d.all_reduce(t, op=op)      # one rank: the identity, through RCCL
        self.calls += 1

    def _shadow(self, b):
        e = self.engine
        if b not in self.shadows:
            sb = self.torch.empty(e.ctx.shadow_bytes(e.R), dtype=self.torch.uint8, device=self.packed[b].device)
            e.ctx.shadow_pack(sb.data_ptr(), self.packed[b].data_ptr(), e.R, e.stream())
            self.shadows[b] = sb
        return self.shadows[b]

    def batch_isend_irecv(self, ops):
        real = []
        for fn, buf, peer in ops:
            if fn == "irecv":
                P = self.P
                b = peer if self.schedule == "direct" else (self.rank - self.hop % max(P - 1, 1) - 1) % P
                forms = {t[b].numel(): t[b] for t in (self.packed, self.wires)}
                if self.engine.ctx.shadow():
                    sb = self._shadow(b)
                    forms[sb.numel()] = sb
                src = forms[buf.numel()]
                real += [self.d.P2POp(self.d.isend, src, 0), self.d.P2POp(self.d.irecv, buf, 0)]
            else:
                n = buf.numel()
                if n not in self.sinks:
                    self.sinks[n] = self.torch.empty_like(buf)
                real += [self.d.P2POp(self.d.isend, buf, 0), self.d.P2POp(self.d.irecv, self.sinks[n], 0)]
        self.hop += 1
        self.calls += 1
        return self.d.batch_isend_irecv(real)


@pytest.mark.parametrize("schedule", ["direct", "ring"])
@pytest.mark.parametrize("P", [2, 8])
@pytest.mark.parametrize("kind", ["int", "int-rescan", "int-wire", "real"])
def test_ring_search_over_rccl(knn, oracle, nccl1, monkeypatch, P, schedule, kind):
    """mpiknn.ring.ring_search -- bench.py's per-rank code -- with its
    transfers on RCCL: byte blocks (int), byte blocks then a forced rescan
    over int16 wire blocks (int-rescan), wire blocks only (int-wire), fp64
    element blocks of real-valued rows (real)."""
    import torch
    import mpiknn.ring as ring
    if kind == "int-rescan":
        monkeypatch.setenv("KNN_FORCE_RESCAN", "1")
    if kind == "int-wire":
        monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    X = datasets.digits_real()[0] if kind == "real" else datasets.mnist_like(3000, 784, seed=5)[0]
    m, n = X.shape
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(X).to(dev)
    R, blocks = ring.partition(m, P)
    engines = []
    for g in range(P):
        base, rows = blocks[g]
        e = ring.GpuEngine(torch, 0, n, R, rows, 30)
        e.pack(Xd[base:base + rows], layout_col=False, elements=True)
        engines.append(e)
    packed = [e.qb.clone() for e in engines]
    metas = torch.stack([e.meta for e in engines])
    wires = []
    for e in engines:
        w = torch.empty(knn.wire_bytes(R, n), dtype=torch.uint8, device=dev)
        knn.wire_pack(w.data_ptr(), e.qb.data_ptr(), R, n, "f64", e.stream())
        wires.append(w)
    for g in sorted({0, P // 2, P - 1}):
        e = engines[g]
        base, rows = blocks[g]
        d = RcclSelfDist(nccl1, torch, g, P, packed, metas, wires, e, schedule)
        ring.ring_search(d, torch, e, g, P, m, base, schedule=schedule, timeout_s=120)
        assert d.calls >= 2          # the meta all-reduce and at least one exchange went through RCCL
        got = e.result()
        ref = oracle.knn(X, 30, rows=(base, rows))
        assert np.array_equal(got["idx"], ref["idx"]), (P, g, kind, schedule)
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), (P, g)
