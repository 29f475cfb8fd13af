"""mpiknn.ring.ring_search -- the code bench.py runs per rank under RCCL --
driven on one GPU through a loopback stand-in for torch.distributed.

Each hop's irecv is a device copy of the block the left neighbour would
send, enqueued on the caller's stream at posting time (where RCCL's stream
would be ordered).  So the real rotation over the STEP_LAG + 2 receive buffers
and the overlapped knn_ctx_step schedule (include/knn.h: the caller's
stream lags KNN_STEP_LAG steps) are exercised with buffer reuse, and every rank's
result must equal the oracle's serial scan of its rows (oracle.knn(X, k,
rows=(base, rows)), serial:72-93) byte for byte -- in each hop form: element
blocks, int16 wire blocks and the search's shadow form (int8 byte blocks on
8-bit data, fp16 shadow rows on wider integers) -- and in both schedules
(neighbour hops, and the direct exchange whose received byte blocks are
folded by one fused launch).  This replaces blk:187-244 / nb:196-259 with
every block visited once.
"""
import types

import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu


class _Req:
    def wait(self):
        pass


def loopback_dist(torch, rank, P, packed, metas, wires, engine, schedule="ring"):
    """A torch.distributed stand-in for rank `rank` of a P-ring whose packed
    blocks are `packed` (block b = rank b's own block), with wire forms
    (mpiknn.wire_pack) `wires`; shadow forms are made on first use with the
    receiving rank's context (knn_ctx_shadow_pack: the form its search
    folds).  An irecv gets the form whose size it asks for."""
    hop = {"n": 0}
    shadows = {}

    def shadow(b):
        if b not in shadows:
            sb = torch.empty(engine.ctx.shadow_bytes(engine.R), dtype=torch.uint8,
                             device=packed[b].device)
            engine.ctx.shadow_pack(sb.data_ptr(), packed[b].data_ptr(), engine.R, engine.stream())
            shadows[b] = sb
        return shadows[b]
    ns = types.SimpleNamespace()
    ns.ReduceOp = types.SimpleNamespace(MAX="max", SUM="sum")

    def all_reduce(t, op):
        if op == "max" and t.numel() == metas.shape[1]:
            t.copy_(metas.max(dim=0).values)

    def P2POp(fn, buf, peer):
        return (fn, buf, peer)

    def isend(*a):
        pass

    def irecv(*a):
        pass

    def batch_isend_irecv(ops):
        for fn, buf, peer in ops:
            if fn is irecv:
                # ring: hop h brings the block that started on rank - h - 1
                # (a rotation is P - 1 hops; the rescan pass's second
                # rotation starts over); direct: the receive from a peer
                # brings the peer's own block
                b = peer if schedule == "direct" else (rank - hop["n"] % max(P - 1, 1) - 1) % P
                forms = {t[b].numel(): t[b] for t in (packed, wires)}
                if engine.ctx.shadow():
                    sb = shadow(b)
                    forms[sb.numel()] = sb
                src = forms[buf.numel()]
                buf.copy_(src, non_blocking=True)
        hop["n"] += 1
        return [_Req()]

    ns.all_reduce, ns.P2POp, ns.isend, ns.irecv = all_reduce, P2POp, isend, irecv
    ns.batch_isend_irecv = batch_isend_irecv
    return ns


@pytest.mark.parametrize("schedule", ["ring", "direct"])
@pytest.mark.parametrize("P", [2, 4, 7, 8])
@pytest.mark.parametrize("kind", ["int", "real", "int-nowire", "int-noshadow", "int-fp16",
                                  "wide-int"])
def test_ring_search_rotation(knn, oracle, P, kind, schedule, monkeypatch):
    import torch
    import mpiknn.ring as ring

    if kind == "int-nowire":
        monkeypatch.setenv("KNN_NO_WIRE", "1")
        monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    if kind == "int-noshadow":
        monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    if kind == "int-fp16":
        monkeypatch.setenv("KNN_NO_I8", "1")      # fp16 shadow rows on the link
    if kind == "real":
        X = datasets.digits_real()[0]
    elif kind == "wide-int":                      # range 512: fp16 shadows, not int8
        X = np.random.default_rng(P).integers(-256, 257, (2200, 300)).astype(np.float64)
        X[40] = X[3]
    else:
        X = datasets.mnist_like(3000, 784, seed=5)[0]
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
    for g, e in enumerate(engines):
        base, rows = blocks[g]
        d = loopback_dist(torch, g, P, packed, metas, wires, e, schedule)
        ring.ring_search(d, torch, e, g, P, m, base, schedule=schedule)
        got = e.result()
        ref = oracle.knn(X, 30, rows=(base, rows))
        assert np.array_equal(got["idx"], ref["idx"]), (P, g)
        assert np.array_equal(got["distance"].view(np.uint64),
                              ref["distance"].view(np.uint64)), (P, g)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_wire_round_trip(knn, dtype):
    """int16 wire form: pack -> unpack restores the packed block byte for
    byte on integer data (knn_wire_ok), including norms and meta."""
    import torch
    import mpiknn.ring as ring
    rng = np.random.default_rng(6)
    X = rng.integers(-32767, 32768, (1000, 37)).astype(np.float64)
    m, n = X.shape
    e = ring.GpuEngine(torch, 0, n, m, m, 8, dtype=dtype)
    e.pack(torch.from_numpy(X if dtype == "f64" else X.astype(np.float32)).to("cuda:0"),
           layout_col=False, elements=True)
    assert knn.wire_ok(e.meta.cpu().numpy())
    w = torch.empty(knn.wire_bytes(m, n, dtype), dtype=torch.uint8, device="cuda:0")
    back = torch.empty_like(e.qb)
    knn.wire_pack(w.data_ptr(), e.qb.data_ptr(), m, n, dtype, e.stream())
    knn.wire_unpack(back.data_ptr(), w.data_ptr(), m, n, dtype, e.stream())
    assert torch.equal(back, e.qb)
    X[0, 0] = 32768.0
    assert not knn.wire_ok(np.array([32768.0, 0, 0, 0, 0, 0, 0, 0]))


@pytest.mark.parametrize("schedule", ["ring", "direct"])
@pytest.mark.parametrize("P", [2, 8])
@pytest.mark.parametrize("shape", ["gist", "sift"])
def test_ring_search_fp32_configs(knn, oracle, P, shape, schedule):
    """configs[4] / configs[3] shapes through the real ring_search at reduced
    m: gist-like (real-valued fp32, n = 960, k = 100: fp32 GEMM filter +
    exact re-rank, element blocks on the link) and sift-like (integer fp32,
    n = 128, k = 32: int8 byte blocks on the link).  Every rank equals the
    oracle on the fp32-rounded points (the fp32 contract, test_gpu_f32.py)."""
    import torch
    import mpiknn.ring as ring

    if shape == "gist":
        X, k = datasets.gist_like(1200, 960, clusters=32), 100
    else:
        X, k = datasets.sift_like(3000, 128, clusters=64, seed=7), 32
    X32 = np.ascontiguousarray(X, dtype=np.float32)
    Xr = X32.astype(np.float64)
    m, n = X32.shape
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(X32).to(dev)
    R, blocks = ring.partition(m, P)
    engines = []
    for g in range(P):
        base, rows = blocks[g]
        e = ring.GpuEngine(torch, 0, n, R, rows, k, dtype="f32")
        e.pack(Xd[base:base + rows], layout_col=False, elements=True)
        engines.append(e)
    packed = [e.qb.clone() for e in engines]
    metas = torch.stack([e.meta for e in engines])
    for g, e in enumerate(engines):
        base, rows = blocks[g]
        d = loopback_dist(torch, g, P, packed, metas, packed, e, schedule)
        ring.ring_search(d, torch, e, g, P, m, base, schedule=schedule)
        got = e.result()
        ref = oracle.knn(Xr, k, rows=(base, rows))
        assert np.array_equal(got["idx"], ref["idx"]), (shape, P, g)
        assert np.array_equal(got["distance"].view(np.uint64),
                              ref["distance"].view(np.uint64)), (shape, P, g)


@pytest.mark.parametrize("fuse", ["rest", "all"])
@pytest.mark.parametrize("P", [3, 12])
def test_direct_fused_many_blocks(knn, oracle, P, fuse, monkeypatch):
    """The direct schedule's fused step over more blocks than one launch
    takes (P = 12: 11 or 12 byte blocks = launches of 8 + 3 / 8 + 4; "all"
    folds the own block in the fused step too), with a forced rescan pass
    over element blocks afterwards; every rank equals the oracle's scan of
    its rows."""
    import torch
    import mpiknn.ring as ring
    monkeypatch.setenv("KNN_FORCE_RESCAN", "1")
    monkeypatch.setenv("KNN_RING_FUSE", fuse)
    X = datasets.mnist_like(2400, 200, seed=11)[0]
    X[1000] = X[17]                                   # a duplicate across blocks
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
    for g in (0, P // 2, P - 1):
        e = engines[g]
        base, rows = blocks[g]
        d = loopback_dist(torch, g, P, packed, metas, wires, e, "direct")
        ring.ring_search(d, torch, e, g, P, m, base, schedule="direct")
        assert e.ctx.shadow() == 2
        got = e.result()
        ref = oracle.knn(X, 30, rows=(base, rows))
        assert np.array_equal(got["idx"], ref["idx"]), (P, g)
        assert np.array_equal(got["distance"].view(np.uint64),
                              ref["distance"].view(np.uint64)), (P, g)
