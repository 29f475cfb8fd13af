"""mpiknn.ring.ring_search -- the code bench.py runs per rank under RCCL --
driven on one GPU through a loopback stand-in for torch.distributed.

Each hop's irecv is a device copy of the block the left neighbour would
send, enqueued on the caller's stream at posting time (where RCCL's stream
would be ordered).  So the real rotation over the STEP_LAG + 2 receive buffers
and the overlapped knn_ctx_step schedule (include/knn.h: the caller's
stream lags KNN_STEP_LAG steps) are exercised with buffer reuse, and every rank's
result must equal the 1-GPU search byte for byte.
"""
import types

import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu


class _Req:
    def wait(self):
        pass


def loopback_dist(torch, rank, P, packed, metas, wires, shadows):
    """A torch.distributed stand-in for rank `rank` of a P-ring whose packed
    blocks are `packed` (block b = rank b's own block), with wire forms
    (mpiknn.wire_pack) `wires` and shadow blocks (mpiknn.shadow_pack)
    `shadows`; an irecv gets the form whose size it asks for."""
    hop = {"n": 0}
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
                # hop h brings the block that started on rank - h - 1
                b = (rank - hop["n"] - 1) % P
                forms = {t[b].numel(): t[b] for t in (packed, wires, shadows)}
                src = forms[buf.numel()]
                buf.copy_(src, non_blocking=True)
        hop["n"] += 1
        return [_Req()]

    ns.all_reduce, ns.P2POp, ns.isend, ns.irecv = all_reduce, P2POp, isend, irecv
    ns.batch_isend_irecv = batch_isend_irecv
    return ns


@pytest.mark.parametrize("P", [2, 4, 7])
@pytest.mark.parametrize("kind", ["int", "real", "int-nowire", "int-noshadow"])
def test_ring_search_rotation(knn, P, kind, monkeypatch):
    import torch
    import mpiknn.ring as ring

    if kind == "int-nowire":
        monkeypatch.setenv("KNN_NO_WIRE", "1")
        monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    if kind == "int-noshadow":
        monkeypatch.setenv("KNN_NO_SHADOW_RING", "1")
    X = datasets.mnist_like(3000, 784, seed=5)[0] if kind != "real" else datasets.digits_real()[0]
    m, n = X.shape
    full, _ = knn.search(X, 30)
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(X).to(dev)
    R, blocks = ring.partition(m, P)
    engines = []
    for g in range(P):
        base, rows = blocks[g]
        e = ring.GpuEngine(torch, 0, n, R, rows, 30)
        e.pack(Xd[base:base + rows], layout_col=False)
        engines.append(e)
    packed = [e.qb.clone() for e in engines]
    metas = torch.stack([e.meta for e in engines])
    wires = []
    for e in engines:
        w = torch.empty(knn.wire_bytes(R, n), dtype=torch.uint8, device=dev)
        knn.wire_pack(w.data_ptr(), e.qb.data_ptr(), R, n, "f64", e.stream())
        wires.append(w)
    shadows = []
    for e in engines:
        sb = torch.empty(knn.shadow_bytes(R, n), dtype=torch.uint8, device=dev)
        knn.shadow_pack(sb.data_ptr(), e.qb.data_ptr(), R, n, "f64", e.stream())
        shadows.append(sb)
    for g, e in enumerate(engines):
        base, rows = blocks[g]
        d = loopback_dist(torch, g, P, packed, metas, wires, shadows)
        ring.ring_search(d, torch, e, g, P, m, base)
        got = e.result()
        assert np.array_equal(got["idx"], full[base:base + rows]["idx"]), (P, g)
        assert np.array_equal(got["distance"].view(np.uint64),
                              full[base:base + rows]["distance"].view(np.uint64)), (P, g)


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
           layout_col=False)
    assert knn.wire_ok(e.meta.cpu().numpy())
    w = torch.empty(knn.wire_bytes(m, n, dtype), dtype=torch.uint8, device="cuda:0")
    back = torch.empty_like(e.qb)
    knn.wire_pack(w.data_ptr(), e.qb.data_ptr(), m, n, dtype, e.stream())
    knn.wire_unpack(back.data_ptr(), w.data_ptr(), m, n, dtype, e.stream())
    assert torch.equal(back, e.qb)
    X[0, 0] = 32768.0
    assert not knn.wire_ok(np.array([32768.0, 0, 0, 0, 0, 0, 0, 0]))
