"""The speculative byte block (knn_block_pack_s8): the int8 contraction's
query/corpus rows x - 128, norm words and block meta straight from the
source, in one pass (replaces the pack of blk:100-109 plus the element ->
byte conversion for 8-bit integer data).

* byte for byte the block k_shadow8 builds from the element block (rows and
  norm words), with the element pack's meta (words 0-5) and word 7 = 1, for
  col-major fp64 (the .mat layout), row-major fp64 and fp32 sources;
* mpiknn.ring.ring_search (bench.py's per-rank code) begun from it at P = 1,
  2 and 8 (loopback transport, both schedules) equals the oracle's scan of
  knn-serial.c:72-93 on every rank, with and without a forced exact rescan
  (which packs the element block after the pass);
* data it cannot hold (a negative value, real values, values above 255)
  falls back to the element block, still exact.
"""
import numpy as np
import pytest

import datasets
from test_gpu_ring_rotation import loopback_dist

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("src", ["col-f64", "col-f64-784", "row-f64", "row-f32"])
def test_s8_block_equals_shadow8(knn, src):
    """(col-f64-784: MNIST's row length, 13 column tiles of the column pack,
    the last one half padding)"""
    import torch
    import mpiknn.ring as ring
    dt = "f32" if src.endswith("f32") else "f64"
    # fp32 INT mode needs n max^2 <= 2^23 (knn_i8_exact): 128 features
    shape = (2500, 784) if src.endswith("784") else (1000, 128 if dt == "f32" else 300)
    X = datasets.mnist_like(*shape, seed=3)[0]
    X[5] = 0.0
    X[7] = 255.0
    m, n = X.shape
    Xs = X.astype(np.float32) if dt == "f32" else X
    if src.startswith("col"):
        Xd = torch.from_numpy(np.ascontiguousarray(Xs.T)).to("cuda:0").t()
    else:
        Xd = torch.from_numpy(np.ascontiguousarray(Xs)).to("cuda:0")
    ref = ring.GpuEngine(torch, 0, n, m, m, 30, dtype=dt)
    ref.pack(Xd, layout_col=src.startswith("col"), elements=True)
    e = ring.GpuEngine(torch, 0, n, m, m, 30, dtype=dt)
    e.pack(Xd, layout_col=src.startswith("col"))
    assert e.spec
    hm = e.meta.cpu().numpy()
    assert knn.s8_spec_ok(hm, n, dt) and hm[7] == 1.0
    assert np.array_equal(hm[:6], ref.meta.cpu().numpy()[:6])
    ref.begin(0, h_meta=ref.meta.cpu().numpy())
    assert ref.ctx.shadow() == 2
    sb = ref.shadow_block()
    torch.cuda.synchronize()
    # real rows (padding rows are masked by index in every kernel; k_shadow8
    # converts their zeros, the direct pack leaves zeros)
    rs = (n + 31) // 32 * 32
    a, b = sb.cpu().numpy(), e.sq.cpu().numpy()
    assert np.array_equal(a[:m * rs], b[:m * rs]), "byte rows differ from k_shadow8's"
    rp = (m + 127) // 128 * 128
    r = np.arange(m)
    rr, w = r & 127, r & 31
    pos = (r & ~127) + (((rr >> 5) * 2 + ((w >> 2) & 1)) * 4 + (w >> 3)) * 4 + (w & 3)
    na = a[rp * rs:rp * rs + 8 * rp].view(np.int32)
    nb = b[rp * rs:rp * rs + 8 * rp].view(np.int32)
    assert np.array_equal(na[pos], nb[pos]), "slot words differ from k_shadow8's"
    assert np.array_equal(na[rp + pos], nb[rp + pos]), "init words differ from k_shadow8's"
    # the two words hold |x'|^2 = sum (x - 128)^2 (knn_device.h: i8_norm_of)
    nrm = ((X.astype(np.int64) - 128) ** 2).sum(1)
    assert np.array_equal(-2 * nb[rp + pos].astype(np.int64) - (nb[pos] >> 5), nrm)


def _engines(torch, ring, knn, X, P, k=30, dtype="f64"):
    m, n = X.shape
    dev = torch.device("cuda", 0)
    Xs = X.astype(np.float32) if dtype == "f32" else X
    Xd = torch.from_numpy(np.ascontiguousarray(Xs)).to(dev)
    R, blocks = ring.partition(m, P)
    engines, packed, emetas = [], [], []
    for g in range(P):
        base, rows = blocks[g]
        el = ring.GpuEngine(torch, 0, n, R, rows, k, dtype=dtype)
        el.pack(Xd[base:base + rows], layout_col=False, elements=True)
        packed.append(el.qb.clone())
        emetas.append(el.meta.clone())
        e = ring.GpuEngine(torch, 0, n, R, rows, k, dtype=dtype)
        e.pack(Xd[base:base + rows], layout_col=False)
        engines.append(e)
    metas = torch.stack([e.meta for e in engines])
    wires = []
    for el_b in packed:
        w = torch.empty(knn.wire_bytes(R, n, dtype), dtype=torch.uint8, device=dev)
        knn.wire_pack(w.data_ptr(), el_b.data_ptr(), R, n, dtype, engines[0].stream())
        wires.append(w)
    return R, blocks, engines, packed, metas, wires, torch.stack(emetas)


def _dist(torch, g, P, packed, metas, wires, e, schedule, emetas):
    """loopback_dist whose second meta all-reduce (after a fallback to
    element blocks) reduces the element packs' metas"""
    d = loopback_dist(torch, g, P, packed, metas, wires, e, schedule)
    calls = {"n": 0}

    def all_reduce(t, op):
        if op == "max" and t.numel() == metas.shape[1]:
            t.copy_((metas if calls["n"] == 0 else emetas).max(dim=0).values)
            calls["n"] += 1
    d.all_reduce = all_reduce
    return d


@pytest.mark.parametrize("rescan", [False, True])
@pytest.mark.parametrize("schedule", ["direct", "ring"])
@pytest.mark.parametrize("P", [1, 2, 8])
def test_ring_search_from_s8(knn, oracle, P, schedule, rescan, monkeypatch):
    """(the loopback's hop model restarts its rotation every P - 1 hops, so
    the neighbour ring's second rotation -- the rescan pass's exchange of
    element blocks after a byte-block search -- runs here too)"""
    import torch
    import mpiknn.ring as ring
    if rescan:
        monkeypatch.setenv("KNN_FORCE_RESCAN", "1")
    X = datasets.mnist_like(2400, 784, seed=9)[0]
    X[2000] = X[11]                                   # a duplicate across blocks
    m, n = X.shape
    R, blocks, engines, packed, metas, wires, emetas = _engines(torch, ring, knn, X, P)
    for g in sorted({0, P // 2, P - 1}):
        e = engines[g]
        base, rows = blocks[g]
        assert e.spec
        d = _dist(torch, g, P, packed, metas, wires, e, schedule, emetas) if P > 1 else None
        ring.ring_search(d, torch, e, g, P, m, base, schedule=schedule)
        assert e.spec and e.ctx.shadow() == 2
        got = e.result()
        ref = oracle.knn(X, 30, rows=(base, rows))
        assert np.array_equal(got["idx"], ref["idx"]), (P, g)
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), (P, g)


def test_ring_search_from_s8_f32_sift(knn, oracle):
    """configs[3]'s form: fp32 rows, k = 32, P = 1 and 4"""
    import torch
    import mpiknn.ring as ring
    X = datasets.sift_like(3000, 128, clusters=64, seed=4)
    Xr = np.ascontiguousarray(X, dtype=np.float32).astype(np.float64)
    for P in (1, 4):
        R, blocks, engines, packed, metas, wires, emetas = _engines(torch, ring, knn, Xr, P, k=32, dtype="f32")
        for g in (0, P - 1):
            e = engines[g]
            base, rows = blocks[g]
            d = _dist(torch, g, P, packed, metas, wires, e, "direct", emetas) if P > 1 else None
            ring.ring_search(d, torch, e, g, P, Xr.shape[0], base, schedule="direct")
            assert e.spec
            got = e.result()
            ref = oracle.knn(Xr, 32, rows=(base, rows))
            assert np.array_equal(got["idx"], ref["idx"]), (P, g)
            assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), (P, g)


@pytest.mark.parametrize("kind", ["negative", "real", "above255"])
@pytest.mark.parametrize("P", [1, 4])
def test_s8_fallback(knn, oracle, P, kind):
    import torch
    import mpiknn.ring as ring
    X = datasets.mnist_like(1600, 196, seed=2)[0]
    if kind == "negative":
        X[P * 100 + 3, 7] = -1.0          # one value below 0 (in one rank's block only)
    elif kind == "real":
        X = X / 255.0 + np.random.default_rng(1).normal(0, 1e-3, X.shape)
    else:
        X[50, 3] = 256.0
    m, n = X.shape
    R, blocks, engines, packed, metas, wires, emetas = _engines(torch, ring, knn, X, P)
    for g in range(P):
        e = engines[g]
        base, rows = blocks[g]
        d = _dist(torch, g, P, packed, metas, wires, e, "direct", emetas) if P > 1 else None
        ring.ring_search(d, torch, e, g, P, m, base, schedule="direct")
        assert not e.spec
        got = e.result()
        ref = oracle.knn(X, 30, rows=(base, rows))
        assert np.array_equal(got["idx"], ref["idx"]), (kind, P, g)
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), (kind, P, g)


def test_s8_speculative_begin_and_mismatch(knn, oracle):
    """P = 1: after a search begun from the byte block, the next one starts
    without reading its meta back (the last one's host meta as the hint) and
    checks it after the search; data the byte block cannot hold (a negative
    value) is then searched again from the element block -- every result
    equal to the oracle's."""
    import torch
    import mpiknn.ring as ring
    X = datasets.mnist_like(1500, 196, seed=8)[0]
    m, n = X.shape
    e = ring.GpuEngine(torch, 0, n, m, m, 30)
    for trial, Y in enumerate((X, X[::-1].copy(), np.where(X > 100, X - 200.0, X))):
        e.try_s8 = True
        e.pack(torch.from_numpy(np.ascontiguousarray(Y)).to("cuda:0"), layout_col=False)
        assert e.spec
        ring.ring_search(None, torch, e, 0, 1, m, 0)
        got = e.result()
        ref = oracle.knn(Y, 30)
        assert np.array_equal(got["idx"], ref["idx"]), trial
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), trial
        assert (e.spec_hint is not None) == (trial < 2), trial


def test_int8_research_of_uncertified(knn, oracle, monkeypatch):
    """Queries a 12-entry lane list cannot certify (tight clusters: most of a
    query's k + 1 nearest fall in one lane) are searched again on the int8
    contraction with 65-entry lists before any fp64 rescan; the results stay
    the oracle's, and fewer (here: no) queries reach the exact rescan.  One
    corpus split (KNN_SPLITS=1: the re-search keeps its own) makes the
    first pass overflow for sure: 2 lane lists of 12 hold a query's 24
    cluster mates."""
    import torch
    import mpiknn.ring as ring
    monkeypatch.setenv("KNN_SPLITS", "1")
    rng = np.random.default_rng(21)
    base = rng.integers(20, 236, (120, 64)).astype(np.float64)
    X = np.repeat(base, 25, axis=0) + rng.integers(-2, 3, (3000, 64))
    m, n = X.shape
    counts = {}
    for mode in ("off", "on"):
        if mode == "off":
            monkeypatch.setenv("KNN_NO_RESEARCH8", "1")
        else:
            monkeypatch.delenv("KNN_NO_RESEARCH8", raising=False)
        e = ring.GpuEngine(torch, 0, n, m, m, 30)
        e.pack(torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0"), layout_col=False)
        counts[mode] = ring.ring_search(None, torch, e, 0, 1, m, 0)
        assert e.ctx.contraction_bits() == 8
        got = e.result()
        ref = oracle.knn(X, 30)
        assert np.array_equal(got["idx"], ref["idx"]), mode
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), mode
    assert counts["off"] > 0, counts
    assert counts["on"] < counts["off"], counts
    # the re-search failing after k_resolve8 has rewritten rows
    # and the device count -- the exact rescan of the first pass's list
    # still gives the oracle's result
    monkeypatch.setenv("KNN_TEST_RESEARCH8_FAIL", "1")
    e = ring.GpuEngine(torch, 0, n, m, m, 30)
    e.pack(torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0"), layout_col=False)
    assert ring.ring_search(None, torch, e, 0, 1, m, 0) > 0   # the first pass's count, not the re-search's
    got = e.result()
    assert np.array_equal(got["idx"], ref["idx"])
    assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64))


@pytest.mark.parametrize("dtype,k", [("f64", 30), ("f32", 64)])
def test_s8_speculative_mismatch_real_valued(knn, oracle, dtype, k):
    """a speculative begin (the last search's host meta as
    the hint) on data that turns out real-valued -- the device meta says GEMM
    while the context holds no element rows.  k <= 32 takes the rank merge,
    k > 32 (fp32) k_merge; neither may read through the missing element
    block, the int8 re-search must not run, and the search is then repeated
    from the element block: every result equal to the oracle's."""
    import torch
    import mpiknn.ring as ring
    X = datasets.mnist_like(1300, 96, seed=12)[0]
    m, n = X.shape
    Xr = X / 255.0 + np.random.default_rng(3).normal(0, 1e-3, X.shape)
    e = ring.GpuEngine(torch, 0, n, m, m, k, dtype=dtype)
    for trial, Y in enumerate((X, Xr, X)):
        e.try_s8 = True
        Ys = Y.astype(np.float32) if dtype == "f32" else Y
        e.pack(torch.from_numpy(np.ascontiguousarray(Ys)).to("cuda:0"), layout_col=False)
        assert e.spec
        ring.ring_search(None, torch, e, 0, 1, m, 0)
        got = e.result()
        Yr = Ys.astype(np.float64)
        ref = oracle.knn(Yr, k)
        assert np.array_equal(got["idx"], ref["idx"]), trial
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), trial
        # the mismatch drops the hint: the search after it reads its meta back
        assert (e.spec_hint is not None) == (trial != 1), trial


@pytest.mark.parametrize("kl", ["12", "17"])
def test_int8_research_every_query_uncertified(knn, oracle, kl, monkeypatch):
    """the int8 re-search with nf == nq -- 2 rows repeated
    750 times, so every query's k nearest nonzero distances are a 750-way
    tie that overflows every 12- or 17-entry lane list of the first pass (a
    list holding only tied entries cannot certify) -- under both lane-list
    lengths: without the re-search all of them take the exact rescan; with
    it the 65-entry re-search over 31 splits gets nf == nq; exact either way."""
    import torch
    import mpiknn.ring as ring
    monkeypatch.setenv("KNN_I8_KL", kl)
    rng = np.random.default_rng(5)
    X = np.repeat(rng.integers(0, 256, (2, 64)).astype(np.float64), 750, axis=0)
    m, n = X.shape
    ref = oracle.knn(X, 30)
    for research in (False, True):
        if research:
            monkeypatch.delenv("KNN_NO_RESEARCH8", raising=False)
        else:
            monkeypatch.setenv("KNN_NO_RESEARCH8", "1")
        e = ring.GpuEngine(torch, 0, n, m, m, 30)
        e.pack(torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0"), layout_col=False)
        unresolved = ring.ring_search(None, torch, e, 0, 1, m, 0)
        assert e.ctx.contraction_bits() == 8
        if not research:
            assert unresolved == m     # the first pass certifies no query: the re-search gets nf == nq
        got = e.result()
        assert np.array_equal(got["idx"], ref["idx"]), research
        assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), research


@pytest.mark.parametrize("P", [2, 4])
def test_int8_research_ring_rank(knn, oracle, P, monkeypatch):
    """a ring rank's uncertified queries (direct schedule,
    byte blocks resident) are searched again on the int8 contraction over
    every byte block the rank holds (knn_ctx_research_blocks) before the
    element-block exchange of the rescan; clustered data with one corpus
    split (KNN_SPLITS=1) leaves some uncertified for sure.  Every rank equals
    the oracle's scan of its rows, with fewer queries left for the rescan
    than with KNN_NO_RESEARCH8=1."""
    import torch
    import mpiknn.ring as ring
    from test_gpu_ring_rotation import loopback_dist
    monkeypatch.setenv("KNN_SPLITS", "1")
    rng = np.random.default_rng(23)
    base_rows = rng.integers(20, 236, (120, 64)).astype(np.float64)
    X = np.repeat(base_rows, 25, axis=0) + rng.integers(-2, 3, (3000, 64))
    X = X[rng.permutation(len(X))]
    m, n = X.shape
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(X).to(dev)
    R, blocks = ring.partition(m, P)
    counts = {}
    for mode in ("off", "on"):
        if mode == "off":
            monkeypatch.setenv("KNN_NO_RESEARCH8", "1")
        else:
            monkeypatch.delenv("KNN_NO_RESEARCH8", raising=False)
        engines = []
        for g in range(P):
            b0, rows = blocks[g]
            e = ring.GpuEngine(torch, 0, n, R, rows, 30)
            e.pack(Xd[b0:b0 + rows], layout_col=False, elements=True)
            engines.append(e)
        packed = [e.qb.clone() for e in engines]
        metas = torch.stack([e.meta for e in engines])
        wires = []
        for e in engines:
            w = torch.empty(knn.wire_bytes(R, n), dtype=torch.uint8, device=dev)
            knn.wire_pack(w.data_ptr(), e.qb.data_ptr(), R, n, "f64", e.stream())
            wires.append(w)
        total = 0
        for g, e in enumerate(engines):
            b0, rows = blocks[g]
            d = loopback_dist(torch, g, P, packed, metas, wires, e, "direct")
            total += ring.ring_search(d, torch, e, g, P, m, b0, schedule="direct")
            assert e.ctx.shadow() == 2
            got = e.result()
            ref = oracle.knn(X, 30, rows=(b0, rows))
            assert np.array_equal(got["idx"], ref["idx"]), (mode, P, g)
            assert np.array_equal(got["distance"].view(np.uint64), ref["distance"].view(np.uint64)), (mode, P, g)
        counts[mode] = total
    assert counts["off"] > 0, counts
    assert counts["on"] < counts["off"], counts
