"""Solo searches (knn_ctx_set_solo): a P = 1 search's distance kernel and
merge on the caller's stream, and the meta check through knn_ctx_search_meta.

ring_search() turns solo on at P = 1 (bench.py's path, knn-serial.c:72-93
over the whole corpus in one step).  Every result must equal the oracle's,
with solo on and off, across the speculative byte-block begin (hint from the
last search, checked after end() against the meta the kernels read), a data
change that invalidates the hint, and a solo context that is handed two
steps after all (the step schedule takes over after the first).
"""
import numpy as np
import pytest

import datasets
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _engine(X, k=30):
    import torch
    import mpiknn.ring as ring
    m, n = X.shape
    e = ring.GpuEngine(torch, 0, n, m, m, k)
    src = torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0")
    return e, src


def test_solo_ring_search_p1_hint_cycle(oracle):
    """P = 1 through ring_search (solo): first search (meta read back), then
    from the hint (checked with knn_ctx_search_meta), then on rescaled data
    (the hint no longer matches: searched again from the element block),
    then real-valued data (no byte block at all) -- every result exact."""
    import torch
    import mpiknn.ring as ring
    X = datasets.mnist_like(3000, 784, seed=61)[0]
    e, _ = _engine(X)
    cases = [X, X, np.clip(X * 0.5, 0, 255).round(), X / 255.0 + 1e-3]
    for i, Xs in enumerate(cases):
        src = torch.from_numpy(np.ascontiguousarray(Xs)).to("cuda:0")
        e.pack(src, layout_col=False)
        ring.ring_search(None, torch, e, 0, 1, Xs.shape[0], 0)
        assert_same(e.result(), oracle.knn(Xs, 30), "solo P=1 search %d" % i)
        meta = e.ctx.search_meta()
        assert meta[0] == float(np.abs(Xs).max()), (i, meta)


@pytest.mark.parametrize("solo", [False, True])
def test_solo_context_two_steps_falls_back(knn, oracle, solo):
    """A solo context given two steps: the first runs on the caller's
    stream, the second goes back to the step schedule -- results exact and
    byte-identical either way."""
    import torch
    X = datasets.mnist_like(2000, 784, seed=62)[0]
    m, n = X.shape
    half = m // 2
    dev = "cuda:0"
    stream = torch.cuda.current_stream().cuda_stream
    src = torch.from_numpy(np.ascontiguousarray(X)).to(dev)
    qb = torch.zeros(knn.block_bytes(m, n), dtype=torch.uint8, device=dev)
    knn.block_pack(qb.data_ptr(), m, m, n, src.data_ptr(), n, knn.ROWMAJOR, stream)
    blocks = []
    for b in range(2):
        bb = torch.zeros(knn.block_bytes(m, n), dtype=torch.uint8, device=dev)
        part = src[b * half:(b + 1) * half].contiguous()
        knn.block_pack(bb.data_ptr(), m, half, n, part.data_ptr(), n, knn.ROWMAJOR, stream)
        blocks.append((bb, part))
    ctx = knn.Context(0, m, n, m, 30, "f64")
    ctx.set_solo(solo)
    out = torch.zeros(m * 30 * 16, dtype=torch.uint8, device=dev)
    meta_ptr = qb.data_ptr() + knn.block_meta_offset(m, n)
    ctx.begin(qb.data_ptr(), m, 0, meta_ptr, stream)
    for b, (bb, _) in enumerate(blocks):
        ctx.step(bb.data_ptr(), half, b * half, stream)
    unresolved = ctx.end(out.data_ptr(), stream)
    if unresolved:
        for b, (bb, _) in enumerate(blocks):
            ctx.rescan_step(bb.data_ptr(), half, b * half, stream)
        ctx.rescan_end(out.data_ptr(), stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(knn.NB_DTYPE).reshape(m, 30)
    assert_same(got, oracle.knn(X, 30), "solo=%s two steps" % solo)
    # and the same context again, one step over the whole query block
    ctx.begin(qb.data_ptr(), m, 0, meta_ptr, stream)
    ctx.step(qb.data_ptr(), m, 0, stream)
    ctx.end(out.data_ptr(), stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(knn.NB_DTYPE).reshape(m, 30)
    assert_same(got, oracle.knn(X, 30), "solo=%s one step after two" % solo)
    ctx.close()
