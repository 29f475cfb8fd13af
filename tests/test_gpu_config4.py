"""BASELINE configs[4] at its stated size: a GIST-shaped 4M x 960 fp32
corpus, k = 100, partitioned over 8 ranks.

One rank's work on the node is mpi-knn-parallel_non_blocking.c:233-258 for
every block: its R = 500K query rows against all eight 500K-row blocks.
Here that share runs through mpiknn.ring.ring_search -- bench.py's per-rank
code, direct schedule -- on one GPU, the other ranks' blocks supplied by the
loopback stand-in for torch.distributed (tests/test_gpu_ring_rotation.py):
the split-fp16 filter (knn_ctx_split), its certificate at 4M rows, the fp64
re-rank and the exact rescan of whatever stays uncertified, at full size.

For ranks 0, 3 and 7 (first, interior, last block): 16 sampled query rows
bit for bit against the oracle's scan of the fp32 points
(oracle.knn_f32 == oracle.knn(X.astype(float64)), serial:72-93), and every
row of the share property-checked (sorted, positive, in range, no self, no
repeats).  The corpus is generated on the device (the 256-centre mixture in
[0, 1) of tools/ring_emulate.py) to keep the generation off the host.
"""
import numpy as np
import pytest

from test_gpu_ring_rotation import loopback_dist

pytestmark = pytest.mark.gpu

M, N, K, P = 4_000_000, 960, 100, 8


def gist_device(torch, m, n, dev, seed=0x6157):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    centres = torch.rand((256, n), generator=g, device=dev) * 0.5 + 0.1
    X = torch.empty((m, n), dtype=torch.float32, device=dev)
    top = float(np.nextafter(np.float32(1), np.float32(0)))
    step = 1 << 18
    for lo in range(0, m, step):
        hi = min(m, lo + step)
        lab = torch.randint(0, 256, (hi - lo,), generator=g, device=dev)
        X[lo:hi] = (centres[lab] + 0.08 * torch.randn((hi - lo, n), generator=g, device=dev)).clamp_(0.0, top)
    return X


@pytest.mark.timeout(900)
def test_gist_4m_rank_shares(knn, oracle):
    import torch
    import mpiknn.ring as ring
    dev = torch.device("cuda", 0)
    Xd = gist_device(torch, M, N, dev)
    R, blocks = ring.partition(M, P)
    nb = knn.block_bytes(R, N, "f32")
    mo = knn.block_meta_offset(R, N, "f32")
    stream = torch.cuda.current_stream(dev).cuda_stream
    packed = []
    for base, rows in blocks:
        t = torch.zeros(nb, dtype=torch.uint8, device=dev)
        knn.block_pack(t.data_ptr(), R, rows, N, Xd[base:base + rows].data_ptr(), N, knn.ROWMAJOR, stream,
                       dtype="f32", src_dtype="f32")
        packed.append(t)
    metas = torch.stack([t[mo:mo + 8 * knn.META_DOUBLES].view(torch.float64) for t in packed])
    X = Xd.cpu().numpy()        # the oracle's copy (15.4 GB); the device copy stays for the packs
    rng = np.random.default_rng(4)
    checked = 0
    for g, nrows in ((0, 6), (3, 5), (7, 5)):
        base, rows = blocks[g]
        e = ring.GpuEngine(torch, 0, N, R, rows, K, dtype="f32")
        e.pack(Xd[base:base + rows], layout_col=False)
        assert not e.spec                              # n = 960 > 896: element blocks
        d = loopback_dist(torch, g, P, packed, metas, packed, e, "direct")
        unresolved = ring.ring_search(d, torch, e, g, P, M, base, schedule="direct")
        assert e.ctx.split() == 1, "configs[4] runs the split fp16 filter"
        got = e.result()
        # every row of the share
        dist, idx = got["distance"], got["idx"]
        assert np.all(np.isfinite(dist)) and np.all(dist > 0)
        assert np.all(dist[:, 1:] >= dist[:, :-1])
        assert np.all((idx >= 1) & (idx <= M))
        assert not np.any(idx == (base + np.arange(rows) + 1)[:, None])
        s = np.sort(idx, axis=1)
        assert not np.any(s[:, 1:] == s[:, :-1])
        # sampled rows bit for bit against the oracle (first, last, random)
        pick = sorted({0, rows - 1, *rng.integers(1, rows - 1, nrows - 2).tolist()})
        ref = oracle.knn_f32(X, K, [base + r for r in pick])    # one thread a row
        for j, r in enumerate(pick):
            assert np.array_equal(got[r]["idx"], ref[j]["idx"]), (g, r, unresolved)
            assert np.array_equal(got[r]["distance"].view(np.uint64), ref[j]["distance"].view(np.uint64)), (g, r)
            checked += 1
        del e, d
        torch.cuda.empty_cache()
    assert checked >= 16
