"""The split fp16 rows of real-valued blocks (knn_split_pack, the conversion
every split-filter step runs on its corpus blocks): byte for byte the
restatement below, for fp64 and fp32 blocks, ragged n (a partial last
32-feature group), values over many binades including ones whose lo half
is subnormal or zero, and several scales.

Restatement (the filter's representation, knn_kernels.hip k_shadow_split):
x = scale * v in the block's precision (scale a power of two: exact), hi =
RN16(x), lo = RN16(x - hi), each rounded once from that precision (numpy's
float64 -> float16 conversion rounds once; x - hi is exact); per row and 32-feature group the 32
hi halves then the 32 lo halves; zero past n.  This is the product's own
representation, not the reference's arithmetic (the reference's S is
recomputed exactly in k_merge), so a numpy restatement is its oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def split_rows(V, n, scale, dt):
    T = np.float64 if dt == "f64" else np.float32
    x = V.astype(T) * T(scale)
    hi = x.astype(np.float16)
    lo = (x - hi.astype(T)).astype(np.float16)
    m = V.shape[0]
    npd = (n + 31) // 32 * 32
    H = np.zeros((m, npd), np.float16)
    L = np.zeros((m, npd), np.float16)
    H[:, :n] = hi
    L[:, :n] = lo
    out = np.concatenate([H.reshape(m, npd // 32, 32), L.reshape(m, npd // 32, 32)], axis=2)
    return out.reshape(m, npd * 2).view(np.uint8)


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("n", [784, 100, 33, 960])
def test_split_pack_matches_restatement(knn, dt, n):
    import torch
    rng = np.random.default_rng(n + (1 if dt == "f32" else 0))
    m = 300
    # magnitudes over ~30 binades, signs, exact zeros, values whose scaled
    # form is an fp16 integer (lo = 0)
    V = rng.standard_normal((m, n)) * np.exp2(rng.integers(-20, 10, (m, n)))
    V[rng.random((m, n)) < 0.05] = 0.0
    V[3] = np.round(rng.uniform(-100, 100, n))
    if dt == "f32":
        V = V.astype(np.float32).astype(np.float64)
    tdt = torch.float32 if dt == "f32" else torch.float64
    src = torch.from_numpy(V).to("cuda:0", tdt).contiguous()
    blk = torch.zeros(knn.block_bytes(m, n, dt), dtype=torch.uint8, device="cuda:0")
    knn.block_pack(blk.data_ptr(), m, m, n, src.data_ptr(), n, knn.ROWMAJOR, dtype=dt, src_dtype=dt)
    maxabs = float(np.abs(V).max())
    e = int(np.floor(np.log2(maxabs)))
    for scale in (2.0 ** (13 - e), 2.0 ** (13 - e - 7), 1.0):
        out = torch.full((knn.split_bytes(m, n),), 0xAB, dtype=torch.uint8, device="cuda:0")
        knn.split_pack(out.data_ptr(), blk.data_ptr(), m, n, dtype=dt, scale=scale)
        torch.cuda.synchronize()
        rs = (n + 31) // 32 * 32 * 4
        got = out.cpu().numpy()[:m * rs].reshape(m, rs)
        want = split_rows(V, n, scale, dt)
        bad = np.argwhere(got != want)
        assert bad.size == 0, (scale, bad[:5])


def test_split_pack_rejects(knn):
    with pytest.raises(knn.KnnError):
        knn.split_pack(1, 1, 10, 8, dtype="f64", scale=3.0)   # not a power of two
    with pytest.raises(knn.KnnError):
        knn.split_pack(0, 1, 10, 8, dtype="f64", scale=1.0)
