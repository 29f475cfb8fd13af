"""GPU vote (knn_classify_device, k_vote) against the host vote
(knn_classify, knn_vote.c -- itself checked against the oracle's vote in
test_abi.py), on device-resident records: predictions, match count and the
filled .label of every record (blk:176), for the three rules."""
import numpy as np
import pytest

import datasets

pytestmark = pytest.mark.gpu


def device_vote(knn, nb, labels, nclasses, rule, q_base=0):
    import torch
    dev = torch.device("cuda", 0)
    d_nb = torch.from_numpy(np.ascontiguousarray(nb).view(np.uint8).reshape(-1).copy()).to(dev)
    d_lab = torch.from_numpy(np.ascontiguousarray(labels, dtype=np.float64)).to(dev)
    m, k = nb.shape
    d_pred = torch.full((max(m, 1),), -7, dtype=torch.int32, device=dev)
    d_match = torch.zeros(1, dtype=torch.int64, device=dev)
    knn.classify_device(d_nb.data_ptr(), m, k, nclasses, rule, d_lab.data_ptr(), len(labels),
                        q_base, d_pred.data_ptr(), d_match.data_ptr(),
                        torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    out = d_nb.cpu().numpy().view(knn.NB_DTYPE).reshape(m, k)
    return out, d_pred.cpu().numpy()[:m], int(d_match.cpu().item())


def expected_labels(nb, labels):
    idx = nb["idx"]
    ok = (idx > 0) & (idx <= len(labels))
    lab = np.zeros(idx.shape, dtype=np.int32)
    lab[ok] = labels[idx[ok] - 1].astype(np.int32)
    return np.where(ok, lab, nb["label"])


@pytest.mark.parametrize("rule", [0, 1, 2])
def test_vote_digits(knn, oracle, rule):
    X, y = datasets.digits()
    nb = oracle.knn(X, 30).view(knn.NB_DTYPE)            # labels not filled
    pred_h, match_h = knn.classify(nb, y, 10, rule)
    out, pred, match = device_vote(knn, nb, y, 10, rule)
    assert (pred == pred_h).all() and match == match_h
    assert (out["label"] == expected_labels(nb, y)).all()
    assert (out["idx"] == nb["idx"]).all()
    if rule == 0:
        assert match == 1636                                # SURVEY sec.4 (serial vote)


def test_vote_after_device_search(knn):
    """search -> vote without leaving the device (fp32, k = 100)."""
    import torch
    import mpiknn.ring as ring
    X, y = datasets.mnist_like(1500, 784, seed=3)
    m, n = X.shape
    dev = torch.device("cuda", 0)
    e = ring.GpuEngine(torch, 0, n, m, m, 100, dtype="f32")
    e.pack(torch.from_numpy(X).to(dev), layout_col=False, elements=True)
    e.begin(0)
    e.step(e.qb, m, 0)
    if e.end():
        e.step(e.qb, m, 0, rescan=True)
        e.rescan_end()
    d_lab = torch.from_numpy(y).to(dev)
    d_pred = torch.zeros(m, dtype=torch.int32, device=dev)
    d_match = torch.zeros(1, dtype=torch.int64, device=dev)
    knn.classify_device(e.out.data_ptr(), m, 100, 10, knn.VOTE_MAJORITY, d_lab.data_ptr(), m, 0,
                        d_pred.data_ptr(), d_match.data_ptr(), e.stream())
    torch.cuda.synchronize()
    host = e.result()
    pred_h, match_h = knn.classify(host, y, 10, knn.VOTE_MAJORITY)
    assert (d_pred.cpu().numpy() == pred_h).all() and int(d_match.item()) == match_h
    assert (host["label"] == expected_labels(host, y)).all()


def test_vote_edges(knn):
    """empty slots, ids past nlabels, labels outside 1..nclasses, k = 1 and
    odd k, m not a multiple of 4, a q_base offset (a ring rank's rows)."""
    rng = np.random.default_rng(4)
    m, k, ncls = 37, 7, 5
    labels = rng.integers(0, 7, 200).astype(np.float64)     # 0 and 6 are out of range
    nb = np.zeros((m, k), dtype=knn.NB_DTYPE)
    nb["idx"] = rng.integers(-1, 230, (m, k))               # <= 0 empty, > 200 unknown
    nb["distance"] = np.sort(rng.uniform(0, 1, (m, k)), axis=1)
    nb["label"] = -5
    for rule in (0, 1, 2):
        for q_base in (0, 150):
            out, pred, match = device_vote(knn, nb, labels, ncls, rule, q_base)
            # host twin (it has no nlabels: ids past 200 get label 0 there,
            # which is out of range, hence skipped like the device does)
            lab_h = np.concatenate([labels, np.zeros(64)])
            pred_h, _ = knn.classify(nb, lab_h, ncls, rule)
            own = lab_h[q_base:q_base + m]
            match_h = int(((pred_h == own) & (np.arange(q_base, q_base + m) < len(labels))).sum())
            assert (pred == pred_h).all(), (rule, q_base)
            assert match == match_h, (rule, q_base)
            assert (out["label"] == expected_labels(nb, labels)).all()
    nb1 = nb[:, :1].copy()
    _, pred, _ = device_vote(knn, nb1, labels, ncls, 0)
    assert (pred == knn.classify(nb1, np.concatenate([labels, np.zeros(64)]), ncls, 0)[0]).all()
