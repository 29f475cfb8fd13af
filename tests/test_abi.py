"""The C-ABI library without a GPU: it loads, exports every entry point
include/knn.h declares, and its host-only pieces (vote, MAT reader, error
paths) behave.  No device compute is attempted here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import datasets

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "knn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(knn_[a-z_0-9]+)\s*\(", src)))


def test_every_declared_symbol_exported(knn):
    names = header_functions()
    assert len(names) >= 19
    out = subprocess.check_output(["nm", "-D", "--defined-only", knn.LIB_PATH]).decode()
    exported = set(re.findall(r" T (knn_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(knn.API_SYMBOLS) == set(names)


def test_internal_symbols_hidden(knn):
    out = subprocess.check_output(["nm", "-D", "--defined-only", knn.LIB_PATH]).decode()
    exported = set(re.findall(r" T (knn_\w+)", out))
    assert exported == set(header_functions()), sorted(exported - set(header_functions()))


def test_strerror(knn):
    assert knn.strerror(0) == "ok"
    assert "device" in knn.strerror(knn.ERR_NODEVICE)
    assert knn.strerror(999) == "unknown status"


def test_invalid_arguments(knn):
    lib = knn.lib
    out = np.zeros((4, 3), dtype=knn.NB_DTYPE)
    X = np.ones((4, 2))
    p = X.ctypes.data_as(ctypes.c_void_p)
    o = out.ctypes.data_as(ctypes.c_void_p)
    assert lib.knn_search(None, 4, 2, 1, None, 3, 1, 0, o) == knn.ERR_INVALID
    assert lib.knn_search(p, 4, 2, 7, None, 3, 1, 0, o) == knn.ERR_INVALID
    assert lib.knn_search(p, 4, 2, 1, None, 33, 1, 0, o) == knn.ERR_UNSUPPORTED
    assert lib.knn_search(p, 4, 2, 1, None, 3, 1, 2, o) == knn.ERR_UNSUPPORTED  # no such dtype
    # k limits: fp64 32, fp32 128 (include/knn.h KNN_MAX_K / KNN_MAX_K_F32)
    assert lib.knn_search(p, 4, 2, 1, None, 129, 1, 1, o) == knn.ERR_UNSUPPORTED
    assert lib.knn_ctx_create_dt(ctypes.byref(h := ctypes.c_void_p()), 0, 4, 2, 4, 33, 0) \
        == knn.ERR_INVALID
    assert lib.knn_ctx_create_dt(ctypes.byref(h), 0, 4, 2, 4, 129, 1) == knn.ERR_INVALID
    assert knn.MAX_K == 32 and knn.MAX_K_F32 == 128
    q = ctypes.c_void_p(8)   # never dereferenced: argument checks come first
    assert lib.knn_classify_device(None, 4, 3, 10, 0, q, 4, 0, None, None, None) == knn.ERR_INVALID
    assert lib.knn_classify_device(q, 4, 3, 10, 9, q, 4, 0, None, None, None) == knn.ERR_INVALID
    assert lib.knn_classify_device(q, 4, 3, 2000, 0, q, 4, 0, None, None, None) == \
        knn.ERR_UNSUPPORTED
    assert lib.knn_search(p, 4, 2, 1, None, 3, 0, 0, o) == knn.ERR_INVALID
    h = ctypes.c_void_p()
    assert lib.knn_ctx_create(ctypes.byref(h), 0, 0, 2, 4, 3) == knn.ERR_INVALID
    assert lib.knn_block_pack(None, 4, 4, 2, None, 4, 0, None) == knn.ERR_INVALID
    assert lib.knn_ctx_create_dt(ctypes.byref(h), 0, 4, 2, 4, 3, 5) == knn.ERR_INVALID
    assert lib.knn_block_pack_dt(None, 1, 4, 4, 2, None, 0, 4, 0, None) == knn.ERR_INVALID
    assert lib.knn_block_pack_dt(p, 3, 4, 4, 2, p, 0, 4, 0, None) == knn.ERR_INVALID


def test_block_layout(knn):
    # rows padded to 128, features to 16, + norms + 8 meta doubles
    assert knn.block_bytes(60000, 784) == (60032 * 784 + 60032 + 8) * 8
    assert knn.block_meta_offset(1, 1) == (128 * 16 + 128) * 8
    # fp32 blocks: features padded to 32 (one 128-byte chunk), fp32 norms,
    # then the same 8 fp64 meta words
    assert knn.block_bytes(60000, 784, "f32") == (60032 * 800 + 60032) * 4 + 64
    assert knn.block_meta_offset(1000, 128, "f32") == (1024 * 128 + 1024) * 4
    assert knn.lib.knn_block_bytes_dt(10, 10, 7) == 0


@pytest.mark.parametrize("rule", [0, 1, 2])
def test_classify_matches_oracle(knn, oracle, rule):
    X, y = datasets.digits()
    nb = oracle.knn(X, 30, labels=y)
    nb2 = nb.view(knn.NB_DTYPE)
    p_ref, m_ref = oracle.classify(nb, y, 10, rule)
    p, m = knn.classify(nb2, y, 10, rule)
    assert m == m_ref and np.array_equal(p, p_ref)


def test_classify_empty_slots(knn):
    # fewer than k neighbours: idx 0 slots are skipped (the reference reads
    # labels[-1] there)
    nb = np.zeros((2, 4), dtype=knn.NB_DTYPE)
    nb["idx"] = [[2, 0, 0, 0], [1, 0, 0, 0]]
    labels = np.array([3.0, 5.0])
    pred, m = knn.classify(nb, labels, 10, knn.VOTE_SERIAL)
    assert list(pred) == [5, 3] and m == 0


def test_no_device_reports_cleanly(knn):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(knn.KnnError) as e:
        knn.search(np.ones((5, 3)), 2)
    assert e.value.status == knn.ERR_NODEVICE


def test_header_constants_mirrored(knn):
    """mpiknn mirrors the knn.h constants the ring drivers size buffers by."""
    import re
    src = open(os.path.join(ROOT, "include", "knn.h")).read()
    assert int(re.search(r"#define KNN_STEP_LAG (\d+)", src).group(1)) == knn.STEP_LAG
