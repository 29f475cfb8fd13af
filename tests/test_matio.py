"""knn_load_mat (csrc/knn_matio.c) against files written by scipy.io.savemat.

Replaces the MATLAB MAT-API calls of serial:40-52 / blk:64-68.  MAT level 5
(-v6, uncompressed) and v7 (zlib miCOMPRESSED) containers, numeric classes
converted to double like mxGetPr of a double array; v7.3 (HDF5) refused.
"""
import os

import numpy as np
import pytest
import scipy.io

import datasets


@pytest.mark.parametrize("compress", [False, True])
@pytest.mark.parametrize("dtype", [np.float64, np.uint8, np.int16, np.float32, np.int32])
def test_roundtrip(knn, tmp_path, compress, dtype):
    X, y = datasets.digits()
    Xd = X[:500].astype(dtype)
    path = str(tmp_path / "mnist_train.mat")
    scipy.io.savemat(path, {"junk": np.arange(7.0), "train_X": Xd,
                            "train_labels": y[:500].reshape(-1, 1)}, do_compression=compress)
    Xr, yr = knn.load_mat(path)
    assert Xr.shape == (500, 64)
    assert np.array_equal(Xr, Xd.astype(np.float64))
    assert np.array_equal(yr, y[:500])


def test_real_valued_exact_bits(knn, tmp_path):
    X, y = datasets.digits_real()
    path = str(tmp_path / "svd.mat")
    scipy.io.savemat(path, {"train_X": X, "train_labels": y}, do_compression=True)
    Xr, yr = knn.load_mat(path)
    assert np.array_equal(Xr.view(np.uint64), X.view(np.uint64))


def test_errors(knn, tmp_path):
    with pytest.raises(knn.KnnError) as e:
        knn.load_mat(str(tmp_path / "absent.mat"))
    assert e.value.status == knn.ERR_IO
    path = str(tmp_path / "other.mat")
    scipy.io.savemat(path, {"A": np.ones((3, 3))})
    with pytest.raises(knn.KnnError) as e:
        knn.load_mat(path)
    assert e.value.status == knn.ERR_FORMAT
    # a v7.3 file: 512-byte MAT header followed by an HDF5 superblock
    h5 = tmp_path / "v73.mat"
    hdr = b"MATLAB 7.3 MAT-file, Platform: GLNXA64, HDF5 schema 1.00 .".ljust(116, b" ")
    h5.write_bytes(hdr + b"\0" * 8 + b"\x00\x02IM" + b"\0" * 384 + b"\x89HDF\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(knn.KnnError) as e:
        knn.load_mat(str(h5))
    assert e.value.status == knn.ERR_UNSUPPORTED
    bad = tmp_path / "bad.mat"
    bad.write_bytes(b"x" * 200)
    with pytest.raises(knn.KnnError) as e:
        knn.load_mat(str(bad))
    assert e.value.status == knn.ERR_FORMAT


def test_no_labels_variable_ok(knn, tmp_path):
    path = str(tmp_path / "x.mat")
    scipy.io.savemat(path, {"train_X": np.arange(12.0).reshape(3, 4)})
    X, lab = knn.load_mat(path, lvar=None)
    assert lab is None and np.array_equal(X, np.arange(12.0).reshape(3, 4))


@pytest.mark.parametrize("dims", [(0x7fffffff, 0x7fffffff), (-5, 3), (5, -3), (0x40000000, 8)])
def test_malformed_dims_rejected(knn, tmp_path, dims):
    """Crafted dims must fail cleanly (KNN_ERR_FORMAT), never size a buffer
    from a wrapped product: 8-byte classes, negative and huge dims."""
    path = tmp_path / "crafted.mat"
    X = np.arange(15, dtype=np.int64).reshape(5, 3)
    scipy.io.savemat(str(path), {"train_X": X}, do_compression=False)
    raw = bytearray(path.read_bytes())
    at = raw.find(np.array([5, 3], dtype="<i4").tobytes())
    assert at > 0
    raw[at:at + 8] = np.array(dims, dtype="<i4").tobytes()
    path.write_bytes(bytes(raw))
    with pytest.raises(knn.KnnError) as e:
        knn.load_mat(str(path), lvar=None)
    assert e.value.status == knn.ERR_FORMAT
