"""The three drop-in executables keep the reference's CLI and stdout
contract (serial:65,98,130; blk:272-273; nb:208-226,290-292) and print the
pinned Matches counts on the digits corpus written as a MAT file."""
import os
import re
import subprocess

import numpy as np
import pytest
import scipy.io

import datasets

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "mpi-knn_amd", "bin")


def _run(tmp_path, exe, args=(), compress=True, extra_env=None):
    X, y = datasets.digits()
    path = tmp_path / "mnist_train.mat"
    scipy.io.savemat(str(path), {"train_X": X, "train_labels": y.reshape(-1, 1)},
                     do_compression=compress)
    env = dict(os.environ)
    env.pop("KNN_MAT", None)
    env.pop("KNN_MPI_COMPAT", None)
    env.update(extra_env or {})
    r = subprocess.run([os.path.join(BIN, exe)] + list(args), cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_knn_serial(tmp_path):
    out = _run(tmp_path, "knn-serial")
    lines = out.splitlines()
    assert lines[0] == "Number of Classes: 10"
    assert lines[1] == "Sorting done"
    assert re.fullmatch(r"Clock time = \d+\.\d{6}", lines[2])
    assert lines[3] == "Matches: 1636"


def test_mpi_blocking_one_gpu(tmp_path):
    out = _run(tmp_path, "mpi-knn-parallel_blocking", ["1", "4"], compress=False)
    lines = out.splitlines()
    assert lines[0] == "Matches: 1635"
    assert re.fullmatch(r"KNN time: \d+\.\d{6}", lines[1])


def test_mpi_non_blocking_one_gpu(tmp_path):
    out = _run(tmp_path, "mpi-knn-parallel_non_blocking", ["1", "1"])
    lines = out.splitlines()
    assert lines[0] == "Matches1635"
    assert re.fullmatch(r"Time :\d+\.\d{6}", lines[1])


def test_mpi_blocking_multi_gpu(tmp_path):
    import torch
    ng = torch.cuda.device_count()
    if ng < 2:
        pytest.skip("needs 2+ GPUs (single-process RCCL ring)")
    out = _run(tmp_path, "mpi-knn-parallel_blocking", [str(ng), "1"])
    counts = [int(v) for v in re.findall(r"Matches: (\d+)", out)]
    assert sum(counts) == 1635 and len(counts) == ng


@pytest.mark.parametrize("exe,fmt", [("mpi-knn-parallel_blocking", r"Matches: (\d+)"),
                                     ("mpi-knn-parallel_non_blocking", r"Matches(\d+)")])
def test_mpi_bug_compat_mode(tmp_path, exe, fmt):
    """KNN_MPI_COMPAT=1: per-rank Matches of the reference's own (F5) lists,
    against the oracle's restatement + the MPI vote rule."""
    import oracle
    X, y = datasets.digits()
    P = 3
    out = _run(tmp_path, exe, [str(P), "1"], extra_env={"KNN_MPI_COMPAT": "1"})
    counts = [int(v) for v in re.findall(fmt, out)]
    nb = oracle.mpi_compat(X, 30, P, labels=y)
    R = X.shape[0] // P
    pred, _ = oracle.classify(nb, y, 10, oracle.VOTE_MPI)
    want = [int((np.asarray(pred[r * R:(r + 1) * R]) == y[r * R:(r + 1) * R]).sum())
            for r in range(P)]
    assert counts == want
