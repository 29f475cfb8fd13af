"""bench.py --gpus N: the rank launcher and the world-size guards (CPU).

VERDICT r05 item 1: `python bench.py --gpus N` with no launcher must run N
ranks (one per GPU) and print ONE rank-0 line with n_gpus = N, or exit
non-zero -- never a P = 1 line.  The multi-rank path runs here under gloo
with the CPU stand-in engine (tests/bench_standin.py, via
KNN_BENCH_TEST_ENGINE); the GPU box's refusal when fewer than N GPUs are
visible is tests/test_gpu_bench_launch.py.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--m", "240", "--n", "784", "--steps", "2", "--warmup", "1", "--secondary-steps", "0",
         "--check", "8"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                              "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env["KNN_BENCH_TEST_ENGINE"] = "bench_standin:make"
    env.update(kw)
    return env


def _lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("gpus,schedule", [(2, "direct"), (3, "ring")])
def test_bench_gpus_n_runs_n_ranks(gpus, schedule):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus)] + SMALL, cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=_env(KNN_RING_SCHEDULE=schedule))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout          # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == gpus
    assert line["config"]["parallelism"] == "ring%d" % gpus
    assert line["launcher"] == "bench.py"
    assert line["rccl_world"] is None         # gloo stand-in, not RCCL
    assert line["check"]["mismatches"] == 0   # rank 0's rows against the oracle
    assert np.isclose(line["value"], 240 / (line["ms_per_step"] * 1e-3))
    assert line["cpu_baseline"] is None       # P > 1: no CPU leg


def test_bench_world_size_must_match_gpus():
    """under a launcher, --gpus and WORLD_SIZE must agree"""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + SMALL, cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
    assert not _lines(r.stdout)


def test_bench_refuses_more_ranks_than_gpus():
    """no stand-in: the launcher counts the visible GPUs (none here) and
    refuses before starting any rank"""
    env = _env()
    env.pop("KNN_BENCH_TEST_ENGINE")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + SMALL, cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "visible GPUs" in r.stderr
    assert not _lines(r.stdout)


def test_bench_failed_rank_fails_the_job():
    """a rank that dies ends the launch with a non-zero exit (its peers are
    stopped, no line is printed)"""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + SMALL, cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=_env(KNN_BENCH_TEST_ENGINE="bench_standin:nosuch"))
    assert r.returncode != 0
    assert not _lines(r.stdout)
