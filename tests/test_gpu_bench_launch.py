"""bench.py --gpus N on the GPU box.

With fewer than N GPUs visible, `bench.py --gpus N` must refuse before any
rank starts (exit 2, no JSON line) -- never print a P = 1 line under an
N-GPU request.  With N GPUs visible (a multi-GPU node) it starts N ranks
over RCCL; that run is the driver's, so only the refusal is tested here.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def test_bench_gpus_more_than_visible_refuses():
    import torch
    n = torch.cuda.device_count()
    want = n + 1
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "KNN_BENCH_TEST_ENGINE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(want), "--steps", "1",
                        "--warmup", "0", "--secondary-steps", "0", "--no-cpu-baseline"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "visible GPUs" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
