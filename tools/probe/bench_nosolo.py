"""bench.py with knn_ctx_set_solo held off (A/B timing of the solo P = 1
stream path; diagnostic only): python tools/probe/bench_nosolo.py ARGS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpi-knn_amd")]
import mpiknn  # noqa: E402

_orig = mpiknn.Context.set_solo
mpiknn.Context.set_solo = lambda self, on: _orig(self, False)
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
