"""Where the host's ~45 us between a search's last kernel and the next
step's first launch goes: bench.py's step under cProfile (P = 1, mnist),
the per-call costs of the Python frames and ctypes calls of one step.

  python tools/probe/host_prof.py [steps]   (GPU box)
"""
import cProfile
import os
import pstats
import sys

sys.argv = [sys.argv[0], "--workload", "mnist", "--steps", sys.argv[1] if len(sys.argv) > 1 else "40",
            "--warmup", "3", "--no-cpu-baseline", "--secondary-steps", "0", "--check", "0"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

out = os.path.join("gpurun_out", "host_prof.out")
os.makedirs("gpurun_out", exist_ok=True)
cProfile.run("bench.main()", out)
st = pstats.Stats(out)
st.sort_stats("tottime").print_stats(45)
