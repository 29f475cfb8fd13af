# round-5 session 12: the own block's GEMM merge shared with the fused step -- parity + P=8 emulation
set -o pipefail
mkdir -p gpurun_out/s12
timeout -k 10 700 python -u -m pytest tests/test_gpu_ring_rotation.py tests/test_gpu_parity.py tests/test_gpu_fullsize_ring.py tests/test_gpu_f32.py tests/test_gpu_rccl_self.py tests/test_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s12/tests.log 2>&1 || { tail -40 gpurun_out/s12/tests.log; exit 1; }
tail -1 gpurun_out/s12/tests.log
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1,2,4,8 --steps 5 > gpurun_out/s12/emu_mr.log 2>&1 || { tail -20 gpurun_out/s12/emu_mr.log; exit 1; }
grep '"P"' gpurun_out/s12/emu_mr.log
timeout -k 10 200 python3 bench.py --workload mnist-real --steps 10 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/s12/mr.log 2>&1 || { tail -20 gpurun_out/s12/mr.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s12/mr.log | tr '\n' ' '; echo " mnist-real"
