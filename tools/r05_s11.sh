# round-5 session 11: k_dist_split32 + shared own-block GEMM merge + ring meta hint -- parity, A/B, P=8 emulation
set -o pipefail
mkdir -p gpurun_out/s11
timeout -k 10 700 python -u -m pytest tests/test_gpu_f32.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_fullsize_ring.py tests/test_gpu_ring_rotation.py tests/test_gpu_rccl_self.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s11/tests.log 2>&1 || { tail -40 gpurun_out/s11/tests.log; exit 1; }
tail -1 gpurun_out/s11/tests.log
for r in 1 2; do
for v in 0 1; do
  export KNN_SPLIT16=$v
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 10 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s11/mr_$v.log 2>&1 || { tail -20 gpurun_out/s11/mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s11/mr_$v.log | tr '\n' ' '; echo " mnist-real SPLIT16=$v"
done
done
unset KNN_SPLIT16
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1,2,4,8 --steps 5 > gpurun_out/s11/emu_mr.log 2>&1 || { tail -20 gpurun_out/s11/emu_mr.log; exit 1; }
grep '"P"' gpurun_out/s11/emu_mr.log
