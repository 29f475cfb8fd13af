# round-5 session 9: fused GEMM step (k_dist_split block table + k_merge table) parity; split ablations; P=8 emulation
set -o pipefail
mkdir -p gpurun_out/s9
timeout -k 10 700 python -u -m pytest tests/test_gpu_ring_rotation.py tests/test_gpu_parity.py tests/test_gpu_fullsize_ring.py tests/test_gpu_f32.py tests/test_gpu_rccl_self.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s9/tests.log 2>&1 || { tail -40 gpurun_out/s9/tests.log; exit 1; }
tail -1 gpurun_out/s9/tests.log
for v in prod noepi noepi_nodma noepi_nofrag noepi_nomfma; do
  if [ $v = prod ]; then unset KNN_LIB_PATH; else export KNN_LIB_PATH=$PWD/tools/abl5/libknn_$v.so; fi
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 5 --warmup 2 --no-cpu-baseline --check 0 --secondary-steps 0 > gpurun_out/s9/mr_$v.log 2>&1 || { tail -20 gpurun_out/s9/mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/s9/mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
done
unset KNN_LIB_PATH
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1,2,4,8 --steps 5 > gpurun_out/s9/emu_mr.log 2>&1 || { tail -20 gpurun_out/s9/emu_mr.log; exit 1; }
grep '"P"' gpurun_out/s9/emu_mr.log
