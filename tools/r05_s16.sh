# round-5 session 16: coalesced multi-block split conversion -- its restatement test, split-filter parity, mnist-real P=1/8 emulation + trace
set -o pipefail
mkdir -p gpurun_out/s16
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_pack.py tests/test_gpu_f32.py tests/test_gpu_parity.py tests/test_gpu_rccl_self.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s16/tests.log 2>&1 || { tail -40 gpurun_out/s16/tests.log; exit 1; }
tail -1 gpurun_out/s16/tests.log
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1,2,4,8 --steps 5 > gpurun_out/s16/emu_mr.log 2>&1 || { tail -20 gpurun_out/s16/emu_mr.log; exit 1; }
grep '"P"' gpurun_out/s16/emu_mr.log
bash tools/gpu.sh emutrace:mnist-real:8
