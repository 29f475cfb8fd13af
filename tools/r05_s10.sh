# round-5 session 10: mnist-real P=8 merge cost -- query order, fuse-all; sift P=8 research; mnist P=1..8
set -o pipefail
mkdir -p gpurun_out/s10
timeout -k 10 200 python -u tools/ring_emulate.py --workload mnist-real --ranks 8 --steps 5 --fuse all > gpurun_out/s10/emu_mr_all.log 2>&1 || { tail -20 gpurun_out/s10/emu_mr_all.log; exit 1; }
grep '"P"' gpurun_out/s10/emu_mr_all.log
KNN_ORDER=1 timeout -k 10 200 python -u tools/ring_emulate.py --workload mnist-real --ranks 8 --steps 5 > gpurun_out/s10/emu_mr_order.log 2>&1 || { tail -20 gpurun_out/s10/emu_mr_order.log; exit 1; }
grep '"P"' gpurun_out/s10/emu_mr_order.log
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist --ranks 1,2,4,8 --steps 10 > gpurun_out/s10/emu_mnist.log 2>&1 || { tail -20 gpurun_out/s10/emu_mnist.log; exit 1; }
grep '"P"' gpurun_out/s10/emu_mnist.log
timeout -k 10 400 python -u tools/ring_emulate.py --workload sift --ranks 1,8 --steps 3 > gpurun_out/s10/emu_sift.log 2>&1 || { tail -20 gpurun_out/s10/emu_sift.log; exit 1; }
grep '"P"' gpurun_out/s10/emu_sift.log
