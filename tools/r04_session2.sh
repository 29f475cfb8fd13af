# round-4 measurement session 2: configs[4] at full size, per-rank ring
# emulation (configs[2], [3], [4]), the gist bench / trace / PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py -x -v --timeout 900 --timeout-method thread > gpurun_out/config4.log 2>&1 || { tail -30 gpurun_out/config4.log; exit 1; }
tail -3 gpurun_out/config4.log
bash tools/gpu.sh emu:mnist:1,2,4,8:5 emu:sift:8:3 emu:mnist-real:1,8:3 || exit $?
timeout -k 10 500 python -u tools/ring_emulate.py --workload gist --ranks 8 --steps 1 --warm 1 > gpurun_out/emu_gist.log 2>&1 || { tail -20 gpurun_out/emu_gist.log; exit 1; }
grep '"P"' gpurun_out/emu_gist.log
bash tools/gpu.sh bench:gist:3 trace:gist:3 pmc:gist:1 || exit $?
