set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ring_emulate.py --steps 5 > gpurun_out/ring_emu.log 2>&1
rc=$?; echo "emu rc=$rc"; grep -E '"[1248]"|rank_ms|dist_busy|splits|shadow' gpurun_out/ring_emu.log | tr -d '\n'; echo; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/emu_trace -o run -- python3 tools/ring_emulate.py --ranks 8 --steps 2 > gpurun_out/emu_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
