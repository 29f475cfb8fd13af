# PMC passes (one counter group per run, kernel-trace only) on one bench step.
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --check 0"
run() { name=$1; shift; timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run --pmc "$@" -- $CMD > gpurun_out/pmc/$name.log 2>&1; echo "$name rc=$?"; }
run fetch FETCH_SIZE && run write WRITE_SIZE && run mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES && run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY
ls gpurun_out/pmc
