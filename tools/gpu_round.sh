# Round evidence for one workload (WL=mnist|sift|gist, default mnist):
# full bench (with CPU leg), kernel-trace stats, PMC traffic + MFMA busy.
# PYTEST=1 also runs the GPU tests and smoke() first.
set -o pipefail
WL=${WL:-mnist}
OUT=gpurun_out/round_$WL
mkdir -p $OUT
if [ "${PYTEST:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "$WL" = mnist ]; then STEPS="--steps 5 --warmup 2"; PSTEPS="--steps 1 --warmup 0"; else STEPS="--steps 3 --warmup 1"; PSTEPS="--steps 1 --warmup 0"; fi
timeout -k 10 500 python -u bench.py --workload $WL $STEPS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.log; exit $rc; }
grep '^{' $OUT/bench.log > $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 bench.py --workload $WL --no-cpu-baseline --check 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD $STEPS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- $CMD $PSTEPS > $OUT/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- $CMD $PSTEPS > $OUT/write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/mfma -o run --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES -- $CMD $PSTEPS > $OUT/mfma.log 2>&1
rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
