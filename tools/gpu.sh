# One GPU session: the steps named on the command line, in order, each under
# its own time limit; the session stops at the first step that fails.
#
#   gpurun -- bash tools/gpu.sh STEP [STEP ...]
#
# Steps (outputs under gpurun_out/<tag>/):
#   tests[:EXPR]          pytest -m gpu (optionally -k EXPR); then smoke()
#   bench:WL[:STEPS]      bench.py --workload WL (CPU leg included)
#   trace:WL[:STEPS]      rocprofv3 --kernel-trace --stats of a bench run (6 warm-up
#                         steps inside the traced process; make_profiles.py
#                         averages the launches after them)
#   pmc:WL:REP            FETCH_SIZE, WRITE_SIZE, MFMA-busy passes (REP
#                         repetitions of each, one counter group per run)
#   emu:WL[:RANKS[:STEPS[:FUSE[:SPLITS]]]] tools/ring_emulate.py (per-rank ring
#                         work; FUSE none|rest|all; SPLITS a comma list to sweep)
#   emutrace:WL:RANKS     the same under --kernel-trace
#   kb8:ARGS              tools/probe/kbench8.py ARGS (commas kept, '+' = space)
#   kb8@NAME:ARGS         the same on an ablated copy (tools/probe/ablate.py NAME)
set -o pipefail
mkdir -p gpurun_out
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
fail() { echo "step $1 rc=$2"; exit "$2"; }

run_step() {
  local spec=$1 kind a b
  kind=${spec%%:*}
  a=$(echo "$spec" | cut -s -d: -f2)
  b=$(echo "$spec" | cut -s -d: -f3)
  case $kind in
  tests)
    local K=()
    [ -n "$a" ] && K=(-k "$a")
    timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread "${K[@]}" \
      > gpurun_out/pytest.log 2>&1 || { rc=$?; tail -30 gpurun_out/pytest.log; fail "$spec" $rc; }
    tail -2 gpurun_out/pytest.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { rc=$?; tail -20 gpurun_out/smoke.log; fail smoke $rc; }
    echo "smoke ok" ;;
  bench)
    local st=${b:-5}
    timeout -k 10 500 python -u bench.py --workload "$a" --steps "$st" --warmup 2 > "gpurun_out/bench_$a.log" 2>&1 \
      || { rc=$?; tail -20 "gpurun_out/bench_$a.log"; fail "$spec" $rc; }
    grep '^{' "gpurun_out/bench_$a.log" | tail -1 ;;
  trace)
    (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
     timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/trace_$a" -o run -- \
       python3 bench.py --workload "$a" --no-cpu-baseline --secondary-steps 0 --check 0 --steps ${b:-10} --warmup 6 \
       > "gpurun_out/trace_$a.log" 2>&1) || fail "$spec" $? ;;
  pmc)
    local rep=${b:-3} i g
    for i in $(seq 1 "$rep"); do
      for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
        local tag
        tag=$(echo "$g" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
        (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
         timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/pmc_$a/${tag}_$i" -o run \
           --pmc $g -- python3 bench.py --workload "$a" --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 \
           > "gpurun_out/pmc_$a/${tag}_$i.log" 2>&1) || fail "$spec:$tag:$i" $?
      done
    done ;;
  pmcx)
    # one SQ counter group per run (slots: 8 SQ, 2 GRBM): instruction mix,
    # cycle buckets or LDS; one bench step, the distance kernel's dispatch
    local cs
    case $b in
    inst) cs="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE" ;;
    cyc) cs="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" ;;
    lds) cs="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" ;;
    *) echo "unknown pmcx group $b"; exit 2 ;;
    esac
    mkdir -p "gpurun_out/pmcx_$a"
    (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
     timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/pmcx_$a/$b" -o run \
       --pmc $cs -- python3 bench.py --workload "$a" --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 \
       > "gpurun_out/pmcx_$a/$b.log" 2>&1) || fail "$spec" $?
    python3 tools/pmc_breakdown.py "gpurun_out/pmcx_$a/$b" ;;
  emu)
    local es fz sw
    es=$(echo "$spec" | cut -s -d: -f4)
    fz=$(echo "$spec" | cut -s -d: -f5)
    sw=$(echo "$spec" | cut -s -d: -f6)
    local lg="emu_${a}_${fz:-rest}_${b//,/-}${sw:+_sweep}.log"
    timeout -k 10 400 python -u tools/ring_emulate.py --workload "$a" --ranks "${b:-1,2,4,8}" --steps "${es:-5}" \
      ${fz:+--fuse $fz} ${sw:+--splits $sw} > "gpurun_out/$lg" 2>&1 \
      || { rc=$?; tail -20 "gpurun_out/$lg"; fail "$spec" $rc; }
    grep '"P"' "gpurun_out/$lg" ;;
  emutrace)
    (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
     timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/emutrace_$a" -o run -- \
       python3 tools/ring_emulate.py --workload "$a" --ranks "${b:-8}" --steps 3 \
       > "gpurun_out/emutrace_$a.log" 2>&1) || fail "$spec" $? ;;
  kb8|kb8@*)
    # kb8@NAME:ARGS times the ablated copy tools/probe/abl/libkbench8_NAME.so
    local args=${spec#*:} so=""
    [ "${kind#kb8@}" != "$kind" ] && so="tools/probe/abl/libkbench8_${kind#kb8@}.so"
    echo "== $spec" >> gpurun_out/kb8.log
    KB8_SO=$so timeout -k 10 300 python -u tools/probe/kbench8.py ${args//+/ } >> gpurun_out/kb8.log 2>&1 \
      || { rc=$?; tail -20 gpurun_out/kb8.log; fail "$spec" $rc; }
    grep '^{' gpurun_out/kb8.log | tail -40 ;;
  *) echo "unknown step $spec"; exit 2 ;;
  esac
  return 0
}

for s in "$@"; do
  [ "${s%%:*}" = pmc ] && mkdir -p "gpurun_out/pmc_$(echo "$s" | cut -d: -f2)"
  run_step "$s" || exit $?
  echo "step $s ok"
done
