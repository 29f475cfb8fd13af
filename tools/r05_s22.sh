# round-5 session 22: LDS and cycle counters of k_dist_split (16x16) vs k_dist_split32 on mnist-real
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/s22
LDS="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
CYC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
INST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for v in 0 1; do
  if [ $v = 1 ]; then export KNN_SPLIT32=1; else unset KNN_SPLIT32; fi
  for g in lds cyc inst; do
    case $g in lds) cs=$LDS ;; cyc) cs=$CYC ;; inst) cs=$INST ;; esac
    (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
     timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/s22/v${v}_$g" -o run \
       --pmc $cs -- python3 bench.py --workload mnist-real --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 \
       > "gpurun_out/s22/v${v}_$g.log" 2>&1) || { echo "pmc $v $g failed"; tail -5 gpurun_out/s22/v${v}_$g.log; exit 1; }
  done
done
python3 tools/pmc_breakdown.py gpurun_out/s22/v0_lds gpurun_out/s22/v0_cyc gpurun_out/s22/v0_inst gpurun_out/s22/v1_lds gpurun_out/s22/v1_cyc gpurun_out/s22/v1_inst > gpurun_out/s22/breakdown.txt
grep -i "split" gpurun_out/s22/breakdown.txt | head -40
