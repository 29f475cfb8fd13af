# round-5 session 13: which change broke test_gemm_state_holds_near_ties (split32 vs the deferred own-block merge)
set -o pipefail
mkdir -p gpurun_out/s13
for v in "KNN_SPLIT16=1" "KNN_NO_PAIR_FUSED=1" "KNN_SPLIT16=1 KNN_NO_PAIR_FUSED=1" "KNN_DUMMY=1"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -q -m gpu -k "near_ties or fp64_blocks or split_filter" --timeout 200 --timeout-method thread > gpurun_out/s13/t.log 2>&1
  echo "$v: $(tail -1 gpurun_out/s13/t.log)"
  grep -E "^E .*assert [0-9]+ == 0|AssertionError: [0-9]+" gpurun_out/s13/t.log | head -3
done
