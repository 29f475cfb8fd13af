# round-4 session 12: P = 8 split hint A/B (same box)
set -o pipefail
mkdir -p gpurun_out
E="timeout -k 10 200 python -u tools/ring_emulate.py --workload mnist --steps 10 --warm 5"
for i in 1 2; do
$E --ranks 1,8 > gpurun_out/s12_hint_$i.log 2>&1 || { tail -20 gpurun_out/s12_hint_$i.log; exit 1; }
$E --ranks 1,8 --no-hint > gpurun_out/s12_nohint_$i.log 2>&1 || { tail -20 gpurun_out/s12_nohint_$i.log; exit 1; }
done
grep '"P"' gpurun_out/s12_*.log
