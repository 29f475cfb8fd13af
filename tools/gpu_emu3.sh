set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ring_emulate.py --steps 5 > gpurun_out/ring_emu.log 2>&1
rc=$?; echo "emu rc=$rc"; [ $rc -eq 0 ] || exit $rc
KNN_NO_H16=1 timeout -k 10 300 python -u tools/ring_emulate.py --steps 5 > gpurun_out/ring_emu_f64.log 2>&1
rc=$?; echo "emu f64 rc=$rc"; exit $rc
