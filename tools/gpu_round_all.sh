# All three workloads' evidence in one call (tests + smoke once, first).
set -o pipefail
PYTEST=1 WL=mnist bash tools/gpu_round.sh && WL=sift bash tools/gpu_round.sh && WL=gist bash tools/gpu_round.sh
